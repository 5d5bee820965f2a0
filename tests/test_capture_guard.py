"""The capture-topology guard (_lib.CaptureTopology) as plain host logic.

Under graph capture, torch's HIP 7.0 runtime files every non-origin stream that waits on a captured
event under the producing stream's list and walks those lists recursively at hipStreamEndCapture; a
cycle never returns (the r5u abort).  The guard keeps that filing per capture and raises
before a wait that would close a cycle.  Stream handles are plain ints here (no GPU)."""
import pytest

from svdformer_pointsea_amd._lib import CaptureTopology

M, S0, S1, S3 = 0x10, 0x20, 0x30, 0x40   # origin (capture) stream and three side streams


def test_flat_and_cross_forks_pass():
    t = CaptureTopology()
    t.wait(S0, M, M, cid=1)   # fork lane 0
    t.wait(S3, M, M, cid=1)   # fork lane 3 from the origin (base="outer")
    t.wait(S0, S3, M, cid=1)  # lane 0 joins lane 3: S0 filed under S3 -- no cycle (the cross shape)
    t.wait(M, S0, M, cid=1)   # origin joins: never filed
    t.wait(M, S3, M, cid=1)
    assert t.filed == {M: {S0, S3}, S3: {S0}}


def test_nested_fork_join_cycle_raises():
    """M -> S0, S0 -> S3 (nested fork), S3 -> S0 (its join): the shape that segfaulted in round 4."""
    t = CaptureTopology()
    t.wait(S0, M, M, cid=7)
    t.wait(S3, S0, M, cid=7)
    with pytest.raises(RuntimeError, match="closes a cycle"):
        t.wait(S0, S3, M, cid=7)


def test_longer_cycle_raises():
    t = CaptureTopology()
    t.wait(S0, M, M, cid=2)
    t.wait(S1, S0, M, cid=2)
    t.wait(S3, S1, M, cid=2)
    with pytest.raises(RuntimeError, match="closes a cycle"):
        t.wait(S0, S3, M, cid=2)


def test_self_wait_raises():
    t = CaptureTopology()
    with pytest.raises(RuntimeError, match="its own work"):
        t.wait(S0, S0, M, cid=3)
    with pytest.raises(RuntimeError, match="its own work"):
        t.wait(M, M, M, cid=3)


def test_new_capture_forgets_old_filing():
    """The filing belongs to one capture: a later capture (new id) may wait the other way round."""
    t = CaptureTopology()
    t.wait(S0, M, M, cid=4)
    t.wait(S3, S0, M, cid=4)
    t.wait(S0, S3, M, cid=5)   # capture 5 starts clean: S0 under S3 only
    assert t.filed == {S3: {S0}}


def test_fork_join_inside_own_block_raises_on_cpu_path():
    """join() inside its own block is refused before any stream call; on CPU tensors fork is a no-op."""
    import torch

    from svdformer_pointsea_amd import _lib

    x = torch.zeros(3)
    with _lib.fork(x.device, inputs=(x,)) as br:   # CPU: not a real fork, join is a pass-through
        assert br.join(x) is x

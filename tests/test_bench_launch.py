"""bench.py --gpus N measures N GPUs: outside torch.distributed.run it starts
one rank per GPU itself (a child `python -m torch.distributed.run
--nproc-per-node N ... bench.py <same args>`, before anything touches the
GPU), and inside a launcher a world size that disagrees with --gpus fails
instead of reporting the wrong n_gpus.  CPU-only: the launcher's argv is
checked by a dry run."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_self_launch_argv():
    args = ["--gpus", "4", "--steps", "7", "--warmup", "2", "--dry-run-launch"]
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=_env(), cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    cmd = json.loads(lines[0])["launch"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert int(cmd[cmd.index("--master-port") + 1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == args          # the ranks see exactly the same arguments


def test_world_size_must_match_gpus():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), cwd=ROOT, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode != 0
    assert "--gpus 4 but WORLD_SIZE=2" in out.stderr
    assert out.stdout.strip() == ""     # no JSON line with a wrong n_gpus


def test_attention_work_parses_both_call_forms():
    """bench.kernel_work reads (B, H, Lq, Lk, D, dtype) from the plain attention entries and from the
    *_colsum ones, which carry extra output pointers before B (the position counts from the end)."""
    sys.path.insert(0, ROOT)
    import bench

    B, H, Lq, Lk, D = 2, 8, 2048, 1024, 64
    strides = (0,) * 12
    tail = (B, H, Lq, Lk, D, 0.125, 1) + strides + (None, 0, None)   # ..., workspace, bytes, stream
    for lead in (7, 8):   # pcops_attention_bwd_dq_delta / _dq_delta_colsum
        assert bench.kernel_work("attention bwd dq", (None,) * lead + tail)[0] == 2.0 * B * H * Lq * Lk * D
    for lead in (7, 9):   # pcops_attention_bwd_dkv / _dkv_colsum
        assert bench.kernel_work("attention bwd dkv", (None,) * lead + tail)[0] == 8.0 * B * H * Lq * Lk * D
    fwd = (None,) * 5 + (B, H, Lq, Lk, D, 0.125, 1) + strides + (None,)
    work, unit, _, bound = bench.kernel_work("attention forward", fwd)
    assert work == 4.0 * B * H * Lq * Lk * D and unit == "TFLOP/s" and bound == "mfma"

"""ctypes binding of libpcops.so (C-ABI: include/pcops.h).

The product path has NO CPU fallback: if the HIP library is missing or a
tensor is not on the GPU, the call raises.  Tensors are passed as raw device
pointers; every launch goes to torch's current HIP stream of the tensor's
device, so the ops compose with torch kernels, streams and hipGraph capture.
"""
import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# PCOPS_LIB_PATH selects an alternative build of the same C-ABI (A/B kernel experiments)
LIB_PATH = os.environ.get("PCOPS_LIB_PATH") or os.path.join(_HERE, "_lib", "libpcops.so")

_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
D = ctypes.c_double
LL = ctypes.c_longlong
ULL = ctypes.c_ulonglong

_SIGS = {
    "pcops_status_string": (ctypes.c_char_p, [I]),
    "pcops_abi_version": (I, []),
    "pcops_fps_workspace_bytes": (ULL, [I, I]),
    "pcops_furthest_point_sampling": (I, [P, I, I, I, P, P, ULL, P]),
    "pcops_furthest_point_sampling_counts": (I, [P, P, I, I, I, P, P, ULL, P]),
    "pcops_gather_points": (I, [P, P, I, I, I, I, P, P]),
    "pcops_gather_points_grad": (I, [P, P, I, I, I, I, P, P]),
    "pcops_group_points": (I, [P, P, I, I, I, I, I, P, P]),
    "pcops_group_points_grad": (I, [P, P, I, I, I, I, I, P, P]),
    "pcops_sa_group": (I, [P, P, P, P, I, I, I, I, I, P, I, P]),
    "pcops_sa_group_grad": (I, [P, I, P, I, I, I, I, I, P, P]),
    "pcops_ball_query": (I, [P, P, I, I, I, F, I, P, P]),
    "pcops_three_nn": (I, [P, P, I, I, I, P, P, P]),
    "pcops_three_interpolate": (I, [P, P, P, I, I, I, I, P, P]),
    "pcops_three_interpolate_grad": (I, [P, P, P, I, I, I, I, P, P]),
    "pcops_knn": (I, [P, P, I, I, I, I, I, I, P, P, P]),
    "pcops_knn_workspace_bytes": (ULL, [I, I, I, I, I]),
    "pcops_knn_ws": (I, [P, P, I, I, I, I, I, I, P, P, P, ULL, P]),
    "pcops_chamfer_forward": (I, [P, P, I, I, I, P, P, P, P, P]),
    "pcops_chamfer_workspace_bytes": (ULL, [I, I, I]),
    "pcops_chamfer_forward_ws": (I, [P, P, I, I, I, P, P, P, P, P, ULL, P]),
    "pcops_chamfer_backward": (I, [P, P, I, I, I, P, P, P, P, P, P, P]),
    "pcops_chamfer_sqrt_mean_grad": (I, [P, F, P, LL, P, LL, P, P, P]),
    "pcops_maxpool3s2_fwd": (I, [P, I, I, I, I, I, P, P, P]),
    "pcops_maxpool3s2_bwd": (I, [P, P, I, I, I, I, I, P, P]),
    "pcops_emd_workspace_bytes": (ULL, [I, I]),
    "pcops_emd_forward": (I, [P, P, I, I, F, I, P, P, P, ULL, P]),
    "pcops_emd_backward": (I, [P, P, P, P, I, I, P, P]),
    "pcops_attention_forward": (I, [P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P]),
    "pcops_attention_bwd_workspace_bytes": (ULL, [I, I, I, I, I]),
    "pcops_attention_backward": (I, [P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_preprocess": (I, [P, P, I, I, I, I, I, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_dq": (I, [P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_dkv": (I, [P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_dq_delta": (I, [P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_colsum_workspace_bytes": (ULL, [I, I, I, I, I]),
    "pcops_attention_bwd_fused_workspace_bytes": (ULL, [I, I, I, I, I, I]),
    "pcops_attention_bwd_fused": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_dq_delta_colsum": (I, [P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_attention_bwd_dkv_colsum": (I, [P, P, P, P, P, P, P, P, P, I, I, I, I, I, F, I, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, LL, P, ULL, P]),
    "pcops_transpose_add": (I, [P, I, P, I, P, I, P, I, I, I, I, P]),
    "pcops_add": (I, [P, I, P, I, P, I, LL, P]),
    "pcops_add_posemb": (I, [P, I, P, P, I, I, I, P, I, P]),
    "pcops_crop_pack": (I, [P, P, P, P, I, I, I, P, P, P]),
    "pcops_add_rows": (I, [P, I, P, I, P, I, LL, I, LL, P]),
    "pcops_linear_skinny": (I, [P, LL, I, P, P, P, I, P]),
    "pcops_edge_group": (I, [P, P, I, I, I, I, P, I, P]),
    "pcops_edge_group_grad": (I, [P, I, P, I, I, I, I, P, P]),
    "pcops_max_k": (I, [P, I, LL, I, I, P, P, P]),
    "pcops_max_k_grad": (I, [P, I, P, LL, I, I, P, P]),
    "pcops_gelu_bwd_colsum": (I, [P, P, I, LL, I, P, P, I, P, ULL, P]),
    "pcops_layernorm_fwd": (I, [P, I, P, I, P, P, F, I, I, P, P, P, P, P]),
    "pcops_layernorm_bwd_workspace_bytes": (ULL, [I, I]),
    "pcops_layernorm_bwd": (I, [P, P, P, I, P, I, P, P, P, I, I, P, P, P, P, P, ULL, P]),
    "pcops_layernorm_bwd_colsum_workspace_bytes": (ULL, [I, I]),
    "pcops_layernorm_bwd_colsum": (I, [P, P, P, I, P, I, P, P, P, I, I, P, P, P, P, P, I, P, ULL, P]),
    "pcops_layernorm_bwd_bf16g": (I, [P, P, P, I, P, I, P, P, P, I, I, P, P, P, P, P, I, P, ULL, P]),
    "pcops_layernorm_bwd_ex": (I, [P, I, LL, P, P, P, I, P, I, P, P, P, I, I, P, P, P, P, P, I, P, ULL, P]),
    "pcops_adam_flat": (I, [P, P, P, LL, LL, P, P, P, P, D, P, D, D, D, D, I, P]),
    "pcops_blend_fwd": (I, [P, I, P, P, LL, P, I, P]),
    "pcops_blend_bwd": (I, [P, I, P, I, P, P, LL, P, P, P, P]),
    "pcops_sum_rows": (I, [P, I, LL, P, I, P]),
    "pcops_wgrad_skinny_workspace_bytes": (ULL, [I, I]),
    "pcops_wgrad_skinny": (I, [P, P, LL, I, I, P, I, P, ULL, P]),
    "pcops_colsum_workspace_bytes": (ULL, [LL, I]),
    "pcops_colsum": (I, [P, I, LL, I, P, I, P, ULL, P]),
    "pcops_colsum_ld": (I, [P, I, LL, I, LL, P, I, P, ULL, P]),
    "pcops_batchnorm_workspace_bytes": (ULL, [LL, I]),
    "pcops_batchnorm_fwd": (I, [P, I, P, I, LL, I, P, P, P, P, F, F, I, I, F, P, P, P, P, ULL, P, P]),
    "pcops_batchnorm_bwd": (I, [P, P, P, I, LL, I, P, P, P, I, I, F, P, P, P, P, P, ULL, P]),
    "pcops_conv3x3_fwd": (I, [P, P, I, I, I, I, P, P]),
    "pcops_conv3x3_fwd_res": (I, [P, P, I, I, I, I, P, P, P]),
    "pcops_conv3x3_wgrad_workspace_bytes": (ULL, [I]),
    "pcops_conv3x3_wgrad": (I, [P, P, I, I, I, I, P, I, I, P, ULL, P]),
    "pcops_conv3x3_c1_fwd": (I, [P, P, I, I, I, P, P]),
    "pcops_conv3x3_c1_wgrad_workspace_bytes": (ULL, []),
    "pcops_conv3x3_c1_wgrad": (I, [P, P, I, I, I, P, I, P, ULL, P]),
    "pcops_pcsa_forward": (I, [P, I, P, I, P, I, I, I, P, P]),
    "pcops_pcsa_backward": (I, [P, I, P, I, P, I, P, I, I, I, P, P, P]),
    "pcops_points2depth_workspace_bytes": (ULL, [I, I, I, I]),
    "pcops_points2depth": (I, [P, P, P, I, I, I, I, I, P, P, ULL, P]),
    "pcops_points2grid": (I, [P, P, P, P, I, I, I, I, I, P, P]),
    "pcops_grid2image_workspace_bytes": (ULL, [I, I, I]),
    "pcops_grid2image": (I, [P, P, I, I, I, P, P, ULL, P]),
}


def exported_symbols():
    return list(_SIGS)


def lib():
    """Load libpcops.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"svdformer_pointsea_amd: HIP library not built ({LIB_PATH}); run "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)"
            )
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def check(status, what):
    if status != 0:
        msg = lib().pcops_status_string(status).decode()
        raise RuntimeError(f"{what} failed: {msg} (status {status})")


class KernelTimer:
    """Opt-in HIP-event timing of every C-ABI launch, per call name.

    Events are recorded on the very stream the call launches on (torch's
    current stream of the current device), so spans are exact per call even
    when the caller uses side streams.  Used by bench.py; off by default."""

    spans = None  # name -> [(start_event, end_event, scalar args)] while enabled

    @classmethod
    def enable(cls):
        cls.spans = {}

    @classmethod
    def disable(cls):
        cls.spans = None

    @classmethod
    def reset(cls):
        if cls.spans is not None:
            cls.spans = {}

    @classmethod
    def summary(cls):
        """name -> (launches, mean ms, total ms); call after synchronising."""
        out = {}
        for name, evs in (cls.spans or {}).items():
            ms = [a.elapsed_time(b) for a, b, _ in evs]
            out[name] = (len(ms), sum(ms) / len(ms), sum(ms))
        return out


def call(what, fn, *args):
    """Run one C-ABI entry point on the current device; raise on failure."""
    spans = KernelTimer.spans
    if spans is None:
        return check(fn(*args), what)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    status = fn(*args)
    e1.record(s)
    # sizes as given; pointers as their address (None for NULL)
    scalars = tuple(a if isinstance(a, (int, float)) else (a.value if isinstance(a, P) else None) for a in args)
    spans.setdefault(what, []).append((e0, e1, scalars))
    check(status, what)


def require_gpu(t, name):
    """utils.h:5-25 CHECK_CUDA / CHECK_CONTIGUOUS, as RuntimeError."""
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")


def require_float(t, name):
    require_gpu(t, name)
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be a float tensor")


def require_int(t, name):
    require_gpu(t, name)
    if t.dtype != torch.int32:
        raise RuntimeError(f"{name} must be an int tensor")


_SIDE = {}
_TLS = threading.local()


class CaptureTopology:
    """Refuses, with a RuntimeError, a stream wait that would kill the process at
    hipStreamEndCapture.

    While capturing, torch's HIP runtime (7.0.51831) files every NON-ORIGIN stream
    that waits on a captured event under the waited (producing) stream's list of
    parallel capture streams and walks those lists recursively at end of capture.
    A cycle in that filing -- a stream waiting on its own event, or a nested fork
    joined back into the stream it forked from -- makes the walk recurse until the
    stack overflows (a segfault inside capture_end, no Python traceback: the r5u
    abort).  `wait(waiter, producer, origin)` is called before every wait the fork /
    join / SharedFPS / fused-sum hand-offs issue; it keeps the filing graph of the
    capture in progress (keyed by its capture id) and raises instead of issuing a
    wait that closes a cycle.  Streams are identified by their integer handle, so
    the check itself is plain host logic (tests/test_capture_guard.py)."""

    def __init__(self):
        self.cid = None
        self.filed = {}   # producer handle -> set of waiter handles filed under it

    def reset(self, cid=None):
        self.cid, self.filed = cid, {}

    def _reaches(self, a, b):
        seen, todo = set(), [a]
        while todo:
            s = todo.pop()
            if s == b:
                return True
            if s in seen:
                continue
            seen.add(s)
            todo.extend(self.filed.get(s, ()))
        return False

    def wait(self, waiter, producer, origin, cid=None):
        """Record (or refuse) `waiter` waiting on work of `producer` in capture `cid`."""
        if cid != self.cid:
            self.reset(cid)
        if waiter == producer:
            raise RuntimeError(
                f"stream {waiter:#x} would wait on its own work while capturing a HIP graph: the runtime's "
                "end-of-capture walk never returns on that (DESIGN.md 1.2); stream order already covers it")
        if waiter == origin:
            return   # the capture's origin stream is never filed
        if self._reaches(waiter, producer):
            raise RuntimeError(
                f"stream {waiter:#x} waiting on stream {producer:#x} closes a cycle among the captured side "
                "streams (each is already filed under the other): hipStreamEndCapture would never return "
                "(DESIGN.md 1.2); fork from the outer origin (fork(..., base='outer')) or run inline")
        self.filed.setdefault(producer, set()).add(waiter)


_TOPO = CaptureTopology()
_CAPINFO = []


def _capture_id(stream):
    """The id of the capture `stream` takes part in (hipStreamGetCaptureInfo of torch's own HIP
    runtime), or None when that entry point cannot be reached."""
    if not _CAPINFO:
        fn = None
        try:
            h = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
            fn = h.hipStreamGetCaptureInfo
            fn.restype = ctypes.c_int
            fn.argtypes = [P, ctypes.POINTER(I), ctypes.POINTER(ULL)]
        except (OSError, AttributeError):
            fn = None
        _CAPINFO.append(fn)
    fn = _CAPINFO[0]
    if fn is None:
        return None
    st, cid = I(0), ULL(0)
    if fn(P(stream.cuda_stream), ctypes.byref(st), ctypes.byref(cid)) != 0 or st.value != 1:
        return None
    return cid.value


def _origin(cur):
    """The capture's origin stream: the outermost fork's base, else the stream current outside any fork."""
    stack = getattr(_TLS, "mains", None)
    return stack[0] if stack else cur


def guarded_wait(waiter, producer, event=None, origin=None):
    """waiter.wait_stream(producer) -- or waiter.wait_event(event) recorded on `producer` --
    after the capture-topology check (a RuntimeError instead of a crash in capture_end).
    `origin` defaults to the outermost fork's base, else the waiter itself (a top-level wait)."""
    if torch.cuda.is_current_stream_capturing():
        origin = origin if origin is not None else _origin(waiter)
        _TOPO.wait(waiter.cuda_stream, producer.cuda_stream, origin.cuda_stream, _capture_id(waiter))
    if event is not None:
        waiter.wait_event(event)
    else:
        waiter.wait_stream(producer)


def on_side_stream():
    """True inside a `fork` block on this thread (the block's ops run on a side stream)."""
    return getattr(_TLS, "side", 0) > 0


class no_stream_k:
    """GEMMs issued inside run on rocBLAS instead of hipBLASLt, with TunableOp
    off.  hipBLASLt's gfx950 bf16 solutions are stream-K (streamK=3 in 208 of
    the 211 solutions of its Tensile library; 85 of the 88 GEMM kernels a PCN
    step launches carry _SK3_): workgroups that own a split tile spin-wait for
    the partial sums of other workgroups of the same launch, which assumes the
    whole grid becomes resident.  Two such launches on two streams can each
    hold the CUs the other's producers need -- the recorded graph-replay hang.
    rocBLAS's gfx950 bf16 Tensile solutions are all streamK=0 (data-parallel,
    no cross-workgroup waits), so side-stream GEMMs go there and at most one
    spinning launch is ever in flight.  The switches are process-global; they
    are flipped around the issue of the side-stream GEMMs only (on the one
    thread issuing them), including at graph-capture time."""

    def __enter__(self):
        import torch.cuda.tunable as tunable

        self.prev = (torch.backends.cuda.preferred_blas_library(), tunable.is_enabled())
        torch.backends.cuda.preferred_blas_library("cublas")
        tunable.enable(False)
        return self

    def __exit__(self, *exc):
        import torch.cuda.tunable as tunable

        torch.backends.cuda.preferred_blas_library(self.prev[0])
        tunable.enable(self.prev[1])
        return False


def side_stream(device, lane=0):
    """Extra HIP streams per device (lane 0, 1, ...) for independent work that
    can run beside the current stream (the point ops fill only B of 256 CUs)."""
    key = (torch.device(device).index, lane)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=device)
    return _SIDE[key]


class fork:
    """`with fork(device, inputs=(x, ...)) as s:` runs the block on the side
    stream after the current stream's pending work; `join(*tensors)` makes the
    stream that is current AT THE JOIN wait for it and marks the tensors as
    used there.  No-op on CPU tensors.

    Memory safety across the two streams (the caching allocator only knows the
    stream a block was allocated on):
      * `inputs` -- every tensor the block reads that was allocated on the
        current stream -- are recorded on the side stream at entry.  The block's
        autograd nodes differentiate on the side stream too, and the saved
        tensors they read there may be released on the host before those
        kernels run; without the record the next current-stream allocation can
        take the block while a side-stream forward or backward kernel still
        reads it.
      * the block's outputs are recorded on the joining stream by `join`.

    Nested forks and HIP-graph capture.  Under stream
    capture the HIP runtime torch ships (7.0.51831) files every non-origin
    stream that waits on a captured event into the waited stream's list of
    "parallel capture streams", and at hipStreamEndCapture walks those lists
    recursively.  A fork opened INSIDE a fork (side stream S0 forks S3, then
    S0 waits on S3 at the join) files S3 under S0 and S0 under S3: the walk
    never ends and the process dies of a stack overflow inside capture_end
    (tools/capture_topology.hip reproduces it without torch; /opt/rocm 7.2's
    runtime has no such cycle).  Hence, while capturing, a nested fork
      * with base="outer" forks from the OUTERMOST fork's origin stream instead
        of the current side stream -- valid when the block reads only tensors
        that were ready there (the caller's promise) -- so the only side-to-side
        edge is the join, and no cycle forms;
      * otherwise runs inline on the current stream (no overlap, same result).
    Eagerly (no capture) both run as ordinary nested forks."""

    # PCOPS_SIDE_STREAMS=0 runs every block on the current stream (A/B runs, and
    # the only safe way to put hipBLASLt GEMMs inside a forked block)
    enabled = os.environ.get("PCOPS_SIDE_STREAMS", "1") != "0"

    def __init__(self, device, lane=0, inputs=(), base="current"):
        if base not in ("current", "outer"):
            raise ValueError(f"fork: base must be 'current' or 'outer', not {base!r}")
        self.on = fork.enabled and torch.device(device).type == "cuda"
        self.inline = False
        if self.on:
            stack = getattr(_TLS, "mains", None) or []
            cur = torch.cuda.current_stream(device)
            if stack and torch.cuda.is_current_stream_capturing():
                if base == "outer":
                    cur = stack[0]
                else:
                    self.on, self.inline = False, True
                    return
            self.main = cur
            self.side = side_stream(device, lane)
            self.inputs = tuple(t for t in inputs if isinstance(t, torch.Tensor) and t.is_cuda)

    def __enter__(self):
        if self.on:
            guarded_wait(self.side, self.main, origin=_origin(self.main))
            for t in self.inputs:
                t.record_stream(self.side)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
            if not hasattr(_TLS, "mains"):
                _TLS.mains = []
            _TLS.mains.append(self.main)
            _TLS.side = getattr(_TLS, "side", 0) + 1
        return self

    def __exit__(self, *exc):
        if self.on:
            _TLS.side -= 1
            _TLS.mains.pop()
            self._ctx.__exit__(*exc)
        return False

    def join(self, *tensors):
        if self.on:
            cur = torch.cuda.current_stream(self.side.device)
            if cur == self.side:
                # inside its own block: stream order already covers the tensors, and under capture the
                # self-wait would hang hipStreamEndCapture -- a misuse, refused either way
                raise RuntimeError("fork.join called on the fork's own side stream (inside its with-block); "
                                   "join after the block")
            guarded_wait(cur, self.side)
            for t in tensors:
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(cur)
        return tensors[0] if len(tensors) == 1 else tensors


class Workspace:
    """Per-device scratch arena reused across calls (grown, never shrunk).

    Keyed by (device, stream) so concurrent streams never share bytes.  A
    buffer that is outgrown is retired, not freed: a HIP graph captured
    earlier may still replay kernels that write to it, so its memory must
    never return to the caching allocator."""

    _bufs = {}
    _retired = []

    @classmethod
    def get(cls, device, nbytes):
        if nbytes <= 0:
            return None
        key = (device, torch.cuda.current_stream(device).cuda_stream)
        buf = cls._bufs.get(key)
        if buf is None or buf.numel() < nbytes:
            if buf is not None:
                cls._retired.append(buf)
            buf = torch.empty(int(nbytes), dtype=torch.uint8, device=device)
            cls._bufs[key] = buf
        return buf

"""Does a hipMemsetAsync captured into a torch CUDA graph run on every replay?

    python tools/capture_memset_probe.py

A  pcops_gather_points_grad (hipMemsetAsync + atomic scatter) into a buffer allocated before the
   capture, poisoned before each replay
B  the same into a buffer allocated inside the capture (graph pool)
C  a bare hipMemsetAsync (torch's libamdhip64 through ctypes) on a pre-allocated buffer
D  torch's zero_() (a fill kernel) for comparison
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from svdformer_pointsea_amd._lib import call, lib, ptr  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.init()
    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    B, C, N, M = 4, 16, 2048, 256
    g_out = torch.randn(B, C, M, device=dev)
    idx = torch.randint(0, N, (B, M), device=dev, dtype=torch.int32)
    ref = torch.zeros(B, C, N, device=dev)
    ref.view(B * C, N).scatter_add_(1, idx.long().repeat_interleave(C, 0), g_out.view(B * C, M))

    def gather_grad(out):
        s = torch.cuda.current_stream().cuda_stream
        call("gg", lib().pcops_gather_points_grad, ptr(g_out), ptr(idx), B, C, N, M, ptr(out), ctypes.c_void_p(s))

    for variant in "ABCD":
        static = torch.empty(B, C, N, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):   # warm-up
            if variant in "AB":
                gather_grad(static)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            if variant == "A":
                out = static
                gather_grad(out)
            elif variant == "B":
                out = torch.empty(B, C, N, device=dev)
                gather_grad(out)
            elif variant == "C":
                out = static
                r = hip.hipMemsetAsync(ctypes.c_void_p(out.data_ptr()), 0, out.numel() * 4,
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                assert r == 0, r
            else:
                out = static
                out.zero_()
        res = []
        for _ in range(4):
            out.fill_(123.0)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            want = ref if variant in "AB" else torch.zeros_like(ref)
            res.append(f"{(out - want).abs().max().item():.2e}")
        print(f"{variant}: max |out - expected| per replay: {' '.join(res)}", flush=True)
        del g


if __name__ == "__main__":
    main()

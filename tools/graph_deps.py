"""Dependency structure of the captured PCN / PointSea forward+backward graph: captures bench.py's
fwd_bwd (model + loss + backward under bf16 autocast, the gt pyramid on its side stream) once with
the HIP graph debug mode on and writes hipGraphDebugDotPrint's DOT file.

    python tools/graph_deps.py [svdformer|pointsea] <out.json>          (GPU: capture + dump)
    python tools/graph_deps.py parse <out.json> <kernel-regex> [depth]   (CPU: the ancestors of the
                                                                          first node whose name matches)
"""
import ctypes
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def capture(name, out):
    import torch

    from bench import Workload
    from svdformer_pointsea_amd import _lib

    dev = torch.device("cuda:0")
    wl = Workload(name)
    torch.manual_seed(0)
    model = wl.Model(wl.cfg).to(dev)
    partial, gt = wl.synth(wl.batch, 1000, dev)
    crop = torch.cuda.default_generators[0] if name == "pointsea" else None

    def fwd_bwd():
        for p in model.parameters():
            p.grad = None
        with _lib.fork(dev, lane=1, inputs=(gt,)) as br:
            gts = wl.gt_pyramid(gt)
        inp = wl.inputs(partial, gt, crop)
        depth = wl.images(inp)
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            pcds = model(inp, depth)
            loss = wl.loss(pcds, inp, gt, br.join(*gts))
        loss.backward()

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            fwd_bwd()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        fwd_bwd()
    dump_graph(g.raw_cuda_graph(), out)
    print(f"wrote {out}", flush=True)


class _KParams(ctypes.Structure):   # hipKernelNodeParams
    _fields_ = [("block", ctypes.c_uint * 3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p),
                ("grid", ctypes.c_uint * 3), ("kernelParams", ctypes.c_void_p), ("shmem", ctypes.c_uint)]


def dump_graph(graph, out):
    """Nodes (creation order: type, kernel name, grid) and edges of a hipGraph_t, through the HIP
    runtime torch loaded, as JSON."""
    import json

    import torch

    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipKernelNameRefByPtr.restype = ctypes.c_char_p
    hip.hipKernelNameRefByPtr.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipKernelNameRef.restype = ctypes.c_char_p
    hip.hipKernelNameRef.argtypes = [ctypes.c_void_p]
    gp = ctypes.c_void_p(graph)
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(gp, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(gp, nodes, ctypes.byref(n)) == 0
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(gp, None, None, ctypes.byref(ne)) == 0
    fr, to = (ctypes.c_void_p * ne.value)(), (ctypes.c_void_p * ne.value)()
    assert hip.hipGraphGetEdges(gp, fr, to, ctypes.byref(ne)) == 0
    index = {nodes[i]: i for i in range(n.value)}
    rows = []
    for i in range(n.value):
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nodes[i]), ctypes.byref(t))
        name, grid = None, None
        if t.value == 0:
            kp = _KParams()
            if hip.hipGraphKernelNodeGetParams(ctypes.c_void_p(nodes[i]), ctypes.byref(kp)) == 0:
                nm = hip.hipKernelNameRefByPtr(kp.func, None) or hip.hipKernelNameRef(kp.func)
                name = nm.decode(errors="replace") if nm else None
                grid = [kp.grid[0], kp.grid[1], kp.grid[2], kp.block[0]]
        rows.append({"i": i, "type": t.value, "name": name, "grid": grid})
    edges = [[index[fr[k]], index[to[k]]] for k in range(ne.value)]
    json.dump({"nodes": rows, "edges": edges}, open(out, "w"))


def parse(path, pat, depth=3):
    import json

    d = json.load(open(path))
    nodes, parents = d["nodes"], {}
    for a, b in d["edges"]:
        parents.setdefault(b, []).append(a)
    rx = re.compile(pat)
    hit = next((r["i"] for r in nodes if r["name"] and rx.search(r["name"])), None)
    print(f"{len(nodes)} nodes ({sum(r['type'] == 0 for r in nodes)} kernels), {len(d['edges'])} edges; "
          f"first match: node {hit}")
    if hit is None:
        return

    def short(i):
        r = nodes[i]
        nm = re.sub(r"\(.*", "", (r["name"] or f"type{r['type']}").replace("(anonymous namespace)::", "")
                    .replace("void ", ""))
        return f"#{i} {nm[:70]} {r['grid'] or ''}"

    def walk(i, dd):
        for p in parents.get(i, []):
            print("   " * (depth - dd + 1) + "<- " + short(p))
            if dd > 1:
                walk(p, dd - 1)

    print(short(hit))
    walk(hit, depth)


if __name__ == "__main__":
    if sys.argv[1] == "parse":
        parse(sys.argv[2], sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 3)
    else:
        capture(sys.argv[1], sys.argv[2])

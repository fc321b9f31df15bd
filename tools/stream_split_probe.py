"""Probe: the headline batch as two half-batches on two HIP streams in one process (each half its own
rasterize_core call; the backward of each half runs on its forward's stream), against one B=64 call.
Measures how much kernel concurrency the latency-bound raster kernels leave to gain.
usage (GPU box): python tools/stream_split_probe.py [steps]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
sys.argv = [sys.argv[0]]
args = bench.parse()
w = bench.workload(args, 0, dev)


def halves(nsplit):
    B = args.batch // nsplit
    out = []
    for h in range(nsplit):
        proj = w["proj"].detach()[h * B:(h + 1) * B].clone().requires_grad_(True)
        g = w["g"][h * B:(h + 1) * B].contiguous()
        tex = w["tex"].detach().clone().requires_grad_(True)
        p = w["params"]
        params = w["nr"].RasterizeParam(vertices_textures=p.vertices_textures[:B], faces_textures=p.faces_textures,
                                        textures=tex[None].expand(B, -1, -1, -1))
        out.append((proj, g, tex, params, torch.cuda.Stream()))
    return out


def run_split(hs):
    from neural_renderer_v2_pytorch_amd.rasterize import rasterize_core
    imgs = []
    cur = torch.cuda.current_stream()
    for proj, g, tex, params, st in hs:
        proj.grad = tex.grad = None
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            imgs.append(rasterize_core(proj, w["faces"], params, w["hp"]))
    torch.autograd.backward(imgs, [h[1] for h in hs])
    for h in hs:
        cur.wait_stream(h[4])


def timeit(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


t1 = timeit(lambda: bench.step(w), steps)
print("one call, B=%d: %.4f ms/step" % (args.batch, 1e3 * t1))
for ns in (2, 4):
    hs = halves(ns)
    t2 = timeit(lambda: run_split(hs), steps)
    print("%d streams x B=%d: %.4f ms/step (%.1f %% faster)" % (ns, args.batch // ns, 1e3 * t2, 100 * (t1 / t2 - 1)))

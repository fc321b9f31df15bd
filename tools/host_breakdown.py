"""Where the host's time per eager step goes (GPU box): the cfg2 teapot step (B=4, the config the
host's launch path bounds) and the headline step, each timed as a whole and in parts, with the GPU
kept out of the measurement by timing host enqueue over many steps (the GPU work of cfg2 is ~0.1 ms
per step, so the queue never fills).

usage: python tools/host_breakdown.py [steps]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench_configs  # noqa: E402
import neural_renderer_v2_pytorch_amd as nr  # noqa: E402
from neural_renderer_v2_pytorch_amd import _lib  # noqa: E402
from neural_renderer_v2_pytorch_amd import rasterize as nrr  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 400


def per_call_us(fn, n=N):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t = time.perf_counter() - t0
    torch.cuda.synchronize()
    tall = time.perf_counter() - t0
    return 1e6 * t / n, 1e6 * tall / n


def teapot():
    v, f = nr.load_obj(os.path.join(bench_configs.DATA, "teapot.obj"))
    B, s = 4, 256
    proj = bench_configs.scene(v, f, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32), device=dev)
    tex.requires_grad_(True)
    vt_d, ft_d = torch.as_tensor(vt, device=dev), torch.as_tensor(ft, device=dev)
    faces = torch.as_tensor(f, device=dev)
    g = torch.randn((B, 5, s, s), device=dev)
    return proj, tex, vt_d, ft_d, faces, g, B, s


def headline():
    """bench.py's headline workload (64 items, 5120 faces, 256^2): (proj, tex, vt, ft, faces, g, B, s)."""
    import bench
    sys.argv = [sys.argv[0]]
    w = bench.workload(bench.parse(), 0, dev)
    vt = w["params"]().vertices_textures[0]
    ft = w["params"]().faces_textures
    return w["proj"], w["tex"], vt, ft, w["faces"], w["g"], w["g"].shape[0], w["g"].shape[2]


def main():
    which = os.environ.get("HOST_WORKLOAD", "teapot")
    proj, tex, vt_d, ft_d, faces, g, B, s = headline() if which == "headline" else teapot()
    print("workload", which)
    out = {}

    def params():
        return nr.RasterizeParam(vertices_textures=vt_d[None].expand(B, -1, -1), faces_textures=ft_d,
                                 textures=tex[None].expand(B, -1, -1, -1))

    def step():
        proj.grad = tex.grad = None
        nr.rasterize_core(proj, faces, params(), nr.RasterizeHyperparam(image_size=s)).backward(g)

    def fwd_grad():
        nr.rasterize_core(proj, faces, params(), nr.RasterizeHyperparam(image_size=s))

    def fwd_nograd():
        with torch.no_grad():
            nr.rasterize_core(proj, faces, params(), nr.RasterizeHyperparam(image_size=s))

    x = torch.zeros(16, device=dev, requires_grad=True)

    def tiny_autograd():  # the engine's own cost: a one-op graph and its backward
        (x * 2).sum().backward()

    L = _lib.lib()

    def ctypes_call():
        L.nr_num_channels(7)

    def empties():
        for _ in range(8):
            torch.empty(1024, device=dev)

    def params_only():
        params()
        nr.RasterizeHyperparam(image_size=s)

    # time spent inside Rasterize.forward / backward (the backward runs on torch's autograd device
    # thread) and inside the library's launch calls, per step
    acc = {}

    def timed(name, fn):
        def w(*a, **k):
            t0 = time.perf_counter()
            r = fn(*a, **k)
            acc[name] = acc.get(name, 0.0) + time.perf_counter() - t0
            return r
        return w
    fwd0, bwd0 = nrr.Rasterize.forward, nrr.Rasterize.backward
    nrr.Rasterize.forward = staticmethod(timed("Rasterize.forward", fwd0))
    nrr.Rasterize.backward = staticmethod(timed("Rasterize.backward", bwd0))
    orig = {fname: getattr(L, fname) for fname in ("nr_rasterize_forward", "nr_rasterize_backward")}
    for fname, f0 in orig.items():
        setattr(L, fname, timed(fname, f0))
    core0 = nrr.rasterize_core
    nr.rasterize_core = timed("rasterize_core", core0)
    h, a = per_call_us(step)
    n = N + 20
    print("instrumented step: host %.1f us/call" % h)
    for k, v in sorted(acc.items()):
        print("  %-28s %8.1f us/step" % (k, 1e6 * v / n))
    nrr.Rasterize.forward, nrr.Rasterize.backward = staticmethod(fwd0), staticmethod(bwd0)
    nr.rasterize_core = core0
    for fname, f0 in orig.items():
        setattr(L, fname, f0)  # back to the configured function objects (argtypes / restype)

    for name, fn in [("step", step), ("forward (grad on)", fwd_grad), ("forward (no_grad)", fwd_nograd),
                     ("tiny autograd fwd+bwd", tiny_autograd), ("ctypes call", ctypes_call),
                     ("8 x torch.empty", empties), ("RasterizeParam + Hyperparam", params_only)]:
        h, a = per_call_us(fn)
        out[name] = (h, a)
        print("%-32s host %8.1f us/call   with GPU %8.1f us/call" % (name, h, a), flush=True)



    # the autograd engine hands a CUDA backward to its device thread and waits for it; with
    # multithreading off it runs the backward in the calling thread (a user-side setting)
    torch.autograd.set_multithreading_enabled(False)
    h, a = per_call_us(step)
    print("%-32s host %8.1f us/call   with GPU %8.1f us/call" % ("step (autograd single-thread)", h, a), flush=True)
    h, a = per_call_us(tiny_autograd)
    print("%-32s host %8.1f us/call   with GPU %8.1f us/call" % ("tiny autograd (single-thread)", h, a), flush=True)
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
    torch.autograd.set_multithreading_enabled(True)


if __name__ == "__main__":
    main()

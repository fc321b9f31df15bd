"""Time the single-GPU BASELINE.json configs other than the headline (bench.py measures that one):

  cfg2  teapot.obj (2464 faces) B=4 at 256^2 (AA, 512^2 internal), rgb + silhouettes + depth
  cfg3  ShapeNet car 4e49873... once midpoint-subdivided (14576 faces), B=64 at 256^2, textured rgba
        with the car's own texture atlas
  cfg5  example2-style loop: torus 250x100 (50000 faces) at 512^2 (1024^2 internal), silhouettes,
        200 fwd+bwd steps with an Adam update of the vertices

One step = rasterize_core forward + backward (cfg5: plus the Adam step), inputs resident on the GPU.
ms_per_step times --steps steps between two synchronisations after --warmup (bench.py's method: the
host enqueues a step while the GPU runs the previous one); synced_ms_per_step is the median with a
synchronisation after every step (host and GPU time in series).  Prints one JSON line per config.
cfg2 is also timed as a HIP-graph replay of the captured step (graph_ms_per_step): at B=4 the eager
step is bound by host launch overhead, not by the kernels.
cfg1 is the reference's CPU-only plumbing case and cfg4 is bench.py --gpus 8.

Each line carries a per-config roofline (algorithmic bytes per kernel and step with the config's real
texture size, HBM fraction per kernel and per step) and, with --pmc, each kernel's measured HBM
traffic and its ratio to the algorithmic bytes.

usage: python tools/bench_configs.py [--steps 50] [--warmup 30] [--loop-steps 200] [--pmc]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import neural_renderer_v2_pytorch_amd as nr  # noqa: E402
from neural_renderer_v2_pytorch_amd import synthetic  # noqa: E402

DATA = os.path.join(ROOT, "tests", "data")


subdivide = synthetic.subdivide  # (moved to the package: tests use it too)


def median_step(fn, steps, warmup):
    """Median of per-step times with a synchronisation after every step (a step's host enqueue and
    its GPU work in series)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def pipelined_step(fn, steps, warmup):
    """bench.py's timing: `steps` steps bracketed by synchronisations, so the host enqueues a step
    while the GPU runs the previous one (what a training loop without a per-step sync sees)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def kernels_ms(fn, n=10):
    """Per-kernel HIP-event durations recorded by the library (nr_profile_*, its ring of event pairs
    averaged) over n steps run back to back after 3 warm-up steps (bench.time_kernels)."""
    import ctypes
    from neural_renderer_v2_pytorch_amd import _lib
    names = ["k_tex_pack", "k_face_setup", "k_raster_fwd", "k_shade", "k_raster_bwd", "k_vertex_grad", "k_tex_out"]
    L = _lib.lib()
    _lib.check(L.nr_profile_enable(1), "nr_profile_enable")
    res = {}
    try:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        _lib.check(L.nr_profile_enable(1), "nr_profile_enable")
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        for k in names:
            ms = ctypes.c_float()
            if L.nr_profile_read(k.encode(), ctypes.byref(ms)) == 0:
                res[k] = round(float(ms.value), 5)
    finally:
        L.nr_profile_enable(0)
    return res


def graphed(step):
    """Capture one step in a HIP graph (torch.cuda.CUDAGraph) after a warm-up on a side stream and
    return its replay: the launch-bound small-batch steps then cost their kernels only."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step()
    return graph.replay


def scene(v, f, B, dev, seed=0):
    vb = torch.as_tensor(synthetic.jittered(v, B, seed_base=1000 + seed))
    eyes = torch.as_tensor(synthetic.viewpoints(B, seed_base=2000 + seed))
    return synthetic.project(vb.to(dev), eyes.to(dev)).contiguous().detach().requires_grad_(True)


def cfg2_step(dev):
    v, f = nr.load_obj(os.path.join(DATA, "teapot.obj"))
    B, s = 4, 256
    proj = scene(v, f, B, dev)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32), device=dev)
    tex.requires_grad_(True)
    vt_d, ft_d = torch.as_tensor(vt, device=dev), torch.as_tensor(ft, device=dev)
    faces = torch.as_tensor(f, device=dev)
    g = torch.randn((B, 5, s, s), device=dev)

    def step():
        proj.grad = tex.grad = None
        # params (the expand of the leaf texture) built per step: graph-capture safe (see graphed)
        params = nr.RasterizeParam(vertices_textures=vt_d[None].expand(B, -1, -1), faces_textures=ft_d,
                                   textures=tex[None].expand(B, -1, -1, -1))
        nr.rasterize_core(proj, faces, params, nr.RasterizeHyperparam(image_size=s)).backward(g)
    meta = dict(batch=B, image_size=s, C=5, V=int(v.shape[0]), F=int(f.shape[0]), tex_shape=tuple(tex.shape))
    return step, meta


def cfg2(dev, a):
    step, m = cfg2_step(dev)
    B, s = m["batch"], m["image_size"]
    t = pipelined_step(step, a.steps, a.warmup)
    ts = median_step(step, a.steps, a.warmup)
    # the same eager steps with the autograd engine in the calling thread (a user-side setting that
    # removes the engine's hand-over to its device thread; see bench.py)
    with torch.autograd.set_multithreading_enabled(False):
        t1 = pipelined_step(step, a.steps, a.warmup)
        t1s = median_step(step, a.steps, a.warmup)
    res = dict(config="cfg2 teapot B=4 256^2 rgb+sil+depth", faces=m["F"], batch=B, image_size=s,
               ms_per_step=round(t * 1e3, 4), mpx_per_s=round(B * s * s / t / 1e6, 1),
               synced_ms_per_step=round(ts * 1e3, 4),
               single_thread_autograd_ms_per_step=round(t1 * 1e3, 4),
               single_thread_autograd_synced_ms_per_step=round(t1s * 1e3, 4),
               kernels_ms=kernels_ms(step))
    tg = median_step(graphed(step), a.steps, a.warmup)
    res.update(graph_ms_per_step=round(tg * 1e3, 4), graph_mpx_per_s=round(B * s * s / tg / 1e6, 1))
    res["roofline"] = roofline(m, res["kernels_ms"], tg * 1e3, "graph_ms_per_step")
    return res


def cfg3_step(dev):
    """The car scene and its fwd+bwd step (also used by tools/fwd_timing.py --workload car)."""
    v, f, vt, ft, tex = nr.load_obj(os.path.join(DATA, "4e49873292196f02574b5684eaec43e9", "model.obj"),
                                    load_textures=True)
    v, f, vt, ft = subdivide(v, f, vt, ft)
    B, s = 64, 256
    proj = scene(v, f, B, dev)
    tex = torch.as_tensor(np.ascontiguousarray(tex), device=dev).float()
    if tex.shape[0] != 3:
        tex = tex.permute(2, 0, 1).contiguous()
    tex.requires_grad_(True)
    params = nr.RasterizeParam(vertices_textures=torch.as_tensor(vt, device=dev)[None].expand(B, -1, -1),
                               faces_textures=torch.as_tensor(ft, device=dev), textures=tex[None].expand(B, -1, -1, -1))
    faces = torch.as_tensor(f, device=dev)
    g = torch.randn((B, 4, s, s), device=dev)

    def step():
        proj.grad = tex.grad = None
        nr.rasterize_rgba(proj, faces, params, nr.RasterizeHyperparam(image_size=s)).backward(g)
    from neural_renderer_v2_pytorch_amd import rasterize as nrr
    # the shared texture windows the backward sums in private copies (k_hot_reduce, bytes in bench.kernel_bytes)
    num_hot = nrr._face_hot(params.faces_textures, params.vertices_textures[0], dev)[1]
    step.meta = dict(batch=B, image_size=s, C=4, V=int(v.shape[0]), F=int(f.shape[0]), tex_shape=tuple(tex.shape),
                     num_hot=num_hot)
    return step, f, B, s


def cfg3(dev, a):
    step, f, B, s = cfg3_step(dev)
    t = pipelined_step(step, a.steps, a.warmup)
    ts = median_step(step, a.steps, a.warmup)
    res = dict(config="cfg3 car (1x subdivided) B=64 256^2 textured rgba", faces=int(f.shape[0]), batch=B,
               image_size=s, ms_per_step=round(t * 1e3, 4), mpx_per_s=round(B * s * s / t / 1e6, 1),
               synced_ms_per_step=round(ts * 1e3, 4), kernels_ms=kernels_ms(step))
    res["roofline"] = roofline(step.meta, res["kernels_ms"], t * 1e3, "ms_per_step")
    return res


def cfg5_step(dev):
    v, f = synthetic.torus(250, 100)
    s = 512
    faces = torch.as_tensor(f, device=dev)
    ren = nr.Renderer()
    ren.image_size = s
    ren.viewpoints = nr.get_points_from_angles(2.732, 30, -15)
    with torch.no_grad():
        target = ren.render_silhouettes(torch.as_tensor(v[None] * 1.1, device=dev), faces)
    verts = torch.nn.Parameter(torch.as_tensor(v[None], device=dev))
    opt = torch.optim.Adam([verts], lr=0.001)

    def step():
        opt.zero_grad()
        loss = ((ren.render_silhouettes(verts, faces) - target) ** 2).sum()
        loss.backward()
        opt.step()
    step.meta = dict(batch=1, image_size=s, C=1, V=int(v.shape[0]), F=int(f.shape[0]), tex_shape=None)
    return step, v, f, s, faces, ren, target, verts


def cfg5(dev, a):
    step, v, f, s, faces, ren, target, verts = cfg5_step(dev)
    t = pipelined_step(step, a.steps, a.warmup)
    ts = median_step(step, a.steps, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.loop_steps):
        step()
    torch.cuda.synchronize()
    loop = time.perf_counter() - t0
    res = dict(config="cfg5 torus 50k faces, 512^2 (1024^2 internal) silhouettes, Renderer + Adam loop",
               faces=int(f.shape[0]), batch=1, image_size=s, ms_per_step=round(t * 1e3, 4),
               mpx_per_s=round(s * s / t / 1e6, 1), synced_ms_per_step=round(ts * 1e3, 4),
               loop_steps=a.loop_steps, loop_s=round(loop, 4),
               kernels_ms=kernels_ms(step))
    # the same loop as one captured HIP graph per step: device-resident viewpoint, capturable Adam
    ren.viewpoints = torch.as_tensor(ren.viewpoints, dtype=torch.float32, device=dev)
    optg = torch.optim.Adam([verts], lr=0.001, capturable=True)

    def stepg():
        loss = ((ren.render_silhouettes(verts, faces) - target) ** 2).sum()
        loss.backward()
        optg.step()
    optg.zero_grad(set_to_none=True)
    replay = graphed(stepg)
    tg = median_step(replay, a.steps, a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.loop_steps):
        replay()
    torch.cuda.synchronize()
    res.update(graph_ms_per_step=round(tg * 1e3, 4), graph_loop_s=round(time.perf_counter() - t0, 4))
    # the step's rasterizer part only (the Adam update, loss and camera are torch's / the camera kernels')
    res["roofline"] = roofline(step.meta, res["kernels_ms"], tg * 1e3, "graph_ms_per_step (incl. Adam, loss, camera)")
    return res


def roofline(meta, kms, step_ms, step_from):
    """Per-config roofline: each kernel's algorithmic (compulsory) HBM bytes per
    launch (bench.kernel_bytes, the formulas of DESIGN.md section 4, with this config's real texture
    size: the car's atlas is 3 x 1190 x 1920 f32 = 27.4 MB) over its HIP-event time, against the 8 TB/s
    HBM roof; and the whole step's bytes B(8S^2 + 8Cs^2 + 36V) + 24F + 2T over the step time."""
    import argparse
    import bench
    w = dict(C=meta["C"], V=meta["V"], F=meta["F"], tex_shape=meta["tex_shape"], num_hot=meta.get("num_hot", 0))
    args = argparse.Namespace(batch=meta["batch"], image_size=meta["image_size"])
    kb, total = bench.kernel_bytes(w, args, kms)
    per = {}
    for k, ms in kms.items():
        if k in kb:
            per[k] = dict(ms=ms, algorithmic_bytes=int(kb[k]),
                          frac=round(kb[k] / (ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 5))
    T = 0 if meta["tex_shape"] is None else 3 * meta["tex_shape"][1] * meta["tex_shape"][2] * 4
    return dict(peak_gbs=bench.HBM_PEAK_GBS, texture_bytes=T, kernels=per, step_algorithmic_bytes=int(total),
                step_ms=round(step_ms, 4), step_from=step_from,
                step_frac=round(total / (step_ms * 1e-3) / 1e9 / bench.HBM_PEAK_GBS, 5))


def pmc_child(name, steps=3):
    """One profiled pass (under rocprofv3 --pmc): `steps` steps of config `name`, then bench.py's 1 GiB
    calibration stream of known byte count (tools/pmc_traffic.py scales the counters with it)."""
    import bench
    dev = torch.device("cuda", 0)
    step = {"cfg2": lambda: cfg2_step(dev)[0], "cfg3": lambda: cfg3_step(dev)[0],
            "cfg5": lambda: cfg5_step(dev)[0]}[name]()
    for _ in range(steps + 1):
        step()
    torch.cuda.synchronize()
    bench.copy_ceiling_gbs(dev)
    torch.cuda.synchronize()


def pmc_traffic(name, timeout_s=240):
    """HBM bytes per launch of each kernel of config `name`: FETCH_SIZE and WRITE_SIZE, each in a
    rocprofv3 --pmc pass of its own over a child process (pmc_child), as bench.py's in-run passes."""
    import shutil
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic as pt
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    d = tempfile.mkdtemp(prefix="nr_cfg_pmc_")
    try:
        for i, counter in enumerate(("FETCH_SIZE", "WRITE_SIZE"), 1):
            cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", os.path.join(d, "p%d" % i), "-o", "run",
                   "--", sys.executable, os.path.abspath(__file__), "--pmc-child", name]
            subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=timeout_s, check=True,
                           cwd=ROOT, env=dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp")))
        # pmc_child runs steps + 1 = 4 steps: per-step bytes (a split forward launches k_raster_fwd twice)
        return pt.summarize(d, [name], verbose=False, steps=4)["hbm_bytes_per_step"]
    finally:
        shutil.rmtree(d, ignore_errors=True)


def config_step(name, dev):
    """(step, meta) of config `name`."""
    if name == "cfg2":
        return cfg2_step(dev)
    st = {"cfg3": cfg3_step, "cfg5": cfg5_step}[name](dev)[0]
    return st, st.meta


def count_child(name):
    """One step of config `name` through the counter build (NR_LIB_PATH = _lib/libnr_raster_count.so,
    set by the parent): prints that step's forward face-test counters (nr_count_read) as JSON."""
    import ctypes
    from neural_renderer_v2_pytorch_amd import _lib
    dev = torch.device("cuda", 0)
    step, _ = config_step(name, dev)
    L = _lib.lib()
    L.nr_count_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 4)()
    step()
    torch.cuda.synchronize()
    _lib.check(L.nr_count_read(out, 1), "nr_count_read")
    step()
    torch.cuda.synchronize()
    _lib.check(L.nr_count_read(out, 1), "nr_count_read")
    print(json.dumps({"tests": out[0], "walked": out[1], "commits": out[2], "walks": out[3]}), flush=True)


def face_tests(name, r, meta):
    """The forward's face-test rate of config `name` (bench.face_test_rate over a counter-build child)."""
    import bench
    counts, note = bench.face_test_counts([sys.executable, os.path.abspath(__file__), "--count-child", name])
    S = meta["image_size"] * 2
    return bench.face_test_rate(counts, note, meta["batch"], S, meta["F"], r["kernels_ms"]["k_raster_fwd"])


def main():
    p = argparse.ArgumentParser()
    # steady state (as bench.py: five warm-up steps left the GPU short of it, profiles/r05_warmup.txt)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--loop-steps", type=int, default=200)
    p.add_argument("--only", default="cfg2,cfg3,cfg5")
    p.add_argument("--calibrate", action="store_true",
                   help="end with bench.py's 1 GiB copy stream (the FETCH_SIZE / WRITE_SIZE calibration of "
                        "tools/pmc_traffic.py when this runs under rocprofv3 --pmc)")
    p.add_argument("--pmc", action="store_true",
                   help="add each config's PMC traffic per kernel (two rocprofv3 --pmc passes per config) and its "
                        "ratio to the algorithmic bytes")
    p.add_argument("--pmc-child", default=None, help=argparse.SUPPRESS)  # one profiled pass (internal)
    p.add_argument("--count-child", default=None, help=argparse.SUPPRESS)  # face-test counts (internal)
    p.add_argument("--no-count", action="store_true", help="skip the face-test counts (counter-build child)")
    a = p.parse_args()
    if a.pmc_child:
        return pmc_child(a.pmc_child)
    if a.count_child:
        return count_child(a.count_child)
    dev = torch.device("cuda", 0)
    for name in a.only.split(","):
        r = globals()[name](dev, a)
        # (not under rocprofv3: the counter-build child would inherit the profiler's preload)
        if not a.no_count and "k_raster_fwd" in r.get("kernels_ms", {}) and \
                not any(k.startswith("ROCPROF") for k in os.environ):
            meta = dict(batch=r["batch"], image_size=r["image_size"], F=r["faces"])
            ftr = face_tests(name, r, meta)
            r["fwd_face_tests_per_px"] = ftr.get("tests_per_px")
            r["fwd_gtests_per_s"] = ftr.get("gtests_per_s")
            r["face_test_rate"] = ftr
        if a.pmc:
            try:
                tr = pmc_traffic(name)
                for k, kr in r["roofline"]["kernels"].items():
                    if k in tr:
                        kr["traffic"] = tr[k]
                        kr["traffic_ratio"] = round(tr[k] / kr["algorithmic_bytes"], 3)
                r["roofline"]["traffic_source"] = "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, calibrated on a 1 GiB stream"
            except Exception as e:  # a profiler failure must not lose the timing line
                r["roofline"]["traffic_source"] = "pmc passes failed: %r" % (e,)
        print(json.dumps(r), flush=True)
    if a.calibrate:
        import bench
        torch.cuda.synchronize()
        print(json.dumps({"copy_ceiling_gbs": round(bench.copy_ceiling_gbs(dev), 1)}), flush=True)


if __name__ == "__main__":
    main()

"""Benchmark: rasterize fwd+bwd Mpixels/s at 256^2, batch 64 per GPU (BASELINE.json metric).

Workload (synthetic, no files): ico-sphere level 4 (V=2562, F=5120), per-item
vertex jitter and viewpoint, projected once outside the timed region; shared 4x4-per-face texture
atlas (create_textures, 3x288x288, U(0,1)) expanded over the batch; RasterizeHyperparam defaults
(anti-aliasing on -> 512^2 internal, draw_backside, rgb + silhouettes + depth -> C = 5).
One step = rasterize_core forward + backward with a fixed N(0,1) upstream gradient (the gradient
of (images * G).sum()), producing d/dvertices and d/dtextures.

Multi-GPU: one process per GPU, each renders its own 64 items (batch sharding, weak scaling, no
collective on the image data path).  The texture atlas is one parameter shared by every item of
every rank, so each timed step ends with the all_reduce(SUM) of its gradient over the ranks (SURVEY
section 8e; also timed on its own as allreduce_ms).  The timed region is bracketed by barriers and
the max over ranks is reported.  Under torchrun the ranks come from its environment; `bench.py --gpus N` started without
a launcher spawns the N rank processes itself (before any GPU call) and exits with their status.
The launched world size must equal --gpus (exit status 2 otherwise).  With N > 1 the rank images
are then all-gathered over RCCL (BASELINE cfg4: 512 items on 8 GPUs "with RCCL gather") and that
time is reported separately as gather_ms.

Output: one JSON line on rank 0 (see README/DESIGN for field meanings).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md "Chip-level parameters"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults: steady state (five warm-up steps left the GPU short of it: 20 timed steps then took
    # 0.380-0.385 ms each against 0.358-0.360 ms after 50, and 0.355 ms over 300; profiles/r05_warmup.txt)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--batch", type=int, default=64, help="items per GPU")
    p.add_argument("--image-size", type=int, default=256)
    p.add_argument("--level", type=int, default=4, help="ico-sphere subdivision level (4 -> 5120 faces)")
    p.add_argument("--mode", choices=["rgbsd", "sil"], default="rgbsd")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=30.0,
                   help="cap on the CPU baseline's timed work (it times the whole batch when that fits)")
    p.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                   help="gloo: rehearse the N > 1 path with ranks sharing GPUs (not for reported numbers)")
    p.add_argument("--graph-steps", type=int, default=0,
                   help="after the eager timing, time this many replays of the step captured in a HIP graph (0: skip)")
    p.add_argument("--no-gather", action="store_true",
                   help="with N > 1, skip the RCCL all_gather of the images timed after the steps (cfg4)")
    p.add_argument("--no-pmc", action="store_true",
                   help="skip the rocprofv3 --pmc passes that measure the roofline's HBM traffic and VALU share")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)  # one profiled pass (internal)
    p.add_argument("--count-child", action="store_true", help=argparse.SUPPRESS)  # face-test counts (internal)
    p.add_argument("--no-count", action="store_true", help="skip the face-test count (counter-build child)")
    return p.parse_args()


def under_profiler():
    """True when this process runs under rocprofv3 (its launcher exports ROCPROF_* settings to the
    profiled program).  A nested rocprofv3 started from here would inherit the outer profiler's
    preload and initialise the GPU before its own exec, so the in-run PMC passes are skipped."""
    return any(k.startswith("ROCPROF") for k in os.environ)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) and exit with the
    worst child status.  Runs before this process makes any GPU call: the parent only spawns and
    waits (a process that has initialised the GPU must not hand over to another program)."""
    import subprocess
    n = args.gpus
    if args.dist_backend == "nccl":
        ndev = torch.cuda.device_count()  # counts devices without initialising the GPU on this image
        if ndev < n:
            sys.stderr.write("bench.py: --gpus %d but %d GPU(s) visible; RCCL needs one GPU per rank "
                             "(use --dist-backend gloo to rehearse with shared GPUs)\n" % (n, ndev))
            return 2
    port = str(free_port())
    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(argv, env=env, cwd=ROOT))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    if bad:
        sys.stderr.write("bench.py: rank exit codes %s\n" % codes)
        return bad[0] if bad[0] > 0 else 1
    return 0


def check_world(args):
    """The launched world size must be the one asked for with --gpus (a torchrun with another
    --nproc-per-node, or a stray WORLD_SIZE, would otherwise report a different n_gpus)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.stderr.write("bench.py: --gpus %d but the launched world size is %d\n" % (args.gpus, world))
        sys.exit(2)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            # rehearsal of the multi-rank code path on a box with fewer GPUs than ranks: gloo, ranks
            # sharing devices (never used for reported numbers)
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", local if world > 1 else 0)


def workload(args, rank, dev):
    import neural_renderer_v2_pytorch_amd as nr
    from neural_renderer_v2_pytorch_amd import synthetic
    B = args.batch
    v, f = synthetic.icosphere(args.level)
    items = np.arange(rank * B, (rank + 1) * B)
    vb = np.stack([synthetic.jittered(v, 1, seed_base=1000 + int(i))[0] for i in items])
    eyes = np.stack([synthetic.viewpoints(1, seed_base=2000 + int(i))[0] for i in items])
    proj = synthetic.project(torch.as_tensor(vb, device=dev), torch.as_tensor(eyes, device=dev)).contiguous()
    proj = proj.detach().requires_grad_(True)
    faces = torch.as_tensor(f, device=dev)
    hp = nr.RasterizeHyperparam(image_size=args.image_size)
    if args.mode == "rgbsd":
        vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
        tex = np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32)
        tex = torch.as_tensor(tex, device=dev).requires_grad_(True)
        vt_d, ft_d = torch.as_tensor(vt, device=dev), torch.as_tensor(ft, device=dev)

        def params():
            # built per step, as a training loop does: a batch-expanded view of the leaf texture made
            # once would keep its autograd node alive across steps (and across a graph capture)
            return nr.RasterizeParam(vertices_textures=vt_d[None].expand(B, -1, -1), faces_textures=ft_d,
                                     textures=tex[None].expand(B, -1, -1, -1))
        C = 5
    else:
        params, tex, C = nr.RasterizeParam, None, 1
        hp.draw_rgb, hp.draw_depth = False, False
    g = torch.as_tensor(np.random.RandomState(7).normal(size=(B, C, args.image_size, args.image_size))
                        .astype(np.float32), device=dev)
    return dict(nr=nr, proj=proj, faces=faces, params=params, hp=hp, tex=tex, g=g, C=C, V=v.shape[0],
                F=f.shape[0], tex_shape=None if tex is None else tuple(tex.shape),
                # parameters every rank's items share: their gradient is summed over the ranks inside
                # the step; the projected vertices are per item, no exchange
                shared=[] if tex is None else [tex])


def step(w):
    """One step: rasterize_core forward + backward of this rank's items and, with more than one
    rank, the all_reduce(SUM) of the shared texture atlas's gradient (every item samples the same
    atlas, so its gradient is the reference's index_put_ scatter summed over the whole global batch,
    rasterize.py:144-148, utils.py:104-114; distributed.allreduce_shared_grads)."""
    from neural_renderer_v2_pytorch_amd.rasterize import rasterize_core
    from neural_renderer_v2_pytorch_amd import distributed
    w["proj"].grad = None
    if w["tex"] is not None:
        w["tex"].grad = None
    images = rasterize_core(w["proj"], w["faces"], w["params"](), w["hp"])
    images.backward(w["g"])
    if w["shared"]:
        distributed.allreduce_shared_grads(w["shared"])  # no-op without a process group of > 1 rank
    return images


def graphed(w):
    """The same step captured in one HIP graph (torch.cuda.CUDAGraph) after a warm-up on a side
    stream; returns its replay.  The replay launches the same kernels on the same buffers (the
    gradients land in the graph's own .grad tensors), without the host's per-launch path and with
    the graph's dispatch of consecutive kernels."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            step(w)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step(w)
    return graph


def kernel_bytes(w, args, measured=None):
    """Algorithmic (compulsory) HBM bytes per launch of each kernel (DESIGN.md "Kernels"): what the
    kernel must read and write at minimum, with stride-0 batch-expanded tensors counted once."""
    B, s, C, V, F = args.batch, args.image_size, w["C"], w["V"], w["F"]
    S = 2 * s
    rgb = w["tex_shape"] is not None
    T = 3 * w["tex_shape"][1] * w["tex_shape"][2] * 4 if rgb else 0
    fim, img, frec = 4 * S * S * B, 4 * C * s * s * B, 36 * F * B
    k = {
        "k_face_setup": 12 * V * B + 12 * F + frec + (24 * F + 12 * F if rgb else 0),
        "k_raster_fwd": frec + fim,
        "k_shade": fim + frec + (24 * F + T if rgb else 0) + img,
        "k_raster_bwd": fim + img + frec + (24 * F + T + T if rgb else 0) + frec,
        "k_vertex_grad": frec + 4 * (V + 1) + 12 * F + 12 * V * B,
        "k_tex_out": 4 * T // 3 + T,  # read the RGBA accumulator, write the planes
        "k_tex_pack": T + (4 * T // 3 if rgb else 0),  # read the planes, write RGBA rows
    }
    # the library carries the texture repacking in k_face_setup's idle threads when it is small
    # (DESIGN.md "Kernels"): its bytes then count to the carrying kernel
    if measured is not None:
        if "k_shade" not in measured:
            # shading fused into the forward (k_raster_fwd<256, true>): no fim read back
            k["k_raster_fwd"] += k.pop("k_shade") - fim
        if "k_tex_pack" not in measured:
            k["k_face_setup"] += k.pop("k_tex_pack")
        if rgb and "k_tex_out" not in measured and "k_vertex_grad" in measured:
            # the texture-gradient output carried by k_vertex_grad's blocks (small enough textures)
            k["k_vertex_grad"] += k.pop("k_tex_out")
    # shared texture windows (NrRasterArgs.face_hot, the car): k_hot_reduce, timed with k_raster_bwd,
    # reads the 32 private copies of each window (16 texels x 16 B) and adds 48 values into the
    # texture gradient; the backward's flushes write the copies (counted as its texture-gradient bytes)
    nh = w.get("num_hot", 0)
    if nh:
        k["k_raster_bwd"] += 32 * nh * 256 + nh * 48 * 4 * 2
    total = B * (8 * S * S + 8 * C * s * s + 36 * V) + 24 * F + (2 * T if T else 0)
    return k, total


KERNELS = ["k_tex_pack", "k_face_setup", "k_raster_fwd", "k_shade", "k_raster_bwd", "k_vertex_grad", "k_tex_out"]


def time_kernels(w, n=20):
    """Per-kernel durations from HIP events the library records on its launch stream around each
    launch (nr_profile_enable/read: a ring of event pairs per kernel, averaged), over n steps run back
    to back as in the timed loop, after 4 warm-up steps with the events on.  (Round 6: sampled one
    step at a time, with a synchronisation before each, the same kernels measured 5-7 % slower than in
    a rocprofv3 trace of a pipelined run on two boxes: the GPU idles for the host's enqueue time before
    every sampled step, and its memory side leaves its busy state, tools/warm_probe.py.)"""
    import ctypes
    from neural_renderer_v2_pytorch_amd import _lib
    L = _lib.lib()
    _lib.check(L.nr_profile_enable(1), "nr_profile_enable")
    res = {}
    try:
        for _ in range(4):
            step(w)
        torch.cuda.synchronize()
        _lib.check(L.nr_profile_enable(1), "nr_profile_enable")  # a new measurement: the n steps only
        t0 = time.perf_counter()
        for _ in range(n):
            step(w)
        torch.cuda.synchronize()
        res["_loop_ms_per_step"] = (time.perf_counter() - t0) / n * 1e3
        for k in KERNELS:
            ms = ctypes.c_float()
            if L.nr_profile_read(k.encode(), ctypes.byref(ms)) == 0:
                res[k] = float(ms.value)
    finally:
        L.nr_profile_enable(0)
    return res


def copy_ceiling_gbs(dev, nbytes=1 << 30, reps=10):
    """Achievable HBM stream rate on this box: a 1 GiB -> 1 GiB elementwise stream (16 B per lane
    loads and stores), read + write bytes.  tools/pmc_traffic.py also uses these launches, of known
    byte count, to calibrate the FETCH_SIZE / WRITE_SIZE counters."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    dst = torch.empty_like(src)
    torch.mul(src, 2.0, out=dst)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        torch.mul(src, 2.0, out=dst)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    return gbs


def host_cpu():
    """(model name, logical CPUs of the machine, CPUs this process may run on)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    return model, os.cpu_count() or 1, allowed


def cpu_baseline(args, budget_s):
    """The CPU oracle (C brute-force kernels with OpenMP + torch CPU stages of rasterize_core), timed
    on this host over the same workload's items, one at a time, until the whole batch is done or
    ~budget_s seconds have been spent.  Threads: every CPU this process may use, capped by the
    OMP_NUM_THREADS allotment when the environment sets one (the GPU box presets 16 host threads
    per GPU)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    import neural_renderer_v2_pytorch_amd as nr
    from neural_renderer_v2_pytorch_amd import synthetic
    model, ncpu, allowed = host_cpu()
    preset = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(allowed, preset) if preset > 0 else allowed
    torch.set_num_threads(threads)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    v, f = synthetic.icosphere(args.level)
    vt, ft, tex = nr.create_textures(f.shape[0], texture_size=4)
    tex = torch.as_tensor(np.random.RandomState(3).uniform(0, 1, tex.shape).astype(np.float32)).requires_grad_(True)
    C = 5 if args.mode == "rgbsd" else 1
    oracle.lib()
    done, t_total = 0, 0.0
    while t_total < budget_s and done < args.batch:
        vb = torch.as_tensor(synthetic.jittered(v, 1, seed_base=1000 + done))
        eye = torch.as_tensor(synthetic.viewpoints(1, seed_base=2000 + done))
        proj = synthetic.project(vb, eye).detach().requires_grad_(True)
        g = torch.as_tensor(np.random.RandomState(7).normal(size=(1, C, args.image_size, args.image_size))
                            .astype(np.float32))
        t0 = time.perf_counter()
        if args.mode == "rgbsd":
            img = oracle.rasterize_core(proj, f, image_size=args.image_size, vertices_textures=torch.as_tensor(vt)[None],
                                        faces_textures=ft, textures=tex[None])
        else:
            img = oracle.rasterize_core(proj, f, image_size=args.image_size, draw_rgb=False, draw_depth=False)
        img.backward(g)
        t_total += time.perf_counter() - t0
        done += 1
    mpx = done * args.image_size ** 2 / t_total / 1e6
    why = ("all %d CPUs this process may use" % threads if threads == allowed else
           "the OMP_NUM_THREADS=%d allotment of the %d CPUs this process may use" % (threads, allowed))
    # the brute-force scan is embarrassingly parallel over pixels, so the rate at every CPU of the
    # machine is at most linear in the thread count; stated, not run (the box allots 16 host
    # threads per GPU, and running 256 would take the other GPUs' share)
    at_nproc = None if threads >= ncpu else dict(
        value_upper_bound=mpx * ncpu / threads, threads=ncpu,
        how="linear extrapolation of the measured rate (an upper bound), not measured")
    return dict(value=mpx, unit="Mpixels/s", cores=threads, kind="port", cpu_model=model, nproc=ncpu,
                cpus_allowed=allowed, threads_why=why, at_nproc=at_nproc,
                sample="%d of the %d items of the headline batch (1 item = 256^2 output, 512^2 internal, %d faces, "
                       "fwd+bwd), %.1f s; oracle/nr_oracle.c brute force (OpenMP, %d threads) + torch-CPU stages"
                       % (done, args.batch, f.shape[0], t_total, threads))


PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",), ("SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "GRBM_GUI_ACTIVE"))
VALU_PEAK_INSTS = 1024 * 2.4e9 / 2  # wave64 VALU instructions/s: 1024 SIMD-32 at 2.4 GHz, 2 cycles each (MI355X_MICROARCH.md)


def pmc_passes(args, timeout_s=240):
    """The roofline's HBM traffic and VALU share, measured in this run: three rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE and the SQ/GRBM counters each in a pass of their own, as
    MI355X_MICROARCH.md's HBM section prescribes), each over a child process that runs 3 steps of
    the same workload plus the 1 GiB -> 1 GiB calibration stream; tools/pmc_traffic.py turns the
    counters into bytes per launch.  Returns (summary or None, note)."""
    import shutil
    import signal
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_traffic
    d = tempfile.mkdtemp(prefix="nr_pmc_")
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    # (the child runs warmup + steps = 4 steps: summarize's per-step traffic divides by that)
    child = [sys.executable, os.path.join(ROOT, "bench.py"), "--pmc-child", "--steps", "3", "--warmup", "1",
             "--batch", str(args.batch), "--image-size", str(args.image_size), "--level", str(args.level),
             "--mode", args.mode]
    try:
        for i, counters in enumerate(PMC_PASSES, 1):
            cmd = [prof, "--pmc", *counters, "--output-format", "csv", "-d", os.path.join(d, "p%d" % i), "-o", "run",
                   "--", *child]
            p = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env,
                                 start_new_session=True, cwd=ROOT)
            try:
                _, err = p.communicate(timeout=timeout_s)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait()
                return None, "pmc pass %d (%s) timed out" % (i, " ".join(counters))
            if p.returncode != 0:
                return None, "pmc pass %d exited %d: %s" % (i, p.returncode, err.decode(errors="replace")[-300:])
        return pmc_traffic.summarize(d, [args.batch, args.image_size, args.level, args.mode], verbose=False, steps=4), \
            "rocprofv3 --pmc, 3 passes in this run over 3 steps each; FETCH_SIZE/WRITE_SIZE calibrated on a 1 GiB stream"
    except Exception as e:  # a profiler failure must not lose the bench line
        return None, "pmc passes failed: %r" % (e,)
    finally:
        shutil.rmtree(d, ignore_errors=True)


def count_child(args):
    """One forward of the workload through the counter build (bench.py --count-child, NR_LIB_PATH =
    _lib/libnr_raster_count.so): prints the forward's face-test counters (nr_count_read) as JSON."""
    import ctypes
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    w = workload(args, 0, dev)
    from neural_renderer_v2_pytorch_amd import _lib
    from neural_renderer_v2_pytorch_amd.rasterize import rasterize_core
    L = _lib.lib()
    L.nr_count_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    out = (ctypes.c_ulonglong * 4)()
    step(w)  # warm-up (caches, layouts)
    torch.cuda.synchronize()
    _lib.check(L.nr_count_read(out, 1), "nr_count_read")
    with torch.no_grad():
        rasterize_core(w["proj"], w["faces"], w["params"](), w["hp"])
    torch.cuda.synchronize()
    _lib.check(L.nr_count_read(out, 1), "nr_count_read")
    print(json.dumps({"tests": out[0], "walked": out[1], "commits": out[2], "walks": out[3]}), flush=True)


def face_test_counts(child_args, timeout_s=180):
    """The forward's face tests, counted by the diagnostic build of the same kernels (-DNR_COUNT_TESTS,
    built by __graft_entry__.build beside the product library) over one forward of the workload in a
    child process.  Returns (counts or None, note)."""
    import subprocess
    lib = os.path.join(ROOT, "neural_renderer_v2_pytorch_amd", "_lib", "libnr_raster_count.so")
    if not os.path.exists(lib):
        return None, "counter build %s missing" % lib
    try:
        p = subprocess.run(child_args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout_s, cwd=ROOT,
                           env=dict(os.environ, NR_LIB_PATH=lib))
        if p.returncode != 0:
            return None, "count child exited %d: %s" % (p.returncode, p.stderr.decode(errors="replace")[-300:])
        return json.loads(p.stdout.decode().strip().splitlines()[-1]), "counter build (-DNR_COUNT_TESTS), one forward"
    except Exception as e:  # a failed count must not lose the bench line
        return None, "count child failed: %r" % (e,)


def face_test_rate(counts, note, B, S, F, fwd_ms):
    """SURVEY 8d's secondary bound in its own unit: the (pixel, face) pass tests the forward's walks
    evaluate per internal pixel and per second of the forward kernel, beside the reference's brute
    force (B S^2 F tests per call, rasterize_cuda_kernel.cu:82-149) over the same time."""
    px = B * S * S
    res = {"source": note, "internal_px": px, "brute_force_tests": px * F}
    if counts is None:
        return res
    t = fwd_ms * 1e-3
    res.update(tests=counts["tests"], tests_per_px=round(counts["tests"] / px, 3),
               gtests_per_s=round(counts["tests"] / t / 1e9, 1),
               brute_force_equivalent_gtests_per_s=round(px * F / t / 1e9, 1),
               tests_vs_brute_force=round(counts["tests"] / (px * F), 6),
               faces_walked_per_walk=round(counts["walked"] / max(counts["walks"], 1), 3),
               commit_batches_per_walk=round(counts["commits"] / max(counts["walks"], 1), 3),
               fwd_ms=round(fwd_ms, 5))
    return res


def pmc_child(args):
    """One profiled pass (bench.py --pmc-child under rocprofv3): the workload's steps, then the
    calibration stream of known byte count."""
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    w = workload(args, 0, dev)
    for _ in range(args.warmup + args.steps):
        step(w)
    torch.cuda.synchronize()
    copy_ceiling_gbs(dev)
    torch.cuda.synchronize()


def main():
    args = parse()
    if args.pmc_child:
        return pmc_child(args)
    if args.count_child:
        return count_child(args)
    if args.gpus < 1:
        sys.stderr.write("bench.py: --gpus must be >= 1\n")
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    check_world(args)
    world, rank, dev = setup_dist(args)
    w = workload(args, rank, dev)
    for _ in range(args.warmup):
        step(w)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        images = step(w)
    # host time to enqueue the steps (Python, autograd, ctypes, launches): below the GPU time, the
    # run is GPU-bound
    host_elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    px = world * args.batch * args.image_size ** 2 * args.steps
    value = px / elapsed / 1e6

    # the shared-gradient all_reduce that every timed step above includes, timed on its own (one
    # warm-up was the steps', then the best of 3, max over ranks), like gather_ms below
    allreduce_ms = None
    if world > 1 and w["shared"]:
        from neural_renderer_v2_pytorch_amd import distributed
        times = []
        for _ in range(3):
            torch.distributed.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            distributed.allreduce_shared_grads(w["shared"])
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t1) * 1e3)
        t = torch.tensor([min(times)], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        allreduce_ms = float(t.item())

    gather_ms = None
    if not args.no_gather and world > 1:
        out = torch.empty((world * images.shape[0],) + tuple(images.shape[1:]), device=dev, dtype=images.dtype)
        src = images.detach().contiguous()
        torch.distributed.all_gather_into_tensor(out, src)  # warm-up: RCCL sets up its channels lazily
        times = []
        for _ in range(3):
            torch.distributed.barrier()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            torch.distributed.all_gather_into_tensor(out, src)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t1) * 1e3)
        t = torch.tensor([min(times)], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        gather_ms = float(t.item())

    # the host's enqueue time per step with the autograd engine running the backward in the calling
    # thread (torch.autograd.set_multithreading_enabled(False), a user-side setting): by default the
    # engine hands a CUDA backward to its device thread and waits, which costs 50-110 us of host time
    # per step on these boxes (tools/host_breakdown.py).  Reported beside host_ms_per_step; the timed
    # steps above run with torch's defaults.
    torch.cuda.synchronize()
    with torch.autograd.set_multithreading_enabled(False):
        for _ in range(2):
            step(w)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(w)
        host_single = (time.perf_counter() - t1) / args.steps * 1e3
        torch.cuda.synchronize()

    # the host's own cost of enqueueing one step, with the GPU idle before each step (synchronised), so
    # that no launch could wait for queue space: a check on host_ms_per_step above, which is measured
    # inside the timed loop (the two agree on the boxes measured in round 6: the loop is not throttled
    # by the launch queue)
    host_idle = []
    for _ in range(10):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step(w)
        host_idle.append(time.perf_counter() - t1)
    torch.cuda.synchronize()
    host_idle_ms = float(np.median(host_idle)) * 1e3

    graph_ms = None
    if args.graph_steps > 0:
        images = images.detach()  # release the last eager step's autograd graph before the capture
        graph = graphed(w)
        for _ in range(args.warmup):
            graph.replay()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.graph_steps):
            graph.replay()
        torch.cuda.synchronize()
        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        ge = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([ge], device=dev, dtype=torch.float64)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            ge = float(t.item())
        graph_ms = ge / args.graph_steps * 1e3
        del graph

    del images
    kms = time_kernels(w)
    timing_loop_ms = kms.pop("_loop_ms_per_step", None)
    kb, total_bytes = kernel_bytes(w, args, kms)
    dominant = max(kms, key=kms.get)
    dom_ms, dom_bytes = kms[dominant], kb[dominant]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    ceiling = copy_ceiling_gbs(dev)

    # HBM traffic and VALU share of the dominant kernel, measured by rocprofv3 --pmc passes in this
    # run (rank 0 at N = 1, like the CPU baseline)
    pmc, pmc_note = None, "not measured (N > 1 or --no-pmc)"
    if world == 1 and rank == 0 and not args.no_pmc:
        if under_profiler():
            pmc_note = ("not measured: bench.py runs under rocprofv3 (ROCPROF_* in the environment); a nested "
                        "profiler pass would inherit the outer one's preload")
        else:
            pmc, pmc_note = pmc_passes(args)
    traffic = valu_busy = valu_insts = wait_share = None
    if pmc is not None:
        # per step (every launch of the kernel in a step; one for k_raster_bwd), like the algorithmic bytes
        traffic = pmc.get("hbm_bytes_per_step", pmc.get("hbm_bytes_per_launch", {})).get(dominant)
        valu_busy = pmc.get("valu_busy", {}).get(dominant)
        valu_insts = pmc.get("valu_insts", {}).get(dominant)
        wait_share = pmc.get("wait_any_share", {}).get(dominant)
    # the forward's face-test rate (SURVEY 8d's secondary bound), rank 0 at N = 1 like the PMC passes
    ftr = None
    # (not under rocprofv3: the child would inherit the profiler's preload, as the PMC passes would)
    if world == 1 and rank == 0 and not args.no_count and "k_raster_fwd" in kms and not under_profiler():
        counts, note = face_test_counts([sys.executable, os.path.join(ROOT, "bench.py"), "--count-child",
                                         "--batch", str(args.batch), "--image-size", str(args.image_size),
                                         "--level", str(args.level), "--mode", args.mode])
        ftr = face_test_rate(counts, note, args.batch, 2 * args.image_size, w["F"], kms["k_raster_fwd"])
    hbm_frac = achieved / HBM_PEAK_GBS
    valu = None
    if valu_insts is not None:
        rate = valu_insts / (dom_ms * 1e-3)
        valu = {"achieved": round(rate / 1e9, 2), "peak": round(VALU_PEAK_INSTS / 1e9, 1),
                "unit": "G wave64-VALU instructions/s", "frac": round(rate / VALU_PEAK_INSTS, 5),
                "busy_share": None if valu_busy is None else round(valu_busy, 4)}
    # the binding roof is the one the kernel comes closest to; with both well below 1 the kernel is
    # latency-bound (dependent memory round trips, barriers), which is stated in `limiter`
    fracs = {"hbm": hbm_frac}
    if valu is not None:
        fracs["valu"] = valu["frac"]
    closest = max(fracs, key=fracs.get)
    limiter = closest if fracs[closest] >= 0.6 else "latency"

    res = {
        "metric": "rasterize Mpixels/s fwd+bwd, 256² batch=64; % HBM roofline at 1 & 8 GPU",
        "value": round(value, 3),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (ico-sphere, jittered per item, random texture atlas)",
        "config": {"workload": "ico-sphere L%d (V=%d, F=%d), %d items/GPU, %d^2 output (AA, %d^2 internal), %s"
                               % (args.level, w["V"], w["F"], args.batch, args.image_size, 2 * args.image_size,
                                  "rgb+sil+depth" if args.mode == "rgbsd" else "silhouettes"),
                   "global_batch": world * args.batch, "image_size": args.image_size, "faces": w["F"],
                   "channels": w["C"], "parallelism": "batch-sharded dp%d" % world},
        "host_ms_per_step": round(host_elapsed / args.steps * 1e3, 4),
        "host_ms_per_step_idle_gpu": round(host_idle_ms, 4),
        "host_ms_per_step_autograd_single_thread": round(host_single, 4),
        # achieved / peak / frac are against the HBM roof (the contract's "bound"); the VALU roof beside
        # it, the closer of the two, and what limits the kernel
        "roofline": {"bound": "hbm", "closest_roof": closest, "kernel": dominant, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(hbm_frac, 5), "traffic": traffic,
                     "traffic_source": pmc_note, "algorithmic_bytes": dom_bytes, "avg_ms": round(dom_ms, 5),
                     "copy_ceiling_gbs": round(ceiling, 1),
                     # the second roof: VALU issue (SQ_INSTS_VALU over the HIP-event duration)
                     "valu": valu, "wait_share": None if wait_share is None else round(wait_share, 4),
                     # what limits the kernel: the closest roof when it is within reach (>= 0.6),
                     # otherwise latency
                     "limiter": limiter},
        "pmc_all_kernels": None if pmc is None else {
            k: {"traffic": pmc.get("hbm_bytes_per_step", pmc["hbm_bytes_per_launch"]).get(k),
                "valu_busy": round(pmc.get("valu_busy", {}).get(k, 0.0), 4),
                "wait_share": round(pmc.get("wait_any_share", {}).get(k, 0.0), 4)} for k in pmc["hbm_bytes_per_launch"]},
        "kernels_ms": {k: round(v, 5) for k, v in kms.items()},
        # the step time of the loop kernels_ms was measured over (its HIP events on), beside ms_per_step
        "kernels_ms_loop_ms_per_step": None if timing_loop_ms is None else round(timing_loop_ms, 4),
        # the forward's compute side in the contract's own unit: face tests per internal pixel and per
        # second (counter build), beside the brute force's B S^2 F
        "fwd_face_tests_per_px": None if ftr is None else ftr.get("tests_per_px"),
        "fwd_gtests_per_s": None if ftr is None else ftr.get("gtests_per_s"),
        "face_test_rate": ftr,
        "step_roofline_frac": round(total_bytes / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
    }
    if graph_ms is not None:
        # the same step replayed from a captured HIP graph (not the headline value)
        res["graph_ms_per_step"] = round(graph_ms, 4)
        res["graph_value"] = round(world * args.batch * args.image_size ** 2 / (graph_ms * 1e-3) / 1e6, 3)
    if allreduce_ms is not None:
        # inside every timed step (ms_per_step includes it); the bytes it sums per rank
        res["allreduce_ms"] = round(allreduce_ms, 4)
        res["allreduce_bytes"] = int(sum(p.numel() * p.element_size() for p in w["shared"]))
    if gather_ms is not None:
        res["gather_ms"] = round(gather_ms, 4)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()

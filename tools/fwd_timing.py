"""Per-wave phase timing of the forward k_raster_fwd on the headline workload (the fused <256, true>
variant) or the car (--workload car: the split forward, its deep launch at 1024 threads and the rest
at 256 on a side stream, each decoded with its own block size) (timing build, NR_FWD_TIMING).
usage (GPU box): python tools/fwd_timing.py [--workload car|cfg2] [extra -D flags...]
Phases: mask words + candidate scan, face staging rounds (summed), candidate expansion + face walk,
the wait at the barrier after each staging round's walks (static blocks: a wave that finished its
block waits for the round's slowest), fim write + bin flag + LDS hand-over, shading epilogue; split by
the bin's candidate count."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib_path = "/tmp/libnr_ftiming.so"
WORKLOAD = "headline"
if len(sys.argv) > 2 and sys.argv[1] == "--workload":
    WORKLOAD = sys.argv[2]
    del sys.argv[1:3]
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402  (the product's hipcc flags)
if os.environ.get("NR_FTIMING_LIB"):  # a timing build made beforehand (on the CPU host)
    lib_path = os.environ["NR_FTIMING_LIB"]
else:
    subprocess.check_call(["/opt/rocm/bin/hipcc", *__graft_entry__.hipcc_flags(), "-DNR_FWD_TIMING", "-I" + ROOT + "/include"]
                          + sys.argv[1:] + [ROOT + "/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip", "-o", lib_path])
os.environ["NR_LIB_PATH"] = lib_path
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

sys.argv = [sys.argv[0]]
torch.cuda.set_device(0)
if WORKLOAD == "car":
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs  # noqa: E402
    step, _, batch, size = bench_configs.cfg3_step(torch.device("cuda", 0))
    waves = 16  # deep bins: the 1024-thread variant
elif WORKLOAD == "cfg5":  # the 50k torus, one item at 1024^2 (deep-first, dealt quarters in its deep bins)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs  # noqa: E402
    step = bench_configs.cfg5_step(torch.device("cuda", 0))[0]
    batch, size, waves = 1, 512, 16
elif WORKLOAD == "cfg2":  # the teapot, B = 4 (the 1024-thread variant: small batches)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs  # noqa: E402
    step, meta = bench_configs.cfg2_step(torch.device("cuda", 0))
    batch, size, waves = meta["batch"], meta["image_size"], 16
else:
    args = bench.parse()
    w = bench.workload(args, 0, torch.device("cuda", 0))
    batch, size, waves = args.batch, args.image_size, 4

    def step():
        bench.step(w)
for _ in range(4):
    step()
torch.cuda.synchronize()
from neural_renderer_v2_pytorch_amd import _lib  # noqa: E402
L = _lib.lib()
S = 2 * size
nbins = (S // 32) ** 2
HALF = (1 << 22) // 2  # NR_FTIMING_MAX / 2: a split forward's second launch stamps the upper half
threads, flags = _lib.last_launch("k_raster_fwd")
split = bool(flags & _lib.NR_LAUNCH_SPLIT)
if not split:
    waves = threads // 64
buf = (ctypes.c_ulonglong * (2 * HALF))()
assert L.nr_debug_fwd_timing(buf, ctypes.c_size_t(2 * HALF)) == 0
raw = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)
if split:
    # part 1: the deep prefix at 1024 threads over a grid capped at Bcap items; part 2: the rest at 256
    bcap = max(8, (batch // 4 + 7) // 8 * 8)
    parts = [("deep launch (1024 threads)", raw[:nbins * bcap * 16 * 10].reshape(nbins * bcap, 16, 10)),
             ("rest launch (256 threads, side stream)", raw[HALF:HALF + nbins * batch * 4 * 10].reshape(nbins * batch, 4, 10))]
else:
    # (a deep-first forward that does not split launches 3 x 16 (NR_QS_CAP) quadrant blocks per list beyond its bins)
    nblk = nbins * batch + (3 * 16 * (8 if batch % 8 == 0 else 1) if flags & _lib.NR_LAUNCH_QUADRANTS else 0)
    parts = [("k_raster_fwd<%d>" % threads, raw[:nblk * waves * 10].reshape(nblk, waves, 10))]
# blocks past their launch's part of the deep-first list return before their first stamp
parts = [(lab, t[t[:, 0, 0] != 0]) for lab, t in parts]


def report(t):
    blocks = t.shape[0]
    nc = t[:, 0, 6]
    st = t[:, :, 2]  # cycles in the staging rounds (face loads + LDS stores + barrier), summed
    wt = t[:, :, 7]  # (static blocks) cycles at the barrier after each round's walks, summed
    ph = np.stack([t[:, :, 1] - t[:, :, 0], st, t[:, :, 3] - t[:, :, 1] - st - wt, wt,
                   t[:, :, 4] - t[:, :, 3], t[:, :, 5] - t[:, :, 4]], axis=2)
    names = ["scan", "stage", "walk", "walk-wait", "fim+flag", "shade"]
    life = t[:, :, 5] - t[:, :, 0]
    print("blocks %d; candidates per bin: zero in %.1f%%, mean %.1f over the rest" % (
        blocks, 100 * (nc == 0).mean(), nc[nc > 0].mean() if (nc > 0).any() else 0))
    ncb = nc
    if (ncb > 0).any():
        print("candidates per non-empty bin p50/p90/p99/max: %s; over 160: %.1f%%, over 512: %.1f%%" % (
            np.percentile(ncb[ncb > 0], [50, 90, 99, 100]).astype(int), 100 * (ncb > 160).mean() / max((ncb > 0).mean(), 1e-9),
            100 * (ncb > 512).mean() / max((ncb > 0).mean(), 1e-9)))
    for lo, hi, lab in ((0, 0, "no candidates"), (1, 10**9, "with candidates")):
        sel = (nc >= lo) & (nc <= hi)
        if not sel.any():
            continue
        print("%s: %d bins, wave lifetime mean %.0f" % (lab, sel.sum(), life[sel].mean()))
        for i, nm in enumerate(names):
            x = ph[sel][:, :, i].ravel()
            print("   %-9s mean %8.0f  p50 %8.0f  p90 %8.0f" % (nm, x.mean(), *np.percentile(x, [50, 90])))
    # where the launch's wave time goes, by the bin's candidate count: share of the summed wave
    # lifetimes (what the chip spends), and the walk's mean per wave
    tot = life.sum()
    print("wave-time share by candidates per bin (and walk mean per wave):")
    for lo, hi in ((0, 0), (1, 64), (65, 160), (161, 512), (513, 2048), (2049, 10**9)):
        sel = (nc >= lo) & (nc <= hi)
        if sel.any():
            print("   %5d-%-9d bins %6d  time share %5.1f%%  walk mean %9.0f  lifetime mean %9.0f" % (
                lo, min(hi, 10**6), sel.sum(), 100 * life[sel].sum() / tot, ph[sel][:, :, 2].mean(), life[sel].mean()))


for lab, t in parts:
    print("== %s" % lab)
    report(t)
# timeline from the chip-wide wall clock (100 MHz): when the bins of each depth class start and end,
# relative to the forward's first wave (over both launches of a split forward)
t0 = min(t[:, :, 8].min() for _, t in parts)
span = (max(t[:, :, 9].max() for _, t in parts) - t0) / 100.0
print("forward span %.1f us (wall clock)" % span)
for lab, t in parts:
    nc = t[:, 0, 6]
    ws_, we_ = t[:, :, 8].min(1), t[:, :, 9].max(1)
    print("  %s: start %.1f end %.1f us" % (lab, (ws_.min() - t0) / 100.0, (we_.max() - t0) / 100.0))
    for lo, hi in ((0, 0), (1, 160), (161, 512), (513, 2048), (2049, 10**9)):
        sel = (nc >= lo) & (nc <= hi)
        if sel.any():
            st_, en_ = (ws_[sel] - t0) / 100.0, (we_[sel] - t0) / 100.0
            print("   %5d-%-9d start mean %7.1f max %7.1f us   end mean %7.1f max %7.1f us   duration mean %6.1f max %6.1f us" % (
                lo, min(hi, 10**6), st_.mean(), st_.max(), en_.mean(), en_.max(), (en_ - st_).mean(), (en_ - st_).max()))

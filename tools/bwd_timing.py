"""Per-wave phase timing of k_raster_bwd on the headline workload or the car (--workload car, BASELINE
cfg3) (timing build, NR_BWD_TIMING).

usage (GPU box): python tools/bwd_timing.py [--workload car] [extra -D flags...]
(NR_BTIMING_LIB=<path>: a timing build made beforehand, -DNR_BWD_TIMING, instead of building here)
Builds the library with -DNR_BWD_TIMING into /tmp, runs bench.py's headline step through it, reads
the per-wave shader-clock stamps of the last backward (nr_debug_bwd_timing) and prints the mean and
percentiles of each phase: step 1 (recompute + staging of I and G), barrier 1, stencil, barrier 2,
record staging + grouping, per-face gather + atomics, and the whole wave lifetime."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib_path = "/tmp/libnr_timing.so"
WORKLOAD = "headline"
if len(sys.argv) > 2 and sys.argv[1] == "--workload":
    WORKLOAD = sys.argv[2]
    del sys.argv[1:3]
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402  (the product's hipcc flags)
if os.environ.get("NR_BTIMING_LIB"):  # a timing build made beforehand (on the CPU host)
    lib_path = os.environ["NR_BTIMING_LIB"]
else:
    subprocess.check_call(["/opt/rocm/bin/hipcc", *__graft_entry__.hipcc_flags(), "-DNR_BWD_TIMING", "-I" + ROOT + "/include"]
                          + sys.argv[1:] + [ROOT + "/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip", "-o", lib_path])
os.environ["NR_LIB_PATH"] = lib_path
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

sys.argv = [sys.argv[0]]
torch.cuda.set_device(0)
if WORKLOAD == "car":  # BASELINE cfg3 (tools/bench_configs.py)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_configs  # noqa: E402
    step, _, batch, size = bench_configs.cfg3_step(torch.device("cuda", 0))
else:
    args = bench.parse()
    w = bench.workload(args, 0, torch.device("cuda", 0))
    batch, size = args.batch, args.image_size

    def step():
        bench.step(w)
for _ in range(4):
    step()
torch.cuda.synchronize()
from neural_renderer_v2_pytorch_amd import _lib  # noqa: E402
L = _lib.lib()
S = 2 * size
blocks = (S // 32) * (S // 16) * batch
n = blocks * 4 * 10
buf = (ctypes.c_ulonglong * n)()
assert L.nr_debug_bwd_timing(buf, ctypes.c_size_t(n)) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(blocks, 4, 10)
names = ["step1", "barrier1", "stencil", "barrier2", "stage+group", "gather+atomics"]
d = np.diff(t[:, :, :7], axis=2)
life = t[:, :, 6] - t[:, :, 0]
print("waves %d, kernel span %.0f clocks" % (blocks * 4, t[:, :, 6].max() - t[:, :, 0].min()))
for i, nm in enumerate(names):
    x = d[:, :, i].ravel()
    print("%-16s mean %8.0f  p10 %8.0f  p50 %8.0f  p90 %8.0f  share %.3f" % (
        nm, x.mean(), *np.percentile(x, [10, 50, 90]), x.mean() / life.mean()))
print("%-16s mean %8.0f  p10 %8.0f  p50 %8.0f  p90 %8.0f" % ("lifetime", life.mean(), *np.percentile(life, [10, 50, 90])))
nf = t[:, :, 7].ravel()
print("faces per wave: mean %.2f p10/p50/p90 %s max %d" % (nf.mean(), np.percentile(nf, [10, 50, 90]), nf.max()))
for k in (1, 2, 3, 4, 6, 8):
    sel = (t[:, :, 7] == k)
    if sel.any():
        print("  %d faces: %6d waves, gather mean %7.0f p50 %7.0f, lifetime mean %7.0f" % (
            k, sel.sum(), d[:, :, 5][sel].mean(), np.median(d[:, :, 5][sel]), life[sel].mean()))
starts = np.sort(t[:, :, 0].min(axis=1) - t[:, :, 0].min())
print("block start times (clocks) p10/p50/p90: %s" % np.percentile(starts, [10, 50, 90]).round())
# SIMD slots a block holds idle: its four waves share the block's LDS until the last one ends, so a
# wave that ends early leaves its slot empty for (block end - wave end)
fg = life.max(axis=1) > 0
end = t[fg][:, :, 6]
bend = end.max(axis=1, keepdims=True)
start = t[fg][:, :, 0]
held = (bend - start).sum()
idle = (bend - end).sum()
print("foreground blocks %d: slot time idle after a wave's end %.3f of the time the block holds its slots"
      % (fg.sum(), idle / held))

# timeline from the chip-wide wall clock (100 MHz), per block: when the foreground (not skipped) and the
# skipped tiles start and end relative to the kernel's first wave
ws_, we_ = t[:, :, 8].min(axis=1), t[:, :, 9].max(axis=1)
t0 = ws_.min()
print("kernel span %.1f us (wall clock)" % ((we_.max() - t0) / 100.0))
for lab, sel in (("skipped tiles", ~fg), ("foreground tiles", fg)):
    if sel.any():
        st_, en_ = (ws_[sel] - t0) / 100.0, (we_[sel] - t0) / 100.0
        print("   %-17s %6d blocks  start mean %7.1f max %7.1f us   end mean %7.1f max %7.1f us   duration mean %6.1f max %6.1f us" % (
            lab, sel.sum(), st_.mean(), st_.max(), en_.mean(), en_.max(), (en_ - st_).mean(), (en_ - st_).max()))

"""Per-wave phase timing of the fused forward k_raster_fwd<256, true> on the headline workload
(timing build, NR_FWD_TIMING).  usage (GPU box): python tools/fwd_timing.py [extra -D flags...]
Phases: mask words + candidate scan, candidate expansion + face staging, face walk, fim write + bin
flag + LDS hand-over, shading epilogue; split by the bin's candidate count."""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib_path = "/tmp/libnr_ftiming.so"
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                       "-ffp-contract=off", "-fno-fast-math", "-fvisibility=hidden", "-DNR_FWD_TIMING", "-I" + ROOT + "/include"]
                      + sys.argv[1:] + [ROOT + "/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip", "-o", lib_path])
os.environ["NR_LIB_PATH"] = lib_path
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402

sys.argv = [sys.argv[0]]
args = bench.parse()
torch.cuda.set_device(0)
w = bench.workload(args, 0, torch.device("cuda", 0))
for _ in range(4):
    bench.step(w)
torch.cuda.synchronize()
from neural_renderer_v2_pytorch_amd import _lib  # noqa: E402
L = _lib.lib()
S = 2 * args.image_size
blocks = (S // 32) ** 2 * args.batch
n = blocks * 4 * 8
buf = (ctypes.c_ulonglong * n)()
assert L.nr_debug_fwd_timing(buf, ctypes.c_size_t(n)) == 0
t = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(blocks, 4, 8)
nc = t[:, 0, 6]
t2 = np.where((nc > 0)[:, None], t[:, :, 2], t[:, :, 1])  # no staging stamp without candidates
ph = np.stack([t[:, :, 1] - t[:, :, 0], t2 - t[:, :, 1], t[:, :, 3] - t2,
               t[:, :, 4] - t[:, :, 3], t[:, :, 5] - t[:, :, 4]], axis=2)
names = ["scan", "stage", "walk", "fim+flag", "shade"]
life = t[:, :, 5] - t[:, :, 0]
print("blocks %d; candidates per bin: zero in %.1f%%, mean %.1f over the rest" % (blocks, 100 * (nc == 0).mean(), nc[nc > 0].mean()))
for lo, hi, lab in ((0, 0, "no candidates"), (1, 10**9, "with candidates")):
    sel = (nc >= lo) & (nc <= hi)
    if not sel.any():
        continue
    print("%s: %d bins, wave lifetime mean %.0f" % (lab, sel.sum(), life[sel].mean()))
    for i, nm in enumerate(names):
        x = ph[sel][:, :, i].ravel()
        print("   %-9s mean %8.0f  p50 %8.0f  p90 %8.0f" % (nm, x.mean(), *np.percentile(x, [50, 90])))

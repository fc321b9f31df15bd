"""Debug count (NR_COUNT_DIRECT build) of the car backward's texture samples: inside their face's 4x4
texel window (gathered per face) or outside it (direct texel atomics).  usage (GPU box):
python tools/count_direct.py"""
import ctypes, os, subprocess, sys
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
lib = "/tmp/libnr_count.so"
sys.path.insert(0, ROOT)
import __graft_entry__  # the product's hipcc flags
subprocess.check_call(["/opt/rocm/bin/hipcc", *__graft_entry__.hipcc_flags(), "-DNR_COUNT_DIRECT", "-I" + ROOT + "/include",
                       ROOT + "/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip", "-o", lib])
os.environ["NR_LIB_PATH"] = lib
sys.path.insert(0, ROOT); sys.path.insert(0, ROOT + "/tools")
import torch, bench_configs
step, f, B, s = bench_configs.cfg3_step(torch.device("cuda", 0))
from neural_renderer_v2_pytorch_amd import _lib
L = _lib.lib()
step(); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 4)()
L.nr_debug_counts(buf)
print("after 1 step: windowed %d direct %d direct-without-window %d; direct whose top-left texel a lower lane of the "
      "wave (same pixel row k) also samples directly: %d" % (buf[0], buf[1], buf[2], buf[3]))

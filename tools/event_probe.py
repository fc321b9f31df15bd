"""Does timing the kernels with the library's HIP events change the step?  One process: 50 warm-up
headline steps, then blocks of 20 back-to-back steps alternately without and with profiling on
(nr_profile_enable: each kernel's launch stamped through hipExtLaunchKernel's events), printing each
block's wall time per step and, for the profiled blocks, the per-kernel event means and their sum.

usage: python tools/event_probe.py
"""
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from neural_renderer_v2_pytorch_amd import _lib  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    w = bench.workload(args, 0, dev)
    L = _lib.lib()
    for _ in range(50):
        bench.step(w)
    torch.cuda.synchronize()
    out = []
    for rep in range(3):
        for prof in (False, True):
            _lib.check(L.nr_profile_enable(1 if prof else 0), "nr_profile_enable")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                bench.step(w)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 20 * 1e3
            rec = {"profiled": prof, "ms_per_step": round(ms, 4)}
            if prof:
                kms = {}
                for k in ("k_face_setup", "k_raster_fwd", "k_raster_bwd", "k_vertex_grad"):
                    v = ctypes.c_float()
                    if L.nr_profile_read(k.encode(), ctypes.byref(v)) == 0:
                        kms[k] = round(v.value, 5)
                rec["kernels_ms"] = kms
                rec["kernel_sum_ms"] = round(sum(kms.values()), 4)
            out.append(rec)
    _lib.check(L.nr_profile_enable(0), "nr_profile_enable")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

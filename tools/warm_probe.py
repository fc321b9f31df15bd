"""Why the first ~50 headline steps of a process run ~7 % slower than later ones (profiles/r05_warmup.txt):
one process times consecutive blocks of 20 steps (bench.py's step and workload), then blocks after an
idle pause and after unrelated GPU work, so that a clock ramp (it comes back after idling and is cut
short by any GPU load) can be told from a one-time cost of the process (it does neither).

usage: python tools/warm_probe.py
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def block(w, k=20):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        bench.step(w)
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / k * 1e3, 4)


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    w = bench.workload(args, 0, dev)
    out = {}
    for _ in range(5):
        bench.step(w)
    out["blocks_after_w5"] = [block(w) for _ in range(6)]
    # the host's enqueue time of each step of a 40-step pipelined block (no synchronisation inside):
    # flat if the host cost is all there is, rising once the runtime's launch queue is full
    torch.cuda.synchronize()
    enq = []
    for _ in range(40):
        t0 = time.perf_counter()
        bench.step(w)
        enq.append(round((time.perf_counter() - t0) * 1e3, 4))
    torch.cuda.synchronize()
    out["enqueue_ms_per_step_pipelined"] = enq
    time.sleep(0.5)
    out["after_idle_0.5s"] = [block(w) for _ in range(3)]
    time.sleep(2.0)
    out["after_idle_2s"] = [block(w) for _ in range(3)]
    time.sleep(2.0)
    a = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.03:  # 30 ms of unrelated GPU work (f32 GEMMs)
        a = (a @ a).clamp_(-1, 1)
        torch.cuda.synchronize()
    out["after_idle_2s_then_30ms_gemm"] = [block(w) for _ in range(3)]
    time.sleep(2.0)
    b = torch.empty(1 << 28, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.03:  # 30 ms of a 1 GiB fill (memory-bound)
        b.fill_(1.0)
        torch.cuda.synchronize()
    out["after_idle_2s_then_30ms_fill"] = [block(w) for _ in range(3)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""bench.py's multi-rank launch (BASELINE cfg4 / the 1-2-4-8 GPU metric).

`python3 bench.py --gpus N` started without a launcher spawns the N rank processes itself, before
any GPU call, and a launched world size that differs from --gpus is an error (exit status 2).  The
GPU test runs the real command line with two gloo ranks sharing the box's one GPU; the CPU test
checks the world-size guard, which fires before anything touches a GPU.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                            "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_world_size_mismatch_exits_nonzero():
    """A torchrun-style environment with WORLD_SIZE=2 and --gpus 4: exit status 2 and a message,
    no bench line."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "1"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 2, (p.returncode, p.stderr[-500:])
    assert "launched world size is 2" in p.stderr
    assert "{" not in p.stdout


@pytest.mark.gpu
def test_bench_cli_two_ranks_gloo():
    """`bench.py --gpus 2 --dist-backend gloo` on the one-GPU box: the script launches its two
    ranks, each renders its own 64 headline items, and rank 0 prints one line with n_gpus = 2,
    global_batch = 128 and the all-gather time of the rank images."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--steps", "3", "--warmup", "1", "--no-pmc", "--no-cpu-baseline"]
    p = subprocess.run(cmd, env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (p.returncode, p.stderr[-2000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2
    assert res["config"]["global_batch"] == 128
    assert res["config"]["parallelism"] == "batch-sharded dp2"
    assert res["gather_ms"] is not None and res["gather_ms"] > 0
    # the shared texture gradient's all_reduce is part of every timed step, and timed on its own
    assert res["allreduce_ms"] is not None and res["allreduce_ms"] > 0
    assert res["allreduce_bytes"] == 3 * 288 * 288 * 4
    assert res["value"] > 0 and res["steps"] == 3


@pytest.mark.gpu
def test_face_test_count_child():
    """The forward's face-test counters (the -DNR_COUNT_TESTS build, bench.py's face-test rate, SURVEY
    8d's secondary bound) through bench.py's own child: a forward of 8 ico-sphere items (level 3,
    1280 faces) at 256^2 internal counts a positive number of (pixel, face) pass tests, 64 per face a
    wave walks over an 8x8 block (no bin here is deep enough for 4x4 quarters), far below the brute
    force's B S^2 F."""
    sys.path.insert(0, ROOT)
    import bench
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--count-child", "--batch", "8", "--level", "3",
           "--image-size", "128"]
    counts, note = bench.face_test_counts(cmd, timeout_s=150)
    assert counts is not None, note
    B, S, F = 8, 256, 1280
    assert counts["tests"] > 0 and counts["tests"] == 64 * counts["walked"]
    assert counts["walks"] > 0 and counts["commits"] > 0
    assert counts["tests"] < B * S * S * F // 100
    r = bench.face_test_rate(counts, note, B, S, F, 0.01)
    assert r["tests_per_px"] == round(counts["tests"] / (B * S * S), 3)
    assert r["brute_force_tests"] == B * S * S * F

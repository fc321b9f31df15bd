"""Build recipe for the CPU oracle (test infrastructure only).

Compiles oracle/nr_oracle.c with gcc into oracle/_build/libnr_oracle.so.  The flags matter
for parity: -ffp-contract=off (the reference kernel is restated with no fused multiply-add)
and no -ffast-math (IEEE division and comparisons).  OpenMP parallelises over pixels.

The reference's own native code (neural_renderer_torch/cuda/*.cu, *.cpp) needs nvcc and
ATen's CUDA headers and is therefore unbuildable in this image; no oracle/_ref is produced
("Oracle").
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "nr_oracle.c")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libnr_oracle.so")

CFLAGS = ["-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-fPIC", "-shared",
          "-fvisibility=hidden", "-Wall"]


def build(force=False, verbose=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    if (not force and os.path.exists(LIB)
            and os.path.getmtime(LIB) >= os.path.getmtime(SRC)):
        return LIB
    cmd = ["gcc", *CFLAGS, SRC, "-o", LIB + ".tmp", "-lm"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True, verbose=True))

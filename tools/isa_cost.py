"""Static VALU cost of the raster kernels (CPU only, no GPU): compiles nr_raster.hip to gfx950 assembly
with the product's flags (plus any extra -D / -f flags given) and prints, per kernel instantiation,
the register budget (VGPRs, spills, scratch, LDS) and a weighted count of the vector instructions in
each barrier-delimited segment.

Weights (MI355X_MICROARCH.md, "Execution model" and the constants table): a wave64 VALU instruction
issues over 2 cycles on a SIMD-32; packed f32 (v_pk_fma/mul/add_f32) does two lanes' worth per lane
in 4 (the same f32 rate as two scalar instructions); transcendentals (v_rcp, v_exp, ...) and 32-bit
integer multiplies (v_mul_lo_u32, v_mad_u64_u32, ...) 8.  Moves
count like any VALU instruction.  The count is static (every branch once, slow paths included), so it
compares builds of the same source rather than predicting time; since the raster kernels issue-bound
their foreground waves, a lower count on the hot path has so far always measured faster.

usage: python tools/isa_cost.py [-DFOO ...] [-fno-...]   (default kernels: the headline's)
       KERNELS="k_raster_bwdILi0ELi2ELi5E,k_raster_fwdILi256ELb1ELi5E" python tools/isa_cost.py
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__  # noqa: E402

KERNELS = os.environ.get("KERNELS", "k_raster_bwdILi0ELi2ELi5E,k_raster_fwdILi256ELb1ELi5E").split(",")


def compile_asm(extra):
    out = os.path.join(tempfile.mkdtemp(), "nr.s")
    flags = [f for f in __graft_entry__.hipcc_flags() if f not in ("-shared", "-fPIC")]
    subprocess.check_call(["/opt/rocm/bin/hipcc", *flags, *extra, "-I" + os.path.join(ROOT, "include"),
                           "--cuda-device-only", "-S", __graft_entry__.SRC, "-o", out],
                          stderr=subprocess.DEVNULL)
    return open(out).read()


def kernel_body(lines, pat):
    start = [i for i, ln in enumerate(lines) if re.match(pat, ln)][0]
    end, j = start, start + 1
    while j < len(lines) and not re.match(r"^_Z\w+:", lines[j]):
        if lines[j].strip().startswith("s_endpgm"):
            end = j
        j += 1
    return lines[start].split(":")[0], lines[start:end]


def metadata(asm, name):
    for blk in asm.split("  - .agpr_count")[1:]:
        if re.search(r"\.name:\s+" + re.escape(name) + r"\n", blk):
            g = lambda k: int(re.search(r"\." + k + r":\s+(\d+)", blk).group(1))  # noqa: E731
            return dict(vgpr=g("vgpr_count"), vgpr_spill=g("vgpr_spill_count"), sgpr_spill=g("sgpr_spill_count"),
                        lds=g("group_segment_fixed_size"), scratch=g("private_segment_fixed_size"))
    return {}


def weight(op):
    if op.startswith("v_pk_") and "mov" not in op:
        return 4
    if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", op) or re.match(r"v_(mul_lo|mul_hi|mad_u64|mad_i64)_", op):
        return 8  # transcendental and 32-bit integer multiplies: quarter rate
    return 2


def cost(body):
    c = n = moves = 0
    for ln in body:
        m = re.match(r"\s+(v_\w+)", ln)
        if m:
            op = m.group(1)
            c += weight(op)
            n += 1
            moves += op.startswith(("v_mov", "v_pk_mov"))
    return c, n, moves


def fast_path(body):
    """The body without the basic blocks that hold an IEEE division (v_div_scale): those are the
    guarded slow paths of the exact shortened divisions, skipped when every lane's operands are in
    range (the headline's case)."""
    out, blk = [], []
    for ln in body:
        ins = ln.strip()
        if ins.startswith((".LBB", "s_cbranch", "s_branch")):
            if not any("v_div_scale" in x for x in blk):
                out += blk
            blk = []
        else:
            blk.append(ln)
    if not any("v_div_scale" in x for x in blk):
        out += blk
    return out


def main():
    asm = compile_asm(sys.argv[1:])
    lines = asm.split("\n")
    for k in KERNELS:
        name, body = kernel_body(lines, r"^_ZN12_GLOBAL__N_1\d+" + k + r".*:")
        bars = [i for i, ln in enumerate(body) if "s_barrier" in ln]
        segs = list(zip([0] + bars, bars + [len(body)]))
        total = cost(body)
        print(k, metadata(asm, name))
        print("   weighted VALU cycles %d (%d instructions, %d moves); per barrier segment: %s"
              % (total[0], total[1], total[2], [cost(body[a:b])[0] for a, b in segs]))
        print("   without the IEEE-division slow paths: %d; per barrier segment: %s"
              % (cost(fast_path(body))[0], [cost(fast_path(body[a:b]))[0] for a, b in segs]))


if __name__ == "__main__":
    main()

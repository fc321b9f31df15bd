"""HBM bytes per kernel launch from the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh.

Calibration (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of a
16-B-per-lane streaming read, WRITE_SIZE the exact bytes of 16-B streaming stores.  Rather than
hard-coding the factor and the counter unit, the bench run itself contains launches of known byte
count -- bench.copy_ceiling_gbs streams 1 GiB -> 1 GiB with torch.mul (MulFunctor kernel, 16 B per
lane) -- and the per-unit scale is taken from them.  The rasterizer's own loads are narrower (4-B
face-index reads, 36-B face records), for which the guide calls the scale uncalibrated; the
corrected figure is reported as the traffic estimate with that caveat.

Writes <dir>/pmc_latest.json (a summary to keep under profiles/ with the round's name; bench.py imports
summarize() for its in-run passes and reads no file): {"config": [batch, image_size, level, mode], "hbm_bytes_per_launch":
{kernel: bytes}, "read_bytes": {...}, "write_bytes": {...}, "raw": {...}, "calibration": {...}}.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAL_BYTES = 1 << 30


def load(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"]
            m = re.search(r"\b(k_\w+)", name)
            key = m.group(1) if m else ("calib_mul" if "MulFunctor" in name else None)
            if key:
                vals[key].append(float(r["Counter_Value"]))
    return vals


SIMDS, XCDS, VALU_CYCLES = 1024, 8, 2  # MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU op issues over 2 cycles


def summarize(d, config=None, verbose=True, steps=None):
    """Per-kernel HBM bytes, VALU instruction counts and shares from the passes under d/p1..p3.  With
    `steps` (the fwd+bwd steps the profiled child ran), also each kernel's bytes per step: the sum
    over its launches / steps (a split forward launches k_raster_fwd twice per step)."""
    fetch, write = load(os.path.join(d, "p1"), "FETCH_SIZE"), load(os.path.join(d, "p2"), "WRITE_SIZE")
    p3 = os.path.join(d, "p3")
    valu, grbm = load(p3, "SQ_INSTS_VALU"), load(p3, "GRBM_GUI_ACTIVE")
    wave_cyc, wait_any = load(p3, "SQ_WAVE_CYCLES"), load(p3, "SQ_WAIT_ANY")
    # the calibration launches are the largest MulFunctor dispatches (1 GiB each)
    cf = sorted(fetch["calib_mul"])[-5:]
    cw = sorted(write["calib_mul"])[-5:]
    rscale = CAL_BYTES / (sum(cf) / len(cf))
    wscale = CAL_BYTES / (sum(cw) / len(cw))
    out = {"config": config or [64, 256, 4, "rgbsd"], "hbm_bytes_per_launch": {}, "read_bytes": {}, "write_bytes": {},
           "raw": {}, "calibration": {"bytes": CAL_BYTES, "fetch_units": sum(cf) / len(cf),
                                      "write_units": sum(cw) / len(cw), "read_scale": rscale, "write_scale": wscale}}
    for k in sorted(set(fetch) | set(write)):
        if k == "calib_mul":
            continue
        f = sum(fetch[k]) / len(fetch[k]) if fetch[k] else 0.0
        w = sum(write[k]) / len(write[k]) if write[k] else 0.0
        out["raw"][k] = {"FETCH_SIZE": f, "WRITE_SIZE": w, "n": [len(fetch[k]), len(write[k])]}
        out["read_bytes"][k] = f * rscale
        out["write_bytes"][k] = w * wscale
        out["hbm_bytes_per_launch"][k] = int(f * rscale + w * wscale)
        if steps:
            # launches per step rounded (a set-up launch outside the steps, e.g. cfg5's target render, is
            # one extra launch, not a second per step), at least one
            lps = max(1, round(max(len(fetch[k]), len(write[k])) / steps))
            out.setdefault("hbm_bytes_per_step", {})[k] = int((f * rscale + w * wscale) * lps)
            out.setdefault("launches_per_step", {})[k] = lps
        if valu.get(k) and grbm.get(k):
            mean = lambda v: sum(v) / len(v)  # noqa: E731
            # VALU issue share: wave-instructions x 2 cycles over the SIMD-cycles of the launch
            # (GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles); memory-wait share of the wave cycles
            out.setdefault("valu_busy", {})[k] = mean(valu[k]) * VALU_CYCLES / (SIMDS * mean(grbm[k]) / XCDS)
            out.setdefault("valu_insts", {})[k] = mean(valu[k])
            out.setdefault("gui_active_cycles", {})[k] = mean(grbm[k]) / XCDS
            if wave_cyc.get(k) and wait_any.get(k):
                out.setdefault("wait_any_share", {})[k] = mean(wait_any[k]) / mean(wave_cyc[k])
        if verbose:
            print("%-16s read %10.2f MB  write %10.2f MB  (raw FETCH %.4g WRITE %.4g)  VALU busy %s  wait %s" %
                  (k, f * rscale / 1e6, w * wscale / 1e6, f, w, "%.2f" % out.get("valu_busy", {}).get(k, float("nan")),
                   "%.2f" % out.get("wait_any_share", {}).get(k, float("nan"))))
    if verbose:
        print("calibration: read_scale %.4g B/unit, write_scale %.4g B/unit" % (rscale, wscale))
    return out


def main(d):
    out = summarize(d)
    json.dump(out, open(os.path.join(d, "pmc_latest.json"), "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) per kernel: mean counter value per dispatch.
usage: python tools/pmc_summary.py <dir> [--all]  (--all: also the non-nr kernels, e.g. the calibration copy)"""
import collections
import csv
import glob
import re
import sys

d = sys.argv[1]
ALL = "--all" in sys.argv[2:]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        m = re.search(r'(k_\w+)', r['Kernel_Name'])
        if not m and not ALL:
            continue
        key = (m.group(1) + ('<1>' if '<true>' in r['Kernel_Name'] else '')) if m else r['Kernel_Name'][:60]
        agg[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k, dd in agg.items():
    print(k)
    for c, v in sorted(dd.items()):
        print('   %-24s %14.4g  (n=%d)' % (c, sum(v) / len(v), len(v)))

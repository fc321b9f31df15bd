# usage: bash tools/pmc_probe.sh <tag> "PASS1" "PASS2" ...: lists the box's counters, then runs each
# pass (a space-separated counter list) whose counters all exist, one rocprofv3 --pmc run per pass,
# over a short bench (PROBE_ARGS: another python program + args, e.g. "tools/bench_configs.py --only cfg3
# --steps 2 --warmup 1"); tools/pmc_summary.py prints per-kernel averages.  The default bench run
# passes --no-pmc: the profiled bench must not start its own nested rocprofv3 passes (bench.py
# also skips them by itself when it sees rocprofv3's ROCPROF_* environment).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-probe}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -oE '\b(TA|TD|TCP|TCC|SQ|GRBM)_[A-Za-z0-9_]+' $OUT/counters.txt | sort -u > $OUT/names.txt
i=0
for PASS in "$@"; do
  i=$((i+1))
  ok=1
  for c in $PASS; do grep -qx "$c" $OUT/names.txt || { echo "pass $i: no counter $c"; ok=0; }; done
  [ $ok = 1 ] || continue
  timeout -k 10 120 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run -- python3 ${PROBE_ARGS:-bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($PASS) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; echo "summary rc=$?"

# usage: bash tools/gpu_check.sh <tag> [pytest selection]: GPU tests, smoke, the bench line (with its
# in-run rocprofv3 --pmc passes), a rocprofv3 --kernel-trace --stats summary of a short bench run, and
# (CONFIGS=cfg2,cfg3,cfg5) the other configs with their per-config rooflines and PMC traffic.
# Every step has its own time limit; the script stops at the first failing step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-check}
SEL=${2:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider --durations=15 > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-pmc --no-count > $OUT/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -8 $OUT/kernel_stats.csv 2>/dev/null | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$CONFIGS" ]; then
  timeout -k 10 600 python tools/bench_configs.py --only $CONFIGS --pmc > $OUT/configs.jsonl 2>&1
  rc=$?; echo "configs rc=$rc"; grep '^{' $OUT/configs.jsonl | cut -c1-300
fi
exit $rc

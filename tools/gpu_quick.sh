# usage: bash tools/gpu_quick.sh <tag>: GPU tests, then the other configs and a headline bench line
# without PMC passes / CPU baseline; stops at the first failing step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python tools/bench_configs.py --only ${CONFIGS:-cfg2,cfg3,cfg5} > $OUT/configs.jsonl 2>&1
rc=$?; echo "configs rc=$rc"; grep '^{' $OUT/configs.jsonl | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels_ms'], 'host', d['host_ms_per_step'])"
exit $rc

# usage: bash tools/gpu_check.sh <tag>: GPU tests, smoke, PMC traffic passes, short bench, rocprofv3 kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
# HBM traffic passes first, so the bench line's roofline.traffic is this build's
bash tools/pmc_traffic.sh $TAG/traffic || exit $?
cp $OUT/traffic/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "rocprof rc=$?"

# usage: ENVS="A=1 A=0,B=2" REPEAT=3 bash tools/ab_env.sh <tag>: the headline bench (no PMC, no CPU
# baseline) under each environment (comma-separated VAR=value lists; "base" = none), interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-abenv}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for r in $(seq 1 ${REPEAT:-1}); do
i=0
for E in ${ENVS:-base}; do
  i=$((i+1))
  EV=""
  if [ "$E" != base ]; then EV=${E//,/ }; fi
  env $EV timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-pmc > $OUT/bench_${i}_$r.log 2>&1
  rc=$?; echo "$E rc=$rc: $(python -c "import json,sys; d=json.loads(open('$OUT/bench_${i}_$r.log').read().strip().splitlines()[-1]); print(d['kernels_ms'], d['ms_per_step'])")"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
done

# usage: bash tools/car_evidence.sh <tag>: BASELINE cfg3 (the car) counter evidence, each step under its
# own time limit: a rocprofv3 kernel trace, the HBM traffic passes (FETCH_SIZE / WRITE_SIZE calibrated on
# a 1 GiB stream, VALU share), the memory-pipeline passes (TA / TD / TCP / TCC), and the forward and
# backward per-wave phases (timing builds).  Summaries land in gpurun_out/<tag>/*.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-car}
OUT=gpurun_out/$TAG
mkdir -p $OUT
RUN="tools/bench_configs.py --only cfg3 --steps 3 --warmup 1 --calibrate"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 tools/bench_configs.py --only cfg3 --steps 10 --warmup 3 > $OUT/prof.log 2>&1
rc=$?; echo "kernel trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
i=0
for PASS in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $PASS --output-format csv -d $OUT/t/p$i -o run -- python3 $RUN > $OUT/t_p$i.log 2>&1
  rc=$?; echo "traffic pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
python3 tools/pmc_traffic.py $OUT/t > $OUT/traffic.txt 2>&1; echo "traffic summary rc=$?"
i=0
while read -r PASS; do
  [ -z "$PASS" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $PASS --output-format csv -d $OUT/mp/p$i -o run -- python3 $RUN > $OUT/mp_p$i.log 2>&1
  rc=$?; echo "memory pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done <<'PASSES'
TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE
TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum
TCC_HIT_sum TCC_MISS_sum
PASSES
python3 tools/pmc_summary.py $OUT/mp > $OUT/memory_pipe.txt 2>&1; echo "memory summary rc=$?"
timeout -k 10 300 python3 tools/fwd_timing.py --workload car > $OUT/fwd_wave_phases_car.txt 2>&1
rc=$?; echo "fwd phases rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/bwd_timing.py --workload car > $OUT/bwd_wave_phases_car.txt 2>&1
rc=$?; echo "bwd phases rc=$rc"; exit $rc

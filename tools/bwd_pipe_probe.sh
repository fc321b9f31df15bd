# usage: bash tools/bwd_pipe_probe.sh <tag>: headline memory-pipeline counters (TA / TD / TCP / TCC and the
# SQ instruction mix) per kernel, the same TCP passes over bench_configs' 1 GiB copy stream (to read
# the L1 access counter's granularity off a kernel of known bytes), and the backward's per-wave phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pipe}
OUT=gpurun_out/$TAG
mkdir -p $OUT
PROBE_ARGS="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc" timeout -k 10 600 bash tools/pmc_probe.sh $TAG/h \
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE" \
  "TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum" \
  "TCC_HIT_sum TCC_MISS_sum" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
rc=$?; echo "headline probe rc=$rc"; [ $rc -ne 0 ] && exit $rc
PROBE_ARGS="tools/bench_configs.py --only cfg2 --steps 2 --warmup 1 --calibrate" timeout -k 10 600 bash tools/pmc_probe.sh $TAG/c \
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_FLAT_READ_WAVEFRONTS_sum" \
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
rc=$?; echo "calibration probe rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/pmc_summary.py $OUT/c --all > $OUT/c/summary_all.txt 2>&1
timeout -k 10 300 python3 tools/bwd_timing.py > $OUT/bwd_wave_phases.txt 2>&1
rc=$?; echo "bwd phases rc=$rc"; exit $rc

# usage: [NR_LIB_PATH=lib.so] bash tools/pmc.sh <tag>: PMC counter passes (one rocprofv3 run per pass) over a short bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
i=0
while read -r PASS; do
  [ -z "$PASS" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($PASS) rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
done <<'PASSES'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS
GRBM_GUI_ACTIVE SQ_INSTS_FLAT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH
PASSES

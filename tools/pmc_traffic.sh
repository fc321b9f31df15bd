# usage: bash tools/pmc_traffic.sh <tag>: HBM traffic per kernel launch from FETCH_SIZE and WRITE_SIZE,
# each in its own rocprofv3 --pmc pass (they do not fit one pass on gfx950), over a short bench run,
# plus a pass for the VALU issue share (SQ_INSTS_VALU, GRBM_GUI_ACTIVE) and the memory-wait share;
# tools/pmc_traffic.py turns them into <out>/pmc_latest.json (a per-kernel summary to copy into
# profiles/ under the round's name; bench.py measures its own roofline traffic in-run and reads no file).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-traffic}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for PASS in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PASS --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($PASS) rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 tools/pmc_traffic.py $OUT > $OUT/traffic.txt 2>&1
rc=$?; cat $OUT/traffic.txt; exit $rc

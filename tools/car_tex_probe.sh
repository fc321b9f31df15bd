# usage: bash tools/car_tex_probe.sh <tag> <lib>...: the car's (cfg3) HBM reads and L2 hit rate per kernel for
# each library (e.g. the product and the NR_ABL_NOTEX timing build, whose texture samples load no texel):
# how much of the forward's reads and L2 misses the shared texture atlas causes.  One FETCH_SIZE pass and
# one TCC_HIT / TCC_MISS pass per library, each under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
RUN="tools/bench_configs.py --only cfg3 --steps 3 --warmup 1 --calibrate --no-count"
j=0
for LIB in "$@"; do
  j=$((j+1))
  NR_LIB_PATH=$LIB timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/l$j/t/p1 -o run -- python3 $RUN > $OUT/l${j}_f.log 2>&1
  rc=$?; echo "$LIB fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
  NR_LIB_PATH=$LIB timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/l$j/mp/p1 -o run -- python3 $RUN > $OUT/l${j}_h.log 2>&1
  rc=$?; echo "$LIB hit rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python3 tools/pmc_traffic.py $OUT/l$j/t > $OUT/l${j}_traffic.txt 2>&1
  python3 tools/pmc_summary.py $OUT/l$j/mp > $OUT/l${j}_l2.txt 2>&1
  echo "== $LIB"; cat $OUT/l${j}_traffic.txt | head -30; grep -A3 "k_raster" $OUT/l${j}_l2.txt
done

# usage: bash tools/ablate.sh <tag>: build NR_ABLATE timing variants of the library and bench each
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ablate}
OUT=gpurun_out/$TAG
mkdir -p $OUT/lib
for A in ${ABLATE:-0 1 2}; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
    -fvisibility=hidden -Iinclude $( [ ${A:0:1} = f ] && echo -DNR_ABLATE_FWD=${A:1} || echo -DNR_ABLATE=$A ) neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip -o $OUT/lib/libnr_$A.so || exit 1
done
for A in ${ABLATE:-0 1 2}; do
  NR_LIB_PATH=$OUT/lib/libnr_$A.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_$A.log 2>&1
  rc=$?; echo "ablate $A rc=$rc: $(python -c "import json,sys; d=json.loads(open('$OUT/bench_$A.log').read().strip().splitlines()[-1]); print(d['kernels_ms'], d['ms_per_step'])")"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
rm -rf $OUT/lib

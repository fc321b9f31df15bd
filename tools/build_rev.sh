# usage: bash tools/build_rev.sh <git-rev> [out.so]: builds the HIP library of an older revision (its
# csrc/ and include/ from git) into build/ for A/B timing with tools/ablate.sh ("lib:build/...")
set -e
REV=${1:?rev}
OUT=${2:-build/libnr_$REV.so}
TMP=$(mktemp -d)
git archive "$REV" neural_renderer_v2_pytorch_amd/csrc include | tar -x -C $TMP
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math \
  -fvisibility=hidden -I$TMP/include $TMP/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip -o $OUT
rm -rf $TMP
echo "built $OUT"

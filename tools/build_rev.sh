# usage: bash tools/build_rev.sh <git-rev> [out.so]: builds the HIP library of an older revision (its
# csrc/ and include/ from git) into build/ for A/B timing with tools/ablate.sh ("lib:build/...")
set -e
# the product's hipcc flags (__graft_entry__.HIPCC_FLAGS without -I); HIPFLAGS overrides them
HIPFLAGS=${HIPFLAGS:-$(cd "$(dirname "$0")/.." && python3 -c 'import __graft_entry__ as g; print(" ".join(g.hipcc_flags()))')}
REV=${1:?rev}
OUT=${2:-build/libnr_$REV.so}
TMP=$(mktemp -d)
git archive "$REV" neural_renderer_v2_pytorch_amd/csrc include | tar -x -C $TMP
mkdir -p $(dirname $OUT)
/opt/rocm/bin/hipcc $HIPFLAGS \
  -I$TMP/include $TMP/neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip -o $OUT
rm -rf $TMP
echo "built $OUT"

# usage: VARIANTS="base lib:abl/libnr_old.so NR_FWD_TIMING A=1,@ENV=2 M:--misched=gcn-max-ilp" bash tools/ablate.sh <tag>
# builds one library per variant (comma-separated -D defines; "base" = none; a token @VAR=value is an
# environment setting of that variant's runs instead, M:<opt> an `-mllvm <opt>` code-generation option)
# and benches each;
# CONFIGS=cfg2,cfg3,cfg5 also times those configs (tools/bench_configs.py); NOHEAD=1 skips the headline.
set -o pipefail
# the product's hipcc flags (__graft_entry__.HIPCC_FLAGS without -I); HIPFLAGS overrides them
HIPFLAGS=${HIPFLAGS:-$(cd "$(dirname "$0")/.." && python3 -c 'import __graft_entry__ as g; print(" ".join(g.hipcc_flags()))')}
cd $GRAFT_REPO_ROOT
TAG=${1:-ablate}
OUT=gpurun_out/$TAG
mkdir -p $OUT/lib
VARIANTS=${VARIANTS:-base}
i=0
for V in $VARIANTS; do
  i=$((i+1))
  # "lib:<path>": a library built beforehand (e.g. from an older revision, tools/build_rev.sh)
  V0=${V%%,*}
  if [ "${V0#lib:}" != "$V0" ]; then cp "${V0#lib:}" $OUT/lib/libnr_$i.so || exit 1; continue; fi
  DEFS=""
  if [ "$V" != base ]; then for d in ${V//,/ }; do case $d in @*) ;; base) ;; lib:*) ;; M:*) DEFS="$DEFS -mllvm ${d#M:}";; *) DEFS="$DEFS -D$d";; esac; done; fi
  /opt/rocm/bin/hipcc $HIPFLAGS \
  -Iinclude $DEFS neural_renderer_v2_pytorch_amd/csrc/nr_raster.hip -o $OUT/lib/libnr_$i.so || exit 1
done
# REPEAT=n runs the whole variant list n times, interleaved (box-to-box and run-to-run spread is a
# few per cent); STEPS sets the timed steps per run
for r in $(seq 1 ${REPEAT:-1}); do
i=0
for V in $VARIANTS; do
  i=$((i+1))
  EV=""
  for d in ${V//,/ }; do case $d in @*) EV="$EV ${d#@}";; esac; done
  if [ -z "$NOHEAD" ]; then
  env $EV NR_LIB_PATH=$OUT/lib/libnr_$i.so timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --no-pmc --no-count > $OUT/bench_${i}_$r.log 2>&1
  rc=$?; echo "$V rc=$rc: $(python -c "import json,sys; d=json.loads(open('$OUT/bench_${i}_$r.log').read().strip().splitlines()[-1]); print(d['kernels_ms'], d['ms_per_step'])")"
  if [ $rc -ne 0 ]; then exit $rc; fi
  fi
  if [ -n "$CONFIGS" ]; then
    env $EV NR_LIB_PATH=$OUT/lib/libnr_$i.so timeout -k 10 300 python tools/bench_configs.py --loop-steps 20 --no-count --only $CONFIGS > $OUT/configs_$i.log 2>&1
    rc=$?; python -c "
import json
for l in open('$OUT/configs_$i.log'):
    if l.startswith('{'): d = json.loads(l); print('   ', '$V', d['config'][:5], d['ms_per_step'], d['kernels_ms'])"
    if [ $rc -ne 0 ]; then exit $rc; fi
  fi
done
done
rm -rf $OUT/lib

# usage: bash tools/gpu_round.sh <tag>: GPU tests + smoke + bench + rocprof stats + ablation timings
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh $1 || exit $?
bash tools/ablate.sh $1/ablate

# usage: bash tools/profile.sh <tag>  -- rocprofv3 kernel trace + stats of a short bench run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1
echo "rocprof rc=$?"
find gpurun_out/$TAG -name "*stats*" | head

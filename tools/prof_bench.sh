# Kernel trace of a short bench run: bash tools/prof_bench.sh <tag> [bench args]
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$tag
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 bench.py --no-cpu-baseline --steps 40 "$@" > gpurun_out/$tag/bench.log 2>&1

set -euo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SWARMRL_AMD_RIDE_ALONG=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3n_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3n_trace.log 2>&1

set -euo pipefail
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3o_bench$r.log 2>&1
done
SWARMRL_AMD_SPEC_VGRID=0 timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3o_bench_spec0.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3o_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3o_trace.log 2>&1

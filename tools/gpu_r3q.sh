set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3q_gpu_tests.log 2>&1
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_PT.so timeout -k 10 120 python tools/build_phases.py 4096 > gpurun_out/r3q_phases.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3q_bench$r.log 2>&1
done
SWARMRL_AMD_VGRID_STAGED=0 timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3q_bench_st0.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3q_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3q_trace.log 2>&1

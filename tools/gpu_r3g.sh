set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_nonperiodic.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3g_gpu_tests.log 2>&1
for v in 1 0; do
SWARMRL_AMD_FUSED_CHECK=$v timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3g_bench_fc$v.log 2>&1
done
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_CALL.so timeout -k 10 200 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3g_bench_call.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3g_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3g_trace.log 2>&1

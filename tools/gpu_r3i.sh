set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_nonperiodic.py tests/test_gpu_parity.py tests/test_gpu_multispecies.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_gpu_tests.log 2>&1 || timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_nonperiodic.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3i_gpu_tests.log 2>&1
for v in PT PTK1; do
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_$v.so timeout -k 10 120 python tools/build_phases.py 4096 > gpurun_out/r3i_phases_$v.log 2>&1
done
for r in 1 2; do
timeout -k 10 200 python bench.py --only head,c2 --no-cpu-baseline > gpurun_out/r3i_bench_main$r.log 2>&1
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_K1.so timeout -k 10 200 python bench.py --only head,c2 --no-cpu-baseline > gpurun_out/r3i_bench_K1_$r.log 2>&1
done

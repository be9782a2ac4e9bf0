set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3aa_gpu_tests.log 2>&1
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_PT.so timeout -k 10 200 python tools/build_phases.py 16384 > gpurun_out/r3aa_phases16k.log 2>&1
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_PT.so timeout -k 10 200 python tools/build_phases.py 4096 > gpurun_out/r3aa_phases.log 2>&1
for r in 1 2; do
timeout -k 10 200 python bench.py --only head,c5 --no-cpu-baseline > gpurun_out/r3aa_bench$r.log 2>&1
done
SWARMRL_AMD_SORT_STAGED=0 timeout -k 10 200 python bench.py --only head,c5 --no-cpu-baseline > gpurun_out/r3aa_bench_st0.log 2>&1

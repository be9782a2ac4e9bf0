set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3v_gpu_tests.log 2>&1
for r in 1 2; do
for v in main bal; do
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_$v.so timeout -k 10 120 python tools/vision_time.py 1 64 > gpurun_out/r3v_vis_${v}_$r.log 2>&1
done
done

set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x_gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3x_smoke.log 2>&1
timeout -k 10 600 python bench.py > gpurun_out/r3x_bench_default.log 2>&1

set -euo pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/vision_time.py 1 64 > gpurun_out/r3s_vis.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3s_trace -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3s_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3s_fetch -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3s_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3s_write -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3s_write.log 2>&1

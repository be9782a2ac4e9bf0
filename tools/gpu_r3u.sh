set -euo pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_BRANCH --output-format csv -d gpurun_out/r3u_pmc1 -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3u_pmc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY --output-format csv -d gpurun_out/r3u_pmc2 -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3u_pmc2.log 2>&1

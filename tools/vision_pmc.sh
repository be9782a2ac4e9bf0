# Vision kernels (tools/vision_time.py E=64): kernel trace, then FETCH_SIZE and
# SQ passes, for the LDS-tile kernel and the record-streaming one.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/vpmc; mkdir -p $out
for t in 0 1; do
  SWARMRL_AMD_VISION_TILE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/t${t}_trace -o run -- python3 tools/vision_time.py 64 > $out/t${t}_trace.log 2>&1
  SWARMRL_AMD_VISION_TILE=$t timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/t${t}_fetch -o run -- python3 tools/vision_time.py 64 > $out/t${t}_fetch.log 2>&1
  SWARMRL_AMD_VISION_TILE=$t timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $out/t${t}_sq -o run -- python3 tools/vision_time.py 64 > $out/t${t}_sq.log 2>&1
done

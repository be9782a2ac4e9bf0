#!/bin/bash
# SQ counter passes over the integrator windows (tools/ablate_integrator.py),
# run on the GPU box from the repo root:  bash tools/pmc_run.sh <tag> <spec...>
# Each pass: its own rocprofv3 process, PMC only (no other trace domains).
set -euo pipefail
tag=$1; shift
out=gpurun_out/pmc_${tag}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
p1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES"
p2="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM"
p3="GRBM_GUI_ACTIVE GRBM_COUNT"
k=0
for p in "$p1" "$p2" "$p3"; do
  k=$((k + 1))
  timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d "$out/p$k" -o run -- \
    python3 tools/ablate_integrator.py "$@" > "$out/p$k.log" 2>&1
done
echo "pmc written to $out"

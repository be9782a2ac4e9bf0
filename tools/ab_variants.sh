#!/bin/bash
# A/B of variant libraries on the GPU box (run from the repo root):
# run-kernel times (tools/run_kernel_time.py, HIP events) and the FETCH_SIZE /
# WRITE_SIZE counters of the run kernel per variant.
#   bash tools/ab_variants.sh TAG "E..." prod smaj minb4 ...
# "prod" is the in-tree library; NAME -> tools/_variants/lib_NAME.so.
set -euo pipefail
tag=$1; envs=$2; shift 2
out=gpurun_out/ab_${tag}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=$PWD/swarmrl_amd/libswarmrl_amd.so
  [ "$v" != prod ] && lib=$PWD/tools/_variants/lib_${v}.so
  SWARMRL_AMD_LIB=$lib timeout -k 10 180 python3 tools/run_kernel_time.py $envs > "$out/${v}_time.log" 2>&1
  cat "$out/${v}_time.log"
  for c in FETCH_SIZE WRITE_SIZE; do
    SWARMRL_AMD_LIB=$lib timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d "$out/${v}_$c" -o run -- \
      python3 tools/run_kernel_time.py $envs > "$out/${v}_$c.log" 2>&1
  done
  echo "variant $v done"
done

#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in separate PMC passes
#   (MI355X_MICROARCH.md "rocprofv3 PMC slots": they do not fit one pass).
# Usage: bash profiles/profile_round.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/prof_${tag}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/trace_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/fetch_bench.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/write_bench.log" 2>&1
echo "profiles written to $out"

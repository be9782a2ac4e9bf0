#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   1. kernel trace + stats of the default bench command
#   2. FETCH_SIZE, 3. WRITE_SIZE, 4. SQ_INSTS_VALU + SQ_WAVES -- separate PMC
#      passes (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE do not fit one
#      pass; PMC passes carry no other trace domains)
# then tools/summarize_profiles.py writes profiles/<tag>_*.
# Usage: bash profiles/profile_round.sh <tag> [bench args...]
set -euo pipefail
tag=$1; shift
out=gpurun_out/prof_${tag}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/trace_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/fetch_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/write_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d "$out/valu" -o run -- \
  python3 bench.py --no-cpu-baseline "$@" > "$out/valu_bench.log" 2>&1
echo "profiles written to $out"

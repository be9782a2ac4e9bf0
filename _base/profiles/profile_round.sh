#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root), one CONFIG-PURE
# run per bench line (bench.py --only <line>), so every kernel row belongs to
# exactly one configuration:
#   1. kernel trace + stats
#   2. FETCH_SIZE, 3. WRITE_SIZE, 4. SQ_INSTS_VALU + SQ_INSTS_VALU_TRANS_F32 +
#      SQ_WAVES -- separate PMC passes (MI355X_MICROARCH.md: FETCH_SIZE and
#      WRITE_SIZE do not fit one pass; PMC passes carry no other trace domains)
# then tools/summarize_profiles.py <tag> writes profiles/<tag>_*.
# Usage: bash profiles/profile_round.sh <tag> [bench args...]
#        (LINES="head batched" to profile a subset, PASSES="trace" to skip the
#        counter passes)
set -euo pipefail
tag=$1; shift
lines=${LINES:-"head batched c2 c4 c5 c3train"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for line in $lines; do
  out=gpurun_out/prof_${tag}/${line}
  mkdir -p "$out"
  run() {  # run <subdir> <rocprofv3 options...>
    local sub=$1; shift
    timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$out/$sub" -o run -- \
      python3 bench.py --only "$line" --no-cpu-baseline "${BENCH_ARGS[@]}" > "$out/${sub}_bench.log" 2>&1
  }
  BENCH_ARGS=("$@")
  passes=${PASSES:-"trace fetch write valu"}
  for p in $passes; do
    case $p in
      trace) run trace --kernel-trace --stats ;;
      fetch) run fetch --pmc FETCH_SIZE ;;
      write) run write --pmc WRITE_SIZE ;;
      valu) run valu --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES ;;
      sq) run sq --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS \
            SQ_INSTS_LDS SQ_ACTIVE_INST_VALU ;;
    esac
  done
  echo "profiled $line"
done
echo "profiles written to gpurun_out/prof_${tag}"

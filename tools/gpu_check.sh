#!/bin/bash
# GPU-box check of the tree (run through gpurun from the repo root):
#   gpu test suite -> smoke -> default bench, outputs under gpurun_out/<tag>.
# Every GPU step has its own time limit and the first failure ends the run.
# Usage: bash tools/gpu_check.sh <tag> [pytest selection, default "tests"]
set -uo pipefail
tag=$1; shift
sel=${*:-tests}
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$out/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 1
tail -2 "$out/smoke.txt"
timeout -k 10 400 python3 bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || exit 1
cut -c1-600 "$out/bench_default.json"

#!/bin/bash
# One GPU-box pass of the round's checks (run from the repo root under gpurun):
# the -m gpu suite, then (unless it crashed) the default bench line.
#   bash tools/gpu_round.sh TAG [pytest selection...]
# Outputs: gpurun_out/TAG/{gpu_tests.txt,bench.json,bench.err}
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
# WORKDIR: run the checks of another copy of the tree (e.g. a baseline
# build unpacked under the repo); outputs still go to gpurun_out/TAG
[ -n "$WORKDIR" ] && { cd "$WORKDIR" || exit 2; }
sel=("$@")
[ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 900 python -u -m pytest "${sel[@]}" -m gpu -v --timeout 150 --timeout-method thread \
  > "$out/gpu_tests.txt" 2>&1
rc=$?
echo "tests rc=$rc" >> "$out/gpu_tests.txt"
# a test failure (1) is not a GPU fault; anything else ends the call here
if [ $rc -le 1 ] && [ -z "$NO_BENCH" ]; then
  timeout -k 10 500 python bench.py > "$out/bench.json" 2> "$out/bench.err"
  echo "bench rc=$?" >> "$out/gpu_tests.txt"
fi
exit $rc

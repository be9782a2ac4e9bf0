#!/bin/bash
# Round-3 final check on the rebuilt tree: gpu suite, smoke, default bench.
set -uo pipefail
out=gpurun_out/r3final
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$out/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 1
tail -2 "$out/smoke.txt"
timeout -k 10 300 python3 bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || exit 1
cat "$out/bench_default.json" | cut -c1-400

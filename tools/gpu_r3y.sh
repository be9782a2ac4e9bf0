#!/bin/bash
# Round-3 session-2 check: full gpu suite on the tree's library, then an
# A/B of the run kernel and the head/batched bench lines against the
# library of HEAD (tools/_variants/lib_head.so, tools/build_rev.sh HEAD head).
set -uo pipefail
out=gpurun_out/r3y
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/gpu_tests.txt" 2>&1
rc=$?
tail -3 "$out/gpu_tests.txt"
[ $rc -eq 0 ] || exit $rc
for v in head prod head prod; do
  lib=$PWD/swarmrl_amd/libswarmrl_amd.so
  [ "$v" != prod ] && lib=$PWD/tools/_variants/lib_${v}.so
  echo "== $v"
  SWARMRL_AMD_LIB=$lib timeout -k 10 150 python3 tools/run_kernel_time.py 1 64 || exit 1
  SWARMRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --only head,batched --no-cpu-baseline \
    > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit 1
  python3 -c "import json;d=json.load(open('$out/bench_$v.json'));print('head',d['value']/1e6,'batched',d['batched']['value']/1e6)"
done

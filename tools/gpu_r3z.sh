#!/bin/bash
# Round-3 final check, part 1: gpu suite, smoke, default bench line, then
# config-pure profiles of LINES (profiles/profile_round.sh r3c).
set -uo pipefail
out=gpurun_out/r3z
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$out/gpu_tests.txt" 2>&1
  rc=$?; tail -3 "$out/gpu_tests.txt"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > "$out/smoke.txt" 2>&1
  rc=$?; tail -3 "$out/smoke.txt"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err"
  rc=$?; [ $rc -eq 0 ] || { tail "$out/bench_default.err"; exit $rc; }
  python3 -c "import json;d=json.load(open('$out/bench_default.json'));print('head',d['value']/1e6,{k:v['value']/1e6 for k,v in d.items() if isinstance(v,dict) and 'value' in v and v.get('unit')=='agent-steps/s'})"
fi
[ -n "${LINES:-}" ] && bash profiles/profile_round.sh "${TAG:-r3c}"
exit 0

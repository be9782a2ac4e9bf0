#!/bin/bash
# A development probe on the GPU box: a -m gpu test subset, then same-box
# bench A/B of library variants (tools/gpu_ab.sh), then rocprofv3 kernel
# traces of one bench line for the working tree and (optional) a baseline
# copy of the tree.  Every step is time-limited; a crash ends the call.
#   TESTS="tests/a.py ..." VARIANTS="prod X" LINES=head,c5 SCHED_LINE=c5 SCHEDS="default obs_side" \
#     PROF_LINE=c5 BASE=_base \
#     bash tools/gpu_probe.sh TAG
tag=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -v --timeout 150 --timeout-method thread \
    > "$out/tests.txt" 2>&1
  rc=$?; echo "tests rc=$rc" >> "$out/tests.txt"
  [ $rc -le 1 ] || exit $rc
fi
if [ -n "$VARIANTS" ]; then
  bash tools/gpu_ab.sh "$tag" $VARIANTS > "$out/ab.txt" 2>&1 || exit $?
fi
if [ -n "$SCHED_LINE" ]; then  # schedule A/B: SCHED_LINE=c5 SCHEDS="default obs_side"
  timeout -k 10 900 python3 tools/sched_ab.py "$SCHED_LINE" $SCHEDS > "$out/sched.txt" 2>&1 || exit $?
fi
if [ -n "$EXTRA" ]; then  # one more command (e.g. a rocprofv3 run of a tool), 300 s
  timeout -k 10 300 bash -c "$EXTRA" > "$out/extra.txt" 2>&1 || exit $?
fi
prof() {  # prof <dir> <name>
  (cd "$1" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$out/prof_$2" -o run -- python3 bench.py --only "$PROF_LINE" --no-cpu-baseline \
     > "$out/prof_$2.log" 2>&1)
}
if [ -n "$PROF_LINE" ]; then
  prof . tree || exit $?
  if [ -n "$BASE" ]; then prof "$BASE" base || exit $?; fi
fi
exit 0

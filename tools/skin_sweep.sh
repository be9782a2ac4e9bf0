#!/bin/bash
# Head line vs the cluster decomposition's Verlet skin (SWARMRL_AMD_SKIN, um):
# results are bit-identical for any skin; the skin trades cluster size (pairs,
# big clusters in k_check) against exact re-runs of failed windows.
set -uo pipefail
out=gpurun_out/skin
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in ${SKINS:-1.25 1.5 1.75 2.0 2.5}; do
  SWARMRL_AMD_SKIN=$s timeout -k 10 200 python3 bench.py --only head --no-cpu-baseline --steps 400 \
    > "$out/head_$s.json" 2> "$out/head_$s.err" || exit 1
  python3 -c "import json;d=json.load(open('$out/head_$s.json'));print('skin $s', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us/slice')"
done

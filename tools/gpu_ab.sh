#!/bin/bash
# A/B of engine libraries on the GPU box: run-kernel HIP-event times
# (tools/run_kernel_time.py) and the head / batched bench lines per variant.
#   bash tools/gpu_ab.sh TAG prod NAME ...   (NAME -> tools/_variants/lib_NAME.so)
set -uo pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  lib=$PWD/swarmrl_amd/libswarmrl_amd.so
  [ "$v" != prod ] && lib=$PWD/tools/_variants/lib_${v}.so
  echo "== $v"
  SWARMRL_AMD_LIB=$lib timeout -k 10 150 python3 tools/run_kernel_time.py 1 64 || exit 1
  SWARMRL_AMD_LIB=$lib timeout -k 10 200 python3 bench.py --only ${LINES:-head,batched} --no-cpu-baseline \
    > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit 1
  python3 -c "import json;d=json.load(open('$out/bench_$v.json'));print({k:(v['value']/1e6 if isinstance(v,dict) and 'value' in v else None) for k,v in d.items() if isinstance(v,dict) and 'value' in v}, 'head', d['value']/1e6)"
done

#!/bin/bash
# Same-box A/B pass: the default bench of a baseline copy of the tree
# (unpacked under BASE, with its own built library), then the -m gpu suite
# and the default bench of the working tree (tools/gpu_round.sh).
#   bash tools/gpu_ab_round.sh TAG BASE [pytest selection...]
tag=$1; base=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 2
out=$PWD/gpurun_out/$tag
mkdir -p "$out"
(cd "$base" && timeout -k 10 400 python bench.py > "$out/base_bench.json" 2> "$out/base_bench.err")
echo "base bench rc=$?" > "$out/ab.txt"
bash tools/gpu_round.sh "$tag" "$@"

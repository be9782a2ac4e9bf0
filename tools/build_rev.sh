# Build the engine library of git revision REV into tools/_variants/lib_NAME.so
# (A/B against an earlier revision of the kernels; never the product path):
#   bash tools/build_rev.sh REV NAME [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
git archive "$rev" swarmrl_amd/csrc include | tar -x -C "$tmp"
mkdir -p tools/_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off "$@" \
  "$tmp/swarmrl_amd/csrc/swarm_engine.hip" -o "tools/_variants/lib_${name}.so"
rm -rf "$tmp"

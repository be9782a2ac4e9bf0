# Timing-ablation variants of the engine library (never used by the product
# path; results are NOT bit-exact): phase timing plus one section removed.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -DSWARM_PHASE_TIMING"
for v in NONE NOTABLE NOSINCOS NOPAIR; do
  /opt/rocm/bin/hipcc $F -DSWARM_ABL_$v swarmrl_amd/csrc/swarm_engine.hip -o tools/_variants/lib_PT_$v.so &
done
wait

# Profiling variants of the engine library (never used by the product path):
#   _nopairs: run kernel without the neighbour loop; _nobd: without the BD update.
set -e
cd "$(dirname "$0")/.."
for v in NO_PAIRS NO_BD PHASE_TIMING; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -DSWARM_$v -DSWARM_ABLATE_$v swarmrl_amd/csrc/swarm_engine.hip -o /tmp/libswarmrl_amd_$v.so &
done
wait
mkdir -p tools/_variants && cp /tmp/libswarmrl_amd_*.so tools/_variants/

# Profiling variant of the engine library (never used by the product path):
#   PHASE_TIMING: shader-clock stamps of the build phases and the run / global
#   path sub-step sections (tools/build_phases.py, tools/rerun_cost.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -DSWARM_PHASE_TIMING swarmrl_amd/csrc/swarm_engine.hip -o tools/_variants/lib_PT.so

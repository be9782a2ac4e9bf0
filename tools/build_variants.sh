# Variant builds of the engine library for A/B measurements (never used by
# the product path; SWARMRL_AMD_LIB=tools/_variants/lib_<name>.so selects one):
#   bash tools/build_variants.sh NAME "-DFLAG ..." [NAME "-DFLAG ..."] ...
#   e.g. PT "-DSWARM_PHASE_TIMING" (shader-clock stamps of the build phases
#   and the run sub-step sections: tools/build_phases.py, tools/rerun_cost.py)
# The builds run in parallel (one hipcc each).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
bid=$(python3 -c "import __graft_entry__ as g; print(g._source_hash())")
pids=()
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -fno-slp-vectorize \
    -DSWARM_BUILD_ID=\"$bid\" $flags swarmrl_amd/csrc/swarm_engine.hip -o tools/_variants/lib_${name}.so &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done

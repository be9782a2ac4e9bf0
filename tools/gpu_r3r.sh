set -euo pipefail
mkdir -p gpurun_out
for r in 1 2; do
for v in main F12 F16; do
L=$PWD/tools/_variants/lib_$v.so
SWARMRL_AMD_LIB=$L timeout -k 10 200 python bench.py --only head,c2 --no-cpu-baseline > gpurun_out/r3r_bench_${v}_$r.log 2>&1
done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_F16.so SWARMRL_AMD_RIDE_ALONG=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3r_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3r_trace.log 2>&1

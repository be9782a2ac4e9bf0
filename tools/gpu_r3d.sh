set -euo pipefail
mkdir -p gpurun_out
true
for x in 0 1; do
  SWARMRL_AMD_XCD_MAP=$x timeout -k 10 120 python tools/run_kernel_time.py 64 > gpurun_out/r3d_run_xcd$x.log 2>&1
  SWARMRL_AMD_XCD_MAP=$x timeout -k 10 120 python tools/vision_time.py 64 > gpurun_out/r3d_vis_xcd$x.log 2>&1
done
for r in 0 1; do
  SWARMRL_AMD_RIDE_ALONG=$r timeout -k 10 300 python bench.py --only head,c2,c4 --no-cpu-baseline > gpurun_out/r3d_bench_ride$r.log 2>&1
done
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_PT.so timeout -k 10 120 python tools/build_phases.py 4096 > gpurun_out/r3d_phases.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for x in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    SWARMRL_AMD_XCD_MAP=$x timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ab_r3d/xcd${x}_$c -o run -- python3 tools/run_kernel_time.py 64 > gpurun_out/r3d_pmc_$x$c.log 2>&1
    SWARMRL_AMD_XCD_MAP=$x timeout -k 10 180 rocprofv3 --pmc $c --output-format csv -d gpurun_out/ab_r3d/visxcd${x}_$c -o run -- python3 tools/vision_time.py 64 > gpurun_out/r3d_vpmc_$x$c.log 2>&1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3d_trace -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3d_trace.log 2>&1
SWARMRL_AMD_LIB=$PWD/tools/_variants/lib_pairs6.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3d_trace_pairs6 -o run -- python3 bench.py --only head --no-cpu-baseline > gpurun_out/r3d_trace_pairs6.log 2>&1
timeout -k 10 400 python bench.py --only batched,c5,c3train --no-cpu-baseline > gpurun_out/r3d_bench.log 2>&1

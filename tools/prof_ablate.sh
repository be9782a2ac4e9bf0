set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/trace -o run -- python3 tools/ablate_integrator.py 1,1,0 1,1,1 4,1,0 4,1,1 16,1,0 16,1,1 64,1 256,1 256,0 > gpurun_out/abl/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS --output-format csv -d gpurun_out/abl/pmc -o run -- python3 tools/ablate_integrator.py 64,1 > gpurun_out/abl/pmc.log 2>&1

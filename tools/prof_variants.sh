set -e
cd $GRAFT_REPO_ROOT
for v in default NO_PAIRS NO_BD; do
  if [ $v = default ]; then unset SWARMRL_AMD_LIB; else export SWARMRL_AMD_LIB=$PWD/tools/_variants/libswarmrl_amd_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python3 tools/ablate_integrator.py 1,1,1 1,1,0 1,0 64,1 256,1
done

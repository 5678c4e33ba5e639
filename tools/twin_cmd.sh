cd $GRAFT_REPO_ROOT
for cfg in "TAG=default" "TAG=noslab DTF_DW_SLAB=0" "TAG=nopiggy DTF_SLAB_PIGGYBACK=0" "TAG=nofused DTF_FUSED_BWD=0" "TAG=nograph DTF_HIP_GRAPH=0" "TAG=nrep1 DTF_UNIFORM_WORK=0"; do
  env $cfg timeout -k 10 200 python tools/twin_check.py 2>&1 | grep -v amdgpu.ids || exit 1
done

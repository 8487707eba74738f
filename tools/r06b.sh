cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06u
bash tools/gpu_steps.sh $O \
 "120|probe|python -u tools/greedy_fused_probe.py"

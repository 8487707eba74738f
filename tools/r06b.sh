cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06r
bash tools/gpu_steps.sh $O \
 "400|ab|python -u tools/greedy_ab.py 2 100"

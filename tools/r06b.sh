cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ms
bash tools/gpu_steps.sh $O \
 "300|probe|python -u -m pytest tests/test_graph_guard_gpu.py -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread"

cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06ag
bash tools/gpu_steps.sh $O \
 "600|greedy|python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k 'greedy or gq or remap'"

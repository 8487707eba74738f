cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06x
bash tools/gpu_steps.sh $O \
 "300|remapoff|python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k 'remap'"

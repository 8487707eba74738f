cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06th
bash tools/gpu_steps.sh $O \
 "300|adaptive|python -u -m pytest tests/test_env_parity_gpu.py -m gpu -q -s -p no:cacheprovider --timeout 200 --timeout-method thread -k 'adaptive'" \
 "700|ab|python -u tools/greedy_ab.py 3 100"

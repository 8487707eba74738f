cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06act
bash tools/gpu_steps.sh $O \
 "400|acttests|python -u -m pytest tests/test_actor_gpu.py tests/test_actor_chain_gpu.py tests/test_configs_gpu.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k 'actor or c5'" \
 "300|actor|python -u bench.py --workload actor --steps 20 --warmup 5 --no-cpu-baseline" \
 "300|actor2|python -u bench.py --workload actor --steps 20 --warmup 5 --no-cpu-baseline"

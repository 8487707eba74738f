set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_distributed_gpu.py > gpurun_out/r04a_dist.log 2>&1; e1=$?
tail -3 gpurun_out/r04a_dist.log
if [ $e1 -ne 0 ] && [ $e1 -ne 1 ]; then exit $e1; fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_configs_gpu.py tests/test_env_parity_gpu.py tests/test_actor_gpu.py -k "c5 or four_million or ksteps or greedy" > gpurun_out/r04a_misc.log 2>&1; e2=$?
tail -3 gpurun_out/r04a_misc.log
exit $(( e1 > e2 ? e1 : e2 ))

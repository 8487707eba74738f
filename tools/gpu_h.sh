set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_distributed_gpu.py tests/test_env_parity_gpu.py tests/test_actor_gpu.py tests/test_capi_cpu.py > gpurun_out/h_pytest.log 2>&1; rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/h_pytest.log | tail -8; exit $rc

set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_distributed_gpu.py > gpurun_out/d_pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/d_pytest.log | tail -14; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/kbench.py --houses 1048576,16777216 --variants w32 --rounds 3 > gpurun_out/d_kb0.log 2>&1 || exit $?
MDR_PIPE_SINGLE=1 timeout -k 10 200 python tools/kbench.py --houses 1048576,16777216 --variants w32 --rounds 3 > gpurun_out/d_kb1.log 2>&1 || exit $?
echo graph; grep "w32" gpurun_out/d_kb0.log | tail -2; echo pipeline; grep "w32" gpurun_out/d_kb1.log | tail -2

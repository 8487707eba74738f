set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py tests/test_env_parity_gpu.py tests/test_distributed_gpu.py > gpurun_out/a_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/a_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cp2 -o run -- python3 tools/count_probe.py > gpurun_out/cp2.log 2>&1 || exit $?
python3 tools/count_probe.py --analyze gpurun_out/cp2/run_kernel_trace.csv
timeout -k 10 300 python tools/kbench.py --houses 1048576,16777216 --variants w32 --rounds 3 > gpurun_out/a_kbench.log 2>&1; rc=$?; tail -6 gpurun_out/a_kbench.log; exit $rc

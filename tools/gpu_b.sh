set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py -k "launch_first or begin" > gpurun_out/b_pytest.log 2>&1; rc=$?; tail -8 gpurun_out/b_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/overhead.py --reps 4 --idle-ms 0 > gpurun_out/b_overhead.log 2>&1; rc=$?; tail -8 gpurun_out/b_overhead.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_bench20.log 2>&1; rc=$?; tail -c 600 gpurun_out/b_bench20.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_bench.log 2>&1; rc=$?; tail -c 300 gpurun_out/b_bench.log; exit $rc

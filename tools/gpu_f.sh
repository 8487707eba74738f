set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py tests/test_division_gpu.py > gpurun_out/f_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/f_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/kbench.py --houses 1048576,16777216 --variants w32 --rounds 3 > gpurun_out/f_kb.log 2>&1 || exit $?
grep w32 gpurun_out/f_kb.log | tail -2
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/f_bench.log 2>&1 || exit $?
python3 -c "
import json; l=[x for x in open('gpurun_out/f_bench.log') if x.startswith('{')][-1]; d=json.loads(l); print('bench %.3e kernel %.1f valu %s'%(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['valu']))"

set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py > gpurun_out/e_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/e_pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/e_b20_$i.log 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('gpurun_out/e_b20_$i.log') if x.startswith('{')][-1]; d=json.loads(l); print('bench20 %.3e  %.1f us/call  kernel %.1f'%(d['value'], d['ms_per_step']*20e3, d['roofline']['kernel_avg_us']))"
done
timeout -k 10 200 python tools/overhead.py --reps 4 --idle-ms 0 > gpurun_out/e_ov.log 2>&1 || exit $?
grep "launch-first" gpurun_out/e_ov.log

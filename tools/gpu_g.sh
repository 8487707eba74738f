set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_window_gpu.py tests/test_env_parity_gpu.py tests/test_division_gpu.py > gpurun_out/g_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/g_pytest.log; [ $rc -ne 0 ] && exit $rc
for v in 1 0 1 0; do
  MDR_WIN_COEF=$v timeout -k 10 200 python tools/kbench.py --houses 1048576,16777216 --variants w32 --rounds 3 > gpurun_out/g_kb$v.log 2>&1 || exit $?
  echo "coef=$v"; grep w32 gpurun_out/g_kb$v.log | tail -2
done
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/g_bench.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g_bench20.log 2>&1 || exit $?
python3 -c "
import json
for f in ['gpurun_out/g_bench.log','gpurun_out/g_bench20.log']:
    l=[x for x in open(f) if x.startswith('{')][-1]; d=json.loads(l); print(f, 'value %.3e kernel %.1f frac %.3f'%(d['value'], d['roofline']['kernel_avg_us'], d['roofline']['frac']))"

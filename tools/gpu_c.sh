set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_env_parity_gpu.py -k greedy > gpurun_out/c_pytest.log 2>&1; rc=$?; tail -6 gpurun_out/c_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cg -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/c_greedy.log 2>&1; rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/c_greedy.log; exit $rc; }
python3 -c "
import csv,json
l=[x for x in open('gpurun_out/c_greedy.log') if x.startswith('{')][-1]; d=json.loads(l); print('value %.3e ms_per_step %.4f kernel_avg_us %.1f'%(d['value'],d['ms_per_step'],d['roofline']['kernel_avg_us']))
for r in list(csv.DictReader(open('gpurun_out/cg/run_kernel_stats.csv')))[:12]: print('  ',r['Name'][:90],r['Calls'],'%.1f'%(float(r['AverageNs'])/1e3))
"

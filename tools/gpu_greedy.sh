#!/bin/bash
# greedy: parity tests (histogram select and the sort form), the bench line + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/greedy; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_env_parity_gpu.py tests/test_distributed_gpu.py tests/test_capi_cpu.py -x -q -k "greedy or capi or symbol" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/gsel.json 2> $O/gsel.err || exit $?
for f in gsel; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', round(d['value']/1e9,2), 'Gsteps/s', round(d['ms_per_step']*1e3,1), 'us/tick; greedy+step tick', round(r['kernel_avg_us'],1), 'us')"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats.log 2>&1 || exit $?
echo done

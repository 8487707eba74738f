#!/bin/bash
# driver-style round check: smoke, the full GPU suite, the driver's bench command three times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit $?
  python3 -c "
import json; d=json.loads(open('$O/bench20_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('bench20', round(d['value']/1e9,1), 'Gsteps/s', round(d['timed_region']['wall_s']*1e6,1), 'us; kern', round(r['kernel_avg_us'],1), 'launches', r['launches_timed'], 'frac', round(r['frac'],3), 'valu', r['valu'] and round(r['valu']['frac'],3))"
done
echo done

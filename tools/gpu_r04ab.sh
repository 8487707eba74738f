#!/bin/bash
# r04ab: final check after the greedy helper refactor: smoke(), the driver's 20-step bench line, the full GPU suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04ab; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.log 2>&1 || { tail -5 $O/bench20.log; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench20.log').read().strip().splitlines()[-1]); r=d['roofline']; am=r.get('above_mall') or {}; print('bench20', round(d['value']/1e11,3), 'e11 k', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), 'traffic', r['traffic'], '16M frac', round(am.get('frac',0),3), 'traffic', am.get('traffic'), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
exit $rc

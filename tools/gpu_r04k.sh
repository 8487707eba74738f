#!/bin/bash
# r04: the select launch's phase split (variant build), then the full GPU suite (the ON-mask buffer
# padded to whole 16-wave count blocks), bench20 and the greedy line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04k; mkdir -p $O
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gqt.so timeout -k 10 150 python tools/gq_timing.py > $O/gq_timing.log 2>&1 || { tail -5 $O/gq_timing.log; exit 1; }
cat $O/gq_timing.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -ge 2 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench20_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; am=r.get('above_mall') or {}; print('bench20', round(d['value']/1e11,3), 'e11 k', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), '16M frac', round(am.get('frac',0),3))"
done
timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/greedy.log').read().strip().splitlines()[-1]); print('greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
exit $rc

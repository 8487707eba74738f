#!/bin/bash
# r04: the binned greedy window (per-bin ranking in k_gq_select1): select phase split, the full GPU
# suite, the greedy line at step TPW 2 / 4 / 8 and its kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04l; mkdir -p $O
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gqt.so timeout -k 10 150 python tools/gq_timing.py > $O/gq_timing.log 2>&1 || { tail -5 $O/gq_timing.log; exit 1; }
cat $O/gq_timing.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -ge 2 ] && exit $rc
for tpw in 2 4 8; do
  timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline --step-tpw $tpw > $O/greedy_t$tpw.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_t$tpw.log').read().strip().splitlines()[-1]); print('greedy tpw $tpw', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_greedy -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_greedy.log 2>&1 || exit 1
exit $rc

#!/bin/bash
# r04: the full GPU suite after the block-parallel gap walk, 16-wave count blocks and the K = 16 last
# layer-2 k-step; greedy bench + kernel stats; k_actor A/B (K = 16 vs 32); count timing; bench20;
# the MFMA cycle probe (16x16x32 vs 16x16x16 bf16)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04j; mkdir -p $O
timeout -k 10 60 ./tools/bin/mfma_probe > $O/mfma_probe.log 2>&1 || exit 1
cat $O/mfma_probe.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -ge 2 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_$i.log').read().strip().splitlines()[-1]); print('greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_greedy -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_greedy.log 2>&1 || exit 1
for r in 1 2; do for v in hip a32; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 120 python tools/actor_kbench.py --reps 20 > $O/akb_${v}_$r.log 2>&1 || exit 1
  echo "$v: $(tail -n 1 $O/akb_${v}_$r.log)"
done; done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so timeout -k 10 120 python tools/count_timing.py --ticks 20 > $O/ct20.log 2>&1 || exit 1
cat $O/ct20.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/bench20_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; am=r.get('above_mall') or {}; print('bench20', round(d['value']/1e11,3), 'e11 k', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), '16M frac', round(am.get('frac',0),3))"
done
timeout -k 10 200 python bench.py --workload actor --steps 50 --warmup 5 --no-cpu-baseline > $O/actor.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/actor.log').read().strip().splitlines()[-1]); print('actor', '%.3e' % d['value'], 'k_actor us', round(d['roofline']['kernel_avg_us'],1))"
exit $rc

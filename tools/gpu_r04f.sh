#!/bin/bash
# r04 check: count-kernel timing split, bench lines (20-step x3, greedy, actor), the actor phase
# profile, then the full GPU suite (the call's limit is 1200 s: the suite gets what is left)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04f; mkdir -p $O
for t in 20 1; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so timeout -k 10 120 python tools/count_timing.py --ticks $t > $O/ct$t.log 2>&1 || { tail -5 $O/ct$t.log; exit 1; }
  cat $O/ct$t.log
done
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench20_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; am=r.get('above_mall') or {}; print('bench20', round(d['value']/1e11,3), 'e11 k', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), '16M k', round(am.get('kernel_avg_us',0),1), 'frac', round(am.get('frac',0),3))"
done
timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/greedy.log').read().strip().splitlines()[-1]); print('greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
timeout -k 10 200 python bench.py --workload actor --steps 50 --warmup 5 --no-cpu-baseline > $O/actor.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/actor.log').read().strip().splitlines()[-1]); print('actor', '%.3e' % d['value'], 'k_actor us', round(d['roofline']['kernel_avg_us'],1))"
timeout -k 10 120 python tools/actor_profile.py > $O/actor_prof.log 2>&1 || exit 1
cat $O/actor_prof.log
# (the r04f run also timed A/B builds — 8 waves per block, the rounded-hi split — built with
#  python marl-demandresponse_amd/build_ext.py --variant aw8 MDR_ACTOR_MAXW=8 / --variant arne MDR_ACTOR_RNE_SPLIT;
#  results in profiles/r04f_actor_ab.log)
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
exit $rc

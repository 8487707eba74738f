#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04e; mkdir -p $O
for t in 20 1; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so timeout -k 10 120 python tools/count_timing.py --ticks $t > $O/ct$t.log 2>&1 || { tail -5 $O/ct$t.log; exit 1; }
  cat $O/ct$t.log
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_window_gpu.py tests/test_configs_gpu.py tests/test_env_parity_gpu.py tests/test_distributed_gpu.py -k "not actor" > $O/win.log 2>&1 || { tail -30 $O/win.log; exit 1; }
tail -2 $O/win.log
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20_$i.log 2>&1 || exit 1
  python3 -c "import json,sys; d=json.loads(open('$O/bench20_$i.log').read().strip().splitlines()[-1]); r=d['roofline']; am=r.get('above_mall') or {}; print('bench20', round(d['value']/1e11,3), 'e11 k', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), '16M k', round(am.get('kernel_avg_us',0),1), 'frac', round(am.get('frac',0),3))"
done
timeout -k 10 300 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/greedy.log').read().strip().splitlines()[-1]); print('greedy', d['ms_per_step']*1e3, 'us/tick; kernel', d['roofline']['kernel_avg_us'], d.get('greedy_select'))"

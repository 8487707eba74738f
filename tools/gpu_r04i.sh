#!/bin/bash
# r04: the greedy select as its own 2-block launch (k_gq_select1) and the count kernel at 4 vs 16
# waves per block: greedy + window parity tests, greedy bench, count timing split, bench20 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_env_parity_gpu.py tests/test_window_gpu.py tests/test_distributed_gpu.py -k "greedy or window or rollout" > $O/pytest.log 2>&1; rc=$?
tail -n 2 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy_$i.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_$i.log').read().strip().splitlines()[-1]); print('greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_greedy -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_greedy.log 2>&1 || exit 1
for v in cwt:4 cwt16:16; do
  lib=${v%%:*}; w=${v##*:}
  for t in 20 1; do
    MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$lib.so timeout -k 10 120 python tools/count_timing.py --ticks $t --waves $w > $O/ct_${lib}_$t.log 2>&1 || { tail -5 $O/ct_${lib}_$t.log; exit 1; }
    cat $O/ct_${lib}_$t.log
  done
done
for r in 1 2; do for v in hip cw16; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --above-mall-houses 0 > $O/b20_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/b20_${v}_$r.log').read().strip().splitlines()[-1]); print('$v bench20', round(d['value']/1e11,3), 'e11')"
done; done
timeout -k 10 60 ./tools/bin/mfma_probe > $O/mfma_probe.log 2>&1 || exit 1
cat $O/mfma_probe.log
exit 0

#!/bin/bash
# r04: greedy A/B — the binned one-block select (default build) vs every call through the 256-block
# k_gq_select with the block-parallel gap walk (gs256); greedy parity tests on the gs256 build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04n; mkdir -p $O
for r in 1 2; do for v in hip gs256; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_${v}_$r.log').read().strip().splitlines()[-1]); print('$v greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2), d.get('greedy_select'))"
done; done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gs256.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_gs256 -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_gs256.log 2>&1 || exit 1
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gs256.so timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_env_parity_gpu.py -k greedy > $O/pytest_gs256.log 2>&1; rc=$?
tail -n 1 $O/pytest_gs256.log
exit $rc

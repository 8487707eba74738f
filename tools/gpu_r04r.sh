#!/bin/bash
# r04: greedy select grid (256 / 64 / 32 blocks) and histogram copies (8 / 2) A/B; greedy parity tests
# on the 32-block / 2-copy build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04r; mkdir -p $O
for r in 1 2; do for v in hip sb32 sb64 cp2 sb32cp2; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_${v}_$r.log').read().strip().splitlines()[-1]); print('$v greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2))"
done; done
for v in sb32 sb32cp2; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$v -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_$v.log 2>&1 || exit 1
done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_sb32cp2.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_env_parity_gpu.py tests/test_distributed_gpu.py -k greedy > $O/pytest_sb32cp2.log 2>&1; rc=$?
tail -n 1 $O/pytest_sb32cp2.log
exit $rc

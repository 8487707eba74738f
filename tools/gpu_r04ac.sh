#!/bin/bash
# r04ac: k_gq_compact with its bin counts and window keys loaded up front (default) against the r04 order (libmdr_late.so), alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04ac; mkdir -p $O
L=marl-demandresponse_amd/mdr_amd
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests -k "greedy" > $O/pytest_greedy.log 2>&1 || { grep -E "^(FAILED|ERROR)" $O/pytest_greedy.log; tail -3 $O/pytest_greedy.log; exit 1; }
tail -n 1 $O/pytest_greedy.log
for k in 1 2 3; do
  for v in hip late; do
    MDR_LIB=$L/libmdr_$v.so timeout -k 10 200 python bench.py --workload greedy --steps 200 --warmup 20 --no-cpu-baseline > $O/greedy_${v}_$k.log 2>&1 || { tail -5 $O/greedy_${v}_$k.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/greedy_${v}_$k.log').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step']*1e3,2), 'us/tick', '%.4g' % d['value'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o greedy -- python3 bench.py --workload greedy --steps 200 --warmup 20 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/greedy_kernel_stats.csv; head -6 $O/greedy_kernel_stats.csv | cut -c1-160

#!/bin/bash
# r04y: the greedy stages after the helper refactor (k_gq_bins / k_gq_compact / k_gq_select bodies
# as shared device functions): the greedy parity tests and the C3 line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04y; mkdir -p $O
timeout -k 10 400 python -u -m pytest -v --timeout 150 --timeout-method thread -m gpu tests -k "greedy" > $O/pytest_greedy.log 2>&1 || { grep -E "^(FAILED|ERROR)" $O/pytest_greedy.log; tail -3 $O/pytest_greedy.log; exit 1; }
tail -n 1 $O/pytest_greedy.log
for k in 1 2; do
  timeout -k 10 200 python bench.py --workload greedy --steps 200 --warmup 20 > $O/greedy_$k.log 2>&1 || { tail -5 $O/greedy_$k.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/greedy_$k.log').read().strip().splitlines()[-1]); print('greedy', d['ms_per_step']*1e3, 'us/tick', d['value'])"
done

#!/bin/bash
# r04: k_actor without the per-tile vmcnt(0) in front of layer 1 (the next tile's prefetch now lands
# beside the MFMAs): kernel bench, phase profile, C5 bench line, actor tests + full suite
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04t; mkdir -p $O
for p in bf16x3 bf16 fp32; do
  timeout -k 10 120 python tools/actor_kbench.py --reps 20 --precision $p > $O/akb_$p.log 2>&1 || exit 1
  tail -n 1 $O/akb_$p.log
done
timeout -k 10 120 python tools/actor_profile.py > $O/actor_prof.log 2>&1 || exit 1
cat $O/actor_prof.log
timeout -k 10 200 python bench.py --workload actor --steps 50 --warmup 5 --no-cpu-baseline > $O/actor.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('$O/actor.log').read().strip().splitlines()[-1]); print('actor', '%.3e' % d['value'], 'k_actor us', round(d['roofline']['kernel_avg_us'],1))"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
exit $rc

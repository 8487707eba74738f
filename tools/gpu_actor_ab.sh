#!/bin/bash
# actor (C5) A/B: default library vs a build variant (MDR_LIB=...): bench lines + phase profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/actor_ab; mkdir -p $O
for v in default ${VARIANTS:-prio}; do
  L=""; [ "$v" != default ] && L="MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so"
  for i in 1 2; do
    timeout -k 10 300 env $L python bench.py --workload actor --steps 50 --warmup 5 --no-cpu-baseline > $O/${v}_$i.json 2> $O/${v}_$i.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', round(d['value']/1e9,2), 'Gsteps/s', round(d['ms_per_step']*1e3,1), 'us/tick; actor', round(r['kernel_avg_us'],1), 'us; mfma frac', round(r['frac'],3))"
  done
  timeout -k 10 120 env $L python tools/actor_profile.py > $O/prof_$v.log 2>&1 || exit $?
  grep -v amdgpu $O/prof_$v.log
done
echo done

#!/bin/bash
# A/B of the rollout path: 20-step (driver) and 2000-step bench lines under variants.
# (wt20/wt2000 need the write-through variant built first: python marl-demandresponse_amd/build_ext.py --variant wt MDR_REWARD_WT)
#   default lib, launch-first graph | MDR_NO_LAUNCH_FIRST | --graph off | write-through reward lib
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/ab; mkdir -p $O
one() {  # name env... -- bench args
  local name=$1; shift
  timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']
print('%-28s %6.1f Gsteps/s  wall %7.1f us  kern %6.1f us  graph/launch %s' % ('$name', d['value']/1e9, d['timed_region']['wall_s']*1e6, r['kernel_avg_us'], r.get('graph_us_per_launch')))"
}
B="python bench.py --no-cpu-baseline"
for i in 1 2 3; do
  one lf20_$i $B --steps 20 --warmup 5
  one nolf20_$i MDR_NO_LAUNCH_FIRST=1 $B --steps 20 --warmup 5
  one nograph20_$i $B --steps 20 --warmup 5 --graph off
  one wt20_$i MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_wt.so $B --steps 20 --warmup 5
done
one lf2000 $B --steps 2000 --warmup 200
one nograph2000 $B --steps 2000 --warmup 200 --graph off
one wt2000 MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_wt.so $B --steps 2000 --warmup 200
echo done

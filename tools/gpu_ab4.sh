#!/bin/bash
# sharded single-window begin (RCCL world 1): tests + 20-step bench lines with / without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/ab7; mkdir -p $O
one() {
  local name=$1; shift
  timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('%-28s %6.1f Gsteps/s  wall %7.1f us  kern %6.1f us  %s' % ('$name', d['value']/1e9, d['timed_region']['wall_s']*1e6, r['kernel_avg_us'], d['config']['sharded_pipeline']))"
}
B="python bench.py --no-cpu-baseline --comm rccl"
for i in 1 2 3 4 5 6; do
  one r20_$i $B --steps 20 --warmup 5 --trace
  one r20noka_$i MDR_NO_KA=1 $B --steps 20 --warmup 5 --trace
done
grep -h "trace (us" $O/*.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu-baseline --comm rccl --steps 20 --warmup 5 > $O/kt.log 2>&1 || exit $?
echo done

#!/bin/bash
# window tests + 20/2000-step bench lines of the default (direct, kernarg drivers) vs the graph policy
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/ab2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_window_gpu.py tests/test_env_parity_gpu.py tests/test_distributed_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
one() {
  local name=$1; shift
  timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']
print('%-28s %6.1f Gsteps/s  wall %7.1f us  kern %6.1f us  graph/launch %s' % ('$name', d['value']/1e9, d['timed_region']['wall_s']*1e6, r['kernel_avg_us'], r.get('graph_us_per_launch')))"
}
B="python bench.py --no-cpu-baseline"
for i in 1 2 3 4; do
  one def20_$i $B --steps 20 --warmup 5 --trace
  one graph20_$i $B --steps 20 --warmup 5 --graph on
done
grep trace $O/def20_*.err
one def2000 $B --steps 2000 --warmup 200
one graph2000 $B --steps 2000 --warmup 200 --graph on
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit $?
echo done

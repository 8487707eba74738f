#!/bin/bash
# launch policies: tests, cold-call host phases, 20/2000-step bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/ab5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_window_gpu.py tests/test_env_parity_gpu.py tests/test_distributed_gpu.py tests/test_integration_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 env MDR_NO_KA=1 python tools/cold_probe.py --kernarg > $O/cold_noka.log 2>&1 || exit $?
timeout -k 10 120 python tools/cold_probe.py --kernarg > $O/cold_ka.log 2>&1 || exit $?
grep rep $O/cold_*.log
one() {
  local name=$1; shift
  timeout -k 10 200 env "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed rc=$?"; tail -5 $O/$name.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$name.json')); r=d['roofline']
print('%-28s %6.1f Gsteps/s  wall %7.1f us  kern %6.1f us' % ('$name', d['value']/1e9, d['timed_region']['wall_s']*1e6, r['kernel_avg_us']))"
}
B="python bench.py --no-cpu-baseline"
for i in 1 2 3 4 5; do
  one ka20_$i $B --steps 20 --warmup 5
  one noka20_$i MDR_NO_KA=1 $B --steps 20 --warmup 5
done
one ka2000 $B --steps 2000 --warmup 200
one noka2000 MDR_NO_KA=1 $B --steps 2000 --warmup 200
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit $?
echo done

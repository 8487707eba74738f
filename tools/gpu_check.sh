#!/bin/bash
# One GPU session: smoke -> GPU tests -> benches -> rocprofv3 kernel trace (STEPS=comma list).
# Every GPU step has its own time limit; a fault / abort / timeout (rc >= 124) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TZ=UTC
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name, stopping"; exit $rc; fi
  return $rc
}
has() { [[ ",${STEPS}," == *",$1,"* ]]; }
STEPS=${STEPS:-smoke,pytest,bench,prof}
has smoke && { step smoke 420 python __graft_entry__.py smoke || true; }
has pytest && { step pytest_gpu 900 python -u -m pytest ${PYTEST_ARGS:-tests} -m gpu -v --maxfail=20 -p no:cacheprovider --timeout 120 --timeout-method thread || true; }
has bench20 && { step bench20 300 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} || true; }
has bench && { step bench 600 python bench.py ${BENCH_ARGS:-} || true; }
has kbench && { step kbench 600 python tools/kbench.py ${KBENCH_ARGS:-} || true; }
has greedy && { step bench_greedy 600 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline || true; }
has actor && { step bench_actor 600 python bench.py --workload actor --steps 200 --warmup 20 --no-cpu-baseline || true; }
if has prof; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python3 bench.py ${PROF_ARGS:---steps 20 --warmup 5 --no-cpu-baseline} || true
fi
echo "== done"

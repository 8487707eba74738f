#!/bin/bash
# One GPU session: smoke -> GPU tests -> bench -> rocprofv3 kernel trace.
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
STEPS=${STEPS:-smoke,pytest,bench,prof}
[[ $STEPS == *smoke* ]] && { step smoke 420 python __graft_entry__.py smoke || true; }
[[ $STEPS == *pytest* ]] && { step pytest_gpu 900 python -u -m pytest tests -m gpu -v --maxfail=20 -p no:cacheprovider --timeout 120 --timeout-method thread || true; }
[[ $STEPS == *bench* ]] && { step bench 600 python bench.py ${BENCH_ARGS:-} || true; }
if [[ $STEPS == *prof* ]]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 500 --warmup 100 --no-cpu-baseline || true
fi
echo "== done"

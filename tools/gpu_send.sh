#!/bin/bash
# Local wrapper: rebuild libmdr_hip.so (stop on a build error, so a stale library never travels),
# then run tools/gpu_check.sh on an MI355X box through gpurun.  Env (STEPS, KBENCH_ARGS, ...) is
# forwarded.  Usage: STEPS=pytest,bench20 tools/gpu_send.sh [gpurun-timeout-s] [extra shell cmd]
set -u
cd "$(dirname "$0")/.."
python marl-demandresponse_amd/build_ext.py > /tmp/mdr_build.log 2>&1 || { tail -20 /tmp/mdr_build.log; echo "BUILD FAILED"; exit 1; }
T=${1:-900}
EXTRA=${2:-true}
VARS="STEPS='${STEPS:-pytest}' PYTEST_ARGS='${PYTEST_ARGS:-tests}' KBENCH_ARGS='${KBENCH_ARGS:-}' BENCH_ARGS='${BENCH_ARGS:-}' PROF_ARGS='${PROF_ARGS:---steps 20 --warmup 5 --no-cpu-baseline}'"
timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- "export $VARS; bash tools/gpu_check.sh && $EXTRA"

#!/bin/bash
# Round-end style check on one box: smoke, the full GPU suite, then tools/profile_r02.sh (bench
# line, rocprofv3 stats of the driver's bench command and of the greedy / actor workloads, PMC).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/r_smoke.log 2>&1 || { tail -20 gpurun_out/r_smoke.log; exit 1; }
tail -1 gpurun_out/r_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r_pytest.log
grep -E "FAILED|ERROR" gpurun_out/r_pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
WORKLOADS="${WORKLOADS-greedy actor}" bash tools/profile_r02.sh

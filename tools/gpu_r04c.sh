#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_window_gpu.py tests/test_actor_chain_gpu.py tests/test_actor_gpu.py > gpurun_out/r04c/actor.log 2>&1; rc=$?
tail -3 gpurun_out/r04c/actor.log; grep -E "max \|p" gpurun_out/r04c/actor.log | head -40
[ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_distributed_gpu.py -k actor > gpurun_out/r04c/dist_actor.log 2>&1; rc2=$?
tail -3 gpurun_out/r04c/dist_actor.log
[ $rc2 -ge 2 ] && exit $rc2
bash tools/count_pmc.sh gpurun_out/r04c/count || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04c/bench20_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r04c/bench20_$i.log | cut -c1-150
done
exit $(( rc > rc2 ? rc : rc2 ))

#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out/r04b
bash tools/count_pmc.sh gpurun_out/r04b/count || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04b/bench20_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/r04b/bench20_$i.log | cut -c1-200
done

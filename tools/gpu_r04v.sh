#!/bin/bash
# r04 final counters: k_count_window (16-wave blocks, 20 ticks: durations vs ticks + SQ passes,
# tools/count_pmc.sh) and k_actor (tools/pmc_actor.sh) on the final build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 500 bash tools/count_pmc.sh $O/count > $O/count.log 2>&1 || { tail -5 $O/count.log; exit 1; }
cat $O/count.log
timeout -k 10 400 bash tools/pmc_actor.sh $O/pmc_actor bf16x3 > $O/pmc_actor.log 2>&1 || { tail -5 $O/pmc_actor.log; exit 1; }
cat $O/pmc_actor.log

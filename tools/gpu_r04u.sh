#!/bin/bash
# r04: HBM bytes of the greedy tick's kernels (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the
# C3 bench, each pass its own run, nothing else traced) -> tools/greedy_pmc_summary.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04u; mkdir -p $O
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $group --output-format csv -d $O/p$i -o run -- python3 bench.py --workload greedy --steps 20 --warmup 3 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
  echo "pass $i ok"
done

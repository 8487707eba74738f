#!/bin/bash
# rocprofv3 counter passes over the C3 greedy bench (one counter group per pass; never combined with
# sys/runtime traces), summed per tick by tools/greedy_pmc_summary.py.  Usage: tools/pmc_greedy.sh OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_greedy}
mkdir -p "$OUT"
CMD="python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline"
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" ; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run -- $CMD \
    > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i ($group) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pmc pass $i ok"
done

#!/bin/bash
# k_count_window evidence: kernel durations vs ticks (rocprofv3 kernel trace
# of tools/count_probe.py), then SQ counter passes on the 20-tick random count (one group per
# pass, nothing else traced).  Usage: tools/count_pmc.sh OUTDIR [HOUSES]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/count}; H=${2:-1048576}
mkdir -p "$OUT"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- \
  python3 tools/count_probe.py --houses $H > "$OUT/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
python3 tools/count_probe.py --analyze "$(ls $OUT/trace/*/run_kernel_trace.csv $OUT/trace/run_kernel_trace.csv 2>/dev/null | head -1)" \
  > "$OUT/durations.txt" && cat "$OUT/durations.txt"
export CP_TICKS=20 CP_MODES=random
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run -- \
    python3 tools/count_probe.py --houses $H > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pmc pass $i ok"
done

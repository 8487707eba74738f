#!/bin/bash
# rocprofv3 counter passes over tools/actor_kbench.py (k_actor alone at 1M houses): MFMA / VALU /
# LDS / stall counters, one group per pass, each its own run (never combined with traces).
# Usage: tools/pmc_actor.sh OUTDIR [PRECISION]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/pmc_actor}; PREC=${2:-bf16x3}
mkdir -p "$OUT"
CMD="python3 tools/actor_kbench.py --houses 1048576 --precision $PREC --reps 5"
i=0
for group in \
  "SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVES" \
  "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
  "GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run -- $CMD \
    > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i ($group) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pmc pass $i ok"
done

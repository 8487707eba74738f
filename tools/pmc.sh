#!/bin/bash
# rocprofv3 counter passes over tools/kbench.py (one counter group per pass; never combined with
# sys/runtime traces).  Usage: tools/pmc.sh HOUSES VARIANT OUTDIR
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
H=${1:-16777216}; V=${2:-w32}; OUT=${3:-gpurun_out/pmc}
mkdir -p "$OUT"
CMD="python3 tools/kbench.py --houses $H --variants $V --ticks 128 --rounds 1"
i=0
for group in \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ TCC_EA0_WRREQ_DRAM" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES" \
  "SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $group --output-format csv -d "$OUT/p$i" -o run -- $CMD \
    > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i ($group) failed rc=$?"; tail -5 "$OUT/p$i.log"; exit 1; }
  echo "pmc pass $i ok"
done

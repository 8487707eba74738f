#!/bin/bash
# rocprofv3 counter passes (one counter group per pass; no sys/runtime traces with --pmc).
# Usage: tools/pmc.sh HOUSES VARIANT OUTTAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
H=${1:-16777216}; V=${2:-fast2}; TAG=${3:-pmc}
CMD="python3 tools/kbench.py --houses $H --variants $V --launches 20 --rounds 1"
i=0
for group in \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_VMEM" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM TCC_HIT TCC_MISS" \
  "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_BRANCH" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d gpurun_out/$TAG/p$i -o run -- $CMD \
    > gpurun_out/$TAG/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc done

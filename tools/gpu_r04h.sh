#!/bin/bash
# r04 HBM-honest counters of the benched window kernel: PMC passes (tools/pmc.sh: FETCH/WRITE
# sizes, EA requests incl. DRAM, SQ instruction and stall counters) at 1M, 4M and 16M houses.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04h; mkdir -p $O
for H in ${PMC_SIZES:-1048576 4194304 16777216}; do
  echo "== pmc $H"
  timeout -k 10 400 bash tools/pmc.sh $H w32 $O/pmc_$H > $O/pmc_$H.log 2>&1 || { tail -5 $O/pmc_$H.log; exit 1; }
  tail -1 $O/pmc_$H.log
done
echo "== done"

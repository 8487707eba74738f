#!/bin/bash
# r04: the select launch's phase split with its shader clock, then the round profile (tools/gpu_r04h.sh:
# bench line, kernel stats, PMC at 1M / 4M / 16M houses)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04m; mkdir -p $O
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gqt.so timeout -k 10 150 python tools/gq_timing.py > $O/gq_timing.log 2>&1 || { tail -5 $O/gq_timing.log; exit 1; }
cat $O/gq_timing.log
bash tools/gpu_r04h.sh

#!/bin/bash
# r04: k_actor's output layer in fp64 FMAs (af64: they issue beside the MFMAs) vs fp32 A/B; the actor
# tests on the af64 build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04s; mkdir -p $O
for r in 1 2 3; do for v in hip af64; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 120 python tools/actor_kbench.py --reps 20 > $O/akb_${v}_$r.log 2>&1 || exit 1
  echo "$v: $(tail -n 1 $O/akb_${v}_$r.log)"
done; done
for v in hip af64; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 120 python tools/actor_kbench.py --reps 20 --precision bf16 > $O/akb16_${v}.log 2>&1 || exit 1
  echo "$v: $(tail -n 1 $O/akb16_${v}.log)"
done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_af64.so timeout -k 10 500 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_actor_gpu.py tests/test_actor_chain_gpu.py tests/test_configs_gpu.py -k "actor or c5" > $O/pytest_af64.log 2>&1; rc=$?
tail -n 1 $O/pytest_af64.log; grep -E "FAILED|max \|p - p_torch\|" $O/pytest_af64.log | head -30
exit $rc

#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out/r04d
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so timeout -k 10 120 python tools/count_timing.py --ticks 20 > gpurun_out/r04d/ct20.log 2>&1 || { tail -5 gpurun_out/r04d/ct20.log; exit 1; }
cat gpurun_out/r04d/ct20.log
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwt.so timeout -k 10 120 python tools/count_timing.py --ticks 1 > gpurun_out/r04d/ct1.log 2>&1 || { tail -5 gpurun_out/r04d/ct1.log; exit 1; }
cat gpurun_out/r04d/ct1.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_actor_chain_gpu.py tests/test_actor_gpu.py > gpurun_out/r04d/actor.log 2>&1; rc=$?
tail -3 gpurun_out/r04d/actor.log; grep -E "max \|p" gpurun_out/r04d/actor.log | head -40
exit $rc

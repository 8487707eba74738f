#!/bin/bash
# r04: count kernel as a tile loop (TPW tiles per wave) vs one tile per wave: timing split, bench20
# A/B, the window tests on the TPW-2 build; then the full suite and smoke() on the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04o; mkdir -p $O
for v in cwt:16:1 cwtp2:16:2 cwtp4w8:8:4; do
  IFS=: read lib w tp <<< "$v"
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$lib.so timeout -k 10 120 python tools/count_timing.py --ticks 20 --waves $w --tpw $tp > $O/ct_$lib.log 2>&1 || { tail -5 $O/ct_$lib.log; exit 1; }
  cat $O/ct_$lib.log
done
for r in 1 2; do for v in hip cwp2 cwp4w8; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --above-mall-houses 0 > $O/b20_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/b20_${v}_$r.log').read().strip().splitlines()[-1]); print('$v bench20', round(d['value']/1e11,3), 'e11')"
done; done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_cwp2.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_window_gpu.py > $O/pytest_cwp2.log 2>&1; echo "cwp2 window tests rc=$?"; tail -n 1 $O/pytest_cwp2.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1; rc=$?
tail -n 1 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -n 3 $O/smoke.log
exit $rc

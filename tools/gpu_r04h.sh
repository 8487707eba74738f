#!/bin/bash
# r04 round profile: the default bench line (with its CPU baseline), rocprofv3 --kernel-trace --stats
# of the driver's bench command, and the HBM-honest counters of the benched window kernel (PMC
# passes, tools/pmc.sh) at 1M, 4M and 16M houses.  tools/collect_profiles.py r04h gpurun_out/r04h
# copies them into profiles/ and profiles/pmc_traffic.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -n 1 $O/bench.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/stats.log 2>&1 || exit 1
for H in ${PMC_SIZES:-1048576 4194304 16777216}; do
  echo "== pmc $H"
  timeout -k 10 400 bash tools/pmc.sh $H w32 $O/pmc_$H > $O/pmc_$H.log 2>&1 || { tail -5 $O/pmc_$H.log; exit 1; }
  tail -n 1 $O/pmc_$H.log
done
echo "== done"

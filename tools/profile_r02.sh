#!/bin/bash
# Round profile: bench line, rocprofv3 --kernel-trace --stats of the driver's bench command, and
# PMC passes for the dominant kernel (k_step_window) at 1M / 4M / 16M houses.  Outputs under
# gpurun_out/round/ (tools/collect_profiles.py copies the summaries into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
OUT=gpurun_out/round
mkdir -p $OUT
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log"; [ $rc -ge 124 ] && exit $rc; return $rc; }
[ -n "${SKIP_BENCH:-}" ] || step bench 600 python bench.py ${BARGS:-} || exit 1
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
# the other workloads' kernels (greedy: hipCUB sort + scan + walk; actor: k_actor + k_obs)
for W in ${WORKLOADS:-}; do
  step bench_$W 600 python bench.py --workload $W --steps 50 --warmup 5 --no-cpu-baseline || exit 1
  step stats_$W 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$W -o run -- python3 bench.py --workload $W --steps 50 --warmup 5 --no-cpu-baseline || exit 1
done
for H in ${PMC_SIZES:-1048576 4194304 16777216}; do
  step pmc_$H 900 bash tools/pmc.sh $H w32 $OUT/pmc_$H || exit 1
done
echo "== done"

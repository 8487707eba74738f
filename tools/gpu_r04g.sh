#!/bin/bash
# r04 profiles: rocprofv3 --kernel-trace --stats of the driver's bench command and of the greedy /
# actor workloads; counter passes (each its own run, never with traces) for the greedy kernels and
# k_actor.  Outputs under gpurun_out/r04g (tools/collect_profiles.py copies them into profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04g; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$O/$name.log"; return $rc; }
step stats 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit 1
for W in greedy actor; do
  step stats_$W 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$W -o run -- python3 bench.py --workload $W --steps 50 --warmup 5 --no-cpu-baseline || exit 1
done
i=0
for group in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  step pmc_greedy_p$i 120 rocprofv3 --pmc $group --output-format csv -d $O/pmc_greedy/p$i -o run -- python3 bench.py --workload greedy --steps 20 --warmup 3 --no-cpu-baseline || exit 1
done
step pmc_actor 400 bash tools/pmc_actor.sh $O/pmc_actor bf16x3 || exit 1
echo "== done"

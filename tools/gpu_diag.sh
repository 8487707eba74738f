#!/bin/bash
# One diagnostic session: the greedy select probe, the actor phase profile + kernel bench + counter
# passes, then tools/profile_r02.sh (bench line, rocprofv3 stats, workloads, PMC).  Each step has
# its own time limit; a timeout / signal ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 4 "gpurun_out/$name.log"; [ $rc -ge 124 ] && exit $rc; return 0; }
run gq_probe 180 python tools/gq_probe.py
run actor_prof 180 python tools/actor_profile.py
run actor_kbench 180 python tools/actor_kbench.py
[ -n "${SKIP_PMC_ACTOR:-}" ] || { timeout -k 10 400 bash tools/pmc_actor.sh gpurun_out/pmc_actor || exit $?; }
[ -n "${SKIP_ROUND:-}" ] || WORKLOADS="${WORKLOADS-greedy actor}" PMC_SIZES="${PMC_SIZES-1048576}" bash tools/profile_r02.sh

#!/bin/bash
# Round profile: bench line + rocprofv3 kernel-trace/stats of the same command + PMC traffic
# passes for the dominant kernel (k_step) at the bench size.  Outputs under gpurun_out/round/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
OUT=gpurun_out/round
mkdir -p $OUT
BARGS=${BARGS:---steps 1000 --warmup 100}
step() { local name=$1 secs=$2; shift 2; echo "== $name"; timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log"; [ $rc -ge 124 ] && exit $rc; return $rc; }
step bench 600 python bench.py $BARGS || exit 1
step stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $BARGS --no-cpu-baseline || exit 1
step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline || exit 1
step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline || exit 1
step pmc_dram 600 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM TCC_EA0_RDREQ_32B TCC_EA0_RDREQ --output-format csv -d $OUT/pmc_dram -o run -- python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline || exit 1
echo "== done"

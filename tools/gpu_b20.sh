#!/bin/bash
# 20-step timed-region probe: phase breakdown (tools/overhead.py), repeated driver-style bench
# lines, and the device timeline of one bench run (rocprofv3 kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
mkdir -p gpurun_out/b20
timeout -k 10 180 python tools/overhead.py --reps 6 > gpurun_out/b20/overhead.log 2>&1 || exit $?
for i in 1 2 3 4; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --trace > gpurun_out/b20/bench_$i.json 2> gpurun_out/b20/bench_$i.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b20/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b20/kt.log 2>&1 || exit $?
echo done

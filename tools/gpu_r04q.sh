#!/bin/bash
# r04: rehearsal of the driver's multi-GPU bench line — 2 ranks sharing cuda:0 over gloo with the
# library's C loops (weak and strong scaling), then the default 1-GPU line for comparison
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04q; mkdir -p $O
for sc in weak strong; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --comm host --scaling $sc --steps 20 --warmup 5 --no-cpu-baseline --above-mall-houses 0 > $O/bench_w2_$sc.log 2>&1; rc=$?
  echo "w2 $sc rc=$rc"
  grep '^{' $O/bench_w2_$sc.log | tail -n 1 | cut -c1-600
  [ $rc -ge 124 ] && exit $rc
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --comm host --steps 2000 --warmup 200 --no-cpu-baseline --above-mall-houses 0 > $O/bench_w2_2000.log 2>&1; echo "w2 2000 rc=$?"
grep '^{' $O/bench_w2_2000.log | tail -n 1 | cut -c1-300
exit 0

#!/bin/bash
# r04: greedy grid sizes A/B — compact houses per block (4096 vs 2048) and the bins grid (256 vs 512
# blocks); per-kernel stats of each; greedy parity tests on the 2048 / 512 build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
O=gpurun_out/r04p; mkdir -p $O
for r in 1 2; do for v in hip gs2k gp512 gs2kp512; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 python bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/greedy_${v}_$r.log 2>&1 || exit 1
  python3 -c "import json; d=json.loads(open('$O/greedy_${v}_$r.log').read().strip().splitlines()[-1]); print('$v greedy', round(d['ms_per_step']*1e3,2), 'us/tick; kernel', round(d['roofline']['kernel_avg_us'],2))"
done; done
for v in hip gs2kp512; do
  MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$v -o run -- python3 bench.py --workload greedy --steps 50 --warmup 5 --no-cpu-baseline > $O/stats_$v.log 2>&1 || exit 1
done
MDR_LIB=marl-demandresponse_amd/mdr_amd/libmdr_gs2kp512.so timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_env_parity_gpu.py tests/test_distributed_gpu.py -k greedy > $O/pytest_gs2kp512.log 2>&1; rc=$?
tail -n 1 $O/pytest_gs2kp512.log
# rehearsal of the driver's multi-GPU bench line: 2 ranks sharing cuda:0 over gloo + the library's C loops
for sc in weak strong; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --comm host --scaling $sc --steps 20 --warmup 5 --no-cpu-baseline --above-mall-houses 0 > $O/bench_w2_$sc.log 2>&1; echo "w2 $sc rc=$?"
  grep '^{' $O/bench_w2_$sc.log | tail -n 1 | cut -c1-400
done
exit $rc

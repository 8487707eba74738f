cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0
O=gpurun_out/r06s
bash tools/gpu_steps.sh $O \
 "600|ab|python -u tools/greedy_ab.py 3 100" \
 "300|actor|python -u bench.py --workload actor --steps 20 --warmup 5 --no-cpu-baseline" \
 "300|actorprof|rocprofv3 --kernel-trace --stats --output-format csv -d $O/actorprof -o actor -- python bench.py --workload actor --steps 10 --warmup 3 --no-cpu-baseline" \
 "200|rccl|rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/rccl -o run -- python bench.py --comm rccl --houses 131072 --steps 200 --chunk 20 --warmup 40 --no-cpu-baseline --kernel-ticks 32 --kernel-reps 1 --kernel-warm-ticks 32" \
 "200|unsh|rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/unsh -o run -- python bench.py --comm none --houses 131072 --steps 200 --chunk 20 --warmup 40 --no-cpu-baseline --kernel-ticks 32 --kernel-reps 1 --kernel-warm-ticks 32" \
 "300|guard|python -u -m pytest -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_graph_guard_gpu.py tests/test_actor_gpu.py"

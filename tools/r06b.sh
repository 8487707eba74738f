cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06y
bash tools/gpu_steps.sh $O \
 "300|greedybench|python -u bench.py --workload greedy --steps 20 --warmup 5 --no-cpu-baseline" \
 "300|prof|rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o greedy -- python bench.py --workload greedy --steps 20 --warmup 5 --no-cpu-baseline"

cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06z
bash tools/gpu_steps.sh $O \
 "600|greedy|python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k 'greedy or gq or remap'" \
 "600|ab|python -u tools/greedy_ab.py 3 100" \
 "300|prof|rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o greedy -- python bench.py --workload greedy --steps 20 --warmup 5 --no-cpu-baseline"

cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06final2
bash tools/gpu_steps.sh $O \
 "1000|gputests|python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "200|smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300|bench20|python -u bench.py --steps 20 --warmup 5" \
 "300|greedy|python -u bench.py --workload greedy --steps 20 --warmup 5 --no-cpu-baseline" \
 "300|actorprof|rocprofv3 --kernel-trace --stats --output-format csv -d $O/actorprof -o actor -- python bench.py --workload actor --steps 10 --warmup 3 --no-cpu-baseline"

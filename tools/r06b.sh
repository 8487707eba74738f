cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06final
bash tools/gpu_steps.sh $O \
 "1000|gputests|python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread" \
 "200|smoke|python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "300|bench20|python -u bench.py --steps 20 --warmup 5" \
 "400|benchprof|rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o step -- python bench.py --no-cpu-baseline"

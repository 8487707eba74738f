cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06mb
bash tools/gpu_steps.sh $O \
 "300|actor|python -u bench.py --workload actor --steps 20 --warmup 5 --no-cpu-baseline" \
 "300|actor2|python -u bench.py --workload actor --steps 20 --warmup 5 --no-cpu-baseline"

for a in "--warmup 5" "--warmup 5" "--warmup 5 --clock-warmup 0"; do
  MDR_TRACE=1 timeout -k 10 120 python bench.py --steps 20 --no-cpu-baseline --trace $a 2> gpurun_out/b20_err.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$a', round(d['value']/1e9,1), 'Gsteps/s wall_us', round(d['timed_region']['wall_s']*1e6), 'ev_us', round(d['timed_region']['launch_stream_event_ms']*1e3))" || exit 1
  grep -E "trace" gpurun_out/b20_err.log; grep mdr_rollout gpurun_out/b20_err.log | tail -3
done

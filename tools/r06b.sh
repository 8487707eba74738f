K="python tools/actor_kbench.py --reps 50"
bash tools/gpu_steps.sh gpurun_out/r06j \
 "100|dbg|python tools/actor_f16_debug.py" \
 "300|t_new|python -u -m pytest -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_actor_gpu.py" \
 "400|t_chain|python -u -m pytest -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_actor_chain_gpu.py tests/test_configs_gpu.py -k 'actor or c5'" \
 "120|kb1|$K --precision fp32 && $K --precision bf16x3 && $K --precision fp32 && $K --precision bf16x3"

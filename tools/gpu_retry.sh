#!/bin/bash
# Retry tools/gpu_send.sh while the pool reports no free box (exit 3 / status=transient).
# Usage: STEPS=... tools/gpu_retry.sh LOG [gpurun-timeout] [extra cmd]
LOG=$1; shift
for i in $(seq 1 20); do
  "$(dirname "$0")/gpu_send.sh" "$@" > "$LOG" 2>&1
  grep -q "status=transient" "$LOG" || break
  sleep 90
done
echo "gpu_retry finished after $i attempt(s)" >> "$LOG"

#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that crashes or
# times out (status >= 124: timeout, abort, segfault), keep going after an ordinary failure.
# Usage: tools/gpu_steps.sh OUTDIR "SECONDS|NAME|COMMAND" ...   (each step's output: OUTDIR/NAME.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp TZ=UTC
out=$1; shift
mkdir -p "$out"
worst=0
for step in "$@"; do
  IFS='|' read -r secs name cmd <<< "$step"
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc"; tail -4 "$out/$name.log"
  [ $rc -gt $worst ] && worst=$rc
  if [ $rc -ge 124 ]; then echo "stopping: $name ended with $rc"; exit $rc; fi
done
exit $worst

#!/bin/bash
# Local wrapper: rebuild the HIP library and the host extension from the tree (stop on a build
# error, so a stale library never travels), then run one command on an MI355X box through gpurun.
# Usage: tools/gpu.sh [--timeout S] -- 'command'
set -u
cd "$(dirname "$0")/.."
python marl-demandresponse_amd/build_ext.py > /tmp/mdr_build.log 2>&1 || { tail -20 /tmp/mdr_build.log; echo "BUILD FAILED"; exit 1; }
exec /usr/local/graft/bin/gpurun "$@"

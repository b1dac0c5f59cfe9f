#!/bin/bash
# Kernel-trace stats of the bench pipeline (no event timing): tools/trace_only.sh <tag> [bench args]
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/trace -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-kernel-times "$@" > $R/gpurun_out/$TAG/trace.log 2>&1
echo done

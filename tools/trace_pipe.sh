#!/bin/bash
# Kernel trace of the pipelined bench (start/end timestamps show the overlap of k4_hist with
# the previous batch's kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tp
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/tp/trace -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-kernel-times --no-roofline-probe > $R/gpurun_out/tp/trace.log 2>&1 && \
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 3 --cpu-seconds 0 --serial --no-roofline-probe > $R/gpurun_out/tp/serial.log 2>&1

#!/bin/bash
# Run the GPU test suite, then one bench line ($@ = extra bench args).
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/b.log 2>&1

#!/bin/bash
# Build, run the GPU test suite, then one bench line per pipeline given ($@ = extra bench args).
# Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
make -s -C api-ratelimit_amd/csrc && \
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/b_v2.log 2>&1

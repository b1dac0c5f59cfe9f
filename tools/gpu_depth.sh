#!/bin/bash
# Pipelined-submission tests, then the GPU suite, then bench at depth 3, 2 and 1.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ab/tp.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-roofline-probe > gpurun_out/ab/b_d3.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-roofline-probe --depth 2 > gpurun_out/ab/b_d2.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --serial --no-roofline-probe > gpurun_out/ab/b_d1.log 2>&1

#!/bin/bash
# Pipelined submission bring-up: new tests first, then the whole GPU suite, then the bench
# (two in flight, and serial for comparison).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipelined.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tp.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/bp.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --serial --no-roofline-probe > gpurun_out/bs.log 2>&1

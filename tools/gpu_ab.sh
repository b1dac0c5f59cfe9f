#!/bin/bash
# GPU suite, then bench A/B: default, stream priorities off, serial.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/t.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-roofline-probe > gpurun_out/ab/b_def.log 2>&1 && \
RL_STREAM_PRIORITIES=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-roofline-probe > gpurun_out/ab/b_noprio.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --serial --no-roofline-probe > gpurun_out/ab/b_serial.log 2>&1

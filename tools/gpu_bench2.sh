#!/bin/bash
# Two bench lines: two batches in flight (default) and one (serial).
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-roofline-probe > gpurun_out/ab/b_def.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 --serial --no-roofline-probe > gpurun_out/ab/b_serial.log 2>&1

#!/bin/bash
# v4 bring-up: smoke, GPU tests (first failure stops), then a short bench of v4 and v3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/b.log 2>&1

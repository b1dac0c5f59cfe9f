#!/bin/bash
# Round-end rehearsal: GPU suite, smoke(), default bench line (as the driver runs them).
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/t.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.log 2>&1

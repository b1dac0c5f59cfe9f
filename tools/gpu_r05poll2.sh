#!/bin/bash
# Completion by k4_group's done word (in-tree) against the completion event (HEAD before it:
# tools/variants/lib_evbase.so), interleaved; config 3; then the pipelined / cache-mirror tests.
set -e
mkdir -p gpurun_out/poll2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipelined.py tests/test_gpu_cache_mirror.py tests/test_gpu_bench_regime.py > gpurun_out/poll2/tests.log 2>&1
tail -1 gpurun_out/poll2/tests.log
bash tools/ab.sh 100 "- tools/variants/lib_evbase.so - tools/variants/lib_evbase.so - tools/variants/lib_evbase.so"
bash tools/ab.sh 20 "- tools/variants/lib_evbase.so - tools/variants/lib_evbase.so"

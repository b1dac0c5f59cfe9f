#!/bin/bash
# No front-stream wait for batch seq-2 when it completed through rl_wait (in-tree) against the
# polled-completion sources with the wait (lib_pollbase); config 3, interleaved; pipelined tests.
set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipelined.py tests/test_gpu_bench_regime.py > gpurun_out/nowait_tests.log 2>&1
tail -1 gpurun_out/nowait_tests.log
bash tools/ab.sh 100 "- tools/variants/lib_pollbase.so - tools/variants/lib_pollbase.so - tools/variants/lib_pollbase.so"
bash tools/ab.sh 20 "- tools/variants/lib_pollbase.so - tools/variants/lib_pollbase.so"

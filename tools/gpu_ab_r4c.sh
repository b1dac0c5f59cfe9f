#!/bin/bash
# Round 4 A/B call 3: the v4 parity tests on the in-tree library (k4_group's four-wave key-list
# layout), then an interleaved A/B against tools/variants/lib_onewave.so (one-wave layout).
# usage (on the GPU box): tools/gpu_ab_r4c.sh <tag>
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_pipelined.py tests/test_gpu_bench_regime.py tests/test_gpu_configs.py tests/test_gpu_combining.py tests/test_gpu_compact.py tests/test_per_second.py tests/test_shadow.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab.sh 40 "- tools/variants/lib_onewave.so - tools/variants/lib_onewave.so - tools/variants/lib_onewave.so" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt

#!/bin/bash
# One GPU call: the routed-step GPU tests, then an interleaved A/B of the routed step on a
# one-rank RCCL communicator (bench.py --force-routed): the in-tree library against
# tools/variants/lib_base.so.
set -u
OUT=gpurun_out/abr; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_combining.py tests/test_gpu_native_router.py \
  tests/test_gpu_routed_bench.py tests/test_gpu_router.py -m gpu -q --timeout 200 --timeout-method thread \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab.sh 30 "- tools/variants/lib_base.so - tools/variants/lib_base.so - tools/variants/lib_base.so" \
  --force-routed --no-kernel-times > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt
[ "${1:-}" = "curve" ] && timeout -k 10 1000 bash tools/gpu_bench_round.sh abr_curve "ls2 ls4 ls8"

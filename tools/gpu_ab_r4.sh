#!/bin/bash
# Round 4 A/B call: the C++ mirror tests, then an interleaved A/B of the in-tree library against
# tools/variants/lib_base.so (HEAD~ kernels) and lib_nosf.so (RL_EPI_NOSYSFENCE) on one box.
# usage (on the GPU box): tools/gpu_ab_r4.sh <tag>
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_cache_mirror.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 1000 bash tools/ab.sh 40 "- tools/variants/lib_base.so tools/variants/lib_nosf.so - tools/variants/lib_base.so tools/variants/lib_nosf.so - tools/variants/lib_base.so tools/variants/lib_nosf.so" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt

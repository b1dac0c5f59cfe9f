#!/bin/bash
# Round 4 A/B call: the C++ mirror and compact-format tests, a bench line (host path included),
# then an interleaved A/B of the in-tree library against tools/variants/lib_ldshot.so (hot table in
# LDS), lib_base.so (the kernels before the round-4 hist / scan changes) and lib_nosf.so
# (RL_EPI_NOSYSFENCE) on one box.
# usage (on the GPU box): tools/gpu_ab_r4.sh <tag>
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_cache_mirror.py tests/test_gpu_compact.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_pipelined.py tests/test_gpu_bench_regime.py tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-roofline-probe > $OUT/bench.json 2> $OUT/bench.err; rc=$?
echo "bench rc=$rc"; python3 -c "import json,sys; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); h=d['host_path']; print(d['ms_per_step'], h['value'], h['ms_per_batch'], h['frac_of_pcie_bound'], h['full_format']['value'])"
[ $rc -ge 124 ] && exit $rc
timeout -k 10 1000 bash tools/ab.sh 40 "- tools/variants/lib_ldshot.so tools/variants/lib_base.so - tools/variants/lib_ldshot.so tools/variants/lib_nosf.so - tools/variants/lib_ldshot.so tools/variants/lib_base.so" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt

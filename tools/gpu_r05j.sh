set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 120 python tools/diag_resolve.py 2>&1 | grep shift
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_resolve.py tests/test_gpu_configs45_regime.py tests/test_gpu_configs.py tests/test_gpu_cache_mirror.py > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh 20 "- tools/variants/lib_res1.so - tools/variants/lib_res1.so" --config 4

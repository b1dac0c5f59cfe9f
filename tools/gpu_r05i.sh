# repack on demand: routed parity, then the one-rank routed step A/B against the previous sources
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_emulated_router.py tests/test_gpu_combining.py tests/test_gpu_routed_regime.py tests/test_gpu_router.py tests/test_gpu_native_router.py > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh 30 "- tools/variants/lib_rp0.so - tools/variants/lib_rp0.so" --force-routed

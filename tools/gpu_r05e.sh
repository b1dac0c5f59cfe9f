set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05e; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh 40 "- tools/variants/lib_prejit.so - tools/variants/lib_prejit.so -"

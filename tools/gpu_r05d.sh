set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_configs45_regime.py > $OUT/pytest.log 2>&1
echo "pytest rc=$?"; tail -3 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --cpu-seconds 2 --no-host-path > $OUT/bench3.json 2> $OUT/bench3.err; rc=$?
echo "bench3 rc=$rc"; tail -c 600 $OUT/bench3.json; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u bench.py --config 5 --cpu-seconds 2 --no-host-path > $OUT/bench5.json 2> $OUT/bench5.err; rc=$?
echo "bench5 rc=$rc"; tail -c 600 $OUT/bench5.json; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 python -u bench.py --config 4 --cpu-seconds 2 --no-host-path > $OUT/bench4.json 2> $OUT/bench4.err; rc=$?
echo "bench4 rc=$rc"; tail -c 600 $OUT/bench4.json; tail -5 $OUT/bench4.err
exit 0

# Round-5 final (polled completion): every GPU test, smoke, the PMC summary, then the bench lines
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05final5; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/pmc_round.sh r05pmc5 20 > $OUT/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 $OUT/pmc.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r05bench.sh; rc=$?
exit $rc

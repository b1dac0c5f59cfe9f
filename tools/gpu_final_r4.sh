#!/bin/bash
# Round 4 final sources, one GPU call: the whole GPU test suite, smoke, then the PMC / trace
# summaries (tools/pmc_round.sh) the bench line's traffic comes from.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 1800 bash tools/pmc_round.sh $1 20 > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -5 $OUT/pmc.log; exit $rc

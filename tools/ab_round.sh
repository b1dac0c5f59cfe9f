# One GPU call: the whole -m gpu suite, then an interleaved A/B of the in-tree library against
# tools/variants/lib_base.so (the previous kernels, built from git HEAD's sources by hand) on
# the same box. A failing or crashing test run stops the call before the A/B.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3l; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab.sh 40 "- tools/variants/lib_base.so - tools/variants/lib_base.so - tools/variants/lib_base.so" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt
[ "${1:-}" = "pmc" ] && { timeout -k 10 600 bash tools/pmc_round.sh abpmc 20 > $OUT/pmc.log 2>&1; echo "pmc rc=$?"; }

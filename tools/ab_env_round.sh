#!/bin/bash
# One GPU call: the -m gpu suite, then an interleaved A/B of environment settings of the
# in-tree library (tools/ab.sh variant syntax: "-,VAR=VAL").
# usage: tools/ab_env_round.sh "<variants>" [steps]
set -u
OUT=gpurun_out/abe; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 bash tools/ab.sh "${2:-40}" "$1" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt

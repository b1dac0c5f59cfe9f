#!/bin/bash
# Round 4: k4_hist writing the tile's hot records in arrival order (RL_HOT_ARRIVAL_ORDER)
# against the in-tree bucket order, single-GPU step, interleaved.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 bash tools/ab.sh 40 "- tools/variants/lib_hotarr.so - tools/variants/lib_hotarr.so - tools/variants/lib_hotarr.so" > $OUT/ab.txt 2>&1; echo "ab rc=$?"; cat $OUT/ab.txt

#!/bin/bash
# Collect PMC counters for the bench pipeline, one counter group per rocprofv3 pass
# (MI355X_MICROARCH.md: TCC FETCH_SIZE and WRITE_SIZE cannot share a pass).
# usage: tools/pmc_run.sh <outdir> [bench args...]
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $R/$OUT/p$i -o run --output-format csv -- \
     python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-times "$@" > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$OUT/p$i.log; exit 1; }
done
echo done

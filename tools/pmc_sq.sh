#!/bin/bash
# SQ instruction / cycle counters per kernel (two passes, 8 SQ counters each).
# usage (GPU box, repo root): tools/pmc_sq.sh <outdir> [bench args...]
set -e
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/$OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $R/$OUT/p$i -o run --output-format csv -- \
     python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-kernel-times --no-roofline-probe "$@" > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/$OUT/p$i.log; exit 1; }
done
echo done

#!/bin/bash
# Round profile: bench line, rocprofv3 kernel-trace stats, PMC traffic passes.
# usage (on the GPU box, from the repo root): tools/profile_round.sh <tag>
set -e
TAG=$1
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/$TAG
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $R/gpurun_out/$TAG/bench.json 2> $R/gpurun_out/$TAG/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/trace -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-kernel-times > $R/gpurun_out/$TAG/trace.log 2>&1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $R/gpurun_out/$TAG/p$i -o run --output-format csv -- \
     python3 $R/bench.py --steps 5 --warmup 2 --cpu-seconds 0 --no-kernel-times > $R/gpurun_out/$TAG/p$i.log 2>&1
done
echo done

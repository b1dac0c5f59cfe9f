#!/bin/bash
# PMC traffic of the routed step on a one-rank RCCL communicator (bench.py --force-routed):
# one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md), then tools/pmc_traffic.py
# over the last STEPS dispatches of each kernel (k_route_pack2 runs twice per step: the pack
# and the repack launch that returns at once; both are averaged under one name).
# usage (on the GPU box, from the repo root): tools/pmc_routed.sh <tag> [steps]
set -u
TAG=$1
STEPS=${2:-30}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
P=/tmp/pmcr_$TAG
mkdir -p "$OUT" "$P"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --force-routed --steps $STEPS --warmup 10 --cpu-seconds 0 --no-kernel-times --no-roofline-probe --no-host-path --prefill 2000"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --pmc $grp -d $P/p$i -o run --output-format csv -- $BENCH \
    > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pmc pass $i rc=$?"; tail -5 "$OUT/p$i.err"; exit 1; }
done
python3 $R/tools/pmc_traffic.py $P "$OUT/pmc_traffic_routed.json" $STEPS "$TAG"

#!/bin/bash
# Per-kernel pipeline counters (occupancy, waits, VMEM instructions, TA / TCP / L2 activity) over a
# short bench, one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md block limits: at
# most 8 SQ, 2 TA, 4 TCP, 4 TCC per pass). Counter names are taken from this box's
# `rocprofv3 --list-avail`: a candidate the box does not list is dropped, so no pass asks for an
# unknown counter. Output: gpurun_out/<tag>/kernel_counters.json (tools/pmc_kernel_counters.py).
# usage (on the GPU box, from the repo root): tools/pmc_kernels.sh <tag> <steps> <bench args...>
set -u
TAG=$1
STEPS=$2
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
P=/tmp/pmck_$TAG
mkdir -p "$OUT" "$P"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --list-avail > "$P/avail.txt" 2>&1 || { echo "list-avail rc=$?"; exit 1; }
grep -o "[A-Za-z][A-Za-z0-9_]*" "$P/avail.txt" | sort -u > "$OUT/avail_names.txt"
pick() {  # the candidates this box lists, at most $1 of them
  local n=$1 out="" k=0
  shift
  for c in "$@"; do
    if [ $k -lt $n ] && grep -qx "$c" "$OUT/avail_names.txt"; then out="$out $c"; k=$((k+1)); fi
  done
  echo $out
}
G1=$(pick 8 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU)
G2=$(pick 2 TA_BUSY_avr TA_TA_BUSY_avr TA_BUSY_max TA_TA_BUSY_max)
G3=$(pick 4 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum)
G4=$(pick 4 TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE)
G5=$(pick 2 TD_BUSY_avr TD_TD_BUSY_avr TD_TC_STALL_sum TD_TC_STALL_avr)
echo "groups: [$G1] [$G2] [$G3] [$G4] [$G5]" | tee "$OUT/groups.txt"
i=0
for grp in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  i=$((i+1))
  [ -z "$grp" ] && continue
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $P/p$i -o run --output-format csv -- \
    python3 $R/bench.py --steps $STEPS --warmup 2 --cpu-seconds 0 --no-kernel-times --no-roofline-probe \
    --no-host-path "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pmc pass $i rc=$?"; tail -5 "$OUT/p$i.err"; exit 1; }
done
python3 $R/tools/pmc_kernel_counters.py $P "$OUT/kernel_counters.json" $STEPS

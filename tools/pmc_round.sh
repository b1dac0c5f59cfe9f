#!/bin/bash
# One GPU call of profiling for the committed round summaries (measurement tooling):
#   1. rocprofv3 --kernel-trace --stats over the bench (prefill, timed steps, kernel-timing
#      steps) and tools/trace_summary.py over the kernel-timing dispatches,
#   2. one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: FETCH_SIZE and
#      WRITE_SIZE cannot share a pass), each over a short bench with the same table fill,
#   3. the same counters over tools/microbench/table_rmw (random 32-B slot reads / RMWs of
#      known count on an 8 GiB table) to calibrate how the counters see random slot traffic,
#   4. tools/pmc_traffic.py -> gpurun_out/<tag>/pmc_traffic.json (per-kernel bytes per launch
#      over the timed dispatches, tagged with bench.source_sha()).
# Raw CSVs stay under /tmp on the box; only summaries come back.
# usage (on the GPU box, from the repo root): tools/pmc_round.sh <tag> [steps] [trace-only|""] [config]
set -u
TAG=$1
STEPS=${2:-20}
CFG=${4:-3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
P=/tmp/pmc_$TAG
mkdir -p "$OUT" "$P"
cd /tmp && export TMPDIR=/tmp
BENCH="python3 $R/bench.py --config $CFG --steps $STEPS --warmup 3 --cpu-seconds 0 --no-kernel-times --no-roofline-probe --no-host-path"
# the trace run keeps bench.py's unoverlapped kernel-timing batches (the last STEPS dispatches)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- \
  python3 $R/bench.py --config $CFG --steps $STEPS --warmup 3 --cpu-seconds 0 --no-roofline-probe --no-host-path \
  > "$OUT/trace.json" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -5 "$OUT/trace.err"; exit 1; }
cp $P/trace/run_kernel_stats.csv "$OUT/kernel_stats.csv"
python3 $R/tools/trace_summary.py $P/trace/run_kernel_trace.csv "$OUT/trace.json" $STEPS "$OUT/kernel_trace_summary.json" > /dev/null
[ "${3:-}" = "trace-only" ] && exit 0
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --pmc $grp -d $P/p$i -o run --output-format csv -- $BENCH \
    > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pmc pass $i rc=$?"; tail -5 "$OUT/p$i.err"; exit 1; }
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $P/c$i -o run --output-format csv -- \
    $R/tools/microbench/table_rmw 28 230000 > "$OUT/c$i.log" 2>&1 || { echo "calibration pass $i rc=$?"; exit 1; }
done
python3 $R/tools/pmc_traffic.py $P "$OUT/pmc_traffic.json" $STEPS "$TAG" $CFG

# routed one-rank timeline (config 3) on the round-5 sources
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/r05h; mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/rtl -o run --output-format csv -- \
  python3 $R/bench.py --force-routed --steps 30 --warmup 5 --cpu-seconds 0 --no-kernel-times --no-roofline-probe --no-host-path > $OUT/rtl.json 2> $OUT/rtl.err || { echo "trace rc=$?"; tail -5 $OUT/rtl.err; exit 1; }
python3 $R/tools/trace_tail.py /tmp/rtl/run_kernel_trace.csv 60 > $OUT/routed_timeline.txt
tail -45 $OUT/routed_timeline.txt

# Round-5 stamps + pipelined timeline of the current sources
set -u
export TMPDIR=/tmp
R=$(pwd)
OUT=$R/gpurun_out/r05f; mkdir -p $OUT
bash tools/stamps_round.sh > $OUT/stamps.txt 2>&1 || { echo "stamps rc=$?"; tail -5 $OUT/stamps.txt; exit 1; }
cp gpurun_out/st/view.txt $OUT/view.txt; cp gpurun_out/st/viewf.txt $OUT/viewf.txt 2>/dev/null
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o run --output-format csv -- \
  python3 $R/bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-kernel-times --no-roofline-probe --no-host-path > $OUT/tl.json 2> $OUT/tl.err || { echo "trace rc=$?"; tail -5 $OUT/tl.err; exit 1; }
python3 $R/tools/timeline.py /tmp/tl/run_kernel_trace.csv 24 > $OUT/timeline.txt
tail -30 $OUT/timeline.txt
cd $R
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c --force-routed --steps 20 --warmup 5 --cpu-seconds 1 --no-host-path > $OUT/routed_c$c.json 2> $OUT/routed_c$c.err; rc=$?
  echo "routed c$c rc=$rc"; tail -c 400 $OUT/routed_c$c.json; [ $rc -ne 0 ] && { tail -5 $OUT/routed_c$c.err; exit $rc; }
done

bash tools/ab.sh 40 "- tools/variants/lib_evdev.so tools/variants/lib_nt1024.so - tools/variants/lib_evdev.so tools/variants/lib_nt1024.so"

set -u
export TMPDIR=/tmp
OUT=gpurun_out/r3c; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v --timeout 120 --timeout-method thread -k "host_path or wait_view" > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -ge 124 ] && exit $rc
mkdir -p /tmp/rp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/rp -o run --output-format csv -- python3 -u bench.py --force-routed --steps 30 --warmup 10 --cpu-seconds 0 --no-host-path --no-roofline-probe --prefill 2000 > $OUT/rprof.json 2> $OUT/rprof.err; rc=$?; echo "rprof rc=$rc"; [ $rc -ge 124 ] && exit $rc
cp /tmp/rp/run_kernel_stats.csv $OUT/routed_kernel_stats.csv; python3 tools/trace_tail.py /tmp/rp/run_kernel_trace.csv 60 > $OUT/routed_timeline.txt 2>&1
timeout -k 10 400 python -u bench.py --cpu-seconds 2 --no-roofline-probe > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"

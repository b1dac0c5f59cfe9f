#!/bin/bash
# Round 4: the router with three steps in flight. Router GPU tests, then the one-rank RCCL routed
# step (records before the older steps' replies, and the in-tree order, depth 3), interleaved,
# then a kernel timeline of the in-tree library.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_combining.py tests/test_gpu_native_router.py \
  tests/test_gpu_emulated_router.py tests/test_gpu_routed_bench.py tests/test_gpu_router.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in recfirst,3 -,3; do
    IFS=, read -r lib dep <<< "$v"
    lp=""; [ "$lib" != "-" ] && lp="--lib tools/variants/lib_$lib.so"
    timeout -k 10 200 python bench.py --force-routed --router-depth $dep --steps 40 --warmup 10 --cpu-seconds 0 \
      --no-roofline-probe --no-host-path $lp > $OUT/r.log 2>&1 || { tail -5 $OUT/r.log; exit 1; }
    python - $v $OUT/r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = (d.get("roofline") or {}).get("kernels_us_per_batch") or {}
print(sys.argv[1], d["ms_per_step"], {n: round(v, 1) for n, v in d.get("router", {}).items() if n.endswith("_us")}, k)
PY
  done
done | tee $OUT/ab.txt
mkdir -p /tmp/rt_$1 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/rt_$1 -o run --output-format csv \
  -- python3 -u bench.py --force-routed --router-depth ${2:-2} --steps 30 --warmup 10 --cpu-seconds 0 --no-host-path \
  --no-roofline-probe --no-kernel-times --prefill 2000 > $OUT/rtrace.log 2>&1 \
  && python3 tools/trace_tail.py /tmp/rt_$1/run_kernel_trace.csv 80 > $OUT/routed_timeline.txt; echo "rtrace rc=$?"

#!/bin/bash
# Round 4 A/B call 2: the pipelined-submission tests with the deferred k4_group (RL_DEFER_GROUP=1),
# then interleaved bench runs: default (depth 2), deferred group at depth 3 and 2, and the
# no-system-fence variant library.
# usage (on the GPU box): tools/gpu_ab_r4b.sh <tag>
set -u
export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
RL_DEFER_GROUP=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_pipelined.py tests/test_gpu_bench_regime.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread > $OUT/pytest_defer.log 2>&1; rc=$?
echo "pytest(defer) rc=$rc"; tail -3 $OUT/pytest_defer.log
[ $rc -ne 0 ] && exit $rc
one() {  # label env lib depth
  local label=$1 envs=$2 lib=$3 depth=$4
  env $envs timeout -k 10 150 python bench.py --steps 40 --warmup 30 --cpu-seconds 0 --no-roofline-probe --no-host-path \
    ${lib:+--lib $lib} --depth $depth > $OUT/ab_one.log 2>&1 || { echo "$label failed"; tail -5 $OUT/ab_one.log; exit 1; }
  python3 - "$label" "$OUT/ab_one.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
k = (d.get("roofline") or {}).get("kernels_us_per_batch") or {}
print(sys.argv[1], d["ms_per_step"], d["config"].get("batches_in_flight"), " ".join(f"{n}={v}" for n, v in k.items()))
PY
}
for r in 1 2 3; do
  one base2 "X=0" "" 2
  one defer3 "RL_DEFER_GROUP=1" "" 3
  one defer2 "RL_DEFER_GROUP=1" "" 2
  one base3 "X=0" "" 3
  [ $r -ne 2 ] && one nosf2 "X=0" tools/variants/lib_nosf.so 2
done 2>&1 | tee $OUT/ab.txt

#!/bin/bash
# A/B bench of variants on one box: tools/ab.sh STEPS "v1 v2 ..." [extra bench args]
# A variant is LIB[,VAR=VAL...]: LIB a variant library or "-" (the in-tree one), with
# optional environment settings. Prints ms/step and batches in flight per run.
steps=$1; vars=$2; shift 2
mkdir -p gpurun_out
for t in $vars; do
  IFS=, read -r lib envs <<< "$t"
  [ "$lib" = "-" ] && lib=""
  env ${envs//,/ } timeout -k 10 150 python bench.py --steps "$steps" --warmup 30 --cpu-seconds 0 --no-roofline-probe \
    --no-host-path ${lib:+--lib $lib} "$@" > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python - "$t" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.log").read().strip().splitlines()[-1])
k = (d.get("roofline") or {}).get("kernels_us_per_batch") or {}
print(sys.argv[1], d["ms_per_step"], d["config"].get("batches_in_flight"), " ".join(f"{n}={v}" for n, v in k.items()))
PY
done

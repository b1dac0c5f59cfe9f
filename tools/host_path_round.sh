#!/bin/bash
# One GPU call: the host-path parity tests, then the bench's host path twice (ms per batch,
# the link's time for the same copies, the fraction of the bound, the copying form).
set -u
OUT=gpurun_out/hp; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -q --timeout 120 --timeout-method thread \
  -k "host_path or wait_view" > $OUT/tests.log 2>&1 || { tail -5 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --cpu-seconds 0 --no-roofline-probe --no-kernel-times --steps 20 \
    > $OUT/b$i.json 2> $OUT/b$i.err || { echo "bench rc=$?"; exit 1; }
  python3 - "$OUT/b$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h = d["host_path"]
print(d["ms_per_step"], h["ms_per_batch"], h["link_ms_per_batch"], h["frac_of_pcie_bound"], h["copy_out"]["ms_per_batch"])
PY
done

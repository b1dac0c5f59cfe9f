#!/bin/bash
# Two against three batches in flight (bench.py --depth), interleaved.
set -e
mkdir -p gpurun_out/depth
for rep in 1 2 3; do
  for dp in 2 3; do
    timeout -k 10 200 python -u bench.py --steps 100 --cpu-seconds 0 --no-host-path --no-roofline-probe --no-kernel-times \
      --depth $dp --json-out gpurun_out/depth/p${dp}_r$rep.json > gpurun_out/depth/p${dp}_r$rep.log 2>&1
    python3 -c "import json;l=json.load(open('gpurun_out/depth/p${dp}_r$rep.json'));print('depth $dp rep $rep', round(l['ms_per_step']*1e3,1), l['engine']['host_us_per_step'])"
  done
done

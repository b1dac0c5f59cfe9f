#!/bin/bash
# Batch structs prebuilt before the timed region (default) against built in the loop
# (--no-prebuilt), interleaved; the driver's step count (20) and 100.
# (--no-prebuilt was an A/B switch of bench.py, removed after this measurement:
# profiles/r05_ab_hist_start.txt.)
set -e
mkdir -p gpurun_out/pre
for steps in 20 100; do
  for rep in 1 2 3; do
    for v in "" "--no-prebuilt"; do
      tag=s${steps}_r${rep}${v:+_np}
      timeout -k 10 200 python -u bench.py --steps $steps --warmup 5 --cpu-seconds 0 --no-host-path --no-roofline-probe \
        --no-kernel-times $v --json-out gpurun_out/pre/$tag.json > gpurun_out/pre/$tag.log 2>&1
      python3 -c "import json;l=json.load(open('gpurun_out/pre/$tag.json'));h=l['engine']['host_us_per_step'];print('$tag', round(l['ms_per_step']*1e3,1), 'step p50', h['step']['p50'], 'submit p50', h['submit']['p50'])"
    done
  done
done

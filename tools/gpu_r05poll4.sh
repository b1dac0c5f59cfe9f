#!/bin/bash
# Polled completion (in-tree) against the completion event (lib_evbase) at configs 5 and 3, with
# the host's time inside submit / wait per step.
set -e
mkdir -p gpurun_out/poll4
for rep in 1 2; do
  for c in 5 3; do
    for v in "-" "tools/variants/lib_evbase.so"; do
      tag=c${c}_r${rep}_$([ "$v" = "-" ] && echo poll || echo event)
      timeout -k 10 300 python -u bench.py --config $c --steps 60 --warmup 10 --cpu-seconds 0 --no-host-path \
        --no-roofline-probe --no-kernel-times $([ "$v" = "-" ] || echo --lib $v) --json-out gpurun_out/poll4/$tag.json > gpurun_out/poll4/$tag.log 2>&1
      python3 -c "import json;l=json.load(open('gpurun_out/poll4/$tag.json'));h=l['engine']['host_us_per_step'];print('$tag', round(l['ms_per_step']*1e3,1), 'step p50', h['step']['p50'], 'submit mean/p50', h['submit']['mean'], h['submit']['p50'], 'wait p50', h['wait']['p50'])"
    done
  done
done

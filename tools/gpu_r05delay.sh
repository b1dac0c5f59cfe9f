#!/bin/bash
# Sensitivity of the pipelined step to when batch k+2's k4_hist is enqueued: the host spins
# D µs before each rl_submit_pipelined (bench.py --host-delay-us), interleaved over D.
set -e
mkdir -p gpurun_out/delay
for rep in 1 2; do
  for d in 0 10 20 35 50; do
    timeout -k 10 200 python -u bench.py --steps 100 --cpu-seconds 0 --no-host-path --no-roofline-probe --no-kernel-times \
      --host-delay-us $d --json-out gpurun_out/delay/d${d}_r$rep.json > gpurun_out/delay/d${d}_r$rep.log 2>&1
    python3 -c "import json;l=json.load(open('gpurun_out/delay/d${d}_r$rep.json'));print('delay $d rep $rep', round(l['ms_per_step']*1e3,1), l['engine']['host_us_per_step'])"
  done
done

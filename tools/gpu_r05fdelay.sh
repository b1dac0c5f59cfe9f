#!/bin/bash
# A device-side delay (one waiting wave, RL_DIAG_FRONT_DELAY_US) in front of the next batch's
# k4_hist at three in flight (its start then no longer depends on the host), against the
# host-timed default; interleaved.
# (RL_DIAG_FRONT_DELAY_US was an A/B switch in the engine, removed after this measurement:
# profiles/r05_ab_hist_start.txt; rerunning needs it back.)
set -e
mkdir -p gpurun_out/fdelay
for rep in 1 2; do
  for v in "2 0" "3 0" "3 5" "3 10" "3 15" "3 20" "3 30"; do
    set -- $v
    RL_DIAG_FRONT_DELAY_US=$2 timeout -k 10 200 python -u bench.py --steps 100 --cpu-seconds 0 --no-host-path \
      --no-roofline-probe --no-kernel-times --depth $1 --json-out gpurun_out/fdelay/p$1d$2_r$rep.json > gpurun_out/fdelay/p$1d$2_r$rep.log 2>&1
    python3 -c "import json;l=json.load(open('gpurun_out/fdelay/p$1d$2_r$rep.json'));h=l['engine']['host_us_per_step'];print('depth $1 delay $2 rep $rep', round(l['ms_per_step']*1e3,1), 'step p50', h['step']['p50'], 'submit p50', h['submit']['p50'])"
  done
done

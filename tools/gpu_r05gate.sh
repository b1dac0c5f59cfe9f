#!/bin/bash
# When the next batch's k4_hist may start: now (host-timed, gate 0), after the batch in
# flight's k4_scan (1) or k4_place (2), at two and three batches in flight; interleaved.
# (RL_DIAG_HIST_GATE was an A/B switch in the engine, removed after this measurement:
# profiles/r05_ab_hist_start.txt; rerunning needs it back.)
set -e
mkdir -p gpurun_out/gate
for rep in 1 2; do
  for v in "2 0" "2 1" "2 2" "3 1" "3 2"; do
    set -- $v
    RL_DIAG_HIST_GATE=$2 timeout -k 10 200 python -u bench.py --steps 100 --cpu-seconds 0 --no-host-path \
      --no-roofline-probe --no-kernel-times --depth $1 --json-out gpurun_out/gate/p$1g$2_r$rep.json > gpurun_out/gate/p$1g$2_r$rep.log 2>&1
    python3 -c "import json;l=json.load(open('gpurun_out/gate/p$1g$2_r$rep.json'));h=l['engine']['host_us_per_step'];print('depth $1 gate $2 rep $rep', round(l['ms_per_step']*1e3,1), 'step p50', h['step']['p50'], 'submit p50', h['submit']['p50'])"
  done
done

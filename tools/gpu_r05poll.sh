#!/bin/bash
# Completion by polling k4_group's done word (RL_DIAG_POLL_DONE=D, then D us of spin) against the
# completion event (unset), interleaved; config 3, 100 steps.
set -e
mkdir -p gpurun_out/poll
timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gpu_pipelined.py > gpurun_out/poll/t_default.log 2>&1
RL_DIAG_POLL_DONE=0 timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread -m gpu tests/test_gpu_pipelined.py > gpurun_out/poll/t_poll.log 2>&1
tail -1 gpurun_out/poll/t_default.log; tail -1 gpurun_out/poll/t_poll.log
for rep in 1 2; do
  for d in off 0 3 6 10; do
    if [ $d = off ]; then unset RL_DIAG_POLL_DONE; else export RL_DIAG_POLL_DONE=$d; fi
    timeout -k 10 200 python -u bench.py --steps 100 --cpu-seconds 0 --no-host-path --no-roofline-probe \
      --no-kernel-times --json-out gpurun_out/poll/d${d}_r$rep.json > gpurun_out/poll/d${d}_r$rep.log 2>&1
    python3 -c "import json;l=json.load(open('gpurun_out/poll/d${d}_r$rep.json'));h=l['engine']['host_us_per_step'];print('poll $d rep $rep', round(l['ms_per_step']*1e3,1), 'step p50', h['step']['p50'], 'wait p50', h['wait']['p50'])"
  done
done

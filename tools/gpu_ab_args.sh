#!/bin/bash
# Bench A/B of bench.py arguments: default vs "$@" (alternating, two runs each).
set -o pipefail
D=gpurun_out/abargs; mkdir -p $D
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-roofline-probe > $D/def$i.json 2>$D/def$i.err || exit 1
  timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-roofline-probe "$@" > $D/var$i.json 2>$D/var$i.err || exit 1
done

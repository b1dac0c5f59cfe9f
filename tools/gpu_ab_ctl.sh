#!/bin/bash
# GPU suite on the current library, then bench A/B: current vs tools/variants/lib_v_old.so (alternating).
set -o pipefail
D=gpurun_out/abctl; mkdir -p $D
L=api-ratelimit_amd/csrc/libratelimit_hip.so
cp $L $D/lib_new.so
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/t.log 2>&1 || exit 1
for i in 1 2; do
  cp $D/lib_new.so $L && timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-roofline-probe > $D/new$i.json 2>$D/new$i.err || exit 1
  cp tools/variants/lib_v_old.so $L && timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-roofline-probe > $D/old$i.json 2>$D/old$i.err || exit 1
done
cp $D/lib_new.so $L

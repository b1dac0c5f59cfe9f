#!/bin/bash
# Bench A/B over library variants tools/variants/lib_<name>.so (alternating rounds); restores the in-tree library.
set -o pipefail
D=gpurun_out/ablibs; mkdir -p $D
L=api-ratelimit_amd/csrc/libratelimit_hip.so
cp $L $D/lib_intree.so
for i in 1 2; do
  for v in "$@"; do
    cp tools/variants/lib_$v.so $L && timeout -k 10 200 python -u bench.py --steps 40 --warmup 5 --cpu-seconds 0 --no-roofline-probe > $D/$v.$i.json 2>$D/$v.$i.err || { cp $D/lib_intree.so $L; exit 1; }
  done
done
cp $D/lib_intree.so $L

#!/bin/bash
# Build timing variants of the HIP library (tools only; not used by the product).
set -e
cd "$(dirname "$0")/../api-ratelimit_amd/csrc"
mkdir -p ../../tools/variants
for v in "A:-DRL_SORT_IPT=16 -DRL_SORT_LB_WIN=16" "B:-DRL_SORT_IPT=16 -DRL_SORT_LB_WIN=32" "C:-DRL_SORT_IPT=8 -DRL_SORT_LB_WIN=16" "D:-DRL_SORT_IPT=8 -DRL_SORT_LB_WIN=32" "E:-DRL_SORT_IPT=16 -DRL_SORT_LB_WIN=16 -DRL_SORT_TICKET" "F:-DRL_SORT_IPT=16 -DRL_SORT_LB_WIN=8"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wno-unused-result $flags -shared \
     -o ../../tools/variants/lib_$name.so rl_kernels.hip rl_engine.cpp rl_cache.cpp -lpthread &
done
wait
ls -la ../../tools/variants

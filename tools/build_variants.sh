#!/bin/bash
# Build timing / diagnostic variants of the HIP library (tools only; not used by the product).
# Usage: tools/build_variants.sh "NAME:-DFLAG ..." ...   -> tools/variants/lib_NAME.so
set -e
cd "$(dirname "$0")/../api-ratelimit_amd/csrc"
mkdir -p ../../tools/variants
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wno-unused-result $flags -shared \
     -o ../../tools/variants/lib_$name.so rl_kernels.hip rl_kernels_v4.hip rl_compact.hip rl_route.hip rl_resolve.hip rl_engine.cpp rl_router.cpp rl_cache.cpp -L/opt/rocm/lib -lrccl -lpthread &
done
wait
ls ../../tools/variants

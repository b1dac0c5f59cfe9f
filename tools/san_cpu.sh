#!/bin/bash
# The CPU test suite under AddressSanitizer + UndefinedBehaviorSanitizer (the
# reference's analog is `go test -race`, /root/reference/Makefile). Builds a copy of the tree with
# SAN=1 — the oracle, the test shims (C++ DoLimit mirror, resolve walk, freecache model) and the
# host code of libratelimit_hip.so (rl_decide_raw, the resolve walk, the config and ABI paths;
# device code is not instrumented) — and runs `pytest -m "not gpu"` there with the clang ASan
# runtime preloaded into Python. Any report fails the run (halt on error, UBSan not recoverable).
# usage: tools/san_cpu.sh [pytest args...]      (CPU only; ~10 min)
set -eu
SRC=$(cd "$(dirname "$0")/.." && pwd)
DST=${SAN_DIR:-/tmp/rl-san}
rm -rf "$DST"
mkdir -p "$DST"
tar -C "$SRC" --exclude=.git --exclude=gpurun_out --exclude='*.so' --exclude='*.o' --exclude=build \
    --exclude=__pycache__ --exclude=tools/variants -cf - . | tar -C "$DST" -xf -
J=$(( $(nproc) < 8 ? $(nproc) : 8 ))
make -s -j"$J" -C "$DST/api-ratelimit_amd/csrc" SAN=1 > "$DST/san_build.log" 2>&1
make -s -C "$DST/oracle" SAN=1 >> "$DST/san_build.log" 2>&1
make -s -C "$DST/tests/cshim" SAN=1 >> "$DST/san_build.log" 2>&1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
cd "$DST"
# leaks: CPython and torch keep allocations to exit by design; everything else halts the run
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
LD_PRELOAD="$RT" python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"

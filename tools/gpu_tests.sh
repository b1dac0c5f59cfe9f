#!/bin/bash
# GPU test passes in one call, each under its own limit; a crash, abort or timeout (rc >= 124)
# stops the call there (a test failure, rc 1, does not).
# usage (on the GPU box, from the repo root): tools/gpu_tests.sh <tag> "<pytest args 1>" ["<pytest args 2>" ...]
set -u
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread $args > "$OUT/pytest$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc: $args" | tee -a "$OUT/steps.txt"
  tail -3 "$OUT/pytest$i.log"
  if [ "$rc" -ge 124 ] || [ "$rc" -lt 0 ]; then echo "stopping after pass $i (rc=$rc)"; exit "$rc"; fi
done

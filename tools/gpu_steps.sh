#!/bin/bash
# One GPU call of several steps (on the GPU box, from the repo root), each a shell command run
# under its own time limit, output to gpurun_out/<tag>/step<i>.log. A test failure (rc 1) goes
# on to the next step; a crash, abort, or time limit (rc >= 124) ends the call there.
# usage: tools/gpu_steps.sh <tag> "<seconds>:<command>" ["<seconds>:<command>" ...]
#   e.g. tools/gpu_steps.sh r6b "600:python -u -m pytest -m gpu tests/test_gpu_resolve.py -x -q" \
#                               "600:bash tools/ab.sh 30 '- tools/variants/lib_r5.so' --config 4"
set -u
export TMPDIR=/tmp
TAG=$1
shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/$TAG
mkdir -p "$OUT"
i=0
for step in "$@"; do
  i=$((i + 1))
  secs=${step%%:*}
  cmd=${step#*:}
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/step$i.log" 2>&1
  rc=$?
  echo "step $i rc=$rc: $cmd" | tee -a "$OUT/steps.txt"
  tail -4 "$OUT/step$i.log"
  if [ "$rc" -ge 124 ]; then echo "stopping after step $i (rc=$rc)"; exit "$rc"; fi
done

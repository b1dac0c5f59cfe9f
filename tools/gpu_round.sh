#!/bin/bash
# One GPU call: GPU tests (bit-exact vs the oracle), smoke, and a bench line, each under its own
# time limit. A normal test failure (rc 1) still runs the later steps; a crash, abort or
# timeout (rc >= 124 or signal) stops the call there.
# usage (on the GPU box, from the repo root): tools/gpu_round.sh <tag> [pytest -k expr] [bench args...]
set -u
TAG=$1
KEXPR=${2:-}
shift 2 || shift $#
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
stop_on_crash() {
  local rc=$1 what=$2
  echo "$what rc=$rc" | tee -a "$OUT/steps.txt"
  if [ "$rc" -ge 124 ] || [ "$rc" -lt 0 ]; then echo "stopping after $what (rc=$rc)"; exit "$rc"; fi
}
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$KEXPR" \
    > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
fi
stop_on_crash $? pytest
tail -5 "$OUT/pytest.log"
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
stop_on_crash $? smoke
timeout -k 10 600 python -u bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
stop_on_crash $? bench
cat "$OUT/bench.json"

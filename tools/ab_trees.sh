#!/bin/bash
# Interleaved A/B of whole trees (bench.py and its built libraries): the in-tree one and one or
# more other checkouts built under tools/variants/<name>/ (e.g. an earlier round's tree, for a
# regression that an ABI change keeps from an A/B of libraries alone). Prints ms/step per run.
# usage: tools/ab_trees.sh STEPS "tree1 tree2 ..." [bench args]   (tree "-" = the in-tree one)
steps=$1; trees=$2; shift 2
R=$(pwd)
mkdir -p gpurun_out
for t in $trees; do
  d=$R; [ "$t" != "-" ] && d=$R/tools/variants/$t
  (cd "$d" && timeout -k 10 200 python bench.py --steps "$steps" --warmup 30 --cpu-seconds 0 --no-roofline-probe \
     --no-host-path --no-kernel-times "$@") > gpurun_out/ab_trees.log 2>&1 || { tail -5 gpurun_out/ab_trees.log; exit 1; }
  python - "$t" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_trees.log").read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d["value"])
PY
done

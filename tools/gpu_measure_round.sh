#!/bin/bash
# The round's measurements of record, in parts that each fit one GPU call (gpurun's 20-min cap).
# Every step under its own limit; a crash or timeout (rc >= 124) ends the call.
#   part A: every GPU test, smoke, the PMC summaries of configs 3 and 4
#   part B: the PMC summaries of config 5 and of the one-rank routed step
#   part C: the bench lines (config 3 twice, configs 4 and 5, one rank over RCCL, logical shards
#           2 / 4 / 8, config 1) — run after the part-A/B summaries are copied into profiles/
# usage (on the GPU box, from the repo root): tools/gpu_measure_round.sh <tag> A|B|C
set -u
TAG=$1
PART=$2
case $PART in
  A) bash tools/gpu_steps.sh "${TAG}A" \
       "600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
       "240:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
       "500:bash tools/pmc_round.sh ${TAG}_c3 20 '' 3" \
       "500:bash tools/pmc_round.sh ${TAG}_c4 20 '' 4" ;;
  B) bash tools/gpu_steps.sh "${TAG}B" \
       "500:bash tools/pmc_round.sh ${TAG}_c5 20 '' 5" \
       "500:bash tools/pmc_routed.sh ${TAG}_routed 30" ;;
  C) bash tools/gpu_bench_round.sh "${TAG}C" "bench bench4 bench5 bench_b routed1 ls2 ls4 ls8 config1" ;;
esac

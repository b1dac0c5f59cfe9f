#!/bin/bash
# The round's measurements of record, in parts that each fit one GPU call (gpurun's 20-min cap).
# Each PMC summary is copied into profiles/ on the box before the bench line of its workload
# runs, so the line's roofline carries its `traffic` (the copies merged back to this tree are the
# gpurun_out/<tag>_c*/pmc_traffic.json files; commit them under profiles/ by the same names).
# Every step under its own limit; a crash or timeout (rc >= 124) ends the call.
#   part A: every GPU test, smoke, PMC summary of config 3, two config-3 bench lines
#   part B: PMC summaries and bench lines of configs 4 and 5
#   part C: PMC summary of the one-rank routed step, the routed line over RCCL, logical shards
#           2 / 4 / 8, config 1
# usage (on the GPU box, from the repo root): tools/gpu_measure_round.sh <tag> A|B|C
set -u
TAG=$1
PART=$2
cp_pmc() {  # pmc tag -> profiles name
  echo "cp gpurun_out/$1/pmc_traffic.json profiles/$2"
}
case $PART in
  A) bash tools/gpu_steps.sh "${TAG}A" \
       "600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
       "240:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
       "500:bash tools/pmc_round.sh ${TAG}_c3 20 '' 3" \
       "30:$(cp_pmc ${TAG}_c3 r06_pmc_traffic.json)" \
       "400:python -u bench.py > gpurun_out/${TAG}A/bench_c3.json" \
       "400:python -u bench.py > gpurun_out/${TAG}A/bench_c3_b.json" ;;
  B) bash tools/gpu_steps.sh "${TAG}B" \
       "500:bash tools/pmc_round.sh ${TAG}_c4 20 '' 4" \
       "30:$(cp_pmc ${TAG}_c4 r06_pmc_traffic_config4.json)" \
       "400:python -u bench.py --config 4 > gpurun_out/${TAG}B/bench_c4.json" \
       "500:bash tools/pmc_round.sh ${TAG}_c5 20 '' 5" \
       "30:$(cp_pmc ${TAG}_c5 r06_pmc_traffic_config5.json)" \
       "400:python -u bench.py --config 5 > gpurun_out/${TAG}B/bench_c5.json" ;;
  C) bash tools/gpu_steps.sh "${TAG}C" "500:bash tools/pmc_routed.sh ${TAG}_routed 30" &&
     bash tools/gpu_bench_round.sh "${TAG}C" "routed1 ls2 ls4 ls8 config1" ;;
esac

# Round-6 follow-up measurements: the config-4 PMC summary with k_resolve named, its bench line,
# an interleaved config-4 A/B against the round-5 library and the previous commit, config-3 lines.
T=r06m
bash tools/gpu_steps.sh ${T}D \
  "500:bash tools/pmc_round.sh ${T}_c4b 20 '' 4" \
  "30:cp gpurun_out/${T}_c4b/pmc_traffic.json profiles/r06_pmc_traffic_config4.json" \
  "400:python -u bench.py --config 4 > gpurun_out/${T}D/bench_c4.json" \
  "500:bash tools/ab.sh 30 '- tools/variants/lib_prev.so tools/variants/lib_r5.so - tools/variants/lib_prev.so tools/variants/lib_r5.so' --config 4" \
  "400:python -u bench.py > gpurun_out/${T}D/bench_c3.json"

bash tools/gpu_steps.sh r6f \
 "400:bash tools/pmc_round.sh r6f_c4 20 trace-only 4"

bash tools/gpu_steps.sh r6d \
 "300:python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resolve.py tests/test_gpu_configs45_regime.py -k 'config4 or resolve'" \
 "600:bash tools/ab.sh 30 '- tools/variants/lib_r5.so - tools/variants/lib_r5.so - tools/variants/lib_r5.so' --config 4"

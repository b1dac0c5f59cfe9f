bash tools/gpu_steps.sh r6h \
 "400:python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_router_processes.py tests/test_gpu_resolve.py" \
 "700:bash tools/ab.sh 30 '- tools/variants/lib_r5.so - tools/variants/lib_r5.so - tools/variants/lib_r5.so' --config 4" \
 "500:bash tools/ab.sh 60 '- tools/variants/lib_r5.so - tools/variants/lib_r5.so'"

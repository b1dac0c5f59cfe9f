set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 ; \
timeout -k 10 240 python -u tools/kernel_variants.py > gpurun_out/kv3.log 2>&1 && \
timeout -k 10 120 python -u tools/stamps4.py 5 lib_S4.so > gpurun_out/st4.log 2>&1

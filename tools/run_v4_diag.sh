set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/stamps4.py 5 lib_S4.so > gpurun_out/st4.log 2>&1

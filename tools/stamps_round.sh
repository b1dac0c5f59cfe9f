set -e
# Phase stamps of the v4 kernels (RL_STAMPS variant; tools/build_variants.sh "st:-DRL_STAMPS",
# optionally "stf:-DRL_STAMPS -DRL_HIST_FINE"), summarised by tools/stamps_view.py.
mkdir -p gpurun_out/st
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-roofline-probe --no-host-path --lib tools/variants/lib_st.so --dump-stamps gpurun_out/st/st.npy > gpurun_out/st/b1.json 2> gpurun_out/st/b1.err
python tools/stamps_view.py gpurun_out/st/st.npy > gpurun_out/st/view.txt
if [ -f tools/variants/lib_stf.so ]; then
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-roofline-probe --no-host-path --lib tools/variants/lib_stf.so --dump-stamps gpurun_out/st/stf.npy > gpurun_out/st/b2.json 2> gpurun_out/st/b2.err
  python tools/stamps_view.py gpurun_out/st/stf.npy fine > gpurun_out/st/viewf.txt
fi
cat gpurun_out/st/view.txt

#!/bin/bash
# One GPU call of measurements: smoke, the N=1 bench line, the routed step on a one-rank RCCL
# communicator (torchrun, two steps in flight), G logical shards (records per owner, step
# breakdown, G-GPU estimate), the config-1 row; on request the PCIe probe and rocprofv3
# timelines (rtrace: routed steps; htrace: host path kernels + copies; strace: single GPU). Each step under its own limit; a crash, abort
# or timeout (rc >= 124) stops the call there.
# usage (on the GPU box, from the repo root): tools/gpu_bench_round.sh <tag> [steps...]
set -u
export TMPDIR=/tmp
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name limit cmd...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc" | tee -a "$OUT/steps.txt"
  tail -c 1500 "$OUT/$name.json"
  echo
  if [ "$rc" -ge 124 ] || [ "$rc" -lt 0 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
for s in "${@:-smoke bench routed1 ls8 ls2 config1}"; do
  for step in $s; do
    case $step in
      smoke) run smoke 240 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
      bench) run bench 600 python -u bench.py ;;
      bench_b) run bench_b 600 python -u bench.py ;;
      bench4) run bench4 600 python -u bench.py --config 4 ;;
      bench5) run bench5 600 python -u bench.py --config 5 ;;
      routed1) run routed1 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
                 --master-port 29533 bench.py --gpus 1 --force-routed --steps 30 --warmup 10 --cpu-seconds 0 \
                 --no-host-path --no-roofline-probe ;;
      ls8) run ls8 600 python -u bench.py --logical-shards 8 --steps 10 --warmup 3 --prefill 40 ;;
      ls2) run ls2 600 python -u bench.py --logical-shards 2 --steps 10 --warmup 3 --prefill 40 ;;
      ls4) run ls4 600 python -u bench.py --logical-shards 4 --steps 10 --warmup 3 --prefill 40 ;;
      rprof) mkdir -p /tmp/rprof_$TAG && run rprof 600 rocprofv3 --kernel-trace --stats -d /tmp/rprof_$TAG -o run \
                 --output-format csv -- python3 -u bench.py --force-routed --steps 30 --warmup 10 --cpu-seconds 0 \
                 --no-host-path --no-roofline-probe && cp /tmp/rprof_$TAG/run_kernel_stats.csv "$OUT/routed_kernel_stats.csv" ;;
      config1) run config1 400 python -u bench.py --config 1 --steps 200 --warmup 20 --cpu-seconds 6 --no-roofline-probe ;;
      pcie) run pcie 120 python -u tools/pcie_probe.py 20 ;;
      rtrace) mkdir -p /tmp/rt_$TAG && run rtrace 600 rocprofv3 --kernel-trace --stats -d /tmp/rt_$TAG -o run \
                 --output-format csv -- python3 -u bench.py --force-routed --steps 30 --warmup 10 --cpu-seconds 0 \
                 --no-host-path --no-roofline-probe --no-kernel-times --prefill 2000 \
                 && python3 tools/trace_tail.py /tmp/rt_$TAG/run_kernel_trace.csv 80 > "$OUT/routed_timeline.txt" ;;
      htrace) mkdir -p /tmp/ht_$TAG && run htrace 600 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ht_$TAG -o run \
                 --output-format csv -- python3 -u bench.py --cpu-seconds 0 --no-roofline-probe --no-kernel-times \
                 --steps 20 --prefill 200 \
                 && python3 tools/copy_timeline.py /tmp/ht_$TAG/run_kernel_trace.csv /tmp/ht_$TAG/run_memory_copy_trace.csv \
                    200 500 > "$OUT/host_copy_timeline.txt" ;;
      hctrace) mkdir -p /tmp/hc_$TAG && run hctrace 600 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/hc_$TAG -o run \
                 --output-format csv -- python3 -u bench.py --cpu-seconds 0 --no-roofline-probe --no-kernel-times \
                 --steps 20 --prefill 200 --host-formats compact --host-no-probe \
                 && python3 tools/copy_timeline.py /tmp/hc_$TAG/run_kernel_trace.csv /tmp/hc_$TAG/run_memory_copy_trace.csv \
                    160 0 > "$OUT/host_compact_timeline.txt" ;;
      strace) mkdir -p /tmp/st_$TAG && run strace 600 rocprofv3 --kernel-trace --stats -d /tmp/st_$TAG -o run \
                 --output-format csv -- python3 -u bench.py --steps 30 --warmup 5 --cpu-seconds 0 --no-host-path \
                 --no-roofline-probe --no-kernel-times \
                 && python3 tools/timeline.py /tmp/st_$TAG/run_kernel_trace.csv 24 > "$OUT/timeline.txt" ;;
    esac
  done
done

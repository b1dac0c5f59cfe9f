# SQ counters of k_resolve (config 4): is it waiting on memory or issuing?
set -u
export TMPDIR=/tmp
R=$(pwd); OUT=$R/gpurun_out/pmcres; mkdir -p $OUT
cd /tmp
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU -d /tmp/pr -o run --output-format csv -- \
  python3 $R/bench.py --config 4 --steps 10 --warmup 2 --prefill 20 --cpu-seconds 0 --no-kernel-times --no-roofline-probe --no-host-path > $OUT/b.json 2> $OUT/b.err || { echo "rc=$?"; tail -5 $OUT/b.err; exit 1; }
python3 - <<'PY' > $OUT/summary.txt
import csv, glob, collections
f = glob.glob('/tmp/pr/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name'].split('(')[0][-40:]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    if r['Counter_Name'] == 'SQ_WAVES': n[k] += 1
for k, d in acc.items():
    if n[k] == 0: continue
    print(k, n[k], {c: round(v / n[k]) for c, v in sorted(d.items())})
PY
cat $OUT/summary.txt

#!/bin/bash
# One rocprofv3 --pmc pass of SQ instruction counters over a short bench (per-kernel VALU /
# SALU / LDS instruction counts and wave cycles), summarised per kernel over the timed
# dispatches. usage (GPU box, repo root): tools/pmc_sq_pass.sh <tag> [steps]
set -u
TAG=$1
STEPS=${2:-10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
P=/tmp/pmcsq_$TAG
mkdir -p "$OUT" "$P"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $P -o run --output-format csv -- python3 $R/bench.py --steps $STEPS --warmup 2 --cpu-seconds 0 \
  --no-kernel-times --no-roofline-probe --no-host-path --prefill 2000 > "$OUT/sq.json" 2> "$OUT/sq.err" || { echo "sq pass rc=$?"; tail -5 "$OUT/sq.err"; exit 1; }
python3 - "$P/run_counter_collection.csv" "$STEPS" > "$OUT/sq_summary.txt" <<'PY'
import collections, csv, sys
rows = collections.defaultdict(lambda: collections.defaultdict(list))
recs = list(csv.DictReader(open(sys.argv[1])))
recs.sort(key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
for r in recs:
    k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].replace("void ", "").strip()
    if k.startswith("k4_"):
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
n = int(sys.argv[2])
for k, c in sorted(rows.items()):
    m = {name: sum(v[-n:]) / len(v[-n:]) for name, v in c.items()}
    valu = m.get("SQ_INSTS_VALU", 0)
    # wave64 VALU issues in 2 cycles on a 32-wide SIMD; 1024 SIMDs; 2.4 GHz
    print(f"{k:10s} waves {m.get('SQ_WAVES',0):9.0f} valu/wave {valu/max(1,m.get('SQ_WAVES',1)):8.0f} "
          f"salu/wave {m.get('SQ_INSTS_SALU',0)/max(1,m.get('SQ_WAVES',1)):7.0f} lds/wave {m.get('SQ_INSTS_LDS',0)/max(1,m.get('SQ_WAVES',1)):6.0f} "
          f"valu_us_if_all_simds_busy {valu*2/1024/2.4e3:7.2f} wait_any/wave_cycles {m.get('SQ_WAIT_INST_ANY',0)/max(1,m.get('SQ_WAVE_CYCLES',1)):.2f} "
          f"busy_cycles {m.get('SQ_BUSY_CYCLES',0):.0f} gui_active {m.get('GRBM_GUI_ACTIVE',0):.0f}")
PY
cat "$OUT/sq_summary.txt"

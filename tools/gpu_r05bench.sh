# Round-5 bench lines of record (config 3 twice, configs 4 and 5, config 3 routed on one rank)
set -u
export TMPDIR=/tmp
OUT=gpurun_out/r05bench; mkdir -p $OUT
for run in a b; do
  timeout -k 10 400 python -u bench.py > $OUT/c3$run.json 2> $OUT/c3$run.err; rc=$?
  echo "c3$run rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/c3$run.err; exit $rc; }
done
for c in 4 5; do
  timeout -k 10 400 python -u bench.py --config $c > $OUT/c$c.json 2> $OUT/c$c.err; rc=$?
  echo "c$c rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/c$c.err; exit $rc; }
done
timeout -k 10 400 python -u bench.py --force-routed --cpu-seconds 1 --no-host-path > $OUT/c3routed.json 2> $OUT/c3routed.err; rc=$?
echo "routed rc=$rc"
exit $rc

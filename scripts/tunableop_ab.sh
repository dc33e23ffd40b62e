#!/bin/bash
# Tune the SMT step's GEMM shapes into a copy of the committed TunableOp table
# (TABLE, default an empty table; shapes already there are skipped), then A/B
# the bench step with the tuned table vs the default heuristics, alternating, on one box.
#   TAG=tune2 bash scripts/tunableop_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-tune2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TABLE" ]; then cp "$TABLE" $OUT/table0.csv; else rm -f $OUT/table0.csv; fi
( while sleep 30; do date >> $OUT/heartbeat; done ) & HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-10} PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/table.csv timeout -k 10 700 python3 -u scripts/tune_gemms.py > $OUT/tune.log 2>&1 \
  || { kill $HB; echo "tune failed"; tail -5 $OUT/tune.log; exit 11; }
kill $HB
COMMON="--cpu-baseline-seconds 0 --ref-mode-steps 0 --roofline-steps 0 --steps 20 --warmup 3"
for i in 1 2; do
  timeout -k 10 400 python3 bench.py $COMMON --out $OUT/base_$i.json > $OUT/base_$i.log 2>&1 || exit 12
  # TunableOp reads and writes <name><device index>.csv (table.csv -> table0.csv)
  cp $OUT/table0.csv $OUT/table_ro0.csv || exit 14
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/table_ro.csv \
    timeout -k 10 400 python3 bench.py $COMMON --out $OUT/tuned_$i.json > $OUT/tuned_$i.log 2>&1 || exit 13
done
echo tune ok

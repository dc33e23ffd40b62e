#!/bin/bash
# TunableOp search for the step's GEMMs with longer timing windows and rotating buffers (operands
# not cache-warm), then the default-vs-table check with rotating inputs. TunableOp reads / writes
# <PYTORCH_TUNABLEOP_FILENAME stem><device index>.csv.
set -o pipefail
OUT=${OUT:-gpurun_out/retune}; mkdir -p $OUT
( while sleep 30; do date >> $OUT/heartbeat; done ) & HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-60} PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=10 \
PYTORCH_TUNABLEOP_ROTATING_BUFFER_SIZE=${ROT_MB:-512} PYTORCH_TUNABLEOP_FILENAME=$OUT/table.csv \
  timeout -k 10 900 python3 -u scripts/tune_gemms.py > $OUT/tune.log 2>&1 || { kill $HB; echo "tune failed"; tail -5 $OUT/tune.log; exit 11; }
kill $HB
cp $OUT/table0.csv $OUT/ro0.csv || exit 12
for r in 1 2; do
  timeout -k 10 200 python3 scripts/diag/tunable_check.py >> $OUT/check.jsonl || exit 13
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/ro.csv \
    timeout -k 10 200 python3 scripts/diag/tunable_check.py >> $OUT/check.jsonl || exit 14
done
echo ok

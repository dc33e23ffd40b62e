#!/bin/bash
# Config 5 (fp8): tune every GEMM shape of the step inline (PyTorch TunableOp: the rowwise-scaled
# torch._scaled_mm calls and the bf16 ones) during a short fp8 bench, then A/B the fp8 step with the
# tuned table vs hipBLASLt's default heuristics, alternating, on one box.
#   TAG=r05_m bash scripts/tunableop_fp8_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-r05_m}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--fp8 --cpu-baseline-seconds 0 --ref-mode-steps 0 --roofline-steps 0 --half-resident-steps 0"
( while sleep 30; do date >> $OUT/heartbeat; done ) & HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=${TUNE_MS:-30} PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5 \
PYTORCH_TUNABLEOP_FILENAME=$OUT/table.csv timeout -k 10 800 python3 -u bench.py $SHORT --steps 2 --warmup 1 \
  > $OUT/tune.log 2>&1 || { kill $HB; echo "tune failed"; tail -5 $OUT/tune.log; exit 11; }
kill $HB
ls -la $OUT; grep -c "" $OUT/table0.csv
for i in 1 2; do
  timeout -k 10 400 python3 bench.py $SHORT --steps 20 --warmup 3 --out $OUT/base_$i.json > $OUT/base_$i.log 2>&1 || exit 12
  cp $OUT/table0.csv $OUT/table_ro0.csv || exit 14
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$OUT/table_ro.csv \
    timeout -k 10 400 python3 bench.py $SHORT --steps 20 --warmup 3 --out $OUT/tuned_$i.json > $OUT/tuned_$i.log 2>&1 || exit 13
done
python3 - <<'PY'
import json, os
o = os.environ.get("OUT_DIR", "gpurun_out/" + os.environ.get("TAG", "r05_m"))
for n in ("base_1", "tuned_1", "base_2", "tuned_2"):
    d = json.load(open(f"{o}/{n}.json"))
    print(n, d["value"], d["median_ms_per_step"], d["peak_hbm_gb"])
PY

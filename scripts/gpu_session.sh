#!/bin/bash
# One GPU call: GPU test suite, headline bench, and (optionally) a GEMM TunableOp tuning pass.
#   STEPS="tests bench tune" bash scripts/gpu_session.sh
set -o pipefail
OUT=gpurun_out/${TAG:-s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for s in ${STEPS:-tests bench}; do
  case $s in
    tests)
      timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
        > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; exit 11; } ;;
    bench)
      timeout -k 10 500 python3 bench.py --out $OUT/bench.json > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -30 $OUT/bench.log; exit 12; } ;;
    dist2)
      # bench.py --gpus 2 starts its two ranks itself (gloo: they share the one GPU of this box)
      timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --model mini --steps 3 --warmup 1 \
        --cpu-baseline-seconds 0 --out $OUT/dist2.json > $OUT/dist2.log 2>&1 || { echo "dist2 failed"; tail -30 $OUT/dist2.log; exit 16; } ;;
    dist4)
      # the 4-rank rehearsal with the DP exchange traced per rank (SMT_DP_TRACE) and per-step times
      SMT_DP_TRACE=$OUT/dptrace SMT_BENCH_STACKS=60 timeout -k 10 600 python3 bench.py --gpus 4 --dist-backend gloo \
        --model mini --full-ft-steps 4 --steps 8 --warmup 2 --cpu-baseline-seconds 0 --out $OUT/dist4.json \
        > $OUT/dist4.log 2>&1 || { echo "dist4 failed"; tail -30 $OUT/dist4.log; exit 17; } ;;
    bench_ckpt)
      timeout -k 10 500 python3 bench.py --grad-ckpt --cpu-baseline-seconds 0 --ref-mode-steps 0 --out $OUT/bench_ckpt.json \
        > $OUT/bench_ckpt.log 2>&1 || { echo "bench_ckpt failed"; tail -30 $OUT/bench_ckpt.log; exit 14; } ;;
    bench_fp8)
      timeout -k 10 500 python3 bench.py --fp8 --cpu-baseline-seconds 0 --out $OUT/bench_fp8.json > $OUT/bench_fp8.log 2>&1 \
        || { echo "bench_fp8 failed"; tail -30 $OUT/bench_fp8.log; exit 15; } ;;
    tune)
      # tuning one large shape can run for minutes without output: keep a heartbeat file growing
      ( while sleep 30; do date >> $OUT/tune_heartbeat; done ) & HB=$!
      GEMM_SHAPES=${GEMM_SHAPES:-} PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
      PYTORCH_TUNABLEOP_FILENAME=$OUT/tunableop_results%d.csv \
        timeout -k 10 900 python3 -u scripts/gemm_bench.py > $OUT/gemm_tuned.jsonl 2> $OUT/gemm_tuned.log \
        || { kill $HB; echo "tune failed"; tail -30 $OUT/gemm_tuned.log; exit 13; }
      kill $HB ;;
  esac
done
echo "session ok"

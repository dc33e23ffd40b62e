#!/bin/bash
# A/B of the dK/dV kernels (SMT_ATTN_DKV=1 lean, 2 one-wave-per-SIMD dual): correctness of the dual
# kernel on the attention tests, then scripts/attn_bench.py alternating, then short benches.
set -o pipefail
OUT=gpurun_out/${TAG:-dkv}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in 2 3; do
  SMT_ATTN_DKV=$v timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/attn_tests_dual$v.log 2>&1 || { echo "dual $v attention tests failed"; tail -30 $OUT/attn_tests_dual$v.log; exit 31; }
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad_full.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/wgrad_full.log 2>&1 || { echo "wgrad tests failed"; tail -30 $OUT/wgrad_full.log; exit 32; }
for r in 1 2; do
  for v in 1 2 3; do
    SMT_ATTN_DKV=$v timeout -k 10 120 python3 scripts/attn_bench.py --impl smt --iters 20 | sed "s/^/{\"dkv\": $v, \"rep\": $r, \"r\": /; s/$/}/" >> $OUT/attn_ab.jsonl || exit 33
  done
done
cat $OUT/attn_ab.jsonl
for v in ${BENCH_DKV:-1 3}; do
  SMT_ATTN_DKV=$v timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 --selective-steps 0 \
    --ref-mode-steps 0 --half-resident-steps 0 --raw-harvest-steps 0 --ref-rounding-steps 20 --out $OUT/bench_dkv$v.json \
    > $OUT/bench_dkv$v.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_dkv$v.log; exit 34; }
  grep "timed:\|rounding:" $OUT/bench_dkv$v.log
done
echo "ab ok"

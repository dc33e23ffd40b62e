#!/bin/bash
# A/B of the attention backward kernels: dQ (SMT_ATTN_DQ 1 lean / 2 dual) x dK/dV (SMT_ATTN_DKV 1 lean /
# 2, 3 dual). Correctness on the attention tests for each dual variant, then scripts/attn_bench.py
# alternating over the combinations (VARIANTS="dq,dkv ..."), then optionally short benches.
set -o pipefail
OUT=gpurun_out/${TAG:-attn}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARIANTS=${VARIANTS:-"1,1 2,1 1,3 2,3"}
for v in $VARIANTS; do
  dq=${v%,*}; dkv=${v#*,}
  [ "$dq,$dkv" = "1,1" ] && continue
  SMT_ATTN_DQ=$dq SMT_ATTN_DKV=$dkv timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -q --timeout 120 \
    --timeout-method thread > $OUT/attn_tests_$dq$dkv.log 2>&1 || { echo "attention tests $v failed"; tail -30 $OUT/attn_tests_$dq$dkv.log; exit 41; }
done
for r in 1 2; do
  for v in $VARIANTS; do
    dq=${v%,*}; dkv=${v#*,}
    SMT_ATTN_DQ=$dq SMT_ATTN_DKV=$dkv timeout -k 10 120 python3 scripts/attn_bench.py --impl smt --iters 20 \
      | sed "s/^/{\"dq\": $dq, \"dkv\": $dkv, \"rep\": $r, \"r\": /; s/$/}/" >> $OUT/attn_ab.jsonl || exit 42
  done
done
cat $OUT/attn_ab.jsonl
for v in ${BENCH_VARIANTS:-}; do
  dq=${v%,*}; dkv=${v#*,}
  SMT_ATTN_DQ=$dq SMT_ATTN_DKV=$dkv timeout -k 10 600 python3 bench.py --steps 20 --warmup 3 --cpu-baseline-seconds 0 \
    --selective-steps 0 --ref-mode-steps 0 --half-resident-steps 0 --raw-harvest-steps 0 --ref-rounding-steps 0 \
    --out $OUT/bench_$dq$dkv.json > $OUT/bench_$dq$dkv.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_$dq$dkv.log; exit 43; }
  grep "timed:" $OUT/bench_$dq$dkv.log
done
echo "ab ok"

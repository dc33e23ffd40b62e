#!/bin/bash
# A/B of the one-wave-per-SIMD pipelined forward (SMT_ATTN_FWD=4) against the default forward:
# the attention tests under it, then scripts/attn_bench.py alternating, ROUNDS rounds.
set -o pipefail
OUT=gpurun_out/${TAG:-fwd_pw}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SMT_ATTN_FWD=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_attention.py -x -v --timeout 120 \
  --timeout-method thread > $OUT/tests_pw.log 2>&1 || { echo "attention tests (pw) failed"; tail -30 $OUT/tests_pw.log; exit 41; }
for r in $(seq ${ROUNDS:-3}); do
  for v in 0 4; do
    SMT_ATTN_FWD=$v timeout -k 10 120 python3 scripts/attn_bench.py --impl smt --iters 20 \
      | sed "s/^/{\"fwd\": $v, \"rep\": $r, \"r\": /; s/$/}/" >> $OUT/ab.jsonl || exit 42
  done
done
cat $OUT/ab.jsonl

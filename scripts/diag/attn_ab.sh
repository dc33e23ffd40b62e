#!/bin/bash
# A/B the in-tree attention kernels against variant builds (scripts/diag/build_variant.py), one GPU call:
#   VARIANTS="ring2" bash scripts/diag/attn_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $OUT/tests.log 2>&1 \
    || { echo "attention tests failed"; tail -30 $OUT/tests.log; exit 11; }
for v in ${VARIANTS}; do
  SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
      --timeout-method thread tests/test_gpu_attention.py > $OUT/tests_$v.log 2>&1 || { echo "tests $v failed"; tail -30 $OUT/tests_$v.log; exit 12; }
done
for r in 1 2; do
  timeout -k 10 120 python3 scripts/attn_bench.py --impl smt >> $OUT/bench_main.jsonl 2>/dev/null || exit 13
  for v in ${VARIANTS}; do
    SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 120 python3 scripts/attn_bench.py --impl smt >> $OUT/bench_$v.jsonl 2>/dev/null || exit 14
  done
done
echo done

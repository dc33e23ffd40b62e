#!/bin/bash
# A/B of attention kernel variants (scripts/attn_bench.py --impl smt), interleaved processes, plus the
# attention parity tests on each variant.  VARIANTS="dkv128" OUT=gpurun_out/x.jsonl bash scripts/diag/ab_attn.sh
set -o pipefail
OUT=${OUT:-gpurun_out/attn_ab.jsonl}
mkdir -p "$(dirname "$OUT")"
for v in ${VARIANTS}; do
  SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_attention.py > "${OUT%.jsonl}_tests_$v.log" 2>&1 || { tail -20 "${OUT%.jsonl}_tests_$v.log"; exit 31; }
done
for r in $(seq ${ROUNDS:-2}); do
  timeout -k 10 120 python3 scripts/attn_bench.py --impl smt | sed 's/}$/, "variant": "default"}/' >> "$OUT" || exit 32
  for v in ${VARIANTS}; do
    SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 120 python3 scripts/attn_bench.py --impl smt \
      | sed "s/}\$/, \"variant\": \"$v\"}/" >> "$OUT" || exit 33
  done
done

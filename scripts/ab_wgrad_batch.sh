#!/bin/bash
# A/B of batched tile-wgrad kernel variants on bench-shaped launches (scripts/wgrad_batch_bench.py),
# interleaved rounds in separate processes; variants built by scripts/diag/build_variant.py.
#   OUT=gpurun_out/ab.jsonl VARIANTS="stagger" ROUNDS=2 bash scripts/ab_wgrad_batch.sh [bench args]
set -o pipefail
OUT=${OUT:-gpurun_out/wgrad_ab.jsonl}
mkdir -p "$(dirname "$OUT")"
for r in $(seq ${ROUNDS:-2}); do
  timeout -k 10 120 python3 scripts/wgrad_batch_bench.py "$@" >> "$OUT" || exit 21
  for v in ${VARIANTS:-}; do
    SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 120 python3 scripts/wgrad_batch_bench.py "$@" >> "$OUT" || exit 22
  done
done

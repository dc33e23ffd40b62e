#!/bin/bash
# round 6, session d: the last-arriver slab sum MEASURED. Kernel-variant builds of
# the same sources (scripts/diag/build_variant.py): la1 = last arriver, chunk-major schedule; la2 = last
# arriver, tile-major schedule (the variant code is in git history at 6eb62e0, removed after this run); default = wgrad_dma_kernel<kOutSlabBF16> + wgrad_reduce_batch_kernel.
# Bench-shaped batched reference-rounding launches (T 32768 = 16 x 2048), alternating builds, then
# FETCH_SIZE / WRITE_SIZE passes per build. Then the fp16 session c steps (fp16 tests, suite, dtype bench).
set -o pipefail
mkdir -p gpurun_out/r06_d
export PYTHONUNBUFFERED=1
V=scripts/diag/_variants
ARGS="--seq-len 2048 --layers 4 --iters 10"
for round in 1 2 3; do
  for lib in default la1 la2; do
    if [ $lib = default ]; then unset SMT_HIP_LIB; else export SMT_HIP_LIB=$V/libsmt_hip_$lib.so; fi
    timeout -k 10 180 python -u scripts/wgrad_batch_bench.py $ARGS --tag $lib >> gpurun_out/r06_d/wgrad_la_ab.jsonl \
      2>> gpurun_out/r06_d/wgrad_la_ab.err || exit 11
  done
done
for lib in default la1 la2; do
  if [ $lib = default ]; then unset SMT_HIP_LIB; else export SMT_HIP_LIB=$V/libsmt_hip_$lib.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex wgrad_ --output-format csv \
      -d gpurun_out/r06_d/pmc_${lib}_$c -o p -- python3 scripts/wgrad_batch_bench.py --seq-len 2048 --layers 4 --iters 2 \
      --tag $lib > gpurun_out/r06_d/pmc_${lib}_$c.log 2>&1 || exit 12
  done
done
unset SMT_HIP_LIB
bash scripts/gpu_r06_c.sh

#!/bin/bash
# round 6, session l: the reference rounding's reduce with 16-B slab loads (8 elements per thread)
# against the round-5 reduce (8-B loads, 4 elements per thread; variant "old" built from the previous
# source by scripts/diag/build_variant.py). Bench-shaped batched launches (T 32768 = 16 x 2048),
# alternating builds (checksums must agree), a kernel trace per build, then the wgrad tests.
set -o pipefail
O=gpurun_out/r06_l; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
V=scripts/diag/_variants
ARGS="--seq-len 2048 --layers 4 --iters 10"
for round in 1 2 3; do
  for lib in new old; do
    if [ $lib = new ]; then unset SMT_HIP_LIB; else export SMT_HIP_LIB=$V/libsmt_hip_$lib.so; fi
    timeout -k 10 180 python -u scripts/wgrad_batch_bench.py $ARGS --tag $lib >> $O/reduce16_ab.jsonl 2>> $O/reduce16_ab.err || exit 11
  done
done
for lib in new old; do
  if [ $lib = new ]; then unset SMT_HIP_LIB; else export SMT_HIP_LIB=$V/libsmt_hip_$lib.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$lib -o t -- \
    python3 scripts/wgrad_batch_bench.py $ARGS --tag $lib > $O/trace_$lib.log 2>&1 || exit 12
done
unset SMT_HIP_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_wgrad_full.py \
  tests/test_gpu_wgrad_batch.py tests/test_gpu_wgrad_dtypes.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 13; }
tail -2 $O/tests.log
cat $O/reduce16_ab.jsonl | cut -c1-300

#!/bin/bash
# One GPU call: write-through (sc1, default) vs plain split-K slab stores of the tile wgrad, on
# bench-shaped batched launches (reference rounding: per-sample bf16 slabs; single: fp32 slabs),
# alternating, then the wgrad GPU tests on the default build.
#   bash scripts/ab_wgrad_slab_sc1.sh      (needs scripts/diag/_variants/libsmt_hip_slabplain.so:
#   python scripts/diag/build_variant.py slabplain -DSMT_WGRAD_SLAB_SC1=0)
set -o pipefail
O=gpurun_out/${TAG:-r05_i}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PLAIN=scripts/diag/_variants/libsmt_hip_slabplain.so
for rep in 1 2; do
  for seq in 2048 0; do
    timeout -k 10 120 python3 scripts/wgrad_batch_bench.py --layers 4 --iters 10 --seq-len $seq --tag sc1 >> $O/slab_ab.jsonl || exit 11
    SMT_HIP_LIB=$PLAIN timeout -k 10 120 python3 scripts/wgrad_batch_bench.py --layers 4 --iters 10 --seq-len $seq --tag plain >> $O/slab_ab.jsonl || exit 12
  done
done
cat $O/slab_ab.jsonl
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_wgrad_full.py tests/test_gpu_wgrad_batch.py tests/test_gpu_kernels.py tests/test_gpu_mx.py -x -q --timeout 300 --timeout-method thread > $O/wgrad_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/wgrad_tests.log; exit 13; }
tail -2 $O/wgrad_tests.log

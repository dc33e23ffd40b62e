#!/bin/bash
# One GPU call: the fp16 / fp32 tile-gradient tests (incl. the channel module), then the batched tile
# wgrad on bench-shaped launches in each operand dtype (reference rounding and single).
#   TAG=r05_p2 bash scripts/gpu_r05_dtypes.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_p2}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_wgrad_dtypes.py tests/test_gpu_channel.py -x -v -s --timeout 200 --timeout-method thread > $O/dtype_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/dtype_tests.log; exit 11; }
tail -2 $O/dtype_tests.log
for dt in bf16 fp16 fp32; do
  for seq in 2048 0; do
    timeout -k 10 180 python3 scripts/wgrad_batch_bench.py --layers 4 --iters 5 --seq-len $seq --dtype $dt >> $O/wgrad_dtypes.jsonl || exit 12
  done
done
cat $O/wgrad_dtypes.jsonl

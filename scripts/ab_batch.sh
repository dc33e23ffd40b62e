#!/bin/bash
# A/B of the batched tile wgrad on one box: bench (bf16 and fp8) with one launch per module vs batched.
#   TAG=ab bash scripts/ab_batch.sh
set -o pipefail
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
COMMON="--cpu-baseline-seconds 0 --ref-mode-steps 0 --steps ${STEPS:-30}"
for mode in ${MODES:-fp8 bf16}; do
  extra=""; [ "$mode" = fp8 ] && extra="--fp8"
  for bt in ${BATCH_TILES:-0 48}; do
    timeout -k 10 500 python3 bench.py $extra $COMMON --wgrad-batch-tiles $bt --out $OUT/${mode}_bt$bt.json \
      > $OUT/${mode}_bt$bt.log 2>&1 || { echo "bench $mode $bt failed"; tail -20 $OUT/${mode}_bt$bt.log; exit 1; }
  done
done
echo ab ok

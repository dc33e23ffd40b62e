#!/bin/bash
# A/B of the engine's wgrad batch size (tiles per batched launch) on one box: the bench's wgrad
# roofline (kernel alone) and step time per setting.
#   TAG=x SIZES="48 96 160" bash scripts/ab_batch_tiles.sh
set -o pipefail
OUT=gpurun_out/${TAG:-abbt}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in ${SIZES:-48 96}; do
  timeout -k 10 400 python3 bench.py --cpu-baseline-seconds 0 --ref-mode-steps 0 --steps ${STEPS:-10} --warmup 3 \
      --wgrad-batch-tiles $n ${BENCH_ARGS:-} --out $OUT/bt_$n.json > $OUT/bt_$n.log 2>&1 \
    || { echo "bench $n failed"; tail -20 $OUT/bt_$n.log; exit 1; }
done
echo ab ok

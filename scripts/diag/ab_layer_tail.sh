#!/bin/bash
# bench.py with the MLP residual add fused into the next layer's input norm (default) vs not
# (SMT_FUSED_LAYER_TAIL=0), alternating; short runs (extra modes off).
set -o pipefail
OUT=${OUT:-gpurun_out/tail}; mkdir -p $OUT
A="--steps 20 --warmup 3 --ref-mode-steps 0 --selective-steps 0 --views-steps 0 --half-resident-steps 0 --ref-rounding-steps 0 --raw-harvest-steps 0 --cpu-baseline-seconds 0 --roofline-steps 0"
for r in 1 2; do
  SMT_FUSED_LAYER_TAIL=0 timeout -k 10 300 python3 bench.py $A --out $OUT/sep_$r.json > $OUT/sep_$r.log 2>&1 || exit 12
  timeout -k 10 300 python3 bench.py $A --out $OUT/tail_$r.json > $OUT/tail_$r.log 2>&1 || exit 13
done
echo ok

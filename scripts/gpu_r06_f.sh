#!/bin/bash
# round 6, session f: the resident headline with and without the W^T copies (alternating, one box):
# the recompute point ran faster without them (profiles/r06_b_bench.json), so the resident step is
# measured both ways before any default changes; then config 4 (LLaMA-2-13B channel path) at the
# reference's recompute policy, where the engine's "auto" now drops the copies.
set -o pipefail
mkdir -p gpurun_out/r06_f
export PYTHONUNBUFFERED=1
SHORT="--steps 20 --warmup 5 --ref-mode-steps 0 --selective-steps 0 --views-steps 0 --half-resident-steps 0 --ref-rounding-steps 0 --raw-harvest-steps 0 --no-transposed-steps 0 --cpu-baseline-seconds 0 --roofline-steps 0"
for round in 1 2; do
  for t in on off; do
    timeout -k 10 400 python -u bench.py $SHORT --transposed-dgrad $t --out gpurun_out/r06_f/headline_t${t}_$round.json \
      > gpurun_out/r06_f/headline_t${t}_$round.log 2>&1 || exit 11
  done
done
timeout -k 10 600 python -u scripts/config4_bench.py --grad-ckpt --out gpurun_out/r06_f/config4_ckpt.json \
  > gpurun_out/r06_f/config4_ckpt.log 2>&1 || exit 12

#!/bin/bash
# One GPU call: fp8 GPU tests, then bench.py --fp8 interleaved on one box: MX tiles with the packed
# gate/up output gradients (default), MX tiles writing the whole gradients (SMT_FP8_PACK_SWIGLU_GRAD=0),
# and the bf16 tile path (SMT_FP8_TILE_WGRAD=bf16).
set -o pipefail
OUT=gpurun_out/${TAG:-fp}
mkdir -p $OUT
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py \
  tests/test_gpu_wgrad_batch.py tests/test_gpu_checkpoint.py > $OUT/tests.log 2>&1 || exit 11
ARGS="--fp8 --steps ${STEPS:-20} --warmup 3 --cpu-baseline-seconds 0 --ref-mode-steps 0 --selective-steps 0 --half-resident-steps 0 --roofline-steps 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $ARGS > $OUT/pack$r.json 2> $OUT/pack$r.log || exit 12
  SMT_FP8_PACK_SWIGLU_GRAD=0 timeout -k 10 300 python bench.py $ARGS > $OUT/full$r.json 2> $OUT/full$r.log || exit 13
  SMT_FP8_TILE_WGRAD=bf16 timeout -k 10 300 python bench.py $ARGS > $OUT/bf16t$r.json 2> $OUT/bf16t$r.log || exit 14
done
echo done

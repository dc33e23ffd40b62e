#!/bin/bash
# round 6, session c: ABI v13 (fp16 fused ops / attention / loss): the new fp16 tests, the whole GPU
# suite (the model-op ABI changed for bf16 too), then the reference's --dtype fp16 vs bf16 at the
# recompute policy on the fused path
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_fused_fp16.py tests/test_gpu_cross_entropy.py \
  > gpurun_out/r06_c_fp16_tests.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r06_c_gpu_suite.log 2>&1 || exit $?
for dt in bf16 fp16; do
  timeout -k 10 300 python -u scripts/dtype_step_bench.py --dtype $dt --steps 10 --out gpurun_out/r06_c_dtype_$dt.json \
    > gpurun_out/r06_c_dtype_$dt.log 2>&1 || exit $?
done

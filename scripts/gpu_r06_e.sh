#!/bin/bash
# round 6, session e: the whole GPU suite on ABI v13, the reference's --dtype fp16 vs bf16 on the fused
# path, and the fp8 MX tile wgrad's kernel trace + FETCH / WRITE counters (item 6)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r06_e_gpu_suite.log 2>&1 || exit $?
for dt in bf16 fp16; do
  timeout -k 10 300 python -u scripts/dtype_step_bench.py --dtype $dt --steps 10 --out gpurun_out/r06_e_dtype_$dt.json \
    > gpurun_out/r06_e_dtype_$dt.log 2>&1 || exit $?
done
PROFILE_TAG=r06_e_fp8 SKIP_BENCH=1 BENCH_ARGS="--fp8" bash scripts/gpu_round_profile.sh

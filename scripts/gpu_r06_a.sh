#!/bin/bash
# round 6, session a: the 8B world-2 DP equivalence and the B = 2 full-depth parity (item 2)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SMT_PARITY_DUMP=gpurun_out/r06_a_parity_8b_full.json timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
  tests/test_gpu_parity_8b_full.py > gpurun_out/r06_a_parity_8b_full.log 2>&1 || exit $?
timeout -k 10 1000 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread tests/test_gpu_dp_8b.py \
  > gpurun_out/r06_a_dp8b.log 2>&1

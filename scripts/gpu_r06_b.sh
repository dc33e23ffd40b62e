#!/bin/bash
# round 6, session b: the reference's memory policy without the W^T copies
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  "tests/test_gpu_parity.py::test_transposed_dgrad_auto_follows_recompute_and_toggles_live" \
  "tests/test_gpu_parity.py::test_transposed_dgrad_matches_plain_dgrad" > gpurun_out/r06_b_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gemm_layout_bench.py > gpurun_out/r06_b_gemm_layout.jsonl 2> gpurun_out/r06_b_gemm_layout.err || exit $?
timeout -k 10 900 python -u bench.py --out gpurun_out/r06_b_bench.json > gpurun_out/r06_b_bench.log 2>&1

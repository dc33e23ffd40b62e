#!/bin/bash
# One GPU call: the whole GPU suite, then config 5 (fp8) and config 4 (LLaMA-2-13B channel path) benches.
#   TAG=r05_x bash scripts/gpu_r05_ext.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_x}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 11; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 bench.py --fp8 --cpu-baseline-seconds 0 --out $O/bench_fp8.json > $O/bench_fp8.log 2>&1 \
  || { echo "fp8 bench failed"; tail -30 $O/bench_fp8.log; exit 12; }
head -c 300 $O/bench_fp8.json; echo
timeout -k 10 700 python3 scripts/config4_bench.py --out $O/config4.json > $O/config4.log 2>&1 \
  || { echo "config4 failed"; tail -30 $O/config4.log; exit 13; }
head -c 300 $O/config4.json

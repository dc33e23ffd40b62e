#!/bin/bash
# One GPU call: the fused LM head + loss (tests, chunk-size micro-benchmark), then the full GPU suite
# and the default bench line.
#   TAG=r05_h bash scripts/gpu_r05_lmhead.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_h}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_cross_entropy.py -x -v -s --timeout 200 --timeout-method thread > $O/ce_tests.log 2>&1 \
  || { echo "ce tests failed"; tail -40 $O/ce_tests.log; exit 11; }
tail -2 $O/ce_tests.log
timeout -k 10 300 python3 -u scripts/lm_head_loss_bench.py --out $O/lm_head_loss.jsonl > $O/lm_head_loss.log 2>&1 \
  || { echo "lm head bench failed"; tail -30 $O/lm_head_loss.log; exit 12; }
cat $O/lm_head_loss.jsonl
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 13; }
tail -2 $O/gpu_tests.log
timeout -k 10 700 python3 bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 14; }
head -c 600 $O/bench.json

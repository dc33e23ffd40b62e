#!/bin/bash
# One GPU call: the tests named in FIRST (verbose, -s), the whole GPU suite, then the default bench line.
#   TAG=r05_j FIRST="tests/test_gpu_shared_blocks.py" bash scripts/gpu_r05_check.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_j}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$FIRST" ]; then
  timeout -k 10 400 python3 -u -m pytest $FIRST -x -v -s --timeout 300 --timeout-method thread > $O/first_tests.log 2>&1 \
    || { echo "first tests failed"; tail -40 $O/first_tests.log; exit 11; }
  tail -2 $O/first_tests.log
fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 12; }
tail -2 $O/gpu_tests.log
timeout -k 10 700 python3 bench.py ${BENCH_ARGS:-} --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 13; }
head -c 400 $O/bench.json

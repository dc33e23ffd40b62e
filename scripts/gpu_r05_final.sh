#!/bin/bash
# One GPU call: the whole GPU suite, smoke(), and the default bench line (the driver's round-end order).
#   TAG=r05_f bash scripts/gpu_r05_final.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_f}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 11; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 12; }
tail -2 $O/smoke.log
timeout -k 10 700 python3 bench.py --out $O/bench.json > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 13; }
head -c 400 $O/bench.json

#!/bin/bash
# The channel GPU tests, then config 4 with the shared q/k/v column gather (default) and without it.
set -o pipefail
O=gpurun_out/${TAG:-r05_c4}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_channel.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/tests.log; exit 11; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 700 python3 scripts/config4_bench.py --out $O/c4_shared_$r.json > $O/c4_shared_$r.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4_shared_$r.log; exit 12; }
  SMT_SHARED_CGATHER=0 timeout -k 10 700 python3 scripts/config4_bench.py --out $O/c4_separate_$r.json > $O/c4_separate_$r.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4_separate_$r.log; exit 13; }
done
echo done

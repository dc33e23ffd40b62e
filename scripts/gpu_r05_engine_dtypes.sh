#!/bin/bash
# One GPU call: the engine in fp16 / fp32 (ABI v12 parameter dtypes, fp16 loss scaling), then the
# AdamW / engine / parity tests the change touches, then smoke.
#   TAG=r05_s bash scripts/gpu_r05_engine_dtypes.sh
set -o pipefail
O=gpurun_out/${TAG:-r05_s}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine_dtypes.py tests/test_gpu_kernels.py tests/test_gpu_parity.py \
  tests/test_gpu_wgrad_dtypes.py -x -v -s --timeout 200 --timeout-method thread > $O/engine_dtype_tests.log 2>&1 \
  || { echo "tests failed"; tail -40 $O/engine_dtype_tests.log; exit 11; }
tail -2 $O/engine_dtype_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 12; }
tail -3 $O/smoke.log

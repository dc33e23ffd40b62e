#!/bin/bash
# round 6, session h: the reference's --dtype fp16 against bf16 at the headline's policy (activations
# resident, W^T copies) on the fused path, then the whole GPU suite and smoke() on the final tree.
set -o pipefail
O=gpurun_out/r06_h; mkdir -p $O
export PYTHONUNBUFFERED=1
for dt in bf16 fp16; do
  timeout -k 10 400 python -u scripts/dtype_step_bench.py --dtype $dt --resident --steps 10 --out $O/dtype_resident_$dt.json \
    > $O/dtype_resident_$dt.log 2>&1 || { tail -30 $O/dtype_resident_$dt.log; exit 11; }
  tail -c 400 $O/dtype_resident_$dt.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gpu_suite.log 2>&1 \
  || { tail -40 $O/gpu_suite.log; exit 12; }
tail -2 $O/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 13; }
tail -3 $O/smoke.log

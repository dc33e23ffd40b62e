#!/bin/bash
# round 6, session i: the extension rows on the final tree (config 5's fp8 bench line, config 4 with
# activations resident), and where fp16's 2 % goes at the resident policy (kernel-trace stats of
# both dtypes' steps).
set -o pipefail
O=gpurun_out/r06_i; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u bench.py --fp8 --out $O/bench_fp8.json > $O/bench_fp8.log 2>&1 || { tail -30 $O/bench_fp8.log; exit 11; }
head -c 300 $O/bench_fp8.json; echo
timeout -k 10 600 python -u scripts/config4_bench.py --out $O/config4.json > $O/config4.log 2>&1 || { tail -30 $O/config4.log; exit 12; }
head -c 300 $O/config4.json; echo
for dt in bf16 fp16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$dt -o s -- \
    python3 scripts/dtype_step_bench.py --dtype $dt --resident --steps 4 --warmup 2 > $O/trace_$dt.log 2>&1 \
    || { tail -30 $O/trace_$dt.log; exit 13; }
done
echo done

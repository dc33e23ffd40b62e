#!/bin/bash
# One GPU call: stream concurrency probe, then kernel traces of a short fp8 bench (overlap on) with
# MX tiles and with bf16 tiles, reduced to per-queue step timelines (scripts/diag/stream_tail.py).
set -o pipefail
OUT=gpurun_out/${TAG:-ft}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--fp8 --steps 4 --warmup 1 --cpu-baseline-seconds 0 --ref-mode-steps 0 --selective-steps 0 --half-resident-steps 0 --roofline-steps 0"
timeout -k 10 180 python3 -u scripts/diag/stream_concurrency.py > $OUT/concurrency.jsonl 2>$OUT/concurrency.err || exit 11
for v in mx bf16; do
  SMT_FP8_TILE_WGRAD=$v timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o bench -- python3 bench.py $SHORT > $OUT/$v.log 2>&1 || exit 12
  python3 scripts/diag/stream_tail.py $OUT/$v/bench_kernel_trace.csv $v > $OUT/${v}_tail.jsonl || exit 13
  python3 scripts/trace_steps.py $OUT/$v/bench_kernel_trace.csv > $OUT/${v}_steps.txt || exit 14
  rm -f $OUT/$v/bench_kernel_trace.csv
done
echo done

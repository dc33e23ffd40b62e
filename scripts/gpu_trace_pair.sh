#!/bin/bash
# One GPU call: rocprofv3 kernel traces of a short bf16 bench and a short fp8 bench (step breakdowns).
set -o pipefail
OUT=gpurun_out/${TAG:-tp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--steps 3 --warmup 1 --cpu-baseline-seconds 0 --ref-mode-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bf16 -o bench -- python3 bench.py $SHORT > $OUT/bf16.log 2>&1 || exit 11
python3 scripts/trace_steps.py $OUT/bf16/bench_kernel_trace.csv > $OUT/bf16_steps.txt || exit 12
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fp8 -o bench -- python3 bench.py --fp8 $SHORT > $OUT/fp8.log 2>&1 || exit 13
python3 scripts/trace_steps.py $OUT/fp8/bench_kernel_trace.csv > $OUT/fp8_steps.txt || exit 14
rm -f $OUT/bf16/bench_kernel_trace.csv $OUT/fp8/bench_kernel_trace.csv
echo done

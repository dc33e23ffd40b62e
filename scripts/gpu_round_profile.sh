#!/bin/bash
# One GPU call: headline bench, kernel-trace stats of a short bench, and the two PMC passes for the
# wgrad kernel (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   PROFILE_TAG=r02_x SKIP_BENCH=1 bash scripts/gpu_round_profile.sh
set -o pipefail
OUT=gpurun_out/${PROFILE_TAG:-r02}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
# the kernel alone (wgrad stream joined), as bench.py measures the roofline: the averages must agree
SHORT="--steps 3 --warmup 1 --cpu-baseline-seconds 0 --ref-mode-steps 0 --selective-steps 0 --views-steps 0 --ref-rounding-steps 0 --raw-harvest-steps 0 --half-resident-steps 0 --no-transposed-steps 0 --no-overlap-wgrad --roofline-steps 0 ${BENCH_ARGS:-}"
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 800 python3 bench.py ${BENCH_ARGS:-} --out $OUT/bench.json > $OUT/bench.log 2>&1 || exit 11
fi
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py $SHORT > $OUT/trace.log 2>&1 || exit 12
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex wgrad_ --output-format csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py $SHORT > $OUT/pmc_fetch.log 2>&1 || exit 13
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex wgrad_ --output-format csv -d $OUT/pmc_write -o write -- python3 bench.py $SHORT > $OUT/pmc_write.log 2>&1 || exit 14
echo done

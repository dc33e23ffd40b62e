#!/bin/bash
# One GPU call: fp8 bench with an env toggle on / off (A/B on one box) and a kernel trace of the "on" arm.
#   TOGGLE=SMT_FP8_FUSED_SWIGLU_FWD bash scripts/diag/fp8_ab.sh
set -o pipefail
OUT=gpurun_out/${TAG:-fab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--steps 3 --warmup 1 --cpu-baseline-seconds 0 --ref-mode-steps 0"
for arm in 1 0 1 0; do
  env $TOGGLE=$arm timeout -k 10 400 python3 bench.py --fp8 --steps 6 --cpu-baseline-seconds 0 --ref-mode-steps 0 --out $OUT/b_$arm.json >> $OUT/b.log 2>&1 || exit 11
  grep -o '"ms_per_step": [0-9.]*' $OUT/b_$arm.json | sed "s/^/$TOGGLE=$arm /" >> $OUT/ab.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tr -o t -- python3 bench.py --fp8 $SHORT > $OUT/tr.log 2>&1 || exit 12
python3 scripts/trace_steps.py $OUT/tr/t_kernel_trace.csv > $OUT/steps.txt || exit 13
rm -f $OUT/tr/t_kernel_trace.csv
echo done

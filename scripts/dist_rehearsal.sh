#!/bin/bash
# Multi-rank rehearsals of bench.py on the one-GPU box (gloo; the ranks share the card), each with the
# DP exchange traced per rank (SMT_DP_TRACE) and per-step times. One variant per argument:
#   base     the defaults
#   hwq1     GPU_MAX_HW_QUEUES=1 (one hardware compute queue per process)
#   nosdma   HSA_ENABLE_SDMA=0 (copies by blit kernels instead of SDMA engines)
#   RANKS=4 TAG=r04_b bash scripts/dist_rehearsal.sh hwq1 nosdma
set -o pipefail
OUT=gpurun_out/${TAG:-dist}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
R=${RANKS:-4}
ARGS="--gpus $R --dist-backend gloo --model mini --full-ft-steps ${FT:-3} --steps 6 --warmup 1 --cpu-baseline-seconds 0 \
  --selective-steps 0 --views-steps 0 --ref-mode-steps 0 --ref-rounding-steps 0 --raw-harvest-steps 0 --roofline-steps 0"
for v in "$@"; do
  case $v in
    base) ENVS="" ;;
    hwq1) ENVS="GPU_MAX_HW_QUEUES=1" ;;
    nosdma) ENVS="HSA_ENABLE_SDMA=0" ;;
    *) echo "unknown variant $v"; exit 2 ;;
  esac
  echo "== $v: $ENVS" | tee -a $OUT/rehearsal.log
  env $ENVS SMT_DP_TRACE=$OUT/dptrace_$v SMT_BENCH_STACKS=120 timeout -k 10 ${LIMIT:-420} python3 bench.py $ARGS \
    --out $OUT/dist${R}_$v.json > $OUT/dist${R}_$v.log 2>&1 || { echo "$v failed rc=$?"; tail -20 $OUT/dist${R}_$v.log; exit 21; }
  grep "warm-up\|timed:" $OUT/dist${R}_$v.log | tee -a $OUT/rehearsal.log
done
echo "rehearsal ok"

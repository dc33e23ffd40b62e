#!/bin/bash
# A/B of kernel environment knobs on one box: the bench's wgrad roofline (kernel alone) per setting.
#   TAG=x VARIANTS="base SMT_JOINT_QKV=0" bash scripts/ab_env.sh
set -o pipefail
OUT=gpurun_out/${TAG:-abenv}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
COMMON="--cpu-baseline-seconds 0 --ref-mode-steps 0 --steps ${STEPS:-10} --warmup 3 ${BENCH_ARGS:-}"
i=0
for v in ${VARIANTS:-base}; do
  i=$((i+1))
  name=${i}_${v//=/_}
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 500 python3 bench.py $COMMON --out $OUT/$name.json > $OUT/$name.log 2>&1 \
    || { echo "bench $v failed"; tail -20 $OUT/$name.log; exit 1; }
done
echo ab ok

#!/bin/bash
# One GPU call: kernel-trace stats and PMC counter passes for the flash-attention kernels
# (attn_fwd / attn_dq / attn_dkdv) at the bench shape B16 Hq32 Hkv8 S2048 D128.
#   TAG=r03_attn bash scripts/attn_pmc.sh
# Each --pmc pass is its own run (gfx950: <= 8 SQ, <= 4 TCC, <= 2 GRBM counters per pass); a pass
# keeps only the counters `rocprofv3 -L` lists on this box.
set -o pipefail
OUT=gpurun_out/${TAG:-attn_pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${ATTN_ARGS:-"--impl smt --iters 5"}
timeout -k 10 120 python3 scripts/attn_bench.py $ARGS > $OUT/attn_bench.jsonl 2> $OUT/attn_bench.log || exit 11
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o attn -- \
  python3 scripts/attn_bench.py $ARGS > $OUT/trace.log 2>&1 || exit 12
pass=0
for set in "${PMC_SETS[@]:-}" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES" \
  "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT" \
  "FETCH_SIZE" "WRITE_SIZE"; do
  [ -z "$set" ] && continue
  keep=""
  for c in $set; do grep -qw "$c" $OUT/counters.txt && keep="$keep $c"; done
  pass=$((pass + 1))
  echo "pass $pass:$keep" >> $OUT/passes.txt
  [ -z "$keep" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $keep --kernel-include-regex attn_ --output-format csv -d $OUT/pmc$pass -o p -- \
    python3 scripts/attn_bench.py --impl smt --iters 2 > $OUT/pmc$pass.log 2>&1 || { echo "pmc pass $pass failed"; exit 13; }
done
echo done

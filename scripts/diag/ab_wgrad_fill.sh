mkdir -p gpurun_out/r03_s2_ab5
O=gpurun_out/r03_s2_ab5/fill.jsonl
for r in 1 2; do
timeout -k 10 120 python3 scripts/wgrad_batch_bench.py --tag default >> $O || exit 1
SMT_WGRAD_SLOTS=5 timeout -k 10 120 python3 scripts/wgrad_batch_bench.py --tag slots5 >> $O || exit 1
for v in noswz nomfma fillnoswz; do SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_$v.so timeout -k 10 120 python3 scripts/wgrad_batch_bench.py --tag $v >> $O || exit 1; done
done

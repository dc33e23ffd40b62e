set -o pipefail
OUT=gpurun_out/r04_bb; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 11; }
A="--steps 20 --warmup 3 --ref-mode-steps 0 --selective-steps 0 --views-steps 0 --half-resident-steps 0 --ref-rounding-steps 0 --raw-harvest-steps 0 --cpu-baseline-seconds 0 --roofline-steps 0"
for r in 1 2; do
  SMT_JOINT_QKV=0 timeout -k 10 300 python3 bench.py $A --out $OUT/sep_$r.json > $OUT/sep_$r.log 2>&1 || exit 12
  timeout -k 10 300 python3 bench.py $A --out $OUT/joint_$r.json > $OUT/joint_$r.log 2>&1 || exit 13
done
echo ok

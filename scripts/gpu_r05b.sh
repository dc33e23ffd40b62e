set -o pipefail
O=gpurun_out/${TAG:-r05b}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 11; }
tail -3 $O/gpu_tests.log
timeout -k 10 600 python3 bench.py --gpus 1 --dist-backend nccl --out $O/bench_nccl.json > $O/bench_nccl.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_nccl.log; exit 12; }
cat $O/bench_nccl.json | head -c 600

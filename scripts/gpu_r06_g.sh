#!/bin/bash
# round 6, session g: norm_dist tie order on the GPU scan (block and channel, incl. the near-tie
# fixtures), then the round's profile of the default bench line: the bench itself, the kernel-trace
# stats of a short run and the wgrad FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_round_profile.sh).
set -o pipefail
O=gpurun_out/r06_g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_channel.py -k "selection or norm_dist or near_tie or ties" \
  > $O/tie_tests.log 2>&1 || { tail -40 $O/tie_tests.log; exit 11; }
tail -3 $O/tie_tests.log
PROFILE_TAG=r06_g bash scripts/gpu_round_profile.sh || exit 12
python scripts/pmc_traffic.py $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv $O/wgrad_pmc.json || exit 13
head -c 600 $O/bench.json

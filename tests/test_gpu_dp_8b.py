"""BASELINE config 3 multi-rank at the real LLaMA-3-8B geometry.

The DP equivalence of tests/test_gpu_dp_equivalence.py, on a 2-layer 512-wide model there, here at
the shapes the bench and the driver's 8-GPU scaling run use: two ranks (gloo, both on cuda:0, one
hardware queue each: DESIGN §7) each run ONE sample of S = 256 and must equal, bit for bit, one rank
running the same two samples as two gradient-accumulation micro-steps (the 1/2 of the average and of
the accumulation are exact power-of-two scalings, and the exchange sums two ranks' gradients as
accumulation adds two micro-steps'). The reference's exchange is DeepSpeed's, implicit in
``model.backward`` (fine_tune.py:712), in ZeRO-2 buckets of ``reduce_bucket_size`` elements
(deepspeed_helpers.py:73). Worker: tests/dp8b_worker.py.

* SMT phase, full depth: 32 layers, 872 tiles in whole-module buckets of the engine's default size
  over the 229 MB packed fp32 tile-gradient buffer, two SMT steps. Asserted equal: the fp32 master,
  exp_avg and exp_avg_sq of all 57.1 M tile parameters, every SMT module's tiles in W (exact) and its
  whole W (bit checksums).
* Warm-up dense buckets at 8B width: 2 decoder layers plus the full 128256-entry embedding and untied
  LM head (1 GB of bf16 each) through DenseGradBuckets at the reference's 1e6-element buckets, one
  full fine-tuning step with the layers recomputed, the harvest, the rank-0 selection broadcast, one
  SMT step. Asserted equal: every parameter and its fp32 master / moments after the warm-up
  (checksums), the harvest accumulators (checksums), the selection, and the SMT state as above.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp8b_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_both(part, tmp_path):
    outs = {}
    for mode in ("acc", "dp"):
        out = str(tmp_path / f"{part}_{mode}.pt")
        if mode == "dp":
            cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--part", part,
                   "--mode", "dp", "--out", out]
        else:
            cmd = [sys.executable, "-u", WORKER, "--part", part, "--mode", "acc", "--out", out]
        # ranks share cuda:0: one hardware queue per process (oversubscribed queues stall)
        env = dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES="1")
        # the children's progress lines are passed through as they come (a long silent GPU test looks hung)
        proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        tail = []
        for line in proc.stdout:
            print(line, end="", flush=True)
            tail = (tail + [line])[-60:]
        rc = proc.wait(timeout=700)
        assert rc == 0, "".join(tail)
        outs[mode] = torch.load(out, weights_only=True)
    return outs["dp"], outs["acc"]


def _assert_smt_state_equal(dp, acc):
    assert dp["world"] == 2 and acc["world"] == 1
    assert dp["n_tiles"] == acc["n_tiles"] and dp["n_modules"] == acc["n_modules"]
    assert len(dp["buckets"]) > 1 and dp["tile_issued"] == len(dp["buckets"]) * dp.get("smt_steps", 1)
    for k in ("master", "exp_avg", "exp_avg_sq"):
        assert torch.equal(dp[k], acc[k]), k
    assert sorted(dp["W_tiles"]) == sorted(acc["W_tiles"])
    for n in acc["W_tiles"]:
        assert torch.equal(dp["W_tiles"][n], acc["W_tiles"][n]), n
        assert dp["W_hash"][n] == acc["W_hash"][n], n


def _bucket_table(dp):
    sizes = [e - s for s, e, _n in dp["buckets"]]
    mods = [n for _s, _e, n in dp["buckets"]]
    return (f"{len(sizes)} tile buckets: {min(sizes) / 1e6:.2f}-{max(sizes) / 1e6:.2f} M elements "
            f"({min(mods)}-{max(mods)} modules each), {sum(sizes) * 4 / 1e6:.1f} MB fp32 in all")


@pytest.mark.timeout(1500)
def test_dp2_llama3_8b_smt_step_equals_gradient_accumulation(tmp_path):
    dp, acc = _run_both("smt", tmp_path)
    dp["smt_steps"] = 2
    assert dp["n_tiles"] == 872 and dp["reduce_bucket_size"] == 4_000_000
    assert dp["sel_att"] == acc["sel_att"] and dp["sel_mlp"] == acc["sel_mlp"]
    print(f"\n8B SMT phase, world 2: {_bucket_table(dp)}; {dp['tile_issued']} all-reduces over 2 steps; "
          f"peak {dp['peak_gb']:.1f} GB per rank (acc {acc['peak_gb']:.1f} GB)")
    _assert_smt_state_equal(dp, acc)
    # the losses of the two micro-steps are rank 0's + rank 1's samples: rank 0 logs its own
    assert dp["losses"] == acc["losses"][0::2], (dp["losses"], acc["losses"])


@pytest.mark.timeout(1500)
def test_dp2_llama3_8b_width_warmup_dense_buckets_equal_gradient_accumulation(tmp_path):
    dp, acc = _run_both("warmup", tmp_path)
    assert dp["dense_buckets"] and dp["dense_issued"] == len(dp["dense_buckets"])
    big = max(dp["dense_buckets"])
    assert big >= 128256 * 4096                       # the embedding / LM head went through a bucket
    print(f"\n8B width, 2 layers, world 2: {len(dp['dense_buckets'])} dense buckets "
          f"({min(dp['dense_buckets']) / 1e6:.3f}-{big / 1e6:.1f} M elements); {_bucket_table(dp)}; "
          f"peak {dp['peak_gb']:.1f} GB per rank")
    assert sorted(dp["warm"]) == sorted(acc["warm"]) and acc["warm"]
    for n in acc["warm"]:
        assert dp["warm"][n] == acc["warm"][n], n     # weight, fp32 master, exp_avg, exp_avg_sq
    assert dp["harvest"] == acc["harvest"] and acc["harvest"]
    assert dp["sel_att"] == acc["sel_att"] and dp["sel_mlp"] == acc["sel_mlp"]
    _assert_smt_state_equal(dp, acc)

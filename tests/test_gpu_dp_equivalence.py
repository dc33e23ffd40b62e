"""Data-parallel equivalence of the real engine.

Two ranks (gloo, both on cuda:0, child processes) each run micro-batch 2 through one full fine-tuning
warm-up step (bucketed dense all-reduce), the harvest, the rank-0 selection broadcast and one SMT step
(bucketed tile all-reduce overlapped with backward, clip, fused AdamW). That must equal, BIT FOR BIT,
one rank running the same two micro-batches as gradient-accumulation micro-steps: the exchange sums
the two ranks' fp32 (tiles) / bf16 (dense) gradients exactly as accumulation adds them (the 1/2 of the
average and of the accumulation are exact power-of-two scalings). Against one rank on the
concatenated batch of 4 (different GEMM shapes, so a few bf16 roundings differ) the state agrees to
fp32-level tolerance. The reference's DP averaging is implicit in DeepSpeed's backward
(fine_tune.py:712).
"""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "dp_equivalence_worker.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(cmd, tmp):
    # ranks share cuda:0: one hardware queue per process (oversubscribed queues stall)
    env = dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_dp2_equals_gradient_accumulation_bit_for_bit(tmp_path):
    outs = {}
    for mode in ("acc", "big", "dp"):
        out = str(tmp_path / f"{mode}.pt")
        if mode == "dp":
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--mode", "dp", "--out", out]
        else:
            cmd = [sys.executable, WORKER, "--mode", mode, "--out", out]
        _run(cmd, tmp_path)
        outs[mode] = torch.load(out, weights_only=True)
    dp, acc, big = outs["dp"], outs["acc"], outs["big"]
    assert dp["buckets"] > 1                                   # the tile exchange really was bucketed
    for n in acc["warm"]:
        assert torch.equal(dp["warm"][n], acc["warm"][n]), n   # warm-up: dense bucketed all-reduce
    assert dp["sel_mlp"] == acc["sel_mlp"] and dp["sel_att"] == acc["sel_att"]
    for k in ("master", "exp_avg", "exp_avg_sq"):
        assert torch.equal(dp[k], acc[k]), k
    for n in acc["W"]:
        assert torch.equal(dp["W"][n], acc["W"][n]), n
    # vs the concatenated batch (other GEMM shapes: bf16 noise in the gradients). The bound, derived:
    # * AdamW's first step (bias-corrected m = g, v = g^2, weight decay 0) moves each fp32 master by
    #   lr * g / (|g| + eps), of magnitude < lr whatever the clip coefficient; the two runs' gradients
    #   differ by rounding, so their masters m1, m2 differ by < 2 lr (a flipped sign of g), else < lr;
    # * each run then stores bf16(m): round to nearest with 8 significant bits, an error of at most
    #   half a unit, 2^-8 |m| (m in [2^e, 2^(e+1)): spacing 2^(e-7)); the two runs round independently,
    #   and |m| <= |bf16(m)| / (1 - 2^-8);
    # so |d - w| <= 2 lr + 2^-8 (|m1| + |m2|) <= 2 lr + 2^-7 max(|d|, |w|) / (1 - 2^-8), plus the fp32
    # rounding of w0 - update (half an fp32 unit of |w| <= 1: 6e-8)
    lr = 1e-3
    for n in big["warm"]:
        d, w = dp["warm"][n].float(), big["warm"][n].float()
        bound = 2 * lr + torch.maximum(d.abs(), w.abs()) * (2.0 ** -7 / (1 - 2.0 ** -8)) + 6e-8
        excess = (d - w).abs() - bound
        assert excess.max().item() <= 0, (n, (d - w).abs().max().item())
    if dp["sel_mlp"] == big["sel_mlp"] and dp["sel_att"] == big["sel_att"]:
        rel = ((dp["exp_avg"] - big["exp_avg"]).norm() / big["exp_avg"].norm()).item()
        assert rel < 5e-2, rel
        assert (dp["master"] - big["master"]).abs().max().item() <= 4.2e-3    # 2 AdamW steps of lr


def test_dp2_equals_gradient_accumulation_fp8_mx(tmp_path):
    """The fp8 path (config 5): per-token e4m3 rows and MX groups of 32 tokens never straddle two
    micro-batches, so 2 ranks equal 2 accumulation micro-steps bit for bit here too."""
    outs = {}
    for mode in ("acc", "dp"):
        out = str(tmp_path / f"{mode}.pt")
        if mode == "dp":
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--mode", "dp", "--fp8",
                   "--out", out]
        else:
            cmd = [sys.executable, WORKER, "--mode", mode, "--fp8", "--out", out]
        _run(cmd, tmp_path)
        outs[mode] = torch.load(out, weights_only=True)
    dp, acc = outs["dp"], outs["acc"]
    assert dp["sel_mlp"] == acc["sel_mlp"] and dp["sel_att"] == acc["sel_att"]
    for k in ("master", "exp_avg", "exp_avg_sq"):
        assert torch.equal(dp[k], acc[k]), k
    for n in acc["W"]:
        assert torch.equal(dp["W"][n], acc["W"][n]), n


def test_rccl_world1_exchange_bit_identical_to_no_process_group(tmp_path):
    """the engine's DP exchange through RCCL itself. One rank under
    torch.distributed.run with the nccl backend (= RCCL) and ``"dp_exchange": "always"``: the dense
    warm-up gradients and the packed tile gradients go through the bucketed all-reduces (issued from the
    comm stream behind per-bucket events; RCCL's ``Work.wait()`` orders the current stream instead of
    blocking the host as gloo's does). At world 1 the sum is the identity, so the state must equal the
    run without a process group bit for bit (``fine_tune.py:81``, ``smt.py:20``: the reference's NCCL)."""
    outs = {}
    for mode in ("plain", "rccl"):
        out = str(tmp_path / f"{mode}.pt")
        if mode == "rccl":
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--mode", "big",
                   "--pg", "nccl", "--exchange", "always", "--out", out]
        else:
            cmd = [sys.executable, WORKER, "--mode", "big", "--out", out]
        env = dict(os.environ, PYTHONPATH=ROOT)
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        outs[mode] = torch.load(out, weights_only=True)
    plain, rccl = outs["plain"], outs["rccl"]
    assert rccl["backend"] == "nccl" and rccl["world"] == 1 and plain["backend"] is None
    assert rccl["buckets"] > 1 and rccl["tile_issued"] == rccl["buckets"]     # one SMT step, every bucket
    assert rccl["dense_issued"] > 1 and plain["tile_issued"] == plain["dense_issued"] == 0
    for n in plain["warm"]:
        assert torch.equal(rccl["warm"][n], plain["warm"][n]), n
    assert rccl["sel_mlp"] == plain["sel_mlp"] and rccl["sel_att"] == plain["sel_att"]
    for k in ("master", "exp_avg", "exp_avg_sq"):
        assert torch.equal(rccl[k], plain[k]), k
    for n in plain["W"]:
        assert torch.equal(rccl["W"][n], plain["W"][n]), n


def test_dp2_fp16_matches_gradient_accumulation(tmp_path):
    """The equivalence in the reference's --dtype fp16 (fp16 model, transformers' ops, the dynamic loss
    scale). Not bit for bit: accumulation halves each micro-step's loss BEFORE the fp16 backward
    (the engine's gas scaling, as DeepSpeed's), the exchange averages after it, and fp16 gradients this
    small are subnormal in places, so the two round differently. Asserted: the warm-up's exchanged
    dense gradients (the loss-scaled fp16 gradients the bucketed all-reduce averaged) within 2e-3
    (relative, per parameter) of the accumulated ones; the same loss-scale state and skipped steps (the
    overflow decision is taken on the exchanged gradients, the same on every rank); the same selection.
    After AdamW the states drift apart further: its first steps move every weight by ~lr times the
    gradient's sign, which turns a flipped sign of a near-zero gradient into a 2 lr difference, so the
    warm-up weights are compared elementwise (< 1 % differ, each within 2.5 lr) and the SMT step's tile
    gradient, computed on those weights, within 1e-2."""
    outs = {}
    for mode in ("acc", "dp"):
        out = str(tmp_path / f"{mode}16.pt")
        if mode == "dp":
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), WORKER, "--mode", "dp",
                   "--dtype", "fp16", "--out", out]
        else:
            cmd = [sys.executable, WORKER, "--mode", mode, "--dtype", "fp16", "--out", out]
        _run(cmd, tmp_path)
        outs[mode] = torch.load(out, weights_only=True)
    dp, acc = outs["dp"], outs["acc"]
    assert dp["buckets"] > 1 and dp["loss_scale"] is not None
    assert dp["loss_scale"] == acc["loss_scale"] and dp["skipped"] == acc["skipped"]
    assert sorted(dp["warm_grads"]) == sorted(acc["warm_grads"]) and acc["warm_grads"]
    worst = 0.0
    for n, ga in acc["warm_grads"].items():
        gd = dp["warm_grads"][n]
        worst = max(worst, ((gd - ga).double().norm() / ga.double().norm().clamp_min(1e-30)).item())
    print(f"\nfp16 dp vs accumulation: warm-up dense gradients within {worst:.2e} (relative, worst parameter)")
    assert worst <= 2e-3, worst
    lr = 1e-3
    for n in acc["warm"]:
        a, d = acc["warm"][n].float(), dp["warm"][n].float()
        assert acc["warm"][n].dtype == torch.float16
        assert (a != d).float().mean().item() < 0.01, n
        assert (a - d).abs().max().item() <= 2.5 * lr, n
    assert dp["sel_mlp"] == acc["sel_mlp"] and dp["sel_att"] == acc["sel_att"]
    g_dp, g_acc = dp["grad"].double(), acc["grad"].double()
    rel = ((g_dp - g_acc).norm() / g_acc.norm()).item()
    print(f"fp16 dp vs accumulation: SMT-step tile gradient {rel:.2e} relative")
    assert rel <= 1e-2, rel

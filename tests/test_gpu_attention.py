"""gfx950 causal flash attention (fused_llama.flash_attention, C ABI include/smt_attention.h) vs an
fp32 reference computed from the same bf16 inputs.

Tolerance (relative Frobenius error vs the fp32 reference): output and each gradient
<= max(8e-3, 1.5 x the error of torch's own bf16 sdpa on the same inputs); lse within 2e-3 abs
(log2 units). Attention is not on the SMT hot path: it is the model's, and its numerics
are held to torch's bf16 sdpa, not to a reference restatement.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from sparse_matrix_tuning_amd.fused_llama import FlashAttnFn, flash_attention

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _ref(q, k, v, g, scale):
    G = q.shape[1] // k.shape[1]
    qf = q.detach().float().requires_grad_(True)
    kf = k.detach().float().requires_grad_(True)
    vf = v.detach().float().requires_grad_(True)
    o = F.scaled_dot_product_attention(qf, kf.repeat_interleave(G, 1), vf.repeat_interleave(G, 1),
                                       is_causal=True, scale=scale)
    o.transpose(1, 2).backward(g.float())
    s = (qf.detach() @ kf.detach().repeat_interleave(G, 1).transpose(-1, -2)) * scale
    S = q.shape[2]
    s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=q.device), 1), float("-inf"))
    lse2 = torch.logsumexp(s, dim=-1) / math.log(2.0)
    return o.transpose(1, 2).detach(), qf.grad, kf.grad, vf.grad, lse2


def _sdpa_bf16(q, k, v, g):
    qs, ks, vs = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    o = F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True).transpose(1, 2)
    o.backward(g)
    return o.detach(), qs.grad, ks.grad, vs.grad


@pytest.mark.parametrize("B,Hq,Hkv,S,layout", [
    (2, 8, 2, 256, "hf"), (1, 4, 4, 200, "hf"), (1, 8, 1, 384, "contig"), (2, 4, 2, 1024, "hf"), (1, 2, 2, 4, "hf"),
    (1, 40, 40, 512, "hf")])                                   # LLaMA-2-13B heads (config 4)
def test_flash_attention_matches_fp32_reference(B, Hq, Hkv, S, layout):
    torch.manual_seed(S + Hq)
    D = 128
    if layout == "hf":      # [B, S, H, D] storage viewed as [B, H, S, D], as transformers hands them over
        mk = lambda H: torch.randn(B, S, H, D, device=DEV).bfloat16().transpose(1, 2).requires_grad_(True)
    else:
        mk = lambda H: torch.randn(B, H, S, D, device=DEV).bfloat16().requires_grad_(True)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    g = torch.randn(B, S, Hq, D, device=DEV).bfloat16()
    scale = D ** -0.5
    o = flash_attention(q, k, v)
    assert o.shape == (B, S, Hq, D) and o.dtype == torch.bfloat16
    lse = o.grad_fn.saved_tensors[4].clone()          # log2 units of the scaled scores
    o.backward(g)
    ro, rdq, rdk, rdv, rlse = _ref(q, k, v, g, scale)
    so, sdq, sdk, sdv = _sdpa_bf16(q, k, v, g)
    for name, mine, sdpa, ref in (("o", o, so, ro), ("dq", q.grad, sdq, rdq), ("dk", k.grad, sdk, rdk),
                                  ("dv", v.grad, sdv, rdv)):
        e, es = _rel(mine, ref), _rel(sdpa, ref)
        assert e <= max(8e-3, 1.5 * es), (name, e, es)
    assert q.grad.stride() == q.stride() and k.grad.stride() == k.stride()
    assert (lse - rlse).abs().max().item() < 2e-3


def test_flash_attention_rejects_unsupported():
    q = torch.zeros(1, 2, 64, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        FlashAttnFn.apply(q, q, q, 0.125)
    q = torch.zeros(1, 2, 66, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        flash_attention(q, q, q)
    with pytest.raises(RuntimeError):
        flash_attention(q.float(), q.float(), q.float())

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

from sparse_matrix_tuning_amd.fused_llama import FlashAttnFn, KeyMask, flash_attention, smt_flash_mask

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


def test_flash_attention_score_far_above_the_first_tiles():
    """A late key whose score beats every earlier one by ~95 in log2 units: the forward's deferred
    running max must move (a rescale of O and l). Output, gradients and lse as the main test."""
    torch.manual_seed(11)
    B, Hq, Hkv, S, D = 1, 4, 2, 512, 128
    mk = lambda H: torch.randn(B, S, H, D, device=DEV).bfloat16().transpose(1, 2)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    q = (q.float() * 0.25 + 0.5).bfloat16()                    # a common positive direction
    k = k.clone()
    k[:, :, 400] = 12.0                                         # q.k ~ 768 -> ~68 natural, ~98 log2 units
    q, k, v = (t.detach().requires_grad_(True) for t in (q, k, v))
    g = torch.randn(B, S, Hq, D, device=DEV).bfloat16()
    o = flash_attention(q, k, v)
    lse = o.grad_fn.saved_tensors[4].clone()
    o.backward(g)
    ro, rdq, rdk, rdv, rlse = _ref(q, k, v, g, D ** -0.5)
    so, sdq, sdk, sdv = _sdpa_bf16(q, k, v, g)
    assert torch.isfinite(o).all() and torch.isfinite(lse).all()
    for name, mine, sdpa, ref in (("o", o, so, ro), ("dq", q.grad, sdq, rdq), ("dk", k.grad, sdk, rdk),
                                  ("dv", v.grad, sdv, rdv)):
        e, es = _rel(mine, ref), _rel(sdpa, ref)
        assert e <= max(8e-3, 1.5 * es), (name, e, es)
    assert (lse - rlse).abs().max().item() < 2e-3 * max(1.0, rlse.abs().max().item() / 64)


def test_flash_attention_rejects_unsupported():
    q = torch.zeros(1, 2, 64, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        FlashAttnFn.apply(q, q, q, 0.125)
    q = torch.zeros(1, 2, 66, 128, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(NotImplementedError):
        flash_attention(q, q, q)
    with pytest.raises(RuntimeError):
        flash_attention(q.float(), q.float(), q.float())


def _ref_masked(q, k, v, g, scale, keep):
    """fp32 reference with a key mask ``keep`` [B, S] (bool) AND causal; a row with no visible key
    has zero output and zero gradients (the kernels' safe-softmax convention)."""
    G = q.shape[1] // k.shape[1]
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    S = q.shape[2]
    causal = torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
    allowed = causal[None, None] & keep[:, None, None, :]
    s = (qf @ kf.repeat_interleave(G, 1).transpose(-1, -2)) * scale
    s = s.masked_fill(~allowed, float("-inf"))
    any_key = allowed.any(-1, keepdim=True)
    p = torch.softmax(s.masked_fill(~any_key, 0.0), -1) * any_key
    o = p @ vf.repeat_interleave(G, 1)
    o.transpose(1, 2).backward(g.float())
    lse2 = torch.logsumexp(s, dim=-1) / math.log(2.0)
    return o.transpose(1, 2).detach(), qf.grad, kf.grad, vf.grad, lse2, any_key.squeeze(-1)


@pytest.mark.parametrize("B,Hq,Hkv,S", [(3, 8, 2, 256), (2, 4, 4, 200), (2, 32, 8, 1024)])
def test_flash_attention_key_mask_matches_fp32_reference(B, Hq, Hkv, S):
    """Padded batches: right padding of mixed lengths plus pad-id holes inside a
    sequence (LLaMA-3's pad id 0 is an ordinary token, deepspeed_helpers.py:600-602, and the collator's
    mask is input_ids != pad, helper.py:194-204), including a row whose first key is masked (its first
    queries see no key at all)."""
    torch.manual_seed(S + B)
    D = 128
    mk = lambda H: torch.randn(B, S, H, D, device=DEV).bfloat16().transpose(1, 2).requires_grad_(True)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    g = torch.randn(B, S, Hq, D, device=DEV).bfloat16()
    keep = torch.ones(B, S, dtype=torch.bool, device=DEV)
    keep[0, S - S // 3:] = False                       # right padding
    keep[1, S // 2 + 7:] = False
    keep[1, 5] = keep[1, 64] = keep[1, 100] = False     # holes (pad id inside the sequence)
    if B > 2:
        keep[2, 0:3] = False                            # queries 0-2 see no key
    km = smt_flash_mask(B, S, S, attention_mask=keep.long())
    assert isinstance(km, KeyMask)
    o = flash_attention(q, k, v, key_mask=km)
    lse = o.grad_fn.saved_tensors[4].clone()
    o.backward(g)
    ro, rdq, rdk, rdv, rlse, visible = _ref_masked(q, k, v, g, D ** -0.5, keep)
    for name, mine, ref in (("o", o, ro), ("dq", q.grad, rdq), ("dk", k.grad, rdk), ("dv", v.grad, rdv)):
        e = _rel(mine, ref)
        assert e <= 8e-3, (name, e)
        assert torch.isfinite(mine.float()).all(), name
    vis = visible.expand_as(rlse)
    assert (lse[vis] - rlse[vis]).abs().max().item() < 2e-3
    assert torch.isinf(lse[~vis]).all() and (lse[~vis] > 0).all()
    # masked keys get exactly zero dK / dV
    dead = ~keep[:, None, :, None].expand(B, Hkv, S, D)
    assert (k.grad.float()[dead] == 0).all() and (v.grad.float()[dead] == 0).all()
    # an all-valid mask is no mask
    assert smt_flash_mask(B, S, S, attention_mask=torch.ones(B, S, device=DEV)) is None

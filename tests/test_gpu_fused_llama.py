"""Fused LLaMA elementwise kernels vs the eager transformers op chains they replace."""
import pytest
import torch

from sparse_matrix_tuning_amd import fused_llama as fl

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _ulp_close(a, b, max_ulp_frac=1e-3):
    """bf16 tensors equal except for a small fraction differing by one rounding step."""
    a, b = a.float(), b.float()
    diff = (a - b).abs()
    tol = b.abs() * 2 ** -7 + 1e-30            # one bf16 ulp (8 significant bits) relative
    bad = (diff > tol).float().mean().item()
    return bad <= max_ulp_frac, bad


def test_rmsnorm_forward_backward_vs_eager():
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    torch.manual_seed(0)
    H = 4096
    norm = LlamaRMSNorm(H, eps=1e-5).to(DEV).bfloat16()
    with torch.no_grad():
        norm.weight.copy_(torch.randn(H) * 0.2 + 1.0)
    x = (torch.randn(3, 257, H, device=DEV) * 3).bfloat16()
    dy = torch.randn(3, 257, H, device=DEV).bfloat16()
    xe = x.clone().requires_grad_(True)
    ye = norm(xe)
    ye.backward(dy)
    dw_e = norm.weight.grad.clone()
    norm.weight.grad = None
    xf = x.clone().requires_grad_(True)
    yf = fl.FusedRMSNormFn.apply(xf, norm.weight, norm.variance_epsilon)
    yf.backward(dy)
    ok, bad = _ulp_close(yf, ye)
    assert ok, bad
    rel = ((xf.grad.float() - xe.grad.float()).norm() / xe.grad.float().norm()).item()
    assert rel < 5e-3, rel
    relw = ((norm.weight.grad.float() - dw_e.float()).norm() / dw_e.float().norm()).item()
    assert relw < 5e-3, relw


def test_rmsnorm_without_weight_grad_small_hidden():
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    norm = LlamaRMSNorm(512, eps=1e-6).to(DEV).bfloat16()
    norm.weight.requires_grad_(False)
    x = torch.randn(64, 512, device=DEV).bfloat16().requires_grad_(True)
    y = fl.FusedRMSNormFn.apply(x, norm.weight, norm.variance_epsilon)
    y.sum().backward()
    x2 = x.detach().clone().requires_grad_(True)
    norm(x2).sum().backward()
    assert ((x.grad.float() - x2.grad.float()).norm() / x2.grad.float().norm()).item() < 5e-3


def _hf_qk(B=2, S=96, Hq=8, Hk=2, D=128):
    # q/k as LlamaAttention builds them: proj(...).view(B, S, H, D).transpose(1, 2)
    q = torch.randn(B, S, Hq * D, device=DEV).bfloat16().view(B, S, Hq, D).transpose(1, 2)
    k = torch.randn(B, S, Hk * D, device=DEV).bfloat16().view(B, S, Hk, D).transpose(1, 2)
    pos = torch.arange(S, device=DEV, dtype=torch.float32)
    inv = 1.0 / (500000.0 ** (torch.arange(0, D, 2, device=DEV, dtype=torch.float32) / D))
    freqs = torch.outer(pos, inv)
    emb = torch.cat((freqs, freqs), dim=-1)
    cos = emb.cos()[None].expand(B, -1, -1).bfloat16().contiguous()
    sin = emb.sin()[None].expand(B, -1, -1).bfloat16().contiguous()
    return q, k, cos, sin


@pytest.mark.parametrize("Hq,Hk", [(8, 2), (32, 8)])
def test_rope_bit_exact_vs_eager_forward_and_backward(Hq, Hk):
    """(32, 8): LLaMA-3-8B's heads, the head-grouped kernel (cos / sin once per 8 heads)."""
    torch.manual_seed(1)
    q, k, cos, sin = _hf_qk(Hq=Hq, Hk=Hk)
    qe, ke = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    oq_e, ok_e = fl.eager_apply_rotary_pos_emb(qe, ke, cos, sin)
    qf, kf = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    oq_f, ok_f = fl.fused_apply_rotary_pos_emb(qf, kf, cos, sin)
    assert torch.equal(oq_f, oq_e) and torch.equal(ok_f, ok_e)
    gq, gk = torch.randn_like(oq_e), torch.randn_like(ok_e)
    (oq_e.float() * gq.float()).sum().add((ok_e.float() * gk.float()).sum()).backward()
    (oq_f.float() * gq.float()).sum().add((ok_f.float() * gk.float()).sum()).backward()
    assert torch.equal(qf.grad, qe.grad) and torch.equal(kf.grad, ke.grad)


@pytest.mark.parametrize("Hq,Hk", [(8, 2), (32, 8)])
def test_rope_shared_cos_sin_zero_batch_stride(Hq, Hk):
    """HF hands one [1, S, D] cos / sin for the whole batch: the fused RoPE reads it with a zero
    batch stride (fused_llama._rope_launch) instead of B materialised copies -- bit-identical to the
    copies, forward and backward, for B = 4."""
    torch.manual_seed(3)
    B = 4
    q, k, cos, sin = _hf_qk(B=B, Hq=Hq, Hk=Hk)
    cos1, sin1 = cos[:1].clone(), sin[:1].clone()           # [1, S, D], as LlamaRotaryEmbedding returns
    outs = []
    for c, s in ((cos, sin), (cos1, sin1)):
        qf, kf = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
        oq, ok = fl.fused_apply_rotary_pos_emb(qf, kf, c, s)
        gq = torch.arange(oq.numel(), device=DEV).remainder(97).view_as(oq).bfloat16() / 97
        gk = torch.arange(ok.numel(), device=DEV).remainder(89).view_as(ok).bfloat16() / 89
        (oq.float() * gq.float()).sum().add((ok.float() * gk.float()).sum()).backward()
        outs.append((oq, ok, qf.grad, kf.grad))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    # and both equal transformers' own rotary on the [1, S, D] embeddings
    qe, ke = q.clone(), k.clone()
    oq_e, ok_e = fl.eager_apply_rotary_pos_emb(qe, ke, cos1, sin1)
    assert torch.equal(outs[1][0], oq_e) and torch.equal(outs[1][1], ok_e)


def test_swiglu_vs_eager():
    torch.manual_seed(2)
    g = (torch.randn(4, 100, 1536, device=DEV) * 3).bfloat16()
    u = torch.randn(4, 100, 1536, device=DEV).bfloat16()
    dh = torch.randn(4, 100, 1536, device=DEV).bfloat16()
    ge, ue = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    he = torch.nn.functional.silu(ge) * ue
    he.backward(dh)
    gf, uf = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    hf = fl.FusedSwiGLUFn.apply(gf, uf)
    hf.backward(dh)
    for a, b in ((hf, he), (gf.grad, ge.grad), (uf.grad, ue.grad)):
        ok, bad = _ulp_close(a, b)
        assert ok, bad


def test_patched_mini_llama_matches_eager():
    import bench
    torch.manual_seed(3)
    model = bench.build_model("mini", DEV)
    ids = torch.randint(0, 4096, (2, 256), device=DEV)
    out_e = model(input_ids=ids, labels=ids, use_cache=False)
    out_e.loss.backward()
    ge = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    model.zero_grad(set_to_none=True)
    try:
        counts = fl.patch_llama(model)
        assert counts["rmsnorm"] == 9 and counts["mlp"] == 4 and counts["attention"] == 4 and counts["decoder"] == 4
        assert model.config._attn_implementation == "smt_flash"
        out_f = model(input_ids=ids, labels=ids, use_cache=False)
        out_f.loss.backward()
    finally:
        fl.unpatch_llama(model)
    assert model.config._attn_implementation == "sdpa"
    rel = abs(out_f.loss.item() - out_e.loss.item()) / abs(out_e.loss.item())
    assert rel < 1e-3, (out_f.loss.item(), out_e.loss.item())
    worst = max(((p.grad.float() - ge[n].float()).norm() / ge[n].float().norm()).item()
                for n, p in model.named_parameters() if p.grad is not None)
    assert worst < 5e-2, worst


def test_layer_tail_fusion_is_bit_identical():
    """The MLP residual add fused with the next layer's input RMSNorm (fused_decoder_layer_forward's
    tail): loss, every parameter gradient (full fine-tuning: the norm weights too) and the hidden
    states bit-identical to the separate add + norm; with per-layer recompute on every other layer
    the tail is not used across a recomputed layer and the results are still identical."""
    import bench

    def run(tail, ckpt_every_other=False):
        torch.manual_seed(3)
        model = bench.build_model("mini", DEV)
        ids = torch.randint(0, 4096, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
        old = fl._LAYER_TAIL
        fl._LAYER_TAIL = tail
        try:
            fl.patch_llama(model)
            if ckpt_every_other:
                model.gradient_checkpointing_enable(gradient_checkpointing_kwargs={"use_reentrant": False})
                for i, layer in enumerate(model.model.layers):
                    layer.gradient_checkpointing = i % 2 == 1
            out = model(input_ids=ids, labels=ids, use_cache=False, output_hidden_states=True)
            out.loss.backward()
        finally:
            fl._LAYER_TAIL = old
            fl.unpatch_llama(model)
        return (out.loss.detach(), [h.detach() for h in out.hidden_states],
                {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})

    for ckpt in (False, True):
        l0, h0, g0 = run(False, ckpt)
        l1, h1, g1 = run(True, ckpt)
        assert torch.equal(l0, l1), ckpt
        assert all(torch.equal(a, b) for a, b in zip(h0, h1)), ckpt
        assert sorted(g0) == sorted(g1)
        for n in g0:
            assert torch.equal(g0[n], g1[n]), (ckpt, n)


@pytest.mark.parametrize("H", [4096, 512])
@pytest.mark.parametrize("weight_grad", [False, True])
def test_fused_add_rmsnorm_vs_eager(H, weight_grad):
    """h = x + residual, y = RMSNorm(h); grads of (x, residual, weight) with a residual-path gradient."""
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    torch.manual_seed(H)
    norm = LlamaRMSNorm(H, eps=1e-5).to(DEV).bfloat16()
    with torch.no_grad():
        norm.weight.copy_(torch.randn(H) * 0.2 + 1.0)
    norm.weight.requires_grad_(weight_grad)
    x = (torch.randn(2, 133, H, device=DEV) * 2).bfloat16()
    r = (torch.randn(2, 133, H, device=DEV) * 3).bfloat16()
    dh = torch.randn(2, 133, H, device=DEV).bfloat16()
    dy = torch.randn(2, 133, H, device=DEV).bfloat16()
    xe, re_ = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    he = re_ + xe
    ye = norm(he)
    torch.autograd.backward([he, ye], [dh, dy])
    dw_e = norm.weight.grad.clone() if weight_grad else None
    norm.weight.grad = None
    xf, rf = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    hf, yf = fl.FusedAddRMSNormFn.apply(xf, rf, norm.weight, norm.variance_epsilon)
    torch.autograd.backward([hf, yf], [dh, dy])
    assert torch.equal(hf, he)
    ok, bad = _ulp_close(yf, ye)
    assert ok, bad
    for a, b in ((xf.grad, xe.grad), (rf.grad, re_.grad)):
        rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
        assert rel < 5e-3, rel
    if weight_grad:
        relw = ((norm.weight.grad.float() - dw_e.float()).norm() / dw_e.float().norm()).item()
        assert relw < 5e-3, relw


@pytest.mark.parametrize("H", [512, 4096, 5120])
@pytest.mark.parametrize("rows", [133, 4133])
def test_rmsnorm_bwd_add_dw_equals_separate_passes(H, rows):
    """smt_rmsnorm_bwd_add_dw (the warm-up's norm backward: weight gradient and residual-path add in
    one pass) gives bit for bit the dx of smt_rmsnorm_bwd followed by autograd's bf16 add, and the
    same dw; dw within bf16 rounding of the fp64 sum of the reference chain's per-row terms."""
    torch.manual_seed(rows + H)
    x = (torch.randn(rows, H, device=DEV) * 2).bfloat16()
    w = (torch.randn(H, device=DEV) * 0.2 + 1.0).bfloat16()
    dy = torch.randn(rows, H, device=DEV).bfloat16()
    dres = torch.randn(rows, H, device=DEV).bfloat16()
    rstd = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    dx0, dw0 = fl._rmsnorm_bwd(x, w, rstd, dy, True)
    dx1, dw1 = fl._rmsnorm_bwd(x, w, rstd, dy, True, dres)
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0 + dres)
    assert torch.equal(dw1, dw0)
    terms = (dy.float() * (x.float() * rstd[:, None]).bfloat16().float()).bfloat16().double()
    truth = terms.sum(0)
    rel = ((dw1.double() - truth).norm() / truth.norm()).item()
    assert rel < 4e-3, rel

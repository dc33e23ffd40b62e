"""The fused LLaMA kernels, the flash attention and the fused loss in fp16 (ABI v13).

The reference trains in the model's dtype, ``--dtype bf16 | fp16 | fp32`` (fine_tune.py:955-959,
deepspeed_helpers.py:53-61). Until round 6 the fused ops were bf16-only, so an fp16 model ran
transformers' eager modules. Each kernel is now one template body for both 16-bit formats, rounding
where the eager chain rounds to the model's dtype; these tests hold the fp16 instances to the same
bars as the bf16 ones (tests/test_gpu_fused_llama.py, test_gpu_attention.py,
test_gpu_cross_entropy.py): eager fp16 transformers chains, or an fp32 reference of the attention on
the same fp16 inputs, and the restated reference path (oracle.ref_convert + eager fp16 on the host)
for a mini-LLaMA's loss and tile gradients."""
import math

import pytest
import torch
import torch.nn.functional as F

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd import fused_llama as fl

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
H16 = torch.float16


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _ulp_close(a, b, max_ulp_frac=1e-3):
    """fp16 tensors equal except for a small fraction differing by one rounding step (11 bits)."""
    a, b = a.float(), b.float()
    bad = ((a - b).abs() > b.abs() * 2 ** -10 + 6e-8).float().mean().item()
    return bad <= max_ulp_frac, bad


@pytest.mark.parametrize("H", [4096, 512, 5120])
def test_rmsnorm_fp16_vs_eager(H):
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    torch.manual_seed(H)
    norm = LlamaRMSNorm(H, eps=1e-5).to(DEV).to(H16)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(H) * 0.2 + 1.0)
    x = (torch.randn(3, 257, H, device=DEV) * 3).to(H16)
    dy = torch.randn(3, 257, H, device=DEV).to(H16)
    xe = x.clone().requires_grad_(True)
    ye = norm(xe)
    ye.backward(dy)
    dw_e = norm.weight.grad.clone()
    norm.weight.grad = None
    xf = x.clone().requires_grad_(True)
    yf = fl.FusedRMSNormFn.apply(xf, norm.weight, norm.variance_epsilon)
    yf.backward(dy)
    assert yf.dtype == H16
    ok, bad = _ulp_close(yf, ye)
    assert ok, bad
    assert _rel(xf.grad, xe.grad) < 2e-3
    assert _rel(norm.weight.grad, dw_e) < 2e-3


@pytest.mark.parametrize("weight_grad", [False, True])
def test_fused_add_rmsnorm_fp16_vs_eager(weight_grad):
    from transformers.models.llama.modeling_llama import LlamaRMSNorm
    torch.manual_seed(5)
    H = 4096
    norm = LlamaRMSNorm(H, eps=1e-5).to(DEV).to(H16)
    with torch.no_grad():
        norm.weight.copy_(torch.randn(H) * 0.2 + 1.0)
    norm.weight.requires_grad_(weight_grad)
    x, r = (torch.randn(2, 133, H, device=DEV) * 2).to(H16), (torch.randn(2, 133, H, device=DEV) * 3).to(H16)
    dh, dy = torch.randn(2, 133, H, device=DEV).to(H16), torch.randn(2, 133, H, device=DEV).to(H16)
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
        assert _rel(a, b) < 2e-3
    if weight_grad:
        assert _rel(norm.weight.grad, dw_e) < 2e-3


@pytest.mark.parametrize("Hq,Hk", [(8, 2), (32, 8)])
def test_rope_fp16_bit_exact_vs_eager(Hq, Hk):
    torch.manual_seed(1)
    B, S, D = 2, 96, 128
    q = torch.randn(B, S, Hq * D, device=DEV).to(H16).view(B, S, Hq, D).transpose(1, 2)
    k = torch.randn(B, S, Hk * D, device=DEV).to(H16).view(B, S, Hk, D).transpose(1, 2)
    pos = torch.arange(S, device=DEV, dtype=torch.float32)
    inv = 1.0 / (500000.0 ** (torch.arange(0, D, 2, device=DEV, dtype=torch.float32) / D))
    emb = torch.cat((torch.outer(pos, inv),) * 2, dim=-1)
    cos, sin = emb.cos()[None].to(H16), emb.sin()[None].to(H16)
    qe, ke = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    oq_e, ok_e = fl.eager_apply_rotary_pos_emb(qe, ke, cos, sin)
    qf, kf = q.clone().requires_grad_(True), k.clone().requires_grad_(True)
    oq_f, ok_f = fl.fused_apply_rotary_pos_emb(qf, kf, cos, sin)
    assert oq_f.dtype == H16 and torch.equal(oq_f, oq_e) and torch.equal(ok_f, ok_e)
    gq, gk = torch.randn_like(oq_e), torch.randn_like(ok_e)
    (oq_e.float() * gq.float()).sum().add((ok_e.float() * gk.float()).sum()).backward()
    (oq_f.float() * gq.float()).sum().add((ok_f.float() * gk.float()).sum()).backward()
    assert torch.equal(qf.grad, qe.grad) and torch.equal(kf.grad, ke.grad)


def test_swiglu_fp16_vs_eager():
    torch.manual_seed(2)
    g = (torch.randn(4, 100, 1536, device=DEV) * 3).to(H16)
    u = torch.randn(4, 100, 1536, device=DEV).to(H16)
    dh = torch.randn(4, 100, 1536, device=DEV).to(H16)
    ge, ue = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    he = F.silu(ge) * ue
    he.backward(dh)
    gf, uf = g.clone().requires_grad_(True), u.clone().requires_grad_(True)
    hf = fl.FusedSwiGLUFn.apply(gf, uf)
    hf.backward(dh)
    for a, b in ((hf, he), (gf.grad, ge.grad), (uf.grad, ue.grad)):
        ok, bad = _ulp_close(a, b)
        assert ok, bad


@pytest.mark.parametrize("op", [_hip.RECOMPUTE_RMSNORM, _hip.RECOMPUTE_SWIGLU])
def test_colblock_recompute_fp16_equals_gathered_output(op):
    """The selective policy's rebuilt column blocks in fp16: bit-identical to the producer's output."""
    torch.manual_seed(7)
    T, C = 1000, 2048
    blocks = torch.tensor([1, 4, 7], dtype=torch.int32, device=DEV)
    if op == _hip.RECOMPUTE_RMSNORM:
        x = (torch.randn(T, C, device=DEV) * 2).to(H16).requires_grad_(True)
        w = (torch.randn(C, device=DEV) * 0.2 + 1).to(H16)
        y = fl.FusedRMSNormFn.apply(x, w, 1e-5)
        rstd = y.grad_fn.saved_tensors[2]                 # the norm's own saved rstd
        got = _hip.colblock_recompute(op, x.detach(), blocks, weight=w, rstd=rstd)
    else:
        g = (torch.randn(T, C, device=DEV) * 3).to(H16)
        u = torch.randn(T, C, device=DEV).to(H16)
        y = fl.FusedSwiGLUFn.apply(g, u)
        got = _hip.colblock_recompute(op, g, blocks, b2d=u)
    want = torch.stack([y.reshape(T, C)[:, b * 256:(b + 1) * 256] for b in blocks.tolist()])
    assert got.dtype == H16 and torch.equal(got, want)


def test_cross_entropy_fp16_vs_transformers():
    torch.manual_seed(9)
    N, V = 300, 32008
    logits = (torch.randn(N, V, device=DEV) * 4).to(H16)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    le = logits.clone().requires_grad_(True)
    loss_e = F.cross_entropy(le.float(), labels, ignore_index=-100)
    loss_e.backward()
    lf = logits.clone().requires_grad_(True)
    denom = (labels != -100).sum().to(torch.float32)
    loss_f = fl.FusedCrossEntropyFn.apply(lf, labels, -100, denom)
    loss_f.backward()
    assert abs(loss_f.item() - loss_e.item()) / loss_e.item() < 1e-5
    ok, bad = _ulp_close(lf.grad, le.grad)
    assert lf.grad.dtype == H16 and ok, bad


@pytest.mark.parametrize("B,Hq,Hkv,S", [(2, 8, 2, 256), (1, 4, 4, 200), (2, 32, 8, 512)])
def test_flash_attention_fp16_matches_fp32_reference(B, Hq, Hkv, S):
    """Same bar as the bf16 instance (tests/test_gpu_attention.py): relative error vs an fp32 reference
    on the same fp16 inputs <= max(8e-3, 1.5 x torch's own fp16 sdpa error); lse within 2e-3."""
    torch.manual_seed(S + Hq)
    D = 128
    mk = lambda H: torch.randn(B, S, H, D, device=DEV).to(H16).transpose(1, 2).requires_grad_(True)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    g = torch.randn(B, S, Hq, D, device=DEV).to(H16)
    scale = D ** -0.5
    o = fl.flash_attention(q, k, v)
    assert o.dtype == H16
    lse = o.grad_fn.saved_tensors[4].clone()
    o.backward(g)
    G = Hq // Hkv
    qf, kf, vf = (t.detach().float().requires_grad_(True) for t in (q, k, v))
    ro = F.scaled_dot_product_attention(qf, kf.repeat_interleave(G, 1), vf.repeat_interleave(G, 1), is_causal=True,
                                        scale=scale)
    ro.transpose(1, 2).backward(g.float())
    s = (qf.detach() @ kf.detach().repeat_interleave(G, 1).transpose(-1, -2)) * scale
    s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=DEV), 1), float("-inf"))
    rlse = torch.logsumexp(s, dim=-1) / math.log(2.0)
    qs, ks, vs = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    so = F.scaled_dot_product_attention(qs, ks, vs, is_causal=True, enable_gqa=True).transpose(1, 2)
    so.backward(g)
    for name, mine, sd, rf in (("o", o, so, ro.transpose(1, 2)), ("dq", q.grad, qs.grad, qf.grad),
                               ("dk", k.grad, ks.grad, kf.grad), ("dv", v.grad, vs.grad, vf.grad)):
        e, es = _rel(mine, rf), _rel(sd, rf)
        print(f"{name}: smt_flash fp16 {e:.2e}, sdpa fp16 {es:.2e}")
        assert e <= max(8e-3, 1.5 * es), (name, e, es)
    assert (lse - rlse).abs().max().item() < 2e-3


def test_patched_mini_llama_fp16_matches_eager_and_reference_path():
    """A mini-LLaMA in fp16 with SMT tiles: the fused model (kernels above, smt_flash, the fused LM head
    + loss, the engine's tile wgrad) against transformers' eager fp16 model with the restated reference
    modules on the host (oracle.ref_convert: what fine_tune.py:710-712 computes in --dtype fp16). Loss
    within 1e-3; every module's tile gradient within max(1e-3, 1.1 x the reference path's own error)
    of the fp64 product of the operands the product saw."""
    import bench
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.smt import smt
    torch.manual_seed(3)
    model = bench.build_model("mini", DEV).to(H16)
    host = bench.build_model("mini", torch.device("cpu")).to(H16)
    host.load_state_dict({k: v.cpu() for k, v in model.state_dict().items()})
    host.config._attn_implementation = "eager"
    sel_mlp = {("gate_proj", 1): [(0, 0), (2, 1)], ("down_proj", 2): [(1, 0)]}
    sel_att = {("q_proj", 0): [(0, 1), (1, 0)], ("v_proj", 3): [(0, 0)]}
    ids = torch.randint(0, 4096, (2, 256), generator=torch.Generator().manual_seed(5))
    counts = fl.patch_llama(model)
    try:
        assert counts["attention"] == 4 and counts["lm_head_loss"] == 1
        smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
        smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
        opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 1e-4), lr=1e-4, betas=(0.9, 0.95))
        # DeepSpeed's fp16 config (deepspeed_helpers.py:53-55) with a small initial scale, so that this
        # one step does not overflow and skip
        eng, *_ = initialize(model=model, optimizer=opt,
                             config={"gradient_clipping": 1.0,
                                     "fp16": {"enabled": True, "loss_scale_window": 100, "initial_scale_power": 8}})
        assert eng.transposed_bytes > 0                 # fp16 frozen weights get W^T copies too
        mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}
        seen = {}

        def cap(name):
            def hook(_m, inp, out):
                x = inp[0].detach().clone()
                out.register_hook(lambda g: seen.__setitem__(name, (x, g.detach().clone())))
            return hook
        hs = [m.register_forward_hook(cap(n)) for n, m in mods.items()]
        loss = eng(input_ids=ids.to(DEV), labels=ids.to(DEV), use_cache=False).loss
        eng.backward(loss)
        torch.cuda.synchronize()
        for h in hs:
            h.remove()
        # the captured output gradients and the sinks are both in loss-scaled units; relative errors below
        grads = {n: m.selected_weight._smt_grad_sink.buffer.detach().cpu() for n, m in mods.items()}
    finally:
        fl.unpatch_llama(model)
    smt.freeze_unselected_matrix_layer(host, sel_mlp, sel_att)
    ref.ref_convert(host, sel_mlp, sel_att)
    out_h = host(input_ids=ids, labels=ids, use_cache=False)
    assert abs(loss.item() - out_h.loss.item()) / abs(out_h.loss.item()) <= 1e-3, (loss.item(), out_h.loss.item())
    for n, (x, g) in seen.items():
        tiles = list(mods[n].index_list)
        fp64 = ref.tile_grads_fp64(g.cpu(), x.cpu(), tiles)
        _gi, gw_ref = ref.linearz_backward(g.cpu(), x.cpu(), mods[n].weight.detach().cpu(), tiles)
        e, er = _rel(grads[n], fp64), _rel(gw_ref, fp64)
        print(f"{n}: tile grad vs fp64 {e:.2e} (reference algorithm {er:.2e})")
        assert e <= max(1e-3, 1.1 * er), (n, e, er)

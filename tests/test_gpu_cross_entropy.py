"""Fused causal-LM cross entropy (csrc/llama_kernels.hip smt_ce_fwd / smt_ce_bwd) vs transformers'
ForCausalLMLoss (logits.float() -> F.cross_entropy, ignore_index -100), both on the GPU.

Tolerances: loss within 1e-5 relative (fp32 log-sum-exp, different summation order); dlogits within
one bf16 rounding step for all but 0.1 % of the elements (both round an fp32 gradient to bf16 once; a
different exp / summation order can move a value across a rounding boundary)."""
import pytest
import torch

from sparse_matrix_tuning_amd import fused_llama as fl

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _reference(logits, labels, num_items=None):
    from transformers.loss.loss_utils import ForCausalLMLoss
    x = logits.detach().clone().requires_grad_(True)
    loss = ForCausalLMLoss(x, labels, vocab_size=logits.shape[-1], num_items_in_batch=num_items)
    loss.backward()
    return loss.detach(), x.grad


def _fused(logits, labels, num_items=None):
    x = logits.detach().clone().requires_grad_(True)
    loss = fl.fused_causal_lm_loss(x, labels, vocab_size=logits.shape[-1], num_items_in_batch=num_items)
    loss.backward()
    return loss.detach(), x.grad


def _check(a_loss, a_grad, b_loss, b_grad):
    rel = abs(a_loss.item() - b_loss.item()) / max(abs(b_loss.item()), 1e-30)
    assert rel < 1e-5, (a_loss.item(), b_loss.item())
    assert a_grad.dtype == b_grad.dtype == torch.bfloat16
    diff = (a_grad.float() - b_grad.float()).abs()
    tol = b_grad.float().abs() * 2 ** -7 + 1e-12
    bad = (diff > tol).float().mean().item()
    assert bad < 1e-3, bad
    relg = ((a_grad.float() - b_grad.float()).norm() / b_grad.float().norm()).item()
    assert relg < 4e-3, relg


@pytest.mark.parametrize("B,S,V", [(2, 64, 4096), (3, 37, 50272), (1, 128, 128256)])
def test_cross_entropy_matches_transformers_loss(B, S, V):
    torch.manual_seed(B * 1000 + V)
    logits = (torch.randn(B, S, V, device=DEV) * 4).bfloat16()
    labels = torch.randint(0, V, (B, S), device=DEV)
    _check(*_fused(logits, labels), *_reference(logits, labels))


def test_cross_entropy_ignore_index_and_num_items():
    torch.manual_seed(7)
    B, S, V = 2, 50, 4096
    logits = (torch.randn(B, S, V, device=DEV) * 2).bfloat16()
    labels = torch.randint(0, V, (B, S), device=DEV)
    labels[0, :13] = -100
    labels[1, 40:] = -100
    _check(*_fused(logits, labels), *_reference(logits, labels))
    n = torch.tensor(77, device=DEV)
    _check(*_fused(logits, labels, n), *_reference(logits, labels, n))


def test_cross_entropy_extreme_logits_stable():
    """Large-magnitude logits (the max-subtraction path), a row spanning [-100, 100]."""
    B, S, V = 1, 8, 8192
    logits = torch.full((B, S, V), -30.0, device=DEV)
    logits[0, :, 5] = 80.0
    logits[0, 3, :] = torch.linspace(-100, 100, V, device=DEV)
    logits = logits.bfloat16()
    labels = torch.full((B, S), 5, device=DEV)
    f_loss, f_grad = _fused(logits, labels)
    r_loss, r_grad = _reference(logits, labels)
    assert torch.isfinite(f_loss) and torch.isfinite(f_grad.float()).all()
    assert abs(f_loss.item() - r_loss.item()) <= 1e-5 * max(1.0, abs(r_loss.item()))
    assert ((f_grad.float() - r_grad.float()).abs() <= r_grad.float().abs() * 2 ** -7 + 1e-6).all()


def test_cross_entropy_out_of_range_label_is_nan_not_silent():
    logits = torch.randn(1, 4, 1024, device=DEV).bfloat16()
    labels = torch.tensor([[1, 2, 5000, 3]], device=DEV)          # shifted: row 1 predicts 5000
    loss = fl.fused_causal_lm_loss(logits, labels, vocab_size=1024)
    assert torch.isnan(loss)


def test_cross_entropy_rejects_fp32_logits():
    with pytest.raises(RuntimeError):
        fl.fused_causal_lm_loss(torch.randn(1, 4, 1024, device=DEV), torch.zeros(1, 4, dtype=torch.long, device=DEV),
                                vocab_size=1024)


# ------------------------------------------------------------------------------------------------
# LM head + loss, chunk by chunk (fl.FusedLMHeadLossFn): against the unfused pair it replaces,
# lm_head (F.linear; data gradient on the transposed copy, as engine.FrozenLinearFn) followed by
# fused_causal_lm_loss. Same kernels and scale per row, so the loss and dh agree to the GEMM
# kernel choice for the chunk shape (printed: bit-identical or not); asserted: loss within 1e-6,
# dh within one bf16 rounding step for all but 0.1 % of the elements.
# ------------------------------------------------------------------------------------------------
class _Head:
    def __init__(self, w, wt):
        self.weight = w
        if wt is not None:
            w._smt_weight_t = wt


def _head_operands(B, S, H, V, seed, transposed=True):
    g = torch.Generator(device=DEV).manual_seed(seed)
    h = (torch.randn(B, S, H, device=DEV, generator=g)).bfloat16()
    w = (torch.randn(V, H, device=DEV, generator=g) * H ** -0.5 * 2).bfloat16()
    wt = w.t().contiguous() if transposed else None
    labels = torch.randint(0, V, (B, S), device=DEV, generator=g)
    return h, w, wt, labels


def _unfused_head(h, w, wt, labels, num_items=None, dloss=1.0):
    from sparse_matrix_tuning_amd.engine import FrozenLinearFn
    x = h.detach().clone().requires_grad_(True)
    logits = FrozenLinearFn.apply(x, w, wt, None) if wt is not None else torch.nn.functional.linear(x, w)
    loss = fl.fused_causal_lm_loss(logits, labels, vocab_size=w.shape[0], num_items_in_batch=num_items)
    (loss * dloss).backward()
    return loss.detach(), x.grad


def _fused_head(h, w, wt, labels, chunk, num_items=None, dloss=1.0):
    x = h.detach().clone().requires_grad_(True)
    w2 = w.detach().clone()              # a fresh tensor to carry this run's transposed copy
    loss = fl.fused_lm_head_loss(x, _Head(w2, wt), labels, num_items_in_batch=num_items, chunk_rows=chunk)
    (loss * dloss).backward()
    return loss.detach(), x.grad


def _close_bf16(a, b):
    diff = (a.float() - b.float()).abs()
    bad = (diff > b.float().abs() * 2 ** -7 + 1e-12).float().mean().item()
    rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
    return bad < 1e-3 and rel < 4e-3, (bad, rel)


@pytest.mark.parametrize("B,S,H,V,chunk,transposed", [
    (2, 100, 256, 4096, 64, True),          # 200 rows: chunks of 64, 64, 64, 8
    (2, 100, 256, 4096, 64, False),         # no transposed copy: dh = dlogits @ W (NN)
    (1, 2048, 4096, 128256, 4096, True),    # the 8B head, one sample; one chunk
    (1, 2048, 4096, 128256, 512, True),     # the 8B head, 4 chunks
])
def test_lm_head_loss_matches_unfused(B, S, H, V, chunk, transposed):
    h, w, wt, labels = _head_operands(B, S, H, V, seed=B * S + V + chunk, transposed=transposed)
    labels[0, : S // 7] = -100
    lu, gu = _unfused_head(h, w, wt, labels)
    lf, gf = _fused_head(h, w, wt, labels, chunk)
    print(f"loss bit-identical {torch.equal(lu, lf)}, dh bit-identical {torch.equal(gu, gf)}")
    assert abs(lf.item() - lu.item()) <= 1e-6 * abs(lu.item()), (lf.item(), lu.item())
    ok, why = _close_bf16(gf, gu)
    assert ok, why


@pytest.mark.parametrize("B,S,H,V,chunk", [(2, 100, 256, 4096, 64), (1, 2048, 4096, 128256, 512)])
def test_lm_head_loss_trainable_head_matches_unfused(B, S, H, V, chunk, monkeypatch):
    """The warm-up's trainable head: dW from an fp32 accumulator over the chunks (one bf16 rounding)
    against autograd's one GEMM over all rows; dh and the loss as for a frozen head. (The chunk floor
    for a trainable head is lifted so that several chunks accumulate.)"""
    monkeypatch.setattr(fl, "LM_HEAD_DW_CHUNK_ROWS", 0)
    h, w, _wt, labels = _head_operands(B, S, H, V, seed=B + S + chunk, transposed=False)
    labels[0, S // 3: S // 3 + 9] = -100
    x0, w0 = h.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    lu = fl.fused_causal_lm_loss(torch.nn.functional.linear(x0, w0), labels, vocab_size=V)
    lu.backward()
    x1, w1 = h.detach().clone().requires_grad_(True), w.detach().clone().requires_grad_(True)
    lf = fl.fused_lm_head_loss(x1, _Head(w1, None), labels, chunk_rows=chunk)
    lf.backward()
    print(f"loss bit-identical {torch.equal(lu, lf)}, dh bit-identical {torch.equal(x0.grad, x1.grad)}, "
          f"dW bit-identical {torch.equal(w0.grad, w1.grad)}")
    assert abs(lf.item() - lu.item()) <= 1e-6 * abs(lu.item())
    for a, b in ((x1.grad, x0.grad), (w1.grad, w0.grad)):
        ok, why = _close_bf16(a, b)
        assert ok, why


def test_lm_head_loss_upstream_gradient_and_num_items():
    """dloss = 0.5 (exact either way: a power of two), 1/3 (fused: applied to the bf16 dh, one more
    rounding; bounded against the fp64 truth at 1.5x the unfused error), and num_items_in_batch."""
    B, S, H, V = 2, 64, 512, 8192
    h, w, wt, labels = _head_operands(B, S, H, V, seed=11)
    n = torch.tensor(100, device=DEV)
    lu, gu = _unfused_head(h, w, wt, labels, n, dloss=0.5)
    lf, gf = _fused_head(h, w, wt, labels, 48, n, dloss=0.5)
    assert abs(lf.item() - lu.item()) <= 1e-6 * abs(lu.item())
    ok, why = _close_bf16(gf, gu)
    assert ok, why
    # fp64 truth of d(loss / 3)/dh
    x = h.double().reshape(-1, H).requires_grad_(True)
    shift = torch.nn.functional.pad(labels, (0, 1), value=-100)[..., 1:].reshape(-1)
    logit = x @ w.double().t()
    truth_loss = torch.nn.functional.cross_entropy(logit, shift, ignore_index=-100, reduction="sum") / 100.0
    (truth_loss / 3).backward()
    truth = x.grad.view(B, S, H)
    _lu, gu3 = _unfused_head(h, w, wt, labels, n, dloss=1 / 3)
    _lf, gf3 = _fused_head(h, w, wt, labels, 48, n, dloss=1 / 3)
    eu = ((gu3.double() - truth).norm() / truth.norm()).item()
    ef = ((gf3.double() - truth).norm() / truth.norm()).item()
    print(f"dloss 1/3: unfused {eu:.3e}, fused {ef:.3e} from fp64")
    assert ef <= max(1.5 * eu, 4e-3), (ef, eu)


def test_lm_head_loss_never_holds_the_full_logits():
    """Peak memory of forward + backward above the operands: one chunk of logits and dh, not the
    [T, V] logits and dlogits of the unfused pair."""
    B, S, H, V, chunk = 4, 2048, 1024, 32768, 1024
    h, w, wt, labels = _head_operands(B, S, H, V, seed=5)
    full = B * S * V * 2

    def peak(fn):
        import gc
        gc.collect()                # garbage of earlier tests freed mid-measurement would lower the peak
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        out = fn()
        torch.cuda.synchronize()
        p = torch.cuda.max_memory_allocated() - base
        del out
        return p

    pu = peak(lambda: _unfused_head(h, w, wt, labels))
    pf = peak(lambda: _fused_head(h, w, wt, labels, chunk))
    print(f"peak above operands: unfused {pu / 2 ** 20:.0f} MiB, fused {pf / 2 ** 20:.0f} MiB")
    assert pu >= 2 * full
    assert pf <= chunk * V * 2 + 3 * B * S * H * 2 + (1 << 22) + w.numel() * 2, pf


def test_lm_head_loss_without_grad_is_the_loss_only():
    B, S, H, V = 2, 64, 256, 4096
    h, w, wt, labels = _head_operands(B, S, H, V, seed=3)
    lu, _ = _unfused_head(h, w, wt, labels)
    with torch.no_grad():
        lf = fl.fused_lm_head_loss(h, _Head(w.clone(), wt), labels, chunk_rows=40)
    assert not lf.requires_grad
    assert abs(lf.item() - lu.item()) <= 1e-6 * abs(lu.item())


def test_lm_head_loss_trainable_head_under_no_grad_skips_the_gradients():
    """``needs_input_grad`` reflects requires_grad even under ``torch.no_grad()``. With a
    trainable head (the warm-up) an evaluation forward with labels must still compute the loss only:
    no dlogits, no dW GEMMs, no fp32 ``[V, H]`` accumulator (here 131 MB)."""
    B, S, H, V = 2, 64, 1024, 32000
    h, w, wt, labels = _head_operands(B, S, H, V, seed=4, transposed=False)
    lu, _ = _unfused_head(h, w, wt, labels)
    head = torch.nn.Linear(H, V, bias=False, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        head.weight.copy_(w)
    assert head.weight.requires_grad
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(DEV)
    torch.cuda.reset_peak_memory_stats(DEV)
    with torch.no_grad():
        lf = fl.fused_lm_head_loss(h.detach(), head, labels)
    torch.cuda.synchronize()
    extra = torch.cuda.max_memory_allocated(DEV) - base
    assert not lf.requires_grad and abs(lf.item() - lu.item()) <= 1e-6 * abs(lu.item())
    assert extra < V * H * 4 // 4, extra                     # far below the fp32 accumulator


def test_patched_model_fuses_the_head():
    """patch_llama's forward: a frozen head (SMT phase) and a trainable one (warm-up) give the fused
    loss (logits None) with the unfused loss and the same gradients; labels None runs transformers'
    forward."""
    import bench
    torch.manual_seed(3)
    model = bench.build_model("mini", DEV)
    model.lm_head.weight.requires_grad_(False)
    ids = torch.randint(0, 4096, (2, 256), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))

    def run(fused):
        model.zero_grad(set_to_none=True)
        counts = fl.patch_llama(model, lm_head_loss=fused)
        try:
            out = model(input_ids=ids, labels=ids, use_cache=False)
            out.loss.backward()
            no_labels = model(input_ids=ids[:, :16], use_cache=False)
        finally:
            fl.unpatch_llama(model)
        assert "forward" not in model.__dict__
        return counts, out, no_labels, {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}

    c0, o0, n0, g0 = run(False)
    c1, o1, n1, g1 = run(True)
    assert c0["lm_head_loss"] == 0 and c1["lm_head_loss"] == 1
    assert o0.logits is not None and o1.logits is None
    assert n1.logits is not None and torch.equal(n0.logits, n1.logits)
    assert abs(o1.loss.item() - o0.loss.item()) <= 1e-6 * abs(o0.loss.item())
    assert sorted(g0) == sorted(g1) and "lm_head.weight" not in g1
    for n in g0:
        ok, why = _close_bf16(g1[n], g0[n])
        assert ok, (n, why)
    # a trainable head (the warm-up): fused too, and the head gets its gradient
    model.lm_head.weight.requires_grad_(True)
    c2, o2, _n2, g2 = run(False)
    c3, o3, _n3, g3 = run(True)
    assert o2.logits is not None and o3.logits is None
    assert abs(o3.loss.item() - o2.loss.item()) <= 1e-6 * abs(o2.loss.item())
    assert sorted(g2) == sorted(g3) and "lm_head.weight" in g3
    for n in g2:
        ok, why = _close_bf16(g3[n], g2[n])
        assert ok, (n, why)

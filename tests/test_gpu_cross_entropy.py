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

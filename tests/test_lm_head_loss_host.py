"""Host logic of the fused LM head + loss (fused_llama.FusedLMHeadLossFn): the label shift, which heads
take the fused path, and patch_llama / unpatch_llama of the model's forward. No kernels run here."""
import torch
from torch import nn

from sparse_matrix_tuning_amd import fused_llama as fl


def test_shifted_labels_follow_for_causal_lm_loss():
    labels = torch.tensor([[5, 6, 7, 8], [1, -100, 3, 4]])
    got = fl._shifted_labels(labels, -100, None)
    assert got.tolist() == [6, 7, 8, -100, -100, 3, 4, -100]
    explicit = torch.tensor([[9, 9, 9, 9], [8, 8, 8, 8]])
    assert fl._shifted_labels(labels, -100, explicit).tolist() == [9] * 4 + [8] * 4


def test_only_bias_free_bf16_device_heads_fuse():
    head = nn.Linear(16, 32, bias=False).bfloat16()
    head.weight.requires_grad_(False)
    assert not fl._fusable_lm_head(head)                 # host tensor: transformers' forward
    meta = nn.Linear(16, 32, bias=False, device="meta", dtype=torch.bfloat16)
    meta.weight.requires_grad_(False)
    assert not fl._fusable_lm_head(meta)                 # meta, not a ROCm device
    biased = nn.Linear(16, 32, bias=True)
    biased.weight.requires_grad_(False)
    assert not fl._fusable_lm_head(biased)
    fp32 = nn.Linear(16, 32, bias=False)
    assert not fl._fusable_lm_head(fp32)
    assert not fl._fusable_lm_head(nn.Identity())


def test_patch_llama_sets_and_removes_the_model_forward(monkeypatch):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=256, hidden_size=64, intermediate_size=128, num_hidden_layers=1,
                      num_attention_heads=2, num_key_value_heads=1)
    model = LlamaForCausalLM(cfg)
    try:
        counts = fl.patch_llama(model, attention=False)
        assert counts["loss"] == 1 and counts["lm_head_loss"] == 1
        assert model.__dict__["forward"].__func__ is fl.fused_causal_lm_forward
        assert model.loss_function is fl.fused_causal_lm_loss
    finally:
        fl.unpatch_llama(model)
    assert "forward" not in model.__dict__
    monkeypatch.setenv("SMT_LM_HEAD_LOSS", "0")
    try:
        counts = fl.patch_llama(model, attention=False)
        assert counts["loss"] == 1 and counts["lm_head_loss"] == 0 and "forward" not in model.__dict__
        counts = fl.patch_llama(model, attention=False, loss=False, lm_head_loss=True)
        assert counts["lm_head_loss"] == 0               # the fused head needs the fused loss
    finally:
        fl.unpatch_llama(model)

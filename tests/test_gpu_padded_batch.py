"""The reference's padded batches on the fused path.

The reference's collator right-pads every batch with the pad id, pads the labels with IGNORE_INDEX and
passes ``attention_mask = input_ids != pad_token_id`` (deepspeed/helpers/helper.py:194-204); for
LLaMA-3 the pad id is 0 (deepspeed_helpers.py:600-602), an ordinary token that can also occur inside a
sequence. One decoder layer at the LLaMA-3-8B geometry (hidden 4096, 32 / 8 heads, intermediate
14336) with SMT modules on q/k/v/o/gate/up/down, a right-padded batch of two sequences of mixed length
(2048 and 1377 tokens) with a pad-id token inside, runs through the product path (fused ops,
smt_flash attention with the key mask, smt_ce with IGNORE_INDEX labels) and through the CPU
restatement (oracle.ref_convert + transformers' eager attention, which applies the same 2-D mask).
Bars: loss relative <= 1e-3; every module's tile gradients vs the fp64 truth of its
own operands <= max(1e-3, 1.1 x the reference algorithm's error) and vs oracle.linearz_backward
<= 1.5 x that error; the host and product output gradients of the padded rows agree."""
from collections import defaultdict

import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
CFG = dict(vocab_size=4096, hidden_size=4096, intermediate_size=14336, num_hidden_layers=1,
           num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0, rms_norm_eps=1e-5,
           tie_word_embeddings=False, max_position_embeddings=4096)
PAD, IGNORE_INDEX = 0, -100


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _build(device):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(**CFG)
    cfg._attn_implementation = "sdpa" if device.type == "cuda" else "eager"
    torch.manual_seed(77)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            return LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)


def _collate(lengths, S):
    """helper.py:194-204 on synthetic token lists: pad ids, IGNORE_INDEX labels, mask = ids != pad."""
    gen = torch.Generator().manual_seed(3)
    ids = torch.full((len(lengths), S), PAD, dtype=torch.int64)
    labels = torch.full((len(lengths), S), IGNORE_INDEX, dtype=torch.int64)
    for b, n in enumerate(lengths):
        seq = torch.randint(1, CFG["vocab_size"], (n,), generator=gen)
        seq[0] = 1                                   # a BOS-like first token
        if b == 1:
            seq[700] = PAD                           # the pad id as an ordinary token inside the text
        ids[b, :n] = seq
        labels[b, :n] = seq
        labels[b, :17] = IGNORE_INDEX                # the prompt part (helper.py:133-135)
    return ids, labels, ids.ne(PAD)


def test_padded_batch_layer_matches_reference_restatement():
    from sparse_matrix_tuning_amd.fused_llama import KeyMask, patch_llama, unpatch_llama
    S = 2048
    ids, labels, mask = _collate([2048, 1377], S)
    assert not bool(mask[1, 1377:].any()) and not bool(mask[1, 700])
    model = _build(DEV)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    sel_att = defaultdict(list, {("q_proj", 0): [(15, 3), (0, 0)], ("k_proj", 0): [(3, 15)], ("v_proj", 0): [(2, 2)]})
    sel_mlp = defaultdict(list, {("gate_proj", 0): [(55, 0)], ("up_proj", 0): [(0, 15), (31, 4)],
                                 ("down_proj", 0): [(15, 55)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    patch_llama(model)
    seen_x, seen_g, masks = {}, {}, []
    try:
        gpu_mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}

        def capture(name):
            def hook(_m, inp, out):
                seen_x[name] = inp[0].detach().clone()
                out.register_hook(lambda g: seen_g.__setitem__(name, g.detach().clone()))
            return hook
        handles = [m.register_forward_hook(capture(n)) for n, m in gpu_mods.items()]
        attn = model.model.layers[0].self_attn
        handles.append(attn.register_forward_pre_hook(
            lambda _m, a, kw: masks.append(kw.get("attention_mask")), with_kwargs=True))
        out = model(input_ids=ids.to(DEV), attention_mask=mask.to(DEV), labels=labels.to(DEV), use_cache=False)
        out.loss.backward()
        torch.cuda.synchronize()
        for h in handles:
            h.remove()
    finally:
        unpatch_llama()
    assert masks and isinstance(masks[0], KeyMask)          # the padded batch took the key-mask path

    cpu = _build(torch.device("cpu"))
    cpu.load_state_dict(sd)
    smt.freeze_unselected_matrix_layer(cpu, sel_mlp, sel_att)
    ref.ref_convert(cpu, sel_mlp, sel_att)
    out_ref = cpu(input_ids=ids, attention_mask=mask, labels=labels, use_cache=False)
    rel = abs(out.loss.item() - out_ref.loss.item()) / abs(out_ref.loss.item())
    print(f"\npadded batch loss: MI355X {out.loss.item():.6f}, reference restatement {out_ref.loss.item():.6f}, "
          f"rel {rel:.2e}")
    assert rel <= 1e-3, (out.loss.item(), out_ref.loss.item())
    for n, m in gpu_mods.items():
        x, g = seen_x[n].cpu(), seen_g[n].cpu()
        truth = ref.tile_grads_fp64(g, x, m.index_list)
        _gi, ref_gw = ref.linearz_backward(g, x, m.weight.detach().cpu(), m.index_list)
        err, ref_err, direct = _rel(m.selected_weight.grad, truth), _rel(ref_gw, truth), _rel(m.selected_weight.grad, ref_gw)
        print(f"{n}: tile grads vs fp64 {err:.2e} (reference {ref_err:.2e}), vs oracle.linearz_backward {direct:.2e}")
        assert err <= max(1e-3, 1.1 * ref_err), (n, err)
        assert direct <= max(1e-3, 1.5 * ref_err), (n, direct)

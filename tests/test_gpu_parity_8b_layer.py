"""End-to-end parity at the LLaMA-3-8B LAYER geometry (hidden 4096, intermediate 14336, 32 query /
8 key-value heads of 128, one sequence of S = 2048): one decoder layer of the product path (fused
RMSNorm / RoPE / SwiGLU, smt_flash attention, smt_ce loss: fused_llama.patch_llama; SMT modules on
q/k/v/o/gate/up/down with tiles in every block row range) against the CPU restatement of the
reference modules (oracle.ref_convert + transformers' eager LLaMA on the host). SURVEY §8(c):
loss relative <= 1e-3; every module's tile gradient vs the fp64 truth of its own bf16 operands
<= max(1e-3, 1.1 x the reference algorithm's error on the same operands). The vocabulary is cut to
4096 (the head is not on the SMT path) so that the host side finishes in seconds."""
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


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _build(device):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(**CFG)
    cfg._attn_implementation = "sdpa" if device.type == "cuda" else "eager"
    torch.manual_seed(2024)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            return LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)


def test_llama3_8b_layer_loss_and_tile_grads_vs_reference_restatement():
    from sparse_matrix_tuning_amd.fused_llama import patch_llama, unpatch_llama
    model = _build(DEV)
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    sel_att = defaultdict(list, {("q_proj", 0): [(15, 3), (0, 0), (7, 12)], ("k_proj", 0): [(3, 15), (0, 1)],
                                 ("v_proj", 0): [(2, 2)]})
    sel_mlp = defaultdict(list, {("gate_proj", 0): [(55, 0), (10, 9)], ("up_proj", 0): [(0, 15), (31, 4), (12, 12)],
                                 ("down_proj", 0): [(15, 55), (4, 20)]})
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    patch_llama(model)
    try:
        _gpu_and_host(model, sd, sel_mlp, sel_att, unpatch_llama)
    finally:
        unpatch_llama()


def _gpu_and_host(model, sd, sel_mlp, sel_att, unpatch_llama):
    gpu_mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    assert len(gpu_mods) == 6
    seen_x, seen_g = {}, {}

    def capture(name):
        def hook(_m, inp, out):
            seen_x[name] = inp[0].detach().clone()
            out.register_hook(lambda g: seen_g.__setitem__(name, g.detach().clone()))
        return hook
    handles = [m.register_forward_hook(capture(n)) for n, m in gpu_mods.items()]
    ids = torch.randint(0, CFG["vocab_size"], (1, 2048), generator=torch.Generator().manual_seed(5))
    out = model(input_ids=ids.to(DEV), labels=ids.to(DEV), use_cache=False)
    out.loss.backward()
    torch.cuda.synchronize()
    for h in handles:
        h.remove()

    unpatch_llama()                     # the host model runs transformers' own modules
    cpu = _build(torch.device("cpu"))
    cpu.load_state_dict(sd)
    smt.freeze_unselected_matrix_layer(cpu, sel_mlp, sel_att)
    ref.ref_convert(cpu, sel_mlp, sel_att)
    out_ref = cpu(input_ids=ids, labels=ids, use_cache=False)
    rel = abs(out.loss.item() - out_ref.loss.item()) / abs(out_ref.loss.item())
    print(f"\nloss: MI355X {out.loss.item():.6f}, reference restatement {out_ref.loss.item():.6f}, rel {rel:.2e}")
    assert rel <= 1e-3, (out.loss.item(), out_ref.loss.item())

    for n, m in gpu_mods.items():
        x, g = seen_x[n].cpu(), seen_g[n].cpu()
        truth = ref.tile_grads_fp64(g, x, m.index_list)
        _gi, ref_gw = ref.linearz_backward(g, x, m.weight.detach().cpu(), m.index_list)
        err, ref_err = _rel(m.selected_weight.grad, truth), _rel(ref_gw, truth)
        print(f"{n}: {len(m.index_list)} tiles, tile-grad rel err {err:.2e} (reference algorithm {ref_err:.2e})")
        assert err <= max(1e-3, 1.1 * ref_err), (n, err)

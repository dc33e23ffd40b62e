"""Full-depth parity at the headline model: the whole 32-layer LLaMA-3-8B
(vocabulary 128256, untied head) through the product path -- fused RMSNorm / RoPE / SwiGLU, smt_flash
attention, smt_ce loss (fused_llama.patch_llama), 872 SMT tiles (436 attention over q/k/v, 436 MLP
over gate/up/down: SURVEY §8's operating point) in every layer, the engine's batched tile wgrad into
its fp32 sinks -- against the CPU restatement of the reference modules (oracle.ref_convert +
transformers' eager LLaMA on the host) with the same weights and one short batch (B = 1, S = 256).

SURVEY §8(c) bars: loss relative <= 1e-3; every SMT module's tile gradient vs the fp64 truth of its
own bf16 operands (input and output gradient as the product saw them) <= max(1e-3, 1.1 x the
reference algorithm's error on the same operands). The host's own tile gradients come from a
different 32-layer bf16 forward/backward (its activations differ from the product's by bf16 rounding
in every layer), so there is no derivable bar for the direct difference; it is printed per module.

The tiles are a seeded draw of SURVEY §8's counts, not a harvest: the selection itself is pinned
separately at this geometry (tests/test_gpu_selection_8b.py), and a warm-up of the 8 B model would
dominate the test."""
import random
from collections import defaultdict

import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd.smt import smt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def _selection(cfg, n_att=436, n_mlp=436, seed=872):
    """{(module, layer): [(row_block, col_block), ...]} draws of the §8 counts over all 32 layers."""
    h, inter, L = cfg["hidden_size"], cfg["intermediate_size"], cfg["num_hidden_layers"]
    kv = h // cfg["num_attention_heads"] * cfg["num_key_value_heads"]
    shapes = {"q_proj": (h, h), "k_proj": (kv, h), "v_proj": (kv, h),
              "gate_proj": (inter, h), "up_proj": (inter, h), "down_proj": (h, inter)}
    rng = random.Random(seed)

    def draw(mods, n):
        pool = [(m, l, i, j) for m in mods for l in range(L)
                for i in range(shapes[m][0] // 256) for j in range(shapes[m][1] // 256)]
        sel = defaultdict(list)
        for m, l, i, j in sorted(rng.sample(pool, n), reverse=True):
            sel[(m, l)].append((i, j))
        return sel
    return draw(("q_proj", "k_proj", "v_proj"), n_att), draw(("gate_proj", "up_proj", "down_proj"), n_mlp)


@pytest.mark.timeout(600)
def test_llama3_8b_full_depth_loss_and_tile_grads_vs_reference_restatement():
    import bench
    from transformers import LlamaConfig, LlamaForCausalLM
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd.fused_llama import patch_llama, unpatch_llama

    cfg = bench.MODELS["llama3-8b"]
    model = bench.build_model("llama3-8b", DEV)
    # the host copy: same parameters and buffers (rotary inv_freq), without a CPU initialisation
    hcfg = LlamaConfig(**cfg)
    hcfg._attn_implementation = "eager"
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device("meta"):
            cpu = LlamaForCausalLM(hcfg)
    finally:
        torch.set_default_dtype(prev)
    cpu = cpu.to_empty(device="cpu")
    with torch.no_grad():
        for (n, p), (n2, q) in zip(model.named_parameters(), cpu.named_parameters()):
            assert n == n2
            q.copy_(p)
        for (n, b), (n2, c) in zip(model.named_buffers(), cpu.named_buffers()):
            assert n == n2
            c.copy_(b)

    patch_llama(model)                      # as bench.py: fused ops, smt_flash, smt_ce
    sel_att, sel_mlp = _selection(cfg)
    assert sum(map(len, sel_att.values())) == 436 and sum(map(len, sel_mlp.values())) == 436
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    opt = SMTFusedAdam(smt.get_optimizer_sparse_grouped_parameters(model, 0.0, 9.865e-6), lr=9.865e-6,
                       betas=(0.9, 0.95))
    engine, *_ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    gpu_mods = {n: m for n, m in model.named_modules() if isinstance(m, smt.LinearLayer_MatrixSparsity)}
    assert sum(len(m.index_list) for m in gpu_mods.values()) == 872
    seen_x, seen_g = {}, {}

    def capture(name):
        def hook(_m, inp, out):
            seen_x[name] = inp[0].detach().clone()
            out.register_hook(lambda g: seen_g.__setitem__(name, g.detach().clone()))
        return hook
    handles = [m.register_forward_hook(capture(n)) for n, m in gpu_mods.items()]
    ids = torch.randint(0, cfg["vocab_size"], (1, 256), generator=torch.Generator().manual_seed(88))
    try:
        loss = engine(input_ids=ids.to(DEV), labels=ids.to(DEV), use_cache=False).loss
        engine.backward(loss)
        torch.cuda.synchronize()
    finally:
        unpatch_llama()                     # the host model runs transformers' own modules
    for h in handles:
        h.remove()
    gpu_loss = loss.item()
    grads = {n: m.selected_weight._smt_grad_sink.buffer.detach().cpu() for n, m in gpu_mods.items()}
    ops = {n: (seen_x[n].cpu(), seen_g[n].cpu(), m.weight.detach().cpu(), list(m.index_list))
           for n, m in gpu_mods.items()}
    del engine, opt, model, gpu_mods, seen_x, seen_g, loss
    torch.cuda.empty_cache()

    smt.freeze_unselected_matrix_layer(cpu, sel_mlp, sel_att)
    ref.ref_convert(cpu, sel_mlp, sel_att)
    out_ref = cpu(input_ids=ids, labels=ids, use_cache=False)
    out_ref.loss.backward()
    rel = abs(gpu_loss - out_ref.loss.item()) / abs(out_ref.loss.item())
    print(f"\nloss: MI355X {gpu_loss:.6f}, reference restatement {out_ref.loss.item():.6f}, rel {rel:.2e}")
    assert rel <= 1e-3, (gpu_loss, out_ref.loss.item())

    cpu_mods = {n: m for n, m in cpu.named_modules() if isinstance(m, ref.RefLinearLayer_MatrixSparsity)}
    assert sorted(cpu_mods) == sorted(ops)
    worst = (0.0, "")
    for n, (x, g, W, tiles) in ops.items():
        truth = ref.tile_grads_fp64(g, x, tiles)
        _gi, ref_gw = ref.linearz_backward(g, x, W, tiles)
        err, ref_err = _rel(grads[n], truth), _rel(ref_gw, truth)
        host = _rel(grads[n], cpu_mods[n].selected_weight.grad)
        print(f"{n}: {len(tiles)} tiles, vs fp64 {err:.2e} (reference algorithm {ref_err:.2e}); "
              f"vs the host model's own tile gradient {host:.2e}")
        assert err <= max(1e-3, 1.1 * ref_err), (n, err, ref_err)
        worst = max(worst, (err, n))
    print(f"worst module vs fp64: {worst}")

"""What one decoder layer keeps for its backward on the fused path, by tensor (distinct storages),
at the LLaMA-3-8B layer geometry with SMT tiles on all seven modules (GPU diagnostic for the
activation policies of bench.py: resident / selective / per-layer recompute).

    python scripts/diag/saved_bytes.py [--batch 16] [--seq 2048] [--policy resident|selective]
"""
import argparse
import json
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

CFG = dict(vocab_size=4096, hidden_size=4096, intermediate_size=14336, num_hidden_layers=2,
           num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0, rms_norm_eps=1e-5,
           tie_word_embeddings=False, max_position_embeddings=4096)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--tiles", type=int, default=8, help="tiles per module")
    ap.add_argument("--policy", default="resident")
    args = ap.parse_args()
    from transformers import LlamaConfig, LlamaForCausalLM
    from sparse_matrix_tuning_amd.smt import smt
    from sparse_matrix_tuning_amd.fused_llama import patch_llama
    dev = torch.device("cuda", 0)
    cfg = LlamaConfig(**CFG)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(0)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        model = LlamaForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    gen = torch.Generator().manual_seed(1)
    shapes = {"q_proj": (16, 16), "k_proj": (4, 16), "v_proj": (4, 16), "o_proj": (16, 16),
              "gate_proj": (56, 16), "up_proj": (56, 16), "down_proj": (16, 56)}
    sel_att, sel_mlp = defaultdict(list), defaultdict(list)
    for layer in range(CFG["num_hidden_layers"]):
        for m, (r, c) in shapes.items():
            picks = torch.randperm(r * c, generator=gen)[: args.tiles].tolist()
            d = sel_mlp if m in ("gate_proj", "up_proj", "down_proj") else sel_att
            d[(m, layer)] = sorted((p // c, p % c) for p in picks)
    smt.freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    smt.convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    patch_llama(model)
    smt.set_activation_policy(args.policy)
    model.model.embed_tokens.weight.requires_grad_(False)

    saved = {}
    order = []

    def pack(t):
        st = t.untyped_storage()
        key = st.data_ptr()
        if key not in saved and t.device.type == "cuda":
            saved[key] = (st.nbytes(), tuple(t.shape), str(t.dtype))
            order.append(key)
        return t

    ids = torch.randint(1, CFG["vocab_size"], (args.batch, args.seq), generator=gen).to(dev)
    layer1 = model.model.layers[1]
    marks = {}
    layer1.register_forward_pre_hook(lambda *_: marks.__setitem__("start", len(order)))
    layer1.register_forward_hook(lambda *_: marks.__setitem__("end", len(order)))
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated(dev)
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        out = model(input_ids=ids, labels=ids, use_cache=False)
    torch.cuda.synchronize()
    after = torch.cuda.memory_allocated(dev)
    keys = order[marks["start"]: marks["end"]]
    by_shape = defaultdict(int)
    for k in keys:
        nb, shp, dt = saved[k]
        by_shape[f"{list(shp)} {dt}"] += nb
    total = sum(saved[k][0] for k in keys)
    out.loss.backward()
    torch.cuda.synchronize()
    print(json.dumps({"policy": args.policy, "batch": args.batch, "seq": args.seq, "tiles_per_module": args.tiles,
                      "layer_saved_gb": round(total / 1e9, 3), "forward_allocated_gb": round((after - base) / 1e9, 3),
                      "by_shape_gb": {k: round(v / 1e9, 3) for k, v in sorted(by_shape.items(), key=lambda kv: -kv[1])}}))


if __name__ == "__main__":
    main()

"""Seeded tile draws at the LLaMA-3-8B operating point (436 attention tiles over q/k/v and
436 MLP tiles over gate/up/down, all 32 layers). Shared by the full-depth parity test and the 8B
data-parallel worker; a helper, never collected by pytest.

The draw is not a harvest: the selection itself is pinned separately at this geometry
(tests/test_gpu_selection_8b.py), and a warm-up of the 8 B model would dominate the tests."""
import random
from collections import defaultdict


def seeded_selection(cfg, n_att=436, n_mlp=436, seed=872):
    """``(sel_att, sel_mlp)``: ``{(module, layer): [(row_block, col_block), ...]}`` draws of the §8
    counts over every layer of the model ``cfg`` describes, in the layout ``select_submatrix``
    returns (each key's tiles in descending order)."""
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
        return dict(sel)
    return draw(("q_proj", "k_proj", "v_proj"), n_att), draw(("gate_proj", "up_proj", "down_proj"), n_mlp)


def bits_hash(t):
    """Two 64-bit checksums of a tensor's bits (plain and position-weighted sums of the bit patterns
    as integers, wrapping), computed where the tensor lives. Used to compare multi-GB states of two
    runs bit for bit without writing them out."""
    import torch
    v = t.detach().contiguous().view(-1)
    iv = v.view({1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[v.element_size()]).to(torch.int64)
    w = torch.arange(iv.numel(), device=iv.device, dtype=torch.int64)
    w.mul_(0x9E3779B1).remainder_(2 ** 31 - 1).add_(1)
    h = (int((iv * w).sum().item()), int(iv.sum().item()), iv.numel())
    del w, iv
    return h

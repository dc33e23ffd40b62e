"""How much config 4's channel selection depends on the order of the bf16 rank sum.

The reference's activation hook (fine_tune.py:651-665) all-reduces every rank's bf16 ``|x|`` in bf16
and adds the sum to an fp32 accumulator. Two ranks give the same bits in any order; from three on the
bf16 sum depends on the collective's internal order, which NCCL / RCCL / gloo choose per element (a
ring starts each chunk's reduction at a different rank). This replays the reference's arithmetic
(``oracle.channel_hook_accumulate_ranks``) on synthetic activation-like inputs at config 4's geometry
(LLaMA-2-13B hidden 5120, B 16 x S 2048 per rank, 2 collection steps, q/k/v of two layers) under
several orders and compares the accumulators and the selections (``oracle.select_channel``, the
reference's heap ranking) with the sequential order's.

    python scripts/channel_rank_order.py --world 4 8 --sigma 1.0 --out profiles/r05_channel_rank_order_s1.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import smt_oracle as ref  # noqa: E402


def ring_chunks(xs):
    """A ring all-reduce's order: the flattened tensor in ``world`` contiguous chunks, chunk c reduced
    starting at rank c+1 and ending at rank c (NCCL's / RCCL's ring reduce-scatter)."""
    w = len(xs)
    flat = [x.reshape(-1) for x in xs]
    n = flat[0].numel()
    out = torch.empty(n, dtype=torch.float32)
    bounds = [n * c // w for c in range(w + 1)]
    for c in range(w):
        a, b = bounds[c], bounds[c + 1]
        out[a:b] = ref.bf16_rank_sum([f[a:b] for f in flat], [(c + 1 + i) % w for i in range(w)])
    return out.view(xs[0].shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[4, 8])
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--H", type=int, default=5120)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--n", type=int, default=1121, help="channels selected over the 6 keys (0.86 %% share)")
    ap.add_argument("--sigma", type=float, default=1.0, help="spread of the per-channel lognormal scales")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    results = {"geometry": {"B": args.B, "S": args.S, "H": args.H, "steps": args.steps, "keys": 6, "n": args.n,
                            "sigma": args.sigma},
               "inputs": f"x = N(0,1) * per-channel lognormal(sigma {args.sigma}) scale (fixed per layer), drawn per rank and "
                         "step, bf16; q/k/v of a layer hook the same input (one accumulator)", "worlds": {}}
    for world in args.world:
        t0 = time.time()
        g = torch.Generator().manual_seed(5 + world)
        orders = {"sequential": list(range(world)), "reversed": list(range(world))[::-1], "pairwise": "pairwise", "ring": "ring"}
        accs = {o: {} for o in orders}
        for layer in range(2):
            scale = torch.exp(args.sigma * torch.randn(args.H, generator=g))
            for _step in range(args.steps):
                xs = [(torch.randn(args.B, args.S, args.H, generator=g) * scale).bfloat16() for _ in range(world)]
                for name, order in orders.items():
                    if order == "ring":
                        s = ring_chunks([x.abs() for x in xs])
                        d = accs[name]
                        d[layer] = s if layer not in d else d[layer] + s
                    else:
                        ref.channel_hook_accumulate_ranks(accs[name], layer, xs, order)
                del xs
        base = accs["sequential"]
        sel = {}
        for name in orders:
            act = {(m, layer): accs[name][layer] for layer in range(2) for m in ("q_proj", "k_proj", "v_proj")}
            sel[name] = ref.select_channel(act, args.n)
        w = {}
        for name in orders:
            diff = sum(int((accs[name][l] != base[l]).sum()) for l in range(2))
            tot = sum(base[l].numel() for l in range(2))
            rel = max(float(((accs[name][l] - base[l]).abs() / base[l].abs().clamp_min(1e-30)).max()) for l in range(2))
            a = {(k, c) for k, v in sel["sequential"].items() for c in v}
            b = {(k, c) for k, v in sel[name].items() for c in v}
            same_lists = all(list(sel[name].get(k, [])) == list(v) for k, v in sel["sequential"].items())
            # the per-key order (the row order of selected_weight, smt.py:196-204): positions that moved
            moved, disp = 0, 0
            for k, v in sel["sequential"].items():
                other = list(sel[name].get(k, []))
                pos = {c: i for i, c in enumerate(other)}
                for i, c in enumerate(v):
                    if i >= len(other) or other[i] != c:
                        moved += 1
                    if c in pos:
                        disp = max(disp, abs(pos[c] - i))
            w[name] = {"acc_elements_differing": diff, "acc_fraction_differing": diff / tot,
                       "acc_max_rel_diff": rel, "selected_channels_differing": len(a ^ b) // 2,
                       "positions_moved": moved, "max_displacement": disp,
                       "selection_identical": a == b and same_lists}
        w["seconds"] = round(time.time() - t0, 1)
        results["worlds"][str(world)] = w
        print(world, json.dumps(w), flush=True)
        del accs
    line = json.dumps(results)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()

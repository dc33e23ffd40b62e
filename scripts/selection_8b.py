#!/usr/bin/env python3
"""LLaMA-3-8B-shaped block selection on the GPU vs the reference's CPU path (SURVEY §8(d)
"Selection fixtures").

    python scripts/selection_8b.py [--layers 32] [--sigma 0.5] [--out file.json]

Builds the warm-up gradient dict of LLaMA-3-8B (32 layers x q 4096^2, k/v 1024x4096 = attention
pool 805 M elements; gate/up 14336x4096, down 4096x14336 = MLP pool 5.64 G elements; fp32) in HBM:
N(0, 1) x per-block lognormal(sigma) x 1e-4, seeded. Then

1. the product (``smt_helper.select_submatrix_based_on_grads``: GPU scan + intervals + host re-score
   of undecided keys): attention pool ``mean_abs`` n=436, MLP pool ``abs_mean`` n=436, as
   fine_tune.py:306-327 dispatches them;
2. the reference's path restated (``oracle.select_submatrix``: ATen fp32 reductions on the host CPU +
   the heap loop of smt_helper.py:111-139) on host copies of the same tensors,

and reports both times (elements/s: BASELINE.md CPU-baseline unit 2), the size of the undecided band
(blocks flagged, keys re-scored) and whether the two selections are identical (keys, key order, tile
order). Test infrastructure: imports the oracle.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DIMS = {"q_proj": [4096, 4096], "k_proj": [1024, 4096], "v_proj": [1024, 4096],
        "gate_proj": [14336, 4096], "up_proj": [14336, 4096], "down_proj": [4096, 14336]}


def make_pool(mods, layers, sigma, gen, dev):
    pool = {}
    for layer in range(layers):
        for m in mods:
            r, c = DIMS[m]
            g = torch.randn(r, c, generator=gen, device=dev)
            scale = torch.exp(sigma * torch.randn(r // 256, c // 256, generator=gen, device=dev))
            g.view(r // 256, 256, c // 256, 256).mul_(scale.view(r // 256, 1, c // 256, 1)).mul_(1e-4)
            pool[(m, layer)] = g
    return pool


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--sigma", type=float, default=0.5)
    ap.add_argument("--n-att", type=int, default=436)
    ap.add_argument("--n-mlp", type=int, default=436)
    ap.add_argument("--skip-cpu", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from oracle import smt_oracle as ref
    from sparse_matrix_tuning_amd import _hip
    from sparse_matrix_tuning_amd.smt import ranking, smt_helper
    _hip.load()
    dev = torch.device("cuda", 0)
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    gen = torch.Generator(device=dev).manual_seed(1234)
    pools = {"attention": (make_pool(("q_proj", "k_proj", "v_proj"), args.layers, args.sigma, gen, dev), "mean_abs", args.n_att),
             "mlp": (make_pool(("gate_proj", "up_proj", "down_proj"), args.layers, args.sigma, gen, dev), "abs_mean", args.n_mlp)}
    torch.cuda.synchronize()
    out = {"layers": args.layers, "sigma": args.sigma, "cpu_threads": cores,
           "cpu_capability": torch.backends.cpu.get_cpu_capability(), "pools": {}}
    for name, (pool, strategy, n) in pools.items():
        elems = sum(g.numel() for g in pool.values())
        smt_helper.select_submatrix_based_on_grads({k: v for k, v in list(pool.items())[:2]}, DIMS, 4,
                                                   calculate_strategy=strategy)          # warm the kernels
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        got = smt_helper.select_submatrix_based_on_grads(pool, DIMS, n, calculate_strategy=strategy)
        t_gpu = time.perf_counter() - t0
        rep = dict(ranking.LAST_REPORT)
        rec = {"strategy": strategy, "n": n, "elements": elems, "blocks": rep["candidates"],
               "gpu_seconds": round(t_gpu, 4), "gpu_elements_per_s": elems / t_gpu,
               "band": {"flagged_blocks": rep["flagged"], "rescored_keys": [list(k) for k in rep["rescored_keys"]],
                        "iterations": rep["iterations"], "worst_case_bound": rep["worst_case_bound"],
                        "ranking_seconds": round(rep["seconds"], 4)},
               "tiles_per_key": {f"{k[0]}.{k[1]}": len(v) for k, v in got.items()}}
        print(f"[sel8b] {name}: GPU {t_gpu:.3f}s, flagged {rep['flagged']}, rescored {len(rep['rescored_keys'])} keys",
              file=sys.stderr, flush=True)
        if not args.skip_cpu:
            t0 = time.perf_counter()
            host = {k: v.cpu() for k, v in pool.items()}
            t_copy = time.perf_counter() - t0
            t0 = time.perf_counter()
            want = ref.select_submatrix(host, DIMS, n, calculate_strategy=strategy)
            t_cpu = time.perf_counter() - t0
            del host
            rec.update({"cpu_seconds": round(t_cpu, 3), "cpu_elements_per_s": elems / t_cpu,
                        "d2h_seconds": round(t_copy, 3),
                        "identical": list(got.items()) == list(want.items()),
                        "same_set": sorted((k, t) for k, v in got.items() for t in v)
                        == sorted((k, t) for k, v in want.items() for t in v)})
            print(f"[sel8b] {name}: reference CPU {t_cpu:.1f}s, identical={rec['identical']}", file=sys.stderr, flush=True)
        out["pools"][name] = rec
        del pool
        torch.cuda.empty_cache()
    line = json.dumps(out)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()

"""LM head + causal-LM loss at the bench geometry (T = 32768 rows, H 4096, V 128256): the unfused pair
(lm_head on the transposed copy + smt_ce) against fused_llama.FusedLMHeadLossFn at several chunk
sizes. Per variant: forward + backward time (HIP events, median of iters), the peak memory above the
operands, and whether the loss and dh are bit-identical to the unfused pair's.

    python scripts/lm_head_loss_bench.py --out gpurun_out/lm_head_loss.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_matrix_tuning_amd import fused_llama as fl            # noqa: E402
from sparse_matrix_tuning_amd.engine import FrozenLinearFn        # noqa: E402


class _Head:
    def __init__(self, w, wt):
        self.weight = w
        w._smt_weight_t = wt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32768)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--chunks", default="2048,4096,8192,16384,32768")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    N, H, V = a.rows, a.hidden, a.vocab
    h = torch.randn(N, H, device=dev, generator=g).bfloat16()
    w = (torch.randn(V, H, device=dev, generator=g) * 0.02).bfloat16()
    wt = w.t().contiguous()
    w._smt_weight_t = wt
    labels = torch.randint(0, V, (1, N), device=dev, generator=g)
    head = _Head(w, wt)

    def unfused():
        x = h.view(1, N, H).detach().requires_grad_(True)
        logits = FrozenLinearFn.apply(x, w, wt, None)
        loss = fl.fused_causal_lm_loss(logits, labels, vocab_size=V)
        loss.backward()
        return loss.detach(), x.grad

    def fused(c):
        def run():
            x = h.view(1, N, H).detach().requires_grad_(True)
            loss = fl.fused_lm_head_loss(x, head, labels, chunk_rows=c)
            loss.backward()
            return loss.detach(), x.grad
        return run

    def measure(fn):
        fn()
        torch.cuda.synchronize()
        times = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
            del out
        base = torch.cuda.memory_allocated()
        torch.cuda.reset_peak_memory_stats()
        out = fn()
        torch.cuda.synchronize()
        peak = torch.cuda.max_memory_allocated() - base
        return sorted(times)[len(times) // 2], peak, out

    rows = []
    ms, peak, (lu, gu) = measure(unfused)
    rows.append({"variant": "unfused", "ms": round(ms, 3), "peak_gib": round(peak / 2 ** 30, 3)})
    print(json.dumps(rows[-1]), flush=True)
    for c in [int(x) for x in a.chunks.split(",")]:
        ms, peak, (lf, gf) = measure(fused(c))
        rows.append({"variant": f"fused_chunk_{c}", "chunk_rows": c, "ms": round(ms, 3),
                     "peak_gib": round(peak / 2 ** 30, 3), "loss_bit_identical": bool(torch.equal(lu, lf)),
                     "dh_bit_identical": bool(torch.equal(gu, gf)),
                     "dh_rel": ((gf.float() - gu.float()).norm() / gu.float().norm()).item()})
        print(json.dumps(rows[-1]), flush=True)
        del lf, gf
    if a.out:
        with open(a.out, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()

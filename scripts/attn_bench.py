"""Time the gfx950 flash attention (fused_llama.flash_attention) against torch sdpa (aotriton) at
the LLaMA-3-8B step shape: B=16, Hq=32, Hkv=8, S=2048, D=128, causal, q/k/v in the HF layout
(transposed views of [B, S, H, D]). FLOPs: fwd 4*B*Hq*S^2*D/2, bwd 2.5x fwd."""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_matrix_tuning_amd.fused_llama import flash_attention  # noqa: E402


def timed(fn, iters):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    e[0].record()
    for _ in range(iters):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=8)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--impl", nargs="*", default=["smt", "sdpa"])
    a = ap.parse_args()
    B, Hq, Hkv, S, D = a.B, a.Hq, a.Hkv, a.S, 128
    torch.manual_seed(0)
    mk = lambda H: torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2).requires_grad_(True)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    g = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    fl = 4 * B * Hq * S * S * D / 2
    for impl in a.impl:
        if impl == "smt":
            f = lambda: flash_attention(q, k, v)
        else:
            f = lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True, enable_gqa=True).transpose(1, 2)
        o = f()
        fwd = timed(f, a.iters)
        def fb():
            q.grad = k.grad = v.grad = None          # no gradient-accumulation adds in the timing
            out = f()
            out.backward(g)
        tot = timed(fb, a.iters)
        bwd = tot - fwd
        print(json.dumps({"impl": impl, "env": {k: v for k, v in os.environ.items() if k.startswith("SMT_ATTN")}, "B": B, "Hq": Hq, "Hkv": Hkv, "S": S, "fwd_ms": round(fwd, 3),
                          "bwd_ms": round(bwd, 3), "fwd_tflops": round(fl / fwd / 1e9, 1),
                          "bwd_tflops": round(2.5 * fl / bwd / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()

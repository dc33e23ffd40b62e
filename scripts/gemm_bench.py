"""Per-shape bf16 GEMM throughput of the LLaMA-3-8B SMT step (T = 16 x 2048 tokens) through
torch.matmul (hipBLASLt), forward (x @ W^T) and data-gradient (g @ W) forms, plus the fused
QKV / gate-up variants. Prints one JSON line per shape."""
import json
import os
import sys

import torch

T = int(os.environ.get("GEMM_T", 32768))
H, I, KV, V = 4096, 14336, 1024, 128256
SHAPES = {  # name: (in, out)
    "q/o": (H, H), "k/v": (H, KV), "gate/up": (H, I), "down": (I, H), "lm_head": (H, V),
    "qkv_fused": (H, H + 2 * KV), "gate_up_fused": (H, 2 * I),
}


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    torch.manual_seed(0)
    only = [n for n in os.environ.get("GEMM_SHAPES", "").split(",") if n]
    for name, (fin, fout) in SHAPES.items():
        if only and name not in only:
            continue
        x = torch.randn(T, fin, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(fout, fin, device="cuda", dtype=torch.bfloat16) * 0.02
        g = torch.randn(T, fout, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * T * fin * fout
        tf = timed(lambda: torch.matmul(x, W.t()))
        tb = timed(lambda: torch.matmul(g, W))
        print(json.dumps({"shape": name, "in": fin, "out": fout, "fwd_ms": round(tf, 3), "fwd_tflops": round(fl / tf / 1e9, 1),
                          "dgrad_ms": round(tb, 3), "dgrad_tflops": round(fl / tb / 1e9, 1)}), flush=True)
        del x, W, g


if __name__ == "__main__":
    main()

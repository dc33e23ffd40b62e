"""Time the step's forward GEMM shapes (F.linear(x, W), T = 32768) with rotating inputs (three x
buffers, so the operands do not stay in the 256 MB MALL between calls), as the default hipBLASLt
heuristics pick them, or, under PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0
PYTORCH_TUNABLEOP_FILENAME=<table>, as a TunableOp table picks them. One JSON line per shape."""
import json
import os

import torch
import torch.nn.functional as F

T = 16 * 2048
SHAPES = {"q/o": (4096, 4096), "k/v": (4096, 1024), "gate/up": (4096, 14336), "down": (14336, 4096),
          "lm_head": (4096, 128256), "qkv_joint": (4096, 6144)}


def main():
    dev = torch.device("cuda", 0)
    tag = "tunableop" if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1" else "default"
    for name, (fin, fout) in SHAPES.items():
        xs = [torch.randn(T, fin, device=dev, dtype=torch.bfloat16) for _ in range(3)]
        w = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16) * 0.02
        n = 6 if name == "lm_head" else 30
        for i in range(3):
            F.linear(xs[i], w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            F.linear(xs[i % 3], w)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / n
        # the data gradient on the transposed copy (g @ (W^T)^T, engine.FrozenLinearFn)
        gs = [torch.randn(T, fout, device=dev, dtype=torch.bfloat16) for _ in range(3)]
        wt = w.t().contiguous()
        for i in range(3):
            torch.matmul(gs[i], wt.t())
        torch.cuda.synchronize()
        e0.record()
        for i in range(n):
            torch.matmul(gs[i % 3], wt.t())
        e1.record()
        torch.cuda.synchronize()
        ms_d = e0.elapsed_time(e1) / n
        print(json.dumps({"tag": tag, "shape": name, "in": fin, "out": fout, "ms": round(ms, 4),
                          "tflops": round(2 * T * fin * fout / ms / 1e9, 1), "dgrad_ms": round(ms_d, 4)}), flush=True)
        del xs, w, gs, wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

"""Dense weight-gradient GEMMs of the full fine-tuning warm-up (fine_tune.py:160-190) at the
LLaMA-3-8B bench shapes (T = 32768): hipBLASLt time of dW = g^T x as autograd issues it against other
operand layouts of the same product. One JSON line per (shape, variant)."""
import json
import torch

T = 32768
SHAPES = {"q/o": (4096, 4096), "k/v": (1024, 4096), "gate/up": (14336, 4096), "down": (4096, 14336)}


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for name, (out_f, in_f) in SHAPES.items():
        g = torch.randn(T, out_f, device=dev, dtype=torch.bfloat16)
        x = torch.randn(T, in_f, device=dev, dtype=torch.bfloat16)
        gt = g.t().contiguous()
        xt = x.t().contiguous()
        flops = 2.0 * T * out_f * in_f
        variants = {
            "autograd: mm(g.t(), x)": lambda: torch.mm(g.t(), x),
            "mm(x.t(), g) (dW^T)": lambda: torch.mm(x.t(), g),
            "mm(gt, x), gt contiguous": lambda: torch.mm(gt, x),
            "mm(g.t(), xt.t())": lambda: torch.mm(g.t(), xt.t()),
            "mm(gt, xt.t())": lambda: torch.mm(gt, xt.t()),
            "mm fp32 out": lambda: torch.mm(g.t(), x, out_dtype=torch.float32),
        }
        for v, fn in variants.items():
            ms = timed(fn)
            print(json.dumps({"shape": name, "out": out_f, "in": in_f, "T": T, "variant": v, "ms": round(ms, 3),
                              "pflops": round(flops / ms / 1e12, 3)}), flush=True)
        del g, x, gt, xt


if __name__ == "__main__":
    main()

"""Compare ROCm SDPA flash backends (aotriton vs CK) at the LLaMA-3-8B step shape."""
import sys
import time
import torch
import torch.nn.functional as F


def run(lib, B=16, H=32, S=2048, D=128, iters=5):
    torch.backends.cuda.preferred_rocm_fa_library(lib)
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
    def step():
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        o.backward(g)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    fwd = bwd = 0.0
    for _ in range(iters):
        e0.record()
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        e1.record()
        o.backward(g)
        e2.record()
        torch.cuda.synchronize()
        fwd += e0.elapsed_time(e1); bwd += e1.elapsed_time(e2)
    fl = 4 * B * H * S * S * D / 2
    print(f"{lib}: fwd {fwd/iters:.2f} ms ({fl/(fwd/iters*1e-3)/1e12:.0f} TF/s)  bwd {bwd/iters:.2f} ms ({2.5*fl/(bwd/iters*1e-3)/1e12:.0f} TF/s)", flush=True)


for lib in sys.argv[1:] or ["aotriton", "ck"]:
    try:
        run(lib)
    except Exception as e:
        print(lib, "failed:", repr(e)[:300])

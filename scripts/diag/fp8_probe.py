"""Probe torch._scaled_mm fp8 paths on gfx950 (tensorwise / rowwise / MX blockwise e8m0) at the
LLaMA-3-8B GEMM shapes; prints capability + TF/s per variant (T = 32768)."""
import json
import statistics
import traceback

import torch

T = 32768
dev = "cuda"
f8 = torch.float8_e4m3fn


def timed(fn, iters=10):
    fn(); torch.cuda.synchronize()
    out = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record(); torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / iters)
    return statistics.median(out)


res = {"device": torch.cuda.get_device_name(0), "arch": torch.cuda.get_device_properties(0).gcnArchName}
for name, (K, N) in {"q/o": (4096, 4096), "gate/up": (4096, 14336), "down": (14336, 4096)}.items():
    x = torch.randn(T, K, device=dev).to(f8)
    w = torch.randn(N, K, device=dev).to(f8)          # [N, K] row-major -> w.t() is column-major [K, N]
    fl = 2.0 * T * K * N
    r = {}
    xb = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
    wb = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    r["bf16_tflops"] = round(fl / timed(lambda: xb @ wb.t()) / 1e9, 1)
    one = torch.ones((), device=dev)
    for variant, (sa, sb) in {
        "tensorwise": (one, one),
        "rowwise": (torch.ones(T, 1, device=dev), torch.ones(1, N, device=dev)),
        "mx_e8m0_b32": (torch.full((T * ((K // 32 + 3) // 4 * 4),), 127, device=dev, dtype=torch.uint8).view(torch.float8_e8m0fnu),
                        torch.full((N * ((K // 32 + 3) // 4 * 4),), 127, device=dev, dtype=torch.uint8).view(torch.float8_e8m0fnu)),
    }.items():
        try:
            y = torch._scaled_mm(x, w.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
            ref = (x.float() @ w.float().t())
            err = ((y.float() - ref).norm() / ref.norm()).item()
            t = timed(lambda: torch._scaled_mm(x, w.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16))
            r[variant] = {"tflops": round(fl / t / 1e9, 1), "rel_err_vs_fp32_of_fp8_inputs": err}
        except Exception as e:  # noqa: BLE001
            r[variant] = {"error": (type(e).__name__ + ": " + str(e))[:300]}
    res[name] = r
    print(json.dumps({name: r}), flush=True)
print(json.dumps(res), flush=True)

"""Fused SwiGLU + fp8 quantisation kernels vs the unfused pairs at the LLaMA-3-8B MLP shape
(T = 32768 rows, 14336 columns), interleaved rounds in one process. Prints one JSON line."""
import json
import statistics

import torch

from sparse_matrix_tuning_amd import _hip
from sparse_matrix_tuning_amd import fp8 as f8

T, N = 32768, 14336


def timed(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    torch.manual_seed(0)
    g = (torch.randn(T, N, device="cuda") * 3).bfloat16()
    u = torch.randn(T, N, device="cuda").bfloat16()
    dh = (torch.randn(T, N, device="cuda") * 1e-3).bfloat16()
    h = torch.empty_like(g)
    dg, du = torch.empty_like(g), torch.empty_like(g)
    lib = _hip.load()
    st = torch.cuda.current_stream().cuda_stream

    def fwd_unfused():
        lib.smt_swiglu_fwd(g.data_ptr(), u.data_ptr(), h.data_ptr(), g.numel(), 0, st)
        f8.quant_rows(h)

    def bwd_unfused():
        lib.smt_swiglu_bwd(g.data_ptr(), u.data_ptr(), dh.data_ptr(), dg.data_ptr(), du.data_ptr(), g.numel(), 0, st)
        f8.quant_rows_cat([dg, du])

    fns = {"fwd_unfused": fwd_unfused,
           "fwd_fused": lambda: f8.swiglu_fwd_quant(g, u, False),
           "fwd_fused_bf16": lambda: f8.swiglu_fwd_quant(g, u, True),
           "bwd_unfused": bwd_unfused,
           "bwd_fused": lambda: f8.swiglu_bwd_quant(g, u, dh, False, False),
           "bwd_fused_bf16": lambda: f8.swiglu_bwd_quant(g, u, dh, True, True)}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            res[k].append(timed(f))
    print(json.dumps({k + "_ms": round(statistics.median(v), 3) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()

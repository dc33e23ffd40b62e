"""The LM head GEMMs of the bench step (LLaMA-3-8B: T = 32768, vocab 128256, hidden 4096) as one
hipBLASLt GEMM vs the vocabulary cut into chunks: forward logits = x @ W^T, data gradient
dx = dlogits @ W (chunks accumulated through the GEMM's C operand). HIP events, interleaved."""
import json

import torch


def timed(fn, iters=5):
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
    T, V, H = 32768, 128256, 4096
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    W = (torch.randn(V, H, device=dev) * 0.02).bfloat16()
    WT = W.t().contiguous()                       # the engine's transposed copy (TN data gradient)
    g = (torch.randn(T, V, device=dev) * 1e-3).bfloat16()
    fl = 2.0 * T * V * H
    for rnd in range(2):
        for n in (1, 2, 3, 4, 8):
            bounds = [V * i // n // 64 * 64 for i in range(n)] + [V]
            outs = [torch.empty(T, bounds[i + 1] - bounds[i], device=dev, dtype=torch.bfloat16) for i in range(n)]

            def fwd():
                for i in range(n):
                    torch.mm(x, W[bounds[i]:bounds[i + 1]].t(), out=outs[i])
            dx = torch.empty(T, H, device=dev, dtype=torch.bfloat16)

            def dgrad():
                torch.mm(g[:, bounds[0]:bounds[1]], WT[:, bounds[0]:bounds[1]].t(), out=dx)
                for i in range(1, n):
                    dx.addmm_(g[:, bounds[i]:bounds[i + 1]], WT[:, bounds[i]:bounds[i + 1]].t())
            full = torch.empty(T, V, device=dev, dtype=torch.bfloat16)

            def fwd_slices():                     # chunk GEMMs writing column slices of one [T, V] buffer
                for i in range(n):
                    torch.mm(x, W[bounds[i]:bounds[i + 1]].t(), out=full[:, bounds[i]:bounds[i + 1]])
            dx32 = torch.empty(T, H, device=dev, dtype=torch.float32)

            def dgrad32():                        # chunks accumulated in fp32 (one bf16 rounding at the end)
                torch.mm(g[:, bounds[0]:bounds[1]], WT[:, bounds[0]:bounds[1]].t(), out_dtype=torch.float32, out=dx32)
                for i in range(1, n):
                    torch.addmm(dx32, g[:, bounds[i]:bounds[i + 1]], WT[:, bounds[i]:bounds[i + 1]].t(),
                                out_dtype=torch.float32, out=dx32)
                return dx32.to(torch.bfloat16)
            tf, td, ts, t32 = timed(fwd), timed(dgrad), timed(fwd_slices), timed(dgrad32)
            if n > 1:
                ref = x @ W.t()
                fwd_slices()
                same = bool(torch.equal(full, ref))
            else:
                same = None
            print(json.dumps({"round": rnd, "chunks": n, "fwd_ms": round(tf, 3), "fwd_tflops": round(fl / tf / 1e9, 1),
                              "fwd_slices_ms": round(ts, 3), "fwd_slices_bit_equal_unchunked": same,
                              "dgrad_ms": round(td, 3), "dgrad_tflops": round(fl / td / 1e9, 1),
                              "dgrad_fp32acc_ms": round(t32, 3)}), flush=True)


if __name__ == "__main__":
    main()

"""Data-gradient GEMM layouts of the LLaMA-3-8B SMT step (T = 32768), interleaved rounds in one
process (DVFS noise): g @ W with W [out, in] row-major (hipBLASLt NN) vs g @ Wt^T with a transposed
copy Wt = W^T [in, out] row-major (hipBLASLt TN, the forward's layout). Prints one JSON line per shape."""
import json
import statistics

import torch

T = 32768
SHAPES = {"q/o": (4096, 4096), "k/v": (4096, 1024), "gate/up": (4096, 14336), "down": (14336, 4096),
          "lm_head": (4096, 128256)}


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    torch.manual_seed(0)
    for name, (fin, fout) in SHAPES.items():
        iters = 2 if name == "lm_head" else 10
        x = torch.randn(T, fin, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(fout, fin, device="cuda", dtype=torch.bfloat16) * 0.02
        Wt = W.t().contiguous()
        g = torch.randn(T, fout, device="cuda", dtype=torch.bfloat16)
        fns = {"fwd": lambda: torch.matmul(x, W.t()), "dgrad_nn": lambda: torch.matmul(g, W),
               "dgrad_tn": lambda: torch.matmul(g, Wt.t())}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                res[k].append(timed(f, iters))
        fl = 2.0 * T * fin * fout
        out = {"shape": name, "in": fin, "out": fout}
        for k, v in res.items():
            med = statistics.median(v)
            out[k + "_ms"] = round(med, 3)
            out[k + "_tflops"] = round(fl / med / 1e9, 1)
        same = torch.equal(torch.matmul(g[:256], W), torch.matmul(g[:256], Wt.t()))
        out["dgrad_bitwise_equal_on_256_rows"] = bool(same)
        print(json.dumps(out), flush=True)
        del x, W, Wt, g


if __name__ == "__main__":
    main()

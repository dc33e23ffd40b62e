"""GEMM fusion probe for the LLaMA-3-8B SMT step (T = 32768), interleaved rounds in one process:
  * q/k/v (4096 -> 4096 + 1024 + 1024) and gate/up (4096 -> 2 x 14336) as separate GEMMs vs one GEMM
    over the concatenated weight, forward and data gradient (separate: mm + addmm_ beta=1, as
    dgrad.py does today; joint: one TN GEMM with K = sum of the outputs);
  * down_proj + residual add as mm + add_ vs addmm (beta = 1 epilogue).
Prints one JSON line per case (median ms over 5 interleaved rounds)."""
import json
import statistics

import torch

T = 32768
GROUPS = {"qkv": (4096, (4096, 1024, 1024)), "gate_up": (4096, (14336, 14336))}


def timed(fn, iters=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def bench(fns, flops):
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    res = {k: [] for k in fns}
    for _ in range(5):
        for k, f in fns.items():
            res[k].append(timed(f))
    out = {}
    for k, v in res.items():
        med = statistics.median(v)
        out[k + "_ms"] = round(med, 3)
        out[k + "_tflops"] = round(flops / med / 1e9, 1)
    return out


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for name, (fin, outs) in GROUPS.items():
        x = torch.randn(T, fin, device=dev, dtype=torch.bfloat16)
        Ws = [torch.randn(o, fin, device=dev, dtype=torch.bfloat16) * 0.02 for o in outs]
        Wts = [w.t().contiguous() for w in Ws]
        Wc = torch.cat(Ws, 0)
        Wct = Wc.t().contiguous()                         # [in, sum(out)]
        gs = [torch.randn(T, o, device=dev, dtype=torch.bfloat16) for o in outs]
        gc = torch.cat(gs, 1)

        def fwd_sep():
            for w in Ws:
                torch.matmul(x, w.t())

        def dgrad_sep():
            acc = torch.matmul(gs[0], Wts[0].t())
            for g, wt in zip(gs[1:], Wts[1:]):
                acc.addmm_(g, wt.t())

        fl = 2.0 * T * fin * sum(outs)
        out = {"case": name, "in": fin, "outs": list(outs)}
        out.update(bench({"fwd_sep": fwd_sep, "fwd_joint": lambda: torch.matmul(x, Wc.t()),
                          "dgrad_sep": dgrad_sep, "dgrad_joint": lambda: torch.matmul(gc, Wct.t())}, fl))
        print(json.dumps(out), flush=True)
        del x, Ws, Wts, Wc, Wct, gs, gc

    a = torch.randn(T, 14336, device=dev, dtype=torch.bfloat16)
    Wd = torch.randn(4096, 14336, device=dev, dtype=torch.bfloat16) * 0.02
    r = torch.randn(T, 4096, device=dev, dtype=torch.bfloat16)
    out = {"case": "down+residual"}
    out.update(bench({"mm_then_add": lambda: torch.matmul(a, Wd.t()).add_(r),
                      "addmm": lambda: torch.addmm(r, a, Wd.t())}, 2.0 * T * 14336 * 4096))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

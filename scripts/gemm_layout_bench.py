"""Data-gradient GEMM layouts of the LLaMA-3-8B SMT step (T = 32768), interleaved rounds in one
process (DVFS noise): g @ W with W [out, in] row-major (hipBLASLt NN) vs g @ Wt^T with a transposed
copy Wt = W^T [in, out] row-major (hipBLASLt TN, the forward's layout). Also the forward from the
transposed copy alone (``fwd_from_wt``: F.linear(x, Wt.t()), W a strided view of Wt, hipBLASLt NN), the
"single copy" storage. Prints one JSON line per shape, then one line pricing the
three storages per step of the reference's recompute policy (every decoder linear's forward twice,
its data gradient once; the LM head's forward and data gradient once): W only, W + W^T copy, W^T only."""
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


# per decoder layer: q, o (q/o shape), k, v, gate, up, down; 32 layers
PER_LAYER = {"q/o": 2, "k/v": 2, "gate/up": 2, "down": 1}


def main():
    torch.manual_seed(0)
    rows = {}
    for name, (fin, fout) in SHAPES.items():
        iters = 2 if name == "lm_head" else 10
        x = torch.randn(T, fin, device="cuda", dtype=torch.bfloat16)
        W = torch.randn(fout, fin, device="cuda", dtype=torch.bfloat16) * 0.02
        Wt = W.t().contiguous()
        g = torch.randn(T, fout, device="cuda", dtype=torch.bfloat16)
        fns = {"fwd": lambda: torch.matmul(x, W.t()), "dgrad_nn": lambda: torch.matmul(g, W),
               "dgrad_tn": lambda: torch.matmul(g, Wt.t()),
               "fwd_from_wt": lambda: torch.nn.functional.linear(x, Wt.t())}
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
        rows[name] = out
        del x, W, Wt, g
    cost = {}
    for store, fwd, dg in (("W only", "fwd", "dgrad_nn"), ("W + W^T copy", "fwd", "dgrad_tn"),
                           ("W^T only (single copy)", "fwd_from_wt", "dgrad_tn")):
        ms = 32 * sum(n * (2 * rows[k][fwd + "_ms"] + rows[k][dg + "_ms"]) for k, n in PER_LAYER.items())
        ms += rows["lm_head"][fwd + "_ms"] + rows["lm_head"][dg + "_ms"]
        cost[store] = round(ms, 1)
    print(json.dumps({"recompute_step_gemm_ms": cost, "note": "decoder linears: 2 forwards (forward + "
                      "per-layer recompute) + 1 data gradient; LM head: 1 + 1; weight gradients excluded"}), flush=True)


if __name__ == "__main__":
    main()

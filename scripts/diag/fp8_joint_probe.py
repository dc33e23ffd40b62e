"""fp8 (rowwise-scaled e4m3, torch._scaled_mm -> hipBLASLt) data-gradient GEMMs of the q/k/v and
gate/up groups at T = 32768: one GEMM per member + bf16 adds (the ungrouped path) vs one joint GEMM
over the concatenated output gradients (Fp8Group). Also the forward per member vs over the joint
weight, and the time of the concatenated-row quantisation. Interleaved rounds in one process;
prints one JSON line per case."""
import json
import statistics

import torch

from sparse_matrix_tuning_amd import fp8 as f8

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


def mm(a8, sa, b8, sb_row):
    return torch._scaled_mm(a8, b8.t(), scale_a=sa.view(-1, 1), scale_b=sb_row, out_dtype=torch.bfloat16)


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for name, (fin, outs) in GROUPS.items():
        Ws = [(torch.randn(o, fin, device=dev) * 0.02).bfloat16() for o in outs]
        g = f8.Fp8Group(Ws)
        fws = [f8.Fp8Weight(w, g, i) for i, w in enumerate(Ws)]
        own = [f8.quant_cols_t(w) for w in Ws]                 # standalone transposed copies
        x8, xs = f8.quant_rows(torch.randn(T, fin, device=dev).bfloat16())
        gos = [torch.randn(T, o, device=dev).bfloat16() for o in outs]
        q_sep = [f8.quant_rows(go) for go in gos]
        q_cat = f8.quant_rows_cat(gos)
        w8c, swc = f8.quant_rows(torch.cat(Ws, 0))

        def dgrad_sep():
            acc = mm(q_sep[0][0], q_sep[0][1], own[0][0], own[0][1].view(1, -1))
            for (a8, sa), (wt8, swt) in zip(q_sep[1:], own[1:]):
                acc = acc + mm(a8, sa, wt8, swt.view(1, -1))

        def fwd_sep():
            for fw in fws:
                mm(x8, xs, fw.w8, fw.sw_row)

        fns = {"dgrad_sep": dgrad_sep,
               "dgrad_joint": lambda: mm(q_cat[0], q_cat[1], g.wt8, g.swt_row),
               "fwd_sep": fwd_sep,
               "fwd_joint": lambda: mm(x8, xs, w8c, swc.view(1, -1)),
               "quant_sep": lambda: [f8.quant_rows(go) for go in gos],
               "quant_cat": lambda: f8.quant_rows_cat(gos)}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(5):
            for k, f in fns.items():
                res[k].append(timed(f))
        fl = 2.0 * T * fin * sum(outs)
        out = {"case": name, "in": fin, "outs": list(outs)}
        for k, v in res.items():
            med = statistics.median(v)
            out[k + "_ms"] = round(med, 3)
            if not k.startswith("quant"):
                out[k + "_tflops"] = round(fl / med / 1e9, 1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

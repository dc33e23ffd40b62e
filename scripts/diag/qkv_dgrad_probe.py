"""The q/k/v data gradient at the bench shape (T = 32768, hidden 4096, q 4096 / k, v 1024 outputs):
three GEMMs accumulating through the C operand (what dgrad.py issues: v, then k and q with
addmm_, on the transposed copies as TN products) vs one joint GEMM over [dq | dk | dv] (T x 6144)
and the joint transposed copy (4096 x 6144). Interleaved rounds, HIP events."""
import argparse
import json

import torch


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--outs", default="4096,1024,1024", help="consumer widths (gate/up: 14336,14336)")
    outs = tuple(int(v) for v in ap.parse_args().outs.split(","))
    dev = torch.device("cuda", 0)
    T, H = 32768, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    J = (torch.randn(T, sum(outs), device=dev, generator=g) * 0.01).bfloat16()
    Wt = (torch.randn(H, sum(outs), device=dev, generator=g) * 0.02).bfloat16()      # joint W^T [in, out]
    offs = [sum(outs[:i]) for i in range(len(outs) + 1)]
    n = len(outs)
    gs = [J[:, offs[i]:offs[i + 1]].contiguous() for i in range(n)]                 # today's separate grads
    gv = [J[:, offs[i]:offs[i + 1]] for i in range(n)]                              # views of J
    wts = [Wt[:, offs[i]:offs[i + 1]].contiguous() for i in range(n)]               # today's separate copies
    mats = [w.t() for w in wts]                                                     # (W^T)^T: TN
    mats_j = [Wt[:, offs[i]:offs[i + 1]].t() for i in range(n)]

    def sep(gl, ml):                                # backward order: the last consumer first
        buf = torch.matmul(gl[-1], ml[-1])
        for i in range(n - 2, -1, -1):
            buf.addmm_(gl[i], ml[i])
        return buf

    def joint():
        return torch.matmul(J, Wt.t())

    ref = sep(gs, mats).float()
    res = {"outs": list(outs), "joint_rel": ((joint().float() - ref).norm() / ref.norm()).item()}
    for r in range(3):
        res[f"sep_ms_{r}"] = round(timeit(lambda: sep(gs, mats)), 4)
        res[f"sep_views_ms_{r}"] = round(timeit(lambda: sep(gv, mats_j)), 4)
        res[f"joint_ms_{r}"] = round(timeit(joint), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""Where does the one-wave-per-SIMD dQ kernel (SMT_ATTN_DQ=2) differ from the lean one? Runs the
attention backward of one test case once per kernel (the choice is read once per process, so each in
a child process), then prints the difference by batch / head / query row and by row position inside
the kernel's 256-row block (wave = row // 64, 32-row block = row // 32 % 2, lane = row % 32).

    python scripts/diag/dq_dual_diag.py [--b 2 --hq 8 --hkv 2 --s 256]"""
import argparse
import os
import subprocess
import sys
import tempfile

import torch


def child(path, B, Hq, Hkv, S):
    sys.path.insert(0, os.getcwd())
    from sparse_matrix_tuning_amd.fused_llama import flash_attention
    dev = torch.device("cuda", 0)
    torch.manual_seed(S + Hq)
    mk = lambda H: torch.randn(B, S, H, 128, device=dev).bfloat16().transpose(1, 2).requires_grad_(True)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    g = torch.randn(B, S, Hq, 128, device=dev).bfloat16()
    o = flash_attention(q, k, v)
    o.backward(g)
    torch.cuda.synchronize()
    torch.save({"dq": q.grad.float().cpu(), "dk": k.grad.float().cpu(), "dv": v.grad.float().cpu()}, path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=2)
    ap.add_argument("--hq", type=int, default=8)
    ap.add_argument("--hkv", type=int, default=2)
    ap.add_argument("--s", type=int, default=256)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        return child(a.child, a.b, a.hq, a.hkv, a.s)
    d = tempfile.mkdtemp()
    out = {}
    for impl in ("1", "2"):
        p = os.path.join(d, f"dq{impl}.pt")
        env = dict(os.environ, SMT_ATTN_DQ=impl)
        subprocess.run([sys.executable, __file__, "--child", p, "--b", str(a.b), "--hq", str(a.hq), "--hkv",
                        str(a.hkv), "--s", str(a.s)], env=env, check=True, timeout=300)
        out[impl] = torch.load(p, weights_only=True)
    for name in ("dk", "dv"):
        print(name, "max |dual - lean|", (out["1"][name] - out["2"][name]).abs().max().item())
    lean, dual = out["1"]["dq"], out["2"]["dq"]                 # [B, Hq, S, D]
    diff = (dual - lean).abs()
    rel_row = diff.norm(dim=-1) / lean.norm(dim=-1).clamp_min(1e-30)     # [B, Hq, S]
    print("dq overall rel", (diff.norm() / lean.norm()).item())
    bad = rel_row > 1e-2
    print("bad rows", int(bad.sum()), "of", bad.numel())
    print("by b", bad.sum(dim=(1, 2)).tolist(), "by h", bad.sum(dim=(0, 2)).tolist())
    rows = torch.arange(a.s)
    r = bad.sum(dim=(0, 1))
    for lbl, key in (("row % 256 // 64 (wave)", rows % 256 // 64), ("row // 32 % 2 (block)", rows // 32 % 2),
                     ("row % 32 (lane)", rows % 32), ("row // 256 (qb)", rows // 256)):
        n = int(key.max()) + 1
        print(lbl, [int(r[key == i].sum()) for i in range(n)])
    print("first bad rows", bad.nonzero()[:20].tolist())
    idx = rel_row.flatten().topk(10).indices
    coords = torch.stack(torch.unravel_index(idx, rel_row.shape), 1).tolist()
    print("worst rows", [(c, round(rel_row[tuple(c)].item(), 4)) for c in coords])
    # columns (features): is the error confined to some dt / g?
    fd = diff.norm(dim=(0, 1, 2))
    print("by feature group of 8", [round(x, 3) for x in fd.view(16, 8).norm(dim=1).tolist()])


if __name__ == "__main__":
    main()

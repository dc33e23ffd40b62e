"""Tune hipBLASLt / rocBLAS solutions (PyTorch TunableOp) for the GEMMs of the LLaMA-3-8B SMT step,
called exactly as the step calls them (same torch ops, layouts and leading dimensions, so the
TunableOp keys match): the forward F.linear(x, W) of every linear and the data gradient
g @ (W^T)^T on the engine's transposed copies (engine.FrozenLinearFn). Run with
    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=<csv> \
        python scripts/tune_gemms.py
(rows already in <csv> are kept; TunableOp writes the file at exit)."""
import torch
import torch.nn.functional as F

T = 16 * 2048
H, I, KV, V = 4096, 14336, 1024, 128256
SHAPES = [(H, H), (H, KV), (H, I), (I, H), (H, V)]      # (in, out): q/o, k/v, gate/up, down, lm_head
JOINT = [(H, H + 2 * KV)]                                 # the joint q/k/v data gradient (dgrad.py)


def main():
    dev = torch.device("cuda", 0)
    for fin, fout in SHAPES:
        x = torch.randn(T, fin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(fout, fin, device=dev, dtype=torch.bfloat16) * 0.02
        g = torch.randn(T, fout, device=dev, dtype=torch.bfloat16)
        wt = w.t().contiguous()
        F.linear(x, w)                       # forward
        torch.matmul(g, wt.t())              # data gradient on the transposed copy
        torch.cuda.synchronize()
        print(f"tuned in={fin} out={fout}", flush=True)
        del x, w, g, wt
    for fin, fout in JOINT:
        g = torch.randn(T, fout, device=dev, dtype=torch.bfloat16)
        wt = torch.randn(fin, fout, device=dev, dtype=torch.bfloat16) * 0.02
        torch.matmul(g, wt.t())              # data gradient only
        torch.cuda.synchronize()
        print(f"tuned joint dgrad in={fin} out={fout}", flush=True)
        del g, wt


if __name__ == "__main__":
    main()

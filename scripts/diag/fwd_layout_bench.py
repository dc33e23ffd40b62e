"""Forward GEMM layout of the bench step's frozen linears (T = 32768): y = x @ W^T as F.linear on
W [out, in] (hipBLASLt NT) vs torch.mm on the transposed copy the engine already keeps for the data
gradient, W^T [in, out] (NN). Interleaved rounds, HIP events; results compared bit for bit."""
import json

import torch
import torch.nn.functional as F


def timed(fn, iters=10):
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
    T = 32768
    dev = torch.device("cuda")
    torch.manual_seed(0)
    shapes = [("q/o", 4096, 4096), ("k/v", 4096, 1024), ("gate/up", 4096, 14336), ("down", 14336, 4096),
              ("lm_head", 4096, 128256)]
    for rnd in range(2):
        for name, fin, fout in shapes:
            x = torch.randn(T, fin, device=dev, dtype=torch.bfloat16)
            W = (torch.randn(fout, fin, device=dev) * 0.02).bfloat16()
            Wt = W.t().contiguous()
            a = timed(lambda: F.linear(x, W))
            b = timed(lambda: torch.mm(x, Wt))
            same = bool(torch.equal(F.linear(x, W), torch.mm(x, Wt)))
            fl = 2.0 * T * fin * fout
            print(json.dumps({"round": rnd, "shape": name, "in": fin, "out": fout, "nt_ms": round(a, 3),
                              "nt_tflops": round(fl / a / 1e9, 1), "nn_ms": round(b, 3),
                              "nn_tflops": round(fl / b / 1e9, 1), "bit_equal": same}), flush=True)
            del x, W, Wt


if __name__ == "__main__":
    main()

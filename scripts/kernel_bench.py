"""Micro-benchmark of the SMT HIP kernels at LLaMA-3-8B shapes (HIP events on the launch stream)."""
import argparse
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(iters):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32768)
    ap.add_argument("--out", type=int, default=14336)
    ap.add_argument("--inp", type=int, default=4096)
    ap.add_argument("--tiles", type=int, nargs="*", default=[1, 8, 27, 64, 128])
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T = args.T
    g = torch.randn(T, args.out, device=dev).bfloat16()
    x = torch.randn(T, args.inp, device=dev).bfloat16()
    rb, cb = args.out // 256, args.inp // 256
    res = []
    for n in args.tiles:
        gen = torch.Generator().manual_seed(n)
        perm = torch.randperm(rb * cb, generator=gen)[:n].tolist()
        tiles = [(p // cb, p % cb) for p in perm]
        rc = _hip.tile_table(tiles, dev)
        out = torch.empty(n * 256, 256, device=dev)
        ws = torch.empty(_hip.wgrad_workspace_bytes(T, n), dtype=torch.uint8, device=dev)
        lib = _hip.load()
        st = torch.cuda.current_stream().cuda_stream

        def run():
            rc_ = lib.smt_tile_wgrad(g.data_ptr(), g.stride(0), x.data_ptr(), x.stride(0), T, rc.data_ptr(), n,
                                     out.data_ptr(), 1, 0, ws.data_ptr(), ws.numel(), st)
            assert rc_ == 0
        t = timeit(run)
        flops = 2.0 * T * 65536 * n
        bytes_alg = n * (T * 256 * 2 * 2 + 65536 * 4)
        res.append(dict(tiles=n, ms=t * 1e3, tflops=flops / t / 1e12, gbs=bytes_alg / t / 1e9,
                        ws_mb=ws.numel() / 2**20))
        print(json.dumps(res[-1]), flush=True)
    # gather / scatter / adamw
    n = 872
    W = torch.randn(14336, 4096, device=dev).bfloat16()
    perm = torch.randperm(56 * 16)[:n % (56 * 16)].tolist()


if __name__ == "__main__":
    main()

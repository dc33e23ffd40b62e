"""Micro-benchmark of smt_tile_wgrad at LLaMA-3-8B shapes (HIP events on the launch stream).

Patterns: 'random' tiles over the [out/256 x in/256] block grid, and 'clustered' tiles confined to
4 column blocks (selections concentrate). Reports algorithmic GB/s (each tile's two
T x 256 bf16 slices + its fp32 output) and the MFMA rate."""
import argparse
import json
import os
import sys

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


def _split(T, n):
    ws = _hip.wgrad_workspace_bytes(T, n)
    return ws // (n * 65536 * 4) if ws else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32768)
    ap.add_argument("--out", type=int, default=14336)
    ap.add_argument("--inp", type=int, default=4096)
    ap.add_argument("--tiles", type=int, nargs="*", default=[1, 8, 27, 64, 128, 256])
    ap.add_argument("--patterns", nargs="*", default=["random", "clustered"])
    ap.add_argument("--orders", nargs="*", type=int, default=[0, 1])
    ap.add_argument("--tag", default="default")
    ap.add_argument("--mx", action="store_true", help="time smt_mx_quant_cols + smt_tile_wgrad_mx instead")
    ap.add_argument("--xblock", action="store_true",
                    help="x from the block-major copy linearZ saves (smt_colblock_gather), as in training")
    args = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    T = args.T
    g = torch.randn(T, args.out, device=dev).bfloat16()
    x = torch.randn(T, args.inp, device=dev).bfloat16()
    rb, cb = args.out // 256, args.inp // 256
    lib = _hip.load()
    for pattern in args.patterns:
        for n in args.tiles:
          for use_order in [bool(o) for o in args.orders]:
            gen = torch.Generator().manual_seed(n)
            if pattern == "random":
                perm = torch.randperm(rb * cb, generator=gen)[:n].tolist()
                tiles = [(p // cb, p % cb) for p in perm]
            else:
                cells = [(r, c) for c in range(4) for r in range(rb)]
                perm = torch.randperm(len(cells), generator=gen)[:n].tolist()
                tiles = [cells[p] for p in perm]
            n = len(tiles)
            rc = _hip.tile_table(tiles, dev)
            order = _hip.order_table(tiles, dev)
            out = torch.empty(n * 256, 256, device=dev)
            wsb = _hip.wgrad_workspace_bytes(T, n)
            ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
            st = torch.cuda.current_stream().cuda_stream

            if args.mx:
                rbs = sorted({r for r, _ in tiles})
                cbs = sorted({c for _, c in tiles})
                rb_dev = torch.tensor(rbs, dtype=torch.int32, device=dev)
                cb_dev = torch.tensor(cbs, dtype=torch.int32, device=dev)
                qg = _hip.mx_quant_cols(g, rb_dev)
                qx = _hip.mx_quant_cols(x, cb_dev)
                prc = _hip.tile_table([(rbs.index(r), cbs.index(c)) for r, c in tiles], dev)
                t_q = timeit(lambda: (_hip.mx_quant_cols(g, rb_dev), _hip.mx_quant_cols(x, cb_dev)))
                t = timeit(lambda: _hip.tile_wgrad_mx(qg, qx, prc, out, order=order if use_order else None))
                flops = 2.0 * T * 65536 * n
                bytes_alg = n * (T * 256 * 2 + 65536 * 4)
                q_bytes = (len(rbs) + len(cbs)) * T * 256 * (2 + 1 + 1 / 32)
                print(json.dumps(dict(tag="mx", pattern=pattern, order=use_order, tiles=n, us=round(t * 1e6, 1),
                                      alg_tbs=round(bytes_alg / t / 1e12, 3), tflops=round(flops / t / 1e12, 1),
                                      quant_us=round(t_q * 1e6, 1), quant_tbs=round(q_bytes / t_q / 1e12, 3))), flush=True)
                continue

            xs, ldx, xbs, rc_x = x, x.stride(0), 256, rc
            if args.xblock:
                cbs = sorted({c for _, c in tiles})
                xs = _hip.colblock_gather(x, torch.tensor(cbs, dtype=torch.int32, device=dev))
                ldx, xbs = 256, T * 256
                rc_x = _hip.tile_table([(r, cbs.index(c)) for r, c in tiles], dev)

            def run():
                assert lib.smt_tile_wgrad(g.data_ptr(), g.stride(0), xs.data_ptr(), ldx, xbs, T, rc_x.data_ptr(),
                                          order.data_ptr() if use_order else None, n,
                                          out.data_ptr(), 1, 0, ws.data_ptr(), wsb, st) == 0
            t = timeit(run)
            flops = 2.0 * T * 65536 * n
            bytes_alg = n * (T * 256 * 2 * 2 + 65536 * 4)
            uniq = (len({r for r, _ in tiles}) + len({c for _, c in tiles})) * T * 512 + n * 65536 * 4
            print(json.dumps(dict(tag=args.tag + ("+xblock" if args.xblock else ""), pattern=pattern, order=use_order, tiles=n, S=_split(T, n), us=round(t * 1e6, 1), alg_tbs=round(bytes_alg / t / 1e12, 3),
                                  unique_slice_tbs=round(uniq / t / 1e12, 3), tflops=round(flops / t / 1e12, 1),
                                  ws_mb=round(wsb / 2**20, 1))), flush=True)


if __name__ == "__main__":
    main()

"""Micro-benchmark of the batched tile wgrad (smt_tile_wgrad_batch) on launches shaped like the
bench's: the SMT linears of LLaMA-3-8B decoder layers with ~8.4 spread tiles each (872 tiles over
104 modules), x as the block-major column-block copy linearZ saves, batches of >= 48 tiles in
backward module order (down, up, gate, o, v, k, q), T = 32768, fp32 outputs (the engine's sink).

Prints one JSON line per run: average launch time (HIP events on the launch stream), distinct and
per-tile operand bytes per launch and their rates, and a checksum of the outputs (kernel variants
must give bit-identical tiles). Compare variants with SMT_HIP_LIB=<variant .so>."""
import argparse
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402

DTYPE = torch.bfloat16

# (name, out_features, in_features) of one LLaMA-3-8B decoder layer, in backward order
LAYER = [("down", 4096, 14336), ("up", 14336, 4096), ("gate", 14336, 4096), ("o", 4096, 4096),
         ("v", 1024, 4096), ("k", 1024, 4096), ("q", 4096, 4096)]


def make_batches(T, tiles_per_module, batch_tiles, n_layers, dev, gen, pattern="spread", g_width=None):
    """Lists of modules (g, x_packed, out, tiles in packed coordinates, distinct-slice keys).
    pattern "rowblock": every tile of a module in ONE row block (one shared g slice, distinct x
    slices), the g row width ``g_width`` (256: contiguous 512-B rows, else a strided column slice)."""
    batches, cur, cur_n = [], [], 0
    for layer in range(n_layers):
        for name, out_f, in_f in LAYER:
            if g_width:
                out_f = g_width
            rb, cb = out_f // 256, in_f // 256
            n = tiles_per_module
            if pattern == "rowblock":
                r0 = int(torch.randint(rb, (1,), generator=gen))
                rc = [(r0, c) for c in torch.randperm(cb, generator=gen)[:n].tolist()]
            else:
                perm = torch.randperm(rb * cb, generator=gen)[:n].tolist()
                rc = [(p // cb, p % cb) for p in perm]
            cols = sorted({c for _r, c in rc})
            pos = {c: i for i, c in enumerate(cols)}
            g = torch.randn(T, out_f, device=dev, dtype=DTYPE)      # this module's output gradient
            x = torch.randn(len(cols), T, 256, device=dev, dtype=DTYPE)   # packed column blocks
            out = torch.zeros(n * 256, 256, device=dev, dtype=torch.float32)
            ktiles = [(r, pos[c]) for r, c in rc]
            keys = {("g", g.data_ptr(), r) for r, _c in rc} | {("x", x.data_ptr(), c) for _r, c in ktiles}
            cur.append((g, x, out, ktiles, keys))
            cur_n += n
            if cur_n >= batch_tiles or len(cur) == _hip.WGRAD_MAX_MODULES:
                batches.append(cur)
                cur, cur_n = [], 0
    if cur:
        batches.append(cur)
    return batches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32768)
    ap.add_argument("--tiles-per-module", type=int, default=8)
    ap.add_argument("--batch-tiles", type=int, default=48)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--pattern", default="spread", choices=("spread", "rowblock"))
    ap.add_argument("--g-width", type=int, default=None, help="override every module's out features")
    ap.add_argument("--seq-len", type=int, default=0, help="reference rounding: T / seq_len samples")
    ap.add_argument("--tag", default=os.environ.get("SMT_HIP_LIB", "default"))
    ap.add_argument("--dtype", default="bf16", choices=("bf16", "fp16", "fp32"),
                    help="operand dtype (the reference's --dtype; fp32 runs wgrad_f32_kernel)")
    args = ap.parse_args()
    global DTYPE
    DTYPE = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    dev = torch.device("cuda")
    gen = torch.Generator().manual_seed(1234)
    torch.manual_seed(0)
    batches = make_batches(args.T, args.tiles_per_module, args.batch_tiles, args.layers, dev, gen, args.pattern,
                           args.g_width)
    prepared = []
    for mods in batches:
        tab, order = _hip.wgrad_batch_table([m[3] for m in mods], dev)
        items = [(m[0], m[1], m[2], False) for m in mods]
        n = sum(len(m[3]) for m in mods)
        keys = set().union(*[m[4] for m in mods])
        eb = torch.tensor([], dtype=DTYPE).element_size()
        distinct = len(keys) * args.T * 256 * eb + n * 65536 * 4
        per_tile = n * (2 * args.T * 256 * eb + 65536 * 4)
        prepared.append((items, tab, order, n, distinct, per_tile))

    def run_all():
        for items, tab, order, *_ in prepared:
            _hip.tile_wgrad_batch(items, tab, order, seq_len=args.seq_len or None)

    run_all()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in prepared]
    times = [0.0] * len(prepared)
    for _ in range(args.iters):
        for i, (items, tab, order, *_r) in enumerate(prepared):
            ev[i][0].record(s)
            _hip.tile_wgrad_batch(items, tab, order, seq_len=args.seq_len or None)
            ev[i][1].record(s)
        torch.cuda.synchronize()
        for i in range(len(prepared)):
            times[i] += ev[i][0].elapsed_time(ev[i][1]) * 1e-3
    h = hashlib.sha256()
    for mods in batches:
        for m in mods:
            h.update(m[2].cpu().numpy().tobytes())
    t = sum(times) / args.iters
    launches = len(prepared)
    distinct = sum(p[4] for p in prepared)
    per_tile = sum(p[5] for p in prepared)
    tiles = sum(p[3] for p in prepared)
    print(json.dumps({"tag": os.path.basename(args.tag), "dtype": args.dtype, "env": {k: v for k, v in os.environ.items()
                                                                    if k.startswith("SMT_WGRAD")},
                      "seq_len": args.seq_len, "T": args.T, "launches": launches,
                      "tiles_per_launch": round(tiles / launches, 1),
                      "avg_launch_us": round(t / launches * 1e6, 2),
                      "distinct_gb_per_launch": round(distinct / launches / 1e9, 4),
                      "distinct_tbs": round(distinct / t / 1e12, 3), "frac_distinct": round(distinct / t / 8e12, 4),
                      "per_tile_tbs": round(per_tile / t / 1e12, 3),
                      "mfma_tflops": round(tiles * 2.0 * args.T * 65536 / t / 1e12, 1),
                      "checksum": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()

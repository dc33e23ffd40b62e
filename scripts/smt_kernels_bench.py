"""Every HBM-bound kernel of the SMT path at the bench's sizes (LLaMA-3-8B, T = B*S = 32768, the
spread selection's ~8.5 tiles per module), timed with HIP events on the launch stream, against the
8 TB/s HBM roof with each kernel's algorithmic bytes. One JSON line per kernel.

    python scripts/smt_kernels_bench.py > profiles/r02_smt_kernels.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402

DEV = torch.device("cuda", 0)
PEAK = 8000.0
T = 32768


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


def report(name, unit, nbytes, seconds, **kw):
    gbs = nbytes / seconds / 1e9
    print(json.dumps(dict(kernel=name, unit=unit, bytes=int(nbytes), us=round(seconds * 1e6, 1),
                          gb_s=round(gbs, 1), frac_of_8tbs=round(gbs / PEAK, 3), **kw)), flush=True)


def main():
    torch.manual_seed(0)
    gen = torch.Generator().manual_seed(0)
    # -- warm-up harvest: fp32 += bf16 over one decoder layer's q/k/v + MLP keys (fine_tune.py:724-741)
    shapes = [(4096, 4096), (1024, 4096), (1024, 4096), (14336, 4096), (14336, 4096), (4096, 14336)]
    accs = [torch.zeros(s, dtype=torch.float32, device=DEV) for s in shapes]
    grads = [torch.randn(s, device=DEV).bfloat16() for s in shapes]
    elems = sum(a.numel() for a in accs)
    plan = _hip.AccumulatePlan(list(zip(accs, grads)), False)
    report("grad_accumulate_kernel", "one layer's harvested keys (fp32 acc += bf16 grad)", elems * 10,
           timeit(plan.launch), elements=elems)
    # -- block scores over the same keys (smt_helper.py:67-78): 4 B per element read
    t = timeit(lambda: _hip.block_scores(accs, [(r // 256, c // 256) for r, c in shapes], _hip.SCORE_ABS_MEAN))
    report("block_score_kernel", "one layer's keys, abs_mean", elems * 4, t, elements=elems)
    del accs, grads, plan
    # -- sparse AdamW over the bench's 872 tiles (57.1 M params): 32 B / param
    n = 872
    grad = torch.randn(n * 65536, device=DEV) * 1e-3
    master = torch.randn(n * 65536, device=DEV)
    m, v = torch.zeros_like(master), torch.zeros_like(master)
    param = master.bfloat16()
    W = torch.zeros(14336, 4096, dtype=torch.bfloat16, device=DEV)
    tiles = [(i % 56, (i * 7) % 16) for i in range(n)]
    descs = _hip.tile_descs([(W, r, c, i * 65536) for i, (r, c) in enumerate(tiles)], DEV)
    norm = _hip.sq_norm(grad)
    args = _hip.AdamWArgs(lr=1e-5, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.0, bias_correction1=0.1,
                          bias_correction2=0.05, max_grad_norm=1.0, grad_scale=1.0, mode=_hip.ADAM_DEEPSPEED,
                          grad_dtype=1)
    t = timeit(lambda: _hip.adamw_step(grad, master, m, v, param, args, tiles=descs, n_tiles=n, grad_sq_norm=norm))
    report("adamw_tiles_kernel", "872 tiles, fp32 grad (the engine's sink)", n * 65536 * 34, t, params=n * 65536,
           bytes_note="fp32 grad 4 + master/m/v read+write 24 + bf16 param 2 + bf16 W scatter 2 + 2 (tile out)")
    t = timeit(lambda: _hip.sq_norm(grad))
    report("sq_norm_*", "872 tiles' fp32 gradient", n * 65536 * 4, t)
    del grad, master, m, v, param, descs
    # -- tile gather / scatter of one module's 8 tiles (smt.py:317-341)
    rc = _hip.tile_table(tiles[:8], DEV)
    buf = torch.empty(8 * 256, 256, dtype=torch.bfloat16, device=DEV)
    t = timeit(lambda: _hip.tile_gather(W, rc, buf))
    report("tile_copy_kernel<gather>", "8 tiles bf16", 8 * 65536 * 4, t)
    # -- linearZ's saved input column blocks: 8 of 16 blocks of a [T, 4096] input, block-major
    x = torch.randn(T, 4096, device=DEV).bfloat16()
    cbs = torch.tensor([0, 2, 3, 5, 8, 11, 12, 15], dtype=torch.int32, device=DEV)
    t = timeit(lambda: _hip.colblock_gather(x, cbs))
    report("colblock_gather_kernel", "8 column blocks of a [32768, 4096] input", T * 8 * 256 * 4, t)
    # -- MX quantiser (fp8 path): 8 column blocks
    t = timeit(lambda: _hip.mx_quant_cols(x, cbs))
    report("mx_quant_cols_kernel", "8 column blocks of a [32768, 4096] input", T * 8 * 256 * (2 + 1 + 1 / 32), t)
    # -- channel path (config 4 shapes): activation harvest and channel scores, [16, 2048, 5120]
    xa = torch.randn(16, 2048, 5120, device=DEV).bfloat16()
    acc = torch.zeros(16, 2048, 5120, device=DEV)
    t = timeit(lambda: _hip.act_accumulate(xa, acc, assign=False))
    report("act_accumulate_kernel", "[16, 2048, 5120] bf16 into fp32", xa.numel() * 10, t)
    t = timeit(lambda: _hip.channel_scores(acc, _hip.SCORE_MEAN_ABS))
    report("channel_score_kernel", "[16, 2048, 5120] fp32", acc.numel() * 4, t)
    idx = torch.randperm(5120, generator=gen)[:1713].sort().values.tolist()
    cols = _hip.index_table(idx, DEV)
    t = timeit(lambda: _hip.column_gather(xa.view(-1, 5120), cols, 1713, 1792))
    report("column_gather_kernel", "1713 of 5120 channels, T = 32768", T * (1713 * 2 + 1792 * 2), t)


if __name__ == "__main__":
    main()

"""Per-tile phase timeline of the forward attention loop (FwdLean) and per-slice timeline of the dK/dV loop (DkvLean) from the shader-clock stamps of a
diagnostic build (SMT_ATTN_STAMPS=1, scripts/diag/build_variant.py; load it with SMT_HIP_LIB): every
64th workgroup's waves record s_memtime at each K/V tile's start, after its compute (QK^T, softmax,
PV issued), after the DMA wait for the next tile, and after the barrier. Prints one JSON summary.

    python scripts/diag/build_variant.py stamps -DSMT_ATTN_STAMPS=1
    SMT_HIP_LIB=scripts/diag/_variants/libsmt_hip_stamps.so python scripts/diag/attn_stamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402
from sparse_matrix_tuning_amd.fused_llama import flash_attention  # noqa: E402


def main():
    B, Hq, Hkv, S, D = 16, 32, 8, 2048, 128
    torch.manual_seed(0)
    mk = lambda H: torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16).transpose(1, 2)
    q, k, v = mk(Hq), mk(Hkv), mk(Hkv)
    for _ in range(3):
        flash_attention(q, k, v)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    flash_attention(q, k, v)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    lib = _hip.load()
    fn = lib.smt_attn_debug_fwd_stamps
    fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    buf = np.zeros((256, 4, 32, 4), dtype=np.uint64)
    rc = fn(buf.ctypes.data, buf.nbytes)
    if rc:
        raise RuntimeError(lib.smt_attn_last_error().decode())
    rows = []
    spans = []
    for blk in range(buf.shape[0]):
        for w in range(4):
            st = buf[blk, w]
            n = int((st[:, 0] > 0).sum())
            if n < 3:
                continue
            st = st[:n].astype(np.int64)
            spans.append(int(st[-1, 3] - st[0, 0]))
            for t in range(1, n - 1):                    # interior tiles (not the first / the diagonal one)
                rows.append((st[t, 1] - st[t, 0], st[t, 2] - st[t, 1], st[t, 3] - st[t, 2], st[t + 1, 0] - st[t, 0]))
    a = np.array(rows, dtype=np.float64)
    med = np.median(a, axis=0)
    mean = a.mean(axis=0)
    out = {"shape": f"B{B} Hq{Hq} Hkv{Hkv} S{S} D{D}", "forward_ms": round(ms, 3), "interior_tiles": len(rows),
           "median_cycles": {"compute": med[0], "dma_wait": med[1], "barrier": med[2], "tile": med[3]},
           "mean_cycles": {"compute": round(mean[0], 1), "dma_wait": round(mean[1], 1), "barrier": round(mean[2], 1),
                           "tile": round(mean[3], 1)},
           "share_of_tile": {"compute": round(mean[0] / mean[3], 3), "dma_wait": round(mean[1] / mean[3], 3),
                             "barrier": round(mean[2] / mean[3], 3)},
           "mfma_cycles_per_tile_per_wave": 32 * 32,
           "block_span_cycles_median": float(np.median(spans)) if spans else None}
    print(json.dumps(out), flush=True)

    # dK/dV kernel: per 32-row query slice of a wave (SMT_ATTN_STAMPS also stamps DkvLean)
    qg, kg, vg = (t.detach().clone().requires_grad_(True) for t in (q, k, v))
    g = torch.randn(B, S, Hq, D, device="cuda", dtype=torch.bfloat16)
    for _ in range(2):
        flash_attention(qg, kg, vg).backward(g)
    torch.cuda.synchronize()
    fn2 = lib.smt_attn_debug_dkv_stamps
    fn2.restype, fn2.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]
    dbuf = np.zeros((256, 8, 64, 5), dtype=np.uint64)
    if fn2(dbuf.ctypes.data, dbuf.nbytes):
        raise RuntimeError(lib.smt_attn_last_error().decode())
    rows = []
    for blk in range(dbuf.shape[0]):
        for w in range(8):
            st = dbuf[blk, w].astype(np.int64)
            n = int((st[:, 0] > 0).sum())
            for i in range(n - 1):
                if st[i, 1] == st[i, 0]:                 # a slice this wave skips (above its diagonal)
                    continue
                rows.append((st[i, 1] - st[i, 0], st[i, 2] - st[i, 1], st[i, 3] - st[i, 2], st[i, 4] - st[i, 3],
                             st[i + 1, 0] - st[i, 0]))
    a = np.array(rows, dtype=np.float64)
    mean = a.mean(axis=0)
    print(json.dumps({"kernel": "attn_dkdv_kernel (DkvLean)", "slices": len(rows),
                      "median_cycles": dict(zip(("s_dp", "dv_dk", "dma_wait", "barrier", "slice"),
                                                np.median(a, axis=0).tolist())),
                      "share_of_slice": dict(zip(("s_dp", "dv_dk", "dma_wait", "barrier"),
                                                 [round(x / mean[4], 3) for x in mean[:4]])),
                      "mfma_cycles_per_slice_per_wave": 32 * 32}), flush=True)


if __name__ == "__main__":
    main()

"""Time smt_column_gather at the config-4 shape (1713 of 5120 channels, T = 32768) for the kernel
SMT_CGATHER_IMPL selects (read once per process), and check it against a torch gather.

    SMT_CGATHER_IMPL=2 python scripts/diag/cgather_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from sparse_matrix_tuning_amd import _hip  # noqa: E402

DEV = torch.device("cuda", 0)


def main():
    gen = torch.Generator().manual_seed(0)
    T, n_in, k, pad = 32768, 5120, 1713, 1792
    x = torch.randn(T, n_in, device=DEV).bfloat16()
    idx = torch.randperm(n_in, generator=gen)[:k].sort().values
    cols = _hip.index_table(idx.tolist(), DEV)
    out = _hip.column_gather(x, cols, k, pad)
    want = torch.zeros(T, pad, dtype=torch.bfloat16, device=DEV)
    want[:, :k] = x[:, idx.to(DEV)]
    exact = bool(torch.equal(out, want))
    for _ in range(3):
        _hip.column_gather(x, cols, k, pad)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        _hip.column_gather(x, cols, k, pad)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    traffic = T * (n_in * 2 + pad * 2)
    print(json.dumps({"impl": os.environ.get("SMT_CGATHER_IMPL", "default"), "us": round(us, 1), "exact": exact,
                      "traffic_tb_s": round(traffic / us / 1e6, 2),
                      "gathered_frac_of_8tbs": round(T * (k * 2 + pad * 2) / us / 1e6 / 8.0, 3)}), flush=True)


if __name__ == "__main__":
    main()

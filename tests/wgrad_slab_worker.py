"""Worker of tests/test_gpu_wgrad_full.py::test_reference_rounding_bf16_slabs_bit_identical (a child
process, so that SMT_WGRAD_SLAB16 -- read once per process by libsmt_hip.so -- can differ from the
parent's). Writes the reference-rounding tile gradients of a few bench-shaped cases (torch.save)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cases():
    from tests.test_gpu_wgrad_full import SHAPES, S, _operands, _tiles
    from sparse_matrix_tuning_amd import _hip
    dev = torch.device("cuda", 0)
    out = {}
    for module, n in (("down_proj", 8), ("q_proj", 27), ("gate_proj", 67)):
        out_f, in_f = SHAPES[module]
        go, x = _operands(out_f, in_f, seed=300 + n)
        tiles = _tiles(out_f, in_f, n, seed=n)
        o = torch.empty(n * 256, 256, dtype=torch.float32, device=dev)
        _hip.tile_wgrad(go, x, _hip.tile_table(tiles, dev), o, order=_hip.order_table(tiles, dev), seq_len=S)
        out[f"{module}-{n}"] = o.cpu()
    return out


if __name__ == "__main__":
    torch.save(cases(), sys.argv[1])

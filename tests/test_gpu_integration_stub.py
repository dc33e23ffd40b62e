"""The reference-side ctypes binding INTEGRATION.md §B shows a maintainer (both stubs, extracted from
the document and run as written, with the library path filled in) computes smt.py:382-404's tile
gradients: the default stub within the fp32-accumulation bar of the fp64 truth, the reference-
rounding stub (ABI v8) against oracle.linearz_tile_grads, the restatement of smt.py:397-404."""
import os
import re

import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd import _hip

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stubs():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = text[text.index("## B. C-ABI binding"):text.index("## Build")]
    blocks = re.findall(r"```python\n(.*?)```", sec, flags=re.S)
    assert len(blocks) == 2
    ns = {}
    code = "\n".join(blocks).replace("/path/to/sparse_matrix_tuning_amd/_lib/libsmt_hip.so", _hip.lib_path())
    _hip.load()                       # torch's HIP runtime first (the stub's own precondition)
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def test_integration_stubs_compute_the_reference_tile_gradients():
    ns = _stubs()
    gen = torch.Generator().manual_seed(11)
    B, S, out_f, in_f = 4, 512, 768, 1024
    g = torch.randn(B, S, out_f, generator=gen).bfloat16()
    x = torch.randn(B, S, in_f, generator=gen).bfloat16()
    index_list = [(2, 3), (0, 0), (1, 2)]
    truth = ref.tile_grads_fp64(g.reshape(-1, out_f), x.reshape(-1, in_f), index_list)
    reference = ref.linearz_tile_grads(g, x, index_list)          # smt.py:397-404, restated
    dev = torch.device("cuda", 0)
    got = ns["tile_wgrad"](g.to(dev), x.to(dev), index_list)
    got_ref = ns["tile_wgrad_reference_rounding"](g.to(dev), x.to(dev), index_list)
    torch.cuda.synchronize()
    err, ref_err = _rel(got, truth), _rel(reference, truth)
    direct = _rel(got_ref, reference)
    print(f"\nstub vs fp64 {err:.2e} (reference {ref_err:.2e}); reference-rounding stub vs restatement {direct:.2e}")
    assert err <= max(1e-3, 1.1 * ref_err)
    assert direct <= 1e-3

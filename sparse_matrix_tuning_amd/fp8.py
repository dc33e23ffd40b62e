"""fp8 (OCP e4m3) frozen linears for the SMT step: BASELINE.json config 5, SURVEY §8(f) row 2.

The reference has no fp8 (bf16/fp16/fp32 only, ``deepspeed/fine_tune.py:955-959``); this path is an
MI355X extension whose parity is stated against the build's own bf16 path
(``tests/test_gpu_fp8.py``). What is fp8 and what is not:

* Every frozen linear weight of the decoder layers (SMT modules and untouched ``nn.Linear``) keeps
  two e4m3 copies made by ``csrc/fp8_kernels.hip``: ``w8 [out, in]`` with one fp32 scale per output
  row (the forward operand) and ``wt8 [in, out]`` with one scale per input column (the data-gradient
  operand, written transposed). Activations and output gradients are quantised per row (token)
  right before each GEMM. The forward ``x @ W^T`` and the data gradient ``g @ W`` then run as
  hipBLASLt rowwise-scaled fp8 GEMMs (``torch._scaled_mm``), 2.4-2.9 PF/s against 1.4-1.6 PF/s in
  bf16 on the LLaMA-3-8B shapes (profiles/r01_fp8_probe.jsonl).
* The 256x256 trainable tiles stay exact: fp32 master and moments, bf16 values in W written by the
  AdamW epilogue, and their weight gradient is the bf16 MFMA tile GEMM on the bf16 activations. After
  each step the rows (for ``w8``) and columns (for ``wt8``) that the tiles touch are re-quantised
  from the bf16 W, so the fp8 copies always describe the current tiles.
* The LM head, embeddings, norms and attention stay bf16.

No CPU path: every entry point raises without a ROCm device.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _hip

F8 = torch.float8_e4m3fn
E4M3_MAX = 448.0


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _bf16_rows(t: torch.Tensor, what: str) -> torch.Tensor:
    if t.dtype != torch.bfloat16 or t.dim() != 2:
        raise RuntimeError(f"{what}: 2-D bf16 ROCm tensor expected (got {t.dtype}, {tuple(t.shape)})")
    if t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def quant_rows(x2d: torch.Tensor, row_blocks: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
               scales: Optional[torch.Tensor] = None):
    """Per-row e4m3 quantisation of a bf16 ``[rows, cols]`` matrix (all rows, or the rows of the
    256-row blocks ``row_blocks``, device int32). Returns ``(q [rows, cols] float8_e4m3fn, scales [rows])``."""
    dev = _hip._require_device(x2d, row_blocks, out, scales)
    x2d = _bf16_rows(x2d, "quant_rows")
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(rows, cols, dtype=torch.uint8, device=dev)
    if scales is None:
        scales = torch.empty(rows, dtype=torch.float32, device=dev)
    raw = out.view(torch.uint8)
    rc = _hip.load().smt_quant_rows_e4m3(x2d.data_ptr(), x2d.stride(0), rows, cols,
                                         None if row_blocks is None else row_blocks.data_ptr(),
                                         0 if row_blocks is None else row_blocks.numel(),
                                         raw.data_ptr(), raw.stride(0), scales.data_ptr(), _stream(dev))
    _hip._check(rc, "smt_quant_rows_e4m3")
    return raw.view(F8), scales


def quant_cols_t(w: torch.Tensor, col_blocks: Optional[torch.Tensor] = None, out_t: Optional[torch.Tensor] = None,
                 scales: Optional[torch.Tensor] = None):
    """Per-column e4m3 quantisation of a bf16 ``[rows, cols]`` matrix, written transposed. Returns
    ``(q_t [cols, rows] float8_e4m3fn, scales [cols])``."""
    dev = _hip._require_device(w, col_blocks, out_t, scales)
    w = _bf16_rows(w, "quant_cols_t")
    rows, cols = w.shape
    if out_t is None:
        out_t = torch.empty(cols, rows, dtype=torch.uint8, device=dev)
    if scales is None:
        scales = torch.empty(cols, dtype=torch.float32, device=dev)
    raw = out_t.view(torch.uint8)
    rc = _hip.load().smt_quant_cols_t_e4m3(w.data_ptr(), w.stride(0), rows, cols,
                                           None if col_blocks is None else col_blocks.data_ptr(),
                                           0 if col_blocks is None else col_blocks.numel(),
                                           raw.data_ptr(), raw.stride(0), scales.data_ptr(), _stream(dev))
    _hip._check(rc, "smt_quant_cols_t_e4m3")
    return raw.view(F8), scales


class Fp8Weight:
    """The two e4m3 copies of one frozen bf16 ``W [out, in]``."""

    def __init__(self, weight: torch.Tensor):
        w = weight.detach()
        self.w8, self.sw = quant_rows(w)                  # [out, in], per output row
        self.wt8, self.swt = quant_cols_t(w)              # [in, out], per input column
        self.sw_row = self.sw.view(1, -1)
        self.swt_row = self.swt.view(1, -1)

    def refresh(self, weight: torch.Tensor, row_blocks: torch.Tensor, col_blocks: torch.Tensor) -> None:
        """Re-quantise the rows / columns of the given 256-blocks from the current bf16 W."""
        w = weight.detach()
        quant_rows(w, row_blocks, out=self.w8, scales=self.sw)
        quant_cols_t(w, col_blocks, out_t=self.wt8, scales=self.swt)

    @property
    def nbytes(self) -> int:
        return self.w8.numel() + self.wt8.numel() + 4 * (self.sw.numel() + self.swt.numel())


def quant_rows_cached(x: torch.Tensor):
    """Per-row e4m3 copy of an activation ``[..., K]``, cached on the tensor (keyed by its version):
    q/k/v (and gate/up) read the same normalised input, which is then quantised once, not 3 (2) times.
    The copy lives exactly as long as the bf16 activation does."""
    c = x.__dict__.get("_smt_q8")
    if c is not None and c[0] == x._version:
        return c[1], c[2]
    x8, sx = quant_rows(x.reshape(-1, x.shape[-1]))
    x._smt_q8 = (x._version, x8, sx)
    return x8, sx


def fp8_matmul(a2d: torch.Tensor, b8: torch.Tensor, b_scales_row: torch.Tensor, a_q=None) -> torch.Tensor:
    """``a2d [M, K] (bf16, quantised per row here unless ``a_q`` = (a8, scales) is given) @ b8 [N, K]^T``
    with ``b8``'s per-row scales: a hipBLASLt rowwise-scaled e4m3 GEMM, bf16 out."""
    a8, sa = a_q if a_q is not None else quant_rows(a2d)
    return torch._scaled_mm(a8, b8.t(), scale_a=sa.view(-1, 1), scale_b=b_scales_row, out_dtype=torch.bfloat16)


def fp8_linear_forward(x: torch.Tensor, fw: Fp8Weight) -> torch.Tensor:
    shape = x.shape
    y = fp8_matmul(None, fw.w8, fw.sw_row, a_q=quant_rows_cached(x))
    return y.view(*shape[:-1], y.shape[-1])


def fp8_linear_dgrad(grad_output: torch.Tensor, fw: Fp8Weight) -> torch.Tensor:
    shape = grad_output.shape
    gi = fp8_matmul(grad_output.reshape(-1, shape[-1]), fw.wt8, fw.swt_row)
    return gi.view(*shape[:-1], gi.shape[-1])


class Fp8LinearFn(torch.autograd.Function):
    """``x @ W^T (+ b)`` of a frozen W through its e4m3 copies; the data gradient through ``wt8``."""

    @staticmethod
    def forward(ctx, x, weight, fw, bias):
        ctx.fw = fw
        y = fp8_linear_forward(x, fw)
        return y if bias is None else y + bias

    @staticmethod
    def backward(ctx, grad_output):
        gi = fp8_linear_dgrad(grad_output, ctx.fw) if ctx.needs_input_grad[0] else None
        return gi, None, None, None

"""Data gradients of frozen linears that read the same input.

In the LLaMA decoder q/k/v_proj read one normalised hidden state and gate/up_proj another. Left to
autograd, each of those linears returns its own ``[T, in]`` gradient and autograd sums them with
separate elementwise adds (2 + 1 per layer; 96 of the step's 224 bf16 add kernels). Here the
consumers accumulate into ONE buffer through the GEMM's C operand (``addmm_``, beta = 1: the
hipBLASLt epilogue reads C once instead of an extra read-read-write pass) and only the last of them
to run hands it to autograd; the others return ``None`` (a zero contribution).

The consumers are counted at forward time on the input tensor (keyed by its version), so every
registered consumer must run its backward for the gradient to be handed over -- true for the
decoder, whose q/k/v and gate/up outputs all feed the loss. A tensor with one consumer takes the
plain path.
"""
from __future__ import annotations

from typing import Optional

import torch


class SharedInputGrad:
    __slots__ = ("version", "consumers", "pending", "buf")

    def __init__(self, version: int):
        self.version = version
        self.consumers = 0
        self.pending = 0
        self.buf: Optional[torch.Tensor] = None


def register(x: torch.Tensor) -> Optional[SharedInputGrad]:
    """Count one more linear consumer of ``x`` (call from the consumer's forward)."""
    if not x.requires_grad:
        return None
    acc = x.__dict__.get("_smt_gacc")
    if acc is None or acc.version != x._version:
        acc = SharedInputGrad(x._version)
        x._smt_gacc = acc
    acc.consumers += 1
    return acc


def input_grad(acc: Optional[SharedInputGrad], grad_output: torch.Tensor, mat: torch.Tensor) -> Optional[torch.Tensor]:
    """``grad_output [..., out] @ mat [out, in]`` for one consumer; with a shared accumulator, the
    summed gradient of all consumers from the last one and ``None`` from the others."""
    lead = grad_output.shape[:-1]
    g2 = grad_output.reshape(-1, grad_output.shape[-1])
    if acc is None or acc.consumers <= 1:
        out = torch.matmul(g2, mat)
        return out.view(*lead, out.shape[-1])
    if acc.buf is None:
        acc.buf = torch.matmul(g2, mat)
        acc.pending = acc.consumers - 1
    else:
        acc.buf.addmm_(g2, mat)
        acc.pending -= 1
    if acc.pending > 0:
        return None
    buf, acc.buf = acc.buf, None
    return buf.view(*lead, buf.shape[-1])

"""Data gradients of frozen linears that read the same input.

In the LLaMA decoder q/k/v_proj read one normalised hidden state and gate/up_proj another. Left to
autograd, each of those linears returns its own ``[T, in]`` gradient and autograd sums them with
separate elementwise adds (2 + 1 per layer; 96 of the step's 224 bf16 add kernels). Here the
consumers accumulate into ONE buffer through the GEMM's C operand (``addmm_``, beta = 1: the
hipBLASLt epilogue reads C once instead of an extra read-read-write pass) and only the last of them
to run hands it to autograd; the others return ``None`` (a zero contribution).

"Last" is decided when each consumer's backward runs, not counted at forward time: every consumer
records its autograd node, and a consumer hands the buffer over as soon as no other consumer that
has not run yet will be executed by the running backward (``torch._C._will_engine_execute_node``).
So a consumer whose output does not reach the loss, a partial ``torch.autograd.grad``, or separate
backward calls over different consumers never strand a contribution: each backward pass hands over
exactly the sum of the consumers it ran. A tensor with one consumer takes the plain path.

Joint product (q/k/v): when a consumer's output gradient is a column slice of a wider row-major
buffer and its weight operand the transpose of a column slice of an equally wide transposed copy
(the flash attention's joint [dq | dk | dv] gradient and the engine's joint q/k/v W^T), its product
is deferred to the last consumer. If the deferred slices then tile both buffers at the same column
offsets, the sum is ONE GEMM over the whole width (fewer, larger GEMMs and no C re-reads; one bf16
rounding of the fp32 sum instead of one per consumer); otherwise the deferred products run one by
one as before.
"""
from __future__ import annotations

import weakref
from typing import List, Optional

import torch


JOINT_PRODUCTS = 0          # joint GEMMs issued by _flush (diagnostics / tests)


class SharedInputGrad:
    __slots__ = ("version", "nodes", "done", "buf", "pending")

    def __init__(self, version: int):
        self.version = version
        # weak references to the consumers' autograd nodes (their ctx): the input tensor keeps this
        # object alive, and the nodes keep the input alive through their saved tensors
        self.nodes: List[weakref.ref] = []
        self.done: List[bool] = []
        self.buf: Optional[torch.Tensor] = None
        self.pending: List[tuple] = []              # deferred (g2, mat) of joint-slice consumers

    @property
    def consumers(self) -> int:
        return len(self.nodes)


class _Slot:
    """What one consumer keeps: the shared accumulator and its own position in it."""
    __slots__ = ("acc", "index")

    def __init__(self, acc: SharedInputGrad, index: int):
        self.acc = acc
        self.index = index


def register(x: torch.Tensor, node=None) -> Optional[_Slot]:
    """Count one more linear consumer of ``x`` (call from the consumer's forward with its ``ctx``)."""
    if not x.requires_grad or node is None:
        return None
    acc = x.__dict__.get("_smt_gacc")
    if acc is None or acc.version != x._version:
        acc = SharedInputGrad(x._version)
        x._smt_gacc = acc
    acc.nodes.append(weakref.ref(node))
    acc.done.append(False)
    return _Slot(acc, len(acc.nodes) - 1)


def _others_pending(acc: SharedInputGrad, me: int) -> bool:
    for i, ref in enumerate(acc.nodes):
        if i == me or acc.done[i]:
            continue
        node = ref()
        if node is not None and torch._C._will_engine_execute_node(node):
            return True
    return False


def input_grad(slot: Optional[_Slot], grad_output: torch.Tensor, mat: torch.Tensor) -> Optional[torch.Tensor]:
    """``grad_output [..., out] @ mat [out, in]`` for one consumer; with a shared accumulator, the
    summed gradient of the consumers this backward runs from the last of them and ``None`` from the
    others."""
    lead = grad_output.shape[:-1]
    g2 = grad_output.reshape(-1, grad_output.shape[-1])
    acc = None if slot is None else slot.acc
    if acc is None or acc.consumers <= 1:
        out = torch.matmul(g2, mat)
        return out.view(*lead, out.shape[-1])
    if _joint_slice(g2, mat):
        acc.pending.append((g2, mat))
    elif acc.buf is None:
        acc.buf = torch.matmul(g2, mat)
    else:
        acc.buf.addmm_(g2, mat)
    acc.done[slot.index] = True
    if _others_pending(acc, slot.index):
        return None
    if acc.pending:
        _flush(acc)
    buf, acc.buf = acc.buf, None
    acc.done = [False] * len(acc.done)           # a later backward over the same graph starts afresh
    return buf.view(*lead, buf.shape[-1])


def _joint_slice(g2: torch.Tensor, mat: torch.Tensor) -> bool:
    """g2 [T, out] a column slice of a wider row-major buffer (row stride C > out), mat [out, in] the
    transpose of a column slice of an [in, C] row-major transposed copy."""
    C = g2.stride(0)
    return (g2.dim() == 2 and g2.stride(1) == 1 and C > g2.shape[1] and mat.dim() == 2
            and mat.stride(0) == 1 and mat.stride(1) == C and mat.dtype == g2.dtype)


def _flush(acc: SharedInputGrad) -> None:
    """Add the deferred products into ``acc.buf``: one GEMM over the whole width when the deferred
    slices tile the gradient buffer and the transposed copy at the same column offsets."""
    items, acc.pending = acc.pending, []
    g0, m0 = items[0]
    C = g0.stride(0)
    og, ow = min(g.storage_offset() for g, _ in items), min(m.storage_offset() for _, m in items)
    spans = sorted((g.storage_offset() - og, g.shape[1], m.storage_offset() - ow) for g, m in items)
    joint = (all(g.untyped_storage().data_ptr() == g0.untyped_storage().data_ptr() and g.shape[0] == g0.shape[0]
                 and g.stride(0) == C for g, _ in items)
             and all(m.untyped_storage().data_ptr() == m0.untyped_storage().data_ptr() and m.shape[1] == m0.shape[1]
                     for _, m in items)
             and all(a == c for a, _w, c in spans)
             and all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(len(spans) - 1))
             and spans[0][0] == 0 and spans[-1][0] + spans[-1][1] == C)
    if joint:
        global JOINT_PRODUCTS
        JOINT_PRODUCTS += 1
        gj = torch.as_strided(g0, (g0.shape[0], C), (C, 1), og)
        mj = torch.as_strided(m0, (C, m0.shape[1]), (1, C), ow)
        items = [(gj, mj)]
    for g, m in items:
        if acc.buf is None:
            acc.buf = torch.matmul(g, m)
        else:
            acc.buf.addmm_(g, m)

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
* The linears that read one input (q/k/v, gate/up) form an :class:`Fp8Group`: their data gradients
  are ONE fp8 GEMM of the concatenated output gradients against the jointly quantised transposed
  weight, so neither a per-member GEMM nor autograd's gradient adds remain.
* The LM head, embeddings, norms and attention stay bf16.

No CPU path: every entry point raises without a ROCm device.
"""
from __future__ import annotations

import os
import threading
import weakref
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


def quant_rows_cat(parts):
    """Per-row e4m3 quantisation of the concatenation ``[p_0 | p_1 | ...]`` of bf16 ``[rows, cols_i]``
    matrices (one scale per row over all of them), without materialising the bf16 concatenation."""
    dev = _hip._require_device(*parts)
    parts = [_bf16_rows(p, "quant_rows_cat") for p in parts]
    rows = parts[0].shape[0]
    if any(p.shape[0] != rows for p in parts) or not 1 <= len(parts) <= 4:
        raise ValueError("quant_rows_cat: 1-4 sources with the same number of rows")
    cols = sum(p.shape[1] for p in parts)
    out = torch.empty(rows, cols, dtype=torch.uint8, device=dev)
    scales = torch.empty(rows, dtype=torch.float32, device=dev)
    srcs = (_hip.QuantSrc * len(parts))(*[_hip.QuantSrc(p.data_ptr(), p.stride(0), p.shape[1], 0) for p in parts])
    rc = _hip.load().smt_quant_rows_cat_e4m3(srcs, len(parts), rows, out.data_ptr(), out.stride(0), scales.data_ptr(),
                                             _stream(dev))
    _hip._check(rc, "smt_quant_rows_cat_e4m3")
    return out.view(F8), scales


class Fp8Group:
    """Frozen linears that read the same input (q/k/v of a LlamaAttention, gate/up of a LlamaMLP).
    Their data gradients run as ONE fp8 GEMM: the concatenated output gradients (quantised per row
    over all of them by ``smt_quant_rows_cat_e4m3``) against the jointly quantised transposed weight
    ``[W_0; W_1; ...]^T`` (one scale per input column over all members). That replaces one GEMM per
    member plus the adds autograd would use to sum their input gradients."""

    def __init__(self, weights):
        self.weights = list(weights)
        self.outs = [w.shape[0] for w in self.weights]
        self.offsets = [sum(self.outs[:i]) for i in range(len(self.outs))]
        # the members' W become row slices of ONE joint [sum(out), in] buffer (same values, same
        # Parameter objects; built before any tile descriptor records a W address), so the per-step
        # re-quantisation of the joint transposed copy reads it in place instead of concatenating
        # the members (was 2 torch.cat copies of 50 + 235 MB per layer and step at the 8B point)
        self.joint = torch.cat([w.detach() for w in self.weights], 0)
        for w, off, n in zip(self.weights, self.offsets, self.outs):
            w.data = self.joint[off:off + n]
        self.wt8, self.swt = quant_cols_t(self._cat())           # [in, sum(out)]
        self.swt_row = self.swt.view(1, -1)
        # the MX column blocks of the members' shared input, quantised once per forward for the union
        # of the column blocks the members' tiles read (set by the engine: set_mx_union)
        self.mx_union = None            # (device int32 blocks, {block: position})
        self._mx_cache = None           # (weakref to the input, its version, MxBlocks)

    def set_mx_union(self, col_blocks, device) -> None:
        cbs = sorted(int(c) for c in col_blocks)
        self.mx_union = (torch.tensor(cbs, dtype=torch.int32).to(device), {c: i for i, c in enumerate(cbs)})
        self._mx_cache = None

    def mx_input_blocks(self, x: torch.Tensor, x2d: torch.Tensor):
        """The MX column blocks (union order) of the input ``x`` the members read: quantised by the
        first member's forward, shared by the others (same tensor object and version)."""
        import weakref
        c = self._mx_cache
        if c is not None and c[0]() is x and c[1] == x._version:
            return c[2]
        mx = _hip.mx_quant_cols(x2d, self.mx_union[0])
        self._mx_cache = (weakref.ref(x), x._version, mx)
        return mx

    def clear_mx_cache(self) -> None:
        self._mx_cache = None

    def _cat(self) -> torch.Tensor:
        """The members' current W stacked: the joint buffer itself while every member still aliases
        its slice of it (a member whose ``.data`` was replaced since is concatenated afresh)."""
        j = self.joint
        row = j.stride(0) * j.element_size()
        if all(w.data_ptr() == j.data_ptr() + off * row and w.shape[0] == n
               for w, off, n in zip(self.weights, self.offsets, self.outs)):
            return j
        return torch.cat([w.detach() for w in self.weights], 0)

    def refresh(self, col_blocks: torch.Tensor) -> None:
        """Re-quantise the joint copy's rows for the given 256-column blocks of the members' W."""
        quant_cols_t(self._cat(), col_blocks, out_t=self.wt8, scales=self.swt)

    def member_wt8(self, i: int) -> torch.Tensor:
        """Member i's transposed copy as a column slice ``[in, out_i]`` of the joint one (same scales)."""
        return self.wt8[:, self.offsets[i]:self.offsets[i] + self.outs[i]]

    @property
    def nbytes(self) -> int:
        return self.wt8.numel() + 4 * self.swt.numel()


class Fp8Weight:
    """The e4m3 copies of one frozen bf16 ``W [out, in]``: ``w8`` (per output row) for the forward,
    and for the data gradient either its own ``wt8 [in, out]`` (per input column) or, as a member of
    an :class:`Fp8Group`, a slice of the group's joint transposed copy."""

    def __init__(self, weight: torch.Tensor, group: "Fp8Group" = None, group_index: int = 0):
        w = weight.detach()
        # the tile weight gradient of an SMT module over this weight: MX-fp8 operands (e4m3, one
        # e8m0 exponent per 32 tokens; smt_tile_wgrad_mx) by default, bf16 with SMT_FP8_TILE_WGRAD=bf16
        self.mx_wgrad = os.environ.get("SMT_FP8_TILE_WGRAD", "mx") != "bf16"
        self.w8, self.sw = quant_rows(w)                  # [out, in], per output row
        self.sw_row = self.sw.view(1, -1)
        self.group = group
        self.group_index = group_index
        if group is None:
            self.wt8, self.swt = quant_cols_t(w)          # [in, out], per input column
        else:
            self.wt8, self.swt = group.member_wt8(group_index), group.swt
        self.swt_row = self.swt.view(1, -1)

    def refresh(self, weight: torch.Tensor, row_blocks: torch.Tensor, col_blocks: torch.Tensor,
                group: bool = True) -> None:
        """Re-quantise the rows / columns of the given 256-blocks from the current bf16 W (the
        columns of a grouped copy only with ``group``: the engine refreshes each group once)."""
        w = weight.detach()
        quant_rows(w, row_blocks, out=self.w8, scales=self.sw)
        if self.group is None:
            quant_cols_t(w, col_blocks, out_t=self.wt8, scales=self.swt)
        elif group:
            self.group.refresh(col_blocks)

    @property
    def nbytes(self) -> int:
        own = self.wt8.numel() + 4 * self.swt.numel() if self.group is None else 0
        return self.w8.numel() + 4 * self.sw.numel() + own


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
    # cached: the RMSNorm backward that produced a residual-stream gradient may have quantised it
    gi = fp8_matmul(None, fw.wt8, fw.swt_row, a_q=quant_rows_cached(grad_output))
    return gi.view(*shape[:-1], gi.shape[-1])


class GroupGrad:
    """The output gradients of one forward's group members, collected until the last one arrives.
    ``prequant``: the members' output gradients already quantised as one row by their producer
    (:func:`swiglu_bwd_quant` for gate/up), used instead of quantising the collected parts."""

    __slots__ = ("version", "group", "nodes", "done", "parts", "prequant")

    def __init__(self, version: int, group: Fp8Group):
        self.version = version
        self.group = group
        self.nodes = []          # weak references to the members' autograd nodes (dgrad.py)
        self.done = []
        self.parts = {}
        self.prequant = None


# SMT_FP8_FUSED_SWIGLU=0 turns the SwiGLU-backward + quantisation fusion off (A/B, parity tests)
FUSED_SWIGLU_QUANT = os.environ.get("SMT_FP8_FUSED_SWIGLU", "1") != "0"
# SMT_FP8_FUSED_SWIGLU_FWD=0: only the forward half (down_proj input quantised by the SwiGLU) off
FUSED_SWIGLU_FWD_QUANT = os.environ.get("SMT_FP8_FUSED_SWIGLU_FWD", "1") != "0"
# SMT_FP8_PACK_SWIGLU_GRAD=0: the SwiGLU backward writes an SMT gate/up module's whole bf16 output
# gradient instead of only the row blocks its MX tile gradient reads (A/B, parity tests)
PACK_SWIGLU_GRAD = os.environ.get("SMT_FP8_PACK_SWIGLU_GRAD", "1") != "0"

# Packed row blocks are requested only by gate/up outputs whose sole consumer is known to be the
# fused SwiGLU: fused_llama.fused_mlp_forward computes them inside this scope. Any other graph (a
# hook, a custom MLP, a second reader of the gate output) gets the whole bf16 gradient, so a valid
# graph never hits the summed-away guard of linearZ.backward.
_sole_swiglu = threading.local()


class sole_swiglu_consumer:
    """Context manager: the SMT linears called inside feed only FusedSwiGLUFn."""

    def __enter__(self):
        _sole_swiglu.depth = getattr(_sole_swiglu, "depth", 0) + 1
        return self

    def __exit__(self, *exc):
        _sole_swiglu.depth -= 1
        return False


def packed_rows_allowed() -> bool:
    return PACK_SWIGLU_GRAD and getattr(_sole_swiglu, "depth", 0) > 0


class MxRowsNeed(tuple):
    """``("mx_rows", tiles)``: an SMT module's request for only its MX tiles' row blocks of its bf16
    output gradient. A producer that hands them over packed sets ``delivered``, so linearZ.backward
    can tell a packed hand-over that autograd summed away (the output had another consumer) from a
    producer that wrote the whole gradient."""

    def __new__(cls, tiles):
        return super().__new__(cls, ("mx_rows", tiles))


def tag_group_output(y: torch.Tensor, reg, fw: "Fp8Weight", needs_bf16_grad) -> torch.Tensor:
    """Mark a group member's output so that its consumer can hand the member's gradient over
    pre-quantised (``needs_bf16_grad``: the member also needs the bf16 gradient itself, e.g. an SMT
    module's tile weight gradient: True, or ``("mx_rows", tiles)`` when only the row blocks of its MX
    tiles are read, which a producer may hand over packed). ``reg``: what :func:`register_group`
    returned."""
    if reg is not None:
        # the last field: produced where the fused SwiGLU is known to be the only consumer
        # (sole_swiglu_consumer), the condition for it to hand the gradients over pre-quantised
        y._smt_gout = (reg[0], fw.group_index, needs_bf16_grad, getattr(_sole_swiglu, "depth", 0) > 0)
    return y


def swiglu_group(gate: torch.Tensor, up: torch.Tensor):
    """``(acc, needs_bf16_gate, needs_bf16_up)`` when gate and up are the two members of one fp8
    group (gate first), else None: their SwiGLU backward can then emit the joint fp8 rows."""
    if not FUSED_SWIGLU_QUANT:
        return None
    tg, tu = gate.__dict__.get("_smt_gout"), up.__dict__.get("_smt_gout")
    if tg is None or tu is None or tg[0] is not tu[0] or (tg[1], tu[1]) != (0, 1) or len(tg[0].group.outs) != 2:
        return None
    if not (tg[3] and tu[3]):
        # gate / up made outside fused_mlp_forward may have other consumers: autograd then sums their
        # gradients, and the group quantises what arrives instead
        return None
    if gate.shape != up.shape or gate.shape[-1] > 16384:
        return None
    return tg[0], tg[2], tu[2]


# SMT_FP8_FUSED_NORM=0: the decoder's RMSNorms stop emitting the e4m3 input of their fp8 consumers
FUSED_NORM_QUANT = os.environ.get("SMT_FP8_FUSED_NORM", "1") != "0"


def norm_consumers(*linears):
    """``(quant, need_bf16)`` for an RMSNorm output read by these linears: quantise it in the norm
    when every consumer runs in fp8; keep the bf16 output only if some consumer reads it (an SMT
    module's tile weight gradient, or a trainable weight)."""
    if not FUSED_NORM_QUANT or any(getattr(m.weight, "_smt_fp8", None) is None for m in linears):
        return False, True
    return True, any(not (type(m) is torch.nn.Linear and not m.weight.requires_grad) for m in linears)


def rmsnorm_quant(x2: torch.Tensor, r2, w: torch.Tensor, eps: float, need_y: bool):
    """RMSNorm (of ``x2 + r2`` when ``r2`` is given) that also emits its output as e4m3 rows
    (``smt_rmsnorm_fwd_quant_e4m3``): returns ``(h or None, y or None, rstd, q, scales)``."""
    dev = _hip._require_device(x2, w)
    rows, H = x2.shape
    h = torch.empty_like(x2) if r2 is not None else None
    y = torch.empty_like(x2) if need_y else None
    rstd = torch.empty(rows, dtype=torch.float32, device=dev)
    q = torch.empty(rows, H, dtype=torch.uint8, device=dev)
    sq = torch.empty(rows, dtype=torch.float32, device=dev)
    rc = _hip.load().smt_rmsnorm_fwd_quant_e4m3(
        x2.data_ptr(), x2.stride(0), None if r2 is None else r2.data_ptr(), 0 if r2 is None else r2.stride(0),
        w.data_ptr(), None if h is None else h.data_ptr(), H, None if y is None else y.data_ptr(), H,
        rstd.data_ptr(), q.data_ptr(), q.stride(0), sq.data_ptr(), rows, H, float(eps), _stream(dev))
    _hip._check(rc, "smt_rmsnorm_fwd_quant_e4m3")
    return h, y, rstd, q.view(F8), sq


def rmsnorm_bwd_add_quant(dy2, x2, w, rstd, dr2):
    """``smt_rmsnorm_bwd_add`` that also emits dx as e4m3 rows: returns ``(dx, q, scales)``."""
    dev = _hip._require_device(dy2, x2, w, rstd, dr2)
    rows, H = x2.shape
    dx = torch.empty_like(x2)
    q = torch.empty(rows, H, dtype=torch.uint8, device=dev)
    sq = torch.empty(rows, dtype=torch.float32, device=dev)
    rc = _hip.load().smt_rmsnorm_bwd_add_quant_e4m3(
        dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), w.data_ptr(), rstd.data_ptr(), dr2.data_ptr(),
        dr2.stride(0), dx.data_ptr(), dx.stride(0), q.data_ptr(), q.stride(0), sq.data_ptr(), rows, H, _stream(dev))
    _hip._check(rc, "smt_rmsnorm_bwd_add_quant_e4m3")
    return dx, q.view(F8), sq


def swiglu_fwd_quant(g: torch.Tensor, u: torch.Tensor, need_h: bool):
    """SwiGLU forward fused with the per-row e4m3 quantisation of its output
    (``smt_swiglu_fwd_quant_e4m3``): returns ``(q [T, n], scales [T], h bf16 or None)``."""
    dev = _hip._require_device(g, u)
    n = g.shape[-1]
    rows = g.numel() // n
    q = torch.empty(rows, n, dtype=torch.uint8, device=dev)
    sq = torch.empty(rows, dtype=torch.float32, device=dev)
    h = torch.empty_like(g) if need_h else None
    rc = _hip.load().smt_swiglu_fwd_quant_e4m3(g.data_ptr(), u.data_ptr(), rows, n, q.data_ptr(), q.stride(0),
                                               sq.data_ptr(), h.data_ptr() if need_h else None, _stream(dev))
    _hip._check(rc, "smt_swiglu_fwd_quant_e4m3")
    return q.view(F8), sq, h


def _grad_out_spec(need, like: torch.Tensor, rows: int, n: int):
    """``(tensor or None, position map or None, ld)`` for one bf16 output gradient: none, the whole
    ``[.., n]`` gradient, or (``("mx_rows", tiles)``) the tiles' row blocks packed ``[rows, n_rb*256]``."""
    if not need:
        return None, None, n
    if need is True:
        return torch.empty_like(like), None, n
    if n % 256:
        raise ValueError(f"swiglu_bwd_quant: packed row blocks need a multiple of 256 features, got {n}")
    n_rb, pos, _ident = need[1].mx_row_pack(n, like.device)
    return torch.empty(rows, n_rb * 256, dtype=like.dtype, device=like.device), pos, n_rb * 256


def swiglu_bwd_quant(g: torch.Tensor, u: torch.Tensor, dh: torch.Tensor, need_dg, need_du):
    """SwiGLU backward fused with the per-row e4m3 quantisation of ``[dgate | dup]``
    (``smt_swiglu_bwd_quant_e4m3``): returns ``(q [T, 2n], scales [T], dgate or None, dup or None)``.
    ``need_dg`` / ``need_du``: False, True (the whole bf16 gradient) or ``("mx_rows", tiles)`` (only
    the tiles' row blocks, packed ``[T, n_rb*256]``: ``smt_swiglu_bwd_quant_e4m3_packed``)."""
    dev = _hip._require_device(g, u, dh)
    n = g.shape[-1]
    rows = g.numel() // n
    q = torch.empty(rows, 2 * n, dtype=torch.uint8, device=dev)
    sq = torch.empty(rows, dtype=torch.float32, device=dev)
    dg, gpos, ldg = _grad_out_spec(need_dg, g, rows, n)
    du, upos, ldu = _grad_out_spec(need_du, u, rows, n)
    ptr = lambda t: None if t is None else t.data_ptr()
    if gpos is None and upos is None:
        rc = _hip.load().smt_swiglu_bwd_quant_e4m3(g.data_ptr(), u.data_ptr(), dh.data_ptr(), rows, n, q.data_ptr(),
                                                   q.stride(0), sq.data_ptr(), ptr(dg), ptr(du), _stream(dev))
        _hip._check(rc, "smt_swiglu_bwd_quant_e4m3")
    else:
        rc = _hip.load().smt_swiglu_bwd_quant_e4m3_packed(
            g.data_ptr(), u.data_ptr(), dh.data_ptr(), rows, n, q.data_ptr(), q.stride(0), sq.data_ptr(),
            ptr(dg), ptr(gpos), ldg, ptr(du), ptr(upos), ldu, _stream(dev))
        _hip._check(rc, "smt_swiglu_bwd_quant_e4m3_packed")
    return q.view(F8), sq, dg, du


def register_group(x: torch.Tensor, fw: Fp8Weight, node=None):
    """Count one more group member reading ``x`` (call from the member's forward with its ``ctx``);
    None when the weight is not grouped or ``x`` needs no gradient. Returns ``(acc, slot)``."""
    if fw.group is None or not x.requires_grad or node is None:
        return None
    acc = x.__dict__.get("_smt_gacc8")
    if acc is None or acc.version != x._version or acc.group is not fw.group:
        acc = GroupGrad(x._version, fw.group)
        x._smt_gacc8 = acc
    acc.nodes.append(weakref.ref(node))
    acc.done.append(False)
    return acc, len(acc.nodes) - 1


def group_input_grad(reg, fw: Fp8Weight, grad_output: torch.Tensor):
    """The summed input gradient of the group members this backward runs, from the last of them to
    run (one joint fp8 GEMM when every member of the group took part), None from the others. "Last" is
    decided by the autograd engine's plan, as in :mod:`..dgrad`: a member whose output does not reach
    the loss never strands the others' contributions."""
    acc, slot = reg
    acc.parts[fw.group_index] = grad_output
    acc.done[slot] = True
    for i, ref in enumerate(acc.nodes):
        if i != slot and not acc.done[i]:
            node = ref()
            if node is not None and torch._C._will_engine_execute_node(node):
                return None
    parts, acc.parts = acc.parts, {}
    acc.done = [False] * len(acc.done)
    g = acc.group
    lead = grad_output.shape[:-1]
    pre, acc.prequant = acc.prequant, None
    if pre is None and any("_smt_gpack" in t.__dict__ for t in parts.values()):
        raise RuntimeError("fp8 group data gradient: a member's output gradient was handed over packed "
                           "(row blocks only) without its producer's e4m3 rows")
    if pre is not None and (sorted(parts) != list(range(len(g.outs)))
                            or any(parts[i] is not t for i, t in enumerate(pre[2]))):
        # the producer's rows hold only its own share of each member's output gradient: a part that
        # autograd summed with another consumer's gradient (or a member that did not run) is not in them
        raise RuntimeError("fp8 group data gradient: a member's output gradient is not the tensor its "
                           "producer quantised (summed with another consumer's gradient); the producer's "
                           "e4m3 rows would miss that share")
    if sorted(parts) == list(range(len(g.outs))):
        if pre is not None:                 # quantised by the producer of the parts
            q, sq, _handed = pre
        else:
            q, sq = quant_rows_cat([parts[i].reshape(-1, g.outs[i]) for i in range(len(g.outs))])
        gi = torch._scaled_mm(q, g.wt8.t(), scale_a=sq.view(-1, 1), scale_b=g.swt_row, out_dtype=torch.bfloat16)
    else:                                   # a subset of the members: per-member GEMMs on the slices
        gi = None
        for i, go in parts.items():
            part = fp8_matmul(go.reshape(-1, g.outs[i]), g.member_wt8(i), g.swt_row)
            gi = part if gi is None else gi.add_(part)
    return gi.view(*lead, gi.shape[-1])


def fp8_input_grad(ctx_acc, fw: Fp8Weight, grad_output: torch.Tensor):
    """Data gradient of one fp8 linear: through its group when it registered with one."""
    if ctx_acc is not None:
        return group_input_grad(ctx_acc, fw, grad_output)
    return fp8_linear_dgrad(grad_output, fw)


class Fp8LinearFn(torch.autograd.Function):
    """``x @ W^T (+ b)`` of a frozen W through its e4m3 copies; the data gradient through ``wt8``
    (jointly with the other members of its group when it has one)."""

    @staticmethod
    def forward(ctx, x, weight, fw, bias):
        ctx.fw = fw
        ctx.gacc = register_group(x, fw, ctx)
        y = fp8_linear_forward(x, fw)
        return tag_group_output(y if bias is None else y + bias, ctx.gacc, fw, False)

    @staticmethod
    def backward(ctx, grad_output):
        gi = fp8_input_grad(ctx.gacc, ctx.fw, grad_output) if ctx.needs_input_grad[0] else None
        return gi, None, None, None

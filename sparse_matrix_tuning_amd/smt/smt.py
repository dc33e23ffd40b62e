"""MI355X drop-in for ``deepspeed/smt/smt.py`` (the matrix-sparsity path).

Same names, signatures, argument meaning and error behaviour as the reference module that
``deepspeed/fine_tune.py:39`` imports, re-implemented over the gfx950 kernels of
``libsmt_hip.so``:

* tile gather (smt.py:317-325) and the per-forward write-back (smt.py:332-341) are one HIP
  launch per module instead of one copy per tile;
* ``linearZ.backward``'s per-tile Python loop of batched GEMM + sum + copy (smt.py:386-404) is
  one grouped bf16 MFMA launch over every tile of the module;
* under :func:`sparse_matrix_tuning_amd.engine.initialize` the tile gradients land in fp32 in the
  engine's packed buffer and the fused AdamW writes the tiles back into ``W``, so the forward
  write-back is skipped.

Differences from the reference, all deliberate:

* no process-group initialisation or rank query at import (smt.py:20-21);
* no ``print_rank_0`` spam;
* the tile-gradient rounding follows the reference by default: every per-sample ``[256, 256]``
  partial is rounded to bf16 and the partials are summed in sample order (smt.py:397-404,
  ``smt_tile_wgrad_batch_seq``; tests/test_gpu_wgrad_full.py). :func:`set_wgrad_rounding("single")`
  (or ``SMT_WGRAD_ROUNDING=single``) sums the whole batch in fp32 and rounds once instead, which is
  closer to exact than the reference. Those two are the global switch; an engine's config key
  ``"wgrad_rounding"`` overrides it for that engine's modules only (an engine without the key takes
  the global mode at its creation, and "single" for fp8 weights). The MX-fp8 tile gradient (config 5)
  sums e4m3 products over all rows and has no per-sample partials: the global mode does not apply to
  it, and an engine that asks for "reference" on it raises.

There is no CPU or eager-PyTorch path: a module built on CPU tensors raises. ``meta`` tensors are
accepted for shape-only construction (used by the CPU tests of the conversion logic).
"""
from __future__ import annotations

import os
import re
import weakref
from typing import Iterable, List, Optional, Sequence, Tuple

import torch
from torch import nn

from .. import _hip, dgrad

Block_dimension = 256

_LAYER_PATTERN = re.compile(r'model\.layers\.(\d+)\.')

# Tile-gradient rounding of linearZ.backward: "reference" (the default, smt.py:397-404: every
# per-sample partial rounded to bf16, then the batch sum) or "single" (fp32 over the whole batch, one
# rounding)
WGRAD_ROUNDINGS = ("single", "reference")
_wgrad_rounding = os.environ.get("SMT_WGRAD_ROUNDING", "reference")
if _wgrad_rounding not in WGRAD_ROUNDINGS:
    raise ValueError(f"SMT_WGRAD_ROUNDING={_wgrad_rounding!r}: one of {WGRAD_ROUNDINGS}")


def set_wgrad_rounding(mode: str) -> str:
    """Select the tile-gradient rounding of every later ``linearZ`` forward; returns the old mode."""
    global _wgrad_rounding
    if mode not in WGRAD_ROUNDINGS:
        raise ValueError(f"wgrad rounding {mode!r}: one of {WGRAD_ROUNDINGS}")
    old, _wgrad_rounding = _wgrad_rounding, mode
    return old


def wgrad_rounding() -> str:
    return _wgrad_rounding


# What linearZ keeps of its input for the tile weight gradient (smt.py:351-358 keeps column slices
# of it): "resident" (the input, or a packed copy of its column blocks when the tiles touch at most
# half of them), "selective" (when the input is an RMSNorm's or SwiGLU's output produced by
# fused_llama, nothing: the backward rebuilds the column blocks from the producer's own saved
# operands with smt_colblock_recompute), "views" (the input itself, always: the reference's views
# of it, which keep the whole input alive, and no copy). Tile gradients are bit-identical under all
# three (same operands, same kernel, same order).
ACTIVATION_POLICIES = ("resident", "selective", "views")
_activation_policy = os.environ.get("SMT_ACTIVATION_POLICY", "resident")
if _activation_policy not in ACTIVATION_POLICIES:
    raise ValueError(f"SMT_ACTIVATION_POLICY={_activation_policy!r}: one of {ACTIVATION_POLICIES}")


def set_activation_policy(mode: str) -> str:
    """Select what every later ``linearZ`` forward keeps of its input; returns the old policy."""
    global _activation_policy
    if mode not in ACTIVATION_POLICIES:
        raise ValueError(f"activation policy {mode!r}: one of {ACTIVATION_POLICIES}")
    old, _activation_policy = _activation_policy, mode
    return old


def activation_policy() -> str:
    return _activation_policy


# Engines whose config names a mode of their own (``"wgrad_rounding"`` / ``"activation_policy"``)
# keep it on the engine: linearZ reads it through the module's gradient sink, so one engine's
# config never leaks into another model or a later test in the same process. The global setting
# above is what modules without such an engine use. Live engines asking for "selective" are counted
# so that the producers tag their outputs (tag_recompute) while any of them exists.
_selective_engines = 0


def _engine_mode(sink, attr: str):
    eng = getattr(sink, "engine", None) if sink is not None else None
    return getattr(eng, attr, None) if eng is not None else None


def register_engine_modes(engine, wgrad_rounding_mode: Optional[str], policy: Optional[str]) -> None:
    """Validate an engine's own modes (None: follow the global setting)."""
    global _selective_engines
    if wgrad_rounding_mode is not None and wgrad_rounding_mode not in WGRAD_ROUNDINGS:
        raise ValueError(f"wgrad rounding {wgrad_rounding_mode!r}: one of {WGRAD_ROUNDINGS}")
    if policy is not None and policy not in ACTIVATION_POLICIES:
        raise ValueError(f"activation policy {policy!r}: one of {ACTIVATION_POLICIES}")
    if policy == "selective":
        import weakref
        _selective_engines += 1

        def _done():
            global _selective_engines
            _selective_engines -= 1
        weakref.finalize(engine, _done)


def tag_recompute(out: torch.Tensor, op: int, a2d: torch.Tensor, b2d: Optional[torch.Tensor] = None,
                  weight: Optional[torch.Tensor] = None, rstd: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Mark ``out`` (a norm's / SwiGLU's output) as rebuildable from the producer's operands (which
    the producer saves for its own backward anyway); read by linearZ under the "selective" policy."""
    if _activation_policy == "selective" or _selective_engines > 0:
        out._smt_recompute = (out._version, op, a2d, b2d, weight, rstd)
    return out


_NO_DECAY = ["bias", "layer_norm.weight", "layernorm.weight", "norm.weight", "ln_f.weight"]


# ------------------------------------------------------------------------------------------------
# naming helpers (the inline expressions of smt.py:105-107, 121-125, 651-653, 726-729)
# ------------------------------------------------------------------------------------------------
def recursive_getattr(model: nn.Module, module_name: str):
    """Same contract as deepspeed.compression.helper.recursive_getattr (imported at smt.py:1)."""
    output = model
    for name in module_name.split('.'):
        output = getattr(output, name)
    return output


def recursive_setattr(model: nn.Module, module_name: str, module: nn.Module) -> None:
    """Same contract as deepspeed.compression.helper.recursive_setattr (imported at smt.py:1)."""
    split_list = module_name.split('.')
    output = model
    for name in split_list[:-1]:
        output = getattr(output, name)
    output.__setattr__(split_list[-1], module)


def _mlp_module_name(name: str) -> str:
    return 'gate_proj' if 'gate_proj' in name else 'up_proj' if 'up_proj' in name else 'down_proj'


def _attn_module_name(name: str) -> Optional[str]:
    return ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
            'v_proj' if 'v_proj' in name else 'o_proj' if 'o_proj' in name else None)


def _layer_number(name: str) -> Optional[int]:
    match = _LAYER_PATTERN.search(name)
    return int(match.group(1)) if match else None


# ------------------------------------------------------------------------------------------------
# tile index: the reference's Python list plus its device copy
# ------------------------------------------------------------------------------------------------
class TileIndex:
    """``index_list`` of smt.py:310 (list of ``(row_block, col_block)`` in selection order) with a
    cached device ``int32 [n, 2]`` table for the kernels."""

    def __init__(self, index_list: Iterable[Sequence[int]]):
        self.index_list: List[Tuple[int, int]] = [(int(i[0]), int(i[1])) for i in index_list]
        self._dev = {}

    def __len__(self) -> int:
        return len(self.index_list)

    def __iter__(self):
        return iter(self.index_list)

    def __getitem__(self, i):
        return self.index_list[i]

    def device_table(self, device: torch.device) -> torch.Tensor:
        key = (device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            t = _hip.tile_table(self.index_list, device)
            self._dev[key] = t
        return t

    def column_blocks(self) -> List[int]:
        """Distinct column blocks of the tiles, in order of first use."""
        seen = {}
        for _r, c in self.index_list:
            seen.setdefault(c, len(seen))
        return list(seen)

    def packed_tables(self, device: torch.device, col_pos: Optional[dict] = None):
        """Device tables for the packed-input backward: int32 [n_cb] column blocks and the int32
        [n, 2] table of (row_block, position of the column block in the packed input). With
        ``col_pos`` the positions in a :class:`ColumnBlockGroup`'s shared copy (the group's blocks)."""
        if col_pos is not None:
            key = ("packed_grp", id(col_pos), device.type, device.index)
            e = self._dev.get(key)
            if e is None or e[0] is not col_pos:
                e = self._dev[key] = (col_pos, (None, _hip.tile_table(self.kernel_tiles(col_pos), device)))
            return e[1]
        key = ("packed", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            cbs = self.column_blocks()
            pos = {c: i for i, c in enumerate(cbs)}
            t = (torch.tensor(cbs, dtype=torch.int32).to(device),
                 _hip.tile_table([(r, pos[c]) for r, c in self.index_list], device))
            self._dev[key] = t
        return t

    def kernel_tiles(self, packed) -> List[Tuple[int, int]]:
        """The ``(row_block, col_block)`` list as the wgrad kernel addresses the input: for the
        block-major packed input of ``colblock_gather`` the column block is its position there
        (``packed`` True: this module's own copy; a dict: a group's column-block positions)."""
        if isinstance(packed, dict):
            key = ("ktiles_grp", id(packed))
            e = self._dev.get(key)
            if e is None or e[0] is not packed:
                e = self._dev[key] = (packed, [(r, packed[c]) for r, c in self.index_list])
            return e[1]
        key = ("ktiles", bool(packed))
        t = self._dev.get(key)
        if t is None:
            if packed:
                pos = {c: i for i, c in enumerate(self.column_blocks())}
                t = [(r, pos[c]) for r, c in self.index_list]
            else:
                t = list(self.index_list)
            self._dev[key] = t
        return t

    def mx_kernel_tiles(self, col_pos: Optional[dict] = None) -> List[Tuple[int, int]]:
        """Host ``(row-block position, column-block position)`` list of :meth:`mx_tables`; with
        ``col_pos`` the column positions in a group's shared MX input blocks instead of this module's."""
        # the entry holds the map itself: an id() of a map that was dropped could be reused
        key = ("mx_ktiles", id(col_pos))
        e = self._dev.get(key)
        if e is None or e[0] is not col_pos:
            rbs = {}
            for r, _c in self.index_list:
                rbs.setdefault(r, len(rbs))
            pos = col_pos if col_pos is not None else {c: i for i, c in enumerate(self.column_blocks())}
            e = self._dev[key] = (col_pos, [(rbs[r], pos[c]) for r, c in self.index_list])
        return e[1]

    def mx_group_table(self, col_pos: dict, device: torch.device) -> torch.Tensor:
        """Device int32 [n, 2] table of :meth:`mx_kernel_tiles` against a group's shared blocks."""
        key = ("mx_group", id(col_pos), device.type, device.index)
        e = self._dev.get(key)
        if e is None or e[0] is not col_pos:
            e = self._dev[key] = (col_pos, _hip.tile_table(self.mx_kernel_tiles(col_pos), device))
        return e[1]

    def block_tables(self, device: torch.device):
        """Device int32 tables of the distinct row blocks and column blocks the tiles touch."""
        key = ("blocks", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            rows = sorted({r for r, _c in self.index_list})
            t = (torch.tensor(rows, dtype=torch.int32).to(device),
                 torch.tensor(sorted(self.column_blocks()), dtype=torch.int32).to(device))
            self._dev[key] = t
        return t

    def mx_tables(self, device: torch.device):
        """Device tables of the MX-fp8 wgrad (fp8 path): int32 [n_rb] row blocks, int32 [n_cb] column
        blocks (both in order of first use) and the int32 [n, 2] table of (row-block position,
        column-block position)."""
        key = ("mx", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            rbs = {}
            for r, _c in self.index_list:
                rbs.setdefault(r, len(rbs))
            cbs = self.column_blocks()
            pos = {c: i for i, c in enumerate(cbs)}
            t = (torch.tensor(list(rbs), dtype=torch.int32).to(device),
                 torch.tensor(cbs, dtype=torch.int32).to(device),
                 _hip.tile_table([(rbs[r], pos[c]) for r, c in self.index_list], device))
            self._dev[key] = t
        return t

    def mx_row_pack(self, out_features: int, device: torch.device):
        """``(n_rb, int32 [out_features / 256] map)`` for an output gradient written packed by its
        producer (``smt_swiglu_bwd_quant_e4m3_packed``): row block ``rb`` of :meth:`mx_tables` (position
        i) goes to columns ``256 i ..``, every other block is not written (-1)."""
        key = ("mx_pack", out_features, device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            pos = [-1] * (out_features // Block_dimension)
            n = 0
            for r, _c in self.index_list:
                if pos[r] < 0:
                    pos[r] = n
                    n += 1
            t = self._dev[key] = (n, torch.tensor(pos, dtype=torch.int32).to(device),
                                  torch.arange(n, dtype=torch.int32).to(device))
        return t

    def transposed_descs(self, weight_t: torch.Tensor) -> torch.Tensor:
        """Device smt_tile_desc[] for the transposed write-back of ``selected_weight`` into W^T."""
        key = ("wt", weight_t.data_ptr(), weight_t.device.index)
        t = self._dev.get(key)
        if t is None:
            t = _hip.tile_descs([(weight_t, r, c, i * _hip.TILE_ELEMS) for i, (r, c) in enumerate(self.index_list)],
                                weight_t.device, weight_t.dtype)
            self._dev[key] = t
        return t

    def schedule(self, device: torch.device) -> torch.Tensor:
        """Device int32 schedule permutation for the wgrad kernel (L2 reuse; speed only)."""
        key = ("order", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            t = _hip.order_table(self.index_list, device)
            self._dev[key] = t
        return t

    def validate(self, rows: int, cols: int) -> None:
        rb, cb = rows // Block_dimension, cols // Block_dimension
        for r, c in self.index_list:
            if not (0 <= r < rb and 0 <= c < cb) or rows % Block_dimension or cols % Block_dimension:
                # the reference's slice assignment fails with a shape-mismatch RuntimeError here
                raise RuntimeError(
                    f"tile ({r}, {c}) outside a [{rows}, {cols}] weight in {Block_dimension}-blocks")


def _as_tile_index(index) -> TileIndex:
    return index if isinstance(index, TileIndex) else TileIndex(index)


class ColumnBlockGroup:
    """SMT linears that read ONE input (q/k/v_proj of an attention module, gate/up_proj of an MLP)
    keep one packed copy of the union of the input's column blocks their tiles read, instead of
    one copy per member: the members' blocks overlap (at the 8B bench point q/k/v read ~19 blocks of
    their 16-block input between them, ~12 distinct). The engine sets it on the members' frozen
    weights (``weight._smt_cb_group``); the first member's forward gathers the union, the others
    reuse that copy (same input object and version), and each member's tile table indexes it. Only
    weak references are held here: the members' saved tensors own the copy, so it is freed with
    the last member's backward, as the per-member copies were."""

    def __init__(self, col_blocks, device: torch.device):
        self.col_blocks = sorted({int(c) for c in col_blocks})
        self.pos = {c: i for i, c in enumerate(self.col_blocks)}
        self.cb_dev = torch.tensor(self.col_blocks, dtype=torch.int32).to(device)
        self._cache = None              # (weakref to the input, its version, weakref to the copy)

    def packed_input(self, x: torch.Tensor, x2d: torch.Tensor, sink) -> torch.Tensor:
        c = self._cache
        if c is not None and c[0]() is x and c[1] == x._version:
            p = c[2]()
            if p is not None:
                return p
        p = _off_stream(sink, lambda: _hip.colblock_gather(x2d, self.cb_dev), x2d)
        self._cache = (weakref.ref(x), x._version, weakref.ref(p))
        return p


# ------------------------------------------------------------------------------------------------
# the SMT module (smt.py:302-344)
# ------------------------------------------------------------------------------------------------
class LinearLayer_MatrixSparsity(torch.nn.Module):
    """Frozen dense ``W`` (aliased, not copied, smt.py:307) plus the trainable 256x256 tiles
    ``selected_weight [n*256, 256]`` listed in ``index_list`` (smt.py:312-327)."""

    def __init__(self, weight, bias=None, index_list=[]):
        super().__init__()
        self.weight = weight
        self.weight.requires_grad = False
        self.bias = bias
        self.tiles = _as_tile_index(index_list)
        self.index_list = self.tiles.index_list
        # True: write the tiles into W at every forward (smt.py:332-341). The SMT engine clears it
        # because its fused AdamW already scatters the updated tiles into W.
        self.writeback_on_forward = True

        w = self.weight.data
        n = len(self.tiles)
        dev = w.device
        if dev.type not in ("cuda", "meta"):
            raise RuntimeError(
                f"LinearLayer_MatrixSparsity: weight on {dev}; the SMT path runs on ROCm devices only")
        if w.dim() != 2:
            raise RuntimeError(f"LinearLayer_MatrixSparsity: 2-D weight expected, got {tuple(w.shape)}")
        self.tiles.validate(w.shape[0], w.shape[1])
        selected = torch.empty(n * Block_dimension, Block_dimension, dtype=w.dtype, device=dev)
        if dev.type == "cuda" and n:
            _hip.tile_gather(w, self.tiles.device_table(dev), selected)
        self.selected_weight = nn.Parameter(selected, requires_grad=True)
        self.fn = linearZ.apply

    def sync_weight(self) -> None:
        """Scatter the tiles into W (smt.py:332-341) with one launch, and into W's transposed copy
        when the data-gradient GEMM uses one (:func:`..engine.attach_transposed_weights`)."""
        w = self.weight.data
        if len(self.tiles) and w.device.type == "cuda":
            _hip.tile_scatter(w, self.tiles.device_table(w.device), self.selected_weight.data)
            wt = getattr(self.weight, "_smt_weight_t", None)
            if wt is not None:
                descs = self.tiles.transposed_descs(wt)
                _hip.tile_scatter_t(descs, len(self.tiles), self.selected_weight.data)
            fw = getattr(self.weight, "_smt_fp8", None)
            if fw is not None:
                rb, cb = self.tiles.block_tables(w.device)
                fw.refresh(w, rb, cb)

    def forward(self, x):
        if self.writeback_on_forward:
            self.sync_weight()
        if not torch.is_grad_enabled():
            # nothing to save for a backward: linearZ.forward's 3-D check and matmul only
            if len(self.tiles) and x.dim() != 3:
                raise IndexError(f"too many indices for tensor of dimension {x.dim()}")
            return _dense_forward(x, self.weight)
        return self.fn(x, self.selected_weight, self.tiles, self.weight)

    def extra_repr(self) -> str:
        return f"in_features={self.weight.shape[1]}, out_features={self.weight.shape[0]}, tiles={len(self.tiles)}"


SMTLinear = LinearLayer_MatrixSparsity


def _dense_forward(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """``x @ W^T`` (smt.py:366): bf16 hipBLASLt, or the e4m3 copy when the fp8 path attached one."""
    fw = getattr(weight, "_smt_fp8", None)
    if fw is not None:
        from ..fp8 import fp8_linear_forward
        return fp8_linear_forward(x, fw)
    return torch.matmul(x, weight.t())


def _rows_ready(t: torch.Tensor) -> torch.Tensor:
    """2-D row-major with 16-byte aligned rows, else a contiguous copy."""
    if t.stride(1) != 1 or t.stride(0) % 8 or t.data_ptr() % 16:
        return t.contiguous()
    return t


def _off_stream(sink, make, *reads: torch.Tensor):
    """Run ``make()`` (the copy / quantisation of the input blocks linearZ keeps for its tile
    gradient) on the engine's wgrad stream when there is one: its only consumer is the tile-gradient
    launch on that stream, so the forward's critical path does not wait for it. The stream first waits
    for the current one (the input is written there); ``reads`` are held for the caching allocator
    until the wgrad stream has passed them."""
    side = None
    if sink is not None and sink.engine is not None:
        side = sink.engine.wgrad_stream
    if side is None:
        return make()
    cur = torch.cuda.current_stream(side.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        out = make()
    for t in reads:
        t.record_stream(side)
    return out


def _recompute_source(input: torch.Tensor):
    """The producer operands ``tag_recompute`` attached to ``input`` (None if absent or if ``input``
    was modified in place since), with their versions for the backward's check."""
    src = input.__dict__.get("_smt_recompute")
    if src is None or src[0] != input._version:
        return None
    ops = src[2:]
    return src[1], ops, tuple(None if t is None else t._version for t in ops)


def _recompute_blocks(rec, cb_dev: torch.Tensor) -> torch.Tensor:
    op, (a2d, b2d, w, rstd), versions = rec
    if any(t is not None and t._version != v for t, v in zip((a2d, b2d, w, rstd), versions)):
        raise RuntimeError("linearZ (selective activation policy): an operand of the input's producer was "
                           "modified in place after the forward; its column blocks cannot be rebuilt")
    return _hip.colblock_recompute(op, a2d, cb_dev, b2d=b2d, weight=w, rstd=rstd)


class linearZ(torch.autograd.Function):
    """``y = x @ W^T`` (smt.py:350-373); backward returns ``(grad_input, grad_tiles, None, None)``
    (smt.py:376-413) with every tile's gradient from one grouped MFMA launch.

    What the forward keeps for the backward: the reference keeps views of the input's column
    slices (``ctx.list1``, smt.py:351-358), which hold the whole input alive. Here, when the tiles
    touch at most half of the input's 256-column blocks, one ``smt_colblock_gather`` launch packs
    exactly those blocks into a ``[T, n_cb*256]`` copy and the input itself is not saved (for a
    down_proj with ~14 tiles that is 14 of its 56 blocks); otherwise the input is saved as is.
    Members of a :class:`ColumnBlockGroup` (q/k/v_proj, gate/up_proj under the engine) share ONE
    packed copy of the union of their blocks, or the input itself when the union covers it. Under
    the "views" activation policy the input is always saved as is (the reference's own choice), and
    under "selective" a norm's / SwiGLU's output is not saved at all (rebuilt in the backward). The
    tile gradients are bit-identical every way (same operands, same kernel, same order). The packed
    copies are of 16-bit inputs; an fp32 model (the reference's --dtype fp32) keeps its input as is.
    Operands may be bf16, fp16 or fp32 (``fine_tune.py:955-959``): the tile gradients are computed in
    that dtype's arithmetic (per-sample partials rounded to it, smt.py:397-404) by the same launches.

    If ``selected_weight`` carries an engine gradient sink (``_smt_grad_sink``), the fp32 tile
    gradients are written straight into the engine's packed buffer and ``None`` is returned for
    ``selected_weight`` (the engine, not autograd, owns those gradients)."""

    @staticmethod
    def forward(ctx, input, selected_weight, matrix_index_list, weight):
        tiles = _as_tile_index(matrix_index_list)
        if len(tiles) and input.dim() != 3:
            # smt.py:354-356 slices input[:, :, cols]; anything but 3-D fails there
            raise IndexError(f"too many indices for tensor of dimension {input.dim()}")
        ctx.tiles = tiles
        ctx.sink = getattr(selected_weight, "_smt_grad_sink", None)
        # the engine's own modes when its config names them, else the global ones
        engine_rounding = _engine_mode(ctx.sink, "wgrad_rounding")
        rounding = engine_rounding or _wgrad_rounding
        policy = _engine_mode(ctx.sink, "activation_policy") or _activation_policy
        # reference rounding: each of the input's B sequences (S rows) is one sample of smt.py:397-404
        ctx.seq_len = int(input.shape[1]) if (rounding == "reference" and len(tiles)) else None
        ctx.packed = False
        ctx.mx = None
        ctx.mx_pos = None
        saved = input
        in_blocks = weight.shape[1] // Block_dimension
        fw = getattr(weight, "_smt_fp8", None)
        if (fw is not None and fw.mx_wgrad and ctx.needs_input_grad[1] and len(tiles)
                and input.device.type == "cuda"):
            # fp8 path: the tile weight gradient runs on MX-fp8 operands; keep only the input's
            # column blocks, quantised (half the bytes of the bf16 blocks)
            if engine_rounding == "reference":
                # the MX kernel sums e4m3 products over all T rows: it has no per-sample bf16 partials
                raise RuntimeError("linearZ: the reference wgrad rounding (smt.py:397-404) exists on the bf16 tile "
                                   "path only; with fp8 weights set SMT_FP8_TILE_WGRAD=bf16 or use rounding 'single'")
            # the global mode is the bf16 tiles' (the reference has no fp8 path whose rounding to follow)
            ctx.seq_len = None
            grp = fw.group
            x2d = _rows_ready(input.reshape(-1, weight.shape[1]))
            if grp is not None and grp.mx_union is not None:
                # q/k/v (gate/up) read one input: its MX blocks are quantised once for the group's
                # union of column blocks and shared
                ctx.mx = _off_stream(ctx.sink, lambda: grp.mx_input_blocks(input, x2d), x2d)
                ctx.mx_pos = grp.mx_union[1]
            else:
                _rb, cb_dev, _table = tiles.mx_tables(input.device)
                ctx.mx = _off_stream(ctx.sink, lambda: _hip.mx_quant_cols(x2d, cb_dev), x2d)
                ctx.mx_pos = None
            saved = None
        elif (policy == "selective" and ctx.needs_input_grad[1] and len(tiles)
                and input.device.type == "cuda" and _recompute_source(input) is not None):
            # rebuilt in the backward from the producer's saved operands: nothing kept here
            ctx.recompute = _recompute_source(input)
            saved = None
            ctx.packed = True
        elif (policy != "views" and ctx.needs_input_grad[1] and len(tiles) and input.device.type == "cuda"
                and input.element_size() == 2 and getattr(weight, "_smt_cb_group", None) is not None
                and len(weight._smt_cb_group.col_blocks) < in_blocks
                and all(c in weight._smt_cb_group.pos for c in tiles.column_blocks())):
            # one packed copy of the group's union of column blocks, shared with the other members
            grp = weight._smt_cb_group
            x2d = _rows_ready(input.reshape(-1, weight.shape[1]))
            saved = grp.packed_input(input, x2d, ctx.sink)
            ctx.packed = grp.pos
        elif (policy != "views" and ctx.needs_input_grad[1] and len(tiles) and input.device.type == "cuda"
                and input.element_size() == 2 and (getattr(weight, "_smt_cb_group", None) is None
                     or not all(c in weight._smt_cb_group.pos for c in tiles.column_blocks()))
                and 2 * len(tiles.column_blocks()) <= in_blocks):
            cb_dev, _ = tiles.packed_tables(input.device)
            x2d = _rows_ready(input.reshape(-1, weight.shape[1]))
            saved = _off_stream(ctx.sink, lambda: _hip.colblock_gather(x2d, cb_dev), x2d)
            ctx.packed = True
        ctx.save_for_backward(saved, weight)
        # q/k/v (gate/up) share their input: their data gradients accumulate in one buffer (bf16)
        # or run as one joint GEMM (fp8 group)
        if fw is None:
            ctx.acc = dgrad.register(input, ctx)
        else:
            from .. import fp8
            ctx.acc = fp8.register_group(input, fw, ctx)
            # the tile weight gradient reads the bf16 output gradient: ask the consumer for it (only
            # the row blocks the MX tiles read, packed, from a producer that can write them so)
            need = fp8.MxRowsNeed(tiles) if ctx.mx is not None and fp8.packed_rows_allowed() else True
            ctx.mx_need = need if need is not True else None
            return fp8.tag_group_output(_dense_forward(input, weight), ctx.acc, fw, need)
        return _dense_forward(input, weight)

    @staticmethod
    def backward(ctx, grad_output):
        saved, weight = ctx.saved_tensors
        tiles = ctx.tiles
        n = len(tiles)
        grad_input = grad_weight = None
        if ctx.needs_input_grad[1] and ctx.mx is not None:
            packed = grad_output.__dict__.get("_smt_gpack")
            need = getattr(ctx, "mx_need", None)
            if need is not None and need.__dict__.pop("delivered", False) and packed is None:
                # the producer wrote only the packed row blocks and left a zero placeholder, but
                # autograd summed that placeholder with another consumer's gradient: the packed
                # blocks never arrived here, and the tile gradient would silently miss them
                raise RuntimeError("linearZ (fp8, MX tile gradient): the packed output gradient was summed "
                                   "with another consumer's gradient; set SMT_FP8_PACK_SWIGLU_GRAD=0 when a "
                                   "gate/up output has more than one consumer")
            if packed is not None:
                # only this module's row blocks, packed in mx_tables order (fp8.swiglu_bwd_quant)
                g2 = packed
                table = tiles.mx_tables(g2.device)[2]
                rb_dev = tiles.mx_row_pack(weight.shape[0], g2.device)[2]
            else:
                g2 = _rows_ready(grad_output.reshape(-1, weight.shape[0]))
                rb_dev, _cb, table = tiles.mx_tables(g2.device)
            if ctx.mx_pos is not None:
                table = tiles.mx_group_table(ctx.mx_pos, g2.device)
            sink = ctx.sink
            if sink is not None and sink.batcher() is not None:
                # quantised and launched with the modules whose backward runs next (one
                # smt_tile_wgrad_mx_batch launch)
                sink.batcher().add_mx(sink, g2, rb_dev, ctx.mx, tiles, ctx.mx_pos)
            elif sink is not None:
                acc, mx, order = sink.take_accumulate(), ctx.mx, tiles.schedule(g2.device)
                sink.run(lambda: _hip.tile_wgrad_mx(_hip.mx_quant_cols(g2, rb_dev), mx, table, sink.buffer,
                                                    accumulate=acc, order=order),
                         g2, mx.q, mx.scales)
                sink.mark_ready()
            else:
                grad_weight = torch.empty(n * Block_dimension, Block_dimension,
                                          dtype=grad_output.dtype, device=grad_output.device)
                _hip.tile_wgrad_mx(_hip.mx_quant_cols(g2, rb_dev), ctx.mx, table, grad_weight,
                                   order=tiles.schedule(g2.device))
            ctx.mx = None
        elif ctx.needs_input_grad[1]:
            out_f = weight.shape[0]
            g2 = _rows_ready(grad_output.reshape(-1, out_f))
            dev = g2.device
            if getattr(ctx, "recompute", None) is not None:
                cb_dev, table = tiles.packed_tables(dev)
                rec, ctx.recompute = ctx.recompute, None
                # rebuilt on the wgrad stream, like the forward's block copies: its only consumer is
                # the tile-gradient launch there, so the data-gradient GEMMs do not wait for it
                x2 = _off_stream(ctx.sink, lambda: _recompute_blocks(rec, cb_dev),
                                 *[t for t in rec[1] if t is not None])
            elif ctx.packed:
                x2 = saved
                table = tiles.packed_tables(dev, ctx.packed if isinstance(ctx.packed, dict) else None)[1]
            else:
                x2, table = _rows_ready(saved.reshape(-1, weight.shape[1])), tiles.device_table(dev)
            sink = ctx.sink
            if sink is not None and sink.batcher() is not None:
                # the engine launches this module's tiles together with those of the modules whose
                # backward runs next (one smt_tile_wgrad_batch launch, deterministic)
                sink.batcher().add(sink, g2, x2, tiles, ctx.packed, ctx.seq_len)
            elif sink is not None:
                acc, order, seq = sink.take_accumulate(), tiles.schedule(dev), ctx.seq_len
                sink.run(lambda: _hip.tile_wgrad(g2, x2, table, sink.buffer, accumulate=acc, order=order,
                                                 seq_len=seq), g2, x2)
                sink.mark_ready()
            else:
                grad_weight = torch.empty(n * Block_dimension, Block_dimension,
                                          dtype=grad_output.dtype, device=grad_output.device)
                if n:
                    _hip.tile_wgrad(g2, x2, table, grad_weight, order=tiles.schedule(dev), seq_len=ctx.seq_len)
        if ctx.needs_input_grad[0]:
            wt = getattr(weight, "_smt_weight_t", None)
            fw = getattr(weight, "_smt_fp8", None)
            # g @ W (smt.py:406); with a transposed copy as the TN product g @ (W^T)^T, the layout
            # hipBLASLt runs 13-19 % faster on these shapes (profiles/r01_gemm_layout.jsonl); on the
            # fp8 path through W's transposed e4m3 copy
            if fw is not None:
                from ..fp8 import fp8_input_grad
                grad_input = fp8_input_grad(ctx.acc, fw, grad_output)
            else:
                grad_input = dgrad.input_grad(ctx.acc, grad_output, weight if wt is None else wt.t())
        return grad_input, grad_weight, None, None


# ------------------------------------------------------------------------------------------------
# model surgery (smt.py:83-179, 416-457, 641-745)
# ------------------------------------------------------------------------------------------------
def _replace(model, name, index_list):
    module = recursive_getattr(model, name)
    tmp = LinearLayer_MatrixSparsity(module.weight, bias=None, index_list=index_list).to(
        module.weight.device).to(module.weight.dtype)
    recursive_setattr(model, name, tmp)


def convert_linear_layer_to_matrix_sparsity(model,
                                            selected_submatrix,
                                            selected_submatrix_attention,
                                            part_module_name=['.layers'],
                                            mixture=False):
    """smt.py:83-179. Replace every trainable ``nn.Linear`` under ``part_module_name`` by an SMT
    module holding its selected tiles; keys are ``(module_name, layer)`` with the layer read by the
    regex ``model\\.layers\\.(\\d+)\\.`` (``None`` when it does not match). Biases are dropped."""
    replace_name = []
    for name, module in model.named_modules():
        if isinstance(module, nn.Linear) and any(part in name for part in part_module_name):
            replace_name.append(name)

    for name in replace_name:
        if "mlp" in name:
            module = recursive_getattr(model, name)
            if module.weight.requires_grad:
                key = (_mlp_module_name(name), _layer_number(name))
                _replace(model, name, selected_submatrix[key])
        if "self_attn" in name:
            module = recursive_getattr(model, name)
            if module.weight.requires_grad:
                key = (_attn_module_name(name), _layer_number(name))
                src = selected_submatrix if mixture else selected_submatrix_attention
                _replace(model, name, src[key])
        if mixture and "embed_tokens" in name:
            module = recursive_getattr(model, name)
            if module.weight.requires_grad:
                _replace(model, name, selected_submatrix[('embed_tokens', None)])
    return model


def convert_matrix_sparsity_to_linear_layer(model, part_module_name=['.layers']):
    """smt.py:416-457: scatter each module's tiles into W and swap back a bias-free ``nn.Linear``
    that shares ``W`` (no copy)."""
    replace_name = []
    for name, module in model.named_modules():
        if isinstance(module, LinearLayer_MatrixSparsity) and any(part in name for part in part_module_name):
            replace_name.append(name)
    for name in replace_name:
        module = recursive_getattr(model, name)
        module.sync_weight()
        for attr in ("_smt_weight_t", "_smt_fp8"):
            if hasattr(module.weight, attr):
                delattr(module.weight, attr)
        weight_shape = module.weight.shape
        new_linear = nn.Linear(weight_shape[1], weight_shape[0], bias=False, device="meta")
        new_linear.weight = module.weight
        recursive_setattr(model, name, new_linear)
        del module
    return model


def freeze_unselected_matrix_layer(model,
                                   select_parameters,
                                   select_attention_parameters,
                                   mixture=False,
                                   layernorm=False):
    """smt.py:641-745: ``requires_grad`` is True exactly for the parameters of selected
    ``(module, layer)`` keys (plus layernorms / embed_tokens in mixture mode)."""
    for name, param in model.named_parameters():
        if mixture:
            if "mlp" in name:
                param.requires_grad = (_mlp_module_name(name), _layer_number(name)) in select_parameters.keys()
            elif "self_attn" in name:
                param.requires_grad = (_attn_module_name(name), _layer_number(name)) in select_parameters.keys()
            elif "embed_tokens" in name:
                param.requires_grad = ('embed_tokens', None) in select_parameters.keys()
            elif ("input_layernorm" in name) or ("post_attention_layernorm" in name):
                param.requires_grad = bool(layernorm)
            else:
                param.requires_grad = False
        else:
            if "mlp" in name:
                param.requires_grad = (_mlp_module_name(name), _layer_number(name)) in select_parameters.keys()
            elif "self_attn" in name:
                param.requires_grad = (_attn_module_name(name), _layer_number(name)) in select_attention_parameters.keys()
            else:
                param.requires_grad = False
    return model


# ------------------------------------------------------------------------------------------------
# optimizer parameter groups (smt.py:465-549, 554-638)
# ------------------------------------------------------------------------------------------------
def _groups(model, weight_decay, lr0, lr1, special, no_decay):
    named = list(model.named_parameters())
    no_decay = list(_NO_DECAY if no_decay is None else no_decay)
    groups = [
        {"params": [p for n, p in named if not any(nd in n.lower() for nd in no_decay)
                    and p.requires_grad and not any(nd in n.lower() for nd in special)],
         "weight_decay": weight_decay, "lr": lr0},
        {"params": [p for n, p in named if not any(nd in n.lower() for nd in no_decay)
                    and p.requires_grad and any(nd in n.lower() for nd in special)],
         "weight_decay": weight_decay, "lr": lr1},
        {"params": [p for n, p in named if any(nd in n.lower() for nd in no_decay) and p.requires_grad],
         "weight_decay": 0.0},
    ]
    return [g for g in groups if g["params"]]


def get_optimizer_sparse_grouped_parameters(
    model,
    weight_decay,
    smt_lr,
    lora_lr=5e-4,
    no_decay_name_list=None,
    lora_name_list=("lora_right_weight", "lora_left_weight"),
):
    """smt.py:465-549: group 0 = trainable non-norm params at ``smt_lr``; empty groups dropped.
    ``no_decay_name_list=None`` means the reference default (bias / *norm.weight / ln_f.weight)."""
    return _groups(model, weight_decay, smt_lr, lora_lr, lora_name_list, no_decay_name_list)


def get_optimizer_qk_augment_grouped_parameters(
    model,
    weight_decay,
    ft_learning_rate,
    module_lr=5e-4,
    no_decay_name_list=None,
    module_name_list=("q_proj", "k_proj"),
):
    """smt.py:554-638: q/k projections get ``module_lr`` (warm-up only, fine_tune.py:160-163)."""
    return _groups(model, weight_decay, ft_learning_rate, module_lr, module_name_list, no_decay_name_list)


# ------------------------------------------------------------------------------------------------
# channel-sparsity path (smt.py:25-80, 185-296, 748-831): SURVEY §8(f) row 1
# ------------------------------------------------------------------------------------------------
class ChannelIndex:
    """``index_list`` of smt.py:186-196 (row / channel indices in selection order) with cached
    device tables: the int32 index table and the all-tiles table of the channel wgrad."""

    def __init__(self, index_list: Iterable[int]):
        self.index_list: List[int] = [int(i) for i in index_list]
        self._dev = {}

    def __len__(self) -> int:
        return len(self.index_list)

    def __iter__(self):
        return iter(self.index_list)

    def __getitem__(self, i):
        return self.index_list[i]

    @property
    def padded(self) -> int:
        """Channel count rounded up to whole 256-blocks (the wgrad operand width)."""
        return -(-len(self.index_list) // Block_dimension) * Block_dimension

    def device_table(self, device: torch.device) -> torch.Tensor:
        key = ("idx", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            t = _hip.index_table(self.index_list, device)
            self._dev[key] = t
        return t

    def long_index(self, device: torch.device) -> torch.Tensor:
        """int64 device index (torch indexing ops: the column write into a transposed W copy)."""
        key = ("long", device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            t = self._dev[key] = torch.tensor(self.index_list, dtype=torch.int64).to(device)
        return t

    def wgrad_tiles(self, out_features: int, device: torch.device) -> torch.Tensor:
        """int32 [(k_pad/256) * (out/256), 2] table covering the [k_pad, out] channel gradient."""
        key = ("tiles", out_features, device.type, device.index)
        t = self._dev.get(key)
        if t is None:
            rc = [(r, c) for r in range(self.padded // Block_dimension)
                  for c in range(out_features // Block_dimension)]
            t = _hip.tile_table(rc, device)
            self._dev[key] = t
        return t

    def validate(self, rows: int) -> None:
        seen = set()
        for i in self.index_list:
            if not -rows <= i < rows:
                # W.data[index, :] in smt.py:203 raises exactly this
                raise IndexError(f"index {i} is out of bounds for dimension 0 with size {rows}")
            if i % rows in seen:
                raise ValueError(f"channel index {i} repeated: the row write-back (smt.py:211-213) would "
                                 "depend on write order")
            seen.add(i % rows)
        self.index_list = [i % rows for i in self.index_list]


def _as_channel_index(index) -> ChannelIndex:
    return index if isinstance(index, ChannelIndex) else ChannelIndex(index)


class ChannelGatherGroup:
    """Channel modules that read ONE input (q/k/v_proj of a layer): their partial inputs
    ``x[:, :, index_list]`` (smt.py:225-233) come from one ``smt_column_gather`` launch into a joint
    ``[T, sum of padded widths]`` buffer, the members' blocks side by side, and each member keeps a
    column-slice view of it. The input rows are read once instead of once per member (a whole row is
    fetched either way: the selected channels touch every 64-B granule). A column index of -1 in the
    joint table writes a zero: each member's block is zero-padded to whole 256-column blocks exactly
    as its own gather pads it, so the tile gradients are bit-identical."""

    def __init__(self, channels: Sequence[ChannelIndex], device: torch.device):
        self.members = list(channels)          # the ChannelIndex objects the joint table was built from
        cols, self.offsets, off = [], [], 0
        for ch in channels:
            cols.extend(ch.index_list)
            cols.extend([-1] * (ch.padded - len(ch)))
            self.offsets.append((off, ch.padded))
            off += ch.padded
        self.width = off
        self.table = _hip.index_table(cols, device)
        # (weakref to the input, its version, weakref to the joint buffer): weak references only, as
        # ColumnBlockGroup holds its copy, so the joint buffer lives exactly as long as a member's
        # saved view of it (until the last member's backward), whoever else keeps the input alive
        self._cache = None

    def partial(self, input: torch.Tensor, x2: torch.Tensor, member: int) -> torch.Tensor:
        """Member ``member``'s ``[T, padded]`` partial input: a view of the joint gather of ``input``,
        made by the first member that asks for it (reused while the input and its version hold)."""
        c = self._cache
        joint = c[2]() if (c is not None and c[0]() is input and c[1] == input._version) else None
        if joint is None:
            joint = _hip.column_gather(x2, self.table, self.width, self.width)
            self._cache = (weakref.ref(input), input._version, weakref.ref(joint))
        off, width = self.offsets[member]
        return joint[:, off:off + width]


class LinearLayer_ChannelSparsity(torch.nn.Module):
    """smt.py:185-214: frozen dense ``W`` (aliased) plus the trainable rows
    ``selected_weight[i, :] = W[index_list[i], :]``; every forward writes the rows back into ``W``
    (one launch) and runs :class:`linearChannel`."""

    def __init__(self, weight, bias=None, index_list=[]):
        super().__init__()
        self.weight = weight
        self.weight.requires_grad = False
        self.bias = bias
        self.channels = _as_channel_index(index_list)
        w = self.weight.data
        dev = w.device
        if dev.type not in ("cuda", "meta"):
            raise RuntimeError(
                f"LinearLayer_ChannelSparsity: weight on {dev}; the SMT path runs on ROCm devices only")
        if w.dim() != 2:
            raise RuntimeError(f"LinearLayer_ChannelSparsity: 2-D weight expected, got {tuple(w.shape)}")
        self.channels.validate(w.shape[0])
        self.index_list = self.channels.index_list
        self.writeback_on_forward = True
        k = len(self.channels)
        selected = torch.empty(k, w.shape[1], dtype=w.dtype, device=dev)
        if dev.type == "cuda" and k:
            _hip.row_gather(w, self.channels.device_table(dev), selected)
        self.selected_weight = nn.Parameter(selected, requires_grad=True)
        self.fn = linearChannel.apply

    def sync_weight(self) -> None:
        """Scatter the rows into W (smt.py:208-213) with one launch, and into the columns of the
        transposed copy W^T when the engine attached one (the data gradient's TN operand)."""
        w = self.weight.data
        if len(self.channels) and w.device.type == "cuda":
            table = self.channels.device_table(w.device)
            _hip.row_scatter(w, table, self.selected_weight.data)
            wt = getattr(self.weight, "_smt_weight_t", None)
            if wt is not None:
                wt.index_copy_(1, self.channels.long_index(w.device), self.selected_weight.data.t())

    def forward(self, x):
        if self.writeback_on_forward:
            self.sync_weight()
        return self.fn(x, self.selected_weight, self.channels, self.weight)

    def extra_repr(self) -> str:
        return f"in_features={self.weight.shape[1]}, out_features={self.weight.shape[0]}, channels={len(self.channels)}"


class linearChannel(torch.autograd.Function):
    """smt.py:217-296. Forward: ``y = x @ W^T``, saving only ``partial_input = x[:, :, index_list]``
    (one gather launch) and ``W``. Backward: ``grad_input = g @ W`` and, as the reference computes
    it, ``grad_weight = sum_b partial_input[b]^T g[b]`` of shape ``[k, out]`` — the tile wgrad
    kernel over the all-tiles grid of the zero-padded ``[T, k_pad]`` operand, then one scatter into
    the dense layout.

    The reference's gradient is ``[k, out]`` while its parameter is ``[k, in]`` (rows of ``W``):
    it only runs for square ``W``, and then it applies the gradient of *column* ``idx`` of ``W`` to
    *row* ``idx``. Both are reproduced: non-square ``W`` raises the same
    autograd shape error, square ``W`` gets the reference's gradient. The batch sum is fp32 with one
    rounding (the reference rounds each per-sample product to bf16 first)."""

    @staticmethod
    def forward(ctx, input, selected_weight, channel_index_list, weight):
        ch = _as_channel_index(channel_index_list)
        if input.dim() != 3:
            # smt.py:226-233 builds [input.shape[0], input.shape[1], k] and slices input[:, :, index]
            raise IndexError(f"too many indices for tensor of dimension {input.dim()}")
        ctx.channels = ch
        ctx.shape = input.shape
        partial = None
        if ctx.needs_input_grad[1] and len(ch):
            x2 = _rows_ready(input.reshape(-1, input.shape[-1]))
            grp = getattr(weight, "_smt_cgather", None)
            if grp is not None and grp[0].members[grp[1]] is ch:
                # q/k/v of a layer: one gather for the group (engine.attach_channel_gather_groups)
                partial = grp[0].partial(input, x2, grp[1])
            else:
                partial = _hip.column_gather(x2, ch.device_table(x2.device), len(ch), ch.padded)
        ctx.save_for_backward(partial, weight)
        # q/k/v share their input: their data gradients accumulate in one buffer (dgrad.py)
        ctx.acc = dgrad.register(input, ctx)
        return torch.matmul(input, weight.t())

    @staticmethod
    def backward(ctx, grad_output):
        partial, weight = ctx.saved_tensors
        ch = ctx.channels
        out_f, in_f = weight.shape
        grad_input = grad_weight = None
        if ctx.needs_input_grad[1]:
            k = len(ch)
            if out_f != in_f:
                raise RuntimeError(
                    f"Function linearChannelBackward returned an invalid gradient at index 1 - got [{k}, {out_f}] "
                    f"but expected shape compatible with [{k}, {in_f}]")
            if out_f % Block_dimension:
                raise NotImplementedError(f"linearChannel: out_features {out_f} not a multiple of {Block_dimension}")
            grad_weight = torch.empty(k, out_f, dtype=grad_output.dtype, device=grad_output.device)
            if k:
                g2 = grad_output.reshape(-1, out_f)
                if g2.stride(1) != 1 or g2.stride(0) % 8 or g2.data_ptr() % 16:
                    g2 = g2.contiguous()
                dev = g2.device
                table = ch.wgrad_tiles(out_f, dev)
                tiles = torch.empty(table.shape[0] * Block_dimension, Block_dimension, dtype=grad_output.dtype,
                                    device=dev)
                _hip.tile_wgrad(partial, g2, table, tiles)
                dense = torch.empty(ch.padded, out_f, dtype=grad_output.dtype, device=dev)
                _hip.tile_scatter(dense, table, tiles)
                grad_weight = dense[:k]
        if ctx.needs_input_grad[0]:
            # g @ W, as the TN product g @ (W^T)^T when the engine attached the transposed copy
            wt = getattr(weight, "_smt_weight_t", None)
            grad_input = dgrad.input_grad(ctx.acc, grad_output, weight if wt is None else wt.t())
        return grad_input, grad_weight, None, None


def _replace_channel(model, name, index_list):
    module = recursive_getattr(model, name)
    tmp = LinearLayer_ChannelSparsity(module.weight, bias=None, index_list=index_list).to(
        module.weight.device).to(module.weight.dtype)
    recursive_setattr(model, name, tmp)


def convert_linear_layer_to_channel_sparsity(model, selected_channel, selected_channel_attention,
                                             part_module_name=['.layers']):
    """smt.py:25-80: every trainable ``nn.Linear`` under ``part_module_name`` becomes a
    :class:`LinearLayer_ChannelSparsity` with ``selected_channel[(gate|up|down_proj, layer)]`` (MLP)
    or ``selected_channel_attention[(q|k|v|o_proj, layer)]`` (attention). Biases are dropped."""
    replace_name = []
    for name, module in model.named_modules():
        if isinstance(module, nn.Linear) and any(part in name for part in part_module_name):
            replace_name.append(name)
    for name in replace_name:
        if "mlp" in name:
            module = recursive_getattr(model, name)
            if module.weight.requires_grad:
                _replace_channel(model, name, selected_channel[(_mlp_module_name(name), _layer_number(name))])
        if "self_attn" in name:
            module = recursive_getattr(model, name)
            if module.weight.requires_grad:
                key = (_attn_module_name(name), _layer_number(name))
                _replace_channel(model, name, selected_channel_attention[key])
    return model


def freeze_unselected_channel_layer(model, select_parameters, select_attention_parameters, mixture=False):
    """smt.py:748-831. Same as the matrix freeze without the layernorm / embedding branches; the
    attention module name has no ``o_proj`` case (so o_proj is never trainable here), and in
    ``mixture`` mode attention keys are looked up in the MLP selection (smt.py:774-777)."""
    for name, param in model.named_parameters():
        if "mlp" in name:
            param.requires_grad = (_mlp_module_name(name), _layer_number(name)) in select_parameters.keys()
        elif "self_attn" in name:
            mod = ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
                   'v_proj' if 'v_proj' in name else None)
            sel = select_parameters if mixture else select_attention_parameters
            param.requires_grad = (mod, _layer_number(name)) in sel.keys()
        else:
            param.requires_grad = False
    return model

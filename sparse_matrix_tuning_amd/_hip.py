"""ctypes binding of ``libsmt_hip.so`` (C ABI: ``include/smt_hip.h``).

PyTorch is used only as plumbing here: device memory (the caching allocator) and the
current HIP stream. Every compute call below goes to a gfx950 kernel; there is no CPU or
eager-PyTorch fallback. If the library is missing or a tensor is not on a ROCm device the
call raises, loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import NamedTuple, Optional, Sequence

import torch  # imported first: its libamdhip64.so.7 is the HIP runtime the library binds to

from . import build as _build

BLOCK = 256
TILE_ELEMS = BLOCK * BLOCK

DTYPE_BF16, DTYPE_FP32, DTYPE_FP16 = 0, 1, 2
SCORE_MEAN_ABS, SCORE_ABS_MEAN, SCORE_L1, SCORE_L2 = 0, 1, 2, 3
ADAM_DEEPSPEED, ADAM_TORCH = 0, 1

_DT = {torch.bfloat16: DTYPE_BF16, torch.float32: DTYPE_FP32, torch.float16: DTYPE_FP16}
ABI_VERSION = 13            # include/smt_hip.h: 16-bit dtype of the model ops / attention (v13),
                            # smt_adamw_args.param_dtype (v12), smt_wgrad_module.operand_dtype (v11)

# Every function the headers declare (include/smt_hip.h, smt_model_ops.h, smt_attention.h); tests check the
# library exports each of them.
ABI_FUNCTIONS = (
    "smt_last_error", "smt_abi_version", "smt_wgrad_workspace_bytes", "smt_tile_wgrad", "smt_wgrad_batch_workspace_bytes",
    "smt_tile_wgrad_batch", "smt_wgrad_seq_workspace_bytes", "smt_tile_wgrad_batch_seq", "smt_colblock_gather", "smt_tile_scatter_t",
    "smt_tile_gather", "smt_tile_scatter", "smt_grad_accumulate", "smt_block_score",
    "smt_sq_norm", "smt_adamw_step", "smt_adamw_multi",
    "smt_mx_quant_cols", "smt_wgrad_mx_workspace_bytes", "smt_tile_wgrad_mx", "smt_tile_wgrad_mx_batch",
    "smt_row_gather", "smt_row_scatter", "smt_column_gather", "smt_act_accumulate",
    "smt_channel_score_workspace_bytes", "smt_channel_score",
    "smt_channel_mean_aten_workspace_bytes", "smt_channel_mean_aten",
    "smt_model_ops_last_error", "smt_rmsnorm_fwd", "smt_rmsnorm_bwd_waves", "smt_rmsnorm_bwd", "smt_rmsnorm_bwd_add_dw",
    "smt_add_rmsnorm_fwd", "smt_rmsnorm_bwd_add", "smt_colblock_recompute",
    "smt_rope_fwd", "smt_rope_bwd", "smt_swiglu_fwd", "smt_swiglu_bwd", "smt_ce_fwd", "smt_ce_bwd",
    "smt_attn_last_error", "smt_attn_fwd", "smt_attn_bwd", "smt_attn_fwd_kmask", "smt_attn_bwd_kmask",
    "smt_fp8_last_error", "smt_quant_rows_e4m3", "smt_quant_cols_t_e4m3", "smt_quant_rows_cat_e4m3",
    "smt_swiglu_fwd_quant_e4m3", "smt_swiglu_bwd_quant_e4m3", "smt_swiglu_bwd_quant_e4m3_packed",
    "smt_rmsnorm_fwd_quant_e4m3",
    "smt_rmsnorm_bwd_add_quant_e4m3",
)


class TileDesc(ctypes.Structure):
    _fields_ = [("weight", ctypes.c_void_p), ("ld_weight", ctypes.c_int64),
                ("row_block", ctypes.c_int32), ("col_block", ctypes.c_int32),
                ("flat_offset", ctypes.c_int64)]


class WgradModule(ctypes.Structure):
    """smt_wgrad_module (include/smt_hip.h): one module of a batched tile wgrad."""
    _fields_ = [("grad_out", ctypes.c_void_p), ("x", ctypes.c_void_p), ("ld_grad_out", ctypes.c_int64),
                ("ld_x", ctypes.c_int64), ("x_block_stride", ctypes.c_int64), ("grad_tiles", ctypes.c_void_p),
                ("accumulate", ctypes.c_int32), ("operand_dtype", ctypes.c_int32)]


class WgradMxModule(ctypes.Structure):
    """smt_wgrad_mx_module (include/smt_hip.h): one module of a batched MX tile wgrad."""
    _fields_ = [("qg", ctypes.c_void_p), ("sg", ctypes.c_void_p), ("qx", ctypes.c_void_p), ("sx", ctypes.c_void_p),
                ("grad_tiles", ctypes.c_void_p), ("accumulate", ctypes.c_int32), ("reserved", ctypes.c_int32)]


WGRAD_MAX_MODULES = 16


class AccumEntry(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("chunk_begin", ctypes.c_int64), ("src_dtype", ctypes.c_int32), ("assign", ctypes.c_int32)]


class ScoreEntry(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("ld", ctypes.c_int64), ("d1", ctypes.c_int32),
                ("d2", ctypes.c_int32), ("block_begin", ctypes.c_int64), ("out", ctypes.c_void_p),
                ("strategy", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class AdamWArgs(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("bias_correction1", ctypes.c_float), ("bias_correction2", ctypes.c_float),
                ("max_grad_norm", ctypes.c_float), ("grad_scale", ctypes.c_float),
                ("mode", ctypes.c_int32), ("grad_dtype", ctypes.c_int32),
                ("param_dtype", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class AdamWTensor(ctypes.Structure):
    _fields_ = [("grad", ctypes.c_void_p), ("master", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("param", ctypes.c_void_p), ("n", ctypes.c_int64)]


class RopeTensor(ctypes.Structure):
    _fields_ = [("inp", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("in_sb", ctypes.c_int64), ("in_sh", ctypes.c_int64), ("in_ss", ctypes.c_int64),
                ("out_sb", ctypes.c_int64), ("out_sh", ctypes.c_int64), ("out_ss", ctypes.c_int64),
                ("heads", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class QuantSrc(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("ld", ctypes.c_int64), ("cols", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class AttnTensor(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("sb", ctypes.c_int64), ("sh", ctypes.c_int64), ("ss", ctypes.c_int64)]


class AttnShape(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int32), ("Hq", ctypes.c_int32), ("Hkv", ctypes.c_int32), ("S", ctypes.c_int32),
                ("scale", ctypes.c_float), ("dtype", ctypes.c_int32)]       # ABI v13: SMT_DTYPE_BF16 / _FP16


ACC_CHUNK = 4096
_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None

_P, _I64, _I32, _SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
_SIGS = {
    "smt_last_error": (ctypes.c_char_p, []),
    "smt_abi_version": (ctypes.c_int, []),
    "smt_wgrad_workspace_bytes": (_SZ, [_I64, _I32]),
    "smt_tile_wgrad": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _I64, _P, _P, _I32, _P, _I32, _I32, _P, _SZ, _P]),
    "smt_wgrad_batch_workspace_bytes": (_SZ, [_I64, _I32]),
    "smt_tile_wgrad_batch": (ctypes.c_int, [ctypes.POINTER(WgradModule), _I32, _I64, _P, _P, _I32, _I32, _P, _SZ, _P]),
    "smt_wgrad_seq_workspace_bytes": (_SZ, [_I64, _I64, _I32]),
    "smt_tile_wgrad_batch_seq": (ctypes.c_int, [ctypes.POINTER(WgradModule), _I32, _I64, _I64, _P, _P, _I32, _I32, _P,
                                                _SZ, _P]),
    "smt_colblock_gather": (ctypes.c_int, [_P, _I64, _I64, _P, _I32, _P, _P]),
    "smt_tile_scatter_t": (ctypes.c_int, [_P, _I32, _P, _P]),
    "smt_tile_gather": (ctypes.c_int, [_P, _I64, _I32, _P, _I32, _P, _P]),
    "smt_tile_scatter": (ctypes.c_int, [_P, _I64, _I32, _P, _I32, _P, _P]),
    "smt_grad_accumulate": (ctypes.c_int, [_P, _I32, _I64, _P]),
    "smt_block_score": (ctypes.c_int, [_P, _I32, _I64, _P]),
    "smt_sq_norm": (ctypes.c_int, [_P, _I64, _P, _I32, _P, _P]),
    "smt_adamw_step": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I32, _I64, _P, ctypes.POINTER(AdamWArgs), _P]),
    "smt_adamw_multi": (ctypes.c_int, [_P, _P, _I32, _I64, _P, ctypes.POINTER(AdamWArgs), _P]),
    "smt_mx_quant_cols": (ctypes.c_int, [_P, _I64, _I64, _P, _I32, _I64, _P, _P, _P]),
    "smt_wgrad_mx_workspace_bytes": (_SZ, [_I64, _I32]),
    "smt_tile_wgrad_mx": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P, _I32, _P, _I32, _I32, _P, _SZ, _P]),
    "smt_tile_wgrad_mx_batch": (ctypes.c_int, [ctypes.POINTER(WgradMxModule), _I32, _I64, _P, _P, _I32, _I32, _P, _SZ, _P]),
    "smt_row_gather": (ctypes.c_int, [_P, _I64, _I32, _I64, _P, _I32, _P, _I64, _P]),
    "smt_row_scatter": (ctypes.c_int, [_P, _I64, _I32, _I64, _P, _I32, _P, _I64, _P]),
    "smt_column_gather": (ctypes.c_int, [_P, _I64, _I64, _I64, _P, _I32, _P, _I64, _P]),
    "smt_act_accumulate": (ctypes.c_int, [_P, _I32, _I64, _I64, _I32, _I32, _I32, _P, _I32, _P]),
    "smt_channel_score_workspace_bytes": (_SZ, [_I32, _I32]),
    "smt_channel_score": (ctypes.c_int, [_P, _I32, _I32, _I32, _I32, _P, _SZ, _P, _P]),
    "smt_channel_mean_aten_workspace_bytes": (_SZ, [_I32, _I32]),
    "smt_channel_mean_aten": (ctypes.c_int, [_P, _I32, _I32, _I32, _P, _SZ, _P, _P]),
    "smt_attn_last_error": (ctypes.c_char_p, []),
    "smt_attn_fwd": (ctypes.c_int, [ctypes.POINTER(AttnTensor)] * 4 + [_P, ctypes.POINTER(AttnShape), _P]),
    "smt_attn_bwd": (ctypes.c_int, [ctypes.POINTER(AttnTensor)] * 5 + [_P, _P] + [ctypes.POINTER(AttnTensor)] * 3
                     + [ctypes.POINTER(AttnShape), _P]),
    "smt_attn_fwd_kmask": (ctypes.c_int, [ctypes.POINTER(AttnTensor)] * 4 + [_P, _P, _I64, ctypes.POINTER(AttnShape), _P]),
    "smt_attn_bwd_kmask": (ctypes.c_int, [ctypes.POINTER(AttnTensor)] * 5 + [_P, _P] + [ctypes.POINTER(AttnTensor)] * 3
                           + [_P, _I64, ctypes.POINTER(AttnShape), _P]),
    "smt_model_ops_last_error": (ctypes.c_char_p, []),
    "smt_rmsnorm_fwd": (ctypes.c_int, [_P, _I64, _P, _P, _I64, _P, _I64, _I32, ctypes.c_float, _I32, _P]),
    "smt_rmsnorm_bwd_waves": (ctypes.c_int, [_I64]),
    "smt_add_rmsnorm_fwd": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _P, _I64, _I32, ctypes.c_float,
                                           _I32, _P]),
    "smt_rmsnorm_bwd_add": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _I64, _P, _I64, _I64, _I32, _I32, _P]),
    "smt_rmsnorm_bwd": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _I64, _P, _P, _I64, _I32, _I32, _P]),
    "smt_rmsnorm_bwd_add_dw": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _I64, _P, _I64, _P, _P, _I64, _I32, _I32, _P]),
    "smt_rope_fwd": (ctypes.c_int, [ctypes.POINTER(RopeTensor), ctypes.POINTER(RopeTensor), _P, _P, _I64, _I64, _I64, _I32,
                                    _I32, _I32, _P]),
    "smt_rope_bwd": (ctypes.c_int, [ctypes.POINTER(RopeTensor), ctypes.POINTER(RopeTensor), _P, _P, _I64, _I64, _I64, _I32,
                                    _I32, _I32, _P]),
    "smt_swiglu_fwd": (ctypes.c_int, [_P, _P, _P, _I64, _I32, _P]),
    "smt_colblock_recompute": (ctypes.c_int, [_I32, _P, _I64, _P, _I64, _P, _P, _I64, _P, _I32, _P, _I32, _P]),
    "smt_swiglu_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _I64, _I32, _P]),
    "smt_ce_fwd": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, _I64, _P, _P, _I32, _P]),
    "smt_ce_bwd": (ctypes.c_int, [_P, _I64, _P, _P, _P, _I64, _I64, _I64, _P, _I64, _I32, _P]),
    "smt_fp8_last_error": (ctypes.c_char_p, []),
    "smt_quant_rows_e4m3": (ctypes.c_int, [_P, _I64, _I64, _I32, _P, _I32, _P, _I64, _P, _P]),
    "smt_quant_cols_t_e4m3": (ctypes.c_int, [_P, _I64, _I32, _I32, _P, _I32, _P, _I64, _P, _P]),
    "smt_quant_rows_cat_e4m3": (ctypes.c_int, [ctypes.POINTER(QuantSrc), _I32, _I64, _P, _I64, _P, _P]),
    "smt_rmsnorm_fwd_quant_e4m3": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _I64, _P, _I64, _P, _P, _I64, _P,
                                                   _I64, _I32, ctypes.c_float, _P]),
    "smt_rmsnorm_bwd_add_quant_e4m3": (ctypes.c_int, [_P, _I64, _P, _I64, _P, _P, _P, _I64, _P, _I64, _P, _I64, _P,
                                                       _I64, _I32, _P]),
    "smt_swiglu_fwd_quant_e4m3": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _I64, _P, _P, _P]),
    "smt_swiglu_bwd_quant_e4m3": (ctypes.c_int, [_P, _P, _P, _I64, _I32, _P, _I64, _P, _P, _P, _P]),
    "smt_swiglu_bwd_quant_e4m3_packed": (ctypes.c_int, [_P, _P, _P, _I64, _I32, _P, _I64, _P, _P, _P, _I64, _P, _P,
                                                         _I64, _P]),
}


def dtype_code16(dtype: torch.dtype, what: str) -> int:
    """SMT_DTYPE_* of a 16-bit model dtype (the model ops and the attention, ABI v13)."""
    if dtype == torch.bfloat16:
        return DTYPE_BF16
    if dtype == torch.float16:
        return DTYPE_FP16
    raise RuntimeError(f"{what}: bf16 or fp16 tensors only (got {dtype})")


def lib_path() -> str:
    return _build.LIB_PATH


def load(build_if_missing: bool = False) -> ctypes.CDLL:
    """Load (and bind) ``libsmt_hip.so``. Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if build_if_missing and _build.is_stale():
                _build.build()
            # SMT_HIP_LIB: load a kernel-variant build of the same sources instead (A/B runs,
            # scripts/diag/build_variant.py); the in-tree library otherwise
            path = os.environ.get("SMT_HIP_LIB") or _build.LIB_PATH
            if not os.path.exists(path):
                raise RuntimeError(
                    f"SMT HIP library not built ({path}); run `python -c 'import __graft_entry__ as g; g.build()'`"
                    " or `python -m sparse_matrix_tuning_amd.build`")
            lib = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            if lib.smt_abi_version() != ABI_VERSION:
                raise RuntimeError(f"{path} implements C ABI v{lib.smt_abi_version()}, this package v{ABI_VERSION}: "
                                   "rebuild it (`python -c 'import __graft_entry__ as g; g.build()'`)")
            _lib = lib
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        lib = load()
        if what.startswith(("smt_quant", "smt_swiglu_fwd_quant", "smt_swiglu_bwd_quant")):
            err = lib.smt_fp8_last_error                 # fp8_kernels.hip
        elif what.startswith(("smt_rmsnorm", "smt_add_rmsnorm", "smt_rope", "smt_swiglu", "smt_ce_",
                              "smt_colblock_recompute")):
            err = lib.smt_model_ops_last_error           # llama_kernels.hip (incl. smt_rmsnorm_fwd_quant_e4m3)
        elif what.startswith("smt_attn"):
            err = lib.smt_attn_last_error
        else:
            err = lib.smt_last_error
        raise RuntimeError(f"{what} failed (status {rc}): {err().decode(errors='replace')}")


def _require_device(*tensors: torch.Tensor) -> torch.device:
    dev = None
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError(
                f"SMT HIP path needs tensors on a ROCm device, got {t.device} "
                "(there is no CPU fallback: the CPU restatement lives in oracle/ and is test-only)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise RuntimeError(f"tensors on different devices: {dev} vs {t.device}")
    return dev


def _stream(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _device_table(structs: Sequence[ctypes.Structure], cls, dev: torch.device) -> torch.Tensor:
    """Copy an array of C structs into device memory (through the caching allocator)."""
    n = len(structs)
    arr = (cls * n)(*structs)
    host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
    return host.to(dev, non_blocking=False)


def tile_table(index_list: Sequence[Sequence[int]], device: torch.device) -> torch.Tensor:
    """Device int32 [n, 2] table of (row_block, col_block)."""
    flat = [int(v) for rc in index_list for v in (rc[0], rc[1])]
    return torch.tensor(flat, dtype=torch.int32).view(-1, 2).to(device)


def schedule_order(index_list: Sequence[Sequence[int]]) -> list:
    """wgrad schedule: tiles sharing the operand slice that is shared most (fewer distinct column
    blocks -> group by column, else by row) become adjacent, so they run on one XCD together."""
    rows = {int(rc[0]) for rc in index_list}
    cols = {int(rc[1]) for rc in index_list}
    if len(cols) <= len(rows):
        key = lambda i: (int(index_list[i][1]), int(index_list[i][0]))
    else:
        key = lambda i: (int(index_list[i][0]), int(index_list[i][1]))
    return sorted(range(len(index_list)), key=key)


def order_table(index_list: Sequence[Sequence[int]], device: torch.device) -> torch.Tensor:
    return torch.tensor(schedule_order(index_list), dtype=torch.int32).to(device)


# ---------------------------------------------------------------------------------------------
# wrappers
# ---------------------------------------------------------------------------------------------
def wgrad_workspace_bytes(T: int, n_tiles: int) -> int:
    return int(load().smt_wgrad_workspace_bytes(int(T), int(n_tiles)))


def tile_wgrad(grad_out2d: torch.Tensor, x: torch.Tensor, tile_rc: torch.Tensor, out: torch.Tensor,
               accumulate: bool = False, order: Optional[torch.Tensor] = None,
               seq_len: Optional[int] = None) -> torch.Tensor:
    """out[i] (+)= grad_out2d[:, r_i-block]^T @ X_{c_i} for every tile (smt.py:397-404): ``x`` is the
    input, row-major [T, in] (X_c = its c-th 256-column block), or the block-major [n_cb, T, 256]
    copy of ``colblock_gather`` (X_c = x[c]). ``order``: optional device int32 schedule permutation
    (speed only). ``seq_len``: the reference's rounding (``smt_tile_wgrad_batch_seq``): T is
    T / seq_len samples, each sample's partial rounded to bf16 before the batch sum. Operands bf16,
    fp16 or fp32 (the reference's --dtype; fp16 / fp32 go through the batched entry point with one
    module), ``out`` the operand dtype or fp32."""
    if grad_out2d.dtype != torch.bfloat16 and grad_out2d.shape[0] == 0:
        if not accumulate:
            out.zero_()
        return out
    if seq_len or grad_out2d.dtype != torch.bfloat16:
        n = tile_rc.shape[0]
        tab = torch.zeros(n, 4, dtype=torch.int32, device=tile_rc.device)
        tab[:, 1:3] = tile_rc
        tab[:, 3] = torch.arange(n, dtype=torch.int32, device=tile_rc.device)
        tile_wgrad_batch([(grad_out2d, x, out, accumulate)], tab, order, seq_len=seq_len)
        return out
    dev = _require_device(grad_out2d, x, tile_rc, out, order)
    if grad_out2d.dtype != torch.bfloat16 or x.dtype != torch.bfloat16:
        raise NotImplementedError(f"tile_wgrad: bf16 operands only (got {grad_out2d.dtype}, {x.dtype})")
    if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous():
        raise ValueError("tile_wgrad: out must be a contiguous bf16/fp32 tensor")
    n = tile_rc.shape[0]
    if out.numel() != n * TILE_ELEMS:
        raise ValueError(f"tile_wgrad: out has {out.numel()} elements, expected {n * TILE_ELEMS}")
    T = grad_out2d.shape[0]
    if x.dim() == 3:                      # block-major [n_cb, T, 256]
        if not x.is_contiguous() or x.shape[1:] != (T, BLOCK):
            raise ValueError("tile_wgrad: a block-major x must be a contiguous [n_cb, T, 256] tensor")
        ld_x, xbs = BLOCK, T * BLOCK
    else:
        if x.dim() != 2 or x.shape[0] != T or x.stride(1) != 1:
            raise ValueError("tile_wgrad: x must be [T, features] with unit feature stride")
        ld_x, xbs = x.stride(0), BLOCK
    if grad_out2d.stride(1) != 1:
        raise ValueError("tile_wgrad: grad_out must be [T, features] with unit feature stride")
    ws_bytes = wgrad_workspace_bytes(T, n)
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    if order is not None and (order.dtype != torch.int32 or order.numel() != n):
        raise ValueError("tile_wgrad: order must be int32 [n_tiles]")
    rc = load().smt_tile_wgrad(_ptr(grad_out2d), grad_out2d.stride(0), _ptr(x), ld_x, xbs, T,
                               _ptr(tile_rc), _ptr(order), n, _ptr(out), _DT[out.dtype], int(bool(accumulate)),
                               _ptr(ws), ws_bytes, _stream(dev))
    _check(rc, "smt_tile_wgrad")
    return out


def _wgrad_x_layout(x: torch.Tensor, T: int, what: str):
    """(ld_x, x_block_stride) of a row-major [T, in] input or a block-major [n_cb, T, 256] copy."""
    if x.dim() == 3:
        if not x.is_contiguous() or x.shape[1:] != (T, BLOCK):
            raise ValueError(f"{what}: a block-major x must be a contiguous [n_cb, T, 256] tensor")
        return BLOCK, T * BLOCK
    if x.dim() != 2 or x.shape[0] != T or x.stride(1) != 1:
        raise ValueError(f"{what}: x must be [T, features] with unit feature stride")
    return x.stride(0), BLOCK


def tile_wgrad_batch(items: Sequence[tuple], tile_tab: torch.Tensor, order: Optional[torch.Tensor] = None,
                     seq_len: Optional[int] = None) -> None:
    """One launch of the tile weight gradients of several modules sharing T (``smt_tile_wgrad_batch``).

    ``items``: per module ``(grad_out2d, x, out, accumulate)`` with the meaning of :func:`tile_wgrad`
    (``out``: that module's contiguous [n_m*256, 256] output; all outputs one dtype). ``tile_tab``:
    device int32 [n, 4] of (module, row_block, col_block, tile index in the module's output), e.g.
    from :func:`wgrad_batch_table`; ``order``: optional int32 [n] schedule permutation (speed only).
    Each tile's result is bit-identical to what :func:`tile_wgrad` gives for the same tile at the
    same T and the same total tile count. ``seq_len``: the reference's per-sample bf16 rounding
    (``smt_tile_wgrad_batch_seq``, include/smt_hip.h)."""
    if not items:
        return
    if len(items) > WGRAD_MAX_MODULES:
        raise ValueError(f"tile_wgrad_batch: {len(items)} modules > {WGRAD_MAX_MODULES}")
    dev = _require_device(tile_tab, order, *[t for it in items for t in it[:3]])
    T = items[0][0].shape[0]
    out_dtype = items[0][2].dtype
    op_dtype = items[0][0].dtype
    if op_dtype not in (torch.bfloat16, torch.float16, torch.float32):
        raise NotImplementedError(f"tile_wgrad_batch: operands bf16, fp16 or fp32 (got {op_dtype})")
    if out_dtype not in (op_dtype, torch.float32) or out_dtype == torch.float64:
        raise ValueError(f"tile_wgrad_batch: {op_dtype} operands give {op_dtype} or fp32 tiles (got {out_dtype})")
    mods = (WgradModule * len(items))()
    for i, (g, x, out, acc) in enumerate(items):
        if g.dtype != op_dtype or x.dtype != op_dtype:
            raise NotImplementedError(f"tile_wgrad_batch: one operand dtype per launch (got {g.dtype}, {x.dtype})")
        if g.dim() != 2 or g.shape[0] != T or g.stride(1) != 1:
            raise ValueError("tile_wgrad_batch: every grad_out must be [T, features] with the same T")
        if out.dtype != out_dtype or not out.is_contiguous():
            raise ValueError("tile_wgrad_batch: outputs must be contiguous and of one dtype")
        ld_x, xbs = _wgrad_x_layout(x, T, "tile_wgrad_batch")
        mods[i] = WgradModule(_ptr(g), _ptr(x), g.stride(0), ld_x, xbs, _ptr(out), int(bool(acc)), _DT[op_dtype])
    if tile_tab.dtype != torch.int32 or tile_tab.dim() != 2 or tile_tab.shape[1] != 4:
        raise ValueError("tile_wgrad_batch: tile_tab must be int32 [n, 4]")
    n = tile_tab.shape[0]
    if order is not None and (order.dtype != torch.int32 or order.numel() != n):
        raise ValueError("tile_wgrad_batch: order must be int32 [n_tiles]")
    if seq_len:
        if T % int(seq_len):
            raise ValueError(f"tile_wgrad_batch: T = {T} is not a whole number of {seq_len}-row samples")
        ws_bytes = int(load().smt_wgrad_seq_workspace_bytes(T, int(seq_len), n))
        ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
        rc = load().smt_tile_wgrad_batch_seq(mods, len(items), T, int(seq_len), _ptr(tile_tab), _ptr(order), n,
                                             _DT[out_dtype], _ptr(ws), ws_bytes, _stream(dev))
        _check(rc, "smt_tile_wgrad_batch_seq")
        return
    ws_bytes = int(load().smt_wgrad_batch_workspace_bytes(T, n))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    rc = load().smt_tile_wgrad_batch(mods, len(items), T, _ptr(tile_tab), _ptr(order), n, _DT[out_dtype],
                                     _ptr(ws), ws_bytes, _stream(dev))
    _check(rc, "smt_tile_wgrad_batch")


def wgrad_batch_table(module_tiles: Sequence[Sequence[Sequence[int]]], device: torch.device):
    """Device tables of a batch: int32 [n, 4] (module, row_block, col_block, tile index) over the
    modules' tile lists (``(row_block, col_block)`` as the kernel sees them: for a block-major input
    the column block is the position in it), and the int32 [n] schedule (tiles of one module stay in
    :func:`schedule_order`'s order, modules in batch order)."""
    rows, order = [], []
    for m, tl in enumerate(module_tiles):
        base = len(rows)
        rows.extend((m, int(r), int(c), k) for k, (r, c) in enumerate(tl))
        order.extend(base + i for i in schedule_order(tl))
    flat = [v for row in rows for v in row]
    tab = torch.tensor(flat, dtype=torch.int32).view(-1, 4).to(device)
    return tab, torch.tensor(order, dtype=torch.int32).to(device)


def colblock_gather(x2d: torch.Tensor, col_blocks: torch.Tensor) -> torch.Tensor:
    """[n_cb, T, 256] block-major copy of the 256-column blocks ``col_blocks`` (device int32) of x2d."""
    dev = _require_device(x2d, col_blocks)
    if x2d.dim() != 2 or x2d.stride(1) != 1 or x2d.element_size() != 2:
        raise ValueError("colblock_gather: x must be a 2-D row-major 16-bit tensor")
    n_cb = col_blocks.numel()
    out = torch.empty(n_cb, x2d.shape[0], BLOCK, dtype=x2d.dtype, device=dev)
    rc = load().smt_colblock_gather(_ptr(x2d), x2d.stride(0), x2d.shape[0], _ptr(col_blocks), n_cb, _ptr(out),
                                    _stream(dev))
    _check(rc, "smt_colblock_gather")
    return out


RECOMPUTE_RMSNORM, RECOMPUTE_SWIGLU = 0, 1


def colblock_recompute(op: int, a2d: torch.Tensor, col_blocks: torch.Tensor, b2d: torch.Tensor = None,
                       weight: torch.Tensor = None, rstd: torch.Tensor = None) -> torch.Tensor:
    """:func:`colblock_gather`'s [n_cb, T, 256] blocks of a norm's (``RECOMPUTE_RMSNORM``: ``a2d`` = its
    input, ``weight``, ``rstd``) or SwiGLU's (``RECOMPUTE_SWIGLU``: ``a2d`` = gate, ``b2d`` = up) output,
    rebuilt from those operands (bit-identical to gathering the producer's output)."""
    dev = _require_device(a2d, col_blocks, b2d, weight, rstd)
    for t in (a2d, b2d):
        if t is not None and (t.dim() != 2 or t.stride(1) != 1 or t.dtype not in (torch.bfloat16, torch.float16)):
            raise ValueError("colblock_recompute: operands must be 2-D row-major bf16 / fp16")
    if b2d is not None and b2d.dtype != a2d.dtype or weight is not None and weight.dtype != a2d.dtype:
        raise ValueError("colblock_recompute: operands of one dtype")
    if b2d is not None and b2d.shape != a2d.shape:
        raise ValueError("colblock_recompute: gate and up shapes differ")
    if rstd is not None and (rstd.dtype != torch.float32 or rstd.numel() != a2d.shape[0] or not rstd.is_contiguous()):
        raise ValueError("colblock_recompute: rstd must be a contiguous fp32 [T]")
    if weight is not None and (weight.numel() != a2d.shape[1] or not weight.is_contiguous()):
        raise ValueError("colblock_recompute: weight must be a contiguous [cols]")
    n_cb = col_blocks.numel()
    out = torch.empty(n_cb, a2d.shape[0], BLOCK, dtype=a2d.dtype, device=dev)
    rc = load().smt_colblock_recompute(op, _ptr(a2d), a2d.stride(0), _ptr(b2d) if b2d is not None else None,
                                       b2d.stride(0) if b2d is not None else 0,
                                       _ptr(weight) if weight is not None else None,
                                       _ptr(rstd) if rstd is not None else None, a2d.shape[0], _ptr(col_blocks), n_cb,
                                       _ptr(out), dtype_code16(a2d.dtype, "colblock_recompute"), _stream(dev))
    _check(rc, "smt_colblock_recompute")
    return out


class MxBlocks(NamedTuple):
    """MX-fp8 column blocks of a [T, C] bf16 matrix (include/smt_hip.h, smt_mx_quant_cols):
    ``q`` uint8 e4m3 [n, ldq/64, 256, 64] (K-major 64-token panels), ``scales`` uint8 e8m0
    [n, ldq/32, 256], ``T`` rows."""
    q: torch.Tensor
    scales: torch.Tensor
    T: int

    @property
    def ldq(self) -> int:
        return self.q.shape[1] * 64


def mx_ld(T: int) -> int:
    return (T + 63) // 64 * 64


def mx_quant_cols(x2d: torch.Tensor, blocks: torch.Tensor) -> MxBlocks:
    """MX-fp8 (e4m3 + one e8m0 exponent per 32 rows) copies of the 256-column blocks ``blocks``
    (device int32) of the bf16 matrix x2d, laid out for smt_tile_wgrad_mx."""
    dev = _require_device(x2d, blocks)
    if x2d.dim() != 2 or x2d.stride(1) != 1 or x2d.dtype != torch.bfloat16:
        raise ValueError("mx_quant_cols: x must be a 2-D row-major bf16 tensor")
    if blocks.dtype != torch.int32 or blocks.dim() != 1:
        raise ValueError("mx_quant_cols: blocks must be device int32 [n]")
    T, n = x2d.shape[0], blocks.numel()
    ldq = mx_ld(T)
    q = torch.empty(n, ldq // 64, BLOCK, 64, dtype=torch.uint8, device=dev)
    sc = torch.empty(n, ldq // 32, BLOCK, dtype=torch.uint8, device=dev)
    rc = load().smt_mx_quant_cols(_ptr(x2d), x2d.stride(0), T, _ptr(blocks), n, ldq, _ptr(q), _ptr(sc), _stream(dev))
    _check(rc, "smt_mx_quant_cols")
    return MxBlocks(q, sc, T)


def tile_wgrad_mx(g: MxBlocks, x: MxBlocks, tile_rc: torch.Tensor, out: torch.Tensor, accumulate: bool = False,
                  order: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[i] (+)= A_i^T B_i over MX column blocks: tile_rc[i] = (block of ``g``, block of ``x``).
    The table is built from a validated host list (no device read-back here, this is per step)."""
    dev = _require_device(g.q, x.q, tile_rc, out, order)
    if out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous():
        raise ValueError("tile_wgrad_mx: out must be a contiguous bf16/fp32 tensor")
    n = tile_rc.shape[0]
    if out.numel() != n * TILE_ELEMS:
        raise ValueError(f"tile_wgrad_mx: out has {out.numel()} elements, expected {n * TILE_ELEMS}")
    if g.T != x.T or g.ldq != x.ldq:
        raise ValueError("tile_wgrad_mx: operands cover different rows")
    if order is not None and (order.dtype != torch.int32 or order.numel() != n):
        raise ValueError("tile_wgrad_mx: order must be int32 [n_tiles]")
    ldq = g.ldq
    ws_bytes = load().smt_wgrad_mx_workspace_bytes(ldq, n)
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    rc = load().smt_tile_wgrad_mx(_ptr(g.q), _ptr(g.scales), _ptr(x.q), _ptr(x.scales), ldq, _ptr(tile_rc),
                                  _ptr(order), n, _ptr(out), _DT[out.dtype], int(bool(accumulate)), _ptr(ws),
                                  ws_bytes, _stream(dev))
    _check(rc, "smt_tile_wgrad_mx")
    return out


def tile_wgrad_mx_batch(items: Sequence[tuple], tile_tab: torch.Tensor, order: Optional[torch.Tensor] = None) -> None:
    """One launch of the MX tile weight gradients of several modules (``smt_tile_wgrad_mx_batch``):
    ``items`` per module ``(g: MxBlocks, x: MxBlocks, out, accumulate)`` as :func:`tile_wgrad_mx`,
    all with the same ldq; ``tile_tab`` int32 [n, 4] of (module, block of its g, block of its x,
    tile index in its output), e.g. :func:`wgrad_batch_table` over the modules' mx tables."""
    if not items:
        return
    if len(items) > WGRAD_MAX_MODULES:
        raise ValueError(f"tile_wgrad_mx_batch: {len(items)} modules > {WGRAD_MAX_MODULES}")
    dev = _require_device(tile_tab, order, *[t for g, x, out, _a in items for t in (g.q, x.q, out)])
    ldq, out_dtype = items[0][0].ldq, items[0][2].dtype
    mods = (WgradMxModule * len(items))()
    for i, (g, x, out, acc) in enumerate(items):
        if g.ldq != ldq or x.ldq != ldq or g.T != x.T:
            raise ValueError("tile_wgrad_mx_batch: every module's MX blocks must cover the same rows")
        if out.dtype != out_dtype or out.dtype not in (torch.bfloat16, torch.float32) or not out.is_contiguous():
            raise ValueError("tile_wgrad_mx_batch: outputs must be contiguous and all bf16 or all fp32")
        mods[i] = WgradMxModule(_ptr(g.q), _ptr(g.scales), _ptr(x.q), _ptr(x.scales), _ptr(out), int(bool(acc)), 0)
    if tile_tab.dtype != torch.int32 or tile_tab.dim() != 2 or tile_tab.shape[1] != 4:
        raise ValueError("tile_wgrad_mx_batch: tile_tab must be int32 [n, 4]")
    n = tile_tab.shape[0]
    if order is not None and (order.dtype != torch.int32 or order.numel() != n):
        raise ValueError("tile_wgrad_mx_batch: order must be int32 [n_tiles]")
    ws_bytes = int(load().smt_wgrad_mx_workspace_bytes(ldq, n))
    ws = torch.empty(max(ws_bytes, 16), dtype=torch.uint8, device=dev)
    rc = load().smt_tile_wgrad_mx_batch(mods, len(items), ldq, _ptr(tile_tab), _ptr(order), n, _DT[out_dtype],
                                        _ptr(ws), ws_bytes, _stream(dev))
    _check(rc, "smt_tile_wgrad_mx_batch")


def tile_gather(weight: torch.Tensor, tile_rc: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    dev = _require_device(weight, tile_rc, out)
    if weight.dim() != 2 or weight.stride(1) != 1 or out.dtype != weight.dtype or not out.is_contiguous():
        raise ValueError("tile_gather: weight must be 2-D row-major and out contiguous of the same dtype")
    rc = load().smt_tile_gather(_ptr(weight), weight.stride(0), weight.element_size(), _ptr(tile_rc),
                                tile_rc.shape[0], _ptr(out), _stream(dev))
    _check(rc, "smt_tile_gather")
    return out


def tile_scatter(weight: torch.Tensor, tile_rc: torch.Tensor, tiles: torch.Tensor) -> None:
    dev = _require_device(weight, tile_rc, tiles)
    if weight.dim() != 2 or weight.stride(1) != 1 or tiles.dtype != weight.dtype or not tiles.is_contiguous():
        raise ValueError("tile_scatter: weight must be 2-D row-major and tiles contiguous of the same dtype")
    rc = load().smt_tile_scatter(_ptr(weight), weight.stride(0), weight.element_size(), _ptr(tile_rc),
                                 tile_rc.shape[0], _ptr(tiles), _stream(dev))
    _check(rc, "smt_tile_scatter")


class AccumulatePlan:
    """Device descriptor table for one multi-tensor warm-up accumulation launch."""

    def __init__(self, pairs: Sequence[tuple], assign: bool):
        entries, chunk = [], 0
        dev = None
        for dst, src in pairs:
            dev = _require_device(dst, src)
            if dst.dtype != torch.float32 or not dst.is_contiguous() or not src.is_contiguous():
                raise ValueError("accumulate: dst must be contiguous fp32 and src contiguous")
            if dst.numel() != src.numel():
                raise ValueError("accumulate: size mismatch")
            n = dst.numel()
            entries.append(AccumEntry(src.data_ptr(), dst.data_ptr(), n, chunk, _DT[src.dtype], int(assign)))
            chunk += (n + ACC_CHUNK - 1) // ACC_CHUNK
        self.n_entries = len(entries)
        self.total_chunks = chunk
        self.device = dev
        self.table = _device_table(entries, AccumEntry, dev) if entries else None

    def launch(self) -> None:
        if not self.n_entries:
            return
        rc = load().smt_grad_accumulate(_ptr(self.table), self.n_entries, self.total_chunks, _stream(self.device))
        _check(rc, "smt_grad_accumulate")


def grad_accumulate(pairs: Sequence[tuple], assign: bool = False) -> None:
    AccumulatePlan(pairs, assign).launch()


def block_scores(grads: Sequence[torch.Tensor], dims: Sequence[tuple], strategy: int) -> list:
    """Per fp32 gradient, an fp64 ``[d1*d2, 2]`` tensor: per 256x256 block (row-major) the sum of the
    strategy's terms and the sum of their magnitudes; one launch for all of them."""
    entries, outs, blk = [], [], 0
    dev = None
    for g, (d1, d2) in zip(grads, dims):
        dev = _require_device(g)
        if g.dtype != torch.float32:
            raise ValueError(f"block_scores: fp32 gradients only (got {g.dtype})")
        g2 = g.reshape(d1 * BLOCK, d2 * BLOCK)
        if g2.stride(1) != 1 or (g2.stride(0) % 4) or (g2.data_ptr() % 16):
            g2 = g2.contiguous()
        out = torch.empty(d1 * d2, 2, dtype=torch.float64, device=dev)
        outs.append((out, g2))
        entries.append(ScoreEntry(g2.data_ptr(), g2.stride(0), d1, d2, blk, out.data_ptr(), strategy, 0))
        blk += d1 * d2
    if not entries:
        return []
    table = _device_table(entries, ScoreEntry, dev)
    rc = load().smt_block_score(_ptr(table), len(entries), blk, _stream(dev))
    _check(rc, "smt_block_score")
    return [o for o, _ in outs]


def sq_norm(x: torch.Tensor, out: Optional[torch.Tensor] = None, n_partials: int = 1024) -> torch.Tensor:
    dev = _require_device(x)
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise ValueError("sq_norm: contiguous fp32 only")
    partials = torch.empty(n_partials, dtype=torch.float64, device=dev)
    if out is None:
        out = torch.empty(1, dtype=torch.float64, device=dev)
    rc = load().smt_sq_norm(_ptr(x), x.numel(), _ptr(partials), n_partials, _ptr(out), _stream(dev))
    _check(rc, "smt_sq_norm")
    return out


_PARAM_DTYPES = (torch.bfloat16, torch.float16, torch.float32)


def _adamw_dtypes(fn: str, grad_dtype: torch.dtype, param_dtype: torch.dtype) -> None:
    """smt_adamw_*: fp32 gradients of a bf16 / fp16 / fp32 parameter, or bf16 / fp16 gradients of a
    parameter of the same dtype (ABI v12; the reference's --dtype, fine_tune.py:955-959)."""
    if param_dtype not in _PARAM_DTYPES:
        raise ValueError(f"{fn}: parameters must be bf16, fp16 or fp32, not {param_dtype}")
    if grad_dtype != torch.float32 and grad_dtype != param_dtype:
        raise ValueError(f"{fn}: {grad_dtype} gradients of a {param_dtype} parameter (fp32, or the parameter's dtype)")


def adamw_step(grad: torch.Tensor, master: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
               param: torch.Tensor, args: AdamWArgs, tiles: Optional[torch.Tensor] = None,
               n_tiles: int = 0, grad_sq_norm: Optional[torch.Tensor] = None) -> None:
    """Fused clip + AdamW over flat buffers; the updated values are written into ``param`` (bf16, fp16
    or fp32) and, with ``tiles``, scattered into the W each descriptor names (W of ``param``'s dtype)."""
    dev = _require_device(grad, master, exp_avg, exp_avg_sq, param, tiles, grad_sq_norm)
    for t in (master, exp_avg, exp_avg_sq):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("adamw_step: master/exp_avg/exp_avg_sq must be contiguous fp32")
    if not param.is_contiguous() or not grad.is_contiguous():
        raise ValueError("adamw_step: param and grad must be contiguous")
    _adamw_dtypes("adamw_step", grad.dtype, param.dtype)
    n = master.numel()
    if not (grad.numel() == n == exp_avg.numel() == exp_avg_sq.numel() == param.numel()):
        raise ValueError("adamw_step: buffer sizes differ")
    args.grad_dtype = _DT[grad.dtype]
    args.param_dtype = _DT[param.dtype]
    rc = load().smt_adamw_step(_ptr(grad), _ptr(master), _ptr(exp_avg), _ptr(exp_avg_sq), _ptr(param),
                               _ptr(tiles), int(n_tiles), n, _ptr(grad_sq_norm), ctypes.byref(args), _stream(dev))
    _check(rc, "smt_adamw_step")


ADAM_MULTI_BLOCK = 2048


def adamw_multi(tensors, args: AdamWArgs, grad_sq_norm: Optional[torch.Tensor] = None) -> None:
    """One ``smt_adamw_multi`` launch over ``tensors`` = [(grad, master, exp_avg, exp_avg_sq, param)]
    (all on one device, one gradient dtype and one parameter dtype, every buffer contiguous and 16-byte
    aligned)."""
    if not tensors:
        return
    dev = _require_device(*[t for row in tensors for t in row], grad_sq_norm)
    gdt, pdt = tensors[0][0].dtype, tensors[0][4].dtype
    _adamw_dtypes("adamw_multi", gdt, pdt)
    rows, starts = [], [0]
    for grad, master, m, v, p in tensors:
        for t in (master, m, v):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError("adamw_multi: master/exp_avg/exp_avg_sq must be contiguous fp32")
        if (p.dtype != pdt or not p.is_contiguous() or not grad.is_contiguous() or grad.dtype != gdt):
            raise ValueError("adamw_multi: params of one dtype, grads of one dtype, all contiguous")
        n = master.numel()
        if not (grad.numel() == n == m.numel() == v.numel() == p.numel()):
            raise ValueError("adamw_multi: buffer sizes differ")
        if any(t.data_ptr() % 16 for t in (grad, master, m, v, p)):
            raise ValueError("adamw_multi: buffers must be 16-byte aligned")
        rows.append(AdamWTensor(_ptr(grad), _ptr(master), _ptr(m), _ptr(v), _ptr(p), n))
        starts.append(starts[-1] + (n + ADAM_MULTI_BLOCK - 1) // ADAM_MULTI_BLOCK)
    # stream-ordered: the caching allocator reuses the tables only after this launch on the stream
    table_dev = _device_table(rows, AdamWTensor, dev)
    starts_dev = torch.tensor(starts, dtype=torch.int64).to(dev)
    args.grad_dtype = _DT[gdt]
    args.param_dtype = _DT[pdt]
    rc = load().smt_adamw_multi(_ptr(table_dev), _ptr(starts_dev), len(tensors), starts[-1], _ptr(grad_sq_norm),
                                ctypes.byref(args), _stream(dev))
    _check(rc, "smt_adamw_multi")


def tile_scatter_t(descs: torch.Tensor, n_tiles: int, tiles: torch.Tensor) -> None:
    """Transposed write-back of 16-bit (bf16 / fp16) tiles into the W^T copies the descriptors point at
    (the kernel moves 16-bit values: one instance for both formats)."""
    dev = _require_device(descs, tiles)
    if tiles.dtype not in (torch.bfloat16, torch.float16) or not tiles.is_contiguous():
        raise ValueError("tile_scatter_t: tiles must be contiguous bf16 / fp16")
    rc = load().smt_tile_scatter_t(_ptr(descs), int(n_tiles), _ptr(tiles), _stream(dev))
    _check(rc, "smt_tile_scatter_t")


def tile_descs(entries: Sequence[tuple], device: torch.device, dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """entries: (weight tensor or None, row_block, col_block, flat_offset) -> device smt_tile_desc[];
    every W is row-major of ``dtype`` (the parameter dtype of the AdamW step that scatters into it)."""
    descs = []
    for w, r, c, off in entries:
        if w is not None:
            if w.dtype != dtype or w.stride(1) != 1:
                raise ValueError(f"tile_descs: W must be {dtype} row-major")
            descs.append(TileDesc(w.data_ptr(), w.stride(0), int(r), int(c), int(off)))
        else:
            descs.append(TileDesc(None, 0, int(r), int(c), int(off)))
    return _device_table(descs, TileDesc, device)


# ---------------------------------------------------------------------------------------------
# channel path (ABI v3)
# ---------------------------------------------------------------------------------------------
def index_table(indices: Sequence[int], device: torch.device) -> torch.Tensor:
    """Device int32 [n] table of row / column indices."""
    return torch.tensor([int(i) for i in indices], dtype=torch.int32).to(device)


def _row_copy(fn: str, weight: torch.Tensor, rows_dev: torch.Tensor, rows: torch.Tensor) -> None:
    dev = _require_device(weight, rows_dev, rows)
    if weight.dim() != 2 or rows.dim() != 2 or weight.stride(1) != 1 or rows.stride(1) != 1:
        raise ValueError(f"{fn}: weight and rows must be 2-D row-major")
    if rows.dtype != weight.dtype or rows.shape[1] != weight.shape[1] or rows.shape[0] != rows_dev.numel():
        raise ValueError(f"{fn}: rows must be [{rows_dev.numel()}, {weight.shape[1]}] of {weight.dtype}")
    rc = getattr(load(), fn)(_ptr(weight), weight.stride(0), weight.element_size(), weight.shape[1], _ptr(rows_dev),
                             rows_dev.numel(), _ptr(rows), rows.stride(0), _stream(dev))
    _check(rc, fn)


def row_gather(weight: torch.Tensor, rows_dev: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[i, :] = weight[rows[i], :] (smt.py:200-204)."""
    _row_copy("smt_row_gather", weight, rows_dev, out)
    return out


def row_scatter(weight: torch.Tensor, rows_dev: torch.Tensor, rows: torch.Tensor) -> None:
    """weight[rows[i], :] = rows[i, :] (smt.py:211-213)."""
    _row_copy("smt_row_scatter", weight, rows_dev, rows)


def column_gather(x2d: torch.Tensor, cols_dev: torch.Tensor, n_cols: int, ld_out: int) -> torch.Tensor:
    """[T, ld_out] with out[:, j] = x2d[:, cols[j]] for j < n_cols and zeros after (smt.py:225-233)."""
    dev = _require_device(x2d, cols_dev)
    if x2d.dim() != 2 or x2d.stride(1) != 1 or x2d.element_size() not in (2, 4):
        raise ValueError("column_gather: x must be a 2-D row-major 16- or 32-bit tensor")
    if x2d.element_size() == 4:
        # an fp32 column c is the 16-bit column pair (2c, 2c + 1) of the same rows: the same kernel
        # over the rows viewed as 16-bit words, with the pairs as its column list
        c = cols_dev[:n_cols].to(torch.int32)
        pairs = torch.stack((2 * c, 2 * c + 1), 1).reshape(-1).contiguous()
        out16 = column_gather(x2d.view(torch.int16), pairs, 2 * int(n_cols), 2 * int(ld_out))
        return out16.view(x2d.dtype)
    out = torch.empty(x2d.shape[0], ld_out, dtype=x2d.dtype, device=dev)
    rc = load().smt_column_gather(_ptr(x2d), x2d.stride(0), x2d.shape[1], x2d.shape[0], _ptr(cols_dev), int(n_cols),
                                  _ptr(out), ld_out, _stream(dev))
    _check(rc, "smt_column_gather")
    return out


def act_accumulate(x3d: torch.Tensor, acc: torch.Tensor, assign: bool) -> None:
    """acc[b, s, c] = |x3d[b, s, c]| (assign) or acc += |x3d| in fp32, elementwise: the reference's
    ``feat[key] = x.abs().float()`` / ``feat[key] += ...`` (fine_tune.py:636-667)."""
    dev = _require_device(x3d, acc)
    if x3d.dim() != 3 or x3d.stride(2) != 1:
        raise ValueError("act_accumulate: x must be [B, S, C] with unit channel stride")
    B, S, C = x3d.shape
    if acc.dtype != torch.float32 or not acc.is_contiguous() or tuple(acc.shape) != (B, S, C):
        raise ValueError(f"act_accumulate: acc must be contiguous fp32 [{B}, {S}, {C}]")
    rc = load().smt_act_accumulate(_ptr(x3d), _DT[x3d.dtype], x3d.stride(1), x3d.stride(0), B, S, C, _ptr(acc),
                                   int(bool(assign)), _stream(dev))
    _check(rc, "smt_act_accumulate")


def channel_mean_aten(acc: torch.Tensor) -> torch.Tensor:
    """fp32 [C]: torch.mean(torch.sum(acc.abs(), 0).abs(), 0) in ATen's CPU summation order
    (``smt_channel_mean_aten``) for a contiguous fp32 [B, S, C] accumulator."""
    dev = _require_device(acc)
    if acc.dtype != torch.float32 or not acc.is_contiguous() or acc.dim() != 3:
        raise ValueError("channel_mean_aten: contiguous fp32 [B, S, C] accumulator expected")
    B, S, C = acc.shape
    out = torch.empty(C, dtype=torch.float32, device=dev)
    ws_bytes = int(load().smt_channel_mean_aten_workspace_bytes(S, C))
    ws = torch.empty(max(ws_bytes // 4, 4), dtype=torch.float32, device=dev)
    rc = load().smt_channel_mean_aten(_ptr(acc), B, S, C, _ptr(ws), ws_bytes, _ptr(out), _stream(dev))
    _check(rc, "smt_channel_mean_aten")
    return out


def channel_scores(acc: torch.Tensor, strategy: int) -> torch.Tensor:
    """fp64 per-channel sums over (batch, sequence) of an fp32 [B, S, C] accumulator: sum_s A_s, or
    sum_s A_s^2 for L2, with A_s = sum_b |acc[b, s, c]|."""
    dev = _require_device(acc)
    if acc.dtype != torch.float32 or not acc.is_contiguous() or acc.dim() != 3:
        raise ValueError("channel_scores: contiguous fp32 [B, S, C] accumulator expected")
    out = torch.empty(acc.shape[2], dtype=torch.float64, device=dev)
    ws_bytes = load().smt_channel_score_workspace_bytes(acc.shape[1], acc.shape[2])
    ws = torch.empty(max(ws_bytes // 8, 2), dtype=torch.float64, device=dev)
    rc = load().smt_channel_score(_ptr(acc), acc.shape[0], acc.shape[1], acc.shape[2], int(strategy), _ptr(ws),
                                  ws_bytes, _ptr(out), _stream(dev))
    _check(rc, "smt_channel_score")
    return out

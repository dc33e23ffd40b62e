"""The C-ABI library builds for gfx950, loads, and exports every symbol include/smt_hip.h declares.
Argument validation paths return error codes before any HIP call (safe without a GPU)."""
import ctypes
import os
import re
import subprocess

from sparse_matrix_tuning_amd import _hip, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include"))) if h.endswith(".h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(smt_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_lists_the_binding_functions():
    assert declared_functions() == sorted(_hip.ABI_FUNCTIONS)


def test_library_exports_every_declared_symbol():
    lib = _hip.load(build_if_missing=True)
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _hip.lib_path()], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}$", out, re.M), name
    assert lib.smt_abi_version() == 13


def test_library_carries_gfx950_code_object():
    blob = open(_hip.lib_path(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob          # the offload bundle's target id


def test_struct_layouts_match_header():
    assert ctypes.sizeof(_hip.TileDesc) == 32
    assert ctypes.sizeof(_hip.AccumEntry) == 40
    assert ctypes.sizeof(_hip.ScoreEntry) == 48
    assert ctypes.sizeof(_hip.AdamWArgs) == 52          # ABI v12: param_dtype + reserved
    assert ctypes.sizeof(_hip.RopeTensor) == 72
    assert ctypes.sizeof(_hip.AdamWTensor) == 48
    assert ctypes.sizeof(_hip.WgradModule) == 56


def test_validation_errors_without_gpu():
    lib = _hip.load()
    assert lib.smt_tile_wgrad(None, 0, None, 0, 256, 16, None, None, -1, None, 0, 0, None, 0, None) == -1
    assert b"negative" in lib.smt_last_error()
    assert lib.smt_tile_wgrad(None, 0, None, 0, 256, 16, None, None, 0, None, 0, 0, None, 0, None) == 0   # no tiles: no-op
    assert lib.smt_adamw_step(None, None, None, None, None, None, 0, 0, None, None, None) == -1
    args = _hip.AdamWArgs(lr=1e-3, beta1=0.9, beta2=0.95, eps=1e-8, weight_decay=0.0, bias_correction1=0.0,
                          bias_correction2=0.1, max_grad_norm=0.0, grad_scale=1.0, mode=0, grad_dtype=0)
    assert lib.smt_adamw_step(None, None, None, None, None, None, 0, 8, None, ctypes.byref(args), None) == -1
    assert b"bias" in lib.smt_last_error()
    assert lib.smt_adamw_multi(None, None, 3, 5, None, ctypes.byref(args), None) == -1
    assert b"bias" in lib.smt_last_error()
    args.bias_correction1 = 0.1
    assert lib.smt_adamw_multi(None, None, 0, 0, None, ctypes.byref(args), None) == 0      # nothing to do
    assert lib.smt_adamw_multi(None, None, 3, 5, None, ctypes.byref(args), None) == -1
    assert b"null table" in lib.smt_last_error()
    # parameter dtypes (ABI v12): 16-bit gradients only of a parameter of their own dtype
    args.grad_dtype, args.param_dtype = _hip.DTYPE_BF16, _hip.DTYPE_FP16
    assert lib.smt_adamw_step(None, None, None, None, None, None, 0, 8, None, ctypes.byref(args), None) == -1
    assert b"param_dtype" in lib.smt_last_error()
    args.grad_dtype, args.param_dtype = _hip.DTYPE_FP16, _hip.DTYPE_FP32
    assert lib.smt_adamw_multi(None, None, 3, 5, None, ctypes.byref(args), None) == -1
    assert b"param_dtype" in lib.smt_last_error()
    args.param_dtype = 7
    assert lib.smt_adamw_step(None, None, None, None, None, None, 0, 8, None, ctypes.byref(args), None) == -1
    for g, p in ((_hip.DTYPE_FP32, _hip.DTYPE_FP32), (_hip.DTYPE_FP32, _hip.DTYPE_FP16), (_hip.DTYPE_FP16, _hip.DTYPE_FP16)):
        args.grad_dtype, args.param_dtype = g, p
        assert lib.smt_adamw_step(None, None, None, None, None, None, 0, 8, None, ctypes.byref(args), None) == -1
        assert b"null buffer" in lib.smt_last_error()
    assert lib.smt_tile_gather(None, 256, 3, None, 1, None, None) == -1
    assert lib.smt_sq_norm(None, 10, None, 0, None, None) == -1
    assert lib.smt_wgrad_workspace_bytes(32768, 27) == 27 * 9 * 65536 * 4
    assert lib.smt_wgrad_workspace_bytes(32768, 8) == 8 * 16 * 65536 * 4       # quarter tiles: 8 x 16 x 4 workgroups
    assert lib.smt_wgrad_workspace_bytes(32768, 6) == 6 * 21 * 65536 * 4       # 504 <= 512 workgroup slots, one round
    assert lib.smt_wgrad_workspace_bytes(32768, 256) == 0          # S == 1: no slabs
    assert lib.smt_wgrad_workspace_bytes(32768, 128) == 128 * 2 * 65536 * 4
    assert lib.smt_wgrad_workspace_bytes(0, 27) == 0
    # reference rounding (ABI v8): per-sample pieces, never crossing a sample boundary
    assert lib.smt_wgrad_seq_workspace_bytes(32768, 2048, 51) == 51 * 16 * 65536 * 4        # 816 >= 256 splits
    assert lib.smt_wgrad_seq_workspace_bytes(32768, 2048, 9) == 9 * 16 * 2 * 65536 * 4      # 9 tiles: 2 pieces
    assert lib.smt_wgrad_seq_workspace_bytes(4096, 2048, 8) == 8 * 2 * 8 * 65536 * 4        # quarter: 8 x 2 x 8 x 4
    assert lib.smt_wgrad_seq_workspace_bytes(4096, 3000, 8) == 0                            # not whole samples
    mods = (_hip.WgradModule * 1)()
    assert lib.smt_tile_wgrad_batch_seq(mods, 1, 4096, 3000, None, None, 8, 0, None, 0, None) == -1
    assert b"null tile table" in lib.smt_last_error()
    tab = ctypes.c_void_p(16)                           # never dereferenced: validation fails first
    assert lib.smt_tile_wgrad_batch_seq(mods, 1, 4096, 3000, tab, None, 8, 0, None, 0, None) == -1
    assert b"whole number" in lib.smt_last_error()
    assert lib.smt_tile_wgrad_batch_seq(mods, 1, 4096, 0, tab, None, 8, 0, None, 0, None) == -1
    # selective activation policy (ABI v9): column blocks rebuilt from the producer's operands
    bf16 = _hip.DTYPE_BF16
    assert lib.smt_colblock_recompute(7, None, 0, None, 0, None, None, 8, None, 1, None, bf16, None) == -1
    assert b"unknown op" in lib.smt_model_ops_last_error()
    assert lib.smt_colblock_recompute(0, None, 0, None, 0, None, None, 0, None, 1, None, bf16, None) == 0   # no rows
    assert lib.smt_colblock_recompute(1, tab, 512, None, 0, None, None, 8, tab, 1, tab, bf16, None) == -1
    assert b"null up" in lib.smt_model_ops_last_error()
    assert lib.smt_colblock_recompute(0, tab, 512, None, 0, None, None, 8, tab, 1, tab, bf16, None) == -1
    assert b"null weight" in lib.smt_model_ops_last_error()
    # ABI v13: the model ops and the attention take the model's 16-bit dtype; anything else is refused
    # before a launch (fp32 = SMT_DTYPE_FP32 and an unknown code)
    for bad in (_hip.DTYPE_FP32, 7):
        assert lib.smt_swiglu_fwd(tab, tab, tab, 8, bad, None) == -1
        assert b"not a 16-bit format" in lib.smt_model_ops_last_error()
        assert lib.smt_ce_fwd(tab, 8, tab, 1, 8, -100, tab, tab, bad, None) == -1
        assert b"not a 16-bit format" in lib.smt_model_ops_last_error()
        shape = _hip.AttnShape(1, 8, 2, 64, 0.088, bad)
        t = _hip.AttnTensor(tab, 0, 0, 0)
        assert lib.smt_attn_fwd(ctypes.byref(t), ctypes.byref(t), ctypes.byref(t), ctypes.byref(t), tab,
                                ctypes.byref(shape), None) == -1
        assert b"not a 16-bit format" in lib.smt_attn_last_error()
    # channel path (ABI v3)
    assert lib.smt_row_gather(None, 256, 2, 256, None, 4, None, 256, None) == -1
    assert lib.smt_row_gather(None, 256, 2, 256, None, 0, None, 256, None) == 0       # no rows: no-op
    assert lib.smt_row_scatter(None, 256, 8, 256, None, 4, None, 256, None) == -1
    assert lib.smt_column_gather(None, 256, 256, 16, None, 300, None, 256, None) == -1      # ld_out < n_cols
    assert lib.smt_act_accumulate(None, 0, 256, 0, 1, 4, 256, None, 1, None) == -1
    assert lib.smt_act_accumulate(None, 7, 256, 0, 1, 4, 256, None, 1, None) == -1     # bad dtype / null acc
    assert lib.smt_act_accumulate(None, 0, 256, 0, 0, 4, 256, None, 1, None) == 0      # empty batch: no-op
    assert lib.smt_channel_score(None, 1, 4, 256, 9, None, 0, None, None) == -1
    assert lib.smt_channel_score_workspace_bytes(2048, 5120) == 64 * 5120 * 8
    assert b"strategy" in lib.smt_last_error()


def test_build_is_up_to_date():
    assert not build.is_stale()

"""Fused gfx950 replacements for the eager elementwise chains of the HF LLaMA decoder.

The SMT step trains ``transformers`` ``LlamaForCausalLM`` (the reference loads it through
``AutoModelForCausalLM``, ``fine_tune.py:150-155``). In eager mode its RMSNorm, rotary embedding and
SwiGLU each run as chains of 4-8 elementwise kernels, several in fp32; on MI355X those chains are
27 % of an SMT step (profiles/r01_bench_step_breakdown.txt). :func:`patch_llama` swaps them for
one-pass HIP kernels (``csrc/llama_kernels.hip``, C ABI ``include/smt_model_ops.h``) wrapped in
autograd Functions. Every intermediate 16-bit rounding of the eager chain is reproduced, so results
match the eager model up to reduction order / exp ulps (tests/test_gpu_fused_llama.py).

It also routes the decoder's attention to a gfx950 causal flash attention (forward + backward,
``csrc/attn_kernels.hip``, C ABI ``include/smt_attention.h``), registered with transformers'
``AttentionInterface`` as ``"smt_flash"``; sdpa on this torch build runs aotriton at 25-27 % of the
step. Tolerances vs an fp32 reference are in tests/test_gpu_attention.py.

The causal-LM loss (transformers ``ForCausalLMLoss``: ``logits.float()`` then cross entropy) becomes
two row kernels over the bf16 logits (``smt_ce_fwd`` / ``smt_ce_bwd``), so the 16.8 GB fp32 logits
copy, its log-softmax and its fp32 gradient are never materialised (tests/test_gpu_cross_entropy.py).

The model's dtype is bf16 or, since ABI v13, fp16 (the reference's ``--dtype fp16``,
``fine_tune.py:955-959``): every kernel is one template body for both formats, rounding where the eager
chain rounds to the model's dtype (tests/test_gpu_fused_fp16.py). fp32 models and mixed dtypes raise
(no silent fallback); the fp8 producer fusions stay bf16-only.
"""
from __future__ import annotations

import ctypes
import os
import weakref

import torch
from torch import nn

from . import _hip


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _need(t: torch.Tensor, what: str, like: torch.Tensor = None):
    """A ROCm tensor of the model's 16-bit dtype: bf16, or fp16 (the reference's --dtype fp16,
    fine_tune.py:955-959; ABI v13) -- and, with ``like``, the same dtype as it."""
    if t.device.type != "cuda" or t.dtype not in (torch.bfloat16, torch.float16):
        raise RuntimeError(f"fused {what}: bf16 / fp16 ROCm tensors only (got {t.dtype} on {t.device})")
    if like is not None and t.dtype != like.dtype:
        raise RuntimeError(f"fused {what}: {t.dtype} beside {like.dtype} (one model dtype)")


def _dt(t: torch.Tensor) -> int:
    """SMT_DTYPE_* of a 16-bit tensor, the kernels' format argument."""
    return _hip.dtype_code16(t.dtype, "fused op")


def _tag(out, op, a2d, b2d=None, w=None, rstd=None):
    """Under the "selective" activation policy, let an SMT linear consuming ``out`` rebuild its column
    blocks from these operands in the backward instead of keeping them (smt.tag_recompute)."""
    from .smt.smt import tag_recompute
    return tag_recompute(out, op, a2d, b2d, w, rstd)


def _rows2d(t: torch.Tensor):
    t2 = t.reshape(-1, t.shape[-1])
    if t2.stride(-1) != 1 or t2.stride(0) % 8 or t2.data_ptr() % 16:
        t2 = t2.contiguous()
    return t2


# ------------------------------------------------------------------------------------------------
# RMSNorm
# ------------------------------------------------------------------------------------------------
class FusedRMSNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, eps):
        _need(x, "rmsnorm")
        _need(weight, "rmsnorm", like=x)
        x2 = _rows2d(x)
        rows, H = x2.shape
        y = torch.empty((rows, H), dtype=x.dtype, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w = weight.contiguous()
        rc = _hip.load().smt_rmsnorm_fwd(x2.data_ptr(), x2.stride(0), w.data_ptr(), y.data_ptr(), y.stride(0),
                                         rstd.data_ptr(), rows, H, float(eps), _dt(x), _stream(x))
        _hip._check(rc, "smt_rmsnorm_fwd")
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        return _tag(y.view(x.shape), _hip.RECOMPUTE_RMSNORM, x2, None, w, rstd)

    @staticmethod
    def backward(ctx, dy):
        x2, w, rstd = ctx.saved_tensors
        dx, dw = _rmsnorm_bwd(x2, w, rstd, dy, ctx.needs_input_grad[1])
        return dx.view(ctx.shape), dw, None


def _rmsnorm_bwd(x2, w, rstd, dy, need_dw: bool, dres=None):
    """dx (+ ``dres``, the gradient reaching the same input by the residual path) and, with
    ``need_dw``, the weight gradient. With both (the full fine-tuning warm-up) one
    ``smt_rmsnorm_bwd_add_dw`` pass; returns ``(dx 2-D, dw or None)``."""
    rows, H = x2.shape
    dy2 = _rows2d(dy)
    dx = torch.empty_like(x2)
    lib = _hip.load()
    dw = partial = None
    if need_dw:
        waves = lib.smt_rmsnorm_bwd_waves(rows)
        partial = torch.empty(waves, H, dtype=torch.float32, device=x2.device)
        dw = torch.empty(H, dtype=w.dtype, device=w.device)
    if dres is not None and need_dw and H % 512 == 0 and H <= 8192:
        dr2 = _rows2d(dres)
        rc = lib.smt_rmsnorm_bwd_add_dw(dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), w.data_ptr(),
                                        rstd.data_ptr(), dr2.data_ptr(), dr2.stride(0), dx.data_ptr(), dx.stride(0),
                                        partial.data_ptr(), dw.data_ptr(), rows, H, _dt(x2), _stream(x2))
        _hip._check(rc, "smt_rmsnorm_bwd_add_dw")
        return dx, dw
    rc = lib.smt_rmsnorm_bwd(dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), w.data_ptr(),
                             rstd.data_ptr(), dx.data_ptr(), dx.stride(0),
                             None if partial is None else partial.data_ptr(),
                             None if dw is None else dw.data_ptr(), rows, H, _dt(x2), _stream(x2))
    _hip._check(rc, "smt_rmsnorm_bwd")
    if dres is not None:
        dx = dx + _rows2d(dres)
    return dx, dw


def fused_rmsnorm_forward(self, hidden_states):
    """Drop-in for ``LlamaRMSNorm.forward``."""
    return FusedRMSNormFn.apply(hidden_states, self.weight, self.variance_epsilon)


class FusedRMSNormResFn(torch.autograd.Function):
    """``LlamaDecoderLayer``'s ``residual = x; y = input_layernorm(x)`` as one node returning
    ``(y, residual)`` (the residual an alias of ``x``), so that the backward receives both gradients
    of ``x`` and sums them inside the norm's backward kernel (``smt_rmsnorm_bwd_add``) instead of an
    autograd add."""

    @staticmethod
    def forward(ctx, x, weight, eps, quant=False, need_y=True):
        if not quant:
            y = FusedRMSNormFn.forward(ctx, x, weight, eps)
            return y, x.view_as(x)
        # fp8 consumers (q/k/v): the norm also emits their e4m3 input (fp8.quant_rows_cached finds it)
        from .fp8 import rmsnorm_quant
        _need(x, "rmsnorm")
        x2, w = _rows2d(x), weight.contiguous()
        _h, y, rstd, q, sq = rmsnorm_quant(x2, None, w, eps, need_y)
        ctx.save_for_backward(x2, w, rstd)
        ctx.shape = x.shape
        ctx.quant_grad = True             # fp8 model: the input gradient feeds the previous down_proj
        y = y.view(x.shape) if y is not None else x.new_zeros(()).expand(x.shape)
        y._smt_q8 = (y._version, q, sq)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dres):
        x2, w, rstd = ctx.saved_tensors              # unpacked once (activation checkpointing)
        if dres is None or ctx.needs_input_grad[1] or x2.shape[1] % 512 or x2.shape[1] > 8192:
            dx, dw = _rmsnorm_bwd(x2, w, rstd, dy, ctx.needs_input_grad[1], dres)
            return dx.view(ctx.shape), dw, None, None, None
        rows, H = x2.shape
        dy2, dr2 = _rows2d(dy), _rows2d(dres)
        if getattr(ctx, "quant_grad", False):
            from .fp8 import rmsnorm_bwd_add_quant
            dx, q, sq = rmsnorm_bwd_add_quant(dy2, x2, w, rstd, dr2)
            dx = dx.view(ctx.shape)
            dx._smt_q8 = (dx._version, q, sq)
            return dx, None, None, None, None
        dx = torch.empty_like(x2)
        rc = _hip.load().smt_rmsnorm_bwd_add(dy2.data_ptr(), dy2.stride(0), x2.data_ptr(), x2.stride(0), w.data_ptr(),
                                             rstd.data_ptr(), dr2.data_ptr(), dr2.stride(0), dx.data_ptr(), H, rows, H,
                                             _dt(x2), _stream(x2))
        _hip._check(rc, "smt_rmsnorm_bwd_add")
        return dx.view(ctx.shape), None, None, None, None


class FusedAddRMSNormFn(torch.autograd.Function):
    """``h = x + residual`` and ``y = RMSNorm(h)`` (LlamaDecoderLayer's attention residual feeding
    ``post_attention_layernorm``) in one pass; the backward adds the gradient that reaches ``h`` by
    the residual path inside the norm's backward. Returns ``(h, y)``."""

    @staticmethod
    def forward(ctx, x, residual, weight, eps, quant=False, need_y=True):
        for t, n in ((x, "x"), (residual, "residual"), (weight, "weight")):
            _need(t, "add+rmsnorm " + n, like=x)
        x2, r2 = _rows2d(x), _rows2d(residual)
        rows, H = x2.shape
        if quant:
            # fp8 consumers (gate/up): the norm also emits their e4m3 input
            from .fp8 import rmsnorm_quant
            w = weight.contiguous()
            h, y, rstd, q, sq = rmsnorm_quant(x2, r2, w, eps, need_y)
            ctx.save_for_backward(h, w, rstd)
            ctx.shape = x.shape
            ctx.quant_grad = True         # fp8 model: the gradient of h feeds o_proj
            y = y.view(x.shape) if y is not None else x.new_zeros(()).expand(x.shape)
            y._smt_q8 = (y._version, q, sq)
            return h.view(x.shape), y
        h = torch.empty((rows, H), dtype=x.dtype, device=x.device)
        y = torch.empty((rows, H), dtype=x.dtype, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        w = weight.contiguous()
        rc = _hip.load().smt_add_rmsnorm_fwd(x2.data_ptr(), x2.stride(0), r2.data_ptr(), r2.stride(0), w.data_ptr(),
                                             h.data_ptr(), H, y.data_ptr(), H, rstd.data_ptr(), rows, H, float(eps),
                                             _dt(x), _stream(x))
        _hip._check(rc, "smt_add_rmsnorm_fwd")
        ctx.save_for_backward(h, w, rstd)
        ctx.shape = x.shape
        return h.view(x.shape), _tag(y.view(x.shape), _hip.RECOMPUTE_RMSNORM, h, None, w, rstd)

    @staticmethod
    def backward(ctx, dh, dy):
        h, w, rstd = ctx.saved_tensors
        rows, H = h.shape
        lib = _hip.load()
        dw = None
        if dy is None:
            dx = dh
        elif ctx.needs_input_grad[2] or dh is None:
            # weight grad (full fine-tuning warm-up; the residual gradient added in the same pass)
            # or no residual gradient: the plain norm backward
            dx, dw = _rmsnorm_bwd(h, w, rstd, dy, ctx.needs_input_grad[2], dh)
            dx = dx.view(ctx.shape)
        elif getattr(ctx, "quant_grad", False):
            from .fp8 import rmsnorm_bwd_add_quant
            dx, q, sq = rmsnorm_bwd_add_quant(_rows2d(dy), h, w, rstd, _rows2d(dh))
            dx = dx.view(ctx.shape)
            dx._smt_q8 = (dx._version, q, sq)
        else:
            dy2, dh2 = _rows2d(dy), _rows2d(dh)
            dx = torch.empty_like(h)
            rc = lib.smt_rmsnorm_bwd_add(dy2.data_ptr(), dy2.stride(0), h.data_ptr(), H, w.data_ptr(), rstd.data_ptr(),
                                         dh2.data_ptr(), dh2.stride(0), dx.data_ptr(), H, rows, H, _dt(h), _stream(h))
            _hip._check(rc, "smt_rmsnorm_bwd_add")
            dx = dx.view(ctx.shape)
        return dx, dx, dw, None, None, None


_RESIDUAL_NORM = os.environ.get("SMT_FUSED_RESIDUAL_NORM", "1") != "0"
# SMT_FUSED_LAYER_TAIL=0: the MLP residual add stays a separate add before the next layer's input norm
_LAYER_TAIL = os.environ.get("SMT_FUSED_LAYER_TAIL", "1") != "0"


def _recomputed(layer) -> bool:
    """transformers' per-layer gradient checkpointing is active for ``layer`` (its forward runs again
    in the backward; the fused tail below must then not span it)."""
    return bool(getattr(layer, "gradient_checkpointing", False) and layer.training)


def _attn_quant(attn, H):
    """(quant, need_y) of a norm feeding this attention's q/k/v (fp8 consumers), as below."""
    if H in (1024, 2048, 4096, 8192) and all(hasattr(attn, n) for n in ("q_proj", "k_proj", "v_proj")):
        from .fp8 import norm_consumers
        return norm_consumers(attn.q_proj, attn.k_proj, attn.v_proj)
    return (False, True)


def fused_decoder_layer_forward(self, hidden_states, attention_mask=None, position_ids=None, past_key_values=None,
                                use_cache=False, position_embeddings=None, **kwargs):
    """Drop-in for ``LlamaDecoderLayer.forward`` with the attention residual add fused into the
    post-attention RMSNorm (:class:`FusedAddRMSNormFn`) and the input norm's two gradients summed in
    its backward (:class:`FusedRMSNormResFn`); the same ops in the same order otherwise."""
    norm1 = self.input_layernorm
    attn, mlp = self.self_attn, self.mlp
    H = hidden_states.shape[-1]
    q1 = q2 = (False, True)
    if H in (1024, 2048, 4096, 8192) and all(hasattr(attn, n) for n in ("q_proj", "k_proj", "v_proj")):
        from .fp8 import norm_consumers
        q1 = norm_consumers(attn.q_proj, attn.k_proj, attn.v_proj)
        if hasattr(mlp, "gate_proj") and hasattr(mlp, "up_proj"):
            q2 = norm_consumers(mlp.gate_proj, mlp.up_proj)
    # the previous layer may have normalised this input already (its fused tail, below): same values
    # as the input norm computes here, and its backward sums the residual gradient the same way
    st = hidden_states.__dict__.pop("_smt_normed", None)
    if (st is not None and st[0] is norm1.weight and st[1] == q1 and st[3] == hidden_states._version
            and not _recomputed(self)):
        residual, hidden_states = hidden_states, st[2]
    elif _RESIDUAL_NORM:
        hidden_states, residual = FusedRMSNormResFn.apply(hidden_states, norm1.weight, norm1.variance_epsilon, *q1)
    else:
        residual = hidden_states
        hidden_states = norm1(hidden_states)
    hidden_states, _ = self.self_attn(hidden_states=hidden_states, attention_mask=attention_mask,
                                      position_ids=position_ids, past_key_values=past_key_values, use_cache=use_cache,
                                      position_embeddings=position_embeddings, **kwargs)
    norm = self.post_attention_layernorm
    residual, hidden_states = FusedAddRMSNormFn.apply(hidden_states, residual, norm.weight, norm.variance_epsilon, *q2)
    hidden_states = self.mlp(hidden_states)
    ref = self.__dict__.get("_smt_next_layer")
    nxt = ref() if ref is not None else None
    if _LAYER_TAIL and _RESIDUAL_NORM and nxt is not None and not _recomputed(self) and not _recomputed(nxt):
        # the MLP residual add fused with the NEXT layer's input RMSNorm (one add+norm pass instead of
        # an add and a norm): the layer still returns h = residual + mlp_out, with the normalised h
        # attached for the next layer, which uses it only if it receives this very tensor unchanged
        # (fp8 attention: the norm also emits the next q/k/v's e4m3 rows, and its backward the
        # down_proj data gradient's, as the next layer's own input norm would)
        qn = _attn_quant(nxt.self_attn, H)
        n1 = nxt.input_layernorm
        h, y = FusedAddRMSNormFn.apply(hidden_states, residual, n1.weight, n1.variance_epsilon, *qn)
        h.__dict__["_smt_normed"] = (n1.weight, qn, y, h._version)
        return h
    return residual + hidden_states


# ------------------------------------------------------------------------------------------------
# RoPE
# ------------------------------------------------------------------------------------------------
def _rope_desc(inp: torch.Tensor, out: torch.Tensor) -> _hip.RopeTensor:
    sb, sh, ss, sd = inp.stride()
    ob, oh, os_, od = out.stride()
    if sd != 1 or od != 1:
        raise RuntimeError("fused rope: head_dim must be the innermost dimension")
    return _hip.RopeTensor(inp.data_ptr(), out.data_ptr(), sb, sh, ss, ob, oh, os_, inp.shape[1], 0)


def _rope_launch(fn_name, q, k, cos, sin, q_layout=None, k_layout=None, in_place=False):
    """Launch the fused rope kernel on q and k; outputs take ``*_layout`` = (shape, stride) (default:
    the input's own layout: [B, S, H, D] storage under the [B, H, S, D] view for HF q/k), or
    overwrite q and k (``in_place``: every thread reads its element pairs before writing them)."""
    B, _Hq, S, D = q.shape
    if cos.dim() != 3 or cos.stride(-1) != 1 or cos.shape != sin.shape or cos.stride() != sin.stride():
        cos, sin = cos.contiguous(), sin.contiguous()
    if cos.shape[0] != B:
        # HF's position embeddings are [1, S, D] for a batch: a zero batch stride instead of B copies
        cos, sin = cos.expand(B, -1, -1), sin.expand(B, -1, -1)
    q = _rope_ready(q)
    k = _rope_ready(k)
    qs, qst = q_layout or (q.shape, q.stride())
    ks, kst = k_layout or (k.shape, k.stride())
    if in_place:
        qo, ko = q, k
    else:
        qo = torch.empty_strided(qs, qst, dtype=q.dtype, device=q.device)
        ko = torch.empty_strided(ks, kst, dtype=k.dtype, device=k.device)
    dq, dk = _rope_desc(q, qo), _rope_desc(k, ko)
    lib = _hip.load()
    rc = getattr(lib, fn_name)(ctypes.byref(dq), ctypes.byref(dk), cos.data_ptr(), sin.data_ptr(), cos.stride(0),
                               cos.stride(1), B, S, D, _dt(q), _stream(q))
    _hip._check(rc, fn_name)
    return qo, ko


def _rope_ready(t: torch.Tensor) -> torch.Tensor:
    """16-byte aligned rows and 8-element strides with head_dim innermost, else a contiguous copy."""
    if t.stride(-1) == 1 and not any(s % 8 for s in t.stride()[:3]) and t.data_ptr() % 16 == 0:
        return t
    return t.contiguous()


class FusedRoPEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, cos, sin):
        for t, n in ((q, "q"), (k, "k"), (cos, "cos"), (sin, "sin")):
            _need(t, "rope " + n, like=q)
        qo, ko = _rope_launch("smt_rope_fwd", q, k, cos, sin)
        ctx.save_for_backward(cos, sin)
        # grads go back in q/k's own layout, so the transpose/view backward of q_proj's output is free
        ctx.layouts = ((q.shape, q.stride()), (k.shape, k.stride()))
        return qo, ko

    @staticmethod
    def backward(ctx, dqo, dko):
        cos, sin = ctx.saved_tensors
        ql, kl = ctx.layouts
        if dqo is None:
            dqo = torch.zeros(ql[0], dtype=cos.dtype, device=cos.device)
        if dko is None:
            dko = torch.zeros(kl[0], dtype=cos.dtype, device=cos.device)
        # the flash attention's joint [dq | dk | dv] gradient (FlashAttnFn joint): rotate the q / k
        # slices in place, so q_proj and k_proj receive slices of the one buffer (dgrad's joint GEMM)
        joint = (getattr(dqo, "_smt_joint", False) and getattr(dko, "_smt_joint", False)
                 and _rope_ready(dqo) is dqo and _rope_ready(dko) is dko)
        dq, dk = _rope_launch("smt_rope_bwd", dqo, dko, cos, sin, ql, kl, in_place=joint)
        return dq, dk, None, None


def fused_apply_rotary_pos_emb(q, k, cos, sin, unsqueeze_dim=1):
    """Drop-in for ``transformers.models.llama.modeling_llama.apply_rotary_pos_emb`` (q/k in
    ``[B, heads, S, head_dim]``, cos/sin ``[B, S, head_dim]``)."""
    if unsqueeze_dim != 1:
        raise NotImplementedError("fused rope: unsqueeze_dim=1 layout only")
    return FusedRoPEFn.apply(q, k, cos, sin)


# ------------------------------------------------------------------------------------------------
# SwiGLU
# ------------------------------------------------------------------------------------------------
class FusedSwiGLUFn(torch.autograd.Function):
    """When gate and up are the two members of one fp8 group (``fp8_linears``), the backward also
    emits their joint e4m3 gradient rows (``fp8.swiglu_bwd_quant``) for the group's single data-
    gradient GEMM, and the bf16 gradients only for a member that needs them (an SMT module's tile
    weight gradient); the others get a zero-stride placeholder that nothing reads."""

    @staticmethod
    def forward(ctx, gate, up, quant_out=False, need_bf16_out=True):
        _need(gate, "swiglu")
        _need(up, "swiglu", like=gate)
        from .fp8 import swiglu_group
        ctx.fp8 = swiglu_group(gate, up)
        g = gate.contiguous()
        u = up.contiguous()
        ctx.save_for_backward(g, u)
        if quant_out:
            # fp8 down_proj: emit its per-row e4m3 input directly (cached on the output, where
            # fp8.quant_rows_cached finds it); the bf16 output only if the consumer reads it
            from .fp8 import swiglu_fwd_quant
            q, sq, h = swiglu_fwd_quant(g, u, need_bf16_out)
            if h is None:
                h = g.new_zeros(()).expand(g.shape)
            h._smt_q8 = (h._version, q, sq)
            return h
        h = torch.empty_like(g)
        rc = _hip.load().smt_swiglu_fwd(g.data_ptr(), u.data_ptr(), h.data_ptr(), g.numel(), _dt(g), _stream(g))
        _hip._check(rc, "smt_swiglu_fwd")
        return _tag(h, _hip.RECOMPUTE_SWIGLU, _rows2d(g), _rows2d(u))

    @staticmethod
    def backward(ctx, dh):
        g, u = ctx.saved_tensors
        dh = dh.contiguous()
        if ctx.fp8 is not None and not ctx.fp8[0].parts and ctx.fp8[0].prequant is None:
            from .fp8 import swiglu_bwd_quant
            acc, need_dg, need_du = ctx.fp8
            q, sq, dg, du = swiglu_bwd_quant(g, u, dh, need_dg, need_du)
            out_g, out_u = _grad_or_placeholder(g, dg, need_dg), _grad_or_placeholder(u, du, need_du)
            # the e4m3 rows stand for exactly these two tensors: the group checks that they reach
            # gate and up unchanged (not summed with another consumer's gradient)
            acc.prequant = (q, sq, (out_g, out_u))
            return out_g, out_u, None, None
        dg = torch.empty_like(g)
        du = torch.empty_like(u)
        rc = _hip.load().smt_swiglu_bwd(g.data_ptr(), u.data_ptr(), dh.data_ptr(), dg.data_ptr(), du.data_ptr(),
                                        g.numel(), _dt(g), _stream(g))
        _hip._check(rc, "smt_swiglu_bwd")
        return dg, du, None, None


def _grad_or_placeholder(like: torch.Tensor, grad, need) -> torch.Tensor:
    """The SwiGLU backward's gradient of gate (up) for autograd: the bf16 gradient itself, or a
    zero-stride placeholder of its shape that nothing reads -- carrying, when the producer wrote only the
    SMT module's row blocks (``need == ("mx_rows", tiles)``), that packed gradient as ``_smt_gpack``
    for linearZ.backward."""
    if grad is not None and need is True:
        return grad
    ph = like.new_zeros(()).expand_as(like)
    if grad is not None:
        ph._smt_gpack = grad
        from .fp8 import MxRowsNeed
        if isinstance(need, MxRowsNeed):
            need.delivered = True
    return ph


def fused_mlp_forward(self, x):
    """Drop-in for ``LlamaMLP.forward`` (SiLU activation). With an fp8 down_proj the SwiGLU also emits
    down_proj's quantised input; a frozen plain down_proj then never reads the bf16 activation."""
    from .fp8 import sole_swiglu_consumer
    with sole_swiglu_consumer():             # gate / up feed only the SwiGLU below
        gate, up = self.gate_proj(x), self.up_proj(x)
    d = self.down_proj
    if getattr(d.weight, "_smt_fp8", None) is not None and gate.shape[-1] <= 16384:
        from . import fp8
        if fp8.FUSED_SWIGLU_QUANT and fp8.FUSED_SWIGLU_FWD_QUANT:
            frozen_plain = type(d) is torch.nn.Linear and not d.weight.requires_grad
            return d(FusedSwiGLUFn.apply(gate, up, True, not frozen_plain))
    return d(FusedSwiGLUFn.apply(gate, up))


# ------------------------------------------------------------------------------------------------
# causal-LM cross entropy
# ------------------------------------------------------------------------------------------------
class FusedCrossEntropyFn(torch.autograd.Function):
    """``F.cross_entropy(logits.float(), labels, ignore_index, reduction=sum) / denom`` over 16-bit
    (bf16 / fp16) logits ``[N, V]`` without the fp32 copy: one pass for the row log-sum-exp, one for the
    gradient in the logits' dtype. ``denom``: fp32 device scalar (valid-label count for the mean, or num_items_in_batch)."""

    @staticmethod
    def forward(ctx, logits2d, labels, ignore_index, denom):
        _need(logits2d, "cross entropy logits")
        if logits2d.stride(1) != 1 or logits2d.stride(0) % 8 or logits2d.data_ptr() % 16:
            logits2d = logits2d.contiguous()
        N, V = logits2d.shape
        labels = labels.to(device=logits2d.device, dtype=torch.int64).contiguous()
        if labels.numel() != N:
            raise ValueError(f"cross entropy: {labels.numel()} labels for {N} logit rows")
        lse = torch.empty(N, dtype=torch.float32, device=logits2d.device)
        rows = torch.empty(N, dtype=torch.float32, device=logits2d.device)
        rc = _hip.load().smt_ce_fwd(logits2d.data_ptr(), logits2d.stride(0), labels.data_ptr(), N, V,
                                    int(ignore_index), lse.data_ptr(), rows.data_ptr(), _dt(logits2d), _stream(logits2d))
        _hip._check(rc, "smt_ce_fwd")
        ctx.save_for_backward(logits2d, labels, lse, denom)
        ctx.ignore_index = int(ignore_index)
        return rows.sum() / denom

    @staticmethod
    def backward(ctx, dloss):
        logits2d, labels, lse, denom = ctx.saved_tensors
        N, V = logits2d.shape
        scale = (dloss.float() / denom).reshape(1).contiguous()
        dlogits = torch.empty_like(logits2d)
        rc = _hip.load().smt_ce_bwd(logits2d.data_ptr(), logits2d.stride(0), labels.data_ptr(), lse.data_ptr(),
                                    scale.data_ptr(), N, V, ctx.ignore_index, dlogits.data_ptr(), dlogits.stride(0),
                                    _dt(logits2d), _stream(logits2d))
        _hip._check(rc, "smt_ce_bwd")
        return dlogits, None, None, None


def fused_causal_lm_loss(logits, labels, vocab_size, num_items_in_batch=None, ignore_index=-100,
                         shift_labels=None, **kwargs):
    """Drop-in for ``transformers.loss.loss_utils.ForCausalLMLoss`` (the loss of
    ``LlamaForCausalLM.forward``): labels shifted left by one with ``ignore_index`` padding, mean over
    non-ignored tokens, or sum / ``num_items_in_batch``."""
    logits2d = logits.reshape(-1, vocab_size)
    shift = _shifted_labels(labels, ignore_index, shift_labels).to(logits2d.device)
    if num_items_in_batch is None:
        denom = (shift != ignore_index).sum().to(torch.float32)
    else:
        denom = torch.as_tensor(num_items_in_batch, device=logits2d.device).to(torch.float32)
    return FusedCrossEntropyFn.apply(logits2d, shift, ignore_index, denom)


def _shifted_labels(labels, ignore_index, shift_labels):
    """ForCausalLMLoss's label shift: position s is scored against token s + 1, the last position
    against ``ignore_index``."""
    if shift_labels is None:
        labels = nn.functional.pad(labels, (0, 1), value=ignore_index)
        shift_labels = labels[..., 1:]
    return shift_labels.reshape(-1)


# ------------------------------------------------------------------------------------------------
# LM head + causal-LM cross entropy, row chunk by row chunk
# ------------------------------------------------------------------------------------------------
LM_HEAD_CHUNK_ROWS = int(os.environ.get("SMT_LM_HEAD_CHUNK_ROWS", "4096"))
# a trainable head (the warm-up) adds each chunk's dlogits^T @ hidden into an fp32 [V, H] accumulator:
# longer chunks mean fewer, longer-K GEMMs (4096-row chunks: 8 x 4.37 ms at the 8B head,
# profiles/r05_k_kernel_stats.csv). The chunk buffer is transient in the forward, below the warm-up's
# peak (the backward's bf16 gradients of every parameter).
LM_HEAD_DW_CHUNK_ROWS = int(os.environ.get("SMT_LM_HEAD_DW_CHUNK_ROWS", "16384"))


class FusedLMHeadLossFn(torch.autograd.Function):
    """``lm_head`` (no bias) followed by :class:`FusedCrossEntropyFn`, without the full ``[T, V]``
    logits. At B 16 x S 2048 x V 128256 the unfused pair keeps the bf16 logits (8.4 GB) for the loss
    backward and allocates the same again for ``dlogits`` at the start of the backward, when every
    activation of the step is still alive: that 16.8 GB is the SMT step's peak HBM (and the
    full fine-tuning warm-up's).

    Here each chunk of ``LM_HEAD_CHUNK_ROWS`` rows runs, inside the forward: the logits GEMM
    (``hidden @ W^T``), the row log-sum-exp (``smt_ce_fwd``), and (when ``hidden`` or ``W`` needs a
    gradient) ``dlogits`` for a unit upstream gradient written over the chunk's logits
    (``smt_ce_bwd`` in place; each element is read and written by one thread), the data gradient
    ``dlogits @ W`` (TN on the engine's transposed copy when there is one, as
    :class:`..engine.FrozenLinearFn` runs it) and, for a trainable head (the warm-up), the chunk's
    ``dlogits^T @ hidden`` added into an fp32 ``[V, H]`` accumulator (hipBLASLt bf16 x bf16 -> fp32,
    beta 1), rounded to bf16 once after the last chunk. Only ``dh [T, H]`` (268 MB) and ``dW``
    are kept; the backward scales them by the upstream gradient.

    Per row this is the unfused arithmetic: the same GEMM products, the same kernels and, for the
    upstream gradient 1 that ``loss.backward()`` gives (``engine.backward`` with one accumulation
    step), the same ``dlogits`` scale ``1 / denom``. Any other upstream gradient is applied to the
    bf16 ``dh`` / ``dW`` (one more rounding than folding it into ``dlogits`` first, exact for powers
    of two). Whether hipBLASLt picks the same kernel for a chunk's GEMM shape as for the whole batch's
    decides bit-identity of the logits and ``dh``; ``dW`` sums the same fp32 products in chunk order
    before its one rounding. tests/test_gpu_cross_entropy.py checks both."""

    @staticmethod
    def forward(ctx, hidden, weight, weight_t, labels, ignore_index, denom, chunk_rows, grad_enabled=True):
        _need(hidden, "lm head loss")
        _need(weight, "lm head loss", like=hidden)
        h2 = _rows2d(hidden)
        N, H = h2.shape
        V = weight.shape[0]
        if weight.shape[1] != H:
            raise ValueError(f"lm head loss: weight {tuple(weight.shape)} for hidden size {H}")
        if V % 8:
            raise ValueError(f"lm head loss: vocabulary {V} is not a multiple of 8")
        labels = labels.to(device=hidden.device, dtype=torch.int64).contiguous()
        if labels.numel() != N:
            raise ValueError(f"lm head loss: {labels.numel()} labels for {N} rows")
        # needs_input_grad reflects requires_grad even under torch.no_grad() (an evaluation forward with
        # labels): the caller passes the grad mode it ran under (inside forward it is always off)
        need_dh = bool(ctx.needs_input_grad[0]) and grad_enabled
        need_dw = bool(ctx.needs_input_grad[1]) and grad_enabled
        lib = _hip.load()
        stream = _stream(hidden)
        dt = _dt(hidden)
        lse = torch.empty(N, dtype=torch.float32, device=hidden.device)
        rows = torch.empty(N, dtype=torch.float32, device=hidden.device)
        dh = torch.empty((N, H), dtype=hidden.dtype, device=hidden.device) if need_dh else None
        scale = (1.0 / denom.to(torch.float32)).reshape(1).contiguous()
        C = max(1, min(max(int(chunk_rows), LM_HEAD_DW_CHUNK_ROWS if need_dw else 0), N))
        buf = torch.empty((C, V), dtype=hidden.dtype, device=hidden.device)
        w_dgrad = weight_t.t() if weight_t is not None else weight
        acc = torch.empty((V, H), dtype=torch.float32, device=hidden.device) if need_dw else None
        for r0 in range(0, N, C):
            c = min(C, N - r0)
            lg = buf[:c]
            hc = h2[r0:r0 + c]
            torch.mm(hc, weight.t(), out=lg)
            rc = lib.smt_ce_fwd(lg.data_ptr(), lg.stride(0), labels[r0:].data_ptr(), c, V, int(ignore_index),
                                lse[r0:].data_ptr(), rows[r0:].data_ptr(), dt, stream)
            _hip._check(rc, "smt_ce_fwd")
            if need_dh or need_dw:
                rc = lib.smt_ce_bwd(lg.data_ptr(), lg.stride(0), labels[r0:].data_ptr(), lse[r0:].data_ptr(),
                                    scale.data_ptr(), c, V, int(ignore_index), lg.data_ptr(), lg.stride(0), dt, stream)
                _hip._check(rc, "smt_ce_bwd")
            if need_dh:
                torch.mm(lg, w_dgrad, out=dh[r0:r0 + c])
            if need_dw:
                if r0 == 0:
                    torch.mm(lg.t(), hc, out_dtype=torch.float32, out=acc)
                else:
                    torch.addmm(acc, lg.t(), hc, out_dtype=torch.float32, out=acc)
        del buf
        dw = None
        if need_dw:
            dw = acc.to(weight.dtype)
            del acc
        ctx.save_for_backward(dh, dw)
        ctx.shape = hidden.shape
        return rows.sum() / denom

    @staticmethod
    def backward(ctx, dloss):
        dh, dw = ctx.saved_tensors
        scale = dloss.float()
        gh = torch.mul(dh, scale).view(ctx.shape) if dh is not None else None
        gw = torch.mul(dw, scale) if dw is not None else None
        return gh, gw, None, None, None, None, None, None


def fused_lm_head_loss(hidden, lm_head: nn.Linear, labels, num_items_in_batch=None, ignore_index=-100,
                       shift_labels=None, chunk_rows=None):
    """``ForCausalLMLoss(lm_head(hidden), labels)`` through :class:`FusedLMHeadLossFn`."""
    shift = _shifted_labels(labels, ignore_index, shift_labels).to(hidden.device)
    if num_items_in_batch is None:
        denom = (shift != ignore_index).sum().to(torch.float32)
    else:
        denom = torch.as_tensor(num_items_in_batch, device=hidden.device).to(torch.float32)
    wt = getattr(lm_head.weight, "_smt_weight_t", None)
    return FusedLMHeadLossFn.apply(hidden, lm_head.weight, wt, shift, ignore_index, denom,
                                   LM_HEAD_CHUNK_ROWS if chunk_rows is None else chunk_rows, torch.is_grad_enabled())


def _fusable_lm_head(head) -> bool:
    w = getattr(head, "weight", None)
    return (type(head) is nn.Linear and head.bias is None and isinstance(w, torch.Tensor)
            and w.device.type == "cuda" and w.dtype in (torch.bfloat16, torch.float16)
            and getattr(w, "_smt_fp8", None) is None)


def fused_causal_lm_forward(self, input_ids=None, attention_mask=None, position_ids=None, past_key_values=None,
                            inputs_embeds=None, labels=None, use_cache=None, logits_to_keep=0, **kwargs):
    """Drop-in for ``LlamaForCausalLM.forward``. With labels, a bias-free bf16 ``lm_head`` (frozen in the
    SMT phase, trainable in the warm-up) and the fused loss patched in, the loss comes from
    :func:`fused_lm_head_loss` and the output carries
    ``logits=None`` (``fine_tune.py:710-711`` reads only ``outputs.loss``); anything else runs
    transformers' own forward."""
    if (labels is None or not _fusable_lm_head(self.lm_head) or not isinstance(logits_to_keep, int)
            or logits_to_keep != 0 or kwargs.get("return_dict") is False
            or getattr(self, "loss_function", None) is not fused_causal_lm_loss):
        return type(self).forward(self, input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids,
                                  past_key_values=past_key_values, inputs_embeds=inputs_embeds, labels=labels,
                                  use_cache=use_cache, logits_to_keep=logits_to_keep, **kwargs)
    kwargs.pop("return_dict", None)
    from transformers.modeling_outputs import CausalLMOutputWithPast
    outputs = self.model(input_ids=input_ids, attention_mask=attention_mask, position_ids=position_ids,
                         past_key_values=past_key_values, inputs_embeds=inputs_embeds, use_cache=use_cache, **kwargs)
    loss = fused_lm_head_loss(outputs.last_hidden_state, self.lm_head, labels,
                              num_items_in_batch=kwargs.get("num_items_in_batch"),
                              shift_labels=kwargs.get("shift_labels"))
    return CausalLMOutputWithPast(loss=loss, logits=None, past_key_values=outputs.past_key_values,
                                  hidden_states=outputs.hidden_states, attentions=outputs.attentions)


# ------------------------------------------------------------------------------------------------
# causal flash attention
# ------------------------------------------------------------------------------------------------
def _attn_tensor(t: torch.Tensor) -> _hip.AttnTensor:
    sb, sh, ss, sd = t.stride()
    if sd != 1:
        raise RuntimeError("flash attention: head_dim must be the innermost dimension")
    return _hip.AttnTensor(t.data_ptr(), sb, sh, ss)


def _attn_ready(t: torch.Tensor) -> torch.Tensor:
    if t.stride(-1) == 1 and not any(s % 8 for s in t.stride()[:3]) and t.data_ptr() % 16 == 0:
        return t
    return t.contiguous()


class KeyMask:
    """The key mask of a padded batch as the smt_flash kernels take it (include/smt_attention.h,
    ``smt_attn_*_kmask``): ``bits`` int64 [B, ceil(S/64)] on the device, bit j%64 of word j/64 set =
    key j takes part. Built by :func:`smt_flash_mask` from transformers' 2-D ``attention_mask``
    (the reference's collator passes ``input_ids != pad_token_id``, helper.py:194-204)."""

    __slots__ = ("bits", "S")

    def __init__(self, bits: torch.Tensor, S: int):
        self.bits, self.S = bits, int(S)

    @classmethod
    def from_padding_mask(cls, mask2d: torch.Tensor) -> "KeyMask":
        B, S = mask2d.shape
        W = -(-S // 64)
        m = torch.zeros(B, W * 64, dtype=torch.int64, device=mask2d.device)
        m[:, :S] = mask2d.to(torch.bool).to(torch.int64)
        shifts = torch.arange(64, dtype=torch.int64, device=mask2d.device)
        # distinct powers of two: the int64 sum is the bitwise OR (bit 63 wraps to the sign bit)
        bits = (m.view(B, W, 64) << shifts).sum(-1)
        return cls(bits.contiguous(), S)


class FlashAttnFn(torch.autograd.Function):
    """Causal GQA attention: q [B, Hq, S, 128], k / v [B, Hkv, S, 128] (any strides with head_dim
    innermost) -> o [B, S, Hq, 128] (the layout transformers' attention functions return).
    ``key_mask``: optional :class:`KeyMask` (padded batches)."""

    @staticmethod
    def forward(ctx, q, k, v, scale, key_mask=None, joint=False):
        for t, n in ((q, "q"), (k, "k"), (v, "v")):
            _need(t, "flash attention " + n, like=q)
        B, Hq, S, D = q.shape
        Hkv = k.shape[1]
        if D != 128 or k.shape != (B, Hkv, S, D) or v.shape != k.shape or Hq % Hkv or S % 4:
            raise NotImplementedError(f"flash attention: head_dim 128, Hq % Hkv == 0, S % 4 == 0 "
                                      f"(q {tuple(q.shape)}, k {tuple(k.shape)})")
        q, k, v = _attn_ready(q), _attn_ready(k), _attn_ready(v)
        for t in (q, k, v):
            if S * t.stride(2) * 2 >= 2 ** 31:
                raise NotImplementedError("flash attention: per-head extent must stay below 2 GiB")
        o = torch.empty(B, S, Hq, D, dtype=q.dtype, device=q.device)
        lse = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
        ov = o.transpose(1, 2)
        shape = _hip.AttnShape(B, Hq, Hkv, S, float(scale), _dt(q))
        km, km_ld = None, 0
        if key_mask is not None:
            if key_mask.S != S or key_mask.bits.shape[0] != B or key_mask.bits.device != q.device:
                raise ValueError(f"flash attention: key mask for [{key_mask.bits.shape[0]}, {key_mask.S}] keys, "
                                 f"batch has [{B}, {S}]")
            km, km_ld = key_mask.bits.data_ptr(), key_mask.bits.shape[1]
        rc = _hip.load().smt_attn_fwd_kmask(ctypes.byref(_attn_tensor(q)), ctypes.byref(_attn_tensor(k)),
                                            ctypes.byref(_attn_tensor(v)), ctypes.byref(_attn_tensor(ov)),
                                            lse.data_ptr(), km, km_ld, ctypes.byref(shape), _stream(q))
        _hip._check(rc, "smt_attn_fwd")
        ctx.save_for_backward(q, k, v, o, lse, key_mask.bits if key_mask is not None else None)
        ctx.scale = float(scale)
        ctx.joint = bool(joint)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, km = ctx.saved_tensors
        B, Hq, S, D = q.shape
        Hkv = k.shape[1]
        do = do if (do.stride(-1) == 1 and not any(s % 8 for s in do.stride()[:3]) and do.data_ptr() % 16 == 0) \
            else do.contiguous()
        if ctx.joint:
            # one [B, S, (Hq + 2 Hkv) D] buffer holding [dq | dk | dv] row by row: q/k/v_proj's data
            # gradients then run as one GEMM (dgrad.py, the engine's joint transposed copy)
            J = torch.empty(B, S, (Hq + 2 * Hkv) * D, dtype=q.dtype, device=q.device)
            dq = J[:, :, :Hq * D].view(B, S, Hq, D).transpose(1, 2)
            dk = J[:, :, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D).transpose(1, 2)
            dv = J[:, :, (Hq + Hkv) * D:].view(B, S, Hkv, D).transpose(1, 2)
            dq._smt_joint = dk._smt_joint = True
        else:
            dq = torch.empty_strided(q.shape, q.stride(), dtype=q.dtype, device=q.device)
            dk = torch.empty_strided(k.shape, k.stride(), dtype=k.dtype, device=k.device)
            dv = torch.empty_strided(v.shape, v.stride(), dtype=v.dtype, device=v.device)
        delta = torch.empty(B, Hq, S, dtype=torch.float32, device=q.device)
        if do.dtype != q.dtype:
            do = do.to(q.dtype)
        shape = _hip.AttnShape(B, Hq, Hkv, S, ctx.scale, _dt(q))
        T = _attn_tensor
        rc = _hip.load().smt_attn_bwd_kmask(ctypes.byref(T(q)), ctypes.byref(T(k)), ctypes.byref(T(v)),
                                            ctypes.byref(T(o.transpose(1, 2))), ctypes.byref(T(do.transpose(1, 2))),
                                            lse.data_ptr(), delta.data_ptr(), ctypes.byref(T(dq)),
                                            ctypes.byref(T(dk)), ctypes.byref(T(dv)),
                                            km.data_ptr() if km is not None else None,
                                            km.shape[1] if km is not None else 0, ctypes.byref(shape), _stream(q))
        _hip._check(rc, "smt_attn_bwd")
        return dq, dk, dv, None, None, None


def flash_attention(q, k, v, scale=None, key_mask: "KeyMask" = None, joint: bool = False):
    """Causal attention ``[B, Hq, S, 128]`` x ``[B, Hkv, S, 128]`` -> ``[B, S, Hq, 128]``; with
    ``key_mask`` the keys it clears take no part (padded batches). ``joint``: the gradients of q, k
    and v go out as slices of one ``[B, S, (Hq + 2 Hkv) * 128]`` buffer (same values)."""
    return FlashAttnFn.apply(q, k, v, scale if scale is not None else q.shape[-1] ** -0.5, key_mask, joint)


def smt_flash_attention_forward(module, query, key, value, attention_mask, dropout=0.0, scaling=None,
                                is_causal=None, **kwargs):
    """transformers attention-function signature (``AttentionInterface``). Causal self-attention,
    unpadded (``attention_mask`` None) or padded (a :class:`KeyMask` from :func:`smt_flash_mask`);
    anything else raises rather than silently changing semantics."""
    if attention_mask is not None and not isinstance(attention_mask, KeyMask):
        raise NotImplementedError("smt_flash attention: only key-padding masks built by smt_flash_mask are "
                                  f"supported (got {type(attention_mask).__name__})")
    if dropout:
        raise NotImplementedError("smt_flash attention: dropout is not supported")
    if is_causal is False or not getattr(module, "is_causal", True):
        raise NotImplementedError("smt_flash attention: causal attention only")
    # the engine marks attention modules whose q/k/v_proj share a joint transposed copy
    return flash_attention(query, key, value, scaling, attention_mask,
                           joint=getattr(module, "_smt_joint_qkv_grad", False)), None


def smt_flash_mask(batch_size, q_length, kv_length, q_offset=0, kv_offset=0, mask_function=None,
                   attention_mask=None, **kwargs):
    """transformers mask-interface builder for ``smt_flash`` (what ``create_causal_mask`` calls):
    ``None`` for a plain causal batch (no mask, or every key valid), a :class:`KeyMask` for a padded
    one: the causal mask AND the 2-D padding mask, exactly the mask ``sdpa_mask`` would materialise
    as [B, 1, S, S]. Anything the kernels do not implement (a KV cache / offsets, packed sequences,
    custom mask functions) raises."""
    from transformers.masking_utils import causal_mask_function
    if mask_function is not None and mask_function is not causal_mask_function:
        raise NotImplementedError("smt_flash attention: custom / packed-sequence masks are not supported")
    if q_offset or kv_offset or q_length != kv_length:
        raise NotImplementedError("smt_flash attention: training-style self-attention only (no KV cache)")
    if attention_mask is None:
        return None
    am = attention_mask
    if am.dim() != 2 or am.shape[0] != batch_size or am.shape[1] < kv_length:
        raise NotImplementedError(f"smt_flash attention: 2-D [B, S] padding mask expected, got {tuple(am.shape)}")
    am = am[:, :kv_length].to(torch.bool)
    if bool(am.all()):
        return None
    return KeyMask.from_padding_mask(am)


ATTN_NAME = "smt_flash"


def register_attention() -> str:
    """Register ``smt_flash`` with transformers (attention function + its mask builder)."""
    from transformers import AttentionInterface
    from transformers.masking_utils import ALL_MASK_ATTENTION_FUNCTIONS
    AttentionInterface.register(ATTN_NAME, smt_flash_attention_forward)
    ALL_MASK_ATTENTION_FUNCTIONS.register(ATTN_NAME, smt_flash_mask)
    return ATTN_NAME


# ------------------------------------------------------------------------------------------------
_EAGER = {}


def _ml():
    from transformers.models.llama import modeling_llama as ml
    if "rope" not in _EAGER:
        _EAGER["rope"] = ml.apply_rotary_pos_emb
    return ml


def eager_apply_rotary_pos_emb(*a, **k):
    """transformers' own apply_rotary_pos_emb (for comparisons while the module global is patched)."""
    return _ml() and _EAGER["rope"](*a, **k)


def patch_llama(model: nn.Module, attention: bool = True, loss: bool = True, lm_head_loss: bool = None) -> dict:
    """Route a transformers LLaMA model's RMSNorm / RoPE / SwiGLU / attention-residual add (and, with ``attention``, its
    attention; with ``loss``, its causal-LM loss) through the fused kernels. RoPE is patched at
    module level (``modeling_llama.apply_rotary_pos_emb``, looked up by ``LlamaAttention.forward`` at
    call time); attention by switching ``config._attn_implementation`` to the registered
    ``smt_flash``; the loss through the model's ``loss_function`` attribute. ``lm_head_loss``
    (default: ``SMT_LM_HEAD_LOSS``, on): with ``loss``, the model's forward runs the LM head and the
    loss together, chunk by chunk, without the full logits (:func:`fused_causal_lm_forward`).
    Returns counts of patched modules. Idempotent."""
    ml = _ml()
    counts = {"rmsnorm": 0, "mlp": 0, "rope": 1, "attention": 0, "loss": 0, "decoder": 0, "lm_head_loss": 0}
    if lm_head_loss is None:
        lm_head_loss = os.environ.get("SMT_LM_HEAD_LOSS", "1") != "0"
    if loss and hasattr(type(model), "loss_function"):
        model.loss_function = fused_causal_lm_loss
        counts["loss"] = 1
        if lm_head_loss and isinstance(model, ml.LlamaForCausalLM):
            model.forward = fused_causal_lm_forward.__get__(model, type(model))
            counts["lm_head_loss"] = 1
    if attention:
        cfg = getattr(model, "config", None)
        if cfg is None:
            raise RuntimeError("patch_llama(attention=True) needs a transformers model with a config")
        if "smt_prev_attn" not in _EAGER:
            _EAGER["smt_prev_attn"] = cfg._attn_implementation
        cfg._attn_implementation = register_attention()
        counts["attention"] = sum(1 for m in model.modules() if isinstance(m, ml.LlamaAttention))
    for m in model.modules():
        if isinstance(m, ml.LlamaRMSNorm):
            m.forward = fused_rmsnorm_forward.__get__(m, type(m))
            counts["rmsnorm"] += 1
        elif isinstance(m, ml.LlamaDecoderLayer):
            m.forward = fused_decoder_layer_forward.__get__(m, type(m))
            counts["decoder"] += 1
        elif isinstance(m, ml.LlamaMLP):
            act = getattr(m, "act_fn", None)
            if act is None or "silu" not in type(act).__name__.lower():
                raise NotImplementedError(f"fused MLP: SiLU activation only (got {type(act).__name__})")
            m.forward = fused_mlp_forward.__get__(m, type(m))
            counts["mlp"] += 1
        elif isinstance(m, nn.ModuleList) and len(m) > 1 and all(isinstance(x, ml.LlamaDecoderLayer) for x in m):
            # each decoder layer's fused tail normalises for the layer after it (a weak reference:
            # not a submodule)
            for i in range(len(m) - 1):
                m[i].__dict__["_smt_next_layer"] = weakref.ref(m[i + 1])
    ml.apply_rotary_pos_emb = fused_apply_rotary_pos_emb
    return counts


def unpatch_llama(model: nn.Module = None) -> None:
    """Undo :func:`patch_llama` (module-level RoPE; per-instance forwards of ``model`` if given)."""
    ml = _ml()
    ml.apply_rotary_pos_emb = _EAGER["rope"]
    if model is not None and "smt_prev_attn" in _EAGER and getattr(model, "config", None) is not None:
        model.config._attn_implementation = _EAGER.pop("smt_prev_attn")
    if model is not None:
        if "_loss_function" in model.__dict__:
            del model.__dict__["_loss_function"]
        if "forward" in model.__dict__:
            del model.__dict__["forward"]
        for m in model.modules():
            if isinstance(m, (ml.LlamaRMSNorm, ml.LlamaMLP, ml.LlamaDecoderLayer)) and "forward" in m.__dict__:
                del m.__dict__["forward"]
            m.__dict__.pop("_smt_next_layer", None)

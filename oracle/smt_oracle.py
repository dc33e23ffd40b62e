"""CPU restatement of the reference SMT hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / CPU baseline. The product (``sparse_matrix_tuning_amd``)
never imports it and has no CPU path.

Every function restates, with torch on the CPU (the library the reference itself computes with),
the reference code at the cited ``file:line`` of yudaohai666/Sparse_Matrix_Tuning. Importing or
running the reference was denied in this environment; the restatement is pinned by
KAT-1 / KAT-2 (derived by reading the reference demos) and by dense-autograd identities,
see tests/test_oracle.py. DeepSpeed's FusedAdam / clipping (external, DeepSpeed 0.16.5) are restated
from their published algorithm: parity unpinned by the reference.
"""
from __future__ import annotations

import heapq
import re
from collections import defaultdict
from typing import Dict, Hashable, List, Sequence, Tuple

import torch

Block_dimension = 256                                   # smt.py:22
_LAYER = re.compile(r'model\.layers\.(\d+)\.')          # smt.py:90, fine_tune.py:718


# ------------------------------------------------------------------------------------------------
# tiles, forward, backward (smt.py:302-413)
# ------------------------------------------------------------------------------------------------
def gather_tiles(weight: torch.Tensor, index_list: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """smt.py:312-325."""
    B = Block_dimension
    out = torch.empty(len(index_list) * B, B, dtype=weight.dtype)
    for i, index in enumerate(index_list):
        out[i * B:(i + 1) * B, :] = weight[index[0] * B:(index[0] + 1) * B, index[1] * B:(index[1] + 1) * B]
    return out


def writeback_tiles(weight: torch.Tensor, selected: torch.Tensor, index_list) -> None:
    """smt.py:332-341 (in place on ``weight``)."""
    B = Block_dimension
    for i, index in enumerate(index_list):
        weight[index[0] * B:(index[0] + 1) * B, index[1] * B:(index[1] + 1) * B] = selected[i * B:(i + 1) * B, :]


def linearz_forward(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """smt.py:366."""
    return torch.matmul(x, weight.t())


def linearz_tile_grads(grad_output: torch.Tensor, x: torch.Tensor, index_list) -> torch.Tensor:
    """smt.py:382-404: per tile, a batched [B,256,S]x[B,S,256] matmul in the input dtype (each
    per-sample partial rounded to that dtype), summed over the batch (``torch.sum(dim=0)``)."""
    B = Block_dimension
    grad_weight = torch.empty(len(index_list) * B, B, dtype=grad_output.dtype)
    for i, index in enumerate(index_list):
        grad_weight[i * B:(i + 1) * B, :] = torch.sum(torch.matmul(
            grad_output.permute(0, 2, 1)[:, index[0] * B:(index[0] + 1) * B, :],
            x[:, :, index[1] * B:(index[1] + 1) * B]), dim=0)
    return grad_weight


def linearz_backward(grad_output: torch.Tensor, x: torch.Tensor, weight: torch.Tensor, index_list):
    """smt.py:382-406: the tile gradients of :func:`linearz_tile_grads`; ``grad_input = g @ W``."""
    grad_weight = linearz_tile_grads(grad_output, x, index_list)
    grad_input = torch.matmul(grad_output, weight)
    return grad_input, grad_weight


def tile_grads_fp64(grad_output: torch.Tensor, x: torch.Tensor, index_list) -> torch.Tensor:
    """Exact-arithmetic truth for the tile gradients from the same (rounded) inputs."""
    B = Block_dimension
    g = grad_output.reshape(-1, grad_output.shape[-1]).double()
    xx = x.reshape(-1, x.shape[-1]).double()
    out = torch.empty(len(index_list) * B, B, dtype=torch.float64)
    for i, (r, c) in enumerate(index_list):
        out[i * B:(i + 1) * B] = g[:, r * B:(r + 1) * B].t() @ xx[:, c * B:(c + 1) * B]
    return out


# ------------------------------------------------------------------------------------------------
# block statistics and selection (smt_helper.py:40-146, 149-251)
# ------------------------------------------------------------------------------------------------
def block_stat(grad: torch.Tensor, d1: int, d2: int, strategy: str) -> torch.Tensor:
    """smt_helper.py:67-78 + 233-251, fp32 CPU reductions exactly as written there."""
    g = grad.reshape(d1, Block_dimension, d2, Block_dimension)
    if strategy == 'mean_abs':
        return g.mean(dim=(1, 3)).abs()
    if strategy == 'abs_mean':
        return g.abs().mean(dim=(1, 3))
    if strategy == 'L1':
        return g.abs().sum(dim=(1, 3))
    if strategy == 'L2':
        return torch.sqrt(torch.sum(g.abs() ** 2, dim=(1, 3)))
    return None


def block_raw_fp64(grad: torch.Tensor, d1: int, d2: int, strategy: str) -> torch.Tensor:
    """What ``smt_block_score`` computes, restated: per block ``[sum of terms, sum of |terms|]`` in
    fp64, with the reference's terms (g, |g|, or the fp32-rounded ``g.abs()**2``)."""
    g = grad.float().reshape(d1, Block_dimension, d2, Block_dimension)
    if strategy == 'mean_abs':
        t = g.double()
    elif strategy in ('abs_mean', 'L1'):
        t = g.abs().double()
    elif strategy == 'L2':
        t = (g * g).double()
    else:
        return None
    return torch.stack([t.sum(dim=(1, 3)), t.abs().sum(dim=(1, 3))], dim=-1).reshape(-1, 2)


def block_stat_fp64(grad: torch.Tensor, d1: int, d2: int, strategy: str) -> torch.Tensor:
    """The same statistic from fp64 sums of the reference's terms, rounded once to fp32 (the
    nominal value the GPU scan reports)."""
    raw = block_raw_fp64(grad, d1, d2, strategy)
    if raw is None:
        return None
    s = raw[:, 0].reshape(d1, d2)
    n = float(Block_dimension * Block_dimension)
    if strategy == 'mean_abs':
        return (s / n).float().abs()
    if strategy == 'abs_mean':
        return (s / n).float()
    if strategy == 'L1':
        return s.float()
    return torch.sqrt(s).float()


def select_submatrix(grads: Dict[Hashable, torch.Tensor], targeted_module_dims, n=660,
                     selection_strategy="no_restriction", calculate_strategy="mean_abs",
                     stat=block_stat, stable=False):
    """smt_helper.py:40-146, including the heap loop of 111-119 and its UnboundLocalError paths.
    ``norm_dist`` calls ``torch.argsort(descending=True)`` on the CPU as smt_helper.py:86 does (ATen's
    std::sort: equal values in its own order); ``stable=True`` only shows where index order differs."""
    block_means = {}
    for key, grad in grads.items():
        d1 = int(targeted_module_dims[key[0]][0] / Block_dimension)
        d2 = int(targeted_module_dims[key[0]][1] / Block_dimension)
        grad.reshape(d1, Block_dimension, d2, Block_dimension)      # RuntimeError on bad dims
        s = stat(grad, d1, d2, calculate_strategy)
        if s is not None:
            block_means[key] = s
    if selection_strategy == "norm_dist":
        ranked_blocks = defaultdict(list)
        if not block_means:
            raise UnboundLocalError("indices")
        for key, block_mean in block_means.items():
            indices = torch.argsort(block_mean.view(-1), descending=True, stable=stable)
            for idx in indices[:n]:
                ranked_blocks[key].append(((idx // block_mean.shape[1]).item(), (idx % block_mean.shape[1]).item()))
        return ranked_blocks
    top_blocks = []
    for key, block_mean in block_means.items():
        for i in range(block_mean.shape[0]):
            for j in range(block_mean.shape[1]):
                abs_mean = block_mean[i, j].item()
                if len(top_blocks) < n:
                    heapq.heappush(top_blocks, (abs_mean, (key, i, j)))
                else:
                    heapq.heappushpop(top_blocks, (abs_mean, (key, i, j)))
    top_blocks.sort(reverse=True)
    if not top_blocks:
        raise UnboundLocalError("mean")
    ranked_blocks = defaultdict(list)
    for _mean, (info, row, col) in top_blocks:
        ranked_blocks[info].append((row, col))
    return ranked_blocks


def select_channel(activation: Dict[Hashable, torch.Tensor], n=660, selection_strategy="no_restriction",
                   calculate_strategy="mean_abs"):
    """smt_helper.py:149-230 (activation channel path; oracle only, product path is 'next')."""
    column_means = {}
    for key, act in activation.items():
        act = torch.sum(act.abs(), dim=0)
        if calculate_strategy == 'mean_abs':
            column_means[key] = torch.mean(act.abs(), dim=0)
        elif calculate_strategy == 'abs_mean':
            column_means[key] = torch.abs(torch.mean(act, dim=0))
        elif calculate_strategy == 'L1':
            column_means[key] = torch.norm(act, p=1, dim=0)
        elif calculate_strategy == 'L2':
            column_means[key] = torch.norm(act, p=2, dim=0)
    if selection_strategy == "norm_dist":
        if not column_means:
            raise UnboundLocalError("indices")          # `del indices` with nothing bound (smt_helper.py:194)
        return {key: torch.argsort(cm, descending=True)[:n].tolist() for key, cm in column_means.items()}
    top_columns = []
    for key, column_mean in column_means.items():
        for idx in range(column_mean.shape[0]):
            value = column_mean[idx].item()
            if len(top_columns) < n:
                heapq.heappush(top_columns, (value, (key, idx)))
            else:
                heapq.heappushpop(top_columns, (value, (key, idx)))
    top_columns.sort(reverse=True)
    if not top_columns:
        raise UnboundLocalError("value")                # `del value` with nothing bound (smt_helper.py:226)
    ranked = defaultdict(list)
    for _value, (key, idx) in top_columns:
        ranked[key].append(idx)
    return ranked


def channel_hook_accumulate(feat: dict, key, x: torch.Tensor) -> None:
    """fine_tune.py:636-667 cache_input_hook at world size 1: ``|x|`` -> fp32 CPU -> first step
    assigns, later steps ``+=`` (the all-reduce over ranks is the identity there)."""
    a = x.abs().detach().cpu().to(torch.float32)
    if key not in feat:
        feat[key] = a
    else:
        feat[key] += a


def bf16_rank_sum(xs: Sequence[torch.Tensor], order=None) -> torch.Tensor:
    """The bf16 sum over ranks of a bf16 ``all_reduce`` (fine_tune.py:655-657), every addition rounded
    to bf16 as a collective's bf16 reduction does: ``order`` is a list of rank indices summed left to
    right (default ``range(len(xs))``) or ``"pairwise"`` (a balanced tree: (x0 + x1) + (x2 + x3) ...).
    For two ranks every order gives the same bits (bf16 addition is commutative); from three ranks on
    the result depends on the order, which is the collective library's (NCCL / RCCL / gloo) internal
    choice -- per element, since ring algorithms start each chunk's reduction at a different rank."""
    xs = [x.to(torch.float32) for x in xs]
    rnd = lambda t: t.to(torch.bfloat16).to(torch.float32)
    if order == "pairwise":
        level = xs
        while len(level) > 1:
            nxt = [rnd(level[i] + level[i + 1]) for i in range(0, len(level) - 1, 2)]
            if len(level) % 2:
                nxt.append(level[-1])
            level = nxt
        return level[0]
    order = list(range(len(xs))) if order is None else list(order)
    if sorted(order) != list(range(len(xs))):
        raise ValueError(f"order {order} is not a permutation of {len(xs)} ranks")
    acc = xs[order[0]]
    for r in order[1:]:
        acc = rnd(acc + xs[r])
    return acc


def channel_hook_accumulate_ranks(feat: dict, key, xs: Sequence[torch.Tensor], order=None) -> None:
    """fine_tune.py:651-665 cache_input_hook at world size len(xs): every rank's ``|x|`` in bf16,
    ``all_reduce`` (sum) in bf16, then fp32 on the CPU, first step assigns, later steps ``+=``. For two
    ranks the collective's one addition is ``bf16(fp32(a) + fp32(b))`` whatever its order; from three
    ranks on the caller names the summation order (:func:`bf16_rank_sum`): the reference's result
    then depends on its collective's internal order (external, unpinned)."""
    if len(xs) == 1:
        return channel_hook_accumulate(feat, key, xs[0])
    if len(xs) > 2 and order is None:
        raise NotImplementedError("above two ranks the bf16 rank sum depends on the collective's order: name one")
    s = bf16_rank_sum([x.detach().cpu().abs() for x in xs], order)
    if key not in feat:
        feat[key] = s
    else:
        feat[key] += s


def channel_raw_fp64(act: torch.Tensor, strategy: str) -> torch.Tensor:
    """What ``smt_channel_score`` computes, restated with its operation order: per channel
    ``sum_s A_s`` (``sum_s A_s^2`` for L2) in fp64, ``A_s = sum_b |act[b, s, c]|`` with b ascending
    from 0; s ascending inside 32-row partials, the partials added in ascending order."""
    a = act.detach().cpu().to(torch.float32).abs().double()
    tot = torch.zeros(a.shape[2], dtype=torch.float64)
    for s0 in range(0, a.shape[1], 32):
        part = torch.zeros(a.shape[2], dtype=torch.float64)
        for s in range(s0, min(a.shape[1], s0 + 32)):
            col = torch.zeros(a.shape[2], dtype=torch.float64)
            for b in range(a.shape[0]):
                col = col + a[b, s]
            part = part + (col * col if strategy == 'L2' else col)
        tot = tot + part
    return tot


def channel_stat_fp64(act: torch.Tensor, strategy: str) -> torch.Tensor:
    """The channel statistic from those fp64 sums, rounded once to fp32 (the GPU's nominal value)."""
    tot = channel_raw_fp64(act, strategy)
    if strategy in ('mean_abs', 'abs_mean'):
        return (tot / act.shape[1]).abs().to(torch.float32)
    if strategy == 'L1':
        return tot.to(torch.float32)
    if strategy == 'L2':
        return tot.sqrt().to(torch.float32)
    raise ValueError(strategy)


def rank_channels(column_means: Dict[Hashable, torch.Tensor], n: int, selection_strategy="no_restriction"):
    """smt_helper.py:186-230 (the heap / argsort half of select_channel) on given fp32 statistics."""
    if selection_strategy == "norm_dist":
        return {key: torch.argsort(cm, descending=True)[:n].tolist() for key, cm in column_means.items()}
    top = []
    for key, cm in column_means.items():
        for idx in range(cm.shape[0]):
            value = cm[idx].item()
            if len(top) < n:
                heapq.heappush(top, (value, (key, idx)))
            else:
                heapq.heappushpop(top, (value, (key, idx)))
    top.sort(reverse=True)
    ranked = defaultdict(list)
    for _value, (key, idx) in top:
        ranked[key].append(idx)
    return ranked


def gather_rows(weight: torch.Tensor, index_list: Sequence[int]) -> torch.Tensor:
    """smt.py:196-204."""
    out = torch.empty(len(index_list), weight.shape[1], dtype=weight.dtype)
    for i, index in enumerate(index_list):
        out[i, :] = weight[index, :]
    return out


def linearchannel_forward(x: torch.Tensor, weight: torch.Tensor, index_list: Sequence[int]):
    """smt.py:221-253: ``(output, partial_input)``."""
    partial = torch.empty(x.shape[0], x.shape[1], len(index_list), dtype=x.dtype)
    for i, index in enumerate(index_list):
        partial[:, :, i] = x[:, :, index]
    return torch.matmul(x, weight.t()), partial


def linearchannel_backward(grad_output: torch.Tensor, partial: torch.Tensor, weight: torch.Tensor):
    """smt.py:256-296: ``grad_weight = sum_b partial[b]^T g[b]`` ([k, out], per-sample products in
    the input dtype), ``grad_input = g @ W``."""
    grad_weight = torch.sum(torch.matmul(partial.permute(0, 2, 1), grad_output), dim=0)
    return torch.matmul(grad_output, weight), grad_weight


def channel_grads_fp64(grad_output: torch.Tensor, x: torch.Tensor, index_list: Sequence[int]) -> torch.Tensor:
    """Exact-arithmetic truth of linearChannel's grad_weight from the same (rounded) inputs."""
    g = grad_output.reshape(-1, grad_output.shape[-1]).double()
    xx = x.reshape(-1, x.shape[-1]).double()[:, list(index_list)]
    return xx.t() @ g


# ------------------------------------------------------------------------------------------------
# trainer segments (fine_tune.py:217-241, 714-767)
# ------------------------------------------------------------------------------------------------
def total_blocks_from_shapes(shapes: Sequence[Tuple[int, ...]]) -> float:
    """fine_tune.py:231-234."""
    total = 0
    for s in shapes:
        if len(s) == 2:
            total += s[0] / 256 * s[1] / 256
    return total


def harvest(named_grads: Sequence[Tuple[str, torch.Tensor]], warmup_grads: dict, attention_warmup_grads: dict,
            num_mlp_blocks: int, num_attention_blocks: int) -> None:
    """fine_tune.py:716-767 on (name, grad) pairs in named_parameters() order (CPU fp32 dicts)."""
    for name, grad in named_grads:
        match = _LAYER.search(name)
        layer_number = int(match.group(1)) if match else None
        if 'mlp' in name and num_mlp_blocks > 0:
            module_name = 'gate_proj' if 'gate_proj' in name else 'up_proj' if 'up_proj' in name else 'down_proj'
            key = (module_name, layer_number)
            if key not in warmup_grads:
                warmup_grads[key] = grad.detach().cpu().to(torch.float32)
            else:
                warmup_grads[key] += grad.detach().cpu().to(torch.float32)
        if 'self_attn' in name and 'weight' in name and num_attention_blocks > 0:
            module_name = 'q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else 'v_proj' if 'v_proj' in name else None
            if module_name is not None:
                key = (module_name, layer_number)
                if key not in attention_warmup_grads:
                    attention_warmup_grads[key] = grad.detach().cpu().to(torch.float32)
                else:
                    attention_warmup_grads[key] += grad.detach().cpu().to(torch.float32)


# ------------------------------------------------------------------------------------------------
# optimizer (DeepSpeed 0.16.5 FusedAdam ADAM_MODE_1 + gradient_clipping; external, restated)
# ------------------------------------------------------------------------------------------------
def clip_coef(grads: List[torch.Tensor], max_norm: float) -> float:
    """DeepSpeed: clip = (||g|| + 1e-6) / max_norm, grads scaled by 1/clip when clip > 1."""
    total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads)).item()
    clip = (total + 1e-6) / max_norm
    return 1.0 / clip if clip > 1 else 1.0


def fused_adam_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
                    lr: float, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.0) -> None:
    """In place on fp32 p, m, v (DeepSpeed multi_tensor_adam.cu, ADAM_MODE_1)."""
    b1, b2 = betas
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    m.mul_(b1).add_((1 - b1) * g)
    v.mul_(b2).add_((1 - b2) * g * g)
    denom = torch.sqrt(v / bc2) + eps
    update = (m / bc1) / denom + weight_decay * p
    p.sub_(lr * update)


# ------------------------------------------------------------------------------------------------
# fp16 training (the reference's --dtype fp16: deepspeed_helpers.py:53-55 sets
# "fp16": {"enabled": True, "loss_scale_window": 100}); DeepSpeed 0.16.5 internals, external and
# restated from its published code (runtime/fp16/loss_scaler.py DynamicLossScaler,
# runtime/zero/stage_1_and_2.py step / unscale_and_clip_grads): parity unpinned by the reference
# ------------------------------------------------------------------------------------------------
class RefDynamicLossScaler:
    """DeepSpeed's dynamic loss scale with its fp16 config defaults (loss_scale 0 = dynamic,
    initial_scale_power 16, loss_scale_window 1000 (the reference: 100), hysteresis 2,
    consecutive_hysteresis False, min_loss_scale 1)."""

    def __init__(self, init_scale=2.0 ** 16, scale_window=1000, min_scale=1.0, delayed_shift=2,
                 consecutive_hysteresis=False, scale_factor=2.0):
        self.cur_scale = float(init_scale)
        self.cur_iter = 0
        self.last_overflow_iter = -1
        self.scale_factor = scale_factor
        self.scale_window = scale_window
        self.min_scale = min_scale
        self.delayed_shift = delayed_shift
        self.cur_hysteresis = delayed_shift
        self.consecutive_hysteresis = consecutive_hysteresis

    def update_scale(self, overflow: bool) -> None:
        if overflow:
            if self.delayed_shift == 1 or self.cur_hysteresis == 1:
                if self.cur_scale == self.min_scale:
                    raise RuntimeError("Current loss scale already at minimum - cannot decrease scale anymore.")
                self.cur_scale = max(self.cur_scale / self.scale_factor, self.min_scale)
            else:
                self.cur_hysteresis -= 1
            self.last_overflow_iter = self.cur_iter
        else:
            if self.consecutive_hysteresis:
                self.cur_hysteresis = self.delayed_shift
            if (self.cur_iter - self.last_overflow_iter) % self.scale_window == 0:
                if not self.consecutive_hysteresis:
                    self.cur_hysteresis = self.delayed_shift
                self.cur_scale *= self.scale_factor
        self.cur_iter += 1


def fp16_step_scales(scaler: RefDynamicLossScaler, grads_scaled: List[torch.Tensor], max_norm: float):
    """One ZeRO-1/2 fp16 step's bookkeeping: overflow = any inf/nan in the (loss-scaled) gradients;
    the scaler updates FIRST, then the gradients are unscaled and clipped with the scale it now holds
    (combined_scale = max(1, (||g_scaled|| / scale + 1e-6) / max_norm) * scale). Returns (overflow,
    multiplier for the scaled gradients; None on overflow: the step is skipped)."""
    overflow = any(not torch.isfinite(g.double()).all().item() for g in grads_scaled)
    scaler.update_scale(overflow)
    if overflow:
        return True, None
    scale = scaler.cur_scale
    combined = scale
    if max_norm > 0:
        total = torch.sqrt(sum((g.double() ** 2).sum() for g in grads_scaled)).item()
        clip = (total / scale + 1e-6) / max_norm
        if clip > 1:
            combined = clip * scale
    return False, 1.0 / combined


# ------------------------------------------------------------------------------------------------
# module-level restatement (smt.py:83-134, 302-413) for end-to-end CPU checks
# ------------------------------------------------------------------------------------------------
class RefLinearZ(torch.autograd.Function):
    """smt.py:347-413."""

    @staticmethod
    def forward(ctx, input, selected_weight, matrix_index_list, weight):
        ctx.save_for_backward(input, weight)
        ctx.index_list = list(matrix_index_list)
        return linearz_forward(input, weight)

    @staticmethod
    def backward(ctx, grad_output):
        input, weight = ctx.saved_tensors
        grad_input, grad_weight = linearz_backward(grad_output, input, weight, ctx.index_list)
        return grad_input, grad_weight, None, None


class RefLinearLayer_MatrixSparsity(torch.nn.Module):
    """smt.py:302-344 (CPU)."""

    def __init__(self, weight, index_list):
        super().__init__()
        self.weight = weight
        self.weight.requires_grad = False
        self.index_list = list(index_list)
        self.selected_weight = torch.nn.Parameter(gather_tiles(weight.data, self.index_list))

    def forward(self, x):
        writeback_tiles(self.weight.data, self.selected_weight.data, self.index_list)
        return RefLinearZ.apply(x, self.selected_weight, self.index_list, self.weight)


def ref_convert(model, selected_mlp, selected_att):
    """smt.py:83-134 (non-mixture branch) with the restated module."""
    names = [n for n, m in model.named_modules() if isinstance(m, torch.nn.Linear) and '.layers' in n]
    for name in names:
        parent = model
        parts = name.split('.')
        for p in parts[:-1]:
            parent = getattr(parent, p)
        module = getattr(parent, parts[-1])
        if not module.weight.requires_grad:
            continue
        match = _LAYER.search(name)
        layer = int(match.group(1)) if match else None
        if "mlp" in name:
            mod = 'gate_proj' if 'gate_proj' in name else 'up_proj' if 'up_proj' in name else 'down_proj'
            setattr(parent, parts[-1], RefLinearLayer_MatrixSparsity(module.weight, selected_mlp[(mod, layer)]))
        elif "self_attn" in name:
            mod = ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
                   'v_proj' if 'v_proj' in name else 'o_proj' if 'o_proj' in name else None)
            setattr(parent, parts[-1], RefLinearLayer_MatrixSparsity(module.weight, selected_att[(mod, layer)]))
    return model


def _attn_name(name):
    return ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else 'v_proj' if 'v_proj' in name
            else 'o_proj' if 'o_proj' in name else None)


def _mlp_name(name):
    return 'gate_proj' if 'gate_proj' in name else 'up_proj' if 'up_proj' in name else 'down_proj'


def _layer_of(name):
    match = _LAYER.search(name)
    return int(match.group(1)) if match else None


def freeze_flags(param_names: Sequence[str], select_parameters, select_attention_parameters,
                 mixture=False, layernorm=False) -> Dict[str, bool]:
    """smt.py:641-745: the requires_grad each named parameter ends up with."""
    out = {}
    for name in param_names:
        if mixture:
            if "mlp" in name:
                out[name] = (_mlp_name(name), _layer_of(name)) in select_parameters.keys()
            elif "self_attn" in name:
                out[name] = (_attn_name(name), _layer_of(name)) in select_parameters.keys()
            elif "embed_tokens" in name:
                out[name] = ('embed_tokens', None) in select_parameters.keys()
            elif ("input_layernorm" in name) or ("post_attention_layernorm" in name):
                out[name] = bool(layernorm)
            else:
                out[name] = False
        else:
            if "mlp" in name:
                out[name] = (_mlp_name(name), _layer_of(name)) in select_parameters.keys()
            elif "self_attn" in name:
                out[name] = (_attn_name(name), _layer_of(name)) in select_attention_parameters.keys()
            else:
                out[name] = False
    return out


def convert_plan(linears: Sequence[Tuple[str, bool]], selected_submatrix, selected_submatrix_attention,
                 part_module_name=('.layers',), mixture=False) -> Dict[str, list]:
    """smt.py:83-179: which ``nn.Linear`` (by name, given whether its weight requires grad) becomes an
    SMT module with which ``index_list`` (``KeyError`` where the reference raises one)."""
    plan = {}
    for name, trainable in linears:
        if not any(part in name for part in part_module_name):
            continue
        if "mlp" in name and trainable:
            plan[name] = list(selected_submatrix[(_mlp_name(name), _layer_of(name))])
        if "self_attn" in name and trainable:
            src = selected_submatrix if mixture else selected_submatrix_attention
            plan[name] = list(src[(_attn_name(name), _layer_of(name))])
        if mixture and "embed_tokens" in name and trainable:
            plan[name] = list(selected_submatrix[('embed_tokens', None)])
    return plan


class RefLinearChannel(torch.autograd.Function):
    """smt.py:217-296."""

    @staticmethod
    def forward(ctx, input, selected_weight, channel_index_list, weight):
        out, partial = linearchannel_forward(input, weight, list(channel_index_list))
        ctx.save_for_backward(partial, weight)
        return out

    @staticmethod
    def backward(ctx, grad_output):
        partial, weight = ctx.saved_tensors
        grad_input, grad_weight = linearchannel_backward(grad_output, partial, weight)
        return grad_input, grad_weight, None, None


class RefLinearLayer_ChannelSparsity(torch.nn.Module):
    """smt.py:185-214 (CPU)."""

    def __init__(self, weight, index_list):
        super().__init__()
        self.weight = weight
        self.weight.requires_grad = False
        self.index_list = list(index_list)
        self.selected_weight = torch.nn.Parameter(gather_rows(weight.data, self.index_list))

    def forward(self, x):
        for i, index in enumerate(self.index_list):
            self.weight.data[index, :] = self.selected_weight.data[i, :]
        return RefLinearChannel.apply(x, self.selected_weight, self.index_list, self.weight)


def ref_convert_channel(model, selected_channel, selected_channel_attention):
    """smt.py:25-80 with the restated channel module."""
    names = [n for n, m in model.named_modules() if isinstance(m, torch.nn.Linear) and '.layers' in n]
    for name in names:
        parent = model
        parts = name.split('.')
        for p in parts[:-1]:
            parent = getattr(parent, p)
        module = getattr(parent, parts[-1])
        if not module.weight.requires_grad:
            continue
        match = _LAYER.search(name)
        layer = int(match.group(1)) if match else None
        if "mlp" in name:
            mod = 'gate_proj' if 'gate_proj' in name else 'up_proj' if 'up_proj' in name else 'down_proj'
            setattr(parent, parts[-1], RefLinearLayer_ChannelSparsity(module.weight, selected_channel[(mod, layer)]))
        elif "self_attn" in name:
            mod = ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
                   'v_proj' if 'v_proj' in name else 'o_proj' if 'o_proj' in name else None)
            setattr(parent, parts[-1], RefLinearLayer_ChannelSparsity(module.weight,
                                                                      selected_channel_attention[(mod, layer)]))
    return model


# ------------------------------------------------------------------------------------------------
# MX-fp8 tile weight gradient (config 5). The reference has no fp8 (fine_tune.py:955-959): this
# restates the build's own documented format (include/smt_hip.h, smt_mx_quant_cols) -- OCP MX with
# 32-element groups along T, e4m3 elements, e8m0 exponents chosen so that nothing saturates -- as the
# checker of the HIP quantiser (bit for bit) and of the MX MFMA kernel (fp64 products of the
# dequantised operands). Its tile gradients are compared with the bf16 path under a stated tolerance.
# ------------------------------------------------------------------------------------------------
def mx_exponent(amax: torch.Tensor) -> torch.Tensor:
    """Smallest e with amax <= 448 * 2^e (amax fp32 >= 0), clamped to >= -127; -127 for amax == 0."""
    bits = amax.float().contiguous().view(torch.int32).to(torch.int64)
    ef = (bits >> 23) & 255
    e = ef - 127 - 8 + ((bits & 0x7FFFFF) > 0x600000).to(torch.int64)
    e = torch.where(ef == 0, torch.full_like(e, -127), e)
    return e.clamp_min(-127)


def mx_quant_cols(x: torch.Tensor, blocks: Sequence[int]):
    """bf16 [T, C] -> (q uint8 [n, ldq/64, 256, 64] e4m3 bits: q[b][t/64][f][t%64] is column f at
    row t; s uint8 [n, ldq/32, 256] e8m0), ldq = ceil64(T)."""
    T = x.shape[0]
    ldq = (T + 63) // 64 * 64
    n = len(blocks)
    q = torch.zeros(n, ldq // 64, 256, 64, dtype=torch.uint8)
    s = torch.empty(n, ldq // 32, 256, dtype=torch.uint8)
    for i, b in enumerate(blocks):
        v = torch.zeros(ldq, 256, dtype=torch.float32)
        v[:T] = x[:, b * 256:(b + 1) * 256].float()
        g = v.view(ldq // 32, 32, 256)
        e = mx_exponent(g.abs().amax(dim=1))                               # [ldq/32, 256]
        inv = torch.pow(2.0, (-e).double()).float()                        # exact powers of two
        qv = (g * inv[:, None, :]).view(ldq, 256)
        q[i] = qv.to(torch.float8_e4m3fn).view(torch.uint8).view(ldq // 64, 64, 256).transpose(1, 2)
        s[i] = (e + 127).to(torch.uint8)
    return q, s


def mx_dequant(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """(q [n, ldq/64, 256, 64], s [n, ldq/32, 256]) -> fp64 [n, ldq, 256] values."""
    n, panels = q.shape[0], q.shape[1]
    vals = q.view(torch.float8_e4m3fn).double().transpose(2, 3).reshape(n, panels * 64, 256)
    scale = torch.pow(2.0, s.double() - 127.0)                             # [n, ldq/32, 256]
    return vals * scale.repeat_interleave(32, dim=1)


def mx_tile_grads_fp64(qg, sg, qx, sx, table: Sequence[Tuple[int, int]]) -> torch.Tensor:
    """fp64 A_i^T B_i over the dequantised MX blocks, [n*256, 256]."""
    a = mx_dequant(qg, sg)
    b = mx_dequant(qx, sx)
    return torch.cat([a[i].t() @ b[j] for i, j in table]) if table else torch.zeros(0, 256, dtype=torch.float64)

"""MI355X drop-in for ``deepspeed/smt/smt_helper.py`` (block scoring and top-n selection).

Scoring (smt_helper.py:54-78, 233-251) runs on the GPU: one multi-tensor launch of the
``block_score`` kernel reads every fp32 gradient once and returns an fp64 raw sum per 256x256
block; the host turns it into the reference's statistic and rounds to fp32, the dtype the
reference compares in (``block_mean[i, j].item()`` of an fp32 tensor, smt_helper.py:114).

Ranking (smt_helper.py:102-146) is host integer/tuple work: the reference keeps the ``n``
largest ``(score, (key, i, j))`` tuples with ``heapq`` and sorts them descending, which is the
first ``n`` of all candidate tuples in descending tuple order (ties fall to the larger module
name, then layer, then i, then j). That order is reproduced exactly; a numpy partition only
pre-filters candidates strictly below the n-th score.

Gradient dicts may live on the CPU (as the reference's warm-up harvest does, fine_tune.py:731);
they are copied to the current ROCm device for scoring. Without a ROCm device the call raises:
there is no CPU scoring path outside ``oracle/``.
"""
from __future__ import annotations

import heapq
import os
from collections import defaultdict
from typing import Dict, Hashable, Optional, Tuple

import numpy as np
import torch

from .. import _hip

Block_dimension = 256

_STRATEGY = {
    "mean_abs": _hip.SCORE_MEAN_ABS,
    "abs_mean": _hip.SCORE_ABS_MEAN,
    "L1": _hip.SCORE_L1,
    "L2": _hip.SCORE_L2,
}


# ------------------------------------------------------------------------------------------------
# statistic helpers with the reference's names (smt_helper.py:233-251); each takes the
# [d1, 256, d2, 256] view and returns the fp32 [d1, d2] block statistic, computed on the GPU.
# ------------------------------------------------------------------------------------------------
def _stat(grad_tensor: torch.Tensor, strategy: str) -> torch.Tensor:
    if grad_tensor.dim() != 4 or grad_tensor.shape[1] != Block_dimension or grad_tensor.shape[3] != Block_dimension:
        raise RuntimeError(f"expected a [d1, 256, d2, 256] view, got {tuple(grad_tensor.shape)}")
    d1, d2 = grad_tensor.shape[0], grad_tensor.shape[2]
    g = _to_device(grad_tensor.reshape(d1 * Block_dimension, d2 * Block_dimension))
    raw = _hip.block_scores([g], [(d1, d2)], _STRATEGY[strategy])[0]
    return torch.from_numpy(finalize_scores(raw.cpu().numpy(), strategy).reshape(d1, d2))


def mean_abs(grad_tensor):
    """``grad_tensor.mean(dim=(1, 3)).abs()`` (smt_helper.py:233-235)."""
    return _stat(grad_tensor, "mean_abs")


def abs_mean_(grad_tensor):
    """``grad_tensor.abs().mean(dim=(1, 3))`` (smt_helper.py:238-240)."""
    return _stat(grad_tensor, "abs_mean")


def L1_norm(grad_tensor):
    """``grad_tensor.abs().sum(dim=(1, 3))`` (smt_helper.py:243-246)."""
    return _stat(grad_tensor, "L1")


def L2_norm(grad_tensor):
    """``sqrt(sum(abs()**2, dim=(1, 3)))`` (smt_helper.py:249-251)."""
    return _stat(grad_tensor, "L2")


def finalize_scores(raw: np.ndarray, strategy: str) -> np.ndarray:
    """fp64 raw block sums -> the reference's fp32 statistic (rounded once)."""
    n = float(Block_dimension * Block_dimension)
    if strategy == "mean_abs":
        return np.abs((raw / n).astype(np.float32))
    if strategy == "abs_mean":
        return (raw / n).astype(np.float32)
    if strategy == "L1":
        return raw.astype(np.float32)
    if strategy == "L2":
        return np.sqrt(raw).astype(np.float32)
    raise ValueError(strategy)


def _to_device(t: torch.Tensor) -> torch.Tensor:
    if t.device.type == "cuda":
        return t if t.dtype == torch.float32 else t.float()
    if not torch.cuda.is_available():
        raise RuntimeError("SMT block scoring runs on a ROCm device; none is available "
                           "(the CPU restatement is oracle/, test-only)")
    return t.to(device=torch.device("cuda", torch.cuda.current_device()), dtype=torch.float32)


def score_blocks(grads: Dict[Hashable, torch.Tensor], targeted_module_dims: Dict[str, list],
                 calculate_strategy: str = "mean_abs") -> Dict[Hashable, np.ndarray]:
    """smt_helper.py:54-78: per key, the fp32 ``[d1, d2]`` block statistic. Keys with an unknown
    strategy are skipped exactly as in the reference (no branch assigns them)."""
    if calculate_strategy not in _STRATEGY:
        return {}
    keys, tensors, dims = [], [], []
    for key, grad in grads.items():
        name = key[0]
        d1 = int(targeted_module_dims[name][0] / Block_dimension)
        d2 = int(targeted_module_dims[name][1] / Block_dimension)
        numel = grad.numel()
        if numel != d1 * Block_dimension * d2 * Block_dimension:
            raise RuntimeError(f"shape '[{d1}, {Block_dimension}, {d2}, {Block_dimension}]' is invalid "
                               f"for input of size {numel}")
        keys.append(key)
        tensors.append(_to_device(grad).reshape(d1 * Block_dimension, d2 * Block_dimension))
        dims.append((d1, d2))
    if not keys:
        return {}
    raws = _hip.block_scores(tensors, dims, _STRATEGY[calculate_strategy])
    host = torch.cat([r for r in raws]).cpu().numpy()
    out, off = {}, 0
    for key, (d1, d2) in zip(keys, dims):
        out[key] = finalize_scores(host[off:off + d1 * d2], calculate_strategy).reshape(d1, d2)
        off += d1 * d2
    return out


def rank_blocks(block_means: Dict[Hashable, np.ndarray], n: int,
                selection_strategy: str = "no_restriction") -> defaultdict:
    """smt_helper.py:81-146 on precomputed fp32 block statistics (host logic)."""
    if not block_means:
        # the reference reaches `del indices` / `del mean` with nothing bound
        raise UnboundLocalError("cannot access local variable 'mean' where it is not associated with a value "
                                "(no candidate blocks: empty gradients or unknown calculate_strategy)")
    ranked_blocks = defaultdict(list)
    if selection_strategy == "norm_dist":
        # per key: the n best blocks by descending score; ties in index order (the reference's
        # unstable torch.argsort leaves tie order unspecified)
        for key, bm in block_means.items():
            flat = np.asarray(bm, dtype=np.float32).reshape(-1)
            order = np.argsort(-flat.astype(np.float64), kind="stable")[:max(n, 0)]
            d2 = bm.shape[1]
            for idx in order:
                ranked_blocks[key].append((int(idx // d2), int(idx % d2)))
        return ranked_blocks

    if n <= 0:
        raise UnboundLocalError("cannot access local variable 'mean' where it is not associated with a value "
                                "(n <= 0 selects no block)")
    # Pre-filter: keep only candidates whose score is >= the n-th largest score (all ties kept),
    # then order them exactly as the reference's tuples.
    all_scores = np.concatenate([np.asarray(v, dtype=np.float32).reshape(-1) for v in block_means.values()])
    if n < all_scores.size:
        thresh = np.partition(all_scores, all_scores.size - n)[all_scores.size - n]
    else:
        thresh = -np.inf
    cands = []
    for key, bm in block_means.items():
        bm = np.asarray(bm, dtype=np.float32)
        d2 = bm.shape[1]
        flat = bm.reshape(-1)
        for idx in np.nonzero(flat >= thresh)[0]:
            cands.append((float(flat[idx]), (key, int(idx // d2), int(idx % d2))))
    top_blocks = heapq.nlargest(n, cands)       # == sorted(cands, reverse=True)[:n]
    for _mean, (info, row, col) in top_blocks:
        ranked_blocks[info].append((row, col))
    return ranked_blocks


def analyze_gradient_distribution(gradients_per_key, key_string, output_dir):
    """smt_helper.py:14-38: histogram of block scores per module (matplotlib, host only)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    n_keys = len(gradients_per_key)
    n_cols = 3
    n_rows = (n_keys + n_cols - 1) // n_cols
    fig, axes = plt.subplots(n_rows, n_cols, figsize=(15, 5 * n_rows))
    axes = np.asarray(axes).flatten()
    for ax, (key, values) in zip(axes, gradients_per_key.items()):
        ax.hist(np.asarray(values), bins=150, alpha=0.7, edgecolor='black')
        ax.set_xlabel('Gradient Magnitude', fontsize=10)
        ax.set_ylabel('Frequency', fontsize=10)
        ax.set_title(f'{key}')
    for i in range(n_keys, len(axes)):
        axes[i].axis('off')
    plt.tight_layout()
    plt.savefig(os.path.join(output_dir, f'gradient_histograms_{key_string}.png'), dpi=300, bbox_inches='tight')
    plt.close()


def select_submatrix_based_on_grads(grads,
                                    targeted_module_dims,
                                    n=660,
                                    selection_strategy="no_restriction",
                                    calculate_strategy="mean_abs",
                                    model="yahma/llama-13b-hf",
                                    do_gradient_distribution_analysis=False,
                                    output_dir=""):
    """smt_helper.py:40-146. ``grads``: ``{(module_name, layer): fp32 [out, in]}``; returns
    ``defaultdict(list)`` ``{(module_name, layer): [(row_block, col_block), ...]}`` with each
    key's list in descending tuple order (the tile order of LinearLayer_MatrixSparsity)."""
    block_means = score_blocks(grads, targeted_module_dims, calculate_strategy)
    if do_gradient_distribution_analysis and selection_strategy != "norm_dist" and block_means:
        per_key = {}
        for key in block_means:
            per_key.setdefault(key[0], [])
        for key, bm in block_means.items():
            per_key[key[0]].extend(float(v) for v in np.asarray(bm).reshape(-1))
        analyze_gradient_distribution(per_key, "_".join(str(k) for k in per_key), output_dir)
    return rank_blocks(block_means, n, selection_strategy)


class ChannelActivation:
    """Device-resident harvested activations of one ``(module, layer)`` key: fp64
    ``acc[s, c] = sum over steps, ranks and batch of |x[b, s, c]|`` (what the reference's CPU
    ``[B, S, in]`` fp32 dict entry holds after ``torch.sum(act.abs(), dim=0)``, smt_helper.py:170)."""

    __slots__ = ("acc", "steps")

    def __init__(self, acc: torch.Tensor, steps: int = 0):
        self.acc = acc
        self.steps = steps


def _channel_acc(act) -> torch.Tensor:
    if isinstance(act, ChannelActivation):
        return act.acc
    if act.dim() != 3:
        raise IndexError(f"activation must be [batch, seq, channels] (the hook input), got {tuple(act.shape)}")
    x = act
    if x.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("SMT channel scoring runs on a ROCm device; none is available "
                               "(the CPU restatement is oracle/, test-only)")
        x = x.to(torch.device("cuda", torch.cuda.current_device()))
    if x.stride(2) != 1 or x.data_ptr() % 16 or x.stride(1) % 8 or x.stride(0) % 8:
        x = x.contiguous()
    acc = torch.empty(x.shape[1], x.shape[2], dtype=torch.float64, device=x.device)
    _hip.act_accumulate(x, acc, assign=True)
    return acc


def finalize_channel_scores(raw: np.ndarray, seq_len: int, strategy: str) -> np.ndarray:
    """fp64 raw column sums over the sequence -> the reference's fp32 statistic (smt_helper.py:171-184;
    the harvested values are non-negative, so mean_abs == abs_mean)."""
    if strategy in ("mean_abs", "abs_mean"):
        return np.abs(raw / float(seq_len)).astype(np.float32)
    if strategy == "L1":
        return raw.astype(np.float32)
    if strategy == "L2":
        return np.sqrt(raw).astype(np.float32)
    raise ValueError(strategy)


def score_channels(activation: Dict[Hashable, object], calculate_strategy: str = "mean_abs") -> Dict[Hashable, np.ndarray]:
    """smt_helper.py:167-184 on the GPU: per key, the fp32 per-channel statistic. Keys with an
    unknown strategy are skipped as in the reference (no branch assigns them)."""
    if calculate_strategy not in _STRATEGY:
        return {}
    out = {}
    for key, act in activation.items():
        acc = _channel_acc(act)
        raw = _hip.channel_scores(acc, _STRATEGY[calculate_strategy])
        out[key] = finalize_channel_scores(raw.cpu().numpy(), acc.shape[0], calculate_strategy)
    return out


def rank_channels(column_means: Dict[Hashable, np.ndarray], n: int,
                  selection_strategy: str = "no_restriction") -> defaultdict:
    """smt_helper.py:186-230 on precomputed fp32 channel statistics (host logic). ``no_restriction``:
    the first ``n`` of all ``(score, (key, idx))`` tuples in descending order, grouped per key in that
    order; ``norm_dist``: the ``n`` best channels of every key."""
    if not column_means:
        raise UnboundLocalError("cannot access local variable 'value' where it is not associated with a value "
                                "(no candidate channels: empty activations or unknown calculate_strategy)")
    ranked = defaultdict(list)
    if selection_strategy == "norm_dist":
        for key, cm in column_means.items():
            flat = np.asarray(cm, dtype=np.float32).reshape(-1)
            # ties in index order (the reference's unstable torch.argsort leaves them unspecified)
            ranked[key] = [int(i) for i in np.argsort(-flat.astype(np.float64), kind="stable")[:max(n, 0)]]
        return ranked
    if n <= 0:
        raise UnboundLocalError("cannot access local variable 'value' where it is not associated with a value "
                                "(n <= 0 selects no channel)")
    all_scores = np.concatenate([np.asarray(v, dtype=np.float32).reshape(-1) for v in column_means.values()])
    thresh = np.partition(all_scores, all_scores.size - n)[all_scores.size - n] if n < all_scores.size else -np.inf
    cands = []
    for key, cm in column_means.items():
        flat = np.asarray(cm, dtype=np.float32).reshape(-1)
        for idx in np.nonzero(flat >= thresh)[0]:
            cands.append((float(flat[idx]), (key, int(idx))))
    for _value, (key, idx) in heapq.nlargest(n, cands):
        ranked[key].append(idx)
    return ranked


def select_channel_based_on_activation(activation, n=660, selection_strategy="no_restriction",
                                       calculate_strategy="mean_abs", model="yahma/llama-13b-hf"):
    """smt_helper.py:149-230. ``activation``: ``{(module_name, layer): act}`` where ``act`` is the
    reference's ``[B, S, in]`` tensor of summed ``|x|`` (any device) or a :class:`ChannelActivation`
    from :class:`sparse_matrix_tuning_amd.trainer.ActivationHarvester`. Returns
    ``defaultdict(list)`` ``{key: [channel, ...]}`` with each list in descending tuple order (the row
    order of LinearLayer_ChannelSparsity)."""
    return rank_channels(score_channels(activation, calculate_strategy), n, selection_strategy)


def get_blocks(model):
    """smt_helper.py:272-294."""
    name = model.__class__.__name__
    if name in ("LlamaForCausalLM", "LlavaLlamaForCausalLM"):
        return model.model.layers
    if name == "OPTForCausalLM":
        return model.model.decoder.layers
    if name == "BloomForCausalLM":
        return model.transformer.h
    low = str(model.__class__).lower()
    if "mpt" in low:
        return model.transformer.blocks
    if "falcon" in low or "bigcode" in low:
        return model.transformer.h
    if "neox" in low:
        return model.gpt_neox.layers
    raise NotImplementedError(type(model))


def get_named_linears(module):
    """smt_helper.py:297-302."""
    import torch.nn as nn
    return {name: m for name, m in module.named_modules() if isinstance(m, nn.Linear)}

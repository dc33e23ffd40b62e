"""MI355X drop-in for ``deepspeed/smt/smt_helper.py`` (block scoring and top-n selection).

Scoring (smt_helper.py:54-78, 233-251) runs on the GPU: one multi-tensor launch of the
``block_score`` kernel reads every fp32 gradient once and returns, per 256x256 block, the fp64 sum
of the reference's terms and of their magnitudes. The host turns that into the reference's
statistic rounded to fp32 (the dtype the reference compares in, ``block_mean[i, j].item()``,
smt_helper.py:114) and into an interval that provably contains the value ATen's fp32 CPU reduction
gives (:mod:`.ranking`).

Ranking (smt_helper.py:102-146) is host integer/tuple work: the first ``n`` of all
``(score, (key, i, j))`` tuples in descending order (ties to the larger module name, then layer,
then i, then j). Where two scores the ranking depends on are too close for the fp64 estimate to
decide, the keys involved are re-scored with the reference's own expression on the host CPU
(``grad.reshape(d1, 256, d2, 256)`` reduced as in smt_helper.py:233-251, over the whole key so
ATen's reduction order per block is the reference's), which makes the selection identical to the
reference's, bit for bit. ``ranking.LAST_REPORT`` says how many blocks that took.

Gradient dicts may live on the CPU (as the reference's warm-up harvest does, fine_tune.py:731);
they are copied to the current ROCm device for scoring. Without a ROCm device the call raises:
the GPU scan has no CPU substitute (the host re-score only decides near-ties).
"""
from __future__ import annotations

import os
from collections import defaultdict
from typing import Dict, Hashable, List, Optional, Tuple

import numpy as np
import torch

from .. import _hip
from . import ranking

Block_dimension = 256

_STRATEGY = {
    "mean_abs": _hip.SCORE_MEAN_ABS,
    "abs_mean": _hip.SCORE_ABS_MEAN,
    "L1": _hip.SCORE_L1,
    "L2": _hip.SCORE_L2,
}


# ------------------------------------------------------------------------------------------------
# statistic helpers with the reference's names (smt_helper.py:233-251); each takes the
# [d1, 256, d2, 256] view and returns the fp32 [d1, d2] block statistic computed on the GPU (the
# fp64 sum rounded once: within the interval of ranking.block_intervals of the reference's value).
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
    """fp64 block sums (``[n, 2]`` from the kernel, or ``[n]`` sums of terms) -> the reference's
    fp32 statistic, rounded once."""
    raw = np.asarray(raw, dtype=np.float64)
    if raw.ndim == 2:
        raw = raw[:, 0]
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


def reference_block_stat(grad: torch.Tensor, d1: int, d2: int, strategy: str) -> np.ndarray:
    """The reference's own expression (smt_helper.py:67-78, 233-251) on the host CPU in fp32: the
    exact values the reference ranks. Used by the ranking for the few keys whose order the GPU
    estimate cannot decide."""
    g = grad.detach()
    if g.device.type != "cpu":
        g = g.cpu()
    g = g.to(torch.float32).reshape(d1, Block_dimension, d2, Block_dimension)
    if strategy == "mean_abs":
        s = g.mean(dim=(1, 3)).abs()
    elif strategy == "abs_mean":
        s = g.abs().mean(dim=(1, 3))
    elif strategy == "L1":
        s = g.abs().sum(dim=(1, 3))
    elif strategy == "L2":
        s = torch.sqrt(torch.sum(g.abs() ** 2, dim=(1, 3)))
    else:
        raise ValueError(strategy)
    return s.numpy().reshape(-1)


# Whether ATen's value of a block equals its value computed over just the block's row of blocks
# (the per-output reduction order does not depend on the other rows): checked against the whole key
# once per (strategy, block grid, host thread count) and process, since ATen's split of a reduction
# depends on the output count and the threads; if it ever differed, whole keys would be re-scored.
_ROW_SLICE_OK: Dict[tuple, bool] = {}


def block_rescorer(grad: torch.Tensor, d1: int, d2: int, strategy: str):
    """``rescore(flat)`` for :class:`ranking.KeyScores`: the reference's values of the 256-row block
    rows holding the requested blocks (reference_block_stat on ``grad[r*256:(r+1)*256]``: the same
    expression over a slice, 1/d1 of the key's bytes to copy and reduce)."""
    def rescore(flat):
        rows = np.unique(np.asarray(flat, dtype=np.int64) // d2)
        key = (strategy, d1, d2, torch.get_num_threads())
        ok = _ROW_SLICE_OK.get(key)
        if ok is None:
            full = reference_block_stat(grad, d1, d2, strategy)
            r0 = int(rows[0])
            part = reference_block_stat(grad[r0 * Block_dimension:(r0 + 1) * Block_dimension], 1, d2, strategy)
            ok = _ROW_SLICE_OK[key] = bool(np.array_equal(part, full[r0 * d2:(r0 + 1) * d2]))
            if not ok:
                return np.arange(d1 * d2), full
        if not ok:
            return np.arange(d1 * d2), reference_block_stat(grad, d1, d2, strategy)
        covered, vals = [], []
        for r in rows:
            r = int(r)
            covered.append(np.arange(r * d2, (r + 1) * d2))
            vals.append(reference_block_stat(grad[r * Block_dimension:(r + 1) * Block_dimension], 1, d2, strategy))
        return np.concatenate(covered), np.concatenate(vals)
    return rescore


def _to_device(t: torch.Tensor) -> torch.Tensor:
    if t.device.type == "cuda":
        return t if t.dtype == torch.float32 else t.float()
    if not torch.cuda.is_available():
        raise RuntimeError("SMT block scoring runs on a ROCm device; none is available "
                           "(the CPU restatement is oracle/, test-only)")
    return t.to(device=torch.device("cuda", torch.cuda.current_device()), dtype=torch.float32)


def score_block_entries(grads: Dict[Hashable, torch.Tensor], targeted_module_dims: Dict[str, list],
                        calculate_strategy: str = "mean_abs") -> List[ranking.KeyScores]:
    """smt_helper.py:54-78 on the GPU: per key, the block statistics as :class:`ranking.KeyScores`
    (nominal fp32 values, intervals holding the reference's values, the host re-score). Keys with an
    unknown strategy are skipped exactly as in the reference (no branch assigns them)."""
    if calculate_strategy not in _STRATEGY:
        return []
    keys, sources, tensors, dims = [], [], [], []
    for key, grad in grads.items():
        name = key[0]
        d1 = int(targeted_module_dims[name][0] / Block_dimension)
        d2 = int(targeted_module_dims[name][1] / Block_dimension)
        numel = grad.numel()
        if numel != d1 * Block_dimension * d2 * Block_dimension:
            raise RuntimeError(f"shape '[{d1}, {Block_dimension}, {d2}, {Block_dimension}]' is invalid "
                               f"for input of size {numel}")
        keys.append(key)
        sources.append(grad)
        tensors.append(_to_device(grad).reshape(d1 * Block_dimension, d2 * Block_dimension))
        dims.append((d1, d2))
    if not keys:
        return []
    raws = _hip.block_scores(tensors, dims, _STRATEGY[calculate_strategy])
    del tensors
    host = torch.cat(raws).cpu().numpy()
    entries, off = [], 0
    for key, src, (d1, d2) in zip(keys, sources, dims):
        raw = host[off:off + d1 * d2]
        off += d1 * d2
        nominal, lo, hi = ranking.block_intervals(raw, calculate_strategy)
        g2 = src.reshape(d1 * Block_dimension, d2 * Block_dimension)
        entries.append(ranking.KeyScores(
            key, (d1, d2), nominal, lo, hi, rescore=block_rescorer(g2, d1, d2, calculate_strategy),
            bounds=lambda worst, raw=raw: ranking.block_intervals(raw, calculate_strategy, worst)[1:]))
    return entries


def score_blocks(grads: Dict[Hashable, torch.Tensor], targeted_module_dims: Dict[str, list],
                 calculate_strategy: str = "mean_abs") -> Dict[Hashable, np.ndarray]:
    """Per key, the nominal fp32 ``[d1, d2]`` block statistic (GPU, fp64 rounded once)."""
    return {e.key: e.nominal.reshape(e.shape)
            for e in score_block_entries(grads, targeted_module_dims, calculate_strategy)}


def _exact_entries(values: Dict[Hashable, np.ndarray]) -> List[ranking.KeyScores]:
    out = []
    for key, v in values.items():
        a = np.asarray(v, dtype=np.float32)
        shape = a.shape if a.ndim else (1,)
        a64 = a.reshape(-1).astype(np.float64)
        e = ranking.KeyScores(key, shape, a, a64, a64, rescore=ranking.whole_key(lambda a=a: a))
        out.append(e)
    return out


def _rank_block_entries(entries: List[ranking.KeyScores], n: int, selection_strategy: str) -> defaultdict:
    if not entries:
        # the reference reaches `del indices` / `del mean` with nothing bound
        raise UnboundLocalError("cannot access local variable 'mean' where it is not associated with a value "
                                "(no candidate blocks: empty gradients or unknown calculate_strategy)")
    to_ij = lambda e, f: (int(f // e.shape[1]), int(f % e.shape[1]))
    if selection_strategy == "norm_dist":
        ranked = defaultdict(list)
        for e, flats in zip(entries, ranking.top_n_per_key(entries, n)):
            for f in flats:                     # a key is only created by an append, as in smt_helper.py:96
                ranked[e.key].append(to_ij(e, f))
        return ranked
    if n <= 0:
        raise UnboundLocalError("cannot access local variable 'mean' where it is not associated with a value "
                                "(n <= 0 selects no block)")
    return ranking.group(entries, ranking.top_n(entries, n), to_ij)


def rank_blocks(block_means: Dict[Hashable, np.ndarray], n: int,
                selection_strategy: str = "no_restriction") -> defaultdict:
    """smt_helper.py:81-146 on given exact fp32 block statistics ``{key: [d1, d2]}`` (host logic)."""
    return _rank_block_entries(_exact_entries(block_means), n, selection_strategy)


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
    key's list in descending tuple order (the tile order of LinearLayer_MatrixSparsity), identical
    to the reference's."""
    entries = score_block_entries(grads, targeted_module_dims, calculate_strategy)
    if do_gradient_distribution_analysis and selection_strategy != "norm_dist" and entries:
        per_key = {}
        for e in entries:
            per_key.setdefault(e.key[0], [])
        for e in entries:
            per_key[e.key[0]].extend(float(v) for v in e.nominal)
        analyze_gradient_distribution(per_key, "_".join(str(k) for k in per_key), output_dir)
    return _rank_block_entries(entries, n, selection_strategy)


class ChannelActivation:
    """Device-resident harvested activations of one ``(module, layer)`` key: the fp32
    ``[B, S, in]`` tensor the reference keeps on the CPU (``feat[key] = |x|`` then ``+= |x|`` over
    steps, fine_tune.py:636-667), here in HBM and updated elementwise by ``smt_act_accumulate``.
    Keys whose linears read the same input (q/k/v, gate/up) share one object."""

    __slots__ = ("acc", "steps")

    def __init__(self, acc: torch.Tensor, steps: int = 0):
        self.acc = acc
        self.steps = steps


def _channel_sources(act) -> Tuple[torch.Tensor, torch.Tensor]:
    """(fp32 [B, S, in] on the device for the GPU scan, the tensor the host re-score reads)."""
    if isinstance(act, ChannelActivation):
        return act.acc, act.acc
    if act.dim() != 3:
        raise IndexError(f"activation must be [batch, seq, channels] (the hook input), got {tuple(act.shape)}")
    x = act
    if x.device.type != "cuda":
        if not torch.cuda.is_available():
            raise RuntimeError("SMT channel scoring runs on a ROCm device; none is available "
                               "(the CPU restatement is oracle/, test-only)")
        x = x.to(torch.device("cuda", torch.cuda.current_device()))
    x = x.to(torch.float32)
    if not x.is_contiguous() or x.data_ptr() % 16 or x.shape[2] % 8:
        if x.shape[2] % 8:
            pad = torch.zeros(x.shape[0], x.shape[1], (-x.shape[2]) % 8, dtype=x.dtype, device=x.device)
            x = torch.cat([x, pad], dim=2)
        x = x.contiguous()
    return x, act


def finalize_channel_scores(raw: np.ndarray, seq_len: int, strategy: str) -> np.ndarray:
    """fp64 column sums over (batch, sequence) -> the reference's fp32 statistic (smt_helper.py:171-184;
    the harvested values are non-negative, so mean_abs == abs_mean)."""
    if strategy in ("mean_abs", "abs_mean"):
        return np.abs(raw / float(seq_len)).astype(np.float32)
    if strategy == "L1":
        return raw.astype(np.float32)
    if strategy == "L2":
        return np.sqrt(raw).astype(np.float32)
    raise ValueError(strategy)


def reference_channel_stat(act: torch.Tensor, strategy: str) -> np.ndarray:
    """The reference's own expression (smt_helper.py:167-184) on the host CPU: the exact fp32 values
    it ranks, for the keys whose order the GPU estimate cannot decide."""
    a = act.detach()
    if a.device.type != "cpu":
        a = a.cpu()
    a = torch.sum(a.to(torch.float32).abs(), dim=0)
    if strategy == "mean_abs":
        s = torch.mean(a.abs(), dim=0)
    elif strategy == "abs_mean":
        s = torch.abs(torch.mean(a, dim=0))
    elif strategy == "L1":
        s = torch.norm(a, p=1, dim=0)
    elif strategy == "L2":
        s = torch.norm(a, p=2, dim=0)
    else:
        raise ValueError(strategy)
    return s.numpy().reshape(-1)


# Whether ATen's value of a channel equals its value computed over just the channel's aligned
# 256-channel window of the [B, S, in] state: checked against the whole key once per (strategy, state
# shape, host thread count) and process (as _ROW_SLICE_OK for blocks). On this host ATen's outer reductions agree on windows of >= 32
# aligned channels and differ on arbitrary column subsets, so a window, never a gather, is re-scored.
_CHANNEL_WINDOW = 256
_CHANNEL_WINDOW_OK: Dict[tuple, bool] = {}


def channel_rescorer(src: torch.Tensor, strategy: str):
    """``rescore(flat)`` for the channel keys: the reference's values (reference_channel_stat) of the
    aligned 256-channel windows holding the requested channels, 1/(in/256) of the key's bytes to copy
    and reduce each; the whole key when a window is partial, when more than a quarter of the key's
    windows are asked for, from the third call on one key, or when the window check failed."""
    C = src.shape[2]
    W = _CHANNEL_WINDOW

    def window(w):
        return reference_channel_stat(src[:, :, w * W:(w + 1) * W].contiguous(), strategy)

    calls = [0]

    def rescore(flat):
        wins = np.unique(np.asarray(flat, dtype=np.int64) // W)
        calls[0] += 1
        # a partial last window, or a key the ranking keeps coming back to (the order of its selected
        # channels is a chain of close values): the whole key at once, in one copy
        if (C % W and int(wins[-1]) == C // W) or calls[0] > 2 or 4 * wins.size > -(-C // W):
            return np.arange(C), reference_channel_stat(src, strategy)
        key = (strategy, tuple(src.shape), torch.get_num_threads())
        ok = _CHANNEL_WINDOW_OK.get(key)
        if ok is None:
            full = reference_channel_stat(src, strategy)
            w0 = int(wins[0])
            ok = _CHANNEL_WINDOW_OK[key] = bool(np.array_equal(window(w0), full[w0 * W:(w0 + 1) * W]))
            if not ok:
                return np.arange(C), full
        if not ok:
            return np.arange(C), reference_channel_stat(src, strategy)
        covered, vals = [], []
        for w in wins:
            w = int(w)
            covered.append(np.arange(w * W, (w + 1) * W))
            vals.append(window(w))
        return np.concatenate(covered), np.concatenate(vals)
    return rescore


# Whether smt_channel_mean_aten (ATen's CPU summation order replayed on the GPU) reproduces the
# reference expression on this host, per accumulator shape: checked once per shape and process
# against reference_channel_stat on the host; a mismatch falls back to the interval ranking.
_ATEN_MEAN_OK: Dict[tuple, bool] = {}
ATEN_MEAN_REPORT: dict = {"exact_keys": 0, "checked_shapes": [], "fallback_shapes": []}


def _exact_channel_means(dev_acc: torch.Tensor, src, C: int, strategy: str) -> Optional[np.ndarray]:
    """The reference's fp32 mean_abs / abs_mean values of one key, computed on the GPU in ATen's
    order, or None when that does not hold on this host for the shape (or for L1 / L2)."""
    if strategy not in ("mean_abs", "abs_mean"):
        return None
    shape = (tuple(dev_acc.shape), torch.get_num_threads())
    ok = _ATEN_MEAN_OK.get(shape)
    if ok is False:
        return None
    vals = _hip.channel_mean_aten(dev_acc).cpu().numpy()[:C]
    if ok is None:
        ref = reference_channel_stat(src, strategy)
        ok = _ATEN_MEAN_OK[shape] = bool(np.array_equal(vals, ref))
        ATEN_MEAN_REPORT["checked_shapes" if ok else "fallback_shapes"].append(shape)
        if not ok:
            return None
    ATEN_MEAN_REPORT["exact_keys"] += 1
    return vals


def score_channel_entries(activation: Dict[Hashable, object], calculate_strategy: str = "mean_abs") -> List[ranking.KeyScores]:
    """smt_helper.py:167-184 on the GPU: per key, the channel statistics as :class:`ranking.KeyScores`.
    mean_abs / abs_mean (the harvested |x| sums are non-negative: the same values) come out exact,
    in ATen's own summation order (smt_channel_mean_aten, checked on the host once per shape); L1 / L2
    (and a shape whose check failed) as fp64 sums with intervals and the window re-score.
    Keys with an unknown strategy are skipped as in the reference (no branch assigns them)."""
    if calculate_strategy not in _STRATEGY:
        return []
    entries = []
    for key, act in activation.items():
        dev_acc, src = _channel_sources(act)
        B, S, C = src.shape
        exact = _exact_channel_means(dev_acc, src, C, calculate_strategy)
        if exact is not None:
            e64 = exact.astype(np.float64)
            entries.append(ranking.KeyScores(key, (C,), exact, e64, e64.copy(),
                                             rescore=channel_rescorer(src, calculate_strategy)))
            continue
        raw = _hip.channel_scores(dev_acc, _STRATEGY[calculate_strategy]).cpu().numpy()[:C]
        nominal, lo, hi = ranking.channel_intervals(raw, B, S, calculate_strategy)
        entries.append(ranking.KeyScores(
            key, (C,), nominal, lo, hi,
            rescore=channel_rescorer(src, calculate_strategy),
            bounds=lambda worst, raw=raw, B=B, S=S: ranking.channel_intervals(raw, B, S, calculate_strategy,
                                                                               worst)[1:]))
    return entries


def score_channels(activation: Dict[Hashable, object], calculate_strategy: str = "mean_abs") -> Dict[Hashable, np.ndarray]:
    """Per key, the nominal fp32 per-channel statistic (GPU, fp64 rounded once)."""
    return {e.key: e.nominal for e in score_channel_entries(activation, calculate_strategy)}


def _rank_channel_entries(entries: List[ranking.KeyScores], n: int, selection_strategy: str) -> defaultdict:
    if not entries:
        raise UnboundLocalError("cannot access local variable 'value' where it is not associated with a value "
                                "(no candidate channels: empty activations or unknown calculate_strategy)")
    if selection_strategy == "norm_dist":
        ranked = defaultdict(list)
        for e, flats in zip(entries, ranking.top_n_per_key(entries, n)):
            ranked[e.key] = [int(f) for f in flats]        # smt_helper.py:195-197 assigns every key
        return ranked
    if n <= 0:
        raise UnboundLocalError("cannot access local variable 'value' where it is not associated with a value "
                                "(n <= 0 selects no channel)")
    return ranking.group(entries, ranking.top_n(entries, n), lambda e, f: int(f))


def rank_channels(column_means: Dict[Hashable, np.ndarray], n: int,
                  selection_strategy: str = "no_restriction") -> defaultdict:
    """smt_helper.py:186-230 on given exact fp32 channel statistics (host logic). ``no_restriction``:
    the first ``n`` of all ``(score, (key, idx))`` tuples in descending order, grouped per key in that
    order; ``norm_dist``: the ``n`` best channels of every key."""
    return _rank_channel_entries(_exact_entries(column_means), n, selection_strategy)


def select_channel_based_on_activation(activation, n=660, selection_strategy="no_restriction",
                                       calculate_strategy="mean_abs", model="yahma/llama-13b-hf"):
    """smt_helper.py:149-230. ``activation``: ``{(module_name, layer): act}`` where ``act`` is the
    reference's fp32 ``[B, S, in]`` tensor of accumulated ``|x|`` (any device) or a
    :class:`ChannelActivation` from :class:`sparse_matrix_tuning_amd.trainer.ActivationHarvester`.
    Returns ``defaultdict(list)`` ``{key: [channel, ...]}`` with each list in descending tuple order
    (the row order of LinearLayer_ChannelSparsity), identical to the reference's."""
    return _rank_channel_entries(score_channel_entries(activation, calculate_strategy), n, selection_strategy)


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

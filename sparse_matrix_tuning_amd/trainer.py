"""The hot segments of ``deepspeed/fine_tune.py`` as reusable host code.

``fine_tune.py`` itself is not imported (it needs DeepSpeed, a hub download and datasets); these
functions restate the parts of it that sit on the SMT path so the bench, the smoke test and the
GPU parity tests drive the exact same sequence:

* :func:`get_targeted_module_dims`      fine_tune.py:217-229
* :func:`count_total_blocks`            fine_tune.py:231-234
* :func:`block_budgets`                 fine_tune.py:236-241
* :class:`GradHarvester`                fine_tune.py:714-767 (fp32 accumulators kept in HBM and
                                        updated by one multi-tensor HIP launch per step instead of a
                                        D2H copy + CPU add per parameter)
* :func:`select_and_convert`            fine_tune.py:257-384
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

from . import _hip
from .engine import SMTFusedAdam, initialize, linear_lr_lambda, safe_get_full_grad
from .smt.smt import (_attn_module_name, _layer_number, _mlp_module_name,
                      convert_linear_layer_to_matrix_sparsity, freeze_unselected_matrix_layer,
                      get_optimizer_sparse_grouped_parameters)
from .smt.smt_helper import select_submatrix_based_on_grads

TARGET_MODULE_NAMES = ('gate_proj', 'up_proj', 'down_proj', 'q_proj', 'k_proj', 'v_proj')


def get_targeted_module_dims(model) -> Dict[str, list]:
    """fine_tune.py:217-229: first-seen ``[out, in]`` per targeted module name."""
    dims: Dict[str, list] = {}
    for name, param in model.named_parameters():
        if 'weight' in name:
            for target in TARGET_MODULE_NAMES:
                if target in name and target not in dims:
                    dims[target] = [param.shape[0], param.shape[1]]
                    break
    return dims


def count_total_blocks(model) -> float:
    """fine_tune.py:231-234: float sum of (rows/256)*(cols/256) over every 2-D parameter."""
    total = 0
    for _name, param in model.named_parameters():
        if isinstance(param, torch.Tensor) and param.ndim == 2:
            total += param.shape[0] / 256 * param.shape[1] / 256
    return total


def block_budgets(num_total_blocks: float, attention_ratio: float, mlp_ratio: float) -> Tuple[int, int]:
    """fine_tune.py:236-241."""
    return int(attention_ratio * num_total_blocks), int(mlp_ratio * num_total_blocks)


class GradHarvester:
    """Warm-up gradient accumulation of fine_tune.py:714-767, kept on the GPU.

    Keys: MLP params match ``'mlp' in name`` (no ``weight`` check) -> ``(gate|up|down_proj, layer)``;
    attention params match ``'self_attn' in name and 'weight' in name`` with module in {q,k,v}
    (o_proj excluded, fine_tune.py:746-747). The first contribution to a key assigns, later ones
    add, in ``named_parameters()`` order; contributions that share a key within one step (e.g. the
    OPT naming where the layer regex never matches) go to successive launches so the fp32 adds
    happen in the reference's order.
    """

    def __init__(self, model, num_mlp_blocks: int, num_attention_blocks: int):
        self.model = model
        self.warmup_grads: Dict[tuple, torch.Tensor] = {}
        self.attention_warmup_grads: Dict[tuple, torch.Tensor] = {}
        self.targets: List[tuple] = []      # (param, dict, key)
        for name, param in model.named_parameters():
            layer = _layer_number(name)
            if 'mlp' in name and num_mlp_blocks > 0:
                self.targets.append((param, self.warmup_grads, (_mlp_module_name(name), layer)))
            if 'self_attn' in name and 'weight' in name and num_attention_blocks > 0:
                mod = ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
                       'v_proj' if 'v_proj' in name else None)
                if mod is not None:
                    self.targets.append((param, self.attention_warmup_grads, (mod, layer)))
        self.steps = 0

    @torch.no_grad()
    def harvest(self) -> None:
        rounds: List[List[tuple]] = []      # launch r holds the r-th contribution of each key
        seen = defaultdict(int)
        assign_rounds: List[List[tuple]] = []
        for param, store, key in self.targets:
            grad = safe_get_full_grad(param)
            if grad is None:
                continue
            grad = grad.detach()
            if not grad.is_contiguous():
                grad = grad.contiguous()
            dk = (id(store), key)
            r = seen[dk]
            seen[dk] += 1
            if key not in store:
                store[key] = torch.empty(grad.shape, dtype=torch.float32, device=grad.device)
                while len(assign_rounds) <= r:
                    assign_rounds.append([])
                assign_rounds[r].append((store[key], grad))
            else:
                while len(rounds) <= r:
                    rounds.append([])
                rounds[r].append((store[key], grad))
        n = max(len(rounds), len(assign_rounds))
        for r in range(n):
            if r < len(assign_rounds) and assign_rounds[r]:
                _hip.grad_accumulate(assign_rounds[r], assign=True)
            if r < len(rounds) and rounds[r]:
                _hip.grad_accumulate(rounds[r], assign=False)
        self.steps += 1

    def release(self) -> None:
        self.warmup_grads = {}
        self.attention_warmup_grads = {}


def select_and_convert(engine, harvester: GradHarvester, targeted_module_dims: dict,
                       num_attention_blocks: int, num_mlp_blocks: int, *, selection_strategy="no_restriction",
                       calculate_strategy="mean_abs", no_limit_mixture=False, w_decay=0.0, smt_lr=9.865e-6,
                       ft_learning_rate=None, smt_lr_warmup_steps=0, num_training_steps=1000,
                       ds_config: Optional[dict] = None, broadcast_selection: bool = True):
    """fine_tune.py:257-384. Returns ``(engine, optimizer, lr_scheduler, selected_mlp, selected_att)``.

    The attention pool is scored with the default ``mean_abs`` (fine_tune.py:306-313 does not pass
    ``calculate_strategy``); the MLP pool uses ``calculate_strategy``. With ``broadcast_selection``
    rank 0's selection is broadcast (the reference relies on every rank computing the same one)."""
    model = engine.module
    selected_att: dict = {}
    selected_mlp: dict = {}
    if no_limit_mixture:
        selected_mlp = select_submatrix_based_on_grads(
            harvester.warmup_grads, targeted_module_dims, num_mlp_blocks + num_attention_blocks,
            selection_strategy=selection_strategy, calculate_strategy=calculate_strategy)
        selected_mlp = _broadcast(selected_mlp, broadcast_selection)
        model = freeze_unselected_matrix_layer(model, selected_mlp, {}, mixture=True)
    else:
        if num_attention_blocks > 0:
            selected_att = select_submatrix_based_on_grads(
                harvester.attention_warmup_grads, targeted_module_dims, num_attention_blocks,
                selection_strategy=selection_strategy)
            selected_att = _broadcast(selected_att, broadcast_selection)
        if num_mlp_blocks > 0:
            selected_mlp = select_submatrix_based_on_grads(
                harvester.warmup_grads, targeted_module_dims, num_mlp_blocks,
                selection_strategy=selection_strategy, calculate_strategy=calculate_strategy)
            selected_mlp = _broadcast(selected_mlp, broadcast_selection)
        model = freeze_unselected_matrix_layer(model, selected_mlp, selected_att)
    engine.release()
    harvester.release()
    model = convert_linear_layer_to_matrix_sparsity(model, selected_mlp, selected_att)
    if hasattr(model, "enable_input_require_grads"):     # make_model_gradient_checkpointing_compatible
        model.enable_input_require_grads()
    groups = get_optimizer_sparse_grouped_parameters(model, w_decay, smt_lr)
    if not groups:
        raise RuntimeError("SMT selection produced no trainable tile (block budgets "
                           f"attention={num_attention_blocks}, mlp={num_mlp_blocks})")
    opt = SMTFusedAdam(groups, lr=ft_learning_rate if ft_learning_rate is not None else smt_lr, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(smt_lr_warmup_steps, num_training_steps))
    torch.cuda.empty_cache()
    new_engine, opt, _, sched = initialize(model=model, optimizer=opt, config=ds_config or {"gradient_clipping": 1.0},
                                           lr_scheduler=sched)
    return new_engine, opt, sched, selected_mlp, selected_att


def _broadcast(selection, enabled: bool):
    import torch.distributed as dist
    if not enabled or not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return selection
    obj = [dict(selection) if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    out = defaultdict(list)
    for k, v in obj[0].items():
        out[k] = list(v)
    return out

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
* :class:`ActivationHarvester`          fine_tune.py:584-709 (channel path: |x| of every targeted
                                        linear's input summed over steps in fp32 HBM accumulators
                                        by one HIP launch per hook; ranks summed in bf16 per hook
                                        and step as the reference does)
* :func:`select_and_convert_channels`   fine_tune.py:406-575
"""
from __future__ import annotations

from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

from . import _hip
from .engine import SMTFusedAdam, initialize, linear_lr_lambda, safe_get_full_grad
from .smt.smt import (_attn_module_name, _layer_number, _mlp_module_name,
                      convert_linear_layer_to_channel_sparsity, convert_linear_layer_to_matrix_sparsity,
                      freeze_unselected_channel_layer, freeze_unselected_matrix_layer,
                      get_optimizer_sparse_grouped_parameters)
from .smt.smt_helper import (ChannelActivation, get_named_linears, select_channel_based_on_activation,
                             select_submatrix_based_on_grads)

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
        """Free the accumulators (the dicts are cleared in place: ``targets`` refers to them)."""
        self.warmup_grads.clear()
        self.attention_warmup_grads.clear()
        self.targets = []


def uses_reentrant_checkpointing(model) -> bool:
    """True when some module runs transformers' gradient checkpointing with the REENTRANT
    ``torch.utils.checkpoint`` (the only variant that needs a grad-requiring input)."""
    for m in model.modules():
        if getattr(m, "gradient_checkpointing", False):
            fn = getattr(m, "_gradient_checkpointing_func", None)
            if (getattr(fn, "keywords", None) or {}).get("use_reentrant", True):
                return True
    return False


def make_gradient_checkpointing_compatible(model) -> bool:
    """fine_tune.py:345 -> deepspeed_helpers.py:151-161: make the embedding output require grad so
    that reentrant activation checkpointing sees a grad-requiring input. Done only when the model
    actually checkpoints reentrantly: otherwise the hook makes autograd run the data-gradient chain
    through every layer down to the (frozen) embeddings, where without it the backward stops at the
    lowest module that holds a trainable tile. Returns whether the hook was installed."""
    if hasattr(model, "enable_input_require_grads") and uses_reentrant_checkpointing(model):
        model.enable_input_require_grads()
        return True
    return False


def checkpointed_layers(model) -> List[torch.nn.Module]:
    """The modules transformers' gradient checkpointing wraps (the decoder layers), in order."""
    try:
        from transformers.modeling_layers import GradientCheckpointingLayer
    except ImportError:                       # older transformers: no per-layer switch
        return []
    return [m for m in model.modules() if isinstance(m, GradientCheckpointingLayer)
            and hasattr(m, "_gradient_checkpointing_func")]


def set_resident_layers(model, n_resident: int) -> int:
    """MI355X memory policy for a model under per-layer recompute (fine_tune.py:192): keep the
    activations of the LAST ``n_resident`` checkpointed layers resident (no recompute), recompute
    the others. The reference recomputes every layer to fit its GPUs; with 288 GB of HBM the full
    fine-tuning warm-up has room for most layers' activations beside the fp32 optimizer state.
    Returns the number of layers left resident. Numerics are those of full recompute (the
    recomputed forward is the same code on the same inputs)."""
    layers = checkpointed_layers(model)
    n = max(0, min(int(n_resident), len(layers)))
    for i, m in enumerate(layers):
        m.gradient_checkpointing = i < len(layers) - n
    return n


@torch.no_grad()
def _rope_for(model, x: torch.Tensor):
    rot = getattr(getattr(model, "model", model), "rotary_emb", None)
    if rot is None:
        return None
    pos = torch.arange(x.shape[1], device=x.device).unsqueeze(0).expand(x.shape[0], -1)
    return rot(x, pos)


def layer_activation_bytes(model, batch: int, seq: int) -> int:
    """HBM one decoder layer's saved activations take beyond its input (which recompute keeps
    anyway) at ``batch`` x ``seq`` tokens, measured: one forward of the first checkpointed layer on a
    random input with autograd recording (its weights' gradient state as it is), then freed."""
    layers = checkpointed_layers(model)
    if not layers:
        return 0
    layer = layers[0]
    p = next(layer.parameters())
    hidden = getattr(getattr(model, "config", None), "hidden_size", None) or p.shape[-1]
    x = torch.randn(batch, seq, hidden, device=p.device, dtype=p.dtype, requires_grad=True)
    pe = _rope_for(model, x)
    was = layer.gradient_checkpointing
    layer.gradient_checkpointing = False
    torch.cuda.synchronize(p.device)
    m0 = torch.cuda.memory_allocated(p.device)
    try:
        with torch.enable_grad():
            out = layer(x, position_embeddings=pe)
            out = out[0] if isinstance(out, tuple) else out
            torch.cuda.synchronize(p.device)
            used = torch.cuda.memory_allocated(p.device) - m0 - out.numel() * out.element_size()
        del out
    finally:
        layer.gradient_checkpointing = was
    del x
    return max(0, int(used))


def resident_layers_for(model, batch: int, seq: int, peak_bytes: int, reserve_frac: float = 0.25) -> int:
    """How many checkpointed layers can keep their activations resident: the HBM left above
    ``peak_bytes`` (a step's peak with every layer recomputed) minus ``reserve_frac`` of the device
    for allocator fragmentation and backward transients, over :func:`layer_activation_bytes`. (At
    the LLaMA-3-8B warm-up, B 16 x S 2048: 3.7 GB per layer; a 12 % reserve put the step's peak at
    280 GB of 309, hence 25 %.)"""
    layers = checkpointed_layers(model)
    if not layers:
        return 0
    dev = next(layers[0].parameters()).device
    total = torch.cuda.get_device_properties(dev).total_memory
    per = layer_activation_bytes(model, batch, seq)
    room = total * (1.0 - reserve_frac) - peak_bytes
    if per <= 0 or room <= 0:
        return 0
    return min(len(layers), int(room // per))


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
    # fine_tune.py:336-337 converts without ``mixture`` in both branches
    new_engine, opt, sched = _convert_and_initialize(model, selected_mlp, selected_att, False, w_decay,
                                                     smt_lr, ft_learning_rate, smt_lr_warmup_steps,
                                                     num_training_steps, ds_config)
    return new_engine, opt, sched, selected_mlp, selected_att


def _convert_and_initialize(model, selected_mlp, selected_att, mixture, w_decay, smt_lr, ft_learning_rate,
                            smt_lr_warmup_steps, num_training_steps, ds_config):
    """fine_tune.py:339-384: convert the frozen model's selected linears, rebuild the optimizer
    groups, scheduler and engine."""
    model = convert_linear_layer_to_matrix_sparsity(model, selected_mlp, selected_att, mixture=mixture)
    make_gradient_checkpointing_compatible(model)
    groups = get_optimizer_sparse_grouped_parameters(model, w_decay, smt_lr)
    if not groups:
        raise RuntimeError("SMT selection produced no trainable tile (selected "
                           f"attention={sum(map(len, selected_att.values()))}, mlp={sum(map(len, selected_mlp.values()))})")
    opt = SMTFusedAdam(groups, lr=ft_learning_rate if ft_learning_rate is not None else smt_lr, betas=(0.9, 0.95))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(smt_lr_warmup_steps, num_training_steps))
    torch.cuda.empty_cache()
    new_engine, opt, _, sched = initialize(model=model, optimizer=opt, config=ds_config or {"gradient_clipping": 1.0},
                                           lr_scheduler=sched)
    return new_engine, opt, sched


def reselect(engine, selected_mlp, selected_att, *, w_decay=0.0, smt_lr=9.865e-6, ft_learning_rate=None,
             smt_lr_warmup_steps=0, num_training_steps=1000, ds_config: Optional[dict] = None):
    """Swap an SMT engine's model over to another tile selection: merge every module's tiles back into
    its W (convert_matrix_sparsity_to_linear_layer, smt.py:416-457), drop the engine's packed state and
    weight copies, freeze / convert / initialise for the new selection (fine_tune.py:264-384). Used by
    the bench to time a second selection of the same model. Returns ``(engine, optimizer, scheduler)``."""
    from .engine import detach_transposed_weights
    from .smt.smt import convert_matrix_sparsity_to_linear_layer
    model = engine.module
    engine.release()
    detach_transposed_weights(model)
    convert_matrix_sparsity_to_linear_layer(model)
    model = freeze_unselected_matrix_layer(model, selected_mlp, selected_att)
    return _convert_and_initialize(model, selected_mlp, selected_att, False, w_decay, smt_lr, ft_learning_rate,
                                   smt_lr_warmup_steps, num_training_steps, ds_config)


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


# ------------------------------------------------------------------------------------------------
# channel path
# ------------------------------------------------------------------------------------------------
class ActivationHarvester:
    """Activation collection of fine_tune.py:584-709, kept on the GPU.

    The reference walks ``model.model.layers`` one by one under ``no_grad`` (a Catcher grabs layer
    0's input), with a forward hook on every ``nn.Linear`` of the layer that takes ``|x|``,
    all-reduces it over ranks, copies it to the CPU in fp32 and adds it to ``activation[(m, i)]``
    (MLP: gate/up/down_proj when ``num_mlp_channel > 0``) or ``attention_activation[(m, i)]``
    (q/k/v_proj when ``num_attention_channel > 0``; o_proj is skipped). The layer index ``i`` is the
    position in ``model.model.layers``.

    Here the hooks stay registered on those linears and one ordinary ``no_grad`` forward of the
    model feeds them the same inputs. Each hook is one ``smt_act_accumulate`` launch that keeps the
    reference's own state, the fp32 ``[B, S, in]`` sum of ``|x|`` over steps, in HBM (bit for bit the
    CPU ``+=``). Linears that read the same input tensor in one forward (q/k/v, gate/up) share one
    accumulator instead of holding identical copies.

    Ranks (``rank_reduction``): ``"reference"`` (default) does what fine_tune.py:651-665 does on
    every hook of every step: ``|x|`` in bf16, summed over ranks in bf16 by one all-reduce, then
    added in fp32 -- so the accumulators, and the selection, are the reference's at any world size
    (one all-reduce per distinct input: the reference's q/k/v hooks each all-reduce the same
    ``|x|`` and get the same sum). ``"fp32_once"`` sums the fp32 accumulators once, in
    :meth:`finalize` (one collective instead of one per input per step; it rounds differently from
    the reference at world size > 1). At world size 1 both are the identity."""

    RANK_REDUCTIONS = ("reference", "fp32_once")

    def __init__(self, model, num_mlp_channel: int, num_attention_channel: int, rank_reduction: str = "reference"):
        if rank_reduction not in self.RANK_REDUCTIONS:
            raise ValueError(f"rank_reduction {rank_reduction!r}: one of {self.RANK_REDUCTIONS}")
        import torch.distributed as dist
        self.model = model
        self.rank_reduction = rank_reduction
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.activation: Dict[tuple, ChannelActivation] = {}
        self.attention_activation: Dict[tuple, ChannelActivation] = {}
        self._handles = []
        self._reduced = False
        self._last = None                   # (input tensor object, accumulator) of the latest hook
        layers = model.model.layers
        for i, layer in enumerate(layers):
            for name, lin in get_named_linears(layer).items():
                store = key = None
                if 'mlp' in name and num_mlp_channel > 0:
                    store, key = self.activation, (_mlp_module_name(name), i)
                if 'self_attn' in name and num_attention_channel > 0:
                    mod = ('q_proj' if 'q_proj' in name else 'k_proj' if 'k_proj' in name else
                           'v_proj' if 'v_proj' in name else None)
                    if mod is not None:
                        store, key = self.attention_activation, (mod, i)
                if store is not None:
                    self._handles.append(lin.register_forward_hook(self._hook(store, key)))

    def _hook(self, store: dict, key: tuple):
        def hook(_module, inputs, _output):
            x_obj = inputs[0]
            last = self._last
            ent = store.get(key)
            if last is not None and last[0] is x_obj and (ent is None or ent is last[1]):
                # same input tensor as the previous linear (q/k/v, gate/up): same accumulator, already
                # updated for this forward
                store[key] = last[1]
                return
            x = x_obj.detach()
            if x.stride(-1) != 1 or x.data_ptr() % 16 or any(st % 8 for st in x.stride()[:-1]):
                x = x.contiguous()
            if ent is None:
                ent = store[key] = ChannelActivation(
                    torch.empty(x.shape, dtype=torch.float32, device=x.device))
            elif tuple(ent.acc.shape) != tuple(x.shape):
                # the reference's `feat_dict[key] += x` needs equal shapes across steps too
                raise RuntimeError(f"activation shape {tuple(x.shape)} differs from earlier steps "
                                   f"({tuple(ent.acc.shape)}) for {key}")
            if self.world > 1 and self.rank_reduction == "reference":
                # fine_tune.py:653-657: x = |x| (bf16), all_reduce (bf16 sum over ranks), then the fp32
                # add; act_accumulate takes |.| of the non-negative sum again, which changes nothing
                import torch.distributed as dist
                x = x.abs()
                dist.all_reduce(x)
            _hip.act_accumulate(x, ent.acc, assign=ent.steps == 0)
            ent.steps += 1
            self._last = (x_obj, ent)
        return hook

    @torch.no_grad()
    def collect(self, batch: dict) -> None:
        """One activation step (fine_tune.py:586-709): eval-mode no-grad forward, back to train."""
        was_training = self.model.training
        self.model.eval()
        try:
            self.model(**batch, use_cache=False)
        finally:
            self._last = None
            self.model.train(was_training)

    def finalize(self) -> None:
        """Sum the accumulators over ranks (the per-hook all-reduce of the reference, done once)."""
        import torch.distributed as dist
        if self._reduced:
            return
        self._reduced = True
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        if self.rank_reduction == "reference":
            return                          # every hook already summed its bf16 |x| over ranks
        seen, accs = set(), []
        for d in (self.activation, self.attention_activation):
            for e in d.values():
                if id(e) not in seen:
                    seen.add(id(e))
                    accs.append(e.acc)
        if not accs:
            return
        flat = torch.cat([a.reshape(-1) for a in accs])
        dist.all_reduce(flat)
        off = 0
        for a in accs:
            a.copy_(flat[off:off + a.numel()].view_as(a))
            off += a.numel()

    def remove(self) -> None:
        for h in self._handles:
            h.remove()
        self._handles = []

    def release(self) -> None:
        self.remove()
        self.activation = {}
        self.attention_activation = {}
        self._last = None


def select_and_convert_channels(model, harvester: ActivationHarvester, num_attention_channel: int,
                                num_mlp_channel: int, *, selection_strategy="no_restriction",
                                calculate_strategy="mean_abs", no_limit_mixture=False, w_decay=0.0,
                                smt_lr=9.865e-6, ft_learning_rate=None, smt_lr_warmup_steps=0,
                                num_training_steps=1000, ds_config: Optional[dict] = None,
                                broadcast_selection: bool = True):
    """fine_tune.py:406-575 (channel path). Returns ``(engine, optimizer, lr_scheduler,
    selected_channel, selected_channel_attention)``.

    As in the reference: with ``no_limit_mixture`` the channels come from the MLP activations only
    with the summed budget; otherwise attention is scored with the default ``mean_abs``
    (fine_tune.py:472-476 does not pass ``calculate_strategy``) and MLP with ``calculate_strategy``;
    the optimizer is FusedAdam at ``ft_learning_rate`` with betas (0.95, 0.999) (fine_tune.py:536-538).
    The selected rows are ordinary dense parameters for the engine (autograd bf16 gradients, fused
    AdamW in flat mode); each forward writes them back into W (smt.py:208-213)."""
    harvester.finalize()
    selected_att: dict = {}
    selected_mlp: dict = {}
    if no_limit_mixture:
        selected_mlp = select_channel_based_on_activation(
            harvester.activation, num_attention_channel + num_mlp_channel,
            selection_strategy=selection_strategy, calculate_strategy=calculate_strategy)
        selected_mlp = _broadcast(selected_mlp, broadcast_selection)
        model = freeze_unselected_channel_layer(model, selected_mlp, {}, mixture=True)
    else:
        if num_attention_channel > 0:
            selected_att = select_channel_based_on_activation(
                harvester.attention_activation, num_attention_channel, selection_strategy=selection_strategy)
        if num_mlp_channel > 0:
            selected_mlp = select_channel_based_on_activation(
                harvester.activation, num_mlp_channel, selection_strategy=selection_strategy,
                calculate_strategy=calculate_strategy)
        # fine_tune.py:506-507 synchronises the attention selection from rank 0 (a file broadcast)
        selected_att = _broadcast(selected_att, broadcast_selection)
        selected_mlp = _broadcast(selected_mlp, broadcast_selection)
        model = freeze_unselected_channel_layer(model, selected_mlp, selected_att)
    harvester.release()
    model = convert_linear_layer_to_channel_sparsity(model, selected_mlp, selected_att)
    make_gradient_checkpointing_compatible(model)
    groups = get_optimizer_sparse_grouped_parameters(model, w_decay, smt_lr)
    if not groups:
        raise RuntimeError("channel selection produced no trainable row (channel budgets "
                           f"attention={num_attention_channel}, mlp={num_mlp_channel})")
    opt = SMTFusedAdam(groups, lr=ft_learning_rate if ft_learning_rate is not None else smt_lr, betas=(0.95, 0.999))
    sched = torch.optim.lr_scheduler.LambdaLR(opt, linear_lr_lambda(smt_lr_warmup_steps, num_training_steps))
    torch.cuda.empty_cache()
    engine, opt, _, sched = initialize(model=model, optimizer=opt, config=ds_config or {"gradient_clipping": 1.0},
                                       lr_scheduler=sched)
    return engine, opt, sched, selected_mlp, selected_att

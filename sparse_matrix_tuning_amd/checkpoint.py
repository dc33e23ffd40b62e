"""SMT checkpoint / resume.

The reference saves only an HF state dict (``deepspeed_helpers.py:341-364``), holding both
``…weight`` and ``…selected_weight``, and cannot resume: the selection and the optimizer state are
lost. Here an SMT checkpoint is what is needed to resume bit-for-bit on top of the
base model:

* ``smt_meta.json``: format tag, per-module ``(name, index_list, weight shape)`` in selection
  order, the optimizer param-group hyper-parameters, step counters, the LR-scheduler state, the fp16
  loss scale's state (the reference's ``--dtype fp16``), and a fingerprint of every frozen parameter (SMT modules' W with their tile blocks masked out);
* ``smt_state.safetensors``: the tiles of every module (in the model's dtype) and, per engine tile group, the fp32
  master / exp_avg / exp_avg_sq (0.8 GB at the LLaMA-3-8B operating point);
* ``smt_frozen.safetensors`` (``include_frozen=True``, the default, as DeepSpeed's
  ``save_checkpoint`` also saves the module): every other weight of the model as it is now. The
  full fine-tuning warm-up (fine_tune.py:160-190) changed all of them before the selection, so a
  freshly loaded base model is NOT what the tiles were trained on. :func:`restore_model` loads them
  when present and, either way, checks every frozen parameter against its fingerprint and raises on
  a mismatch instead of resuming on the wrong weights.

Only rank 0 writes (the tiles and the optimizer state are replicated), each file to a temporary
name first and then renamed; rank 0 then broadcasts whether the save succeeded, so a failed write
raises on every rank instead of leaving the others waiting. Every file carries the save's random id
(safetensors metadata, and ``save_id`` in the meta file written last): a directory overwritten by a
save that crashed half-way, holding files of two saves, is refused on load.

:func:`save_merged_model` writes the plain HF-style state dict with the tiles merged into W and
no ``selected_weight`` keys (``convert_matrix_sparsity_to_linear_layer`` semantics, smt.py:416-457).
Loaders never unpickle: JSON + safetensors only.
"""
from __future__ import annotations

import json
import os
import uuid
from collections import defaultdict
from typing import Dict, Optional, Tuple

import torch
from safetensors import safe_open
from safetensors.torch import load_file, save_file

from .smt.smt import (LinearLayer_MatrixSparsity, _attn_module_name, _layer_number, _mlp_module_name,
                      convert_linear_layer_to_matrix_sparsity, freeze_unselected_matrix_layer)

FORMAT = "smt-mi355x-v2"
META = "smt_meta.json"
STATE = "smt_state.safetensors"
FROZEN = "smt_frozen.safetensors"


def _smt_modules(model):
    return [(n, m) for n, m in model.named_modules() if isinstance(m, LinearLayer_MatrixSparsity)]


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


@torch.no_grad()
def fingerprint(t: torch.Tensor, tiles=None) -> str:
    """Order-sensitive integer digest of a tensor's bits (exact, so independent of the reduction
    order): ``sum_i bits[i] * (i mod 1000003 + 1)`` mod 2^64, with the 256x256 ``tiles`` of a 2-D
    weight masked to zero first."""
    t = t.detach()
    if tiles:
        t = t.clone()
        for r, c in tiles:
            t[r * 256:(r + 1) * 256, c * 256:(c + 1) * 256] = 0
    t = t.contiguous()
    itype = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[t.element_size()]
    bits = t.view(itype).reshape(-1).to(torch.int64)
    w = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 1000003 + 1
    digest = int((bits * w).sum().item()) & ((1 << 64) - 1)
    return f"{t.dtype}:{tuple(t.shape)}:{digest:016x}"


def _frozen_fingerprints(model) -> Dict[str, str]:
    """Every parameter except the trainable tiles; SMT modules' W with the tile blocks masked (they
    hold the tiles, restored from the checkpoint)."""
    tiles_of = {id(m.weight): m.index_list for _n, m in _smt_modules(model)}
    out = {}
    for name, p in model.named_parameters():
        if name.endswith("selected_weight"):
            continue
        out[name] = fingerprint(p, tiles_of.get(id(p)))
    return out


def _atomic(path: str, write) -> None:
    tmp = path + ".tmp"
    write(tmp)
    os.replace(tmp, path)


def save_checkpoint(engine, save_dir: str, client_state: Optional[dict] = None, include_frozen: bool = True) -> str:
    """Write selection + tiles + optimizer state of an :class:`SMTEngine` (DeepSpeed
    ``engine.save_checkpoint`` counterpart), and with ``include_frozen`` every frozen weight.
    Returns the directory. Raises on every rank if rank 0's write failed."""
    dist = _dist()
    rank = dist.get_rank() if dist is not None else 0
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    err = None
    if rank == 0:
        try:
            _write_checkpoint(engine, save_dir, client_state, include_frozen)
        except Exception as e:          # reported to every rank below, then re-raised here
            err = e
    if dist is not None:
        msg = [None if err is None else f"{type(err).__name__}: {err}"]
        dist.broadcast_object_list(msg, src=0)
        if err is None and msg[0] is not None:
            raise RuntimeError(f"save_checkpoint failed on rank 0: {msg[0]}")
    if err is not None:
        raise err
    return save_dir


def _write_checkpoint(engine, save_dir: str, client_state: Optional[dict], include_frozen: bool) -> None:
    model = engine.module
    save_id = uuid.uuid4().hex
    os.makedirs(save_dir, exist_ok=True)
    tensors: Dict[str, torch.Tensor] = {}
    modules = []
    for name, m in _smt_modules(model):
        modules.append({"name": name, "index_list": [list(t) for t in m.index_list],
                        "weight_shape": list(m.weight.shape), "trainable": bool(m.selected_weight.requires_grad)})
        tensors[f"tiles/{name}"] = m.selected_weight.detach().contiguous().cpu()
    groups = []
    for gi, tg in enumerate(engine.tile_groups):
        names = [n for n, m in _smt_modules(model) if any(m is x for x in tg.modules)]
        groups.append({"modules": names, "step": tg.step,
                       "hyper": {k: (list(v) if isinstance(v, tuple) else v) for k, v in tg.group.items() if k != "params"}})
        tensors[f"master/{gi}"] = tg.master.cpu()
        tensors[f"exp_avg/{gi}"] = tg.exp_avg.cpu()
        tensors[f"exp_avg_sq/{gi}"] = tg.exp_avg_sq.cpu()
    scaler = getattr(engine, "loss_scaler", None)
    meta = {"format": FORMAT, "modules": modules, "groups": groups, "global_steps": engine.global_steps,
            "micro_steps": engine.micro_steps, "skipped_steps": getattr(engine, "skipped_steps", 0),
            "loss_scaler": scaler.state_dict() if scaler is not None else None,
            "lr_scheduler": engine.lr_scheduler.state_dict() if engine.lr_scheduler is not None else None,
            "client_state": client_state or {}, "frozen_fingerprints": _frozen_fingerprints(model),
            "includes_frozen": bool(include_frozen), "save_id": save_id}
    tag = {"smt_save_id": save_id}
    _atomic(os.path.join(save_dir, STATE), lambda p: save_file(tensors, p, metadata=tag))
    if include_frozen:
        frozen = {n: p.detach().contiguous().cpu() for n, p in model.named_parameters()
                  if not n.endswith("selected_weight")}
        _atomic(os.path.join(save_dir, FROZEN), lambda p: save_file(frozen, p, metadata=tag))

    def write_meta(p):
        with open(p, "w") as f:
            json.dump(meta, f, indent=1, default=_json_default)
    _atomic(os.path.join(save_dir, META), write_meta)          # last: its presence marks a complete save


def _load_checked(path: str, meta: dict) -> Dict[str, torch.Tensor]:
    """load_file, after checking that the file belongs to the save ``meta`` describes."""
    want = meta.get("save_id")
    if want is not None:
        with safe_open(path, framework="pt") as f:
            got = (f.metadata() or {}).get("smt_save_id")
        if got != want:
            raise ValueError(f"{os.path.basename(path)} is from another save ({got}) than {META} ({want}): "
                             "the checkpoint directory was overwritten by an incomplete save")
    return load_file(path)


def _json_default(o):
    if isinstance(o, torch.Tensor):
        return o.tolist()
    raise TypeError(type(o))


def read_selection(load_dir: str) -> Tuple[dict, dict]:
    """``(selected_mlp, selected_attention)`` dicts (the reference's selection format) of a
    checkpoint, keyed like fine_tune.py: ``(module_name, layer)``."""
    with open(os.path.join(load_dir, META)) as f:
        meta = json.load(f)
    if meta.get("format") not in (FORMAT, "smt-mi355x-v1"):
        raise ValueError(f"not an SMT checkpoint: {meta.get('format')}")
    sel_mlp, sel_att = defaultdict(list), defaultdict(list)
    for mod in meta["modules"]:
        name = mod["name"]
        tiles = [tuple(t) for t in mod["index_list"]]
        if "mlp" in name:
            sel_mlp[(_mlp_module_name(name), _layer_number(name))] = tiles
        elif "self_attn" in name:
            sel_att[(_attn_module_name(name), _layer_number(name))] = tiles
    return sel_mlp, sel_att


def restore_model(model, load_dir: str):
    """Re-apply a checkpoint to a model of the same architecture: load the saved frozen weights when
    the checkpoint has them (the post-warm-up weights), freeze -> convert (smt.py:641-745, 83-134),
    load the saved tiles and scatter them into W, then check every frozen parameter against the
    checkpoint's fingerprint. A model whose weights are not the ones the checkpoint was saved from
    (e.g. the pre-warm-up base) raises ``ValueError``. Returns the model."""
    with open(os.path.join(load_dir, META)) as f:
        meta = json.load(f)
    sel_mlp, sel_att = read_selection(load_dir)
    frozen_path = os.path.join(load_dir, FROZEN)
    if meta.get("includes_frozen") and os.path.exists(frozen_path):
        frozen = _load_checked(frozen_path, meta)
        params = dict(model.named_parameters())
        missing = [n for n in frozen if n not in params]
        if missing:
            raise KeyError(f"checkpoint weights not in the model: {missing[:5]}")
        with torch.no_grad():
            for n, t in frozen.items():
                params[n].data.copy_(t.to(params[n].device))
    freeze_unselected_matrix_layer(model, sel_mlp, sel_att)
    convert_linear_layer_to_matrix_sparsity(model, sel_mlp, sel_att)
    state = _load_checked(os.path.join(load_dir, STATE), meta)
    for name, m in _smt_modules(model):
        t = state.get(f"tiles/{name}")
        if t is None:
            raise KeyError(f"checkpoint has no tiles for {name}")
        with torch.no_grad():
            m.selected_weight.data.copy_(t.to(m.selected_weight.device))
        m.sync_weight()
    want = meta.get("frozen_fingerprints") or {}
    got = _frozen_fingerprints(model)
    bad = [n for n, fp in want.items() if got.get(n) != fp]
    if bad:
        raise ValueError(f"{len(bad)} frozen weights differ from the checkpoint's (first: {bad[:3]}): restore "
                         "onto the model the checkpoint was saved from (after the full fine-tuning warm-up), or "
                         "save with include_frozen=True")
    return model


def load_optimizer_state(engine, load_dir: str) -> dict:
    """Load tile-group optimizer state and counters into an engine built on a restored model
    (same param-group order as at save time). Returns the saved ``client_state``."""
    with open(os.path.join(load_dir, META)) as f:
        meta = json.load(f)
    state = _load_checked(os.path.join(load_dir, STATE), meta)
    if len(meta["groups"]) != len(engine.tile_groups):
        raise ValueError(f"checkpoint has {len(meta['groups'])} tile groups, engine {len(engine.tile_groups)}")
    for gi, (g, tg) in enumerate(zip(meta["groups"], engine.tile_groups)):
        for key, dst in (("master", tg.master), ("exp_avg", tg.exp_avg), ("exp_avg_sq", tg.exp_avg_sq)):
            src = state[f"{key}/{gi}"]
            if src.numel() != dst.numel():
                raise ValueError(f"{key}/{gi}: {src.numel()} elements, engine has {dst.numel()}")
            dst.copy_(src.to(dst.device))
        tg.step = int(g["step"])
        for k, v in g["hyper"].items():       # current lr (set by the scheduler), betas, eps, decay
            tg.group[k] = tuple(v) if isinstance(v, list) else v
    engine.global_steps = int(meta["global_steps"])
    engine.micro_steps = int(meta["micro_steps"])
    engine.skipped_steps = int(meta.get("skipped_steps", 0))
    saved_scaler = meta.get("loss_scaler")
    scaler = getattr(engine, "loss_scaler", None)
    if (saved_scaler is None) != (scaler is None):
        raise ValueError("the checkpoint was saved " + ("with" if saved_scaler is not None else "without")
                         + " an fp16 loss scale and this engine runs " + ("with" if scaler is not None else "without")
                         + " one: resume with the same \"fp16\" config")
    if scaler is not None:
        scaler.load_state_dict(saved_scaler)     # the dynamic scale's schedule continues where it stopped
    if engine.lr_scheduler is not None and meta.get("lr_scheduler") is not None:
        engine.lr_scheduler.load_state_dict(meta["lr_scheduler"])
    return meta.get("client_state", {})


def save_merged_model(model, path: str) -> None:
    """HF-style state dict (safetensors) with every SMT module's tiles merged into its W and no
    ``selected_weight`` entries."""
    sd = {}
    for name, m in _smt_modules(model):
        m.sync_weight()
    torch.cuda.synchronize()
    for k, v in model.state_dict().items():
        if k.endswith("selected_weight"):
            continue
        sd[k] = v.detach().contiguous().cpu()
    save_file(sd, path)

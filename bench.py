#!/usr/bin/env python3
"""SMT-phase training throughput of LLaMA-3-8B SMT(0.71%) on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU (RCCL over xGMI for N > 1, weak scaling: B=16 x S=2048 per GPU). Per rank:

1. LLaMA-3-8B architecture (HF ``LlamaForCausalLM``), random init (seed 1234), bf16, synthetic
   uniform token batches, labels = input ids. Gradient checkpointing (fine_tune.py:192) is on for
   the full-FT warm-up; in the SMT phase the activations stay resident in HBM (its peak is then
   still below the warm-up's), and a short second measurement with checkpointing on (the
   reference's memory policy) is reported under ``grad_ckpt_mode``.
2. Warm-up: ``--full-ft-steps`` full fine-tuning steps through the engine (fp32-master AdamW over
   all 8.03 B params) with the gradient harvest of fine_tune.py:714-767 in HBM.
3. Selection + conversion (fine_tune.py:257-384): 436 attention + 436 MLP tiles of 256x256
   (ratios 0.00356, = 57.1 M trainable params = 0.71 %), MLP scored ``abs_mean``, attention
   ``mean_abs``.
4. SMT phase: W untimed steps, then K timed steps (forward + engine.backward + engine.step),
   bracketed by barrier + synchronize; the max over ranks is reported.

Rank 0 prints ONE JSON line. ``roofline`` is for the dominant hand-written kernel (the grouped
tile-wgrad, smt_tile_wgrad = wgrad_dma + wgrad_reduce), timed with HIP events on its launch
stream over the timed region. ``cpu_baseline`` times the oracle's restatement of the reference path
(oracle/smt_oracle.py) on this host's cores.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "train tokens/sec + peak GB HBM, LLaMA-3-8B SMT(0.71%) at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0          # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0              # MI355X HBM3E spec (MI355X_MICROARCH.md)
F_ALG_GFLOP_PER_TOKEN = 31.744     # fwd 15.009 + dgrad 15.009 + wgrad 0.114 + attn 1.611

MODELS = {
    "llama3-8b": dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                      num_attention_heads=32, num_key_value_heads=8, rope_theta=500000.0, rms_norm_eps=1e-5,
                      max_position_embeddings=8192, tie_word_embeddings=False, initializer_range=0.02),
    # small config for smoke runs (dims multiples of 256)
    "mini": dict(vocab_size=4096, hidden_size=512, intermediate_size=1536, num_hidden_layers=4,
                 num_attention_heads=4, num_key_value_heads=2, rope_theta=500000.0, rms_norm_eps=1e-5,
                 max_position_embeddings=4096, tie_word_embeddings=False, initializer_range=0.02),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=16, help="per-GPU micro batch (deepspeed/README.md:39)")
    ap.add_argument("--seq", type=int, default=2048)
    ap.add_argument("--full-ft-steps", type=int, default=2)
    ap.add_argument("--att-ratio", type=float, default=None, help="default 0.00356 (8B), 0.03 (mini)")
    ap.add_argument("--mlp-ratio", type=float, default=None, help="default 0.00356 (8B), 0.03 (mini)")
    ap.add_argument("--calculate-strategy", default="abs_mean")
    ap.add_argument("--smt-lr", type=float, default=9.865e-6)
    ap.add_argument("--grad-ckpt", action="store_true",
                    help="recompute each decoder layer in the SMT phase's backward (the reference's "
                         "fine_tune.py:192 memory policy) for the timed steps; default: activations stay "
                         "resident in HBM (the SMT phase then peaks below the warm-up phase)")
    ap.add_argument("--no-grad-ckpt", action="store_true", help=argparse.SUPPRESS)   # the default now
    ap.add_argument("--ref-mode-steps", type=int, default=4,
                    help="after the timed steps, also time this many steps with gradient checkpointing "
                         "(reported under 'grad_ckpt_mode'; 0 disables)")
    ap.add_argument("--sdpa-attention", action="store_true",
                    help="keep transformers' sdpa (aotriton) attention instead of the gfx950 flash attention")
    ap.add_argument("--eager-ops", action="store_true",
                    help="keep transformers' eager RMSNorm/RoPE/SwiGLU instead of the fused HIP kernels")
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE config 5 (DeepSeek-R1-Distill-LLaMA-8B = the LLaMA-3-8B architecture, "
                         "SMT(0.86%%)): the decoder layers' frozen linears run as rowwise-scaled e4m3 GEMMs")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0, help="0 disables the CPU leg")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (functional tests)")
    args = ap.parse_args()
    default_ratio = (0.0043 if args.fp8 else 0.00356) if args.model == "llama3-8b" else 0.03
    args.att_ratio = default_ratio if args.att_ratio is None else args.att_ratio
    args.mlp_ratio = default_ratio if args.mlp_ratio is None else args.mlp_ratio
    return args


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


class WgradTimer:
    """HIP events around every smt_tile_wgrad call (on the stream it is launched on)."""

    def __init__(self):
        self.enabled = False
        self.records = []      # (start, end, algorithmic bytes, flops)

    def hook(self, T, n_tiles, out_bytes, stream_fn):
        if not self.enabled:
            return stream_fn()
        s = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = stream_fn()
        e1.record(s)
        self.records.append((e0, e1, n_tiles * (T * 256 * 2 * 2 + 65536 * out_bytes), 2.0 * T * 65536 * n_tiles))
        return r

    def summary(self):
        if not self.records:
            return None
        torch.cuda.synchronize()
        t = sum(a.elapsed_time(b) for a, b, _, _ in self.records) * 1e-3
        by = sum(r[2] for r in self.records)
        fl = sum(r[3] for r in self.records)
        return dict(launches=len(self.records), seconds=t, bytes=by, flops=fl)


def install_wgrad_timer(timer: WgradTimer):
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.tile_wgrad

    def timed(g2, x2, rc, out, accumulate=False, order=None):
        return timer.hook(g2.shape[0], rc.shape[0], out.element_size(),
                          lambda: orig(g2, x2, rc, out, accumulate=accumulate, order=order))
    _hip.tile_wgrad = timed


class AttnTimer:
    """HIP events around every smt_flash forward / backward launch (current stream), with the causal
    attention FLOPs each one does: forward 2 GEMM-equivalents (QK^T, PV) over the causal half,
    backward 5 (S and dP recomputed, dV, dK, dQ) plus the 2 recomputed ones of the separate dQ
    kernel (S, dP): 7 in this implementation, 5 algorithmic."""

    def __init__(self):
        self.enabled = False
        self.records = []      # (start, end, algorithmic flops)

    def wrap(self, fn, flops_fn):
        def timed(*a, **k):
            if not self.enabled:
                return fn(*a, **k)
            fl = flops_fn(*a)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = fn(*a, **k)
            e1.record(s)
            self.records.append((e0, e1, fl))
            return r
        return timed

    def summary(self):
        if not self.records:
            return None
        torch.cuda.synchronize()
        t = sum(a.elapsed_time(b) for a, b, _ in self.records) * 1e-3
        return dict(launches=len(self.records), seconds=t, flops=sum(r[2] for r in self.records))


def install_attn_timer(timer: AttnTimer):
    from sparse_matrix_tuning_amd import fused_llama as fl
    fn_cls = fl.FlashAttnFn

    def unit(q):                  # one causal QK^T-sized GEMM: 2 * B * Hq * S^2 / 2 * D
        B, Hq, S, D = q.shape
        return 2.0 * B * Hq * S * S / 2 * D

    fwd, bwd = fn_cls.forward, fn_cls.backward
    fn_cls.forward = staticmethod(timer.wrap(fwd, lambda ctx, q, *r: 2 * unit(q)))
    fn_cls.backward = staticmethod(timer.wrap(bwd, lambda ctx, do: 5 * unit(ctx.saved_tensors[0])))


def build_model(name, device):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(**MODELS[name])
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            model = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    return model


def batches(n, B, S, vocab, rank, device, offset=0):
    out = []
    for step in range(n):
        gen = torch.Generator().manual_seed(1234 + 1000 * rank + offset + step)
        ids = torch.randint(0, vocab, (B, S), generator=gen, dtype=torch.int64)
        ids = ids.to(device)
        out.append(dict(input_ids=ids, attention_mask=torch.ones_like(ids), labels=ids))
    return out


def pmc_traffic(args):
    """HBM bytes per wgrad launch from the committed rocprofv3 --pmc passes of this same bench
    configuration (scripts/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE), or None."""
    path = os.path.join(ROOT, "profiles", "r01_wgrad_pmc.json")
    if args.model != "llama3-8b" or not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return round(d.get("hbm_bytes_per_call", d.get("hbm_bytes_per_launch"))), f"profiles/r01_wgrad_pmc.json ({d['correction']})"


def cpu_baseline(seconds: float, selection_tiles: dict, model_name: str):
    """Oracle restatement of the reference's SMT linears (smt.py:350-413, per-tile loop, bf16) for
    one decoder layer at B=1, S=512, timed on this host; scaled to tokens/s of the 32-layer stack."""
    if seconds <= 0:
        return None
    from oracle import smt_oracle as ref
    # the GPU box grants each GPU a CPU share (OMP_NUM_THREADS, 16 per GPU there); use that many threads
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    cfg = MODELS[model_name]
    h, inter, kv = cfg["hidden_size"], cfg["intermediate_size"], cfg["hidden_size"] // cfg["num_attention_heads"] * cfg["num_key_value_heads"]
    shapes = {"q_proj": (h, h), "k_proj": (kv, h), "v_proj": (kv, h), "o_proj": (h, h),
              "gate_proj": (inter, h), "up_proj": (inter, h), "down_proj": (h, inter)}
    S = 512                      # bounded sample: B=1, S=512 tokens per layer pass
    gen = torch.Generator().manual_seed(0)
    mods = []
    for name, (o, i) in shapes.items():
        tiles = selection_tiles.get(name, [])
        W = (torch.randn(o, i, generator=gen) * 0.02).bfloat16()
        x = torch.randn(1, S, i, generator=gen).bfloat16()
        g = torch.randn(1, S, o, generator=gen).bfloat16()
        mods.append((W, x, g, tiles))
    t0 = time.perf_counter()
    layers = 0
    while True:
        for W, x, g, tiles in mods:
            ref.linearz_forward(x, W)
            if tiles:
                ref.linearz_backward(g, x, W, tiles)
            else:
                torch.matmul(g, W)
        layers += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    per_layer = el / layers
    tok_s = S / (per_layer * cfg["num_hidden_layers"])
    ntiles = sum(len(t) for t in selection_tiles.values())
    return {"value": tok_s, "unit": "tokens/s", "cores": cores, "kind": "port",
            "sample": (f"oracle linearZ fwd+bwd (reference per-tile loop, bf16 CPU) of the 7 linears of one "
                       f"decoder layer, B=1 S={S}, {ntiles} tiles; {layers} layer passes in {el:.1f}s, "
                       f"scaled x{cfg['num_hidden_layers']} layers; excludes attention/norms/head (optimistic)")}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; more ranks than GPUs (functional multi-rank runs on a 1-GPU box with gloo)
    # share devices round-robin
    dev_index = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(args.dist_backend)

    from sparse_matrix_tuning_amd import _hip
    _hip.load(build_if_missing=True)
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize, linear_lr_lambda
    from sparse_matrix_tuning_amd import trainer

    timer = WgradTimer()
    install_wgrad_timer(timer)
    atimer = AttnTimer()
    if not (args.eager_ops or args.sdpa_attention):
        install_attn_timer(atimer)

    t_setup = time.time()
    model = build_model(args.model, device)
    if not args.eager_ops:
        from sparse_matrix_tuning_amd.fused_llama import patch_llama
        patch_llama(model, attention=not args.sdpa_attention)
    # warm-up (full fine-tuning: fp32 master/moments for all 8 B params) always checkpoints;
    # --no-grad-ckpt turns it off for the SMT phase only (keeps activations in the 288 GB HBM)
    model.gradient_checkpointing_enable()
    model.train()
    log(f"model built in {time.time() - t_setup:.1f}s, params {sum(p.numel() for p in model.parameters()) / 1e9:.3f} B")
    vocab = MODELS[args.model]["vocab_size"]
    B, S = args.batch, args.seq

    dims = trainer.get_targeted_module_dims(model)
    total_blocks = trainer.count_total_blocks(model)
    n_att, n_mlp = trainer.block_budgets(total_blocks, args.att_ratio, args.mlp_ratio)
    log(f"num_total_blocks={total_blocks} attention budget={n_att} mlp budget={n_mlp}")

    # ---- warm-up: full fine-tuning + gradient harvest (fine_tune.py:710-775) ----
    ds_config = {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": B, "train_batch_size": B * world}
    smt_config = dict(ds_config, fp8_linears=bool(args.fp8))
    from sparse_matrix_tuning_amd.smt.smt import _NO_DECAY
    groups = [{"params": [p for n, p in model.named_parameters() if not any(nd in n.lower() for nd in _NO_DECAY)],
               "weight_decay": 0.0},
              {"params": [p for n, p in model.named_parameters() if any(nd in n.lower() for nd in _NO_DECAY)],
               "weight_decay": 0.0}]
    opt = SMTFusedAdam(groups, lr=9.865e-6, betas=(0.9, 0.95))
    engine, opt, _, _ = initialize(model=model, optimizer=opt, config=ds_config)
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    warm_batches = batches(args.full_ft_steps, B, S, vocab, rank, device, offset=100000)
    torch.cuda.reset_peak_memory_stats(device)
    t_w = time.time()
    for b in warm_batches:
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        harvester.harvest()
        engine.step()
    torch.cuda.synchronize()
    warm_peak = torch.cuda.max_memory_allocated(device) / 1e9
    log(f"warm-up {args.full_ft_steps} full-FT steps in {time.time() - t_w:.1f}s, peak {warm_peak:.1f} GB, loss {loss.item():.4f}")
    del warm_batches, loss

    # ---- selection + conversion (fine_tune.py:257-384) ----
    t_s = time.time()
    total_steps = args.full_ft_steps + args.warmup + args.steps
    engine, opt, sched, sel_mlp, sel_att = trainer.select_and_convert(
        engine, harvester, dims, n_att, n_mlp, calculate_strategy=args.calculate_strategy,
        smt_lr=args.smt_lr, num_training_steps=total_steps, ds_config=smt_config)
    del groups, opt
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    n_tiles = sum(len(v) for v in sel_mlp.values()) + sum(len(v) for v in sel_att.values())
    trainable = sum(p.numel() for p in engine.module.parameters() if p.requires_grad)
    total_params = sum(p.numel() for p in engine.module.parameters())
    log(f"selection+conversion {time.time() - t_s:.1f}s: {n_tiles} tiles, trainable {trainable} "
        f"({100.0 * trainable / total_params:.3f}% of {total_params})")
    tile_layers = sorted({l for (_m, l) in list(sel_mlp) + list(sel_att) if l is not None})
    log(f"tiles in {len(sel_mlp) + len(sel_att)} modules of layers {tile_layers}")

    # ---- SMT phase ----
    if not args.grad_ckpt:
        engine.module.gradient_checkpointing_disable()
        if hasattr(engine.module, "disable_input_require_grads"):
            engine.module.disable_input_require_grads()
    smt_batches = batches(args.warmup + args.steps, B, S, vocab, rank, device)
    log(f"SMT phase starts with {torch.cuda.memory_allocated(device) / 1e9:.1f} GB allocated")
    torch.cuda.reset_peak_memory_stats(device)

    def step(b):
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        engine.step()
        return loss

    for i in range(args.warmup):
        step(smt_batches[i])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timer.enabled = True
    atimer.enabled = True
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(smt_batches[args.warmup + i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    atimer.enabled = False
    t_max = torch.tensor([elapsed], dtype=torch.float64, device=device)
    peak = torch.tensor([torch.cuda.max_memory_allocated(device) / 1e9], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    elapsed = t_max.item()
    tokens = world * B * S * args.steps
    value = tokens / elapsed
    w = timer.summary()
    a_sum = atimer.summary()

    # ---- the reference's memory policy (per-layer recompute), same engine and tiles ----
    ckpt_mode = None
    if args.ref_mode_steps > 0 and not args.grad_ckpt:
        engine.module.gradient_checkpointing_enable()
        ref_batches = batches(1 + args.ref_mode_steps, B, S, vocab, rank, device, offset=50000)
        step(ref_batches[0])
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
        if world > 1:
            dist.barrier()
        t1 = time.perf_counter()
        for b in ref_batches[1:]:
            step(b)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        r = torch.tensor([time.perf_counter() - t1, torch.cuda.max_memory_allocated(device) / 1e9],
                         dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(r, op=dist.ReduceOp.MAX)
        ckpt_mode = {"grad_ckpt": True, "steps": args.ref_mode_steps,
                     "value": round(world * B * S * args.ref_mode_steps / r[0].item(), 1),
                     "ms_per_step": round(r[0].item() / args.ref_mode_steps * 1e3, 2),
                     "peak_hbm_gb": round(r[1].item(), 2)}
        del ref_batches

    if rank == 0:
        per_gpu = value / world
        roofline = None
        if w and w["seconds"] > 0:
            achieved = w["bytes"] / w["seconds"] / 1e9
            traffic, tsrc = pmc_traffic(args)
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic, "traffic_source": tsrc,
                        "kernel": "smt_tile_wgrad (wgrad_dma_kernel + wgrad_reduce_kernel)",
                        "launches": w["launches"], "avg_launch_us": round(w["seconds"] / w["launches"] * 1e6, 2),
                        "algorithmic_bytes_per_launch": round(w["bytes"] / w["launches"]),
                        "mfma_tflops": round(w["flops"] / w["seconds"] / 1e12, 1)}
        tiles_by_module = {}
        for (m, _l), v in list(sel_mlp.items()) + list(sel_att.items()):
            tiles_by_module.setdefault(m, [])
            tiles_by_module[m].extend(v)
        per_layer = {m: v[: max(1, round(len(v) / MODELS[args.model]["num_hidden_layers"]))] for m, v in tiles_by_module.items()}
        # the CPU baseline is a property of the N = 1 line; a multi-GPU run does not repeat it
        cpu = cpu_baseline(args.cpu_baseline_seconds, per_layer, args.model) if world == 1 else None
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "tokens/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp8-e4m3 (rowwise-scaled decoder GEMMs) + bf16" if args.fp8 else "bf16",
            "data": "synthetic (uniform token ids, labels=inputs; random-init weights)",
            "config": {"workload": (f"{'LLaMA-3-8B' if args.model == 'llama3-8b' else args.model} SMT(0.71%) "
                                    "training step (fwd+bwd+sparse AdamW)") if not args.fp8 else
                                   (f"{'DeepSeek-R1-Distill-LLaMA-8B (LLaMA-3-8B architecture)' if args.model == 'llama3-8b' else args.model}"
                                    " SMT(0.86%) fp8 training step (fwd+bwd+sparse AdamW)"),
                       "global_batch": B * world, "seq_len": S, "parallelism": f"dp{world}",
                       "tiles": n_tiles, "trainable_params": trainable,
                       "grad_ckpt": bool(args.grad_ckpt), "full_ft_steps": args.full_ft_steps,
                       "fused_llama_ops": not args.eager_ops,
                       "attention": "sdpa" if (args.eager_ops or args.sdpa_attention) else "smt_flash",
                       "loss": "transformers" if args.eager_ops else "smt_ce"},
            "peak_hbm_gb": round(peak.item(), 2), "warmup_peak_hbm_gb": round(warm_peak, 2),
            "grad_ckpt_mode": ckpt_mode,
            "step_mfma_frac": (round(per_gpu * F_ALG_GFLOP_PER_TOKEN * 1e9 / (PEAK_BF16_TFLOPS * 1e12), 4)
                               if args.model == "llama3-8b" else None),
            "roofline": roofline,
            "roofline_attention": None if not a_sum else {
                "bound": "mfma", "kernel": "smt_flash causal GQA attention (attn_fwd / attn_delta + attn_dq + attn_dkdv)",
                "achieved": round(a_sum["flops"] / a_sum["seconds"] / 1e12, 1), "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(a_sum["flops"] / a_sum["seconds"] / 1e12 / PEAK_BF16_TFLOPS, 4),
                "launches": a_sum["launches"], "avg_launch_us": round(a_sum["seconds"] / a_sum["launches"] * 1e6, 1),
                "flops_note": "algorithmic causal FLOPs: fwd 2, bwd 5 QK^T-sized GEMMs per launch"},
            "cpu_baseline": cpu,
            "final_loss": round(loss.item(), 5),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

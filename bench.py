#!/usr/bin/env python3
"""SMT-phase training throughput of LLaMA-3-8B SMT(0.71%) on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]      # N > 1: starts N ranks itself
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
   bracketed by barrier + synchronize; the max over ranks is reported. ``value`` is the K steps'
   tokens over their wall time; HIP events at the step boundaries also give the median step
   (BASELINE.md's definition: median over steps 10-60 after the conversion = the defaults).
   The reference's memory policy (per-layer recompute) is then timed over as many steps
   (``grad_ckpt_mode``).

Rank 0 prints ONE JSON line. ``roofline`` is for the dominant hand-written kernel (the tile
wgrad: smt_tile_wgrad_batch / smt_tile_wgrad = wgrad_dma | wgrad_quarter + wgrad_reduce), timed
with HIP events on its launch stream over extra steps with the wgrad stream joined (the kernel
alone); its algorithmic bytes count each distinct operand slice of a launch once, and the roof
(HBM or MFMA) follows the launch's intensity on those bytes; counter bytes beside it.
``cpu_baseline`` times the oracle's restatement of the reference path (oracle/smt_oracle.py) on this
host's cores for BASELINE.md's four units, each beside the same unit on the GPU.
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
# what a streaming kernel reaches in practice (MI355X_MICROARCH.md: a 1.2 GB in-order LDS-DMA sweep
# 6.0-6.1 TB/s, the LDS-DMA weight stream 6.4-6.8 TB/s): reported beside the spec peak, not used as it
PRACTICAL_HBM_GBS = 6300.0
PEAK_MXFP8_TFLOPS = 5000.0         # block-scaled e4m3 MFMA, 2x bf16 per clock (MI355X_MICROARCH.md)
WGRAD_ROUNDING_NOTE = {
    "reference": "reference: per-sample bf16 partials summed in sample order, rounded to bf16 (smt.py:397-404; "
                 "smt_tile_wgrad_batch_seq)",
    "single": "single: fp32 over the whole batch, rounded once (smt_tile_wgrad_batch)"}
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
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one GPU each). Without an external launcher (WORLD_SIZE unset) and N > 1, "
                         "bench.py starts N ranks itself through torch.distributed.run before touching the GPU; "
                         "under a launcher N must equal WORLD_SIZE (default: WORLD_SIZE, else 1)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)  # CPU test of the launch path
    # defaults: BASELINE.md's definition, steps 10-60 after the conversion (10 untimed, 50 timed)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
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
    ap.add_argument("--warmup-resident", default="auto",
                    help="full fine-tuning warm-up: decoder layers whose activations stay resident after the "
                         "first step ('auto': as many as the HBM above the first step's peak allows, for warm-ups of "
                         "more than RESIDENT_BREAK_EVEN_STEPS steps; 0: recompute every layer, the reference's policy)")
    ap.add_argument("--ref-mode-steps", type=int, default=None,
                    help="after the timed steps, also time this many steps with gradient checkpointing "
                         "(reported under 'grad_ckpt_mode'; default: as many as --steps; 0 disables)")
    ap.add_argument("--views-steps", type=int, default=None,
                    help="also time this many steps with the 'views' activation policy (SMT linears keep their "
                         "whole input, as the reference's ctx.list1 views do, instead of packed copies of the "
                         "column blocks their tiles read); reported under 'views_mode'; default: as many as "
                         "--steps; 0 disables")
    ap.add_argument("--selective-steps", type=int, default=None,
                    help="after the timed steps, also time this many steps with the 'selective' activation "
                         "policy (SMT linears fed by RMSNorm / SwiGLU keep no input blocks; the backward rebuilds "
                         "them; reported under 'selective_mode'; default: as many as --steps; 0 disables)")
    ap.add_argument("--half-resident-steps", type=int, default=None,
                    help="after the recompute point, also time this many steps with the same per-layer recompute "
                         "but the last half of the decoder layers resident (reported under "
                         "'grad_ckpt_half_resident_mode'; default: min(--steps, 20); 0 disables)")
    ap.add_argument("--no-transposed-steps", type=int, default=None,
                    help="after the recompute point, time this many steps of the same per-layer recompute without "
                         "the W^T copies of the data-gradient GEMMs (the engine's transposed_dgrad 'auto' default "
                         "under recompute; reported under 'grad_ckpt_no_transposed_mode' and in memory_vs_full_ft; "
                         "default: min(--steps, 20); 0 disables)")
    ap.add_argument("--transposed-dgrad", default="on", choices=("on", "off"),
                    help="the headline engine's W^T copies of the frozen linears' data-gradient GEMMs (engine key "
                         "transposed_dgrad; default on: the resident headline keeps them)")
    ap.add_argument("--ref-rounding-steps", type=int, default=None,
                    help="after the selective point, also time this many steps with the other tile-gradient rounding "
                         "than the engine's (default engine: the reference's per-sample bf16 partials, smt.py:397-404; "
                         "the point: single fp32 rounding; reported under 'wgrad_rounding_alt_mode'; default: "
                         "min(--steps, 20); 0 disables)")
    ap.add_argument("--raw-harvest-steps", type=int, default=None,
                    help="with --tile-spread layers: at the end, swap the model over to the selection the raw "
                         "(unscaled) harvest gives and time this many steps (reported under 'raw_harvest_mode'; "
                         "default: min(--steps, 20); 0 disables)")
    ap.add_argument("--tile-spread", default="layers", choices=("layers", "none"),
                    help="layers: scale each layer's harvested gradients to a common mean |g| before the "
                         "selection, so the 872 tiles spread over all 32 layers as in a real fine-tune (random "
                         "init + uniform tokens otherwise concentrate them in layers 0-4); none: select on the "
                         "raw harvest")
    ap.add_argument("--sdpa-attention", action="store_true",
                    help="keep transformers' sdpa (aotriton) attention instead of the gfx950 flash attention")
    ap.add_argument("--eager-ops", action="store_true",
                    help="keep transformers' eager RMSNorm/RoPE/SwiGLU instead of the fused HIP kernels")
    ap.add_argument("--fp8", action="store_true",
                    help="BASELINE config 5 (DeepSeek-R1-Distill-LLaMA-8B = the LLaMA-3-8B architecture, "
                         "SMT(0.86%%)): the decoder layers' frozen linears run as rowwise-scaled e4m3 GEMMs")
    ap.add_argument("--wgrad-batch-tiles", type=int, default=48,
                    help="the engine launches the tile wgrad of consecutive modules together once they hold "
                         "this many tiles (smt_tile_wgrad_batch); 0 = one launch per module")
    ap.add_argument("--no-overlap-wgrad", action="store_true",
                    help="run the tile weight gradients on the current stream (default: their own stream, "
                         "overlapped with the data-gradient GEMMs)")
    ap.add_argument("--roofline-steps", type=int, default=5,
                    help="extra SMT steps after the timed region with the wgrad stream joined, on which the "
                         "tile-wgrad roofline is measured (the kernel alone; in the timed region it shares the "
                         "chip with the data-gradient GEMM)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0, help="0 disables the CPU leg")
    ap.add_argument("--out", default=None, help="also write the JSON line here")
    ap.add_argument("--dist-backend", default=None,
                    help="nccl (= RCCL on ROCm; the default with N > 1) or gloo (functional tests). Given with "
                         "one rank, a world-1 process group of that backend is created and the engine runs its "
                         "DP exchange anyway (engine config dp_exchange: always), so the line measures the "
                         "step with the RCCL all-reduces in it")
    args = ap.parse_args()
    default_ratio = (0.0043 if args.fp8 else 0.00356) if args.model == "llama3-8b" else 0.03
    args.att_ratio = default_ratio if args.att_ratio is None else args.att_ratio
    args.mlp_ratio = default_ratio if args.mlp_ratio is None else args.mlp_ratio
    if args.ref_mode_steps is None:
        args.ref_mode_steps = args.steps
    if args.selective_steps is None:
        args.selective_steps = args.steps
    if args.views_steps is None:
        args.views_steps = args.steps
    if args.half_resident_steps is None:
        args.half_resident_steps = min(args.steps, 20)
    if args.ref_rounding_steps is None:
        args.ref_rounding_steps = min(args.steps, 20)
    if args.no_transposed_steps is None:
        args.no_transposed_steps = min(args.steps, 20)
    if args.raw_harvest_steps is None:
        args.raw_harvest_steps = min(args.steps, 20)
    return args


# The resident-layer warm-up policy saves ~0.15 s per full fine-tuning step at the 8B point (18
# layers resident: 1.70 -> 1.55 s) but its first step pays ~2 s for the fresh HBM it allocates
# (profiles/r02_warmup_resident.json): 'auto' applies it only to warm-ups long enough to gain.
RESIDENT_BREAK_EVEN_STEPS = 16


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def launch_plan(gpus, environ) -> tuple:
    """How this process runs ``--gpus N`` (no GPU call is made here).

    * ``("run", world)``: run as one rank of ``world`` in this process (under an external launcher:
      torch.distributed.run as the driver uses it, or the reference's ``deepspeed --include=...``
      launcher, deepspeed/README.md:36 + fine_tune.py:968-971, which exports the same variables);
    * ``("spawn", n)``: WORLD_SIZE is unset and N > 1: start N ranks through torch.distributed.run
      as a child process and exit with its status;
    * ``("error", message)``: ``--gpus`` disagrees with the launcher's WORLD_SIZE."""
    env_world = environ.get("WORLD_SIZE")
    if env_world is None:
        n = 1 if gpus is None else int(gpus)
        if n < 1:
            return ("error", f"--gpus {n}: need at least one rank")
        return ("spawn", n) if n > 1 else ("run", 1)
    world = int(env_world)
    if gpus is not None and int(gpus) != world:
        return ("error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("run", world)


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Start ``n`` ranks of this script (``torch.distributed.run``, one node, 127.0.0.1) as a child
    process; SIGINT / SIGTERM are passed on to it. Returns its exit status (the launcher's: non-zero
    when any rank failed)."""
    import signal
    import subprocess
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    n_dev = torch.cuda.device_count()       # counts devices without initialising one (this image)
    if n > n_dev:
        # ranks share a GPU (gloo rehearsals): one hardware queue per process. With the box's 4 per
        # process, 4 processes on one card oversubscribe its hardware queues and a step stalls for
        # 2-3 minutes (profiles/r04_b_dist4_*: GPU_MAX_HW_QUEUES=1 removes it, HSA_ENABLE_SDMA=0 does not)
        env["GPU_MAX_HW_QUEUES"] = "1"
    log("launching", n, "ranks:", " ".join(cmd), f"({n_dev} GPUs; GPU_MAX_HW_QUEUES={env.get('GPU_MAX_HW_QUEUES')})")
    proc = subprocess.Popen(cmd, env=env)

    def forward(sig, _frame):
        if proc.poll() is None:
            proc.send_signal(sig)
    old = {s: signal.signal(s, forward) for s in (signal.SIGINT, signal.SIGTERM)}
    try:
        rc = proc.wait()
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    return rc if rc >= 0 else 128 - rc


def launch_check(args, world, rank):
    """--launch-check (CPU tests of the launch path): every rank joins the process group (gloo), sums
    its rank, and rank 0 prints the line fields that identify the ranks -- no GPU is touched."""
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank)])
    dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "world_size": dist.get_world_size(), "backend": dist.get_backend(),
                          "parallelism": f"dp{world}", "rank_sum": t.item()}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


class WgradTimer:
    """HIP events around every tile-wgrad launch (smt_tile_wgrad per module, smt_tile_wgrad_batch
    for the engine's batches, smt_tile_wgrad_mx on the fp8 path), on the stream it is launched on,
    with its algorithmic bytes counted two ways: per tile (2 operand slices + the output tile), and
    per DISTINCT operand slice (a g row-block or x column-block slice that several tiles of the
    launch read counts once: the least HBM traffic the launch can have)."""

    def __init__(self):
        self.enabled = False
        self.records = []      # (start, end, bytes per tile, unique-slice bytes, flops)
        self._host_tabs = {}

    def host_rows(self, tab):
        """Host copy of a (cached, never rewritten) device tile table."""
        key = (tab.data_ptr(), tuple(tab.shape))
        rows = self._host_tabs.get(key)
        if rows is None:
            rows = self._host_tabs[key] = tab.cpu().tolist()
        return rows

    def hook(self, T, n_tiles, out_bytes, stream_fn, operand_bytes=2, slices=None):
        if not self.enabled:
            return stream_fn()
        s = torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = stream_fn()
        e1.record(s)
        per_tile = n_tiles * (T * 256 * operand_bytes * 2 + 65536 * out_bytes)
        n_slices = 2 * n_tiles if slices is None else slices
        unique = n_slices * T * 256 * operand_bytes + n_tiles * 65536 * out_bytes
        self.records.append((e0, e1, per_tile, unique, 2.0 * T * 65536 * n_tiles))
        return r

    def summary(self):
        if not self.records:
            return None
        torch.cuda.synchronize()
        t = sum(a.elapsed_time(b) for a, b, *_ in self.records) * 1e-3
        return dict(launches=len(self.records), seconds=t, bytes=sum(r[2] for r in self.records),
                    unique_bytes=sum(r[3] for r in self.records), flops=sum(r[4] for r in self.records))


def _slice_keys(g, x, rows):
    """Distinct operand slices of one module's tiles: (address of the g row-block column slice),
    (address of the x column block), from the (row_block, col_block) rows the kernel reads."""
    xbs = 256 * x.shape[1] if x.dim() == 3 else 256
    return ({g.data_ptr() + 512 * r for r, _c in rows} | {x.data_ptr() + 2 * xbs * c for _r, c in rows})


def install_wgrad_timer(timer: WgradTimer):
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.tile_wgrad

    def timed(g2, x2, rc, out, accumulate=False, order=None, seq_len=None):
        n_slices = len(_slice_keys(g2, x2, timer.host_rows(rc))) if timer.enabled else None
        return timer.hook(g2.shape[0], rc.shape[0], out.element_size(),
                          lambda: orig(g2, x2, rc, out, accumulate=accumulate, order=order, seq_len=seq_len),
                          slices=n_slices)
    _hip.tile_wgrad = timed


def install_wgrad_batch_timer(timer: WgradTimer):
    """The engine's batched launches (smt_tile_wgrad_batch: the tiles of several modules at once)."""
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.tile_wgrad_batch

    def timed(items, tab, order=None, seq_len=None):
        n_slices = None
        if timer.enabled:
            keys, rows = set(), timer.host_rows(tab)
            for m, (g2, x2, _out, _acc) in enumerate(items):
                keys |= _slice_keys(g2, x2, [(r, c) for mm, r, c, _k in rows if mm == m])
            n_slices = len(keys)
        return timer.hook(items[0][0].shape[0], tab.shape[0], items[0][2].element_size(),
                          lambda: orig(items, tab, order, seq_len=seq_len), slices=n_slices)
    _hip.tile_wgrad_batch = timed


def install_mx_wgrad_batch_timer(timer: WgradTimer):
    """The engine's batched MX launches (smt_tile_wgrad_mx_batch; the quantisation of the output
    gradients is a launch of its own, as on the per-module path)."""
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.tile_wgrad_mx_batch

    def timed(items, tab, order=None):
        n_slices = None
        if timer.enabled:
            keys, rows = set(), timer.host_rows(tab)
            for m, (g, x, _out, _acc) in enumerate(items):
                for mm, r, c, _k in rows:
                    if mm == m:
                        keys.add((g.q.data_ptr(), r))
                        keys.add((x.q.data_ptr(), c))
            n_slices = len(keys)
        return timer.hook(items[0][0].ldq, tab.shape[0], items[0][2].element_size(),
                          lambda: orig(items, tab, order), operand_bytes=1, slices=n_slices)
    _hip.tile_wgrad_mx_batch = timed


def install_mx_wgrad_timer(timer: WgradTimer):
    """The fp8 path's smt_tile_wgrad_mx (1-byte operands; T = the MX blocks' padded rows)."""
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.tile_wgrad_mx

    def timed(g, x, rc, out, accumulate=False, order=None):
        n_slices = None
        if timer.enabled:
            rows = timer.host_rows(rc)
            n_slices = len({r for r, _c in rows}) + len({c for _r, c in rows})
        return timer.hook(g.ldq, rc.shape[0], out.element_size(),
                          lambda: orig(g, x, rc, out, accumulate=accumulate, order=order), operand_bytes=1,
                          slices=n_slices)
    _hip.tile_wgrad_mx = timed


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


class LaunchTimer:
    """HIP events around the launches of one wrapped function (current stream)."""

    def __init__(self):
        self.enabled = False
        self.records = []      # (start, end, units)

    def wrap(self, fn, units_fn):
        def timed(*a, **k):
            if not self.enabled:
                return fn(*a, **k)
            s = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            r = fn(*a, **k)
            e1.record(s)
            self.records.append((e0, e1, units_fn(*a, **k)))
            return r
        return timed

    def summary(self):
        if not self.records:
            return None
        torch.cuda.synchronize()
        t = sum(a.elapsed_time(b) for a, b, _ in self.records) * 1e-3
        return dict(launches=len(self.records), seconds=t, units=sum(r[2] for r in self.records))


def install_adam_timer(timer: LaunchTimer):
    """The fused clip + AdamW + scatter over the packed tiles (engine.step), params per launch."""
    from sparse_matrix_tuning_amd import _hip
    orig = _hip.adamw_step

    def units(grad, master, *a, tiles=None, n_tiles=0, **k):
        return master.numel() if tiles is not None else 0
    _hip.adamw_step = timer.wrap(orig, units)


class SelectionTimer:
    """Wall time (device-synchronised) and gradient elements of the product's selection calls
    (smt_helper.select_submatrix_based_on_grads as trainer.select_and_convert calls it)."""

    def __init__(self):
        self.seconds = 0.0
        self.elements = 0
        self.reports = []

    def install(self):
        from sparse_matrix_tuning_amd import trainer
        from sparse_matrix_tuning_amd.smt import ranking
        orig = trainer.select_submatrix_based_on_grads

        def timed(grads, *a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = orig(grads, *a, **k)
            torch.cuda.synchronize()
            self.seconds += time.perf_counter() - t0
            self.elements += sum(g.numel() for g in grads.values())
            rep = dict(ranking.LAST_REPORT)
            self.reports.append({"flagged_blocks": rep.get("flagged"), "rescored_keys": len(rep.get("rescored_keys", [])),
                                 "worst_case_bound": rep.get("worst_case_bound")})
            return r
        trainer.select_submatrix_based_on_grads = timed


@torch.no_grad()
def spread_over_layers(harvester):
    """--tile-spread layers: scale every layer's harvested gradients (per pool) to a common mean |g|,
    so that the reference's selection picks blocks from every layer (a stand-in for the spread a real
    fine-tune's gradients have; uniform random tokens on a random-init model concentrate the gradient
    in the first layers). The selection itself is unchanged."""
    for pool in (harvester.warmup_grads, harvester.attention_warmup_grads):
        by_layer = {}
        for key, g in pool.items():
            by_layer.setdefault(key[1], []).append(g)
        for layer, gs in by_layer.items():
            m = torch.stack([g.abs().mean() for g in gs]).mean()
            for g in gs:
                g.div_(m)


def raw_selection(harvester, dims, n_att, n_mlp, calculate_strategy):
    """The reference's selection (fine_tune.py:304-327) on the harvest as it is, without the bench's
    per-layer scaling: ``(selected_mlp, selected_att)``, rank 0's on every rank."""
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.smt.smt_helper import select_submatrix_based_on_grads
    att = select_submatrix_based_on_grads(harvester.attention_warmup_grads, dims, n_att) if n_att > 0 else {}
    mlp = (select_submatrix_based_on_grads(harvester.warmup_grads, dims, n_mlp, calculate_strategy=calculate_strategy)
           if n_mlp > 0 else {})
    return trainer._broadcast(mlp, True), trainer._broadcast(att, True)


def tile_distribution(sel_mlp, sel_att):
    layers = sorted({l for (_m, l) in list(sel_mlp) + list(sel_att) if l is not None})
    per_layer = {}
    for (_m, l), v in list(sel_mlp.items()) + list(sel_att.items()):
        per_layer[l] = per_layer.get(l, 0) + len(v)
    return {"tiles": sum(len(v) for v in sel_mlp.values()) + sum(len(v) for v in sel_att.values()),
            "tile_modules": len(sel_mlp) + len(sel_att), "tile_layers": len(layers),
            "tiles_per_layer": {str(l): per_layer[l] for l in sorted(per_layer, key=lambda x: (x is None, x))},
            "max_tiles_per_module": max([len(v) for v in list(sel_mlp.values()) + list(sel_att.values())] or [0])}


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


def pmc_traffic(args, rounding):
    """HBM bytes per wgrad launch from the committed rocprofv3 --pmc passes of this same bench
    configuration (scripts/pmc_traffic.py; FETCH_SIZE x2 + WRITE_SIZE), or None."""
    path = None
    # the counters of the launch pattern this run uses: batched (engine default) or one per module
    if args.wgrad_batch_tiles <= 0:
        cands = ("r02_wgrad_pmc.json", "r01_wgrad_pmc.json")
    elif rounding == "reference":             # the per-sample slabs of smt_tile_wgrad_batch_seq
        cands = ("r06_g_wgrad_pmc.json", "r05_end_wgrad_pmc.json", "r05_k_wgrad_pmc.json", "r05_p_wgrad_pmc.json", "r04_s_wgrad_pmc.json", "r04_e_wgrad_pmc.json", "r04_final_wgrad_pmc.json")
    else:
        cands = ("r03_final_wgrad_pmc.json", "r02_final_wgrad_pmc.json", "r02_wgrad_batch_pmc.json")
    for cand in cands:
        if os.path.exists(os.path.join(ROOT, "profiles", cand)):
            path = os.path.join(ROOT, "profiles", cand)
            break
    if args.model != "llama3-8b" or args.fp8 or path is None:
        return None, None
    with open(path) as f:
        d = json.load(f)
    return round(d.get("hbm_bytes_per_call", d.get("hbm_bytes_per_launch"))), f"profiles/{os.path.basename(path)} ({d['correction']})"


def _host_cores() -> int:
    """The GPU box grants each GPU a CPU share (OMP_NUM_THREADS, 16 per GPU there)."""
    n = len(os.sched_getaffinity(0))
    return min(n, int(os.environ.get("OMP_NUM_THREADS", "0")) or n)


def _layer_shapes(cfg):
    h, inter = cfg["hidden_size"], cfg["intermediate_size"]
    kv = h // cfg["num_attention_heads"] * cfg["num_key_value_heads"]
    return {"q_proj": (h, h), "k_proj": (kv, h), "v_proj": (kv, h), "o_proj": (h, h),
            "gate_proj": (inter, h), "up_proj": (inter, h), "down_proj": (h, inter)}


def _layer_operands(cfg, S, gen, dtype=torch.bfloat16):
    ops = {}
    for name, (o, i) in _layer_shapes(cfg).items():
        ops[name] = ((torch.randn(o, i, generator=gen) * 0.02).to(dtype), torch.randn(1, S, i, generator=gen).to(dtype),
                     torch.randn(1, S, o, generator=gen).to(dtype))
    return ops


def cpu_unit_layer(seconds, tiles, cfg, S=2048):
    """Unit 1, CPU: the reference's SMT linears of one decoder layer (smt.py:350-413: dense forward,
    per-tile batched-matmul + sum loop, dense data gradient) in bf16 on the host, B=1."""
    from oracle import smt_oracle as ref
    ops = _layer_operands(cfg, S, torch.Generator().manual_seed(0))
    t0 = time.perf_counter()
    passes = 0
    while True:
        for name, (W, x, g) in ops.items():
            ref.linearz_forward(x, W)
            if tiles.get(name):
                ref.linearz_backward(g, x, W, tiles[name])
            else:
                torch.matmul(g, W)
        passes += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return S * passes / el, f"{passes} passes in {el:.1f}s"


def gpu_unit_layer(tiles, cfg, device, S=2048, iters=10):
    """Unit 1, GPU: the same layer through the product's SMT modules (linearZ)."""
    from sparse_matrix_tuning_amd.smt.smt import LinearLayer_MatrixSparsity
    ops = _layer_operands(cfg, S, torch.Generator().manual_seed(0))
    mods = []
    for name, (W, x, g) in ops.items():
        Wd = torch.nn.Parameter(W.to(device), requires_grad=False)
        m = LinearLayer_MatrixSparsity(Wd, index_list=tiles.get(name, [])) if tiles.get(name) else None
        mods.append((m, Wd, x.to(device).requires_grad_(True), g.to(device)))

    def run():
        for m, Wd, x, g in mods:
            y = m(x) if m is not None else torch.nn.functional.linear(x, Wd)
            y.backward(g)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    return S * iters / (e0.elapsed_time(e1) * 1e-3)


def cpu_unit_selection(model_name, layers=4):
    """Unit 2, CPU: the reference's block scan + heap selection (smt_helper.py:40-146, fp32 ATen on the
    host) over `layers` layers of the LLaMA-3-8B-shaped pools (bounded sample; elements/s scale
    linearly in the layer count). Attention: mean_abs, MLP: abs_mean, n = 436 each."""
    from oracle import smt_oracle as ref
    cfg = MODELS[model_name]
    shapes = _layer_shapes(cfg)
    gen = torch.Generator().manual_seed(5)
    dims = {k: list(v) for k, v in shapes.items()}
    pools = {"att": {}, "mlp": {}}
    for layer in range(layers):
        for m in ("q_proj", "k_proj", "v_proj"):
            pools["att"][(m, layer)] = torch.randn(*shapes[m], generator=gen) * 1e-4
        for m in ("gate_proj", "up_proj", "down_proj"):
            pools["mlp"][(m, layer)] = torch.randn(*shapes[m], generator=gen) * 1e-4
    elems = sum(g.numel() for p in pools.values() for g in p.values())
    t0 = time.perf_counter()
    ref.select_submatrix(pools["att"], dims, 436)
    ref.select_submatrix(pools["mlp"], dims, 436, calculate_strategy="abs_mean")
    el = time.perf_counter() - t0
    return elems / el, f"{layers} of {cfg['num_hidden_layers']} layers ({elems / 1e9:.2f} G elements) in {el:.1f}s"


def cpu_unit_adam(n_params, seconds=5.0):
    """Unit 3, CPU: DeepSpeed FusedAdam's update restated (oracle.fused_adam_step, fp32 torch on the
    host) plus the global-norm clip, over n_params parameters."""
    from oracle import smt_oracle as ref
    gen = torch.Generator().manual_seed(3)
    p = torch.randn(n_params, generator=gen) * 0.02
    g = torch.randn(n_params, generator=gen) * 1e-4
    m, v = torch.zeros(n_params), torch.zeros(n_params)
    t0 = time.perf_counter()
    steps = 0
    while True:
        steps += 1
        coef = ref.clip_coef([g], 1.0)
        ref.fused_adam_step(p, g * coef, m, v, steps, 9.865e-6, (0.9, 0.95))
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return n_params * steps / el, f"{steps} steps over {n_params / 1e6:.1f} M params in {el:.1f}s"


OPT_125M = dict(vocab_size=50272, hidden_size=768, ffn_dim=3072, num_hidden_layers=12, num_attention_heads=12,
                word_embed_proj_dim=768, max_position_embeddings=2048)


def _opt_model(device):
    from transformers import OPTConfig, OPTForCausalLM
    cfg = OPTConfig(**OPT_125M)
    cfg._attn_implementation = "sdpa"
    torch.manual_seed(1234)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device(device):
            return OPTForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)


def _opt_batch(step, B=4, S=128):
    g = torch.Generator().manual_seed(777 + step)
    ids = torch.randint(2, OPT_125M["vocab_size"], (B, S), generator=g)
    return {"input_ids": ids, "attention_mask": torch.ones_like(ids), "labels": ids}


def gpu_unit_opt(device, steps=10):
    """Unit 4, GPU: config 1 (OPT-125m SMT(1%): 19 attention tiles, MLP ratio < 0) through the
    product: one full-FT warm-up step with the harvest, selection + conversion, then timed SMT steps
    (B=4, S=128 synthetic). Returns (steps/s, selection)."""
    from sparse_matrix_tuning_amd import trainer
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    model = _opt_model(device)
    dims = trainer.get_targeted_module_dims(model)
    n_att, n_mlp = trainer.block_budgets(trainer.count_total_blocks(model), 0.01, -1)
    opt = SMTFusedAdam(model.parameters(), lr=1e-5, betas=(0.9, 0.95))
    engine, _, _, _ = initialize(model=model, optimizer=opt, config={"gradient_clipping": 1.0})
    harvester = trainer.GradHarvester(model, n_mlp, n_att)
    b = {k: v.to(device) for k, v in _opt_batch(0).items()}
    engine.backward(engine(**b, use_cache=False).loss)
    harvester.harvest()
    engine.step()
    engine, _o, _s, sel_mlp, sel_att = trainer.select_and_convert(engine, harvester, dims, n_att, n_mlp,
                                                                 smt_lr=1e-4, num_training_steps=100)
    batches_ = [{k: v.to(device) for k, v in _opt_batch(1 + i).items()} for i in range(steps + 2)]

    def step(b):
        engine.backward(engine(**b, use_cache=False).loss)
        engine.step()
    for b in batches_[:2]:
        step(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in batches_[2:]:
        step(b)
    torch.cuda.synchronize()
    rate = steps / (time.perf_counter() - t0)
    del engine, model
    torch.cuda.empty_cache()
    return rate, dict(sel_att)


def cpu_unit_opt(sel_att, seconds=10.0):
    """Unit 4, CPU: the reference's SMT step of config 1 on the host (oracle modules: tile write-back
    every forward, per-tile wgrad loop; clip + FusedAdam restated), bf16, B=4, S=128."""
    from oracle import smt_oracle as ref
    model = _opt_model("cpu")
    names = [n for n, _ in model.named_parameters()]
    flags = ref.freeze_flags(names, {}, sel_att)
    for n, p in model.named_parameters():
        p.requires_grad = flags[n]
    ref.ref_convert(model, {}, sel_att)
    tiles = [m.selected_weight for m in model.modules() if isinstance(m, ref.RefLinearLayer_MatrixSparsity)]
    master = [t.detach().float() for t in tiles]
    mom = [(torch.zeros_like(t), torch.zeros_like(t)) for t in master]
    steps = 0
    t0 = time.perf_counter()
    while True:
        out = model(**_opt_batch(100 + steps), use_cache=False)
        out.loss.backward()
        grads = [t.grad.float() for t in tiles]
        coef = ref.clip_coef(grads, 1.0)
        steps += 1
        for t, p, g, (m, v) in zip(tiles, master, grads, mom):
            ref.fused_adam_step(p, g * coef, m, v, steps, 1e-4)
            t.data.copy_(p)
            t.grad = None
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return steps / el, f"{steps} steps in {el:.1f}s"


def cpu_baseline(seconds: float, tiles_one_layer: dict, model_name: str, gpu: dict, device):
    """BASELINE.md CPU-baseline units 1-4 (the oracle's restatement of the reference path timed on this
    host's cores), each next to the same unit on the GPU. Unit 1 is the headline ``value``."""
    if seconds <= 0:
        return None
    cores = _host_cores()
    torch.set_num_threads(cores)
    cfg = MODELS[model_name]
    units = []
    gpu_layer = gpu_unit_layer(tiles_one_layer, cfg, device)
    log("cpu baseline: unit 1 (decoder layer)")
    cpu_layer, s1 = cpu_unit_layer(seconds, tiles_one_layer, cfg)
    units.append({"unit": 1, "what": "one decoder layer's 7 SMT linears, fwd + bwd, B=1 S=2048 "
                  f"({sum(len(v) for v in tiles_one_layer.values())} tiles)", "metric": "tokens/s",
                  "cpu": round(cpu_layer, 2), "gpu": round(gpu_layer, 1), "cpu_sample": s1})
    if gpu.get("selection"):
        log("cpu baseline: unit 2 (selection)")
        cpu_sel, s2 = cpu_unit_selection(model_name)
        units.append({"unit": 2, "what": "block scan + top-n selection (attention mean_abs, MLP abs_mean, n=436 each)",
                      "metric": "elements/s", "cpu": round(cpu_sel), "gpu": round(gpu["selection"]["elements_per_s"]),
                      "cpu_sample": s2, "gpu_sample": gpu["selection"]["sample"]})
    if gpu.get("adam"):
        log("cpu baseline: unit 3 (sparse AdamW)")
        cpu_adam, s3 = cpu_unit_adam(gpu["adam"]["params"])
        units.append({"unit": 3, "what": "sparse AdamW (clip + update) over the trainable tiles", "metric": "params/s",
                      "cpu": round(cpu_adam), "gpu": round(gpu["adam"]["params_per_s"]), "cpu_sample": s3,
                      "gpu_sample": gpu["adam"]["sample"]})
    try:
        log("cpu baseline: unit 4 (OPT-125m step)")
        gpu_opt, sel = gpu_unit_opt(device)
        cpu_opt, s4 = cpu_unit_opt(sel)
        units.append({"unit": 4, "what": "config 1: OPT-125m SMT(1%) training step (19 attention tiles), B=4 S=128",
                      "metric": "steps/s", "cpu": round(cpu_opt, 3), "gpu": round(gpu_opt, 2), "cpu_sample": s4})
    except Exception as exc:                     # keep the headline line even if the side unit fails
        units.append({"unit": 4, "error": repr(exc)[:300]})
    for u in units:
        if "cpu" in u and u["cpu"]:
            u["gpu_over_cpu"] = round(u["gpu"] / u["cpu"], 1)
    return {"value": round(cpu_layer, 2), "unit": units[0]["metric"] + " (unit 1: " + units[0]["what"] + ")",
            "cores": cores, "kind": "port",
            "sample": "oracle/smt_oracle.py restatement of the reference path on the host CPU; " + s1,
            "units": units}


def memory_vs_full_ft(ckpt_mode, no_t_mode, full_ft_gb, harvest_gb, ckpt_copies=True):
    """The reference's one published figure for this path: SMT cuts the GPU memory footprint of full
    fine-tuning by 67 % (README.md:5). Same activation policy on both sides (every layer recomputed,
    fine_tune.py:192); the harvest accumulators, which the reference keeps on the host, are taken out of
    the full fine-tuning peak. One point per W^T setting, tokens/s beside each; ``reduction`` is the
    engine's default at this policy (transposed_dgrad "auto": no copies when layers are recomputed)."""
    points = []
    for mode, copies in ((ckpt_mode, ckpt_copies), (no_t_mode, False)):
        if mode is not None:
            points.append({"transposed_dgrad": copies, "smt_peak_gb": mode["peak_hbm_gb"],
                           "reduction": round(1.0 - mode["peak_hbm_gb"] / full_ft_gb, 4),
                           "tokens_per_s": mode["value"], "median_ms_per_step": mode["median_ms_per_step"]})
    default = points[-1]
    return {"policy": "every layer recomputed (fine_tune.py:192) in both",
            "smt_peak_gb": default["smt_peak_gb"], "full_ft_peak_gb": round(full_ft_gb, 2),
            "harvest_accumulators_gb": round(harvest_gb, 2), "reduction": default["reduction"],
            "default_transposed_dgrad": default["transposed_dgrad"], "points": points,
            "reference_claim": {"reduction": 0.67, "source": "README.md:5", "gpu": "unspecified"}}


def _median(xs):
    xs = sorted(xs)
    n = len(xs)
    return xs[n // 2] if n % 2 else 0.5 * (xs[n // 2 - 1] + xs[n // 2])


def timed_steps(step, batch_list, world, device):
    """Run the steps between barrier + synchronize on both sides; HIP events at every step boundary
    give per-step durations (for the median) without synchronising inside the region."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(len(batch_list) + 1)]
    t0 = time.perf_counter()
    evs[0].record()
    loss = None
    for i, b in enumerate(batch_list):
        loss = step(b)
        evs[i + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_step = [evs[i].elapsed_time(evs[i + 1]) * 1e-3 for i in range(len(batch_list))]
    return elapsed, per_step, loss


def main():
    args = parse()
    if os.environ.get("SMT_BENCH_STACKS"):
        # diagnostics: every thread's Python stack to stderr every N seconds (a stalled multi-rank run)
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["SMT_BENCH_STACKS"]), repeat=True)
    # decided before any GPU call: a parent that starts ranks must not initialise the device
    mode, what = launch_plan(args.gpus, os.environ)
    if mode == "error":
        print(f"bench.py: {what}", file=sys.stderr, flush=True)
        sys.exit(2)
    if mode == "spawn":
        sys.exit(spawn_ranks(what, sys.argv[1:]))
    world = what
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        launch_check(args, world, rank)
        return
    n_dev = torch.cuda.device_count()
    dist_backend = args.dist_backend or "nccl"
    pg1 = world == 1 and args.dist_backend is not None     # a world-1 group: the exchange runs anyway
    if dist_backend == "nccl" and world > n_dev:
        # RCCL needs one GPU per rank: never report N ranks that shared fewer devices as N GPUs
        raise SystemExit(f"bench.py: {world} ranks with the nccl (RCCL) backend need {world} GPUs; "
                         f"this node has {n_dev}")
    # one process per GPU; more ranks than GPUs (functional multi-rank runs on a 1-GPU box with gloo)
    # share devices round-robin
    if world > n_dev and os.environ.get("GPU_MAX_HW_QUEUES") != "1":
        log(f"warning: {world} ranks share {n_dev} GPU(s) with GPU_MAX_HW_QUEUES="
            f"{os.environ.get('GPU_MAX_HW_QUEUES')}: hardware-queue oversubscription stalls steps (DESIGN §7); "
            "bench.py --gpus N sets 1 when it starts the ranks itself")
    dev_index = local % max(1, n_dev)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1 or pg1:
        kw = {} if (world > 1 or "MASTER_ADDR" in os.environ) else {"store": dist.HashStore(), "rank": 0,
                                                                  "world_size": 1}
        if dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device, **kw)
        else:
            dist.init_process_group(dist_backend, **kw)
    backend = dist.get_backend() if dist.is_initialized() else None
    devices_used = n_dev if world > n_dev else world

    from sparse_matrix_tuning_amd import _hip
    _hip.load(build_if_missing=True)
    from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
    from sparse_matrix_tuning_amd import trainer

    timer = WgradTimer()
    install_wgrad_timer(timer)
    install_wgrad_batch_timer(timer)
    mx_timer = WgradTimer()
    install_mx_wgrad_timer(mx_timer)
    install_mx_wgrad_batch_timer(mx_timer)
    atimer = AttnTimer()
    if not (args.eager_ops or args.sdpa_attention):
        install_attn_timer(atimer)
    adam_timer = LaunchTimer()
    install_adam_timer(adam_timer)
    sel_timer = SelectionTimer()
    sel_timer.install()

    t_setup = time.time()
    model = build_model(args.model, device)
    if not args.eager_ops:
        from sparse_matrix_tuning_amd.fused_llama import patch_llama
        patch_llama(model, attention=not args.sdpa_attention)
    # warm-up (full fine-tuning: fp32 master/moments for all 8 B params) always checkpoints
    # (fine_tune.py:192); the SMT phase keeps activations resident unless --grad-ckpt
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
    ds_config = {"gradient_clipping": 1.0, "train_micro_batch_size_per_gpu": B, "train_batch_size": B * world,
                 "dp_exchange": "always" if pg1 else "auto"}
    # the headline keeps activations resident, so its engine keeps the W^T copies of the data-gradient
    # GEMMs (the model still recomputes its layers from the warm-up when the engine is built, which
    # the "auto" default would read as the reference's memory policy)
    smt_config = dict(ds_config, fp8_linears=bool(args.fp8), overlap_wgrad=not args.no_overlap_wgrad,
                      wgrad_batch_tiles=args.wgrad_batch_tiles, transposed_dgrad=args.transposed_dgrad == "on")
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
    warm_times, resident = [], 0
    for i, b in enumerate(warm_batches):
        t0 = time.time()
        loss = engine(**b, use_cache=False).loss
        engine.backward(loss)
        harvester.harvest()
        engine.step()
        torch.cuda.synchronize()
        warm_times.append(time.time() - t0)
        if i == 0 and args.warmup_resident != "0" and len(warm_batches) > 1 and (
                args.warmup_resident != "auto" or len(warm_batches) - 1 >= RESIDENT_BREAK_EVEN_STEPS):
            # the first step ran with every layer recomputed (the reference's policy); its peak
            # holds all persistent state (fp32 optimizer state, harvest accumulators): keep as many
            # layers' activations resident as the HBM above it allows
            n = (trainer.resident_layers_for(model, B, S, torch.cuda.max_memory_allocated(device))
                 if args.warmup_resident == "auto" else int(args.warmup_resident))
            resident = trainer.set_resident_layers(model, n)
    warm_peak = torch.cuda.max_memory_allocated(device) / 1e9
    # the fp32 harvest accumulators live in HBM here; the reference keeps them on the host
    # (fine_tune.py:714-767), so they are not part of its full fine-tuning footprint
    harvest_gb = sum(t.numel() * t.element_size() for pool in (harvester.warmup_grads, harvester.attention_warmup_grads)
                     for t in pool.values() if t.is_cuda) / 1e9
    warm_s = time.time() - t_w
    trainer.set_resident_layers(model, 0)
    log(f"warm-up {args.full_ft_steps} full-FT steps in {warm_s:.1f}s ({', '.join(f'{t:.2f}' for t in warm_times)} s; "
        f"{resident} layers resident after the first), peak {warm_peak:.1f} GB, loss {loss.item():.4f}")
    del warm_batches, loss
    raw_sel = None
    if args.tile_spread == "layers" and args.raw_harvest_steps > 0 and not args.fp8:
        # the selection the raw harvest gives (smt_helper.py:102-139 on the unscaled gradients), kept
        # for the raw_harvest_mode point at the end
        raw_sel = raw_selection(harvester, dims, n_att, n_mlp, args.calculate_strategy)
    if args.tile_spread == "layers":
        spread_over_layers(harvester)

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
    log(f"selection+conversion {time.time() - t_s:.1f}s (selection {sel_timer.seconds:.2f}s over "
        f"{sel_timer.elements / 1e9:.2f} G elements; band {sel_timer.reports}): {n_tiles} tiles, trainable "
        f"{trainable} ({100.0 * trainable / total_params:.3f}% of {total_params})")
    tile_layers = sorted({l for (_m, l) in list(sel_mlp) + list(sel_att) if l is not None})
    n_modules = len(sel_mlp) + len(sel_att)
    log(f"tiles in {n_modules} modules of {len(tile_layers)} layers {tile_layers}")

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
    torch.cuda.synchronize()
    log(f"{args.warmup} untimed SMT steps done; timing {args.steps}")
    timer.enabled = mx_timer.enabled = atimer.enabled = adam_timer.enabled = True
    elapsed, per_step, loss = timed_steps(step, smt_batches[args.warmup:], world, device)
    timer.enabled = mx_timer.enabled = atimer.enabled = adam_timer.enabled = False
    t_max = torch.tensor([elapsed, _median(per_step)], dtype=torch.float64, device=device)
    peak = torch.tensor([torch.cuda.max_memory_allocated(device) / 1e9], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(peak, op=dist.ReduceOp.MAX)
    elapsed, med = t_max[0].item(), t_max[1].item()
    tokens = world * B * S * args.steps
    value = tokens / elapsed
    w = timer.summary()
    w_mx = mx_timer.summary()
    a_sum = atimer.summary()
    adam = adam_timer.summary()
    del smt_batches
    log(f"timed: {value:.1f} tokens/s ({elapsed / args.steps * 1e3:.1f} ms/step), peak {peak[0].item():.1f} GB")

    # ---- the tile wgrad alone (its roofline): the same steps with the wgrad stream joined ----
    overlapped = {"bf16": w, "mx": w_mx}

    def isolated_wgrad(n_steps, offset):
        """Timer summaries of the tile wgrad over n_steps SMT steps with the wgrad stream joined."""
        side = engine.wgrad_stream
        engine.wgrad_stream = None
        for tg in engine.tile_groups:
            if tg.buckets is not None:
                tg.buckets.side_stream = None
        iso = batches(n_steps, B, S, vocab, rank, device, offset=offset)
        timer.records, mx_timer.records = [], []
        timer.enabled = mx_timer.enabled = True
        for b in iso:
            step(b)
        torch.cuda.synchronize()
        timer.enabled = mx_timer.enabled = False
        engine.wgrad_stream = side
        for tg in engine.tile_groups:
            if tg.buckets is not None:
                tg.buckets.side_stream = side
        del iso
        return timer.summary(), mx_timer.summary()

    if engine.wgrad_stream is not None and args.roofline_steps > 0:
        w, w_mx = isolated_wgrad(args.roofline_steps, 70000)
        log(f"roofline steps done ({args.roofline_steps}, wgrad stream joined)")

    # ---- the selective activation policy: GEMM outputs, attention O / LSE resident; the SMT linears'
    # RMSNorm / SwiGLU input blocks rebuilt in the backward (smt.set_activation_policy) ----
    def policy_point(n_steps, offset, label):
        pb = batches(1 + n_steps, B, S, vocab, rank, device, offset=offset)
        step(pb[0])
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
        el, per, _ = timed_steps(step, pb[1:], world, device)
        r = torch.tensor([el, _median(per), torch.cuda.max_memory_allocated(device) / 1e9],
                         dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(r, op=dist.ReduceOp.MAX)
        del pb
        return {label: True, "steps": n_steps,
                "value": round(world * B * S * n_steps / r[0].item(), 1),
                "ms_per_step": round(r[0].item() / n_steps * 1e3, 2),
                "median_ms_per_step": round(r[1].item() * 1e3, 2),
                "median_tokens_per_s": round(world * B * S / r[1].item(), 1),
                "peak_hbm_gb": round(r[2].item(), 2)}

    selective_mode = None
    if args.selective_steps > 0 and not args.grad_ckpt and not args.fp8:
        from sparse_matrix_tuning_amd.smt import smt as _smt
        old_policy = _smt.set_activation_policy("selective")
        selective_mode = policy_point(args.selective_steps, 60000, "selective")
        selective_mode["recomputed"] = ("the column blocks SMT linears read of RMSNorm / SwiGLU outputs "
                                        "(smt_colblock_recompute in the backward)")
        _smt.set_activation_policy(old_policy)
        log(f"selective policy: {selective_mode['value']} tokens/s at {selective_mode['peak_hbm_gb']} GB")

    # ---- the "views" activation policy: the SMT linears keep their whole input,
    # as the reference's ctx.list1 views do (smt.py:351-358), instead of the packed copies of the
    # column blocks their tiles read (smt_colblock_gather on the wgrad stream, beside the GEMMs) ----
    views_mode = None
    if args.views_steps > 0 and not args.grad_ckpt and not args.fp8:
        from sparse_matrix_tuning_amd.smt import smt as _smt
        old_policy = _smt.set_activation_policy("views")
        views_mode = policy_point(args.views_steps, 65000, "views")
        views_mode["kept"] = "every SMT linear's whole input (no column-block copies)"
        views_mode["median_step_vs_headline"] = round(views_mode["median_ms_per_step"] / (med * 1e3), 4)
        _smt.set_activation_policy(old_policy)
        log(f"views policy: {views_mode['value']} tokens/s at {views_mode['peak_hbm_gb']} GB "
            f"(median step x{views_mode['median_step_vs_headline']})")

    # ---- the other tile-gradient rounding, same engine and tiles: the headline
    # runs the engine's default, the reference's per-sample bf16 partials (smt.py:397-404); this point
    # runs fp32 over the whole batch, rounded once ----
    alt_round_mode = None
    headline_rounding = engine.wgrad_rounding
    if args.ref_rounding_steps > 0 and not args.fp8 and engine.tile_groups:
        alt = "single" if headline_rounding == "reference" else "reference"
        engine.wgrad_rounding = alt
        alt_round_mode = policy_point(args.ref_rounding_steps, 30000, "wgrad_rounding_" + alt)
        engine.wgrad_rounding = headline_rounding
        alt_round_mode["wgrad_rounding"] = WGRAD_ROUNDING_NOTE[alt]
        alt_round_mode["median_step_vs_headline"] = round(alt_round_mode["median_ms_per_step"] / (med * 1e3), 4)
        if engine.wgrad_stream is not None and args.roofline_steps > 0:
            # the tile wgrad kernel alone under this rounding, as the headline's roofline is measured
            engine.wgrad_rounding = alt
            wa, _wm = isolated_wgrad(args.roofline_steps, 35000)
            engine.wgrad_rounding = headline_rounding
            if wa and wa["seconds"] > 0:
                avg_a = wa["seconds"] / wa["launches"]
                uniq_a = wa["unique_bytes"] / wa["launches"]
                traffic_a, tsrc_a = pmc_traffic(args, alt)
                alt_round_mode["wgrad_kernel"] = {
                    "launches": wa["launches"], "avg_launch_us": round(avg_a * 1e6, 2),
                    "algorithmic_bytes_per_launch": round(uniq_a),
                    "hbm_frac_on_algorithmic_bytes": round(uniq_a / avg_a / 1e9 / PEAK_HBM_GBS, 4),
                    "traffic": traffic_a, "traffic_source": tsrc_a}
        log(f"{alt} rounding: {alt_round_mode['value']} tokens/s (median step x{alt_round_mode['median_step_vs_headline']})")

    # ---- the reference's memory policy (per-layer recompute), same engine and tiles ----
    ckpt_mode = half_mode = no_t_mode = None
    if args.ref_mode_steps > 0 and not args.grad_ckpt:
        engine.module.gradient_checkpointing_enable()
        ref_batches = batches(1 + args.ref_mode_steps, B, S, vocab, rank, device, offset=50000)
        step(ref_batches[0])
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(device)
        el2, per2, _ = timed_steps(step, ref_batches[1:], world, device)
        r = torch.tensor([el2, _median(per2), torch.cuda.max_memory_allocated(device) / 1e9],
                         dtype=torch.float64, device=device)
        if world > 1:
            dist.all_reduce(r, op=dist.ReduceOp.MAX)
        ckpt_mode = {"grad_ckpt": True, "steps": args.ref_mode_steps,
                     "value": round(world * B * S * args.ref_mode_steps / r[0].item(), 1),
                     "ms_per_step": round(r[0].item() / args.ref_mode_steps * 1e3, 2),
                     "median_ms_per_step": round(r[1].item() * 1e3, 2),
                     "median_tokens_per_s": round(world * B * S / r[1].item(), 1),
                     "peak_hbm_gb": round(r[2].item(), 2)}
        del ref_batches
        log(f"recompute policy: {ckpt_mode['value']} tokens/s at {ckpt_mode['peak_hbm_gb']} GB")
        # a point between the two: the same per-layer recompute, with the last half of the decoder
        # layers resident (trainer.set_resident_layers: the MI355X memory-budget policy)
        if args.half_resident_steps > 0:
            n_half = trainer.set_resident_layers(engine.module, len(trainer.checkpointed_layers(engine.module)) // 2)
            half_mode = policy_point(args.half_resident_steps, 40000, "grad_ckpt")
            half_mode["resident_layers"] = n_half
            trainer.set_resident_layers(engine.module, 0)
            log(f"recompute policy, {n_half} layers resident: {half_mode['value']} tokens/s at "
                f"{half_mode['peak_hbm_gb']} GB")
        # the same recompute without the W^T copies: every data gradient then runs
        # g @ W on hipBLASLt's NN layout, and the 14 GB of copies are gone. This is what an engine built
        # on a recomputing model gets by default (transposed_dgrad "auto", fine_tune.py:192)
        if args.no_transposed_steps > 0 and not args.fp8 and engine.transposed_bytes:
            copies_gb = engine.transposed_bytes / 1e9
            engine.set_transposed_dgrad(False)
            torch.cuda.empty_cache()
            no_t_mode = policy_point(args.no_transposed_steps, 45000, "grad_ckpt")
            no_t_mode["transposed_dgrad"] = False
            no_t_mode["transposed_copies_dropped_gb"] = round(copies_gb, 2)
            no_t_mode["median_step_vs_with_copies"] = round(no_t_mode["median_ms_per_step"] /
                                                            ckpt_mode["median_ms_per_step"], 4)
            engine.set_transposed_dgrad(True)
            log(f"recompute policy without W^T copies: {no_t_mode['value']} tokens/s at "
                f"{no_t_mode['peak_hbm_gb']} GB (median step x{no_t_mode['median_step_vs_with_copies']})")
        engine.module.gradient_checkpointing_disable()

    # ---- the raw harvest's selection (no per-layer scaling), swapped in at the end ----
    raw_mode = None
    if raw_sel is not None:
        t_r = time.time()
        engine, _o, _s = trainer.reselect(engine, raw_sel[0], raw_sel[1], smt_lr=args.smt_lr,
                                          num_training_steps=total_steps, ds_config=smt_config)
        del _o, _s
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        reconvert_s = time.time() - t_r
        raw_mode = policy_point(args.raw_harvest_steps, 20000, "raw_harvest")
        raw_mode.update(tile_distribution(*raw_sel))
        raw_mode["reconversion_s"] = round(reconvert_s, 2)
        raw_mode["median_step_vs_headline"] = round(raw_mode["median_ms_per_step"] / (med * 1e3), 4)
        log(f"raw-harvest selection: {raw_mode['value']} tokens/s, {raw_mode['tiles']} tiles in "
            f"{raw_mode['tile_modules']} modules of {raw_mode['tile_layers']} layers")

    if rank == 0:
        per_gpu = value / world
        roofline = None
        mx = bool(w_mx and w_mx["seconds"] > 0)
        if mx:                              # the fp8 path: the MX-fp8 tile wgrad is the SMT kernel
            w = w_mx
        w_ov = overlapped["mx" if mx else "bf16"]
        if w and w["seconds"] > 0:
            avg = w["seconds"] / w["launches"]
            tflops = w["flops"] / w["seconds"] / 1e12
            alg_bytes = w["bytes"] / w["launches"]
            uniq_bytes = w["unique_bytes"] / w["launches"]
            alg_gbs = alg_bytes / avg / 1e9
            uniq_gbs = uniq_bytes / avg / 1e9
            traffic, tsrc = (None, None) if mx else pmc_traffic(args, headline_rounding)
            peak_mfma = PEAK_MXFP8_TFLOPS if mx else PEAK_BF16_TFLOPS
            # The roof: the launch's intensity on its DISTINCT operand slices (each g row-block / x
            # column-block slice once, however many tiles read it) against the ridge peak_mfma / HBM.
            # The spread selection shares few slices: ~128-190 F/B, below the 312 F/B bf16 ridge.
            intensity = w["flops"] / max(1.0, w["unique_bytes"])
            ridge = peak_mfma * 1e12 / (PEAK_HBM_GBS * 1e9)
            hbm_bound = intensity < ridge
            hbm = {"achieved": round(uniq_gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                   "frac": round(uniq_gbs / PEAK_HBM_GBS, 4),
                   "on_per_tile_bytes": round(alg_gbs, 1), "frac_on_per_tile_bytes": round(alg_gbs / PEAK_HBM_GBS, 4),
                   "on_counter_bytes": None if traffic is None else round(traffic / avg / 1e9, 1),
                   "frac_on_counter_bytes": None if traffic is None else round(traffic / avg / 1e9 / PEAK_HBM_GBS, 4),
                   "practical_streaming_gbs": PRACTICAL_HBM_GBS,
                   "frac_of_practical_on_per_tile_bytes": round(alg_gbs / PRACTICAL_HBM_GBS, 4)}
            mfma = {"achieved": round(tflops, 1), "peak": peak_mfma, "unit": "TFLOP/s",
                    "frac": round(tflops / peak_mfma, 4), "intensity_flop_per_byte": round(intensity, 1),
                    "ridge_flop_per_byte": round(ridge, 1)}
            roof = hbm if hbm_bound else mfma
            roofline = {"bound": "hbm" if hbm_bound else "mfma", "achieved": roof["achieved"], "peak": roof["peak"],
                        "unit": roof["unit"], "frac": roof["frac"], "traffic": traffic, "traffic_source": tsrc,
                        "kernel": ("smt_tile_wgrad_mx (wgrad_mx_kernel, + wgrad_reduce_kernel when split; MX-fp8 operands)"
                                   if mx else "smt_tile_wgrad (wgrad_dma_kernel | wgrad_quarter_kernel, + "
                                              "wgrad_reduce_kernel when split)"),
                        "launches": w["launches"], "avg_launch_us": round(avg * 1e6, 2),
                        "measured_on": (f"{args.roofline_steps} SMT steps after the timed region with the wgrad "
                                        "stream joined (the kernel alone)" if engine.wgrad_stream is not None
                                        and args.roofline_steps > 0 else "the timed region"),
                        "timed_region_avg_launch_us": (round(w_ov["seconds"] / w_ov["launches"] * 1e6, 2)
                                                       if w_ov and w_ov["launches"] else None),
                        "timed_region_note": ("in the timed region the tile wgrad runs on its own stream beside "
                                              "the MFMA-bound data-gradient GEMM: its launches stretch over the "
                                              "GEMM's duration while the step gets shorter"
                                              if engine.wgrad_stream is not None else None),
                        "algorithmic_bytes_per_launch": round(uniq_bytes),
                        "per_tile_bytes_per_launch": round(alg_bytes),
                        "tiles_per_launch": round(w["flops"] / w["launches"] / (2.0 * 65536 * B * S), 1),
                        "flops_per_launch": round(w["flops"] / w["launches"]),
                        "hbm": hbm, "mfma": mfma,
                        "bytes_note": (("algorithmic bytes per launch = distinct operand slices (T x 256 x 1 B each: "
                                        "a g row-block or x column-block slice several tiles read counts once) + the "
                                        "fp32 tiles; the MX quantisation of the operands is a separate launch")
                                       if mx else
                                       ("algorithmic bytes per launch = distinct operand slices (T x 256 x 2 B each: a g "
                                        "row-block or x column-block slice several tiles of the launch read counts once) "
                                        "+ the fp32 tiles; per_tile_bytes counts both slices of every tile; traffic = "
                                        "FETCH_SIZE x2 + WRITE_SIZE (rocprofv3 --pmc) per launch, including the split-K "
                                        "slabs and their reduce"))}
        tiles_by_module = {}
        for (m, _l), v in list(sel_mlp.items()) + list(sel_att.items()):
            tiles_by_module.setdefault(m, []).extend(v)
        nl = MODELS[args.model]["num_hidden_layers"]
        per_layer = {m: v[: max(1, round(len(v) / nl))] for m, v in tiles_by_module.items()}
        gpu_units = {}
        if sel_timer.seconds > 0:
            gpu_units["selection"] = {"elements_per_s": sel_timer.elements / sel_timer.seconds,
                                      "sample": f"{sel_timer.elements / 1e9:.2f} G harvested elements in "
                                                f"{sel_timer.seconds:.2f}s (GPU scan + host ranking + re-score)"}
        if adam and adam["units"]:
            gpu_units["adam"] = {"params": adam["units"] // adam["launches"],
                                 "params_per_s": adam["units"] / adam["seconds"],
                                 "sample": f"{adam['launches']} launches of smt_adamw_step over the tiles"}
        # the CPU baseline is a property of the N = 1 line; a multi-GPU run does not repeat it
        cpu = (cpu_baseline(args.cpu_baseline_seconds, per_layer, args.model, gpu_units, device)
               if world == 1 else None)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "tokens/s", "n_gpus": world,
            "world_size": dist.get_world_size() if dist.is_initialized() else 1, "backend": backend, "devices_used": devices_used,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2),
            "median_ms_per_step": round(med * 1e3, 2), "median_tokens_per_s": round(world * B * S / med, 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp8-e4m3 (rowwise-scaled decoder GEMMs) + bf16" if args.fp8 else "bf16",
            "data": "synthetic (uniform token ids, labels=inputs; random-init weights)",
            "config": {"workload": (f"{'LLaMA-3-8B' if args.model == 'llama3-8b' else args.model} SMT(0.71%) "
                                    "training step (fwd+bwd+sparse AdamW)") if not args.fp8 else
                                   (f"{'DeepSeek-R1-Distill-LLaMA-8B (LLaMA-3-8B architecture)' if args.model == 'llama3-8b' else args.model}"
                                    " SMT(0.86%) fp8 training step (fwd+bwd+sparse AdamW)"),
                       "global_batch": B * world, "seq_len": S, "parallelism": f"dp{world}",
                       "tiles": n_tiles, "tile_modules": n_modules, "tile_layers": len(tile_layers),
                       "trainable_params": trainable,
                       "tile_spread": ("layer-normalised harvest (tiles over all layers, as in a real fine-tune)"
                                       if args.tile_spread == "layers" else "raw harvest"),
                       "activations": "recomputed per layer (fine_tune.py:192)" if args.grad_ckpt else
                                      "resident in HBM (MI355X default; the reference's recompute policy: grad_ckpt_mode)",
                       "grad_ckpt": bool(args.grad_ckpt), "full_ft_steps": args.full_ft_steps,
                       "transposed_dgrad": args.transposed_dgrad == "on",
                       "wgrad_rounding": WGRAD_ROUNDING_NOTE.get(headline_rounding, headline_rounding),
                       "fused_llama_ops": not args.eager_ops,
                       "attention": "sdpa" if (args.eager_ops or args.sdpa_attention) else "smt_flash",
                       "loss": "transformers" if args.eager_ops else "smt_ce"},
            "peak_hbm_gb": round(peak.item(), 2), "warmup_peak_hbm_gb": round(warm_peak, 2),
            "warmup_full_ft_s_per_step": round(warm_s / max(1, args.full_ft_steps), 2),
            "warmup_full_ft": {"s_per_step": [round(t, 3) for t in warm_times], "resident_layers": resident,
                       "policy": ("every layer recomputed (fine_tune.py:192)" if not resident else
                                  "first step: every layer recomputed (fine_tune.py:192); later steps: the last "
                                  f"{resident} layers' activations resident (HBM above the first step's peak)")},
            "selection": {"seconds": round(sel_timer.seconds, 3), "elements": sel_timer.elements,
                          "band": sel_timer.reports},
            "grad_ckpt_mode": ckpt_mode, "grad_ckpt_half_resident_mode": half_mode,
            # the reference's one published figure for this path: SMT cuts the GPU memory footprint of
            # full fine-tuning by 67 % (README.md:5). Same activation policy on both sides (every layer
            # recomputed, fine_tune.py:192); the harvest accumulators, which the reference keeps on
            # the host, are taken out of the full fine-tuning peak
            "memory_vs_full_ft": None if (ckpt_mode is None or resident or args.fp8) else memory_vs_full_ft(
                ckpt_mode, no_t_mode, warm_peak - harvest_gb, harvest_gb, args.transposed_dgrad == "on"),
            "grad_ckpt_no_transposed_mode": no_t_mode,
            "selective_mode": selective_mode,
            "views_mode": views_mode,
            "wgrad_rounding_alt_mode": alt_round_mode,
            "raw_harvest_mode": raw_mode,
            "tile_distribution": tile_distribution(sel_mlp, sel_att),
            "step_mfma_frac": (round(per_gpu * F_ALG_GFLOP_PER_TOKEN * 1e9 / (PEAK_BF16_TFLOPS * 1e12), 4)
                               if args.model == "llama3-8b" else None),
            "roofline": roofline,
            "roofline_attention": None if not a_sum else {
                "bound": "mfma", "kernel": "smt_flash causal GQA attention (attn_fwd / attn_dq + attn_dkdv)",
                "achieved": round(a_sum["flops"] / a_sum["seconds"] / 1e12, 1), "peak": PEAK_BF16_TFLOPS,
                "unit": "TFLOP/s", "frac": round(a_sum["flops"] / a_sum["seconds"] / 1e12 / PEAK_BF16_TFLOPS, 4),
                "launches": a_sum["launches"], "avg_launch_us": round(a_sum["seconds"] / a_sum["launches"] * 1e6, 1),
                "flops_note": "algorithmic causal FLOPs: fwd 2, bwd 5 QK^T-sized GEMMs per launch"},
            "cpu_baseline": cpu,
            "step_ms": [round(t * 1e3, 2) for t in per_step],
            "final_loss": round(loss.item(), 5),
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

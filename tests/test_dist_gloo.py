"""The N>1 path on CPU with gloo, world_size 2 and 4: the packed tile-gradient all-reduce + dense averaging
of the engine, the bucketed backward-overlapped tile all-reduce, and the rank-0 selection broadcast
(SURVEY §8(e))."""
import os
import socket
from collections import defaultdict

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import allreduce_gradients
    from sparse_matrix_tuning_amd.trainer import _broadcast
    torch.manual_seed(rank)
    tiles = torch.randn(3 * 65536)
    dense = [torch.randn(7, 5), torch.randn(11)]
    all_tiles = [torch.zeros_like(tiles) for _ in range(world)]
    dist.all_gather(all_tiles, tiles)
    all_dense = [[torch.zeros_like(d) for _ in range(world)] for d in dense]
    for d, bucket in zip(dense, all_dense):
        dist.all_gather(bucket, d)
    allreduce_gradients([tiles], dense, world)
    # raw sum (1/world is folded into the kernels); bit-equal for two ranks, otherwise up to the
    # collective's own summation order
    ok = torch.equal(tiles, sum(all_tiles)) if world == 2 else torch.allclose(tiles, sum(all_tiles), rtol=0, atol=1e-5)
    ok &= all(torch.allclose(d, sum(b) / world) for d, b in zip(dense, all_dense))
    # every rank proposes a different selection; rank 0's wins everywhere
    sel = defaultdict(list, {("up_proj", rank): [(rank, 1), (0, 0)]})
    got = _broadcast(sel, True)
    ok &= dict(got) == {("up_proj", 0): [(0, 1), (0, 0)]}
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_tile_allreduce_and_selection_broadcast(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import TileGradBuckets
    sizes = [3, 1, 4, 1, 5, 2]                         # tiles per module, forward order
    ranges, off = [], 0
    for k in sizes:
        ranges.append((off * 16, (off + k) * 16))      # 16 "elements" per tile keeps it small
        off += k
    buf = torch.zeros(off * 16)
    buckets = TileGradBuckets(buf, ranges, bucket_elems=5 * 16)
    ok = [b[:2] for b in buckets.buckets] == [[0, 128], [128, 224], [224, 256]]
    ok &= buckets.bucket_of == [0, 0, 0, 1, 1, 2]
    for step in range(2):
        buckets.arm()
        for i in reversed(range(len(sizes))):         # backward order; module 2 never reports
            s, e = ranges[i]
            buf[s:e] = float(rank + 1) * (i + 1) + step
            if i != 2:
                buckets.ready(i)
        ok &= buckets.works[2] is not None and buckets.works[1] is not None and buckets.works[0] is None
        buckets.finish()
        tri = world * (world + 1) // 2                 # sum of the ranks' (rank + 1)
        want = torch.cat([torch.full((e - s,), float(tri * (i + 1) + world * step)) for i, (s, e) in enumerate(ranges)])
        ok &= torch.equal(buf, want)
    buckets.ready(0)                                   # not armed: ignored
    ok &= not buckets.armed
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_bucketed_tile_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _dense_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import DenseGradBuckets
    torch.manual_seed(0)                                # same weights on both ranks
    net = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))
    unused = torch.nn.Parameter(torch.ones(3))          # never gets a gradient
    params = [unused] + list(net.parameters())         # reversed: last layer first, `unused` last
    buckets = DenseGradBuckets(params, bucket_elems=50, world=world)
    ok = [[p.numel() for p in b] for b in buckets.buckets] == [[4, 64], [16, 128], [3]]
    x = torch.randn(5, 8, generator=torch.Generator().manual_seed(10 + rank))
    for step in range(2):
        # this rank's own gradients (p.grad becomes the bucket buffer, reduced in flight, once armed)
        local = list(torch.autograd.grad(net(x).pow(2).sum(), list(net.parameters())))
        for p in params:
            p.grad = None
        buckets.arm()
        net(x).pow(2).sum().backward()
        ok &= buckets.next >= 1                         # the last layer's bucket went out during backward
        gathered = [[torch.zeros_like(g) for _ in range(world)] for g in local]
        buckets.finish()
        for g, bucket in zip(local, gathered):
            dist.all_gather(bucket, g)
        ok &= all(torch.allclose(p.grad, sum(b) / world) for p, b in zip(net.parameters(), gathered))
        ok &= torch.equal(unused.grad, torch.zeros(3))
        # the averaged gradients ARE the bucket buffers (no copy back): p.grad views of one flat tensor
        b0 = buckets.buckets[0]
        ok &= b0[1].grad.data_ptr() == b0[0].grad.data_ptr() + 4 * b0[0].numel()
    # a gradient accumulated again after its bucket went out would be lost: that raises
    buckets.arm()
    net(x).pow(2).sum().backward()
    last = buckets.buckets[0][0]
    try:
        buckets._hook(last)
        ok = False
    except RuntimeError as e:
        ok &= "again" in str(e)
    buckets.finish()
    buckets.remove()
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_bucketed_dense_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dense_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _order_worker(rank, world, port, q):
    """Buckets are issued in the same order on every rank whatever order their modules report in."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import TileGradBuckets
    ranges = [(i * 16, (i + 1) * 16) for i in range(4)]
    buf = torch.full((64,), float(rank + 1))
    b = TileGradBuckets(buf, ranges, bucket_elems=16)  # one module per bucket
    b.arm()
    order = [0, 3, 1, 2] if rank == 0 else [3, 2, 1, 0]
    issued = []
    for i in order:
        b.ready(i)
        issued.append([w is not None for w in b.works])
    b.finish()
    ok = torch.equal(buf, torch.full((64,), float(world * (world + 1) // 2)))
    if rank == 0:           # 0 first: nothing may go out before bucket 3 (the last) does
        ok &= issued[0] == [False] * 4 and issued[1] == [False, False, False, True]
    b2 = TileGradBuckets(buf, ranges, bucket_elems=0)  # <= 0: one bucket
    ok &= len(b2.buckets) == 1
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_bucket_issue_order_is_rank_independent(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_order_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _mixed_dtype_worker(rank, world, port, q):
    """A mixed-precision model (fp32 norm-like scale beside bf16 weights): each dtype
    fills buckets of its own, and every p.grad comes back DP-averaged in its own dtype."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import DenseGradBuckets
    torch.manual_seed(0)
    lin1 = torch.nn.Linear(8, 16).to(torch.bfloat16)
    scale = torch.nn.Parameter(torch.rand(16) + 0.5)     # fp32
    lin2 = torch.nn.Linear(16, 4).to(torch.bfloat16)
    params = list(lin1.parameters()) + [scale] + list(lin2.parameters())
    buckets = DenseGradBuckets(params, bucket_elems=40, world=world)
    ok = all(len({p.dtype for p in b}) == 1 for b in buckets.buckets)
    ok &= sorted(p.numel() for b in buckets.buckets for p in b) == sorted(p.numel() for p in params)
    x = torch.randn(5, 8, generator=torch.Generator().manual_seed(10 + rank)).to(torch.bfloat16)

    def loss():
        return lin2((lin1(x).float() * scale).to(torch.bfloat16)).float().pow(2).sum()
    local = list(torch.autograd.grad(loss(), params))
    buckets.arm()
    loss().backward()
    buckets.finish()
    for p, g in zip(params, local):
        got = [torch.zeros_like(g) for _ in range(world)]
        dist.all_gather(got, g)
        want = sum(t.float() for t in got) / world
        ok &= p.grad.dtype == p.dtype
        ok &= torch.allclose(p.grad.float(), want, rtol=2e-2, atol=1e-3)
    buckets.remove()
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_dense_buckets_mixed_dtypes():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mixed_dtype_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


def _fp16_headroom_worker(rank, world, port, q):
    """loss-scaled fp16 gradients that are finite on every rank but whose cross-rank SUM
    exceeds 65504. The dense buckets divide fp16 buckets by the world size before the all-reduce (as
    DeepSpeed's ZeRO-2 reduction does), so the average comes back finite and exact."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from sparse_matrix_tuning_amd.engine import DenseGradBuckets
    p16 = torch.nn.Parameter(torch.zeros(64, dtype=torch.float16))
    p32 = torch.nn.Parameter(torch.zeros(8))
    buckets = DenseGradBuckets([p16, p32], bucket_elems=16, world=world)
    buckets.arm()
    big = 40000.0 + 64.0 * rank                       # fp16-exact, as are their halves and their mean
    ((p16.float() * big).sum() + (p32 * (rank + 1.0)).sum()).backward()
    buckets.finish()
    want16 = sum(40000.0 + 64.0 * r for r in range(world)) / world      # any two sum past 65504
    ok = p16.grad.dtype == torch.float16 and bool(torch.isfinite(p16.grad).all())
    ok &= torch.equal(p16.grad.float(), torch.full((64,), want16))
    ok &= torch.equal(p32.grad, torch.full((8,), sum(r + 1.0 for r in range(world)) / world))   # fp32: sum, then divide
    buckets.remove()
    q.put((rank, bool(ok)))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_dense_fp16_buckets_average_without_overflow():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fp16_headroom_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}

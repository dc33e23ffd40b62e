"""Host logic of the SMT checkpoint: a save whose rank-0 write fails raises on every rank
(gloo world 2) instead of leaving the others at a barrier, and a directory holding files of two
different saves (an overwrite that crashed half-way) is refused on load. CPU only: an engine-shaped
object without tile groups."""
import os
import shutil
import socket
from types import SimpleNamespace

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from sparse_matrix_tuning_amd import checkpoint


def _engine(seed=0):
    torch.manual_seed(seed)
    return SimpleNamespace(module=torch.nn.Linear(8, 4), tile_groups=[], global_steps=3, micro_steps=3,
                           lr_scheduler=None)


def test_save_ids_tie_the_files_of_one_save(tmp_path):
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    checkpoint.save_checkpoint(_engine(0), a)
    checkpoint.save_checkpoint(_engine(1), b)
    eng = _engine(0)
    assert checkpoint.load_optimizer_state(eng, a) == {}
    # an overwrite of `a` by another save that died before its meta file: STATE from b, META from a
    shutil.copy(os.path.join(b, checkpoint.STATE), os.path.join(a, checkpoint.STATE))
    with pytest.raises(ValueError, match="another save"):
        checkpoint.load_optimizer_state(eng, a)
    shutil.copy(os.path.join(b, checkpoint.FROZEN), os.path.join(a, checkpoint.FROZEN))
    with pytest.raises(ValueError, match="another save"):
        checkpoint.restore_model(torch.nn.Linear(8, 4), a)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, bad_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        checkpoint.save_checkpoint(_engine(), bad_dir)
        q.put((rank, "no error"))
    except Exception as e:             # noqa: BLE001 - the test inspects it
        q.put((rank, type(e).__name__))
    dist.barrier()
    dist.destroy_process_group()


def test_failed_rank0_write_raises_on_every_rank(tmp_path):
    bad = tmp_path / "file"
    bad.write_text("not a directory")                    # makedirs fails on rank 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(bad / "ckpt"), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert res[0] in ("FileExistsError", "NotADirectoryError") and res[1] == "RuntimeError", res

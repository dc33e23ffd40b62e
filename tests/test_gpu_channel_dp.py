"""Config 4's activation harvest at world size 2: the reference all-reduces every
hook's bf16 ``|x|`` each step and adds it in fp32 (fine_tune.py:651-665). Two ranks (gloo, both on
cuda:0) collect activations of different batches; the product's accumulators equal
``oracle.channel_hook_accumulate_ranks`` applied to the two ranks' hooked inputs BIT FOR BIT, on both
ranks, and the channel selections of both pools equal the restatement's."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_channel_harvest_world2_matches_reference_rank_reduction(tmp_path):
    out = str(tmp_path / "c.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "channel_dp_worker.py"), "--out", out]
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT, GPU_MAX_HW_QUEUES="1"), capture_output=True, text=True,
                       timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = torch.load(out, weights_only=True)
    assert res["keys"] == 2 * (3 + 3)
    assert res["ranks_equal"]
    assert res["acc_equal_restatement"]
    assert res["differs_from_rank0_alone"]          # the other rank's activations are really in there
    assert res["sel_att"] == res["ref_att"]
    assert res["sel_mlp"] == res["ref_mlp"]

"""bench.py's multi-rank launch: ``--gpus N`` starts N ranks itself when no
launcher is present, refuses a mismatch with a launcher's WORLD_SIZE, and refuses more RCCL ranks
than GPUs. CPU only: the launch-check mode joins a gloo group and touches no GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update({k: str(v) for k, v in kw.items()})
    return env


def test_launch_plan():
    assert bench.launch_plan(None, {}) == ("run", 1)
    assert bench.launch_plan(1, {}) == ("run", 1)
    assert bench.launch_plan(8, {}) == ("spawn", 8)
    assert bench.launch_plan(None, {"WORLD_SIZE": "4"}) == ("run", 4)
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}) == ("run", 4)
    mode, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"})
    assert mode == "error" and "WORLD_SIZE=1" in msg
    assert bench.launch_plan(0, {})[0] == "error"


@pytest.mark.timeout(180)
def test_gpus_2_spawns_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--launch-check"], env=_env(), capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out == {"n_gpus": 2, "world_size": 2, "backend": "gloo", "parallelism": "dp2", "rank_sum": 1.0}


def test_gpus_mismatch_with_launcher_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--launch-check"],
                       env=_env(WORLD_SIZE=2, RANK=0, LOCAL_RANK=0, MASTER_ADDR="127.0.0.1", MASTER_PORT=1),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_nccl_ranks_beyond_devices_refused():
    # this container has no GPU: two RCCL ranks cannot each own one
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "mini"],
                       env=_env(WORLD_SIZE=2, RANK=0, LOCAL_RANK=0, MASTER_ADDR="127.0.0.1", MASTER_PORT=1),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "need 2 GPUs" in r.stderr


def test_memory_vs_full_ft_reports_both_transposed_settings():
    """the reference's one published figure (README.md:5, 67 % less GPU memory than
    full fine-tuning) reported at the recompute policy with and without the W^T copies, tokens/s beside
    each; the headline ``reduction`` is the engine's default at that policy (no copies)."""
    ck = {"peak_hbm_gb": 49.02, "value": 28510.0, "median_ms_per_step": 1145.25}
    nt = {"peak_hbm_gb": 34.26, "value": 29109.5, "median_ms_per_step": 1125.11}
    m = bench.memory_vs_full_ft(ck, nt, 133.99, 25.77)
    assert [p["transposed_dgrad"] for p in m["points"]] == [True, False]
    assert m["default_transposed_dgrad"] is False and m["smt_peak_gb"] == 34.26
    assert m["reduction"] == round(1 - 34.26 / 133.99, 4) and m["reduction"] > m["reference_claim"]["reduction"]
    assert m["points"][0]["reduction"] == round(1 - 49.02 / 133.99, 4)
    assert m["points"][1]["tokens_per_s"] == 29109.5
    only = bench.memory_vs_full_ft(ck, None, 133.99, 25.77)          # --no-transposed-steps 0
    assert len(only["points"]) == 1 and only["default_transposed_dgrad"] is True
    off = bench.memory_vs_full_ft(nt, None, 133.99, 25.77, ckpt_copies=False)   # --transposed-dgrad off
    assert off["points"][0]["transposed_dgrad"] is False

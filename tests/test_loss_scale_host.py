"""fp16 loss scaling of the engine (the reference's --dtype fp16: deepspeed_helpers.py:53-55), host logic.

The engine's ``DynamicLossScale`` against the oracle's restatement of DeepSpeed 0.16.5's
DynamicLossScaler (external; parity unpinned by the reference): the same scale, tolerance and
iteration state after every update, over random overflow sequences and the config variants DeepSpeed
exposes (hysteresis, consecutive_hysteresis, window, minimum, static scale). No GPU.
"""
import random

import pytest
import torch
from torch import nn

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd.engine import DynamicLossScale, initialize


def _pair(cfg):
    prod = DynamicLossScale(cfg)
    oracle = ref.RefDynamicLossScaler(init_scale=2.0 ** cfg.get("initial_scale_power", 16),
                                      scale_window=cfg.get("loss_scale_window", 1000),
                                      min_scale=cfg.get("min_loss_scale", 1),
                                      delayed_shift=cfg.get("hysteresis", 2),
                                      consecutive_hysteresis=cfg.get("consecutive_hysteresis", False))
    return prod, oracle


@pytest.mark.parametrize("cfg", [
    {"enabled": True, "loss_scale_window": 100},                     # the reference's fp16 config
    {"enabled": True, "loss_scale_window": 3, "hysteresis": 1},
    {"enabled": True, "loss_scale_window": 5, "hysteresis": 3, "initial_scale_power": 8},
    {"enabled": True, "loss_scale_window": 4, "consecutive_hysteresis": True, "hysteresis": 2},
    {"enabled": True, "loss_scale_window": 2, "min_loss_scale": 4, "initial_scale_power": 4},
])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_dynamic_loss_scale_follows_the_restatement(cfg, seed):
    prod, oracle = _pair(cfg)
    rng = random.Random(seed)
    p_overflow = rng.choice([0.05, 0.3, 0.6])
    for it in range(400):
        overflow = rng.random() < p_overflow
        try:
            oracle.update_scale(overflow)
        except RuntimeError:
            with pytest.raises(RuntimeError):
                prod.update(overflow)
            return
        prod.update(overflow)
        assert prod.scale == oracle.cur_scale, it
        assert prod.tolerance == oracle.cur_hysteresis, it
        assert prod.iteration == oracle.cur_iter and prod.last_overflow == oracle.last_overflow_iter


def test_dynamic_loss_scale_known_sequence():
    """The reference's config (window 100, hysteresis 2, 2**16): the first overflow is tolerated,
    the second halves; 100 clean iterations after the last overflow double it."""
    s = DynamicLossScale({"enabled": True, "loss_scale_window": 100})
    assert s.scale == 65536.0
    s.update(True)
    assert s.scale == 65536.0 and s.tolerance == 1
    s.update(True)
    assert s.scale == 32768.0
    for _ in range(99):
        s.update(False)
    assert s.scale == 32768.0
    s.update(False)                                  # iteration 101 - last overflow 1 = 100
    assert s.scale == 65536.0 and s.tolerance == 2


def test_static_loss_scale_never_moves():
    s = DynamicLossScale({"enabled": True, "loss_scale": 128})
    for o in (True, True, False, True):
        s.update(o)
    assert s.scale == 128.0


def test_overflow_at_the_minimum_raises():
    s = DynamicLossScale({"enabled": True, "initial_scale_power": 1, "hysteresis": 1, "min_loss_scale": 1})
    s.update(True)
    assert s.scale == 1.0
    with pytest.raises(RuntimeError):
        s.update(True)


def test_fp16_step_scales_unscale_with_the_updated_scale():
    """The restated ZeRO-1/2 step: the scale grows BEFORE the gradients are unscaled, so the step on
    which it doubles divides by the new scale; the clip uses the same scale."""
    scaler = ref.RefDynamicLossScaler(init_scale=4.0, scale_window=1, delayed_shift=2)
    g = [torch.full((4,), 8.0)]
    overflow, mult = ref.fp16_step_scales(scaler, g, 0.0)
    assert not overflow and scaler.cur_scale == 8.0 and mult == 1.0 / 8.0
    overflow, mult = ref.fp16_step_scales(scaler, [torch.tensor([float("inf")])], 0.0)
    assert overflow and mult is None and scaler.cur_scale == 8.0          # tolerated
    # clip: ||g|| / scale = 16 / 16 = 1 > 0.5 -> combined = (1 + 1e-6) / 0.5 * 16
    scaler = ref.RefDynamicLossScaler(init_scale=16.0, scale_window=1000)
    overflow, mult = ref.fp16_step_scales(scaler, [torch.tensor([16.0])], 0.5)
    assert mult == pytest.approx(1.0 / ((1.0 + 1e-6) / 0.5 * 16.0), rel=1e-12)


def test_engine_checks_the_config_dtype_against_the_model():
    """DeepSpeed casts the model to the config's dtype; this engine takes it in that dtype and says
    so when it is not."""
    net = nn.Linear(8, 8).to(torch.bfloat16)
    with pytest.raises(ValueError, match="fp16 enabled"):
        initialize(model=net, optimizer=None, config={"fp16": {"enabled": True}})
    with pytest.raises(ValueError, match="bf16 enabled"):
        initialize(model=nn.Linear(8, 8), optimizer=None, config={"bf16": {"enabled": True}})
    eng, _, _, _ = initialize(model=nn.Linear(8, 8).half(), optimizer=None,
                              config={"fp16": {"enabled": True, "loss_scale_window": 100}})
    assert eng.loss_scaler is not None and eng.loss_scaler.scale == 65536.0 and eng.loss_scaler.window == 100
    eng, _, _, _ = initialize(model=nn.Linear(8, 8), optimizer=None, config={"fp16": {"enabled": False}})
    assert eng.loss_scaler is None                    # the reference's fp32 (fp16 disabled)


def test_loss_scale_state_round_trip():
    """The state a checkpoint carries (checkpoint.py meta "loss_scaler") restores the schedule: the
    restored scaler and the original stay equal under the same later overflows."""
    import json
    a = DynamicLossScale({"enabled": True, "loss_scale_window": 3, "initial_scale_power": 10})
    for o in (True, False, True, True, False, False):
        a.update(o)
    b = DynamicLossScale({"enabled": True})
    b.load_state_dict(json.loads(json.dumps(a.state_dict())))      # through the JSON meta file
    assert b.state_dict() == a.state_dict()
    for o in (False, False, False, True, False, True, True):
        a.update(o)
        b.update(o)
        assert b.state_dict() == a.state_dict()

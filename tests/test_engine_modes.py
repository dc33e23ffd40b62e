"""Engine-scoped modes: an engine's ``"wgrad_rounding"`` / ``"activation_policy"`` config
keys stay on the engine (linearZ reads them through the module's gradient sink) and never change the
global setting that other models and later engines see."""
import gc

import pytest
import torch

from sparse_matrix_tuning_amd.smt import smt


class _Eng:
    pass


class _Sink:
    def __init__(self, engine):
        self.engine = engine


def test_engine_modes_are_scoped_to_the_engine():
    before = (smt.wgrad_rounding(), smt.activation_policy())
    e = _Eng()
    e.wgrad_rounding, e.activation_policy = "reference", "selective"
    smt.register_engine_modes(e, e.wgrad_rounding, e.activation_policy)
    assert (smt.wgrad_rounding(), smt.activation_policy()) == before
    assert smt._engine_mode(_Sink(e), "wgrad_rounding") == "reference"
    assert smt._engine_mode(_Sink(e), "activation_policy") == "selective"
    assert smt._engine_mode(None, "wgrad_rounding") is None
    other = _Eng()
    other.wgrad_rounding = other.activation_policy = None
    assert smt._engine_mode(_Sink(other), "wgrad_rounding") is None
    # producers tag their outputs while an engine asks for "selective", and stop when it is gone
    n = smt._selective_engines
    assert n >= 1
    out = torch.zeros(2)
    smt.tag_recompute(out, 0, torch.zeros(2))
    assert "_smt_recompute" in out.__dict__
    del e
    gc.collect()
    assert smt._selective_engines == n - 1


def test_engine_mode_values_validated():
    with pytest.raises(ValueError):
        smt.register_engine_modes(_Eng(), "double", None)
    with pytest.raises(ValueError):
        smt.register_engine_modes(_Eng(), None, "offload")

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


def test_default_rounding_is_the_reference():
    """without SMT_WGRAD_ROUNDING the global tile-gradient rounding is the
    reference's (smt.py:397-404); "views" is an accepted activation policy."""
    import os
    assert smt.wgrad_rounding() == os.environ.get("SMT_WGRAD_ROUNDING", "reference")
    assert "views" in smt.ACTIVATION_POLICIES
    old = smt.set_activation_policy("views")
    assert smt.set_activation_policy(old) == "views"


def _dp_exchange_worker(q):
    """One process, a world-1 gloo group: an engine with dp_exchange "always" arms the dense buckets
    and all-reduces them (the identity at world 1); "auto" does not; an unknown value raises."""
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1)
        from sparse_matrix_tuning_amd.engine import SMTFusedAdam, initialize
        res = {}
        for mode in ("auto", "always"):
            torch.manual_seed(0)
            net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Linear(32, 4))
            opt = SMTFusedAdam(net.parameters(), lr=1e-3)
            eng, *_ = initialize(model=net, optimizer=opt, config={"dp_exchange": mode, "reduce_bucket_size": 100})
            x = torch.randn(8, 16)
            eng.backward(eng(x).square().sum())
            grads = [p.grad.clone() for p in net.parameters()]
            res[mode] = (eng.exchange, eng.dense_buckets.issued if eng.dense_buckets else 0, grads)
        ok = (res["auto"][:2] == (False, 0) and res["always"][0] and res["always"][1] > 1
              and all(torch.equal(a, b) for a, b in zip(res["auto"][2], res["always"][2])))
        try:
            initialize(model=net, optimizer=SMTFusedAdam(net.parameters(), lr=1e-3), config={"dp_exchange": "never"})
            ok = False
        except ValueError:
            pass
        q.put(bool(ok))
    except Exception as e:          # reported to the parent
        q.put(repr(e))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_dp_exchange_always_at_world_one_gloo():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_dp_exchange_worker, args=(q,))
    p.start()
    res = q.get(timeout=120)
    p.join(timeout=60)
    assert res is True, res


def test_transposed_dgrad_key():
    """``transposed_dgrad``: "auto" (default) keeps W^T copies for resident activations and none when
    the model recomputes its layers (fine_tune.py:192); booleans force it; other strings raise."""
    from sparse_matrix_tuning_amd.engine import transposed_dgrad_wanted

    class M:
        is_gradient_checkpointing = False
    m = M()
    assert transposed_dgrad_wanted({}, m) is True
    m.is_gradient_checkpointing = True
    assert transposed_dgrad_wanted({}, m) is False
    assert transposed_dgrad_wanted({"transposed_dgrad": "auto"}, m) is False
    assert transposed_dgrad_wanted({"transposed_dgrad": True}, m) is True
    assert transposed_dgrad_wanted({"transposed_dgrad": False}, M()) is False
    assert transposed_dgrad_wanted({}, torch.nn.Linear(2, 2)) is True       # no checkpointing attribute
    with pytest.raises(ValueError):
        transposed_dgrad_wanted({"transposed_dgrad": "always"}, m)

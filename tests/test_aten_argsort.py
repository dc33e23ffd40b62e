"""norm_dist's tie order: the reference ranks with the unstable
``torch.argsort(v, descending=True)`` on CPU tensors (smt_helper.py:86, 191; the harvests are
``.cpu()``, fine_tune.py:733, 657). ATen's CPU kernel runs std::sort over (value, index) pairs, so
equal values come out in libstdc++ introsort's order, not index order. The product restates that
sort (ranking.aten_argsort_desc) and uses it wherever equal values decide ``indices[:n]``.

Pinned two ways on this host: against torch.argsort itself (torch 2.10 here; the reference pins
2.1.2, whose CPU sort kernel makes the same std::sort call), and against g++'s std::sort /
std::partial_sort on the same pairs (tests/stdsort_probe.cpp)."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest
import torch

from oracle import smt_oracle as ref
from sparse_matrix_tuning_amd.smt import ranking, smt_helper

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
SIZES = (0, 1, 2, 3, 15, 16, 17, 18, 31, 33, 64, 100, 256, 257, 896, 1000, 4096, 5120)


def _tie_arrays(seed: int):
    """Arrays with runs of equal values (few distinct levels, zeros, -0.0, inf, NaN)."""
    rng = np.random.default_rng(seed)
    for n in SIZES:
        for kind in range(5):
            if kind == 0:
                v = rng.integers(0, 4, n).astype(np.float32)
            elif kind == 1:
                v = (rng.integers(0, max(1, n // 3), n) / 7.0).astype(np.float32)
            elif kind == 2:
                v = rng.standard_normal(n).astype(np.float32)
                v[rng.integers(0, max(n, 1), n // 4)] = 0.0
            elif kind == 3:
                v = rng.choice(np.array([0.0, -0.0, 1.5, np.inf, -np.inf], np.float32), n)
            else:
                v = rng.integers(0, 3, n).astype(np.float32)
                v[rng.integers(0, max(n, 1), n // 6)] = np.nan
            yield v


def test_aten_argsort_matches_torch_cpu_argsort():
    checked = 0
    for seed in range(3):
        for v in _tie_arrays(seed):
            want = torch.argsort(torch.from_numpy(v.copy()), descending=True).numpy()
            got = ranking.aten_argsort_desc(v)
            assert np.array_equal(got, want), (v.size, v[:20])
            checked += 1
    assert checked == 3 * len(SIZES) * 5
    # sorted, presorted and reversed runs (the median-of-three pivot's easy and adversarial shapes)
    for n in (17, 100, 1000, 4097):
        for v in (np.arange(n, dtype=np.float32), np.arange(n, 0, -1, dtype=np.float32),
                  np.repeat(np.arange(n // 4 + 1, dtype=np.float32), 4)[:n],
                  np.tile(np.arange(5, dtype=np.float32), n // 5 + 1)[:n]):
            want = torch.argsort(torch.from_numpy(v.copy()), descending=True).numpy()
            assert np.array_equal(ranking.aten_argsort_desc(v), want), n


@pytest.fixture(scope="module")
def stdsort_probe(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("stdsort") / "stdsort_probe")
    subprocess.run([gxx, "-O2", "-o", exe, os.path.join(HERE, "stdsort_probe.cpp")], check=True)
    return exe


def _probe(exe: str, mode: str, v: np.ndarray) -> np.ndarray:
    text = f"{mode} {v.size}\n" + "\n".join(float(x).hex() if x == x else "nan" for x in v.tolist()) + "\n"
    out = subprocess.run([exe], input=text, capture_output=True, text=True, check=True).stdout.split()
    return np.asarray([int(t) for t in out], dtype=np.int64)


def test_aten_argsort_matches_libstdcxx_sort_and_heap_fallback(stdsort_probe):
    for v in _tie_arrays(7):
        assert np.array_equal(ranking.aten_argsort_desc(v), _probe(stdsort_probe, "sort", v)), v.size
        # the introsort's depth-limit fallback (std::partial_sort over the whole range)
        assert np.array_equal(ranking.aten_argsort_desc(v, heap_only=True), _probe(stdsort_probe, "partial", v)), v.size


def _exact_entry(key, vals):
    a = np.asarray(vals, np.float32)
    a64 = a.astype(np.float64)
    return ranking.KeyScores(key, a.shape, a, a64, a64, rescore=ranking.whole_key(lambda a=a: a))


def test_top_n_per_key_ties_follow_aten_on_exact_values():
    rng = np.random.default_rng(3)
    for n_blocks in (16, 17, 64, 896):
        vals = rng.integers(0, 5, n_blocks).astype(np.float32)
        for n in (1, 5, 17, n_blocks - 1, n_blocks + 3, -2):
            got = ranking.top_n_per_key([_exact_entry(("q_proj", 0), vals)], n)[0]
            want = torch.argsort(torch.from_numpy(vals), descending=True)[:n].tolist()
            assert got == want, (n_blocks, n)


def test_top_n_per_key_ties_decided_through_intervals():
    """GPU-style entries: inexact values in intervals, exact zeros (all-zero blocks) and a re-score
    that returns the reference's values. Equal values at the cut make the key exact and sorted the
    way ATen sorts; distinct values still take the interval path without a re-score."""
    rng = np.random.default_rng(11)
    exact = rng.integers(1, 4, 64).astype(np.float32) * np.float32(0.125)
    exact[rng.integers(0, 64, 20)] = 0.0
    calls = []

    def rescore(_flat):
        calls.append(1)
        return np.arange(exact.size), exact

    nominal = exact.copy()
    lo = exact.astype(np.float64) * (1 - 1e-6)
    hi = exact.astype(np.float64) * (1 + 1e-6)
    e = ranking.KeyScores(("gate_proj", 3), (8, 8), nominal, lo, hi, rescore=rescore)
    assert e.exact.sum() == (exact == 0).sum()               # only the zero blocks start exact
    got = ranking.top_n_per_key([e], 30)[0]
    assert got == torch.argsort(torch.from_numpy(exact), descending=True)[:30].tolist()
    assert ranking.LAST_REPORT["tie_sorted_keys"] == [("gate_proj", 3)] and calls
    # distinct values: no tie sort, the order is decided by the intervals alone
    distinct = np.linspace(1.0, 2.0, 64, dtype=np.float32)[rng.permutation(64)]
    d = ranking.KeyScores(("q_proj", 0), (8, 8), distinct, distinct * (1 - 1e-9), distinct * (1 + 1e-9),
                          rescore=lambda f: (_ for _ in ()).throw(AssertionError("no re-score expected")))
    assert ranking.top_n_per_key([d], 10)[0] == np.argsort(-distinct, kind="stable")[:10].tolist()
    assert ranking.LAST_REPORT["tie_sorted_keys"] == []


def test_norm_dist_tie_goldens_through_the_interval_path():
    """The product's GPU-path ranking on the CPU: the fp64 per-block sums smt_block_score computes
    (oracle.block_raw_fp64), ranking.block_intervals, and the product's host re-score."""
    from tests.golden.make_golden import tie_inputs
    spec = json.load(open(os.path.join(GOLDEN, "norm_dist_ties_expected.json")))
    grads = tie_inputs()
    dims = spec["dims"]
    for case in spec["cases"][::3]:
        st = case["strategy"]
        entries = []
        for key, g in grads.items():
            d1, d2 = dims[key[0]][0] // 256, dims[key[0]][1] // 256
            raw = ref.block_raw_fp64(g, d1, d2, st).numpy()
            nominal, lo, hi = ranking.block_intervals(raw, st)
            entries.append(ranking.KeyScores(key, (d1, d2), nominal, lo, hi,
                                             rescore=smt_helper.block_rescorer(g, d1, d2, st)))
        out = smt_helper._rank_block_entries(entries, case["n"], "norm_dist")
        assert [[k[0], k[1], [list(t) for t in v]] for k, v in out.items()] == case["expected"], (st, case["n"])


def test_norm_dist_tie_goldens_on_host():
    """The committed tie fixtures (oracle = the reference's unstable argsort on this host) through
    the product's host ranking on ATen's own statistics."""
    from tests.golden.make_golden import digest, tie_channel_inputs, tie_inputs
    spec = json.load(open(os.path.join(GOLDEN, "norm_dist_ties_expected.json")))
    grads = tie_inputs()
    assert digest(grads) == spec["inputs_sha256"], "seeded generator drifted: regenerate goldens"
    assert sum(c["index_order_differs"] for c in spec["cases"]) >= 10
    dims = spec["dims"]
    for case in spec["cases"]:
        scores = {k: ref.block_stat(g, dims[k[0]][0] // 256, dims[k[0]][1] // 256, case["strategy"]).numpy()
                  for k, g in grads.items()}
        out = smt_helper.rank_blocks(scores, case["n"], "norm_dist")
        assert [[k[0], k[1], [list(t) for t in v]] for k, v in out.items()] == case["expected"], case
        oracle_out = ref.select_submatrix(grads, dims, case["n"], selection_strategy="norm_dist",
                                          calculate_strategy=case["strategy"])
        assert [[k[0], k[1], [list(t) for t in v]] for k, v in oracle_out.items()] == case["expected"]
    act = tie_channel_inputs()
    assert digest(act) == spec["channel"]["inputs_sha256"]
    for case in spec["channel"]["cases"]:
        stats = {}
        for k, a in act.items():
            s = torch.sum(a.abs(), dim=0)                     # smt_helper.py:167-184 on ATen
            stats[k] = {"mean_abs": lambda: torch.mean(s.abs(), dim=0), "abs_mean": lambda: torch.abs(torch.mean(s, dim=0)),
                        "L1": lambda: torch.norm(s, p=1, dim=0), "L2": lambda: torch.norm(s, p=2, dim=0)}[case["strategy"]]().numpy()
        out = smt_helper.rank_channels(stats, case["n"], "norm_dist")
        assert [[k[0], k[1], list(v)] for k, v in out.items()] == case["expected"], case


def test_near_tie_channel_fixture_norm_dist_on_host():
    """The near-tie channel fixture holds an exact tie under norm_dist (two channels of one key with
    equal ATen means; ATen's sort puts the larger index first): the oracle's unstable argsort and
    the product's host ranking on ATen's statistics both give the committed order."""
    from tests.golden.make_golden import near_tie_channel_inputs
    spec = json.load(open(os.path.join(GOLDEN, "near_tie_expected.json")))["channel"]
    act = near_tie_channel_inputs()
    cases = [c for c in spec["cases"] if c["selection_strategy"] == "norm_dist"]
    assert cases
    for case in cases:
        out = ref.select_channel(act, case["n"], selection_strategy="norm_dist", calculate_strategy=case["strategy"])
        assert [[k[0], k[1], list(v)] for k, v in out.items()] == case["expected"], (case["strategy"], case["n"])
        if case["strategy"] in ("mean_abs", "abs_mean"):
            stats = {k: torch.mean(torch.sum(a.abs(), dim=0).abs(), dim=0).numpy() for k, a in act.items()}
            got = smt_helper.rank_channels(stats, case["n"], "norm_dist")
            assert [[k[0], k[1], list(v)] for k, v in got.items()] == case["expected"], (case["strategy"], case["n"])

"""Bit-identical top-n ranking of SMT block / channel scores (host logic).

The reference ranks the fp32 values of ATen's CPU reductions (``grad.reshape(d1,256,d2,256)``
reduced over dims (1, 3), smt_helper.py:67-78, 233-251; the channel statistic of
smt_helper.py:167-184) by the tuple ``(score, (key, i, j))`` (smt_helper.py:111-139) or, for
``norm_dist``, per key with ``argsort`` (smt_helper.py:81-100, 186-199). The GPU scan computes each
score's terms in fp64, which is within a few fp32 ulps of ATen's value but not always equal to it,
so two blocks a few ulps apart could swap.

Here every score is carried as an interval ``[lo, hi]`` that provably contains the reference's
fp32 value (bounds in :func:`block_intervals` / :func:`channel_intervals`), plus a nominal value
inside it (the fp64 value rounded once). The ranking only depends on comparisons, so it is the
reference's ranking as soon as every comparison it depends on is decided:

* membership: every block of the top ``n`` vs every block just below it;
* the tile order: blocks of the same key inside the top ``n`` (the order is the tile layout of
  LinearLayer_MatrixSparsity, smt.py:312-325);
* the dict order: the first block of each key (its position decides the key's insertion order).

A comparison is decided when both values are exact or the two intervals are disjoint. Every block
with an undecided comparison is re-scored together with its whole key, with the reference's own
expression on the host CPU (so ATen's per-output reduction order is the reference's); its interval
collapses to the exact value, and the check repeats until nothing is undecided. Typical runs re-score
a handful of keys; the report of the last call is kept in :data:`LAST_REPORT`.

An exact value outside its interval would mean the bound's assumption about ATen's reduction
(:data:`BLOCK_DEPTH`) does not hold on this host: the ranking then restarts with the
order-independent worst-case bound.
"""
from __future__ import annotations

import heapq
import time
from collections import defaultdict
from typing import Callable, Dict, Hashable, List, Optional, Sequence

import numpy as np

U32 = 2.0 ** -24                       # unit roundoff of fp32 (round to nearest)
BLOCK_ELEMS = 256 * 256
# ATen reduces each 256-element row of a block (one contiguous inner reduction, any tree: depth
# <= 255) and adds the 256 row results into the output one after another (depth <= 256), so every
# term passes through at most 511 fp32 additions; +2 for the square of L2 and the final rounding.
BLOCK_DEPTH = 514
# No assumption about the order at all: a chain through every term of the block.
BLOCK_DEPTH_WORST = BLOCK_ELEMS + 2

LAST_REPORT: dict = {}


def gamma(k: int) -> float:
    """Higham's gamma_k = k u / (1 - k u): relative bound of k fp32 roundings."""
    return k * U32 / (1.0 - k * U32)


class KeyScores:
    """Scores of one key (module, layer): nominal fp32 values and an interval around each that
    contains the reference's value, with a callable that computes exact reference values.

    ``rescore(flat_indices) -> (covered_flat_indices, fp32 values)`` returns the reference's values
    of at least the requested elements (a whole key, or the block rows holding them)."""

    __slots__ = ("key", "shape", "nominal", "lo", "hi", "exact", "_rescore", "_bounds")

    def __init__(self, key: Hashable, shape: tuple, nominal: np.ndarray, lo: np.ndarray, hi: np.ndarray,
                 rescore: Callable, bounds: Optional[Callable[[bool], tuple]] = None):
        self.key = key
        self.shape = tuple(shape)
        self.nominal = np.asarray(nominal, dtype=np.float32).reshape(-1)
        self.lo = np.asarray(lo, dtype=np.float64).reshape(-1)
        self.hi = np.asarray(hi, dtype=np.float64).reshape(-1)
        # an interval of width zero is an exact value (an all-zero block)
        self.exact = self.lo == self.hi
        self._rescore = rescore
        self._bounds = bounds

    @property
    def size(self) -> int:
        return self.nominal.size

    @property
    def all_exact(self) -> bool:
        return bool(self.exact.all())

    def make_exact(self, flat: Optional[np.ndarray] = None) -> bool:
        """Replace the estimates of (at least) ``flat`` (default: every element) by the reference's
        values; False if one fell outside its interval."""
        if flat is None:
            flat = np.arange(self.size)
        covered, vals = self._rescore(np.asarray(flat, dtype=np.int64))
        covered = np.asarray(covered, dtype=np.int64).reshape(-1)
        vals = np.asarray(vals, dtype=np.float32).reshape(-1)
        if vals.size != covered.size:
            raise RuntimeError(f"re-score of {self.key} returned {vals.size} values for {covered.size} elements")
        v64 = vals.astype(np.float64)
        finite = np.isfinite(v64)
        lo, hi = self.lo[covered], self.hi[covered]
        ok = bool(np.all((v64[finite] >= lo[finite]) & (v64[finite] <= hi[finite])))
        self.nominal[covered] = vals
        self.lo[covered] = v64
        self.hi[covered] = v64
        self.exact[covered] = True
        return ok

    def widen(self) -> None:
        """Switch the inexact elements to the order-independent bound."""
        if not self.all_exact and self._bounds is not None:
            lo, hi = self._bounds(True)
            keep = ~self.exact
            self.lo[keep] = np.asarray(lo, dtype=np.float64).reshape(-1)[keep]
            self.hi[keep] = np.asarray(hi, dtype=np.float64).reshape(-1)[keep]


def whole_key(values_fn: Callable[[], np.ndarray]) -> Callable:
    """A ``rescore`` that computes every element of the key at once."""
    def rescore(_flat):
        vals = np.asarray(values_fn(), dtype=np.float32).reshape(-1)
        return np.arange(vals.size), vals
    return rescore


# ------------------------------------------------------------------------------------------------
# intervals
# ------------------------------------------------------------------------------------------------
def _pad(lo: np.ndarray, hi: np.ndarray) -> tuple:
    """Cover the final fp32 rounding(s) of the statistic (division, sqrt): 4 ulps, plus the
    smallest subnormal for results that underflow."""
    return lo * (1.0 - 4 * U32) - 1.5e-45, hi * (1.0 + 4 * U32) + 1.5e-45


def block_intervals(raw: np.ndarray, strategy: str, worst_case: bool = False) -> tuple:
    """``raw``: fp64 ``[n, 2]`` per block (sum of terms, sum of |terms|) from ``smt_block_score``.
    Returns ``(nominal fp32, lo, hi)`` with lo <= reference fp32 value <= hi."""
    raw = np.asarray(raw, dtype=np.float64).reshape(-1, 2)
    s, m = raw[:, 0], raw[:, 1]
    n = float(BLOCK_ELEMS)
    depth = BLOCK_DEPTH_WORST if worst_case else BLOCK_DEPTH
    # ATen's fp32 sum of the same terms: |err| <= gamma_depth * sum|terms|; the fp64 sum itself is
    # off by at most 65536 * 2^-53 * sum|terms| (< 1e-11)
    err = (gamma(depth) + 1e-11) * m
    if strategy == "mean_abs":
        a = np.abs(s)
        lo, hi = np.maximum(a - err, 0.0) / n, (a + err) / n
        nominal = np.abs((s / n).astype(np.float32))
    elif strategy == "abs_mean":
        lo, hi = np.maximum(s - err, 0.0) / n, (s + err) / n
        nominal = (s / n).astype(np.float32)
    elif strategy == "L1":
        lo, hi = np.maximum(s - err, 0.0), s + err
        nominal = s.astype(np.float32)
    elif strategy == "L2":
        lo, hi = np.sqrt(np.maximum(s - err, 0.0)), np.sqrt(s + err)
        nominal = np.sqrt(s).astype(np.float32)
    else:
        raise ValueError(strategy)
    lo, hi = _pad(lo, hi)
    zero = m == 0.0                      # every term zero: the reference's value is exactly 0
    lo[zero] = 0.0
    hi[zero] = 0.0
    return nominal, lo, hi


def channel_depth(batch: int, seq: int) -> int:
    """fp32 roundings on the way from the accumulated [B, S, in] activations to the reference's
    channel statistic: the batch sum (B-1), the sequence reduction (S-1), the square of L2 (which
    doubles the batch sum's relative error), the division / sqrt; all terms are non-negative, so
    the bound is relative."""
    return 2 * batch + seq + 6


def channel_intervals(raw: np.ndarray, batch: int, seq: int, strategy: str, worst_case: bool = False) -> tuple:
    """``raw``: fp64 per-channel sums from ``smt_channel_score`` (sum_s A_s, or sum_s A_s^2 for L2).
    Returns ``(nominal fp32, lo, hi)``."""
    raw = np.asarray(raw, dtype=np.float64).reshape(-1)
    depth = channel_depth(batch, seq) if not worst_case else 2 * batch * seq + 6
    g = gamma(depth) + 1e-12
    if strategy in ("mean_abs", "abs_mean"):
        v = raw / float(seq)
        nominal = np.abs(v).astype(np.float32)
    elif strategy == "L1":
        v = raw
        nominal = raw.astype(np.float32)
    elif strategy == "L2":
        v = np.sqrt(raw)
        nominal = v.astype(np.float32)
    else:
        raise ValueError(strategy)
    lo, hi = _pad(v * (1.0 - g), v * (1.0 + g))
    zero = raw == 0.0
    lo[zero] = 0.0
    hi[zero] = 0.0
    return nominal, lo, hi


# ------------------------------------------------------------------------------------------------
# deciding the comparisons
# ------------------------------------------------------------------------------------------------
def _overlaps_in_order(pos: np.ndarray, lo: np.ndarray, hi: np.ndarray) -> np.ndarray:
    """``pos``: element ids sorted by descending value. For i before j the two intervals overlap
    iff hi[j] >= lo[i] (both contain their nominal values). Returns, per position, whether the
    element overlaps any other element of ``pos``."""
    k = pos.size
    if k < 2:
        return np.zeros(k, dtype=bool)
    l, h = lo[pos], hi[pos]
    suffix_max_hi = np.maximum.accumulate(h[::-1])[::-1]          # max over positions >= i
    prefix_min_lo = np.minimum.accumulate(l)                       # min over positions <= i
    later = np.empty(k, dtype=bool)
    later[:-1] = suffix_max_hi[1:] >= l[:-1]
    later[-1] = False
    earlier = np.empty(k, dtype=bool)
    earlier[0] = False
    earlier[1:] = prefix_min_lo[:-1] <= h[1:]
    return later | earlier


class _Flat:
    """All keys' scores as flat arrays (element id = position in the concatenation)."""

    def __init__(self, entries: Sequence[KeyScores]):
        self.owner = np.concatenate([np.full(e.size, i, dtype=np.int64) for i, e in enumerate(entries)])
        self.flat = np.concatenate([np.arange(e.size, dtype=np.int64) for e in entries])
        self.val = np.concatenate([e.nominal.astype(np.float64) for e in entries])
        self.lo = np.concatenate([e.lo for e in entries])
        self.hi = np.concatenate([e.hi for e in entries])
        self.exact = np.concatenate([e.exact for e in entries])


def _key_ranks(entries: Sequence[KeyScores]) -> np.ndarray:
    """Rank of each key under Python's tuple ordering (the heap compares the keys themselves)."""
    order = sorted(range(len(entries)), key=lambda i: entries[i].key)
    rank = np.empty(len(entries), dtype=np.int64)
    r = -1
    prev = object()
    for i in order:
        if r < 0 or entries[i].key != prev:
            r += 1
            prev = entries[i].key
        rank[i] = r
    return rank


def _rescore(entries: Sequence[KeyScores], owners: np.ndarray, flats: np.ndarray, report: dict) -> bool:
    ok = True
    for o in np.unique(owners):
        e = entries[int(o)]
        want = flats[owners == o]
        want = want[~e.exact[want]]
        if not want.size:
            continue
        before = int(e.exact.sum())
        ok &= e.make_exact(want)
        report["rescored_keys"].append(e.key)
        report["rescored_elements"] += int(e.exact.sum()) - before
    return ok


def _new_report(kind: str, n: int, entries: Sequence[KeyScores]) -> dict:
    return {"kind": kind, "n": n, "keys": len(entries), "candidates": int(sum(e.size for e in entries)),
            "flagged": 0, "rescored_keys": [], "rescored_elements": 0, "iterations": 0, "worst_case_bound": False,
            "seconds": 0.0}


def _restart_worst_case(entries: Sequence[KeyScores], report: dict) -> None:
    report["worst_case_bound"] = True
    for e in entries:
        e.widen()


def top_n(entries: Sequence[KeyScores], n: int) -> List[tuple]:
    """The first ``n`` of all ``(score, (key, flat index))`` tuples in descending order, as the
    reference's heap + sort produce them (smt_helper.py:111-139), as ``[(entry index, flat index)]``."""
    t0 = time.perf_counter()
    report = _new_report("no_restriction", n, entries)
    rank = _key_ranks(entries)
    result = None
    for _ in range(sum(e.size for e in entries) + 2):
        report["iterations"] += 1
        F = _Flat(entries)
        if not np.all(np.isfinite(F.val)):
            result = _literal_heap(entries, n, report)
            break
        # descending tuple order: value, then key, then flat index
        order = np.lexsort((F.flat, rank[F.owner], F.val))[::-1]
        top, rest = order[:n], order[n:]
        undecided = np.zeros(F.val.size, dtype=bool)
        if rest.size and top.size:
            near = rest[F.hi[rest] >= F.lo[top].min()]
            if near.size:
                undecided[near] = True
                undecided[top[F.lo[top] <= F.hi[near].max()]] = True
        for o in np.unique(F.owner[top]):                      # tile order inside each key
            pos = top[F.owner[top] == o]
            undecided[pos[_overlaps_in_order(pos, F.lo, F.hi)]] = True
        _, first_at = np.unique(F.owner[top], return_index=True)   # key order: first block of each key
        firsts = top[np.sort(first_at)]
        undecided[firsts[_overlaps_in_order(firsts, F.lo, F.hi)]] = True
        undecided &= ~F.exact
        if not undecided.any():
            result = [(int(F.owner[i]), int(F.flat[i])) for i in top]
            break
        report["flagged"] += int(undecided.sum())
        if not _rescore(entries, F.owner[undecided], F.flat[undecided], report):
            _restart_worst_case(entries, report)
    if result is None:                     # cannot happen: every round makes at least one key exact
        raise RuntimeError("SMT ranking did not converge")
    report["seconds"] = time.perf_counter() - t0
    LAST_REPORT.clear()
    LAST_REPORT.update(report)
    return result


# ------------------------------------------------------------------------------------------------
# ATen's CPU argsort(descending=True), ties included
# ------------------------------------------------------------------------------------------------
# The reference's norm_dist ranks with torch.argsort(v, descending=True) on CPU tensors (the
# harvests are .cpu(), fine_tune.py:733, 657; smt_helper.py:86, 191). With stable=False, ATen's CPU
# sort kernel (aten/src/ATen/native/cpu/SortingKernel.cpp, torch 2.x) runs std::sort over
# (value, index) pairs with KeyValueCompDesc: lhs before rhs iff lhs is NaN and rhs is not, or
# lhs > rhs. std::sort is libstdc++'s introsort (bits/stl_algo.h): median-of-three pivot moved to
# the front, unguarded Hoare partition, recursion on the right part, heap sort past 2*floor(log2 n)
# levels, then one insertion sort over the 16-element runs. That algorithm is deterministic, so
# equal values come out in one definite order, which is restated below and pinned against this
# host's torch.argsort and a g++ std::sort / std::partial_sort (tests/test_aten_argsort.py).
_S_THRESHOLD = 16


def _before(a, b) -> bool:
    x, y = a[0], b[0]
    return (x != x and y == y) or x > y


def _unguarded_linear_insert(a: list, last: int) -> None:
    val = a[last]
    nxt = last - 1
    while _before(val, a[nxt]):
        a[last] = a[nxt]
        last = nxt
        nxt -= 1
    a[last] = val


def _insertion_sort(a: list, first: int, last: int) -> None:
    for i in range(first + 1, last):
        if _before(a[i], a[first]):
            val = a[i]
            a[first + 1:i + 1] = a[first:i]
            a[first] = val
        else:
            _unguarded_linear_insert(a, i)


def _push_heap(a: list, first: int, hole: int, top: int, value) -> None:
    while hole > top:
        parent = (hole - 1) // 2
        if not _before(a[first + parent], value):
            break
        a[first + hole] = a[first + parent]
        hole = parent
    a[first + hole] = value


def _adjust_heap(a: list, first: int, hole: int, length: int, value) -> None:
    top = second = hole
    while second < (length - 1) // 2:
        second = 2 * (second + 1)
        if _before(a[first + second], a[first + second - 1]):
            second -= 1
        a[first + hole] = a[first + second]
        hole = second
    if (length & 1) == 0 and second == (length - 2) // 2:
        second = 2 * (second + 1)
        a[first + hole] = a[first + second - 1]
        hole = second - 1
    _push_heap(a, first, hole, top, value)


def _pop_heap(a: list, first: int, last: int, result: int) -> None:
    value = a[result]
    a[result] = a[first]
    _adjust_heap(a, first, 0, last - first, value)


def _partial_sort(a: list, first: int, middle: int, last: int) -> None:
    length = middle - first
    if length >= 2:                                      # make_heap
        parent = (length - 2) // 2
        while True:
            _adjust_heap(a, first, parent, length, a[first + parent])
            if parent == 0:
                break
            parent -= 1
    for i in range(middle, last):                        # heap_select
        if _before(a[i], a[first]):
            _pop_heap(a, first, middle, i)
    while middle - first > 1:                            # sort_heap
        middle -= 1
        _pop_heap(a, first, middle, middle)


def _move_median_to_first(a: list, result: int, x: int, y: int, z: int) -> None:
    if _before(a[x], a[y]):
        if _before(a[y], a[z]):
            m = y
        elif _before(a[x], a[z]):
            m = z
        else:
            m = x
    elif _before(a[x], a[z]):
        m = x
    elif _before(a[y], a[z]):
        m = z
    else:
        m = y
    a[result], a[m] = a[m], a[result]


def _introsort_loop(a: list, first: int, last: int, depth: int) -> None:
    while last - first > _S_THRESHOLD:
        if depth == 0:
            _partial_sort(a, first, last, last)
            return
        depth -= 1
        _move_median_to_first(a, first, first + 1, first + (last - first) // 2, last - 1)
        lo, hi = first + 1, last                         # unguarded partition around a[first]
        while True:
            while _before(a[lo], a[first]):
                lo += 1
            hi -= 1
            while _before(a[first], a[hi]):
                hi -= 1
            if not lo < hi:
                break
            a[lo], a[hi] = a[hi], a[lo]
            lo += 1
        _introsort_loop(a, lo, last, depth)
        last = lo


def aten_argsort_desc(values, heap_only: bool = False) -> np.ndarray:
    """``torch.argsort(torch.tensor(values, dtype=float32), descending=True)`` as ATen's CPU kernel
    computes it (std::sort, see above), equal values included. ``heap_only``: std::partial_sort over
    the whole range instead (the introsort's depth-limit fallback, for the tests)."""
    a = [(v, i) for i, v in enumerate(np.asarray(values, dtype=np.float32).reshape(-1).tolist())]
    n = len(a)
    if heap_only:
        _partial_sort(a, 0, n, n)
    elif n > 1:
        _introsort_loop(a, 0, n, 2 * (n.bit_length() - 1))
        if n > _S_THRESHOLD:
            _insertion_sort(a, 0, _S_THRESHOLD)
            for i in range(_S_THRESHOLD, n):
                _unguarded_linear_insert(a, i)
        else:
            _insertion_sort(a, 0, n)
    return np.fromiter((i for _v, i in a), dtype=np.int64, count=n)


def _ties_decide(e: KeyScores, top: np.ndarray, rest: np.ndarray) -> bool:
    """Do two EXACT values, one of them in ``top``, compare equal? Then ``order[:n]`` depends on the
    sort's tie order. A tie that involves an inexact value shows as overlapping intervals instead,
    which the caller re-scores; once everything it depends on is decided, no such tie is left."""
    t = top[e.exact[top]]
    if not t.size:
        return False
    v = e.nominal[t]
    if np.unique(v).size < v.size:
        return True
    r = rest[e.exact[rest]]
    return bool(r.size and np.isin(e.nominal[r], v).any())


def top_n_per_key(entries: Sequence[KeyScores], n: int) -> List[List[int]]:
    """``norm_dist``: per key ``torch.argsort(values, descending=True)[:n]`` (smt_helper.py:86-94,
    191-195): the order is decided from the intervals; where equal values make the result depend on
    the sort's tie order, the key is re-scored exactly and ATen's CPU sort restated
    (:func:`aten_argsort_desc`) gives it."""
    t0 = time.perf_counter()
    report = _new_report("norm_dist", n, entries)
    report["tie_sorted_keys"] = []
    out = []
    for e in entries:
        for _ in range(e.size + 3):
            report["iterations"] += 1
            val = e.nominal.astype(np.float64)
            idx = np.arange(e.size)
            if not np.all(np.isfinite(val)):
                if not e.all_exact:
                    e.make_exact()
                    report["rescored_keys"].append(e.key)
                    continue
                order = aten_argsort_desc(e.nominal)
                out.append([int(i) for i in order[:n]])
                break
            order = np.lexsort((idx, -val))
            top, rest = order[:n], order[n:]        # Python slicing, as indices[:n] of smt_helper.py:93
            if _ties_decide(e, top, rest):
                # equal values at stake: ATen's std::sort order over the key's exact values
                if not e.all_exact:
                    before = int(e.exact.sum())
                    e.make_exact()
                    report["rescored_keys"].append(e.key)
                    report["rescored_elements"] += int(e.exact.sum()) - before
                report["tie_sorted_keys"].append(e.key)
                out.append([int(i) for i in aten_argsort_desc(e.nominal)[:n]])
                break
            if e.all_exact or not top.size:
                out.append([int(i) for i in top])
                break
            undecided = np.zeros(e.size, dtype=bool)
            if rest.size:
                near = rest[e.hi[rest] >= e.lo[top].min()]
                if near.size:
                    undecided[near] = True
                    undecided[top[e.lo[top] <= e.hi[near].max()]] = True
            undecided[top[_overlaps_in_order(top, e.lo, e.hi)]] = True
            undecided &= ~e.exact
            if not undecided.any():
                out.append([int(i) for i in top])
                break
            report["flagged"] += int(undecided.sum())
            before = int(e.exact.sum())
            if not e.make_exact(np.nonzero(undecided)[0]):
                report["worst_case_bound"] = True
                e.widen()
            report["rescored_keys"].append(e.key)
            report["rescored_elements"] += int(e.exact.sum()) - before
        else:
            raise RuntimeError("SMT per-key ranking did not converge")
    report["seconds"] = time.perf_counter() - t0
    LAST_REPORT.clear()
    LAST_REPORT.update(report)
    return out


def _literal_heap(entries: Sequence[KeyScores], n: int, report: dict) -> List[tuple]:
    """Non-finite scores (a diverged warm-up): NaN breaks the total order the fast path relies on,
    so every key is re-scored and the reference's heap loop (smt_helper.py:111-119) runs as written."""
    for i, e in enumerate(entries):
        if not e.all_exact:
            e.make_exact()
            report["rescored_keys"].append(e.key)
    report["literal_heap"] = True
    heap: list = []
    for o, e in enumerate(entries):
        for f in range(e.size):
            item = (float(e.nominal[f]), (e.key, f, o))
            if len(heap) < n:
                heapq.heappush(heap, item)
            else:
                heapq.heappushpop(heap, item)
    heap.sort(reverse=True)
    return [(o, f) for _v, (_k, f, o) in heap]


def group(entries: Sequence[KeyScores], picks: List[tuple], to_index: Callable[[KeyScores, int], object]) -> defaultdict:
    """``[(entry, flat)]`` in order -> ``defaultdict(list)`` keyed as the reference (smt_helper.py:135-139)."""
    out = defaultdict(list)
    for o, f in picks:
        out[entries[o].key].append(to_index(entries[o], f))
    return out

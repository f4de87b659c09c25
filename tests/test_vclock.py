"""partisan_vclock: dense-lane kernels (csrc/vclock.hip) vs the oracle
(oracle/vclock.c, pinned by the eunit KATs of src/partisan_vclock.erl:206-257).

CPU part: the dense encoding itself (absent = 0, counter c = c + 1) is
checked against the oracle with a numpy statement of the lane ops, so the
encoding is validated without a GPU.  GPU part: the kernels through the C ABI.
"""
import json
import os

import numpy as np
import pytest

import pyoracle as O
from partisan_amd.vclock import LANES, to_dense, to_sparse

ACTORS = list(range(100, 100 + LANES))


def random_clock(rng, p_present=0.3, zero_p=0.2):
    clk = []
    for a in ACTORS:
        if rng.random() < p_present:
            c = 0 if rng.random() < zero_p else int(rng.integers(1, 50))
            clk.append([a, c])
    rng.shuffle(clk)        # reference clocks are unordered lists (increment prepends)
    return clk


def related(rng, base):
    """a clock near `base` so that descends/dominates are often true."""
    out = [[a, max(0, c + int(rng.integers(-1, 2)))] for a, c in base if rng.random() < 0.95]
    if rng.random() < 0.3:
        out.append([ACTORS[int(rng.integers(LANES))], int(rng.integers(0, 5))])
    seen = set()
    uniq = []
    for a, c in out:
        if a not in seen:
            seen.add(a)
            uniq.append([a, c])
    return uniq


def pairs(n, seed):
    rng = np.random.default_rng(seed)
    A, B = [], []
    for i in range(n):
        a = random_clock(rng)
        b = related(rng, a) if i % 2 else random_clock(rng)
        if i % 7 == 0:
            b = []
        if i % 11 == 0:
            a = []
        A.append(a)
        B.append(b)
    return A, B


# numpy statement of the lane ops (test-side model of the kernels)
def np_descends(a, b):
    return (a >= b).all(axis=1)


def np_merge(a, b):
    return np.maximum(a, b)


def sorted_clock(c):
    return sorted([list(x) for x in c])


def test_dense_encoding_matches_oracle():
    A, B = pairs(600, 1)
    da, db = to_dense(A, ACTORS), to_dense(B, ACTORS)
    d = np_descends(da, db)
    dom = d & ~np_descends(db, da)
    m = np_merge(da, db)
    for i in range(len(A)):
        assert d[i] == O.vc_descends(A[i], B[i]), (A[i], B[i])
        assert dom[i] == O.vc_dominates(A[i], B[i])
        assert sorted_clock(to_sparse(m[i:i + 1], ACTORS)[0]) == sorted_clock(O.vc_merge([A[i], B[i]]))


def np_glb(a, b):
    return np.minimum(a, b)


def np_subtract_dots(d, c):
    return np.where(d > np.maximum(c, 1), d, 0).astype(np.uint32)


def np_get_counter(a, act):
    x = a[np.arange(len(a)), act].astype(np.int64)
    return np.where(x > 0, x - 1, 0)


def test_dense_encoding_rest_matches_oracle():
    """glb/2, subtract_dots/2, get_counter/2 and equal/2 as lane ops (the
    kernels' statement) against the oracle's list restatement."""
    A, B = pairs(600, 4)
    da, db = to_dense(A, ACTORS), to_dense(B, ACTORS)
    g = np_glb(da, db)
    sd = np_subtract_dots(da, db)
    eq = (da == db).all(axis=1)
    rng = np.random.default_rng(5)
    act = rng.integers(0, LANES, len(A))
    gc = np_get_counter(da, act)
    for i in range(len(A)):
        assert to_sparse(g[i:i + 1], ACTORS)[0] == O.vc_glb(A[i], B[i]), i
        assert to_sparse(sd[i:i + 1], ACTORS)[0] == O.vc_subtract_dots(A[i], B[i]), i
        assert eq[i] == O.vc_equal(A[i], B[i]), i
        assert gc[i] == O.vc_get_counter(ACTORS[act[i]], A[i]), i
    # equal/2 compares sorted lists: a permuted clock is equal
    assert O.vc_equal([[101, 2], [100, 1]], [[100, 1], [101, 2]])


# the example in subtract_dots/2's doc comment (src/partisan_vclock.erl:81-83):
# [{a,3},{b,2},{d,14},{g,22}] minus [{a,4},{b,1},{c,1},{d,14},{e,5},{f,2}] = [{b,2},{g,22}]
SUBTRACT_DOC = ([[1, 3], [2, 2], [4, 14], [7, 22]], [[1, 4], [2, 1], [3, 1], [4, 14], [5, 5], [6, 2]],
                [[2, 2], [7, 22]])


def test_subtract_dots_doc_example():
    dots, clock, want = SUBTRACT_DOC
    assert O.vc_subtract_dots(dots, clock) == want
    actors = list(range(1, 8))
    d = np_subtract_dots(to_dense([dots], actors), to_dense([clock], actors))
    assert to_sparse(d, actors)[0] == want


def test_dense_encoding_kats(golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "vclock_kat.json")))
    actors = list(range(1, 8))
    for c in kat["merge"]:
        if len(c["in"]) != 2:
            continue
        da, db = to_dense([c["in"][0]], actors), to_dense([c["in"][1]], actors)
        assert to_sparse(np_merge(da, db), actors)[0] == c["out"]


@pytest.fixture(scope="module")
def ops():
    import partisan_amd as pa
    from partisan_amd.vclock import VClockOps
    sim = pa.Simulator()
    yield VClockOps(sim)
    sim.close()


@pytest.mark.gpu
def test_kernels_match_oracle(ops):
    A, B = pairs(5000, 2)
    da, db = to_dense(A, ACTORS), to_dense(B, ACTORS)
    d = ops.descends(da, db)
    dom = ops.dominates(da, db)
    m = ops.merge(da, db)
    rng = np.random.default_rng(3)
    act = rng.integers(0, LANES, len(A)).astype(np.uint32)
    inc = ops.increment(da, act)
    for i in range(len(A)):
        assert d[i] == O.vc_descends(A[i], B[i]), i
        assert dom[i] == O.vc_dominates(A[i], B[i]), i
        assert sorted_clock(to_sparse(m[i:i + 1], ACTORS)[0]) == sorted_clock(O.vc_merge([A[i], B[i]])), i
        want = O.vc_increment(ACTORS[act[i]], A[i])
        assert sorted_clock(to_sparse(inc[i:i + 1], ACTORS)[0]) == sorted_clock(want), i


@pytest.mark.gpu
def test_kernel_kats(ops, golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "vclock_kat.json")))
    actors = list(range(1, 8)) + list(range(100, 157))
    for c in kat["merge"]:
        if len(c["in"]) != 2:
            continue
        da, db = to_dense([c["in"][0]], actors), to_dense([c["in"][1]], actors)
        assert to_sparse(ops.merge(da, db), actors)[0] == c["out"]
    # example_test (:212-227) through the kernels; actors a=1, b=2, c=3
    z = np.zeros((1, LANES), np.uint32)
    lane = {1: 0, 2: 1, 3: 2}
    A1 = ops.increment(z, [lane[1]])
    B1 = ops.increment(z, [lane[2]])
    assert ops.descends(A1, z)[0] and ops.descends(B1, z)[0]
    assert not ops.descends(A1, B1)[0]
    A2 = ops.increment(A1, [lane[1]])
    Cc = ops.merge(A2, B1)
    C1 = ops.increment(Cc, [lane[3]])
    assert ops.descends(C1, A2)[0] and ops.descends(C1, B1)[0]
    assert not ops.descends(B1, C1)[0] and not ops.descends(B1, A1)[0]


@pytest.mark.gpu
def test_large_batch_properties(ops):
    rng = np.random.default_rng(9)
    n = 1 << 20
    a = rng.integers(0, 40, (n, LANES), dtype=np.uint32)
    b = rng.integers(0, 40, (n, LANES), dtype=np.uint32)
    m = ops.merge(a, b)
    assert np.array_equal(m, np.maximum(a, b))
    assert ops.descends(m, a).all() and ops.descends(m, b).all()
    assert np.array_equal(ops.descends(a, b), (a >= b).all(axis=1))


@pytest.mark.gpu
def test_kernels_rest_match_oracle(ops):
    """Device glb / subtract_dots / get_counter / equal against the oracle,
    plus the accessor KAT (src/partisan_vclock.erl:212-220) and the
    subtract_dots doc example."""
    A, B = pairs(5000, 6)
    A += [[[100, 3], [101, 1]], [[100, 0]]]
    B += [[[101, 1], [100, 3]], [[100, 0]]]      # permuted equal; zero counters equal
    da, db = to_dense(A, ACTORS), to_dense(B, ACTORS)
    g = ops.glb(da, db)
    sd = ops.subtract_dots(da, db)
    eq = ops.equal(da, db)
    rng = np.random.default_rng(7)
    act = rng.integers(0, LANES, len(A)).astype(np.uint32)
    gc = ops.get_counter(da, act)
    for i in range(len(A)):
        assert to_sparse(g[i:i + 1], ACTORS)[0] == O.vc_glb(A[i], B[i]), i
        assert to_sparse(sd[i:i + 1], ACTORS)[0] == O.vc_subtract_dots(A[i], B[i]), i
        assert bool(eq[i]) == O.vc_equal(A[i], B[i]), i
        assert int(gc[i]) == O.vc_get_counter(ACTORS[act[i]], A[i]), i
    assert eq[-1] and eq[-2]
    actors = list(range(1, 8))
    dots, clock, want = SUBTRACT_DOC
    assert to_sparse(ops.subtract_dots(to_dense([dots], actors), to_dense([clock], actors)), actors)[0] == want


@pytest.mark.gpu
def test_accessor_kat_on_device(ops, golden_dir):
    kat = json.load(open(os.path.join(golden_dir, "vclock_kat.json")))["accessor"]
    actors = list(range(1, 8))
    clk = to_dense([kat["clock"]] * len(kat["get_counter"]), actors)
    act = np.array([actors.index(a) for a, _ in kat["get_counter"]], np.uint32)
    got = ops.get_counter(clk, act)
    assert got.tolist() == [c for _, c in kat["get_counter"]]

"""The oracle against the reference's own eunit known-answer tests.

Fixtures: tests/golden/*_kat.json, transcribed from
  src/partisan_interval_sets.erl:849-1019, src/partisan_vclock.erl:206-257,
  src/partisan_plumtree_util.erl:102-261 (script: tests/golden/transcribe_eunit.py).
"""
import json
import os

import pytest

import pyoracle as O


def load(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


# ----------------------------------------------------------- interval sets
@pytest.fixture(scope="module")
def iset(golden_dir):
    return load(golden_dir, "interval_sets_kat.json")


def test_from_list(iset):
    for c in iset["from_list"]:
        assert O.iset_from_list(c["in"]) == c["out"]


def test_seq(iset):
    for c in iset["seq"]:
        assert O.iset_seq(c["in"]) == c["out"]


def test_is_type(iset):
    for c in iset["is_type"]:
        assert O.iset_is_type(c["in"]) is c["out"]


def test_is_element(iset):
    for c in iset["is_element"]:
        assert O.iset_is_element(c["el"], c["set"]) is c["out"], c


def test_flat_size_min_max(iset):
    for c in iset["flat_size"]:
        assert O.iset_flat_size(c["in"]) == c["out"]
    for c in iset["min"]:
        assert O.iset_min(c["in"]) == c["out"]
    for c in iset["max"]:
        assert O.iset_max(c["in"]) == c["out"]


def test_element_precedes_meets(iset):
    for c in iset["element_precedes"]:
        assert O.iset_element_precedes(c["a"], c["b"]) is c["out"], c
    for c in iset["element_meets"]:
        assert O.iset_element_meets(c["a"], c["b"]) is c["out"], c


def test_element_subtract(iset):
    for c in iset["element_subtract"]:
        assert O.iset_element_subtract(c["a"], c["b"]) == c["out"], c


def _ordset_union(a, b):
    return sorted(set(a) | set(b))


def test_add_element(iset):
    for c in iset["add_element"]:
        got = O.iset_add_element(c["el"], c["set"])
        assert got == c["out"], c
        # the second assertion of each eunit case
        assert _ordset_union(O.iset_seq([c["el"]]), O.iset_seq(c["set"])) == O.iset_seq(got)


def test_del_element(iset):
    for c in iset["del_element"]:
        got = O.iset_del_element(c["el"], c["set"])
        assert got == c["out"], c
        assert sorted(set(O.iset_seq(c["set"])) - set(O.iset_seq([c["el"]]))) == O.iset_seq(got)


def test_del_element_overlap_with_tail_is_badarg():
    # faithful quirk: del_element/2 recurses with a LIST remainder (App. A)
    with pytest.raises(ValueError):
        O.iset_del_element([3, 5], [[0, 8], [10, 12]])


def test_heartbeat_dedup_sequence():
    # the backend's use: from_list([M]) then add_element(M', ISet), in order
    s = O.iset_from_list([1])
    for m in range(2, 40):
        s = O.iset_add_element(m, s)
    assert s == [[1, 39]]
    assert O.iset_is_element(17, s) and not O.iset_is_element(40, s)
    s = O.iset_add_element(45, s)
    assert s == [[1, 39], 45]
    assert not O.iset_is_element(42, s)


# ----------------------------------------------------------- vclock
@pytest.fixture(scope="module")
def vc(golden_dir):
    return load(golden_dir, "vclock_kat.json")


def test_vclock_example(vc):
    env = {}
    for op in vc["example"]:
        if op[0] == "fresh":
            env[op[1]] = []
        elif op[0] == "increment":
            env[op[1]] = O.vc_increment(op[2], env[op[3]])
        elif op[0] == "merge":
            env[op[1]] = O.vc_merge([env[x] for x in op[2]])
        elif op[0] == "assert_descends":
            assert O.vc_descends(env[op[2]], env[op[3]]) is op[1], op


def test_vclock_accessor(vc):
    a = vc["accessor"]
    for actor, expect in a["get_counter"]:
        assert O.vc_get_counter(actor, a["clock"]) == expect
    assert O.vc_all_nodes(a["clock"]) == a["all_nodes"]


def test_vclock_merge(vc):
    for c in vc["merge"]:
        assert O.vc_merge(c["in"]) == c["out"]


def test_vclock_quirks():
    # Q22: an actor of B absent from A fails descends even with counter 0
    assert not O.vc_descends([[1, 5]], [[2, 0]])
    assert O.vc_descends([[1, 5], [2, 0]], [[2, 0]])
    # Q23: merge of one clock is returned unsorted; increment prepends
    assert O.vc_merge([[[3, 1], [1, 1]]]) == [[3, 1], [1, 1]]
    assert O.vc_increment(2, [[1, 1], [2, 4]]) == [[2, 5], [1, 1]]
    assert O.vc_equal([[2, 5], [1, 1]], [[1, 1], [2, 5]])
    # dominates = descends and not descends back
    assert O.vc_dominates([[1, 2]], [[1, 1]]) and not O.vc_dominates([[1, 1]], [[1, 1]])


# ----------------------------------------------------------- build_tree
def test_build_tree(golden_dir):
    for c in load(golden_dir, "build_tree_kat.json")["cases"]:
        assert O.build_tree(c["arity"], c["nodes"], c["cycles"]) == c["out"], c

"""Writes the reference's eunit known-answer tests as JSON fixtures.

The vectors below are DATA transcribed by hand from the reference's eunit
blocks (inputs and expected outputs only; no reference code is copied):

  * src/partisan_interval_sets.erl:849-1019   -> interval_sets_kat.json
  * src/partisan_vclock.erl:206-257            -> vclock_kat.json
  * src/partisan_plumtree_util.erl:102-261     -> build_tree_kat.json
  * test/partisan_SUITE.erl:500-586 (causal_test scenario) -> causal_kat.json
  * src/partisan_membership_set.erl:269-522   -> membership_set_kat.json

Term encoding: an interval-set element N is the JSON int N and {H, T} is the
list [H, T].  vclock actors are mapped to integers preserving Erlang term
order (a<b<c ; <<"1">> < <<"2">> < ... < <<"7">>).  build_tree nodes
node1..node8 are the integers 1..8 (atom order == integer order for <= 9).

Run:  python tests/golden/transcribe_eunit.py   (rewrites the JSON files)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

IV = lambda a, b: [a, b]  # noqa: E731  interval term {A, B}
EXP = [IV(1, 2), 4, IV(6, 10)]

interval_sets = {
    "source": "src/partisan_interval_sets.erl:849-1019",
    # from_list_test_ (:852-860)
    "from_list": [
        {"in": [1, 2, 4, 6, 7, 8, 9, 10], "out": EXP},
        {"in": [IV(1, 2), 4, 6, 7, 8, 9, 10], "out": EXP},
        {"in": [IV(1, 2), 4, IV(6, 7), 8, 9, 10], "out": EXP},
        {"in": [IV(1, 2), 4, IV(6, 7), 8, IV(9, 10)], "out": EXP},
        {"in": EXP, "out": EXP},
    ],
    # seq_test_ (:863-870)
    "seq": [
        {"in": [1, 2, 4, 6, 7, 8, 9, 10], "out": [1, 2, 4, 6, 7, 8, 9, 10]},
        {"in": [IV(1, 2), 4, 6, 7, 8, 9, 10], "out": [1, 2, 4, 6, 7, 8, 9, 10]},
        {"in": [IV(1, 2), 4, IV(6, 7), 8, 9, 10], "out": [1, 2, 4, 6, 7, 8, 9, 10]},
        {"in": [IV(1, 2), 4, IV(6, 10)], "out": [1, 2, 4, 6, 7, 8, 9, 10]},
    ],
    # is_type_test_ (:873-884); the three non-integer cases (0.23, atom, <<>>)
    # are not representable in the integer domain and are recorded as such.
    "is_type": [
        {"in": [1, 2, 4, 6, 7, 8, 9, 10], "out": True},
        {"in": [IV(1, 2), 4, 6, 7, 8, 9, 10], "out": True},
        {"in": [IV(1, 2), 4, IV(6, 7), 8, 9, 10], "out": True},
        {"in": [IV(1, 2), 4, IV(6, 7), 8, IV(9, 10)], "out": True},
        {"in": [IV(1, 2), 4, IV(6, 10)], "out": True},
    ],
    "is_type_non_integer_terms": ["[0.23]", "[atom]", "[<<>>]"],
    # is_element_test_ (:887-905)
    "is_element": [
        {"el": e, "set": EXP, "out": o}
        for e, o in [
            (1, True), (2, True), (3, False), (4, True), (5, False), (6, True),
            (7, True), (8, True), (9, True), (10, True), (11, False),
            (IV(1, 6), False), (IV(6, 7), True), (IV(7, 10), True), (IV(8, 11), False),
        ]
    ],
    # flat_size_test_ / min_test_ / max_test_ (:908-934)
    "flat_size": [
        {"in": s, "out": 8}
        for s in [
            [1, 2, 4, 6, 7, 8, 9, 10],
            [IV(1, 2), 4, 6, 7, 8, 9, 10],
            [IV(1, 2), 4, IV(6, 7), 8, 9, 10],
            [IV(1, 2), 4, IV(6, 7), 8, IV(9, 10)],
            [IV(1, 2), 4, IV(6, 10)],
        ]
    ],
    "min": [{"in": s, "out": 1} for s in [
        [1, 2, 4, 6, 7, 8, 9, 10], [IV(1, 2), 4, 6, 7, 8, 9, 10],
        [IV(1, 2), 4, IV(6, 7), 8, 9, 10], [IV(1, 2), 4, IV(6, 7), 8, IV(9, 10)],
        [IV(1, 2), 4, IV(6, 10)]]],
    "max": [{"in": s, "out": 10} for s in [
        [1, 2, 4, 6, 7, 8, 9, 10], [IV(1, 2), 4, 6, 7, 8, 9, 10],
        [IV(1, 2), 4, IV(6, 7), 8, 9, 10], [IV(1, 2), 4, IV(6, 7), 8, IV(9, 10)],
        [IV(1, 2), 4, IV(6, 10)]]],
    # element_precedes_test_ (:937-947)
    "element_precedes": [
        {"a": 0, "b": IV(2, 3), "out": True},
        {"a": 1, "b": IV(2, 3), "out": True},
        {"a": IV(0, 1), "b": IV(2, 3), "out": True},
        {"a": IV(1, 1), "b": 1, "out": False},
        {"a": IV(0, 1), "b": IV(0, 1), "out": False},
        {"a": IV(0, 3), "b": IV(2, 3), "out": False},
        {"a": IV(3, 4), "b": IV(2, 3), "out": False},
        {"a": IV(4, 5), "b": IV(2, 3), "out": False},
    ],
    # element_meets_test_ (:949-957)
    "element_meets": [
        {"a": IV(1, 1), "b": 1, "out": False},
        {"a": IV(0, 1), "b": IV(0, 1), "out": False},
        {"a": IV(0, 3), "b": IV(2, 3), "out": False},
        {"a": IV(3, 4), "b": IV(2, 3), "out": False},
        {"a": IV(0, 1), "b": IV(2, 3), "out": True},
        {"a": IV(4, 5), "b": IV(2, 3), "out": True},
    ],
    # element_subtract_test_ (:959-977)
    "element_subtract": [
        {"a": 16, "b": 16, "out": []},
        {"a": IV(0, 16), "b": IV(0, 16), "out": []},
        {"a": IV(4, 16), "b": IV(0, 16), "out": []},
        {"a": IV(0, 5), "b": IV(0, 10), "out": []},
        {"a": IV(5, 10), "b": IV(3, 20), "out": []},
        {"a": IV(0, 16), "b": IV(2, 16), "out": [IV(0, 1)]},
        {"a": IV(0, 16), "b": IV(0, 8), "out": [IV(9, 16)]},
        {"a": IV(4, 16), "b": IV(4, 8), "out": [IV(9, 16)]},
        {"a": IV(4, 16), "b": IV(4, 8), "out": [IV(9, 16)]},
        {"a": IV(3, 20), "b": IV(0, 10), "out": [IV(11, 20)]},
        {"a": IV(0, 16), "b": IV(8, 20), "out": [IV(0, 7)]},
        {"a": IV(0, 16), "b": IV(2, 8), "out": [IV(0, 1), IV(9, 16)]},
        {"a": IV(0, 16), "b": IV(4, 8), "out": [IV(0, 3), IV(9, 16)]},
        {"a": IV(3, 20), "b": IV(5, 10), "out": [IV(3, 4), IV(11, 20)]},
    ],
    # add_element_test_ (:979-1000): {Expected, Element, Set}; each case also
    # asserts ordsets:union(seq([E]), seq(Set)) == seq(add_element(E, Set))
    "add_element": [
        {"out": [IV(0, 1), IV(3, 4)], "el": IV(0, 1), "set": [IV(3, 4)]},
        {"out": [0, IV(3, 4)], "el": 0, "set": [IV(3, 4)]},
        {"out": [1, IV(3, 4)], "el": 1, "set": [IV(3, 4)]},
        {"out": [IV(0, 3)], "el": IV(0, 1), "set": [IV(2, 3)]},
        {"out": [IV(0, 3)], "el": IV(0, 2), "set": [IV(2, 3)]},
        {"out": [IV(0, 3)], "el": IV(0, 3), "set": [IV(2, 3)]},
        {"out": [IV(0, 4)], "el": IV(0, 4), "set": [IV(2, 3)]},
        {"out": [IV(0, 4)], "el": IV(0, 4), "set": [IV(0, 3)]},
        {"out": [IV(0, 4)], "el": IV(0, 4), "set": [IV(0, 4)]},
        {"out": [IV(2, 10)], "el": IV(3, 10), "set": [IV(2, 3)]},
        {"out": [IV(2, 3), IV(20, 30)], "el": IV(20, 30), "set": [IV(2, 3)]},
    ],
    # del_element_test_ (:1003-1019); each case also asserts
    # ordsets:subtract(seq(Set), seq([E])) == seq(del_element(E, Set))
    "del_element": [
        {"out": [2], "el": 1, "set": [2]},
        {"out": [IV(2, 3)], "el": 1, "set": [IV(2, 3)]},
        {"out": [], "el": 1, "set": [1]},
        {"out": [], "el": 1, "set": [IV(1, 1)]},
        {"out": [], "el": IV(1, 2), "set": [IV(1, 2)]},
        {"out": [IV(3, 4)], "el": IV(0, 1), "set": [IV(3, 4)]},
        {"out": [IV(2, 4)], "el": IV(0, 1), "set": [IV(0, 4)]},
        {"out": [IV(0, 2), IV(15, 16)], "el": IV(3, 14), "set": [IV(0, 16)]},
    ],
}

# vclock eunit (:206-257).  Actors: a=1, b=2, c=3; <<"N">> = N.
vclock = {
    "source": "src/partisan_vclock.erl:206-257",
    "actor_map": {"a": 1, "b": 2, "c": 3, "<<\"1\">>..<<\"7\">>": "1..7"},
    # example_test (:212-227) as an op script over named clocks
    "example": [
        ["fresh", "A"], ["fresh", "B"],
        ["increment", "A1", 1, "A"], ["increment", "B1", 2, "B"],
        ["assert_descends", True, "A1", "A"], ["assert_descends", True, "B1", "B"],
        ["assert_descends", False, "A1", "B1"],
        ["increment", "A2", 1, "A1"],
        ["merge", "C", ["A2", "B1"]],
        ["increment", "C1", 3, "C"],
        ["assert_descends", True, "C1", "A2"], ["assert_descends", True, "C1", "B1"],
        ["assert_descends", False, "B1", "C1"], ["assert_descends", False, "B1", "A1"],
    ],
    # accessor_test (:229-235)
    "accessor": {"clock": [[1, 1], [2, 2]],
                 "get_counter": [[1, 1], [2, 2], [3, 0]],
                 "all_nodes": [1, 2]},
    # merge_test, merge_less_left_test, merge_less_right_test, merge_same_id_test (:237-257)
    "merge": [
        {"in": [[]], "out": []},
        {"in": [[[1, 1], [2, 2], [4, 4]], [[3, 3], [4, 3]]], "out": [[1, 1], [2, 2], [3, 3], [4, 4]]},
        {"in": [[[5, 5]], [[6, 6], [7, 7]]], "out": [[5, 5], [6, 6], [7, 7]]},
        {"in": [[[6, 6], [7, 7]], [[5, 5]]], "out": [[5, 5], [6, 6], [7, 7]]},
        {"in": [[[1, 1], [2, 1]], [[1, 1], [3, 1]]], "out": [[1, 1], [2, 1], [3, 1]]},
    ],
}


def _tree(arity, n, cycles):
    return {"arity": arity, "nodes": list(range(1, n + 1)), "cycles": cycles}


# build_tree arity_test (:106-199) and cycles_test (:201-261); expected as
# orddict lists [[Node, [Children]]]
build_tree = {
    "source": "src/partisan_plumtree_util.erl:102-261",
    "cases": [
        # 1-ary
        {**_tree(1, 1, False), "out": [[1, []]]},
        {**_tree(1, 2, False), "out": [[1, [2]], [2, []]]},
        {**_tree(1, 3, False), "out": [[1, [2]], [2, [3]], [3, []]]},
        {**_tree(1, 4, False), "out": [[1, [2]], [2, [3]], [3, [4]], [4, []]]},
        # 2-ary
        {**_tree(2, 1, False), "out": [[1, []]]},
        {**_tree(2, 2, False), "out": [[1, [2]], [2, []]]},
        {**_tree(2, 3, False), "out": [[1, [2, 3]], [2, []], [3, []]]},
        {**_tree(2, 4, False), "out": [[1, [2, 3]], [2, [4]], [3, []], [4, []]]},
        {**_tree(2, 5, False), "out": [[1, [2, 3]], [2, [4, 5]], [3, []], [4, []], [5, []]]},
        {**_tree(2, 6, False), "out": [[1, [2, 3]], [2, [4, 5]], [3, [6]], [4, []], [5, []], [6, []]]},
        # 3-ary
        {**_tree(3, 1, False), "out": [[1, []]]},
        {**_tree(3, 2, False), "out": [[1, [2]], [2, []]]},
        {**_tree(3, 3, False), "out": [[1, [2, 3]], [2, []], [3, []]]},
        {**_tree(3, 4, False), "out": [[1, [2, 3, 4]], [2, []], [3, []], [4, []]]},
        {**_tree(3, 5, False), "out": [[1, [2, 3, 4]], [2, [5]], [3, []], [4, []], [5, []]]},
        {**_tree(3, 6, False), "out": [[1, [2, 3, 4]], [2, [5, 6]], [3, []], [4, []], [5, []], [6, []]]},
        {**_tree(3, 7, False), "out": [[1, [2, 3, 4]], [2, [5, 6, 7]], [3, []], [4, []], [5, []], [6, []], [7, []]]},
        {**_tree(3, 8, False), "out": [[1, [2, 3, 4]], [2, [5, 6, 7]], [3, [8]], [4, []], [5, []], [6, []], [7, []], [8, []]]},
        # cycles, 1-ary
        {**_tree(1, 1, True), "out": [[1, [1]]]},
        {**_tree(1, 2, True), "out": [[1, [2]], [2, [1]]]},
        {**_tree(1, 3, True), "out": [[1, [2]], [2, [3]], [3, [1]]]},
        {**_tree(1, 4, True), "out": [[1, [2]], [2, [3]], [3, [4]], [4, [1]]]},
        # cycles, 2-ary
        {**_tree(2, 1, True), "out": [[1, [1, 1]]]},
        {**_tree(2, 2, True), "out": [[1, [2, 1]], [2, [2, 1]]]},
        {**_tree(2, 3, True), "out": [[1, [2, 3]], [2, [1, 2]], [3, [3, 1]]]},
        {**_tree(2, 4, True), "out": [[1, [2, 3]], [2, [4, 1]], [3, [2, 3]], [4, [4, 1]]]},
        {**_tree(2, 5, True), "out": [[1, [2, 3]], [2, [4, 5]], [3, [1, 2]], [4, [3, 4]], [5, [5, 1]]]},
        {**_tree(2, 6, True), "out": [[1, [2, 3]], [2, [4, 5]], [3, [6, 1]], [4, [2, 3]], [5, [4, 5]], [6, [6, 1]]]},
        # cycles, 3-ary
        {**_tree(3, 1, True), "out": [[1, [1, 1, 1]]]},
        {**_tree(3, 2, True), "out": [[1, [2, 1, 2]], [2, [1, 2, 1]]]},
        {**_tree(3, 3, True), "out": [[1, [2, 3, 1]], [2, [2, 3, 1]], [3, [2, 3, 1]]]},
        {**_tree(3, 4, True), "out": [[1, [2, 3, 4]], [2, [1, 2, 3]], [3, [4, 1, 2]], [4, [3, 4, 1]]]},
        {**_tree(3, 5, True), "out": [[1, [2, 3, 4]], [2, [5, 1, 2]], [3, [3, 4, 5]], [4, [1, 2, 3]], [5, [4, 5, 1]]]},
        {**_tree(3, 6, True), "out": [[1, [2, 3, 4]], [2, [5, 6, 1]], [3, [2, 3, 4]], [4, [5, 6, 1]], [5, [2, 3, 4]], [6, [5, 6, 1]]]},
    ],
}

# causal_test (test/partisan_SUITE.erl:500-586): Node3 emits m1 then m2 to
# Node4 on one label; m2 is handed to Node4's backend first, then m1.
# Expected: m2 not delivered on receipt; m1 delivered on receipt; m2
# delivered on the next redelivery tick.
causal = {
    "source": "test/partisan_SUITE.erl:500-586",
    "sender": 3, "receiver": 4,
    "emit": ["m1", "m2"],
    "receive_order": ["m2", "m1"],
    "expect": {
        "after_receive_m2": [],
        "after_receive_m1": ["m1"],
        "after_redelivery_tick": ["m1", "m2"],
    },
}


# partisan_membership_set eunit (:269-522) as op scripts over named states.
# Elements are node_spec() maps, numbered in Erlang term order (maps compare
# channels, then listen_addrs, then name; here the specs differ only by ip):
#   1 = node1@127.0.0.1 ip {127,0,0,1}; 2 = node1@127.0.0.1 ip {192,168,0,1};
#   11, 12, 13 = node1/2/3 with ips {192,168,0,1..3} (compare_test).
# Actors a, b, c = 1, 2, 3.  Every add draws a fresh unique token (the
# reference's tokens are random; no assertion depends on their values).
#   ["new", X] | ["add", X, Elem, Actor, Y] (X = add(Elem, Actor, Y))
#   ["remove", X, Elem, Actor, Y] | ["merge", X, Y, Z] (X = merge(Y, Z))
#   ["alias", X, Y] | ["to_list", X, [Elems]] | ["same_term", X, Y]
#   ["equal", Bool, X, Y] | ["compare", [List], X, [Joiners], [Leavers]]
membership_set = {
    "source": "src/partisan_membership_set.erl:269-522",
    "tests": {
        "add_remove_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["to_list", "A", [1]],
                            ["remove", "A1", 1, 1, "A"], ["to_list", "A1", []]],
        "one_side_updates_test": [["new", "A"], ["alias", "B", "A"], ["add", "A1", 1, 1, "A"],
                                  ["to_list", "A1", [1]], ["merge", "M", "A1", "B"], ["to_list", "M", [1]]],
        "concurrent_updates_test": [["new", "A"], ["alias", "B", "A"], ["add", "A1", 1, 1, "A"],
                                    ["add", "B1", 2, 2, "B"], ["to_list", "A1", [1]], ["to_list", "B1", [2]],
                                    ["merge", "M", "A1", "B1"], ["to_list", "M", [1, 2]]],
        "compare_test": [["new", "S0"], ["add", "S1", 11, 1, "S0"], ["add", "S2", 12, 1, "S1"],
                         ["compare", [], "S2", [], []], ["compare", [11, 12], "S2", [], []],
                         ["compare", [11, 12, 13], "S2", [13], []], ["compare", [11, 13], "S2", [13], [12]]],
        "concurrent_remove_update_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["remove", "A1", 1, 1, "A"],
                                          ["alias", "B", "A"], ["add", "B1", 2, 2, "B"], ["to_list", "A", [1]],
                                          ["to_list", "A1", []], ["to_list", "B1", [1, 2]],
                                          ["merge", "M", "A1", "B1"], ["to_list", "M", [2]]],
        "assoc_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["add", "B", 1, 2, "N"], ["remove", "B2", 1, 2, "B"],
                       ["alias", "C", "A"], ["remove", "C3", 1, 3, "C"],
                       ["merge", "L1", "B2", "C3"], ["merge", "L", "A", "L1"],
                       ["merge", "R1", "A", "B2"], ["merge", "R", "R1", "C3"], ["same_term", "L", "R"],
                       ["merge", "P1", "A", "C3"], ["merge", "P", "P1", "B2"],
                       ["to_list", "P", None], ["same_list", "P", "R"], ["same_term", "P", "R"]],
        "clock_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["alias", "B", "A"], ["add", "B2", 2, 2, "B"],
                       ["remove", "A2", 1, 1, "A"], ["add", "A4", 2, 1, "A2"], ["merge", "AB", "A4", "B2"],
                       ["to_list", "AB", [2]]],
        "remfield_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["alias", "B", "A"], ["remove", "A2", 1, 1, "A"],
                          ["add", "A4", 2, 1, "A2"], ["merge", "AB", "A4", "B"], ["to_list", "AB", [2]]],
        "present_but_removed_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["alias", "C", "A"],
                                     ["remove", "A2", 1, 1, "A"], ["add", "B", 2, 2, "N"],
                                     ["merge", "A3", "B", "A2"], ["remove", "B2", 2, 2, "B"],
                                     ["merge", "M1", "C", "A3"], ["merge", "M", "B2", "M1"], ["to_list", "M", []]],
        "no_dots_left_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["add", "B", 2, 2, "N"], ["alias", "C", "A"],
                              ["remove", "A2", 1, 1, "A"], ["merge", "A3", "A2", "B"], ["remove", "B2", 2, 2, "B"],
                              ["merge", "B3", "B2", "C"], ["merge", "M1", "B3", "A3"], ["merge", "M", "C", "M1"],
                              ["to_list", "M", []]],
        "equals_test": [["new", "N"], ["add", "A", 1, 1, "N"], ["add", "B", 1, 2, "N"], ["equal", False, "A", "B"],
                        ["merge", "C", "A", "B"], ["merge", "D", "B", "A"], ["equal", True, "C", "D"],
                        ["equal", True, "A", "A"]],
    },
}


def main():
    for name, obj in [("interval_sets_kat.json", interval_sets), ("vclock_kat.json", vclock),
                      ("build_tree_kat.json", build_tree), ("causal_kat.json", causal),
                      ("membership_set_kat.json", membership_set)]:
        with open(os.path.join(HERE, name), "w") as f:
            json.dump(obj, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()

"""ctypes wrapper around oracle/liboracle.so.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package partisan_amd.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class IEl(C.Structure):
    _fields_ = [("lo", C.c_int64), ("hi", C.c_int64), ("iv", C.c_int32), ("_pad", C.c_int32)]


class Dot(C.Structure):
    _fields_ = [("actor", C.c_uint32), ("_pad", C.c_uint32), ("ctr", C.c_int64)]


class Msg(C.Structure):
    _fields_ = [("type", C.c_uint32), ("src", C.c_uint32), ("dst", C.c_uint32), ("round", C.c_uint32),
                ("root", C.c_uint32), ("id_node", C.c_uint32), ("id_epoch", C.c_uint32),
                ("id_mono", C.c_uint32), ("seq", C.c_uint64)]


class RoundStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 6), ("delivered_new", C.c_uint64), ("active", C.c_uint64),
                ("outstanding", C.c_uint64), ("outstanding_live", C.c_uint64),
                ("max_per_edge", C.c_uint64)]


class DmStats(C.Structure):
    _fields_ = [("rm_sent", C.c_uint64), ("push_sent", C.c_uint64), ("pull_sent", C.c_uint64),
                ("delivered_new", C.c_uint64), ("complete", C.c_uint64)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class HvConfig(C.Structure):
    _fields_ = [(k, C.c_uint32) for k in ("active_max_size", "active_min_size", "active_rwl", "passive_max_size",
                                           "passive_rwl", "shuffle_k_active", "shuffle_k_passive",
                                           "shuffle_rounds", "promotion_rounds")]


class HvStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 10), ("draws", C.c_uint64), ("error", C.c_uint64)]

    def as_dict(self):
        return {"sent": [int(x) for x in self.sent[1:10]], "draws": int(self.draws), "error": int(self.error)}


class CausalStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("emitted", "received", "delivered", "checks", "buffered")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class FmStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("sent", "processed", "merges", "updates", "inflight", "member_sum")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class ScampStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 7)] + [(k, C.c_uint64) for k in (
        "dropped", "processed", "draws", "stopped", "error", "pv_sum", "inview_sum", "resub")]

    def as_dict(self):
        d = {"sent": [int(x) for x in self.sent[1:7]]}
        d.update({k: int(getattr(self, k)) for k, _ in self._fields_[1:]})
        return d


class C3Stats(C.Structure):
    _fields_ = [("scamp", ScampStats), ("pt", RoundStats)] + [(k, C.c_uint64) for k in (
        "updates", "pt_dropped", "delivered_live", "live")]

    def as_dict(self):
        d = {"scamp": self.scamp.as_dict(), "pt": stats_dict(self.pt)}
        d.update({k: int(getattr(self, k)) for k, _ in self._fields_[2:]})
        return d


HV_DEFAULTS = dict(active_max_size=6, active_min_size=3, active_rwl=6, passive_max_size=30, passive_rwl=6,
                   shuffle_k_active=3, shuffle_k_passive=4, shuffle_rounds=10, promotion_rounds=5)

MSG_NAMES = {1: "broadcast", 2: "prune", 3: "i_have", 4: "ignored_i_have", 5: "graft"}

_lib = None


class RelayRound(C.Structure):
    _fields_ = [(f, C.c_uint64) for f in ("direct", "relay", "dropped", "lost", "arrived")]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        sz = C.c_size_t
        L.orc_iset_from_list.argtypes = [P(IEl), sz, P(IEl), sz, P(sz)]
        L.orc_iset_is_element.argtypes = [P(IEl), P(IEl), sz]
        L.orc_iset_add_element.argtypes = [P(IEl), P(IEl), sz, P(IEl), sz, P(sz)]
        L.orc_iset_del_element.argtypes = [P(IEl), P(IEl), sz, P(IEl), sz, P(sz)]
        L.orc_iset_element_subtract.argtypes = [P(IEl), P(IEl), P(IEl), sz, P(sz)]
        L.orc_iset_element_precedes.argtypes = [P(IEl), P(IEl)]
        L.orc_iset_element_meets.argtypes = [P(IEl), P(IEl)]
        for f in ("orc_iset_flat_size", "orc_iset_min", "orc_iset_max"):
            getattr(L, f).argtypes = [P(IEl), sz]
            getattr(L, f).restype = C.c_int64
        L.orc_iset_is_type.argtypes = [P(IEl), sz]
        L.orc_iset_seq.argtypes = [P(IEl), sz, P(C.c_int64), sz, P(sz)]
        for f in ("orc_iset_union", "orc_iset_intersection", "orc_iset_subtract"):
            getattr(L, f).argtypes = [P(IEl), sz, P(IEl), sz, P(IEl), sz, P(sz)]
        L.orc_vc_descends.argtypes = [P(Dot), sz, P(Dot), sz]
        L.orc_vc_dominates.argtypes = [P(Dot), sz, P(Dot), sz]
        L.orc_vc_merge.argtypes = [P(Dot), P(sz), sz, P(Dot), sz, P(sz)]
        L.orc_vc_get_counter.argtypes = [C.c_uint32, P(Dot), sz]
        L.orc_vc_get_counter.restype = C.c_int64
        L.orc_vc_increment.argtypes = [C.c_uint32, P(Dot), sz, P(Dot), sz, P(sz)]
        L.orc_vc_equal.argtypes = [P(Dot), sz, P(Dot), sz]
        L.orc_vc_all_nodes.argtypes = [P(Dot), sz, P(C.c_uint32), sz, P(sz)]
        L.orc_vc_glb.argtypes = [P(Dot), sz, P(Dot), sz, P(Dot), sz, P(sz)]
        L.orc_vc_subtract_dots.argtypes = [P(Dot), sz, P(Dot), sz, P(Dot), sz, P(sz)]
        L.orc_build_tree.argtypes = [C.c_uint32, P(C.c_uint32), sz, C.c_int,
                                     P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.orc_pt_create.argtypes = [C.c_uint32, P(C.c_uint64), P(C.c_uint32), C.c_uint32]
        L.orc_pt_create.restype = C.c_void_p
        L.orc_pt_destroy.argtypes = [C.c_void_p]
        L.orc_pt_set_alive.argtypes = [C.c_void_p, P(C.c_uint8)]
        L.orc_pt_heartbeat.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_pt_heartbeat.restype = C.c_uint32
        L.orc_pt_update.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), sz]
        L.orc_pt_reset_peers_all.argtypes = [C.c_void_p]
        L.orc_pt_step.argtypes = [C.c_void_p, C.c_uint32, P(RoundStats)]
        L.orc_pt_step.restype = C.c_uint32
        L.orc_pt_run.argtypes = [C.c_void_p, C.c_uint32, P(RoundStats), sz]
        L.orc_pt_run.restype = C.c_uint32
        L.orc_pt_pending.argtypes = [C.c_void_p, P(Msg), sz]
        L.orc_pt_pending.restype = sz
        L.orc_pt_get_peers.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint32), P(sz),
                                       P(C.c_uint32), P(sz), sz]
        L.orc_pt_get_outstanding.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32),
                                             P(C.c_uint32), sz]
        L.orc_pt_get_outstanding.restype = sz
        L.orc_pt_get_delivered.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint8)]
        L.orc_pt_get_recv_round.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint32)]
        L.orc_pt_dump_state.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, P(C.c_uint64), P(C.c_uint32),
                                        C.c_uint32, C.c_uint32, P(C.c_uint32), P(C.c_uint32), P(C.c_uint32),
                                        P(C.c_uint16)]
        L.orc_pt_inflight_words.argtypes = [C.c_void_p, P(C.c_uint64), P(C.c_uint32), C.c_uint32, C.c_uint32,
                                            P(C.c_uint32)]
        L.orc_pt_restart_backend.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_pt_epoch.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_pt_epoch.restype = C.c_uint32
        L.orc_pt_set_omissions.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint32), sz]
        L.orc_pt_omitted.argtypes = [C.c_void_p]
        L.orc_pt_omitted.restype = C.c_uint64
        L.orc_pt_set_delays.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint32), P(C.c_uint8), sz]
        L.orc_pt_inflight.argtypes = [C.c_void_p]
        L.orc_pt_inflight.restype = C.c_uint64
        L.orc_relay_run.argtypes = [C.c_uint32, P(C.c_uint64), P(C.c_uint32), P(C.c_uint64), P(C.c_uint32),
                                    P(C.c_uint8), C.c_uint32, P(C.c_uint32), P(C.c_uint32), C.c_uint32,
                                    P(C.c_uint64), P(C.c_uint32), P(RelayRound), sz, sz]
        L.orc_relay_run.restype = C.c_int64
        L.orc_philox4x32_10.argtypes = [P(C.c_uint32), P(C.c_uint32), P(C.c_uint32)]
        L.orc_dm_select2.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, P(C.c_uint32)]
        L.orc_dm_draws_per_call.argtypes = [C.c_uint32]
        L.orc_dm_draws_per_call.restype = C.c_uint64
        L.orc_dm_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32]
        L.orc_dm_create.restype = C.c_void_p
        L.orc_dm_destroy.argtypes = [C.c_void_p]
        L.orc_dm_origin.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_dm_origin.restype = C.c_uint32
        L.orc_dm_full_mask.argtypes = [C.c_void_p]
        L.orc_dm_full_mask.restype = C.c_uint64
        L.orc_dm_broadcast_all.argtypes = [C.c_void_p]
        L.orc_dm_step.argtypes = [C.c_void_p, C.c_uint32, P(DmStats)]
        L.orc_dm_run.argtypes = [C.c_void_p, C.c_uint32, P(DmStats), sz]
        L.orc_dm_run.restype = C.c_uint32
        L.orc_dm_get_seen.argtypes = [C.c_void_p, P(C.c_uint64)]
        L.orc_dm_pending.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint32), P(C.c_uint32), P(C.c_uint32),
                                     P(C.c_uint64), sz]
        L.orc_dm_pending.restype = sz
        L.orc_hv_create.argtypes = [C.c_uint32, C.c_uint64, P(HvConfig)]
        L.orc_hv_create.restype = C.c_void_p
        L.orc_hv_destroy.argtypes = [C.c_void_p]
        L.orc_hv_set_alive.argtypes = [C.c_void_p, P(C.c_uint8)]
        L.orc_hv_join.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_hv_step.argtypes = [C.c_void_p, C.c_uint32, P(HvStats)]
        L.orc_hv_inflight.argtypes = [C.c_void_p]
        L.orc_hv_inflight.restype = sz
        L.orc_hv_views.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32), P(C.c_uint32),
                                   P(C.c_uint32)]
        L.orc_hv_draws.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_hv_draws.restype = C.c_uint64
        L.orc_hv_idmap.argtypes = [C.c_void_p, C.c_uint32, C.c_int, P(C.c_uint32), P(C.c_uint32), P(C.c_uint32), sz]
        L.orc_hv_idmap.restype = sz
        L.orc_causal_create.argtypes = [C.c_uint32] * 5 + [C.c_uint64]
        L.orc_causal_create.restype = C.c_void_p
        L.orc_causal_destroy.argtypes = [C.c_void_p]
        L.orc_causal_emit.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_causal_emit.restype = C.c_uint32
        L.orc_causal_receive.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_causal_tick.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_causal_log.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), sz]
        L.orc_causal_log.restype = sz
        L.orc_causal_step.argtypes = [C.c_void_p, C.c_uint32, P(CausalStats)]
        L.orc_causal_clock.argtypes = [C.c_void_p, C.c_uint32, P(Dot), sz]
        L.orc_causal_clock.restype = sz
        L.orc_causal_buffered.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint32), sz]
        L.orc_causal_buffered.restype = sz
        L.orc_causal_delivered.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_causal_delivered.restype = C.c_uint64
        L.orc_causal_emitter.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_causal_emitter.restype = C.c_uint32
        L.orc_orset_new.restype = C.c_void_p
        L.orc_orset_clone.argtypes = [C.c_void_p]
        L.orc_orset_clone.restype = C.c_void_p
        L.orc_orset_free.argtypes = [C.c_void_p]
        L.orc_orset_add.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64]
        L.orc_orset_remove.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_orset_merge.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_orset_merge.restype = C.c_void_p
        L.orc_orset_equal.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_orset_to_list.argtypes = [C.c_void_p, P(C.c_uint32), sz]
        L.orc_orset_to_list.restype = sz
        L.orc_orset_dump.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint64), P(C.c_uint8), sz]
        L.orc_orset_dump.restype = sz
        L.orc_fm_create.argtypes = [C.c_uint32, C.c_uint32]
        L.orc_fm_create.restype = C.c_void_p
        L.orc_fm_destroy.argtypes = [C.c_void_p]
        L.orc_fm_set_alive.argtypes = [C.c_void_p, P(C.c_uint8)]
        L.orc_fm_join.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_fm_leave.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_fm_step.argtypes = [C.c_void_p, C.c_uint32, P(FmStats)]
        L.orc_fm_inflight.argtypes = [C.c_void_p]
        L.orc_fm_inflight.restype = sz
        L.orc_fm_members.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), sz]
        L.orc_fm_members.restype = sz
        L.orc_fm_state.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_fm_state.restype = C.c_void_p
        L.orc_fm_alive.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_orset_put.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint8]
        L.orc_fm_messages.argtypes = [C.c_void_p, P(C.c_uint32), P(C.c_uint32), P(C.c_uint64), sz]
        L.orc_fm_messages.restype = sz
        L.orc_fm_message_state.argtypes = [C.c_void_p, sz]
        L.orc_fm_message_state.restype = C.c_void_p
        L.orc_fm_take.argtypes = [C.c_void_p, C.c_uint32, P(C.c_uint32), P(C.c_uint64), P(C.c_void_p), sz]
        L.orc_fm_take.restype = sz
        L.orc_fm_put.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint64, C.c_void_p]
        L.orc_scamp_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64]
        L.orc_scamp_create.restype = C.c_void_p
        L.orc_scamp_destroy.argtypes = [C.c_void_p]
        L.orc_scamp_set_alive.argtypes = [C.c_void_p, P(C.c_uint8)]
        L.orc_scamp_join.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_scamp_leave.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_scamp_crash.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_scamp_step.argtypes = [C.c_void_p, C.c_uint32, P(ScampStats)]
        L.orc_scamp_inflight.argtypes = [C.c_void_p]
        L.orc_scamp_inflight.restype = sz
        L.orc_scamp_pending.argtypes = [C.c_void_p, P(C.c_uint32), sz]
        L.orc_scamp_pending.restype = sz
        L.orc_scamp_view.argtypes = [C.c_void_p, C.c_uint32, C.c_int, P(C.c_uint32), sz]
        L.orc_scamp_view.restype = sz
        L.orc_scamp_draws.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_scamp_draws.restype = C.c_uint64
        L.orc_scamp_alive.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_scamp_last_ping.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_scamp_last_ping.restype = C.c_int64
        L.orc_c3_create.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64]
        L.orc_c3_create.restype = C.c_void_p
        L.orc_c3_destroy.argtypes = [C.c_void_p]
        L.orc_c3_scamp.argtypes = [C.c_void_p]
        L.orc_c3_scamp.restype = C.c_void_p
        L.orc_c3_plumtree.argtypes = [C.c_void_p]
        L.orc_c3_plumtree.restype = C.c_void_p
        L.orc_c3_join.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32]
        L.orc_c3_crash.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_c3_heartbeat.argtypes = [C.c_void_p, C.c_uint32]
        L.orc_c3_heartbeat.restype = C.c_uint32
        L.orc_c3_step.argtypes = [C.c_void_p, C.c_uint32, P(C3Stats)]
        _lib = L
    return _lib


# ---------------------------------------------------------------- interval sets
def _to_iels(terms):
    arr = (IEl * max(1, len(terms)))()
    for i, t in enumerate(terms):
        if isinstance(t, (list, tuple)):
            arr[i].lo, arr[i].hi, arr[i].iv = t[0], t[1], 1
        else:
            arr[i].lo, arr[i].hi, arr[i].iv = t, t, 0
    return arr


def _from_iels(arr, n):
    out = []
    for i in range(n):
        e = arr[i]
        out.append([e.lo, e.hi] if e.iv else e.lo)
    return out


def _iset_call(fn, *args, cap=256):
    out = (IEl * cap)()
    n = C.c_size_t(0)
    rc = fn(*args, out, cap, C.byref(n))
    if rc < 0:
        raise ValueError("badarg")
    return _from_iels(out, n.value)


def iset_from_list(terms):
    return _iset_call(lib().orc_iset_from_list, _to_iels(terms), len(terms))


def iset_is_element(el, s):
    rc = lib().orc_iset_is_element(_to_iels([el]), _to_iels(s), len(s))
    if rc < 0:
        raise ValueError("badarg")
    return bool(rc)


def iset_add_element(el, s):
    return _iset_call(lib().orc_iset_add_element, _to_iels([el]), _to_iels(s), len(s))


def iset_del_element(el, s):
    return _iset_call(lib().orc_iset_del_element, _to_iels([el]), _to_iels(s), len(s))


def iset_element_subtract(a, b):
    return _iset_call(lib().orc_iset_element_subtract, _to_iels([a]), _to_iels([b]))


def iset_element_precedes(a, b):
    return bool(lib().orc_iset_element_precedes(_to_iels([a]), _to_iels([b])))


def iset_element_meets(a, b):
    return bool(lib().orc_iset_element_meets(_to_iels([a]), _to_iels([b])))


def iset_flat_size(s):
    return lib().orc_iset_flat_size(_to_iels(s), len(s))


def iset_min(s):
    return lib().orc_iset_min(_to_iels(s), len(s))


def iset_max(s):
    return lib().orc_iset_max(_to_iels(s), len(s))


def iset_is_type(s):
    return bool(lib().orc_iset_is_type(_to_iels(s), len(s)))


def iset_seq(s, cap=4096):
    out = (C.c_int64 * cap)()
    n = C.c_size_t(0)
    lib().orc_iset_seq(_to_iels(s), len(s), out, cap, C.byref(n))
    return list(out[: n.value])


def iset_union(a, b):
    return _iset_call(lib().orc_iset_union, _to_iels(a), len(a), _to_iels(b), len(b))


def iset_subtract(a, b):
    return _iset_call(lib().orc_iset_subtract, _to_iels(a), len(a), _to_iels(b), len(b))


# ---------------------------------------------------------------- vclock
def _to_dots(clock):
    arr = (Dot * max(1, len(clock)))()
    for i, (a, c) in enumerate(clock):
        arr[i].actor, arr[i].ctr = a, c
    return arr


def _from_dots(arr, n):
    return [[arr[i].actor, arr[i].ctr] for i in range(n)]


def vc_descends(a, b):
    return bool(lib().orc_vc_descends(_to_dots(a), len(a), _to_dots(b), len(b)))


def vc_dominates(a, b):
    return bool(lib().orc_vc_dominates(_to_dots(a), len(a), _to_dots(b), len(b)))


def vc_merge(clocks):
    flat = [d for c in clocks for d in c]
    lens = (C.c_size_t * max(1, len(clocks)))(*[len(c) for c in clocks])
    cap = max(1, len(flat))
    out = (Dot * cap)()
    n = C.c_size_t(0)
    lib().orc_vc_merge(_to_dots(flat), lens, len(clocks), out, cap, C.byref(n))
    return _from_dots(out, n.value)


def vc_get_counter(actor, clock):
    return lib().orc_vc_get_counter(actor, _to_dots(clock), len(clock))


def vc_increment(actor, clock):
    cap = len(clock) + 1
    out = (Dot * cap)()
    n = C.c_size_t(0)
    lib().orc_vc_increment(actor, _to_dots(clock), len(clock), out, cap, C.byref(n))
    return _from_dots(out, n.value)


def vc_equal(a, b):
    return bool(lib().orc_vc_equal(_to_dots(a), len(a), _to_dots(b), len(b)))


def vc_glb(a, b):
    cap = max(1, len(a))
    out = (Dot * cap)()
    n = C.c_size_t(0)
    lib().orc_vc_glb(_to_dots(a), len(a), _to_dots(b), len(b), out, cap, C.byref(n))
    return _from_dots(out, n.value)


def vc_subtract_dots(dots, clock):
    cap = max(1, len(dots))
    out = (Dot * cap)()
    n = C.c_size_t(0)
    lib().orc_vc_subtract_dots(_to_dots(dots), len(dots), _to_dots(clock), len(clock), out, cap, C.byref(n))
    return _from_dots(out, n.value)


def vc_all_nodes(clock):
    cap = max(1, len(clock))
    out = (C.c_uint32 * cap)()
    n = C.c_size_t(0)
    lib().orc_vc_all_nodes(_to_dots(clock), len(clock), out, cap, C.byref(n))
    return list(out[: n.value])


# ---------------------------------------------------------------- build_tree
def build_tree(arity, nodes, cycles):
    n = len(nodes)
    keys = (C.c_uint32 * n)()
    ch = (C.c_uint32 * (n * arity))()
    cnt = (C.c_uint32 * n)()
    lib().orc_build_tree(arity, (C.c_uint32 * n)(*nodes), n, 1 if cycles else 0, keys, ch, cnt)
    return [[keys[i], list(ch[i * arity: i * arity + cnt[i]])] for i in range(n)]


# ---------------------------------------------------------------- plumtree
def _u64p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def _u32p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


class Plumtree:
    """Round-synchronous plumtree + heartbeat backend over a membership CSR."""

    def __init__(self, row_ptr, col, lazy_tick_rounds=1):
        self.row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        self.col = np.ascontiguousarray(col, dtype=np.uint32)
        self.n = len(self.row_ptr) - 1
        self._h = lib().orc_pt_create(self.n, _u64p(self.row_ptr), _u32p(self.col), lazy_tick_rounds)

    def close(self):
        if self._h:
            lib().orc_pt_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        lib().orc_pt_set_alive(self._h, a.ctypes.data_as(C.POINTER(C.c_uint8)))

    def heartbeat(self, root):
        """The Monotonic; after a backend restart, epoch << 24 | Monotonic (psim's id form)."""
        m = lib().orc_pt_heartbeat(self._h, root)
        return (self.epoch(root) << 24) | m

    def update(self, v, members):
        m = np.ascontiguousarray(members, dtype=np.uint32)
        lib().orc_pt_update(self._h, v, _u32p(m), len(m))

    def reset_peers_all(self):
        lib().orc_pt_reset_peers_all(self._h)

    def restart_backend(self, v):
        """v's heartbeat backend restarts: newer epoch, Monotonic 0, empty table."""
        lib().orc_pt_restart_backend(self._h, v)

    def epoch(self, v):
        return int(lib().orc_pt_epoch(self._h, v))

    def set_omissions(self, pairs):
        """Omission faults on directed (src, dst) pairs; [] heals."""
        p = np.asarray(pairs, dtype=np.uint32).reshape(-1, 2)
        s, d = np.ascontiguousarray(p[:, 0]), np.ascontiguousarray(p[:, 1])
        lib().orc_pt_set_omissions(self._h, _u32p(s), _u32p(d), len(p))

    def omitted(self):
        return int(lib().orc_pt_omitted(self._h))

    def set_delays(self, pairs, delays):
        """Delay faults: messages over directed (src, dst) arrive delays[i]
        rounds late; [] removes them.  Refused while messages are in flight."""
        p = np.asarray(pairs, dtype=np.uint32).reshape(-1, 2)
        s, d = np.ascontiguousarray(p[:, 0]), np.ascontiguousarray(p[:, 1])
        dl = np.ascontiguousarray(delays, dtype=np.uint8)
        assert len(dl) == len(p)
        rc = lib().orc_pt_set_delays(self._h, _u32p(s), _u32p(d), dl.ctypes.data_as(C.POINTER(C.c_uint8)), len(p))
        if rc:
            raise RuntimeError("orc_pt_set_delays: messages in flight")

    def inflight(self):
        return int(lib().orc_pt_inflight(self._h))

    def step(self, rounds=1):
        st = (RoundStats * rounds)()
        lib().orc_pt_step(self._h, rounds, st)
        return [stats_dict(s) for s in st]

    def run(self, max_rounds=100000, cap=4096):
        st = (RoundStats * cap)()
        r = lib().orc_pt_run(self._h, max_rounds, st, cap)
        return [stats_dict(st[i]) for i in range(min(r, cap))], r

    def pending(self):
        n = lib().orc_pt_pending(self._h, None, 0)
        arr = (Msg * max(1, n))()
        lib().orc_pt_pending(self._h, arr, n)
        return [(m.src, m.dst, m.type, m.round) for m in arr[:n]]

    def pending_full(self, packed=False):
        """(src, dst, kind, Round, Monotonic) of the messages the next round
        delivers, in handling order; packed: the id as psim reports it,
        epoch << 24 | Monotonic (a prune carries no id: 0)."""
        n = lib().orc_pt_pending(self._h, None, 0)
        arr = (Msg * max(1, n))()
        lib().orc_pt_pending(self._h, arr, n)
        if packed:
            return [(m.src, m.dst, m.type, m.round, (m.id_epoch << 24 | m.id_mono) if m.type != 2 else 0)
                    for m in arr[:n]]
        return [(m.src, m.dst, m.type, m.round, m.id_mono) for m in arr[:n]]

    def peers(self, v, root, cap=4096):
        e = (C.c_uint32 * cap)()
        l_ = (C.c_uint32 * cap)()
        ne, nl = C.c_size_t(0), C.c_size_t(0)
        lib().orc_pt_get_peers(self._h, v, root, e, C.byref(ne), l_, C.byref(nl), cap)
        return list(e[: ne.value]), list(l_[: nl.value])

    def outstanding(self, v, cap=4096):
        p = (C.c_uint32 * cap)()
        r = (C.c_uint32 * cap)()
        m = (C.c_uint32 * cap)()
        n = lib().orc_pt_get_outstanding(self._h, v, p, r, m, cap)
        return [(p[i], r[i], m[i]) for i in range(min(n, cap))]

    def delivered(self, origin, mono):
        """is_stale({origin, epoch, mono}) at every vertex; mono is psim's id
        form, epoch << 24 | Monotonic (epoch 0 until a backend restart)."""
        out = np.zeros(self.n, dtype=np.uint8)
        lib().orc_pt_get_delivered(self._h, origin, mono, out.ctypes.data_as(C.POINTER(C.c_uint8)))
        return out

    def recv_round(self, origin, mono):
        out = np.zeros(self.n, dtype=np.uint32)
        lib().orc_pt_get_recv_round(self._h, origin, mono, _u32p(out))
        return out

    def dump_state(self, root, mono, slot_row_ptr, slot_col, lo=0, hi=None):
        """Vertices [lo, hi) as psim_get_plumtree returns them: (eager, lazy,
        outstanding) masks over the slot layout (slot_row_ptr, slot_col) --
        the handle's global layout, rows sorted by id -- and the accepted
        Round as u16 (0xFFFF none, 0xFFFE the origin)."""
        hi = self.n if hi is None else hi
        k = hi - lo
        rp = np.ascontiguousarray(slot_row_ptr, dtype=np.uint64)
        cl = np.ascontiguousarray(slot_col, dtype=np.uint32)
        e, l_, o = (np.zeros(max(1, k), np.uint32) for _ in range(3))
        rr = np.zeros(max(1, k), np.uint16)
        rc = lib().orc_pt_dump_state(self._h, root, mono, _u64p(rp), _u32p(cl), lo, hi, _u32p(e),
                                     _u32p(l_), _u32p(o), rr.ctypes.data_as(C.POINTER(C.c_uint16)))
        if rc:
            raise RuntimeError("orc_pt_dump_state: a peer outside its slot row")
        return e[:k], l_[:k], o[:k], rr[:k]

    def inflight_words(self, slot_row_ptr, slot_col, lo=0, hi=None):
        """The next round's messages to receivers [lo, hi) as psim_get_inflight
        words over slots slot_row_ptr[lo] .. slot_row_ptr[hi] (Round kept for
        broadcast / i_have only)."""
        hi = self.n if hi is None else hi
        rp = np.ascontiguousarray(slot_row_ptr, dtype=np.uint64)
        cl = np.ascontiguousarray(slot_col, dtype=np.uint32)
        k = int(rp[hi] - rp[lo])
        w = np.zeros(max(1, k), np.uint32)
        rc = lib().orc_pt_inflight_words(self._h, _u64p(rp), _u32p(cl), lo, hi, _u32p(w))
        if rc:
            raise RuntimeError("orc_pt_inflight_words: > 4 messages on a slot or a sender off the row")
        return w[:k]


def inflight_protocol_words(words):
    """psim_get_inflight words with the Round kept only where the word holds a
    broadcast or an i_have (the others carry the sender's pushed Round as an
    echo the protocol never reads) -- comparable with Plumtree.inflight_words."""
    w = np.asarray(words, dtype=np.uint32)
    f = w & np.uint32(0xFFFF)
    nib = [(f >> np.uint32(4 * i)) & np.uint32(0xF) for i in range(4)]
    keep = np.zeros(w.shape, bool)
    for x in nib:
        keep |= (x == 1) | (x == 3)
    return np.where(keep, w, f).astype(np.uint32)


def stats_dict(s):
    d = {MSG_NAMES[t]: int(s.sent[t]) for t in range(1, 6)}
    d.update(delivered_new=int(s.delivered_new), active=int(s.active),
             outstanding=int(s.outstanding), outstanding_live=int(s.outstanding_live),
             max_per_edge=int(s.max_per_edge))
    return d


# ---------------------------------------------------------------- philox / demers
def philox(ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def select2(seed, v, kind, n, j):
    """Demers select_random_sublist(usort(Members), 2) over 0..n-1 for the call
    whose first draw is draw j of process (v, kind) (oracle/demers.c)."""
    o = (C.c_uint32 * 2)()
    k = lib().orc_dm_select2(seed, v, kind, n, j, o)
    return list(o[:k])


def draws_per_call(n):
    """Draws one select_random_sublist call consumes: n (faithful) or 2 (scaled)."""
    return int(lib().orc_dm_draws_per_call(n))


class Demers:
    def __init__(self, n, m, seed, ae_period=2, rm_on=True):
        self.n, self.m = n, m
        mode = 2 if rm_on == "direct_mail" else (1 if rm_on else 0)   # direct mail: demers_direct_mail.erl
        self._h = lib().orc_dm_create(n, m, seed, ae_period, mode)
        if not self._h:
            raise ValueError("bad demers config")

    def close(self):
        if self._h:
            lib().orc_dm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def origins(self):
        return [lib().orc_dm_origin(self._h, i) for i in range(self.m)]

    def full_mask(self):
        return lib().orc_dm_full_mask(self._h)

    def broadcast_all(self):
        lib().orc_dm_broadcast_all(self._h)

    def step(self, rounds=1):
        st = (DmStats * rounds)()
        lib().orc_dm_step(self._h, rounds, st)
        return [s.as_dict() for s in st]

    def run(self, max_rounds=10000, cap=4096):
        st = (DmStats * cap)()
        r = lib().orc_dm_run(self._h, max_rounds, st, cap)
        return [st[i].as_dict() for i in range(min(r, cap))], r

    def seen(self):
        out = np.zeros(self.n, dtype=np.uint64)
        lib().orc_dm_get_seen(self._h, out.ctypes.data_as(C.POINTER(C.c_uint64)))
        return out

    def pending(self):
        n = lib().orc_dm_pending(self._h, None, None, None, None, None, 0)
        t, s, d, m = (np.zeros(max(1, n), np.uint32) for _ in range(4))
        p = np.zeros(max(1, n), np.uint64)
        P = C.POINTER
        lib().orc_dm_pending(self._h, t.ctypes.data_as(P(C.c_uint32)), s.ctypes.data_as(P(C.c_uint32)),
                             d.ctypes.data_as(P(C.c_uint32)), m.ctypes.data_as(P(C.c_uint32)),
                             p.ctypes.data_as(P(C.c_uint64)), n)
        return t[:n], s[:n], d[:n], m[:n], p[:n]


# ---------------------------------------------------------------- hyparview
class HyParView:
    def __init__(self, n, seed, **cfg):
        c = dict(HV_DEFAULTS)
        c.update(cfg)
        self.n = n
        self.cfg = HvConfig(**c)
        self._h = lib().orc_hv_create(n, seed, C.byref(self.cfg))

    def close(self):
        if self._h:
            lib().orc_hv_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        lib().orc_hv_set_alive(self._h, a.ctypes.data_as(C.POINTER(C.c_uint8)))

    def join(self, v, contact):
        lib().orc_hv_join(self._h, v, contact)

    def step(self, rounds=1):
        st = (HvStats * rounds)()
        lib().orc_hv_step(self._h, rounds, st)
        return [s.as_dict() for s in st]

    def inflight(self):
        return lib().orc_hv_inflight(self._h)

    def views(self, v):
        a = (C.c_uint32 * 8)()
        p = (C.c_uint32 * 32)()
        na, np_ = C.c_uint32(), C.c_uint32()
        lib().orc_hv_views(self._h, v, a, C.byref(na), p, C.byref(np_))
        return list(a[:na.value]), list(p[:np_.value])

    def draws(self, v):
        return lib().orc_hv_draws(self._h, v)

    def idmap(self, v, which, cap=4096):
        pe, ep, cn = (C.c_uint32 * cap)(), (C.c_uint32 * cap)(), (C.c_uint32 * cap)()
        k = lib().orc_hv_idmap(self._h, v, which, pe, ep, cn, cap)
        return sorted((pe[i], ep[i], cn[i]) for i in range(min(k, cap)))


class Causal:
    """Causal delivery backend.  m = 0: the primitive API (emit/receive/tick);
    m > 0: the round workload of DESIGN.md "Causal delivery"."""

    def __init__(self, n, m=0, period=1, dmax=1, redeliver=1, seed=0):
        self.n, self.m = n, m
        if m == 0:
            lib().orc_causal_reset_handles()
        self._h = lib().orc_causal_create(n, m, period, dmax, redeliver, seed)

    def close(self):
        if self._h:
            lib().orc_causal_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def emit(self, node, dest):
        return lib().orc_causal_emit(self._h, node, dest)

    def receive(self, node, msg):
        lib().orc_causal_receive(self._h, node, msg)

    def tick(self, node):
        lib().orc_causal_tick(self._h, node)

    def log(self, node, cap=4096):
        out = (C.c_uint32 * cap)()
        k = lib().orc_causal_log(self._h, node, out, cap)
        return list(out[:min(k, cap)])

    def step(self, rounds=1):
        st = (CausalStats * rounds)()
        lib().orc_causal_step(self._h, rounds, st)
        return [x.as_dict() for x in st]

    def clock(self, v, cap=4096):
        out = (Dot * cap)()
        k = lib().orc_causal_clock(self._h, v, out, cap)
        return [(out[i].actor, out[i].ctr) for i in range(min(k, cap))]

    def buffered(self, v, cap=4096):
        k_, r_ = (C.c_uint32 * cap)(), (C.c_uint32 * cap)()
        k = lib().orc_causal_buffered(self._h, v, k_, r_, cap)
        return [(k_[i], r_[i]) for i in range(min(k, cap))]

    def delivered(self, v):
        return lib().orc_causal_delivered(self._h, v)

    def emitter(self, k):
        return lib().orc_causal_emitter(self._h, k)


# ---------------------------------------------------------------- OR-set / full membership
class ORSet:
    """state_orset (types 0.1.8) as partisan_membership_set wraps it; tokens
    are supplied by the caller (unique ints)."""

    def __init__(self, handle=None):
        self._h = handle if handle is not None else lib().orc_orset_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_orset_free(self._h)
            self._h = None

    def add(self, elem, token):
        c = ORSet(lib().orc_orset_clone(self._h))
        lib().orc_orset_add(c._h, elem, token)
        return c

    def remove(self, elem):
        c = ORSet(lib().orc_orset_clone(self._h))
        if lib().orc_orset_remove(c._h, elem) < 0:
            raise KeyError(f"precondition: {elem} not present")
        return c

    def merge(self, other):
        return ORSet(lib().orc_orset_merge(self._h, other._h))

    def equal(self, other):
        return bool(lib().orc_orset_equal(self._h, other._h))

    def to_list(self, cap=65536):
        out = (C.c_uint32 * cap)()
        k = lib().orc_orset_to_list(self._h, out, cap)
        return list(out[:min(k, cap)])

    def dump(self, cap=65536):
        e, t, a = (C.c_uint32 * cap)(), (C.c_uint64 * cap)(), (C.c_uint8 * cap)()
        k = lib().orc_orset_dump(self._h, e, t, a, cap)
        return [(e[i], t[i], bool(a[i])) for i in range(min(k, cap))]


class FullMembership:
    """Round-synchronous full-membership strategy (oracle/fullmem.c)."""

    def __init__(self, n, periodic_rounds=0):
        self.n = n
        self._h = lib().orc_fm_create(n, periodic_rounds)

    def close(self):
        if self._h:
            lib().orc_fm_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        lib().orc_fm_set_alive(self._h, a.ctypes.data_as(C.POINTER(C.c_uint8)))

    def join(self, v, peer):
        lib().orc_fm_join(self._h, v, peer)

    def leave(self, v, leaving):
        lib().orc_fm_leave(self._h, v, leaving)

    def step(self, rounds=1):
        st = (FmStats * rounds)()
        lib().orc_fm_step(self._h, rounds, st)
        return [x.as_dict() for x in st]

    def inflight(self):
        return lib().orc_fm_inflight(self._h)

    def members(self, v, cap=65536):
        out = (C.c_uint32 * cap)()
        k = lib().orc_fm_members(self._h, v, out, cap)
        return list(out[:min(k, cap)])

    def alive(self, v):
        return bool(lib().orc_fm_alive(self._h, v))

    def payload(self, v):
        """(elem, token, active) rows of node v's state_orset."""
        return _dump_orset(lib().orc_fm_state(self._h, v))

    def messages(self):
        """The wire: [(src, dst, seq, payload rows)] in handling order (dst, src, seq)."""
        k = lib().orc_fm_messages(self._h, None, None, None, 0)
        src, dst, seq = (C.c_uint32 * max(1, k))(), (C.c_uint32 * max(1, k))(), (C.c_uint64 * max(1, k))()
        lib().orc_fm_messages(self._h, src, dst, seq, k)
        return [(src[i], dst[i], seq[i], _dump_orset(lib().orc_fm_message_state(self._h, i))) for i in range(k)]

    def take(self, dst, cap=1 << 16):
        """dst's messages off the wire: [(src, dst, seq, payload rows)] in handling order."""
        src, seq, st = (C.c_uint32 * cap)(), (C.c_uint64 * cap)(), (C.c_void_p * cap)()
        k = lib().orc_fm_take(self._h, dst, src, seq, st, cap)
        assert k <= cap
        out = []
        for i in range(k):
            out.append((src[i], dst, seq[i], _dump_orset(st[i])))
            lib().orc_orset_free(st[i])
        return out

    def put(self, msgs):
        """[(src, dst, seq, payload rows)] onto the wire for the next round."""
        for src, dst, seq, rows in msgs:
            h = lib().orc_orset_new()
            for e, t, a in rows:
                lib().orc_orset_put(h, e, t, 1 if a else 0)
            lib().orc_fm_put(self._h, src, dst, seq, h)
            lib().orc_orset_free(h)


def _dump_orset(h, cap=65536):
    """(elem, token, active) rows of a state_orset handle."""
    e, t, a = (C.c_uint32 * cap)(), (C.c_uint64 * cap)(), (C.c_uint8 * cap)()
    k = lib().orc_orset_dump(h, e, t, a, cap)
    return [(e[i], t[i], bool(a[i])) for i in range(min(k, cap))]


# ---------------------------------------------------------------- SCAMP
class Scamp:
    """Round-synchronous SCAMP v1/v2 membership (oracle/scamp.c)."""

    def __init__(self, n, version=2, c=5, periodic_rounds=10, seed=0):
        self.n = n
        self._h = lib().orc_scamp_create(n, version, c, periodic_rounds, seed)
        if not self._h:
            raise ValueError("bad scamp config")

    def close(self):
        if self._h:
            lib().orc_scamp_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_alive(self, alive):
        a = np.ascontiguousarray(alive, dtype=np.uint8)
        lib().orc_scamp_set_alive(self._h, a.ctypes.data_as(C.POINTER(C.c_uint8)))

    def join(self, v, contact):
        lib().orc_scamp_join(self._h, v, contact)

    def leave(self, v, node):
        lib().orc_scamp_leave(self._h, v, node)

    def crash(self, v):
        lib().orc_scamp_crash(self._h, v)

    def step(self, rounds=1):
        st = (ScampStats * rounds)()
        lib().orc_scamp_step(self._h, rounds, st)
        return [x.as_dict() for x in st]

    def inflight(self):
        return lib().orc_scamp_inflight(self._h)

    def pending(self):
        """Next round's messages as (type, src, dst, seq, a, b) tuples in handling order."""
        n = lib().orc_scamp_pending(self._h, None, 0)
        buf = np.zeros(max(1, 6 * n), np.uint32)
        lib().orc_scamp_pending(self._h, _u32p(buf), n)
        return [tuple(int(x) for x in buf[6 * i:6 * i + 6]) for i in range(n)]

    def view(self, v, which=0, cap=4096):
        out = (C.c_uint32 * cap)()
        k = lib().orc_scamp_view(self._h, v, which, out, cap)
        return list(out[:min(k, cap)])

    def draws(self, v):
        return lib().orc_scamp_draws(self._h, v)

    def alive(self, v):
        return bool(lib().orc_scamp_alive(self._h, v))

    def last_ping(self, v):
        return lib().orc_scamp_last_ping(self._h, v)


# ---------------------------------------------------------------- C3
class C3:
    """Plumtree over churning SCAMP v2 (oracle/c3.c)."""

    def __init__(self, n, c=5, periodic_rounds=10, seed=0):
        self.n = n
        self._h = lib().orc_c3_create(n, c, periodic_rounds, seed)
        self.scamp = Scamp.__new__(Scamp)
        self.scamp.n, self.scamp._h = n, lib().orc_c3_scamp(self._h)
        self.pt = Plumtree.__new__(Plumtree)
        self.pt.n, self.pt._h = n, lib().orc_c3_plumtree(self._h)

    def close(self):
        if self._h:
            self.scamp._h = None   # owned by the composition
            self.pt._h = None
            lib().orc_c3_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def join(self, v, contact):
        lib().orc_c3_join(self._h, v, contact)

    def crash(self, v):
        lib().orc_c3_crash(self._h, v)

    def heartbeat(self, root):
        return lib().orc_c3_heartbeat(self._h, root)

    def step(self, rounds=1):
        st = (C3Stats * rounds)()
        lib().orc_c3_step(self._h, rounds, st)
        return [x.as_dict() for x in st]


def relay_run(act_ptr, act, ol_ptr, ol, alive, src, dst, relay_ttl=5, max_copies=50_000_000, cap=64):
    """Transitive relay (oracle/relay.c): returns (per-round stats dicts, delivered[k], first_round[k])."""
    ap = np.ascontiguousarray(act_ptr, dtype=np.uint64)
    ai = np.ascontiguousarray(act, dtype=np.uint32)
    op = np.ascontiguousarray(ol_ptr, dtype=np.uint64)
    oi = np.ascontiguousarray(ol, dtype=np.uint32)
    al = np.ascontiguousarray(alive, dtype=np.uint8)
    s = np.ascontiguousarray(src, dtype=np.uint32)
    d = np.ascontiguousarray(dst, dtype=np.uint32)
    k = len(s)
    n = len(ap) - 1
    dv = np.zeros(k, dtype=np.uint64)
    fr = np.zeros(k, dtype=np.uint32)
    st = (RelayRound * cap)()
    r = lib().orc_relay_run(n, _u64p(ap), _u32p(ai), _u64p(op), _u32p(oi),
                            al.ctypes.data_as(C.POINTER(C.c_uint8)), k, _u32p(s), _u32p(d), relay_ttl,
                            dv.ctypes.data_as(C.POINTER(C.c_uint64)), _u32p(fr), st, cap, max_copies)
    if r < 0:
        raise ValueError(f"orc_relay_run: {r}")
    rows = [{f: int(getattr(st[i], f)) for f, _ in RelayRound._fields_} for i in range(min(r, cap))]
    return rows, dv, fr

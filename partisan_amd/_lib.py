"""ctypes binding of libpsim.so (include/psim.h).

The library is the product: there is no CPU fallback anywhere in this
package.  If libpsim.so is missing or no gfx950 device is usable, the calls
raise.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PSIM_LIB_PATH") or os.path.join(HERE, "libpsim.so")   # override: kernel experiments

PSIM_ABI_VERSION = 3
PSIM_CFG_BINNED = 1   # psim_config.flags: binned Plumtree engine on one GPU
PSIM_CFG_CSR = 2      # slot-scatter engine keeps CSR rows instead of ELL rows
PSIM_CFG_CHUNK_TIMING = 4   # one hipEvent pair per chunk of rounds instead of per round
ERRORS = {
    0: "PSIM_OK", -1: "PSIM_EINVAL", -2: "PSIM_ENOMEM", -3: "PSIM_EHIP", -4: "PSIM_ERCCL",
    -5: "PSIM_ESTATE", -6: "PSIM_EOVERFLOW", -7: "PSIM_EBUSY", -8: "PSIM_ENODEV", -9: "PSIM_ENOSPC", -10: "PSIM_ENOTSUP",
}
MSG_KINDS = {1: "broadcast", 2: "prune", 3: "i_have", 4: "ignored_i_have", 5: "graft"}


class PsimError(RuntimeError):
    def __init__(self, code, detail=""):
        self.code = code
        self.name = ERRORS.get(code, str(code))
        super().__init__(f"{self.name}: {detail}" if detail else self.name)


class FmMsg(C.Structure):
    _fields_ = [("src", C.c_uint32), ("dst", C.c_uint32), ("seq", C.c_uint32), ("reserved", C.c_uint32)]


class Config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("device", C.c_int32), ("lazy_tick_rounds", C.c_uint32),
                ("exchange_tick_rounds", C.c_uint32), ("flags", C.c_uint32), ("max_roots", C.c_uint32),
                ("seed", C.c_uint64)]


class RoundStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 6), ("delivered_new", C.c_uint64), ("active", C.c_uint64),
                ("senders", C.c_uint64), ("sender_degree_sum", C.c_uint64),
                ("outstanding_vertices", C.c_uint64), ("algo_bytes", C.c_uint64), ("kernel_ms", C.c_double),
                ("words_stored", C.c_uint64)]

    def as_dict(self):
        d = {MSG_KINDS[t]: int(self.sent[t]) for t in range(1, 6)}
        d.update(delivered_new=int(self.delivered_new), active=int(self.active), senders=int(self.senders),
                 sender_degree_sum=int(self.sender_degree_sum),
                 outstanding_vertices=int(self.outstanding_vertices), algo_bytes=int(self.algo_bytes),
                 kernel_ms=float(self.kernel_ms), words_stored=int(self.words_stored))
        return d


class DemersStats(C.Structure):
    _fields_ = [("rm_sent", C.c_uint64), ("push_sent", C.c_uint64), ("pull_sent", C.c_uint64),
                ("delivered_new", C.c_uint64), ("complete", C.c_uint64), ("algo_bytes", C.c_uint64),
                ("kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if k == "kernel_ms" else int(getattr(self, k))) for k, _ in self._fields_}


class HvConfig(C.Structure):
    _fields_ = [(k, C.c_uint32) for k in ("active_max_size", "active_min_size", "active_rwl", "passive_max_size",
                                           "passive_rwl", "shuffle_k_active", "shuffle_k_passive",
                                           "shuffle_rounds", "promotion_rounds")]


HV_MSG_KINDS = {1: "join", 2: "neighbor", 3: "forward_join", 4: "disconnect", 5: "neighbor_request",
                6: "neighbor_rejected", 7: "neighbor_accepted", 8: "shuffle", 9: "shuffle_reply"}


class HvStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 10), ("draws", C.c_uint64), ("error", C.c_uint64), ("processed", C.c_uint64),
                ("active", C.c_uint64), ("algo_bytes", C.c_uint64), ("kernel_ms", C.c_double)]

    def as_dict(self):
        return {"sent": [int(x) for x in self.sent[1:10]], "draws": int(self.draws), "error": int(self.error),
                "processed": int(self.processed), "active": int(self.active), "algo_bytes": int(self.algo_bytes),
                "kernel_ms": float(self.kernel_ms)}


class CausalStats(C.Structure):
    _fields_ = [("emitted", C.c_uint64), ("received", C.c_uint64), ("delivered", C.c_uint64),
                ("checks", C.c_uint64), ("buffered", C.c_uint64), ("algo_bytes", C.c_uint64),
                ("kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if k == "kernel_ms" else int(getattr(self, k))) for k, _ in self._fields_}


class FmStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("sent", "processed", "merges", "updates", "inflight", "member_sum",
                                           "algo_bytes")] + [("kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if k == "kernel_ms" else int(getattr(self, k))) for k, _ in self._fields_}


SCAMP_MSG_KINDS = {1: "forward_subscription", 2: "keep_subscription", 3: "ping", 4: "remove_subscription",
                   5: "replace_subscription", 6: "bootstrap_remove_subscription"}


class ScampMsg(C.Structure):
    """psim_scamp_msg: one membership message on the wire (PSIM_SC_* type, a / b node ids)."""
    _fields_ = [(k, C.c_uint32) for k in ("type", "src", "dst", "seq", "a", "b")]


class ScampStats(C.Structure):
    _fields_ = [("sent", C.c_uint64 * 7)] + [(k, C.c_uint64) for k in (
        "dropped", "processed", "draws", "stopped", "error", "pv_sum", "inview_sum", "resub", "algo_bytes")] + \
        [("kernel_ms", C.c_double)]

    def as_dict(self):
        d = {"sent": [int(x) for x in self.sent[1:7]]}
        for k, _ in self._fields_[1:]:
            d[k] = float(getattr(self, k)) if k == "kernel_ms" else int(getattr(self, k))
        return d


class C3Stats(C.Structure):
    _fields_ = [("scamp", ScampStats), ("pt_sent", C.c_uint64 * 6)] + [(k, C.c_uint64) for k in (
        "pt_dropped", "delivered_new", "active", "updates", "delivered_live", "live", "outstanding_live",
        "pt_algo_bytes")] + [("pt_kernel_ms", C.c_double)]

    def as_dict(self):
        d = {"scamp": self.scamp.as_dict(), "pt_sent": {MSG_KINDS[t]: int(self.pt_sent[t]) for t in range(1, 6)}}
        for k, _ in self._fields_[2:]:
            d[k] = float(getattr(self, k)) if k == "pt_kernel_ms" else int(getattr(self, k))
        return d


class ExchangeStats(C.Structure):
    _fields_ = [("rounds", C.c_uint64), ("fabric_bytes", C.c_uint64), ("exchange_ms", C.c_double),
                ("kernel_ms", C.c_double)]

    def as_dict(self):
        return {k: (float(getattr(self, k)) if k.endswith("_ms") else int(getattr(self, k))) for k, _ in self._fields_}


# psim_transport callbacks (include/psim.h): all-to-all-v of u32 words over host buffers, int64 sum all-reduce
ALLTOALLV_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint32),
                           C.POINTER(C.c_uint64), C.c_int)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_size_t)


class Transport(C.Structure):
    _fields_ = [("ctx", C.c_void_p), ("alltoallv", ALLTOALLV_FN), ("allreduce", ALLREDUCE_FN)]


PSIM_RCCL_ID_BYTES = 128


# every entry point of include/psim.h: name -> (restype, argtypes)
class RelayStats(C.Structure):
    _fields_ = [(k, C.c_uint64) for k in ("direct", "relay", "dropped", "lost", "arrived")]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_P = C.POINTER
_H = C.c_void_p
SIGNATURES = {
    "psim_create": (C.c_int, [_P(Config), _P(C.c_void_p)]),
    "psim_destroy": (C.c_int, [_H]),
    "psim_strerror": (C.c_char_p, [C.c_int]),
    "psim_last_error": (C.c_char_p, [_H]),
    "psim_device_info": (C.c_int, [_H, C.c_char_p, C.c_size_t]),
    "psim_load_csr": (C.c_int, [_H, C.c_uint32, _P(C.c_uint64), _P(C.c_uint32), C.c_uint64]),
    "psim_num_slots": (C.c_int, [_H, _P(C.c_uint64)]),
    "psim_get_slots": (C.c_int, [_H, _P(C.c_uint64), _P(C.c_uint32)]),
    "psim_set_alive": (C.c_int, [_H, _P(C.c_uint8), C.c_size_t]),
    "psim_plumtree_reset_trees": (C.c_int, [_H]),
    "psim_plumtree_restart_backend": (C.c_int, [_H, C.c_uint32]),
    "psim_plumtree_broadcast": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32)]),
    "psim_plumtree_broadcast_many": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t, _P(C.c_uint32)]),
    "psim_plumtree_broadcast_run": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), C.c_uint32, _P(RoundStats), C.c_size_t,
                                              _P(C.c_uint32)]),
    "psim_plumtree_broadcast_run_n": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P(RoundStats),
                                                C.c_size_t, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32)]),
    "psim_step": (C.c_int, [_H, C.c_uint32, _P(RoundStats), C.c_size_t]),
    "psim_run": (C.c_int, [_H, C.c_uint32, _P(RoundStats), C.c_size_t, _P(C.c_uint32)]),
    "psim_get_plumtree": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint16),
                                    C.c_size_t]),
    "psim_get_delivered": (C.c_int, [_H, _P(C.c_uint8), C.c_size_t]),
    "psim_get_inflight": (C.c_int, [_H, _P(C.c_uint32), C.c_uint64]),
    "psim_trace_hash": (C.c_int, [_H, _P(C.c_uint64)]),
    "psim_plumtree_focus": (C.c_int, [_H, C.c_uint32]),
    "psim_forest_set_lanes": (C.c_int, [_H, C.c_uint32]),
    "psim_set_omissions": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_set_delays": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint8), C.c_size_t]),
    "psim_get_messages": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32),
                                    _P(C.c_uint32), C.c_size_t, _P(C.c_size_t)]),
    "psim_get_rows": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t,
                                _P(C.c_size_t)]),
    "psim_get_delivered_mono": (C.c_int, [_H, C.c_uint32, _P(C.c_uint8), C.c_size_t]),
    "psim_get_delivered_range": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_size_t, _P(C.c_uint8)]),
    "psim_get_timing": (C.c_int, [_H, _P(C.c_double), _P(C.c_uint64)]),
    "psim_set_chunk_timing": (C.c_int, [_H, C.c_int]),
    "psim_shard_init": (C.c_int, [_H, C.c_int, C.c_int]),
    "psim_shard_info": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint64), _P(C.c_uint32)]),
    "psim_shard_layout": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_shard_broadcast": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), C.c_void_p, C.c_uint64, _P(C.c_uint64),
                                       _P(C.c_int64)]),
    "psim_shard_round": (C.c_int, [_H, C.c_void_p, C.c_uint64, _P(C.c_uint64), _P(RoundStats), _P(C.c_int64)]),
    "psim_shard_ingest": (C.c_int, [_H, C.c_void_p, C.c_uint64]),
    "psim_set_stream": (C.c_int, [_H, C.c_void_p]),
    "psim_shard_recv_layout": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_shard_broadcast_dense": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), C.c_void_p]),
    "psim_shard_round_async": (C.c_int, [_H, C.c_void_p]),
    "psim_shard_ingest_dense": (C.c_int, [_H, C.c_void_p]),
    "psim_shard_collect": (C.c_int, [_H, _P(RoundStats), C.c_size_t, _P(C.c_uint32), _P(C.c_int64)]),
    "psim_shard_uncount": (C.c_int, [_H, C.c_uint32]),
    "psim_rccl_unique_id": (C.c_int, [_P(C.c_uint8)]),
    "psim_shard_init_rccl": (C.c_int, [_H, C.c_int, C.c_int, _P(C.c_uint8)]),
    "psim_shard_set_transport": (C.c_int, [_H, _P(Transport)]),
    "psim_shard_transport_info": (C.c_int, [_H, _P(C.c_int), _P(C.c_int), _P(C.c_int)]),
    "psim_shard_broadcast_x": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32)]),
    "psim_shard_run": (C.c_int, [_H, C.c_uint32, _P(RoundStats), C.c_size_t, _P(C.c_uint32), _P(ExchangeStats)]),
    "psim_shard_step": (C.c_int, [_H, C.c_uint32, _P(RoundStats), C.c_size_t, _P(ExchangeStats)]),
    "psim_demers_setup": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "psim_demers_broadcast_all": (C.c_int, [_H]),
    "psim_demers_step": (C.c_int, [_H, C.c_uint32, _P(DemersStats), C.c_size_t]),
    "psim_demers_run": (C.c_int, [_H, C.c_uint32, _P(DemersStats), C.c_size_t, _P(C.c_uint32)]),
    "psim_demers_get_seen": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_demers_origins": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t]),
    "psim_demers_shard_setup": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.c_int,
                                          _P(C.c_uint64)]),
    "psim_demers_shard_info": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint64)]),
    "psim_demers_shard_broadcast_all": (C.c_int, [_H, C.c_void_p, C.c_void_p]),
    "psim_demers_shard_round": (C.c_int, [_H, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, _P(DemersStats),
                                          _P(C.c_uint32)]),
    "psim_demers_shard_ingest": (C.c_int, [_H, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "psim_demers_shard_broadcast_x": (C.c_int, [_H]),
    "psim_demers_shard_step": (C.c_int, [_H, C.c_uint32, _P(DemersStats), C.c_size_t]),
    "psim_demers_shard_run": (C.c_int, [_H, C.c_uint32, _P(DemersStats), C.c_size_t, _P(C.c_uint32)]),
    "psim_demers_shard_set_exchange": (C.c_int, [_H, C.c_int]),
    "psim_demers_shard_exchange_stats": (C.c_int, [_H, _P(C.c_uint64), _P(C.c_uint32), _P(C.c_uint32),
                                                   _P(C.c_uint32)]),
    "psim_demers_shard_get_seen": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_hv_setup": (C.c_int, [_H, C.c_uint32, _P(HvConfig)]),
    "psim_hv_set_alive": (C.c_int, [_H, _P(C.c_uint8), C.c_size_t]),
    "psim_hv_join": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_hv_step": (C.c_int, [_H, C.c_uint32, _P(HvStats), C.c_size_t]),
    "psim_hv_join_seq": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t, C.c_uint32, _P(HvStats), C.c_size_t]),
    "psim_hv_get_views": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint8), _P(C.c_uint32), _P(C.c_uint8), C.c_size_t]),
    "psim_hv_get_draws": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_hv_get_idmap": (C.c_int, [_H, C.c_uint32, C.c_int, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32),
                                    C.c_size_t, _P(C.c_size_t)]),
    "psim_hv_inflight": (C.c_int, [_H, _P(C.c_uint64)]),
    "psim_causal_setup": (C.c_int, [_H] + [C.c_uint32] * 5),
    "psim_causal_step": (C.c_int, [_H, C.c_uint32, _P(CausalStats), C.c_size_t]),
    "psim_causal_get_clocks": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_causal_get_buffered": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t,
                                           _P(C.c_size_t)]),
    "psim_causal_get_delivered": (C.c_int, [_H, _P(C.c_uint64), C.c_size_t]),
    "psim_causal_emitters": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t]),
    "psim_causal_shard_setup": (C.c_int, [_H] + [C.c_uint32] * 5 + [C.c_int, C.c_int]),
    "psim_causal_shard_info": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32)]),
    "psim_causal_shard_round": (C.c_int, [_H, C.c_void_p, _P(CausalStats)]),
    "psim_causal_shard_ingest": (C.c_int, [_H, C.c_void_p]),
    "psim_causal_shard_step": (C.c_int, [_H, C.c_uint32, _P(CausalStats), C.c_size_t]),
    "psim_fm_setup": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32]),
    "psim_fm_set_alive": (C.c_int, [_H, _P(C.c_uint8), C.c_size_t]),
    "psim_fm_join": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_fm_leave": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_fm_step": (C.c_int, [_H, C.c_uint32, _P(FmStats), C.c_size_t]),
    "psim_fm_get_state": (C.c_int, [_H, _P(C.c_uint64), _P(C.c_uint64), _P(C.c_uint8), C.c_size_t, C.c_size_t]),
    "psim_fm_tokens": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t, _P(C.c_uint32)]),
    "psim_fm_inflight": (C.c_int, [_H, _P(C.c_uint64)]),
    "psim_fm_messages": (C.c_int, [_H, _P(FmMsg), _P(C.c_uint64), _P(C.c_uint64), C.c_size_t, C.c_size_t,
                              _P(C.c_size_t)]),
    "psim_fm_take": (C.c_int, [_H, C.c_uint32, _P(FmMsg), _P(C.c_uint64), _P(C.c_uint64), C.c_size_t, C.c_size_t,
                          _P(C.c_size_t)]),
    "psim_fm_put": (C.c_int, [_H, _P(FmMsg), _P(C.c_uint64), _P(C.c_uint64), C.c_size_t, C.c_size_t]),
    "psim_scamp_setup": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]),
    "psim_scamp_set_alive": (C.c_int, [_H, _P(C.c_uint8), C.c_size_t]),
    "psim_scamp_join": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_scamp_leave": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_scamp_crash": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t]),
    "psim_scamp_step": (C.c_int, [_H, C.c_uint32, _P(ScampStats), C.c_size_t]),
    "psim_scamp_get_views": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32),
                                       C.c_size_t]),
    "psim_scamp_get_nodes": (C.c_int, [_H, _P(C.c_uint64), _P(C.c_int32), _P(C.c_uint8), C.c_size_t]),
    "psim_scamp_inflight": (C.c_int, [_H, _P(C.c_uint64)]),
    "psim_scamp_messages": (C.c_int, [_H, _P(ScampMsg), C.c_size_t, _P(C.c_size_t)]),
    "psim_scamp_take": (C.c_int, [_H, C.c_uint32, _P(ScampMsg), C.c_size_t, _P(C.c_size_t)]),
    "psim_scamp_put": (C.c_int, [_H, _P(ScampMsg), C.c_size_t]),
    "psim_c3_setup": (C.c_int, [_H, C.c_uint32, C.c_uint32, C.c_uint32]),
    "psim_c3_join": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_c3_crash": (C.c_int, [_H, _P(C.c_uint32), C.c_size_t]),
    "psim_c3_heartbeat": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32)]),
    "psim_c3_step": (C.c_int, [_H, C.c_uint32, _P(C3Stats), C.c_size_t]),
    "psim_c3_run": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32),
                              _P(C.c_uint32), C.c_uint32, C.c_uint32, _P(C3Stats), C.c_size_t]),
    "psim_c3_get_plumtree": (C.c_int, [_H, C.c_uint32, _P(C.c_uint32), _P(C.c_size_t), _P(C.c_uint32),
                                       _P(C.c_size_t), _P(C.c_uint32), _P(C.c_size_t), C.c_size_t,
                                       _P(C.c_uint32), _P(C.c_uint32)]),
    "psim_vclock_descends": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint8), C.c_size_t]),
    "psim_vclock_dominates": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint8), C.c_size_t]),
    "psim_vclock_merge": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_vclock_increment": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_vclock_equal": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint8), C.c_size_t]),
    "psim_vclock_glb": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_vclock_subtract_dots": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_vclock_get_counter": (C.c_int, [_H, _P(C.c_uint32), _P(C.c_uint32), _P(C.c_uint32), C.c_size_t]),
    "psim_relay_run": (C.c_int64, [_H, C.c_uint32, _P(C.c_uint64), _P(C.c_uint32), C.c_uint64, _P(C.c_uint64),
                                   _P(C.c_uint32), C.c_uint64, _P(C.c_uint8), C.c_uint32, _P(C.c_uint32), _P(C.c_uint32), C.c_uint32,
                                   _P(C.c_uint64), _P(C.c_uint32), _P(RelayStats), C.c_size_t, C.c_size_t]),
}

_lib = None


def lib():
    """Load libpsim.so once; raise loudly if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; "
                              f"g.build()'` (hipcc --offload-arch=gfx950)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("PSIM_LIB_PATH") and not hasattr(L, name):
                continue            # an older experiment build: bind what it exports
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, h=None):
    if rc != 0:
        raise PsimError(rc, lib().psim_last_error(h).decode())
    return rc

"""Deterministic overlay generators (membership CSR: row_ptr u64[n+1], col u32).

* random_regular: HyParView-shaped overlay for the large benches -- every
  vertex gets `peers` random symmetric neighbours (configuration model with
  self-loops and multi-edges dropped), i.e. an active view of at most
  `active_max_size - 1` = 5 peers (partisan.hrl:204-217).  Building
  10M-peer views by simulated joins is the HyParView row of SURVEY 8; this
  generator only supplies the topology for the Plumtree hot path.
* complete: full membership (config C1: every member eager, Q1).
* from_edges: symmetric CSR from an undirected edge list.
"""
import numpy as np


def _csr_from_directed(n, src, dst):
    order = np.argsort(src, kind="stable")
    col = dst[order].astype(np.uint32)
    counts = np.bincount(src, minlength=n)
    row_ptr = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(counts, out=row_ptr[1:])
    return row_ptr, col


def from_edges(n, a, b):
    """Symmetric membership CSR for undirected edges {a[i], b[i]}."""
    a = np.asarray(a, dtype=np.int64)
    b = np.asarray(b, dtype=np.int64)
    src = np.concatenate([a, b])
    dst = np.concatenate([b, a])
    return _csr_from_directed(n, src, dst)


def random_regular(n, peers=5, seed=0):
    """Random symmetric overlay, degree <= peers (mostly == peers)."""
    rng = np.random.default_rng(seed)
    stubs = np.repeat(np.arange(n, dtype=np.int64), peers)
    rng.shuffle(stubs)
    stubs = stubs[: len(stubs) // 2 * 2]
    a, b = stubs[0::2], stubs[1::2]
    keep = a != b
    a, b = a[keep], b[keep]
    lo, hi = np.minimum(a, b), np.maximum(a, b)
    key = np.unique(lo * n + hi)
    return from_edges(n, key // n, key % n)


def complete(n):
    """Every vertex lists every other vertex (full membership)."""
    src = np.repeat(np.arange(n, dtype=np.int64), n)
    dst = np.tile(np.arange(n, dtype=np.int64), n)
    keep = src != dst
    return _csr_from_directed(n, src[keep], dst[keep])


def ring_lattice(n, k=2):
    """Each vertex connected to its k nearest successors (and predecessors)."""
    a = np.repeat(np.arange(n, dtype=np.int64), k)
    b = (a + np.tile(np.arange(1, k + 1, dtype=np.int64), n)) % n
    return from_edges(n, a, b)


# ---------------------------------------------------------------- workload draws
_PHILOX_M0, _PHILOX_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_PHILOX_W0, _PHILOX_W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32_10(c0, c1, c2, c3, seed):
    """Vectorised Philox4x32-10 (Random123), the simulation's RNG, for host-side
    workload generation (crash lists, contacts).  Arrays of uint32 counters."""
    m = np.uint64(0xFFFFFFFF)
    x = [np.asarray(c, dtype=np.uint64) & m for c in (c0, c1, c2, c3)]
    x = list(np.broadcast_arrays(*x))
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for r in range(10):
        p0 = _PHILOX_M0 * x[0]
        p1 = _PHILOX_M1 * x[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & m
        hi1, lo1 = p1 >> np.uint64(32), p1 & m
        x = [(hi1 ^ x[1] ^ k0) & m, lo1, (hi0 ^ x[3] ^ k1) & m, lo0]
        k0 = (k0 + np.uint64(_PHILOX_W0)) & m
        k1 = (k1 + np.uint64(_PHILOX_W1)) & m
    return [a.astype(np.uint32) for a in x]


def philox_uniform(seed, ctr, kind, n):
    """floor(r * n / 2^64) for the 64-bit draw r of counter {ctr, 0, kind, 0}."""
    ctr = np.asarray(ctr, dtype=np.uint64)
    r = philox4x32_10(ctr, 0, kind, 0, seed)
    lo, hi = r[0].astype(np.uint64), r[1].astype(np.uint64)
    n64 = np.uint64(n)
    # mulhi(hi:lo * n) without 128-bit ints: (hi*n + (lo*n >> 32)) >> 32
    t = hi * n64 + ((lo * n64) >> np.uint64(32))
    return (t >> np.uint64(32)).astype(np.uint32)

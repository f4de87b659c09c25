"""partisan_amd -- MI355X-native round-synchronous simulator of the gossip hot
path of loong/partisan (Plumtree eager/lazy push with graft/prune, heartbeat
handler), driven through the C ABI of libpsim.so (include/psim.h).

Importing this package loads libpsim.so and fails loudly if it is absent.
"""
from ._lib import PsimError, lib  # noqa: F401  (loads libpsim.so now)
from .sim import Simulator  # noqa: F401
from . import c3, causal, demers, fullmem, hyparview, membership, overlay, relay, scamp, vclock  # noqa: F401
from .plumtree import PlumtreeBackend, PlumtreeBroadcast, PlumtreeBroadcastHandler  # noqa: F401

lib()

%% partisan_gpu_sim -- Erlang binding of libpsim.so through the NIF in
%% ../c_src/partisan_gpu_sim_nif.c.  Every function is replaced by the NIF
%% at load time; the bodies below only run if the NIF failed to load.
%%
%% Binary conventions: vertex ids and masks are little-endian u32, row
%% pointers u64, byte maps one byte per vertex (see include/psim.h).
-module(partisan_gpu_sim).

-export([new/1, load_csr/3, set_alive/2, reset_trees/1, restart_backend/2, broadcast/2, broadcast_many/2,
         step/2, run/2, broadcast_run/3, broadcast_run_n/5,
         peers/1, slots/1, delivered/1, trace_hash/1, focus/2, set_omissions/3, set_delays/4, delivered_mono/2, is_delivered/3, rows/2, messages/1, shard_step/2,
         relay_run/10,
         hv_setup/3, hv_join/3, hv_step/2, hv_views/1,
         demers_setup/5, demers_run/2,
         vclock/4,
         scamp_setup/5, scamp_join/3, scamp_leave/3, scamp_crash/2, scamp_step/2, scamp_views/1,
         scamp_messages/1, scamp_messages_from/2, scamp_take/2, scamp_put/2,
         fm_setup/4, fm_join/3, fm_leave/3, fm_step/2, fm_state/1, fm_tokens/1,
         fm_messages/1, fm_messages_from/2, fm_take/2, fm_put/2,
         c3_setup/4, c3_join/3, c3_crash/2, c3_heartbeat/2, c3_step/2, c3_run/8,
         causal_setup/6, causal_step/2, causal_clocks/1,
         rccl_unique_id/0, shard_init_rccl/4, shard_broadcast/2, shard_run/2,
         demers_shard_setup/7, demers_shard_run/2, causal_shard_setup/8, causal_shard_step/2]).
-export([active_views/1, csr_from_views/1]).

-on_load(init/0).

-type sim() :: reference().
-type error() :: {error, einval | enomem | ehip | erccl | estate | eoverflow | ebusy | enodev | psim_error}.
-export_type([sim/0]).

init() ->
    Dir = case code:priv_dir(partisan) of
              {error, bad_name} -> filename:join(filename:dirname(code:which(?MODULE)), "../priv");
              D -> D
          end,
    erlang:load_nif(filename:join(Dir, "partisan_gpu_sim"), 0).

-spec new(#{device => integer(), seed => non_neg_integer(), lazy_tick_rounds => pos_integer(),
            max_roots => non_neg_integer(), forest_lanes => non_neg_integer(),
            exchange_tick_rounds => pos_integer()}) -> {ok, sim()} | error().
new(_Opts) -> erlang:nif_error(nif_not_loaded).

-spec load_csr(sim(), binary(), binary()) -> ok | error().
load_csr(_Sim, _RowPtr, _Col) -> erlang:nif_error(nif_not_loaded).

-spec set_alive(sim(), binary()) -> ok | error().
set_alive(_Sim, _Alive) -> erlang:nif_error(nif_not_loaded).

-spec reset_trees(sim()) -> ok | error().
reset_trees(_Sim) -> erlang:nif_error(nif_not_loaded).

%% Vertex's heartbeat backend restarts (backend init/1): newer epoch,
%% Monotonic 0, empty timestamp table.  Ids are Epoch bsl 24 bor Monotonic.
-spec restart_backend(sim(), non_neg_integer()) -> ok | error().
restart_backend(_Sim, _V) -> erlang:nif_error(nif_not_loaded).

%% {ok, Id}: Id = Epoch bsl 24 bor Monotonic (Epoch 0 until a restart)
-spec broadcast(sim(), non_neg_integer()) -> {ok, non_neg_integer()} | error().
broadcast(_Sim, _Root) -> erlang:nif_error(nif_not_loaded).

%% Heartbeats from every listed root at once (the backend's timer firing at
%% each node, partisan_plumtree_backend.erl:341-368): Roots and the returned
%% Ids are u32-little binaries.  On a handle created with max_roots > 16 (the
%% forest) every root's trees are kept: {error, enospc} past max_roots,
%% {error, ebusy} for a root whose last heartbeat is still in flight.
-spec broadcast_many(sim(), binary()) -> {ok, binary()} | error().
broadcast_many(_Sim, _Roots) -> erlang:nif_error(nif_not_loaded).

-spec step(sim(), pos_integer()) -> {ok, [map()]} | error().
step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).

-spec run(sim(), pos_integer()) -> {ok, non_neg_integer(), [map()]} | error().
run(_Sim, _MaxRounds) -> erlang:nif_error(nif_not_loaded).
%% one heartbeat interval of one root: broadcast/2 then run/2 in one call
-spec broadcast_run(sim(), non_neg_integer(), pos_integer()) ->
    {ok, non_neg_integer(), non_neg_integer(), [map()]} | error().
broadcast_run(_Sim, _Root, _MaxRounds) -> erlang:nif_error(nif_not_loaded).
%% Count heartbeat intervals of one root back to back (reset_trees/1 before
%% each when Reset is 1): the same as Count broadcast_run/3 calls
-spec broadcast_run_n(sim(), non_neg_integer(), pos_integer(), 0 | 1, pos_integer()) ->
    {ok, [{non_neg_integer(), non_neg_integer()}], [map()]} | error().
broadcast_run_n(_Sim, _Root, _Count, _Reset, _MaxRounds) -> erlang:nif_error(nif_not_loaded).

-spec peers(sim()) -> {ok, binary(), binary(), binary(), binary()} | error().
peers(_Sim) -> erlang:nif_error(nif_not_loaded).

-spec slots(sim()) -> {ok, binary(), binary()} | error().
slots(_Sim) -> erlang:nif_error(nif_not_loaded).

-spec delivered(sim()) -> {ok, binary()} | error().
delivered(_Sim) -> erlang:nif_error(nif_not_loaded).

%% Point the per-vertex getters at Root's heartbeat lane (psim_plumtree_focus).
-spec focus(sim(), non_neg_integer()) -> ok | error().
focus(_Sim, _Root) -> erlang:nif_error(nif_not_loaded).

%% Omission faults on directed pairs: native-endian u32 binaries (psim_set_omissions).
-spec set_omissions(sim(), binary(), binary()) -> ok | error().
set_omissions(_Sim, _Src, _Dst) -> erlang:nif_error(nif_not_loaded).

%% Delay faults on directed pairs (psim_set_delays): Src / Dst native-endian
%% u32 binaries, Rounds one byte per pair; refused while messages are in flight.
-spec set_delays(sim(), binary(), binary(), binary()) -> ok | error().
set_delays(_Sim, _Src, _Dst, _Rounds) -> erlang:nif_error(nif_not_loaded).

%% Mod:is_stale({Root, Epoch, Mono}) per vertex of the focused root, any
%% heartbeat of a window lane (psim_get_delivered_mono).
-spec delivered_mono(sim(), non_neg_integer()) -> {ok, binary()} | error().
delivered_mono(_Sim, _Mono) -> erlang:nif_error(nif_not_loaded).

%% Mod:is_stale/1 at ONE vertex of the focused root (Mono 0: the newest
%% heartbeat): psim_get_delivered_range over one vertex, no whole-set copy.
-spec is_delivered(sim(), non_neg_integer(), non_neg_integer()) -> {ok, boolean()} | error().
is_delivered(_Sim, _V, _Mono) -> erlang:nif_error(nif_not_loaded).

%% Vertex V's outstanding i_have rows {Peer, Round, Mono} in insertion order.
-spec rows(sim(), non_neg_integer()) -> {ok, [{non_neg_integer(), non_neg_integer(), non_neg_integer()}]} | error().
rows(_Sim, _V) -> erlang:nif_error(nif_not_loaded).

%% The next round's messages {Src, Dst, Kind, Round, Mono} in handling order.
-spec messages(sim()) -> {ok, [tuple()]} | error().
messages(_Sim) -> erlang:nif_error(nif_not_loaded).

%% Exactly Rounds collective rounds of a sharded handle (psim_shard_step).
-spec shard_step(sim(), non_neg_integer()) -> {ok, [map()], tuple()} | error().
shard_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).

%% Transitive relay (psim_relay_run): forward_message(Node, Message,
%% #{transitive => true}) for a batch of sends over active views (ActPtr u64 /
%% Act u32 binaries) and out-links (OlPtr / Ol), Alive one byte per vertex.
%% Returns the rounds run, per-round {Direct, Relay, Dropped, Lost, Arrived},
%% copies delivered per send (u64 binary) and first arrival rounds (u32).
-spec relay_run(sim(), binary(), binary(), binary(), binary(), binary(), binary(), binary(),
                pos_integer(), pos_integer()) ->
    {ok, non_neg_integer(), [tuple()], binary(), binary()} | error().
relay_run(_Sim, _ActPtr, _Act, _OlPtr, _Ol, _Alive, _Src, _Dst, _RelayTTL, _MaxCopies) ->
    erlang:nif_error(nif_not_loaded).

%% Order-independent digest of the Plumtree state (psim_trace_hash).
-spec trace_hash(sim()) -> {ok, {non_neg_integer(), non_neg_integer(), non_neg_integer(), non_neg_integer()}} | error().
trace_hash(_Sim) -> erlang:nif_error(nif_not_loaded).

-spec hv_setup(sim(), pos_integer(), map()) -> ok | error().
hv_setup(_Sim, _N, _Config) -> erlang:nif_error(nif_not_loaded).

-spec hv_join(sim(), binary(), binary()) -> ok | error().
hv_join(_Sim, _Joiners, _Contacts) -> erlang:nif_error(nif_not_loaded).

-spec hv_step(sim(), pos_integer()) -> {ok, [map()]} | error().
hv_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).

-spec hv_views(sim()) -> {ok, binary(), binary(), binary(), binary()} | error().
hv_views(_Sim) -> erlang:nif_error(nif_not_loaded).

-spec demers_setup(sim(), pos_integer(), 1..64, non_neg_integer(), boolean()) -> ok | error().
demers_setup(_Sim, _N, _M, _AePeriod, _RumorMongering) -> erlang:nif_error(nif_not_loaded).

-spec demers_run(sim(), pos_integer()) -> {ok, non_neg_integer(), binary()} | error().
demers_run(_Sim, _MaxRounds) -> erlang:nif_error(nif_not_loaded).

%% partisan_vclock on dense 64-lane clocks: B is a clock binary, or u32 actor
%% lanes for increment / get_counter; descends / dominates / equal return one
%% byte per clock, get_counter one u32 per clock, the others clocks.
-spec vclock(sim(), descends | dominates | equal | merge | glb | subtract_dots | increment | get_counter,
             binary(), binary()) -> {ok, binary()} | error().
vclock(_Sim, _Op, _A, _B) -> erlang:nif_error(nif_not_loaded).

%% ---- SCAMP v1 / v2 (psim_scamp_*): joins / leaves / crashes are u32 binaries,
%% handled by the next round; views are rows of 128 (partial) and 64 (in-view)
%% u32 ids in the reference's list order, with u32 lengths.
-spec scamp_setup(sim(), pos_integer(), 1 | 2, pos_integer(), pos_integer()) -> ok | error().
scamp_setup(_Sim, _N, _Version, _C, _PeriodicRounds) -> erlang:nif_error(nif_not_loaded).
-spec scamp_join(sim(), binary(), binary()) -> ok | error().
scamp_join(_Sim, _Joiners, _Contacts) -> erlang:nif_error(nif_not_loaded).
-spec scamp_leave(sim(), binary(), binary()) -> ok | error().
scamp_leave(_Sim, _Vs, _Leaving) -> erlang:nif_error(nif_not_loaded).
-spec scamp_crash(sim(), binary()) -> ok | error().
scamp_crash(_Sim, _Vs) -> erlang:nif_error(nif_not_loaded).
-spec scamp_step(sim(), pos_integer()) -> {ok, [map()]} | error().
scamp_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
-spec scamp_views(sim()) -> {ok, binary(), binary(), binary(), binary()} | error().
scamp_views(_Sim) -> erlang:nif_error(nif_not_loaded).

%% The membership messages on the wire: {Src, Dst, Seq, {membership_strategy,
%% Msg}} with Msg in partisan_scamp_v2_membership_strategy's own shapes
%% ({forward_subscription, A}, {replace_subscription, A, B}, ...; vertex ids).
-type wire_msg() :: {non_neg_integer(), non_neg_integer(), non_neg_integer(), {membership_strategy, tuple()}}.
%% the next round's messages in handling order (dst, src, seq)
-spec scamp_messages(sim()) -> {ok, [wire_msg()]} | error().
scamp_messages(_Sim) -> erlang:nif_error(nif_not_loaded).

%% scamp_messages/1 restricted to the messages sent by Src (filtered in the NIF).
-spec scamp_messages_from(sim(), non_neg_integer()) -> {ok, [wire_msg()]} | error().
scamp_messages_from(_Sim, _Src) -> erlang:nif_error(nif_not_loaded).
%% takes Dst's messages off the wire (the next round does not deliver them)
-spec scamp_take(sim(), non_neg_integer()) -> {ok, [wire_msg()]} | error().
scamp_take(_Sim, _Dst) -> erlang:nif_error(nif_not_loaded).
%% puts messages on the wire for the next round (a node's handle_message/2)
-spec scamp_put(sim(), [wire_msg()]) -> ok | error().
scamp_put(_Sim, _Msgs) -> erlang:nif_error(nif_not_loaded).

%% ---- full membership (psim_fm_*): state_orset token bitmaps per node ----------
-spec fm_setup(sim(), pos_integer(), pos_integer(), pos_integer()) -> ok | error().
fm_setup(_Sim, _N, _PeriodicRounds, _MaxTokens) -> erlang:nif_error(nif_not_loaded).
-spec fm_join(sim(), binary(), binary()) -> ok | error().
fm_join(_Sim, _Vs, _Peers) -> erlang:nif_error(nif_not_loaded).
-spec fm_leave(sim(), binary(), binary()) -> ok | error().
fm_leave(_Sim, _Vs, _Leaving) -> erlang:nif_error(nif_not_loaded).
-spec fm_step(sim(), pos_integer()) -> {ok, [map()]} | error().
fm_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
-spec fm_state(sim()) -> {ok, binary(), binary(), binary()} | error().
fm_state(_Sim) -> erlang:nif_error(nif_not_loaded).
-spec fm_tokens(sim()) -> {ok, binary(), non_neg_integer()} | error().
fm_tokens(_Sim) -> erlang:nif_error(nif_not_loaded).

%% The full-membership gossip on the wire (psim_fm_messages / _take / _put):
%% [{Src, Dst, Seq, Known, Removed}] in handling order, Known / Removed the
%% message's state_orset as little-endian u64 token bitmaps.
-spec fm_messages(sim()) -> {ok, [{non_neg_integer(), non_neg_integer(), non_neg_integer(), binary(), binary()}]} | error().
fm_messages(_Sim) -> erlang:nif_error(nif_not_loaded).

%% fm_messages/1 restricted to the messages sent by Src (filtered in the NIF).
-spec fm_messages_from(sim(), non_neg_integer()) -> {ok, [{non_neg_integer(), non_neg_integer(), non_neg_integer(), binary(), binary()}]} | error().
fm_messages_from(_Sim, _Src) -> erlang:nif_error(nif_not_loaded).
-spec fm_take(sim(), non_neg_integer()) ->
          {ok, [{non_neg_integer(), non_neg_integer(), non_neg_integer(), binary(), binary()}]} | error().
fm_take(_Sim, _Dst) -> erlang:nif_error(nif_not_loaded).
-spec fm_put(sim(), [{non_neg_integer(), non_neg_integer(), non_neg_integer(), binary(), binary()}]) -> ok | error().
fm_put(_Sim, _Msgs) -> erlang:nif_error(nif_not_loaded).

%% ---- C3: Plumtree over churning SCAMP v2 (psim_c3_*) -------------------------
-spec c3_setup(sim(), pos_integer(), pos_integer(), pos_integer()) -> ok | error().
c3_setup(_Sim, _N, _C, _PeriodicRounds) -> erlang:nif_error(nif_not_loaded).
-spec c3_join(sim(), binary(), binary()) -> ok | error().
c3_join(_Sim, _Joiners, _Contacts) -> erlang:nif_error(nif_not_loaded).
-spec c3_crash(sim(), binary()) -> ok | error().
c3_crash(_Sim, _Vs) -> erlang:nif_error(nif_not_loaded).
-spec c3_heartbeat(sim(), non_neg_integer()) -> {ok, non_neg_integer()} | error().
c3_heartbeat(_Sim, _Root) -> erlang:nif_error(nif_not_loaded).
-spec c3_step(sim(), pos_integer()) -> {ok, [{map(), map()}]} | error().
c3_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
%% R churn rounds in one call (psim_c3_run): offsets are <<u32>> of R + 1 entries
-spec c3_run(sim(), binary(), binary(), binary(), binary(), binary(), non_neg_integer(), non_neg_integer()) ->
          {ok, [{map(), map()}]} | error().
c3_run(_Sim, _CrashOff, _CrashV, _JoinOff, _JoinV, _JoinC, _HbEvery, _Root) -> erlang:nif_error(nif_not_loaded).

%% ---- causal delivery (psim_causal_*) ------------------------------------------
-spec causal_setup(sim(), pos_integer(), 1..64, pos_integer(), pos_integer(), pos_integer()) -> ok | error().
causal_setup(_Sim, _N, _M, _Period, _DMax, _Redeliver) -> erlang:nif_error(nif_not_loaded).
-spec causal_step(sim(), pos_integer()) -> {ok, [map()]} | error().
causal_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).
-spec causal_clocks(sim()) -> {ok, binary(), binary()} | error().
causal_clocks(_Sim) -> erlang:nif_error(nif_not_loaded).

%% ---- vertex sharding with the library's own RCCL communicator --------------------
%% One BEAM per GPU: rank 0 calls rccl_unique_id/0 and ships the id to the
%% other ranks (e.g. erpc); each calls shard_init_rccl/4 before load_csr/3;
%% shard_broadcast/2 and shard_run/2 are collective.
-spec rccl_unique_id() -> {ok, binary()} | error().
rccl_unique_id() -> erlang:nif_error(nif_not_loaded).
-spec shard_init_rccl(sim(), non_neg_integer(), pos_integer(), binary()) -> ok | error().
shard_init_rccl(_Sim, _Rank, _World, _Id) -> erlang:nif_error(nif_not_loaded).
-spec shard_broadcast(sim(), non_neg_integer()) -> {ok, non_neg_integer()} | error().
shard_broadcast(_Sim, _Root) -> erlang:nif_error(nif_not_loaded).
-spec shard_run(sim(), pos_integer()) ->
    {ok, non_neg_integer(), [map()], {non_neg_integer(), non_neg_integer(), non_neg_integer()}} | error().
shard_run(_Sim, _MaxRounds) -> erlang:nif_error(nif_not_loaded).

%% Active views (self excluded) as a list of id lists, vertex order.
-spec active_views(sim()) -> {ok, [[non_neg_integer()]]} | error().
active_views(Sim) ->
    case hv_views(Sim) of
        {ok, Act, Len, _Pas, _PLen} -> {ok, rows(Act, Len, 0, [])};
        Err -> Err
    end.

rows(<<>>, <<>>, _V, Acc) ->
    lists:reverse(Acc);
rows(<<Row:32/binary, RestA/binary>>, <<L, RestL/binary>>, V, Acc) ->
    Ids = [I || <<I:32/little>> <= binary:part(Row, 0, L * 4), I =/= V],
    rows(RestA, RestL, V + 1, [Ids | Acc]).

%% The active views as the membership CSR load_csr/3 takes (the peer
%% service feeding partisan_plumtree_broadcast).
-spec csr_from_views([[non_neg_integer()]]) -> {binary(), binary()}.
csr_from_views(Views) ->
    {RowPtr, _} = lists:foldl(fun(Ids, {Acc, Off}) -> Next = Off + length(Ids),
                                                      {<<Acc/binary, Next:64/little>>, Next} end,
                              {<<0:64/little>>, 0}, Views),
    Col = << <<I:32/little>> || Ids <- Views, I <- Ids >>,
    {RowPtr, Col}.

%% C4 / C5 vertex-sharded over World ranks, the exchange on the handle's RCCL
%% communicator (shard_init_rccl first; psim_demers_shard_* / psim_causal_shard_step).
-spec demers_shard_setup(sim(), pos_integer(), pos_integer(), non_neg_integer(), boolean(), non_neg_integer(),
                         pos_integer()) -> {ok, non_neg_integer(), non_neg_integer()} | error().
demers_shard_setup(_Sim, _N, _M, _AePeriod, _RumorMongering, _Rank, _World) -> erlang:nif_error(nif_not_loaded).
-spec demers_shard_run(sim(), pos_integer()) -> {ok, non_neg_integer(), binary()} | error().
demers_shard_run(_Sim, _MaxRounds) -> erlang:nif_error(nif_not_loaded).
-spec causal_shard_setup(sim(), pos_integer(), pos_integer(), pos_integer(), pos_integer(), non_neg_integer(),
                         non_neg_integer(), pos_integer()) -> {ok, non_neg_integer(), non_neg_integer()} | error().
causal_shard_setup(_Sim, _N, _M, _Period, _DMax, _Redeliver, _Rank, _World) -> erlang:nif_error(nif_not_loaded).
-spec causal_shard_step(sim(), pos_integer()) -> {ok, [map()]} | error().
causal_shard_step(_Sim, _Rounds) -> erlang:nif_error(nif_not_loaded).

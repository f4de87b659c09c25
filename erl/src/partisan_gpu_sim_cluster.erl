%% partisan_gpu_sim_cluster -- one simulated Partisan cluster of N virtual
%% peers in HBM, driven through the partisan_gpu_sim NIF (include/psim.h).
%%
%% This is what the two behaviour adapters
%% (partisan_gpu_sim_membership_strategy, partisan_gpu_sim_plumtree_handler)
%% call: the cluster owns one libpsim handle; the strategy callbacks of the
%% simulated nodes queue their joins / leaves on it, and the cluster runs the
%% device rounds -- one periodic interval (`periodic_rounds' rounds, the
%% strategy's periodic/1 inside them, src/partisan_pluggable_peer_service_manager.erl
%% :1386-1419) once every live simulated node's periodic/1 has been called
%% for the interval.  Membership messages travel on the device; outgoing/1,
%% incoming/1 and deliver/2 render, take and put them in the wire form
%% {membership_strategy, Msg} the pluggable manager carries.
%%
%% Simulated node v is named 'nXXXXXXXX' (zero-padded v) with listen port
%% 10000 + v, so every Erlang term order of node specs equals vertex order
%% (SURVEY App. A Q28).
-module(partisan_gpu_sim_cluster).

-export([start/1, stop/0, sim/0, n/0,
         node_spec/1, vertex/1, self_vertex/0, set_self/1,
         join/2, leave/2, periodic/1, members/1, run_interval/0,
         load_overlay/2, heartbeat/1, restart_backend/1, delivered/3, is_stale/4, graft/4,
         outgoing/1, incoming/1, deliver/2]).

-define(KEY, ?MODULE).
-define(HIST, partisan_gpu_sim_heartbeats).

%% Opts: n, strategy (scamp_v2 | scamp_v1 | full), seed, device,
%% periodic_rounds (10), scamp_c (5), lazy_tick_rounds (1), max_tokens (2n).
-spec start(map()) -> {ok, partisan_gpu_sim:sim()} | {error, term()}.
start(#{n := N, strategy := Strategy} = Opts) ->
    Periodic = maps:get(periodic_rounds, Opts, 10),
    NewOpts = #{seed => maps:get(seed, Opts, 0), device => maps:get(device, Opts, 0),
                lazy_tick_rounds => maps:get(lazy_tick_rounds, Opts, 1)},
    case partisan_gpu_sim:new(NewOpts) of
        {ok, Sim} ->
            Setup = case Strategy of
                        scamp_v2 -> partisan_gpu_sim:scamp_setup(Sim, N, 2, maps:get(scamp_c, Opts, 5), Periodic);
                        scamp_v1 -> partisan_gpu_sim:scamp_setup(Sim, N, 1, maps:get(scamp_c, Opts, 5), Periodic);
                        full -> partisan_gpu_sim:fm_setup(Sim, N, Periodic, maps:get(max_tokens, Opts, 2 * N))
                    end,
            case Setup of
                ok ->
                    %% 1: periodic calls this interval; 2: wire seq; 3: heartbeats started
                    Calls = atomics:new(3, []),
                    catch ets:delete(?HIST),
                    ?HIST = ets:new(?HIST, [named_table, public, set]),
                    %% token words of a full-membership state (psim_fm_setup:
                    %% ceil(max_tokens / 64)), kept here so deliver/2 never
                    %% downloads the cluster's states to learn it (ADVICE r4)
                    FmWords = (maps:get(max_tokens, Opts, 2 * N) + 63) div 64,
                    persistent_term:put(?KEY, #{sim => Sim, n => N, strategy => Strategy,
                                                periodic => Periodic, calls => Calls,
                                                live => maps:get(live, Opts, N),
                                                fm_words => FmWords}),
                    {ok, Sim};
                Err ->
                    Err
            end;
        Err ->
            Err
    end.

-spec stop() -> ok.
stop() ->
    catch ets:delete(?HIST),
    _ = persistent_term:erase(?KEY),
    ok.

sim() -> maps:get(sim, persistent_term:get(?KEY)).
n() -> maps:get(n, persistent_term:get(?KEY)).

%% ---- node identity (SURVEY Q28) ----------------------------------------------
-spec node_spec(non_neg_integer()) -> map().
node_spec(V) ->
    Name = list_to_atom(lists:flatten(io_lib:format("n~8..0B", [V]))),
    #{name => Name,
      listen_addrs => [#{ip => {127, 0, 0, 1}, port => 10000 + V}],
      channels => #{undefined => #{parallelism => 1}}}.

-spec vertex(map() | atom()) -> non_neg_integer().
vertex(#{name := Name}) -> vertex(Name);
vertex(Name) when is_atom(Name) ->
    [Base | _] = string:split(atom_to_list(Name), "@"),
    "n" ++ Digits = Base,
    list_to_integer(Digits).

%% The simulated node the calling process acts for: set_self/1, else the
%% node name.
-spec self_vertex() -> non_neg_integer().
self_vertex() ->
    case get(partisan_gpu_sim_vertex) of
        undefined -> vertex(node());
        V -> V
    end.

set_self(V) -> put(partisan_gpu_sim_vertex, V), ok.

%% ---- membership strategy side ---------------------------------------------------
%% join/leave calls are queued on the device and handled by the next round
%% (psim_scamp_join / psim_fm_join: {connected, ...} -> Strategy:join/3).
join(V, Peer) -> batch(join, V, Peer).
leave(V, Node) -> batch(leave, V, Node).

batch(What, V, Other) ->
    #{sim := Sim, strategy := S} = persistent_term:get(?KEY),
    A = <<V:32/little>>,
    B = <<Other:32/little>>,
    case {S, What} of
        {full, join} -> partisan_gpu_sim:fm_join(Sim, A, B);
        {full, leave} -> partisan_gpu_sim:fm_leave(Sim, A, B);
        {_, join} -> partisan_gpu_sim:scamp_join(Sim, A, B);
        {_, leave} -> partisan_gpu_sim:scamp_leave(Sim, A, B)
    end.

%% periodic/1 of node V for the current interval: the last live node's call
%% runs the interval on the device.
periodic(_V) ->
    #{calls := C, live := Live} = persistent_term:get(?KEY),
    case atomics:add_get(C, 1, 1) >= Live of
        true ->
            atomics:put(C, 1, 0),
            run_interval();
        false ->
            ok
    end.

-spec run_interval() -> ok | {error, term()}.
run_interval() ->
    #{sim := Sim, strategy := S, periodic := P} = persistent_term:get(?KEY),
    Res = case S of
              full -> partisan_gpu_sim:fm_step(Sim, P);
              _ -> partisan_gpu_sim:scamp_step(Sim, P)
          end,
    case Res of
        {ok, _Stats} -> ok;
        Err -> Err
    end.

%% The members node V's strategy holds, as node specs in term order.
-spec members(non_neg_integer()) -> [map()].
members(V) ->
    #{sim := Sim, strategy := S, n := N} = persistent_term:get(?KEY),
    Ids = case S of
              full ->
                  {ok, Known, Removed, _Alive} = partisan_gpu_sim:fm_state(Sim),
                  W = byte_size(Known) div (N * 8),
                  K = binary:part(Known, V * W * 8, W * 8),
                  R = binary:part(Removed, V * W * 8, W * 8),
                  Live = [Bit || {Kw, Rw, Word} <- lists:zip3(words(K), words(R), lists:seq(0, W - 1)),
                                 Bit <- bits(Kw band (bnot Rw), Word * 64)],
                  {ok, TokNodes, _Used} = partisan_gpu_sim:fm_tokens(Sim),
                  lists:usort([token_node(TokNodes, T) || T <- Live]);
              _ ->
                  {ok, Pv, Npv, _Iv, _Niv} = partisan_gpu_sim:scamp_views(Sim),
                  Skip = V * 4,
                  <<_:Skip/binary, Len:32/little, _/binary>> = Npv,
                  Row = binary:part(Pv, V * 128 * 4, Len * 4),
                  lists:usort([I || <<I:32/little>> <= Row])
          end,
    [node_spec(I) || I <- Ids].

words(Bin) -> [W || <<W:64/little>> <= Bin].
bits(0, _Base) -> [];
bits(W, Base) -> [Base + I || I <- lists:seq(0, 63), (W bsr I) band 1 =:= 1].

%% the node token T adds (psim_fm_tokens: token v is node v's init/1 add, a
%% self-leave takes a fresh token)
token_node(TokNodes, T) ->
    Skip = T * 4,
    <<_:Skip/binary, Node:32/little, _/binary>> = TokNodes,
    Node.

%% ---- plumtree side ------------------------------------------------------------------
%% The peer service's members as Plumtree sees them (partisan_plumtree_broadcast
%% start_link/0): row_ptr u64 / col u32 binaries.
load_overlay(RowPtr, Col) -> partisan_gpu_sim:load_csr(sim(), RowPtr, Col).

%% backend heartbeat at Root (src/partisan_plumtree_backend.erl:341-368), run to
%% quiescence.  Returns the broadcast id {Node, Epoch, Monotonic}: Epoch counts
%% Root's backend restarts (restart_backend/1; erlang:system_time() at init/1
%% in the reference -- only its order matters, :229-244).  The delivered set
%% of Root's previous heartbeat is kept for is_stale/1 of older ids.
-spec heartbeat(non_neg_integer()) ->
          {ok, {node(), non_neg_integer(), pos_integer()}, non_neg_integer()} | {error, term()}.
heartbeat(Root) ->
    Sim = sim(),
    ok = snapshot_latest(Sim, Root),
    case partisan_gpu_sim:broadcast(Sim, Root) of
        {ok, Id} ->
            S = atomics:add_get(calls(), 3, 1),
            ets:insert(?HIST, {{latest, Root}, Id, S}),
            {ok, Rounds, _Stats} = partisan_gpu_sim:run(Sim, 100000),
            {ok, {maps:get(name, node_spec(Root)), Id bsr 24, Id band 16#FFFFFF}, Rounds};
        Err ->
            Err
    end.

%% V's heartbeat backend crashes and its supervisor starts it again (backend
%% init/1 :316-329): newer epoch, Monotonic 0, an empty timestamp table -- V
%% forgets every origin's heartbeats.  Heartbeats started before this are
%% not in V's table any more.
-spec restart_backend(non_neg_integer()) -> ok | {error, term()}.
restart_backend(V) ->
    Sim = sim(),
    %% No delivered-set snapshot here (VERDICT r3: N bytes per origin per
    %% call): the restart changes only V's own entries, which ts_row/2 no
    %% longer reads for heartbeats started before it ({restart, V} below), and
    %% every other vertex's newest-heartbeat bit is still on the device, read
    %% one vertex at a time (psim_get_delivered_range).
    case partisan_gpu_sim:restart_backend(Sim, V) of
        ok ->
            ets:insert(?HIST, {{restart, V}, atomics:get(calls(), 3)}),
            ok;
        Err ->
            Err
    end.

calls() -> maps:get(calls, persistent_term:get(?KEY)).

%% the delivered set of Origin's newest heartbeat, kept as {{hb, Origin, S}, Id, D}
snapshot_latest(Sim, Origin) ->
    case ets:lookup(?HIST, {latest, Origin}) of
        [{_, Id, S}] ->
            ok = partisan_gpu_sim:focus(Sim, Origin),
            {ok, D} = partisan_gpu_sim:delivered(Sim),
            ets:insert(?HIST, {{hb, Origin, S}, Id, D}),
            ok;
        [] ->
            ok
    end.

%% ---- membership messages on the wire (SURVEY 8(f) row 3) ------------------
%% What the pluggable manager of simulated node V would put on
%% ?MEMBERSHIP_CHANNEL for its strategy's Outgoing messages
%% (src/partisan_pluggable_peer_service_manager.erl:1396-1407, 1764-1776):
%% [{DstSpec, {membership_strategy, Msg}}] with Msg in the strategy's own
%% shape and node specs for node ids.  The simulated nodes' messages travel
%% on the device; this renders the ones V sent that the next round delivers.
-spec outgoing(non_neg_integer()) -> [{map(), {membership_strategy, tuple()}}].
outgoing(V) ->
    case strategy() of
        full ->
            {ok, Msgs} = partisan_gpu_sim:fm_messages_from(sim(), V),
            [{node_spec(Dst), {membership_strategy, {node_spec(Src), full_state(Src, K, R)}}}
             || {Src, Dst, _Seq, K, R} <- Msgs];
        _ ->
            {ok, Msgs} = partisan_gpu_sim:scamp_messages_from(sim(), V),
            [{node_spec(Dst), {membership_strategy, spec_msg(M)}}
             || {_Src, Dst, _Seq, {membership_strategy, M}} <- Msgs]
    end.

%% The messages for V the next round would deliver, taken off the device:
%% what V's manager receives as {membership_strategy, Msg} and hands to
%% handle_message/2 (:1739-1808) -- e.g. for a node that is run outside the
%% simulation.  [{SrcSpec, Msg}] in handling order; full membership's Msg is
%% {SrcSpec, #full_v1{}} (partisan_full_membership_strategy.erl:135-166, 247-267).
-spec incoming(non_neg_integer()) -> [{map(), tuple()}].
incoming(V) ->
    case strategy() of
        full ->
            {ok, Msgs} = partisan_gpu_sim:fm_take(sim(), V),
            [{node_spec(Src), {node_spec(Src), full_state(Src, K, R)}} || {Src, _Dst, _Seq, K, R} <- Msgs];
        _ ->
            {ok, Msgs} = partisan_gpu_sim:scamp_take(sim(), V),
            [{node_spec(Src), spec_msg(M)} || {Src, _Dst, _Seq, {membership_strategy, M}} <- Msgs]
    end.

%% handle_message(Msg, State) at simulated node V: Msg, as a manager received
%% it, goes onto the device for V's next round.  A SCAMP message does not
%% name its sender (the manager does not pass it), so it is ordered after the
%% simulated senders (source id N, by arrival); a full-membership message
%% {SenderSpec, #full_v1{}} carries it (a sender outside the cluster: N).
-spec deliver(non_neg_integer(), tuple()) -> ok | {error, term()}.
deliver(V, Msg) ->
    #{sim := Sim, n := N, calls := Calls} = persistent_term:get(?KEY),
    Seq = atomics:add_get(Calls, 2, 1),
    case Msg of
        {#{name := _} = From, {full_v1, _Actor, Membership}} ->
            Src = case catch vertex(From) of
                      I when is_integer(I), I >= 0, I < N -> I;
                      _ -> N
                  end,
            case full_bits(Membership) of
                {ok, K, R} -> partisan_gpu_sim:fm_put(Sim, [{Src, V, Seq, K, R}]);
                Err -> Err
            end;
        _ ->
            partisan_gpu_sim:scamp_put(Sim, [{N, V, Seq, {membership_strategy, id_msg(Msg)}}])
    end.

strategy() -> maps:get(strategy, persistent_term:get(?KEY)).

%% ---- #full_v1{} terms <-> token bitmaps ------------------------------------------
%% The device keeps a node's state_orset (partisan_membership_set) as two
%% bitmaps over the cluster's token universe (psim_fm_get_state): Known and
%% Removed.  The term is {full_v1, Actor, {state_orset, Payload}} with
%% Payload = orddict NodeSpec -> orddict Token -> Active (types 0.1.8), token
%% T rendered as {psim_token, T} (the device numbers tokens: T = V is node V's
%% init/1 add, a self-leave takes the next free one; psim_fm_tokens).
full_state(Src, K, R) ->
    W = byte_size(K) div 8,
    <<KI:(W * 64)/little>> = K,
    <<RI:(W * 64)/little>> = R,
    {ok, TokNodes, _Used} = partisan_gpu_sim:fm_tokens(sim()),
    Rows = [{token_node(TokNodes, T), {{psim_token, T}, (RI bsr T) band 1 =:= 0}}
            || T <- lists:seq(0, W * 64 - 1), (KI bsr T) band 1 =:= 1],
    Payload = lists:foldl(fun({E, Tok}, Acc) -> orddict:append(E, Tok, Acc) end, orddict:new(), Rows),
    Spec = fun(E) -> node_spec(E) end,
    {full_v1, {psim_actor, Src},
     {state_orset, orddict:from_list([{Spec(E), orddict:from_list(Toks)} || {E, Toks} <- Payload])}}.

full_bits({state_orset, Payload}) ->
    W = fm_words(),
    try
        {KI, RI} = lists:foldl(
                     fun({_Spec, Toks}, Acc0) ->
                             lists:foldl(fun({{psim_token, T}, Active}, {K0, R0}) when is_integer(T), T >= 0,
                                                                                        T < W * 64 ->
                                                 {K0 bor (1 bsl T),
                                                  case Active of true -> R0; false -> R0 bor (1 bsl T) end}
                                         end, Acc0, Toks)
                     end, {0, 0}, Payload),
        {ok, <<KI:(W * 64)/little>>, <<RI:(W * 64)/little>>}
    catch
        _:_ -> {error, foreign_state}     % a token the simulated cluster did not allocate
    end;
full_bits(_) ->
    {error, foreign_state}.

fm_words() ->
    maps:get(fm_words, persistent_term:get(?KEY)).

spec_msg({replace_subscription, A, B}) -> {replace_subscription, node_spec(A), node_spec(B)};
spec_msg({Tag, A}) -> {Tag, node_spec(A)}.

id_msg({replace_subscription, A, B}) -> {replace_subscription, vertex(A), vertex(B)};
id_msg({Tag, A}) -> {Tag, vertex(A)}.

%% V's timestamp-table row for Origin: the ids of Origin's heartbeats V
%% delivered since its backend last restarted, of the newest epoch among them
%% (add_timestamp/1 :400-417: a newer epoch replaces the set).  {Epoch, Ids}
%% or none.
ts_row(V, Origin) ->
    Since = case ets:lookup(?HIST, {restart, V}) of [{_, R}] -> R; [] -> 0 end,
    Latest = ets:lookup(?HIST, {latest, Origin}),
    LS = case Latest of [{_, _, S0}] -> S0; [] -> 0 end,
    Old = [{S, Id} || {{hb, _, S}, Id, D} <- ets:match_object(?HIST, {{hb, Origin, '_'}, '_', '_'}),
                      S > Since, S =/= LS, binary:at(D, V) =:= 1],
    New = case Latest of
              [{_, Id, S}] when S > Since ->
                  %% the newest heartbeat: one vertex, psim_get_delivered_range, O(1)
                  Sim = sim(),
                  ok = partisan_gpu_sim:focus(Sim, Origin),
                  case partisan_gpu_sim:is_delivered(Sim, V, 0) of
                      {ok, true} -> [{S, Id}];
                      _ -> []
                  end;
              _ ->
                  []
          end,
    case lists:sort(Old ++ New) of
        [] ->
            none;
        Got ->
            {_, Last} = lists:last(Got),
            E = Last bsr 24,
            {E, [Id || {_, Id} <- Got, Id bsr 24 =:= E]}
    end.

%% Mod:is_stale({Origin, Epoch, Monotonic}) at vertex V (backend :229-244)
-spec is_stale(non_neg_integer(), non_neg_integer(), non_neg_integer(), non_neg_integer()) -> boolean().
is_stale(V, Origin, Epoch, Mono) ->
    case ts_row(V, Origin) of
        none -> false;
        {Epoch, Ids} -> lists:member(Epoch bsl 24 bor Mono, Ids);
        {Epoch0, _} -> Epoch0 > Epoch
    end.

%% Mod:graft({Origin, Epoch, Monotonic}) at vertex V (backend :254-280):
%% ok (the payload is the id itself) | stale | not_found
-spec graft(non_neg_integer(), non_neg_integer(), non_neg_integer(), non_neg_integer()) -> ok | stale | not_found.
graft(V, Origin, Epoch, Mono) ->
    case ts_row(V, Origin) of
        none -> not_found;
        {Epoch, Ids} ->
            case lists:member(Epoch bsl 24 bor Mono, Ids) of
                true -> ok;
                false -> not_found
            end;
        {Epoch0, _} when Epoch0 > Epoch -> stale;
        _ -> not_found
    end.

%% is_stale/4 for an id in psim's packed form, Epoch bsl 24 bor Monotonic
-spec delivered(non_neg_integer(), non_neg_integer(), non_neg_integer()) -> boolean().
delivered(V, Origin, Id) ->
    is_stale(V, Origin, Id bsr 24, Id band 16#FFFFFF).

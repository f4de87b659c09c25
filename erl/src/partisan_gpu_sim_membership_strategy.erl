%% partisan_gpu_sim_membership_strategy -- the partisan_membership_strategy
%% behaviour (src/partisan_membership_strategy.erl:55-77) for a node of a
%% simulated cluster (partisan_gpu_sim_cluster): the pluggable peer service
%% manager calls it exactly as it calls partisan_scamp_v2_membership_strategy
%% or partisan_full_membership_strategy
%% (src/partisan_pluggable_peer_service_manager.erl:1386-1419, 1532-1597,
%% 1739-1808), and the strategy the cluster was started with runs on the GPU
%% (psim_scamp_* / psim_fm_*, the same restatement the oracle checks).
%%
%% The simulated nodes' membership messages travel on the device, so every
%% callback returns no outgoing messages (the manager would send them twice);
%% partisan_gpu_sim_cluster:outgoing/1 renders them as the manager puts them
%% on the wire, [{DstSpec, {membership_strategy, Msg}}], and incoming/1 takes
%% a node's messages off the device.  A {membership_strategy, Msg} the node's
%% manager receives (full membership: {SenderSpec, #full_v1{}}; SCAMP:
%% forward_subscription, keep_subscription, ping, remove_subscription,
%% replace_subscription, bootstrap_remove_subscription) goes onto the device
%% for the node's next round (handle_message/2).
%% Members are read back from the device after the interval runs.
-module(partisan_gpu_sim_membership_strategy).

-behaviour(partisan_membership_strategy).

-export([init/1, join/3, leave/2, compare/2, periodic/1, prune/2, handle_message/2]).

-record(gpu_state, {
    vertex :: non_neg_integer(),
    actor :: term()
}).

%% init/1 (scamp_v2 :75-85, full :70-74): the node knows itself
init(Identity) ->
    V = partisan_gpu_sim_cluster:self_vertex(),
    {ok, partisan_gpu_sim_cluster:members(V), #gpu_state{vertex = V, actor = Identity}}.

%% {connected, Node, ...} -> join/3 (pluggable :1532-1597): queued on the device
join(NodeSpec, _PeerState, #gpu_state{vertex = V} = State) ->
    ok = partisan_gpu_sim_cluster:join(V, partisan_gpu_sim_cluster:vertex(NodeSpec)),
    {ok, partisan_gpu_sim_cluster:members(V), [], State}.

%% internal_leave (pluggable :2059-2109) -> leave/2
leave(NodeSpec, #gpu_state{vertex = V} = State) ->
    ok = partisan_gpu_sim_cluster:leave(V, partisan_gpu_sim_cluster:vertex(NodeSpec)),
    {ok, partisan_gpu_sim_cluster:members(V), [], State}.

%% handle_info(periodic) (pluggable :1386-1419): the last live node's call of
%% the interval runs it on the device
periodic(#gpu_state{vertex = V} = State) ->
    ok = partisan_gpu_sim_cluster:periodic(V),
    {ok, partisan_gpu_sim_cluster:members(V), [], State}.

%% {membership_strategy, Msg} (pluggable :1739-1808): onto the device for V --
%% full membership's {SenderSpec, #full_v1{}} (:135-166) and the SCAMP
%% strategies' atom-tagged messages
handle_message({#{name := _}, {full_v1, _, _}} = Msg, #gpu_state{vertex = V} = State) ->
    ok = partisan_gpu_sim_cluster:deliver(V, Msg),
    {ok, partisan_gpu_sim_cluster:members(V), [], State};
handle_message(Msg, #gpu_state{vertex = V} = State) when is_tuple(Msg), is_atom(element(1, Msg)) ->
    ok = partisan_gpu_sim_cluster:deliver(V, Msg),
    {ok, partisan_gpu_sim_cluster:members(V), [], State};
handle_message(_Msg, #gpu_state{vertex = V} = State) ->
    {ok, partisan_gpu_sim_cluster:members(V), [], State}.

%% {Joiners, Leavers}: the specs of List that are not members, the members
%% that are not in List
compare(Members, #gpu_state{vertex = V}) ->
    Current = partisan_gpu_sim_cluster:members(V),
    {Members -- Current, Current -- Members}.

prune(NodeSpecs, #gpu_state{vertex = V} = State) ->
    lists:foreach(fun(N) -> ok = partisan_gpu_sim_cluster:leave(V, partisan_gpu_sim_cluster:vertex(N)) end,
                  NodeSpecs),
    {ok, partisan_gpu_sim_cluster:members(V), State}.

%% partisan_gpu_sim_plumtree_handler -- the partisan_plumtree_broadcast_handler
%% behaviour (src/partisan_plumtree_broadcast_handler.erl:47-78) for the
%% heartbeat broadcasts of a simulated cluster: the same callbacks and return
%% shapes as the default handler partisan_plumtree_backend
%% (src/partisan_plumtree_backend.erl:180-293), answered from the device
%% state (psim_get_delivered on the origin's heartbeat lane) for the node the
%% calling process acts for (partisan_gpu_sim_cluster:self_vertex/0).
%%
%% The device runs merge/add_timestamp itself inside each round (the
%% simulated broadcast servers call this handler on device); from the host,
%% merge/2 is the read-only view "not stale".
-module(partisan_gpu_sim_plumtree_handler).

-behaviour(partisan_plumtree_broadcast_handler).

-export([broadcast_data/1, broadcast_channel/0, merge/2, is_stale/1, graft/1, exchange/1]).

-record(broadcast, {timestamp}).

%% backend :192-195
broadcast_data(#broadcast{timestamp = Timestamp}) ->
    {Timestamp, Timestamp};
broadcast_data(#{timestamp := Timestamp}) ->
    {Timestamp, Timestamp}.

%% backend :180-181 (?MEMBERSHIP_CHANNEL)
broadcast_channel() ->
    partisan_membership.

%% backend :205-215
merge(Timestamp, Timestamp) ->
    not is_stale(Timestamp);
merge(_Id, _Payload) ->
    false.

%% backend :229-244: the origin's row {Node, Epoch0, ISet} of the node's table
is_stale({Node, Epoch, Monotonic}) ->
    partisan_gpu_sim_cluster:is_stale(partisan_gpu_sim_cluster:self_vertex(),
                                      partisan_gpu_sim_cluster:vertex(Node), Epoch, Monotonic).

%% backend :254-280
graft({Node, Epoch, Monotonic} = Timestamp) ->
    case partisan_gpu_sim_cluster:graft(partisan_gpu_sim_cluster:self_vertex(),
                                        partisan_gpu_sim_cluster:vertex(Node), Epoch, Monotonic) of
        ok -> {ok, Timestamp};
        stale -> stale;
        not_found -> {error, {not_found, Timestamp}}
    end.

%% backend :292-293
exchange(_Peer) ->
    ignore.

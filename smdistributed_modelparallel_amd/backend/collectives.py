"""Object collectives over the native mailbox.

Semantics follow the reference object channel (`smp/backend/collectives.py:15-348`):
pickled-object broadcast / send / recv / allgather / gather / barrier over the named
groups WORLD, PP, TP, RDP, DP and MP, matched by transaction id.

Transaction ids are derived per (operation kind, group-or-peer) from a counter that
every participant advances identically, so no id negotiation is needed.  User-API
traffic and internal traffic use disjoint id spaces (``is_user_api`` bit), matching the
reference's ``2 * id + is_user_api`` convention.
"""
import pickle
from enum import Enum

from .exceptions import SMPInvalidArgumentError

USER_CHANNEL = 0
SERVER_CHANNEL = 1


class CommGroup(Enum):
    WORLD = 0
    PP_GROUP = 1
    TP_GROUP = 2
    RDP_GROUP = 3
    DP_GROUP = 4
    MP_GROUP = 5


class RankType(Enum):
    WORLD_RANK = 0
    PP_RANK = 1
    TP_RANK = 2
    RDP_RANK = 3
    DP_RANK = 4
    MP_RANK = 5


_KIND = {"p2p": 1, "bcast": 2, "allgather": 3, "gather": 4, "barrier": 5, "large": 6}


class TransactionIdentifier:
    """Deterministic transaction ids: (kind, key) -> counter."""

    def __init__(self):
        self._counters = {}

    def next(self, kind, key, is_user_api):
        k = (kind, key, bool(is_user_api))
        c = self._counters.get(k, 0)
        self._counters[k] = c + 1
        return ((_KIND[kind] * 2 + int(bool(is_user_api))) << 48) | (c & ((1 << 48) - 1))

    def reset(self):
        self._counters.clear()


def dumps(obj):
    return pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)


def loads(b):
    return pickle.loads(b)


class CollectiveCommunicator:
    """Group-aware object communication. `core` supplies rank/group queries."""

    def __init__(self, core, mailbox):
        self.core = core
        self.mailbox = mailbox
        self.tids = TransactionIdentifier()
        self.timeout = -1.0

    # --------------------------------------------------------------- helpers
    def _group_ranks(self, group):
        if isinstance(group, CommGroup):
            return self.core.get_group_ranks(group)
        if isinstance(group, (list, tuple)):
            return list(group)
        raise SMPInvalidArgumentError(f"invalid group {group}")

    def _to_global(self, rank, rank_type):
        if rank_type is None or rank_type == RankType.WORLD_RANK:
            return rank
        group = {
            RankType.PP_RANK: CommGroup.PP_GROUP,
            RankType.TP_RANK: CommGroup.TP_GROUP,
            RankType.RDP_RANK: CommGroup.RDP_GROUP,
            RankType.DP_RANK: CommGroup.DP_GROUP,
            RankType.MP_RANK: CommGroup.MP_GROUP,
        }[rank_type]
        return self._group_ranks(group)[rank]

    # ------------------------------------------------------------ primitives
    def send(self, obj, dest, rank_type=RankType.WORLD_RANK, is_user_api=False, payload=None):
        dst = self._to_global(dest, rank_type)
        tid = self.tids.next("p2p", (self.core.rank(), dst), is_user_api)
        self.mailbox.send(dst, tid, USER_CHANNEL, payload if payload is not None else dumps(obj))

    def recv_from(self, src, rank_type=RankType.WORLD_RANK, is_user_api=False, raw=False):
        s = self._to_global(src, rank_type)
        tid = self.tids.next("p2p", (s, self.core.rank()), is_user_api)
        b = self.mailbox.recv(s, tid, self.timeout)
        return b if raw else loads(b)

    def broadcast(self, obj, group=CommGroup.WORLD, is_user_api=False, root=None):
        """Root sends `obj` to every other group member; returns nothing on the root."""
        # one point-to-point message per member, numbered in the (root, member) sequence that
        # send / recv_from use: a receiver may take it with recv_from(root) -- the reference's
        # broadcast + recv_from pairing (`test/backend/test_collectives.py:54-72`) -- or with
        # recv_broadcast; messages between a pair are matched in program order
        ranks = self._group_ranks(group)
        root = self.core.rank() if root is None else root
        others = [r for r in ranks if r != root]
        if not others:
            return
        payload = dumps(obj)
        for dst in others:
            self.mailbox.send(dst, self.tids.next("p2p", (root, dst), is_user_api), USER_CHANNEL, payload)

    def recv_broadcast(self, root, group=CommGroup.WORLD, is_user_api=False):
        return self.recv_from(root, RankType.WORLD_RANK, is_user_api)

    def bcast(self, obj, root, group=CommGroup.WORLD, is_user_api=False):
        """Symmetric broadcast: every member calls, the root's object is returned everywhere."""
        if self.core.rank() == root:
            self.broadcast(obj, group, is_user_api, root=root)
            return obj
        return self.recv_broadcast(root, group, is_user_api)

    def allgather(self, obj, group=CommGroup.WORLD, is_user_api=False):
        ranks = self._group_ranks(group)
        me = self.core.rank()
        tid = self.tids.next("allgather", tuple(ranks), is_user_api)
        payload = dumps(obj)
        others = [r for r in ranks if r != me]
        if others:
            self.mailbox.broadcast(others, tid, USER_CHANNEL, payload)
        out = []
        for r in ranks:
            out.append(obj if r == me else loads(self.mailbox.recv(r, tid, self.timeout)))
        return out

    def gather(self, obj, group=CommGroup.WORLD, rank=0, is_user_api=False):
        """Gather to the group member `rank` (group-local index). Non-roots get None."""
        ranks = self._group_ranks(group)
        root = ranks[rank]
        me = self.core.rank()
        tid = self.tids.next("gather", (tuple(ranks), root), is_user_api)
        if me != root:
            self.mailbox.send(root, tid, USER_CHANNEL, dumps(obj))
            return None
        return [obj if r == me else loads(self.mailbox.recv(r, tid, self.timeout)) for r in ranks]

    def barrier(self, group=CommGroup.WORLD, is_user_api=False):
        self.allgather(None, group, is_user_api)

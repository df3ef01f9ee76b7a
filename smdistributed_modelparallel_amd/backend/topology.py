"""Rank placement.

A global rank is a mixed-radix number whose digits are the (pipeline, reduced-data,
tensor) coordinates.  The placement string (a permutation of ``P``, ``D``, ``T``) gives
the digit order, most significant first, so the *rightmost* axis varies fastest between
neighbouring ranks.  ``cluster`` == ``DPT`` (TP groups are adjacent ranks -> adjacent
GPUs on one xGMI-connected node) and ``spread`` == ``TPD``.

Derived groups follow the reference's definitions (`smp/backend/core.py:26-162`):
* DP group = all ranks with the same pipeline coordinate (TP ranks included), ordered
  by the relative placement of D and T;
* MP group = all ranks with the same reduced-data coordinate (pipeline x tensor).
"""
from functools import lru_cache

_AXES = ("P", "D", "T")


class Ranker:
    def __init__(self, placement_strategy, rdp_size, pp_size, tp_size):
        ps = {"cluster": "DPT", "spread": "TPD"}.get(placement_strategy, placement_strategy)
        if sorted(ps) != sorted(_AXES):
            raise ValueError(f"invalid placement strategy {placement_strategy}")
        self.ps = ps
        self.size_map = {"P": pp_size, "D": rdp_size, "T": tp_size}
        self.size = pp_size * rdp_size * tp_size
        # stride of each axis in the mixed-radix number
        self._stride = {}
        stride = 1
        for axis in reversed(ps):
            self._stride[axis] = stride
            stride *= self.size_map[axis]

    # ---------------------------------------------------------------- digits
    def coords(self, rank):
        return {a: (rank // self._stride[a]) % self.size_map[a] for a in _AXES}

    def compose(self, coords):
        return sum(coords[a] * self._stride[a] for a in _AXES)

    def translate(self, pp_rank, tp_rank, rdp_rank):
        return self.compose({"P": pp_rank, "T": tp_rank, "D": rdp_rank})

    def _axis_group(self, rank, axis):
        c = self.coords(rank)
        out = []
        for i in range(self.size_map[axis]):
            c[axis] = i
            out.append(self.compose(c))
        return out

    def _pair_group(self, rank, a, b):
        """All ranks sharing `rank`'s third coordinate, ordered by the placement order of a/b."""
        outer, inner = (a, b) if self.ps.index(a) < self.ps.index(b) else (b, a)
        c = self.coords(rank)
        out = []
        for i in range(self.size_map[outer]):
            for j in range(self.size_map[inner]):
                c[outer], c[inner] = i, j
                out.append(self.compose(c))
        return out

    def _pair_rank(self, rank, a, b):
        outer, inner = (a, b) if self.ps.index(a) < self.ps.index(b) else (b, a)
        c = self.coords(rank)
        return c[outer] * self.size_map[inner] + c[inner]

    # -------------------------------------------------------------- ranks
    def get_pp_rank(self, rank):
        return self.coords(rank)["P"]

    def get_tp_rank(self, rank):
        return self.coords(rank)["T"]

    def get_rdp_rank(self, rank):
        return self.coords(rank)["D"]

    def get_dp_rank(self, rank):
        return self._pair_rank(rank, "D", "T")

    def get_mp_rank(self, rank):
        return self._pair_rank(rank, "P", "T")

    # ------------------------------------------------------------- groups
    def get_pp_group(self, rank):
        return self._axis_group(rank, "P")

    def get_tp_group(self, rank):
        return self._axis_group(rank, "T")

    def get_rdp_group(self, rank):
        return self._axis_group(rank, "D")

    def get_dp_group(self, rank):
        return self._pair_group(rank, "D", "T")

    def get_mp_group(self, rank):
        return self._pair_group(rank, "P", "T")

    # ------------------------------------------------------ group-rank maps
    def _split_pair(self, idx, a, b):
        outer, inner = (a, b) if self.ps.index(a) < self.ps.index(b) else (b, a)
        return {outer: idx // self.size_map[inner], inner: idx % self.size_map[inner]}

    def get_rdp_rank_from_dp_rank(self, dp_rank):
        return self._split_pair(dp_rank, "D", "T")["D"]

    def get_tp_rank_from_dp_rank(self, dp_rank):
        return self._split_pair(dp_rank, "D", "T")["T"]

    def get_pp_rank_from_mp_rank(self, mp_rank):
        return self._split_pair(mp_rank, "P", "T")["P"]

    def get_tp_rank_from_mp_rank(self, mp_rank):
        return self._split_pair(mp_rank, "P", "T")["T"]

    @lru_cache(maxsize=None)
    def all_groups(self, kind):
        """Every distinct group of a kind, in a deterministic order (for collective creation)."""
        fn = getattr(self, f"get_{kind}_group")
        seen, out = set(), []
        for r in range(self.size):
            g = tuple(fn(r))
            if g not in seen:
                seen.add(g)
                out.append(list(g))
        return out

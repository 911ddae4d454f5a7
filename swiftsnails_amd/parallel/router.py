"""Hash-fragment router (key -> fragment -> server).

Parity with ``BasicHashFrag`` (/root/reference/src/core/parameter/hashfrag.h):

* ``init``: fragment ``i`` belongs to server id ``i // (frag_num // num_nodes) + 1``
  clamped to ``[1, num_nodes]`` (hashfrag.h:30-46; ids start at 1 because the
  master is node 0).
* ``to_node_id(key) = map[fmix64(key) % frag_num]`` (hashfrag.h:48-53).
* wire format ``{int32 num_nodes, int32 num_frags, uint32 map[num_frags]}``
  (hashfrag.h:55-85) — identical bytes to the reference BinaryBuffer codec.

Differences (deliberate): ``frag_num < num_nodes`` raises instead of dividing
by zero (SURVEY §5 known defects), and ``rank_map`` translates server ids to
the ranks of the communicator so the device router (fused into the dedup
kernel) sends straight to a GPU rank.  The map is computed deterministically
on every rank (no master round-trip is needed for correctness, though the
master still broadcasts it for protocol parity).
"""
from __future__ import annotations

import struct
from typing import Sequence

import numpy as np
import torch

from ..utils.hashing import as_u64, fmix64


class HashFrag:
    def __init__(self, num_nodes: int = 0, frag_num: int = 0):
        self.num_nodes = 0
        self.num_frags = 0
        self.map_table: np.ndarray | None = None
        if num_nodes and frag_num:
            self.init(num_nodes, frag_num)

    def init(self, num_nodes: int, frag_num: int) -> "HashFrag":
        if num_nodes <= 0:
            raise ValueError("num_nodes must be > 0")
        if frag_num < num_nodes:
            raise ValueError(f"frag_num ({frag_num}) must be >= num_nodes ({num_nodes})")
        self.num_nodes = int(num_nodes)
        self.num_frags = int(frag_num)
        each = frag_num // num_nodes
        ids = np.arange(frag_num, dtype=np.int64) // each + 1
        self.map_table = np.clip(ids, 1, num_nodes).astype(np.uint32)
        return self

    # -- routing -------------------------------------------------------------
    def frag_of(self, keys) -> np.ndarray:
        self._check()
        return (fmix64(keys) % np.uint64(self.num_frags)).astype(np.int64)

    def to_node_id(self, keys) -> np.ndarray:
        """1-based server node ids (reference numbering)."""
        return self.map_table[self.frag_of(keys)].astype(np.int64)

    def rank_map(self, server_ranks: Sequence[int] | None = None) -> np.ndarray:
        """fragment -> communicator rank. ``server_ranks[k-1]`` hosts server id k."""
        self._check()
        if server_ranks is None:
            server_ranks = list(range(self.num_nodes))
        if len(server_ranks) != self.num_nodes:
            raise ValueError("need one rank per server node")
        sr = np.asarray(server_ranks, dtype=np.int32)
        return sr[self.map_table.astype(np.int64) - 1]

    def rank_map_tensor(self, server_ranks=None, device=None) -> torch.Tensor:
        return torch.from_numpy(self.rank_map(server_ranks).astype(np.int32)).to(device)

    # -- codec ---------------------------------------------------------------
    def serialize(self) -> bytes:
        self._check()
        return struct.pack("<ii", self.num_nodes, self.num_frags) + self.map_table.astype(
            "<u4").tobytes()

    @classmethod
    def deserialize(cls, data: bytes) -> "HashFrag":
        n, f = struct.unpack_from("<ii", data, 0)
        if f <= 0:
            raise ValueError("bad hashfrag payload")
        h = cls()
        h.num_nodes, h.num_frags = n, f
        h.map_table = np.frombuffer(data, dtype="<u4", count=f, offset=8).astype(np.uint32)
        return h

    def _check(self):
        if self.map_table is None:
            raise RuntimeError("map_table has not been inited")

    def __repr__(self):
        return f"HashFrag(num_nodes={self.num_nodes}, num_frags={self.num_frags})"


def route_keys_np(keys, frag_rank_map: np.ndarray) -> np.ndarray:
    """Reference (host) routing: key -> rank via a fragment->rank map."""
    f = fmix64(keys) % np.uint64(len(frag_rank_map))
    return frag_rank_map[f.astype(np.int64)].astype(np.int64)


__all__ = ["HashFrag", "route_keys_np", "as_u64"]

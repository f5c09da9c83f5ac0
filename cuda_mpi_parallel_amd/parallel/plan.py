"""Row partition + halo plan (thin typed view over csrc/host/partition.cpp)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

from .. import native


@dataclass(frozen=True)
class Layout:
    """One rank's share: owned rows, column window, ext-vector layout and halo plan.

    ``sends`` / ``recvs`` are ``(peer, first_global_row, count)`` triples; a range is
    sent straight out of the owner's owned block and lands straight in the
    receiver's ghost block (ext index = global - col_lo + pad).
    """

    rank: int
    world: int
    n_global: int
    row_begin: int
    row_end: int
    col_lo: int
    col_hi: int
    pad: int
    ext_len: int
    own_off: int
    interior_begin: int
    interior_end: int
    allgather: bool  # ghosts = every other rank's block, refreshed by one all-gather (own_off = rank * block)
    block: int
    sends: Tuple[Tuple[int, int, int], ...]
    recvs: Tuple[Tuple[int, int, int], ...]

    @property
    def n_local(self) -> int:
        return self.row_end - self.row_begin

    def ext_index(self, g: int) -> int:
        return g - self.col_lo + self.pad


def partition_rows(spec, world: int, halo_mode: int = -1) -> List[int]:
    ns = spec.native() if hasattr(spec, "native") else spec
    return list(native().partition_rows(ns, world, halo_mode))


def layout(spec, world: int, rank: int, halo_mode: int = -1) -> Layout:
    ns = spec.native() if hasattr(spec, "native") else spec
    d = native().make_layout(ns, world, rank, halo_mode)
    d["sends"] = tuple(tuple(x) for x in d["sends"])
    d["recvs"] = tuple(tuple(x) for x in d["recvs"])
    return Layout(**d)

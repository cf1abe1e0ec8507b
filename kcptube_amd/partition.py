"""Multi-GPU partition of shard groups.

Shard groups are independent: the encoding matrix is shared and read-only, decode coefficients are
per group.  A job of G_total groups over W ranks gives rank r the contiguous range
[r * G_total // W, (r + 1) * G_total // W); each rank generates / owns its groups' bytes on its own GPU,
runs the same kernels, and nothing crosses xGMI.  The only cross-rank traffic is control: the timing
barrier, a max-reduce of the elapsed time, and (for the parity check) a combine of per-rank digests --
all over gloo on the host, never over RCCL, because there is no data-path exchange to accelerate.
"""
from __future__ import annotations

import hashlib


def group_range(total_groups: int, world: int, rank: int) -> tuple[int, int]:
    """[g0, g1) of the global group space owned by `rank` (contiguous, sizes differ by at most 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    return total_groups * rank // world, total_groups * (rank + 1) // world


def combine_digests(per_rank_hex: list[str]) -> str:
    """Order-fixed digest of per-rank digests (a checksum of checksums), independent of timing."""
    h = hashlib.sha256()
    for d in per_rank_hex:
        h.update(bytes.fromhex(d))
    return h.hexdigest()

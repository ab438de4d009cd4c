"""Multi-GPU plumbing for config 5 (independent streams sharded over ranks).

One process per GPU. Units (windows or whole streams) are split into
contiguous, balanced shards with no data-path collective; the only exchange is
the final gather of decoded symbols to rank 0 (RCCL over xGMI under the
"nccl" backend; gloo on CPU for tests), which then frames them as ip.proto
ToReceiver messages.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np


def shard_range(total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous balanced shard of `total` units: (first, count)."""
    if world < 1 or not 0 <= rank < world or total < 0:
        raise ValueError("bad shard request")
    base, extra = divmod(total, world)
    first = rank * base + min(rank, extra)
    return first, base + (1 if rank < extra else 0)


def gather_symbols(local, total_units: int, world: int, unit: int = 1, group=None):
    """All-gather every rank's symbol shard; returns the full uint8 tensor
    (same device as `local`) on every rank. Rank r holds the symbols of units
    shard_range(total_units, r, world), `unit` symbols per unit (e.g. windows
    per stream). Uneven shards are padded to the largest, then trimmed."""
    import torch
    import torch.distributed as dist

    per = (-(-total_units // world) if world else 0) * unit
    buf = torch.zeros(per, dtype=torch.uint8, device=local.device)
    buf[: local.numel()] = local.reshape(-1)
    out = torch.empty(per * world, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    parts = []
    for r in range(world):
        _, cnt = shard_range(total_units, r, world)
        parts.append(out[r * per: r * per + cnt * unit])
    return torch.cat(parts) if parts else out[:0]


def gather_blocks(local, world: int, block: int, group=None):
    """All-gather one variable-length byte block per rank (at most `block`
    bytes each, padded to it): returns [world][block] uint8 on every rank.
    Configs[4]'s bucketed step gathers each rank's frames of S steps this
    way (bench.py), one collective per S steps."""
    import torch
    import torch.distributed as dist

    buf = torch.zeros(block, dtype=torch.uint8, device=local.device)
    buf[: local.numel()] = local.reshape(-1)
    out = torch.empty(block * world, dtype=torch.uint8, device=local.device)
    dist.all_gather_into_tensor(out, buf, group=group)
    return out.view(world, block)


def frame_symbols(A, symbols: np.ndarray, k: int) -> bytes:
    """Rank-0 framing of the gathered symbol stream (delimited ToReceiver)."""
    return A.frame_symbols(np.ascontiguousarray(symbols, dtype=np.uint8), A.bits_per_symbol(k))


def unframe_symbols(A, stream: bytes, n: int, k: int) -> np.ndarray:
    """Inverse of frame_symbols (the receiver side, network.cpp:409-430)."""
    bits = A.bits_per_symbol(k)
    per = A.DEMOD_MAX_FRAME_PAYLOAD * 8 // bits
    out, got = [], 0
    for payload in A.iter_frames(stream):
        cnt = min(per, n - got)
        out.append(A.unpack_symbols(payload, cnt, bits))
        got += cnt
    return np.concatenate(out) if out else np.zeros(0, np.uint8)

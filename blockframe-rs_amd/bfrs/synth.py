"""Deterministic synthetic BlockFrame workloads (tests and bench.py).

Bytes come from splitmix64 over a counter, so the same (seed, segment,
length) gives identical bytes from numpy on the host and torch on the GPU.
Word i of segment s is mix((seed << 44) + (s << 24) + i); shards up to
128 MiB.  Block shapes follow the reference's tier-3 commit: blocks of up to
30 segments (src/chunker/commit.rs:359,402-416), S = 32 MiB
(src/utils.rs:68).
"""
from __future__ import annotations

import numpy as np

SEGMENT_SIZE = 32 * 1024 * 1024  # src/utils.rs:68 on any real host
BLOCK_SEGMENTS = 30              # src/chunker/commit.rs:359
PARITY_SHARDS = 3

_G = 0x9E3779B97F4A7C15
_M1 = 0xBF58476D1CE4E5B9
_M2 = 0x94D049BB133111EB


def block_shapes(n_segments: int, per_block: int = BLOCK_SEGMENTS):
    """Original counts per block, as commit_blocked forms them."""
    full, rest = divmod(n_segments, per_block)
    return [per_block] * full + ([rest] if rest else [])


def _base(seed: int, seg: int) -> int:
    return ((seed << 44) + (seg << 24)) & 0xFFFFFFFFFFFFFFFF


def segment_np(seed: int, seg: int, nbytes: int) -> np.ndarray:
    nwords = (nbytes + 7) // 8
    with np.errstate(over="ignore"):
        z = (np.arange(nwords, dtype=np.uint64) + np.uint64(_base(seed, seg))) * np.uint64(_G)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
        z = z ^ (z >> np.uint64(31))
    return z.view(np.uint8)[:nbytes].copy()


def _i64(x: int) -> int:
    x &= 0xFFFFFFFFFFFFFFFF
    return x - (1 << 64) if x >= 1 << 63 else x


def _lsr(z, s: int):
    import torch
    return (z >> s) & ((1 << (64 - s)) - 1)


def fill_segment_torch(out, seed: int, seg: int) -> None:
    """Fill a uint8 torch tensor (any device, length multiple of 8) in place."""
    import torch
    n = out.numel()
    assert n % 8 == 0
    w = out.view(torch.int64)
    torch.arange(n // 8, dtype=torch.int64, device=out.device, out=w)
    w.add_(_i64(_base(seed, seg))).mul_(_i64(_G))
    w.bitwise_xor_(_lsr(w, 30)).mul_(_i64(_M1))
    w.bitwise_xor_(_lsr(w, 27)).mul_(_i64(_M2))
    w.bitwise_xor_(_lsr(w, 31))

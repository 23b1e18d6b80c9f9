"""Shard / chunk plan of the multi-GPU allreduce -- the same arithmetic as
``inccl_shard_elems`` (csrc/inccl_internal.h) and the chunk loop of
``inccl_allreduce_f32_pipelined`` (csrc/api.c).  Used by bench.py to report
per-rank shapes and by the gloo tests of the N>1 decomposition.
"""
from __future__ import annotations

SHARD_ALIGN = 64   # elements: every shard starts 256-B aligned for dwordx4


def shard_elems(n: int, world: int) -> int:
    per = (n + world - 1) // world
    return (per + SHARD_ALIGN - 1) // SHARD_ALIGN * SHARD_ALIGN


def chunk_plan(n: int, world: int, chunks: int = 1):
    """[(offset, count, shard)] for each pipelined chunk of an n-element bucket."""
    chunks = max(1, int(chunks))
    unit = world * SHARD_ALIGN
    per = ((n + chunks - 1) // chunks + unit - 1) // unit * unit
    per = max(per, unit)
    out = []
    off = 0
    while off < n:
        cnt = min(per, n - off)
        out.append((off, cnt, shard_elems(cnt, world)))
        off += cnt
    return out


def xgmi_bytes_per_rank(n: int, world: int) -> int:
    """Bytes each rank sends over xGMI: reduce-scatter (int32) + all-gather (fp32)."""
    shard = shard_elems(n, world)
    return 2 * (world - 1) * shard * 4

"""Multi-GPU group-by (key-hash exchange of partial groups) and sample sort over
torch.distributed.

One process per GPU; backend "nccl" is RCCL over xGMI on ROCm ("gloo" on CPU for tests).
Each rank pre-aggregates its row shard on its GPU (nut_groupby), partitions the partial
groups by owner = mix64(key tuple) % P on the device (nut_groups_partition), and the
ranks exchange them with ONE all-to-all of counts and ONE all-to-all of records.  Each
owner merges what it received (nut_groupby_accumulate: SUM/COUNT partials add, MIN/MAX
re-min/max) and rank 0 gathers the owners' final groups.  xGMI is a full point-to-point
mesh, so the all-to-all uses every link directly.

The record layout is the library's column-major segment format: segment p holds
counts[p] groups as (nkeys + naggs) consecutive 64-bit columns.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

MASK64 = (1 << 64) - 1


def owner_of(k1: np.ndarray, k2: Optional[np.ndarray], nparts: int) -> np.ndarray:
    """Host restatement of the device owner hash (csrc/common.hpp owner_hash) for tests
    and host-side tooling: mix64(k1 ^ 0x6A09E667F3BCC908) [then mix64(h ^ k2)] % P."""
    def mix(z):
        z = z.astype(np.uint64)
        with np.errstate(over="ignore"):
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

    h = mix(k1.view(np.uint64) ^ np.uint64(0x6A09E667F3BCC908))
    if k2 is not None:
        h = mix(h ^ k2.view(np.uint64))
    return (h % np.uint64(nparts)).astype(np.int64)


def exchange_partials(buf: torch.Tensor, counts: List[int], width: int, group=None) -> List[torch.Tensor]:
    """All-to-all of partitioned partial groups.  `buf` holds P column-major segments
    (segment p: counts[p] groups x `width` int64 words).  Returns the P segments this
    rank receives, each a [width, c] int64 view (c may be 0)."""
    world = dist.get_world_size(group)
    dev = buf.device
    send = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    rc = [int(x) for x in recv.tolist()]
    out = torch.empty(width * sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, buf.reshape(-1)[: width * sum(counts)].contiguous(),
                           [width * c for c in rc], [width * c for c in counts], group=group)
    segs, off = [], 0
    for c in rc:
        segs.append(out[width * off: width * (off + c)].view(width, c))
        off += c
    assert len(segs) == world
    return segs


def gather_groups(mine: torch.Tensor, group=None, dst: int = 0) -> Optional[torch.Tensor]:
    """Collect every owner's [width, n_r] groups on rank `dst` (padded all_gather: the
    final group count is small).  Returns [width, sum n_r] on dst, None elsewhere."""
    world = dist.get_world_size(group)
    width = mine.shape[0]
    dev = mine.device
    cnt = torch.tensor([mine.shape[1]], dtype=torch.int64, device=dev)
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    ns = [int(c.item()) for c in cnts]
    mx = max(max(ns), 1)
    pad = torch.zeros((width, mx), dtype=torch.int64, device=dev)
    pad[:, : mine.shape[1]] = mine
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    if dist.get_rank(group) != dst:
        return None
    return torch.cat([b[:, :n] for b, n in zip(bufs, ns)], dim=1)


def distributed_groupby(ex, local, merge_query: Callable[[torch.Tensor], "object"], group_hint: int,
                        group=None) -> Optional[torch.Tensor]:
    """Full multi-GPU group-by step after the local scan.

    `local` is this rank's nut_groups result (Groups); `merge_query(seg)` builds the
    AggQuery that merges one received [width, c] segment.  Returns the final groups as a
    [width, G] int64 tensor on rank 0 (unordered; f64 words as bits), None elsewhere."""
    world = dist.get_world_size(group)
    width = local.nkeys + local.naggs
    buf, counts = local.partition(world)
    segs = exchange_partials(buf, counts, width, group)
    owner = None
    for seg in segs:
        if seg.shape[1] == 0:
            continue
        q = merge_query(seg)
        if owner is None:
            owner = ex.groupby(q, group_hint=group_hint)
        else:
            ex.accumulate(q, owner)
    if owner is not None:
        mine = owner.to_device()
        owner.free()
    else:
        mine = torch.empty((width, 0), dtype=torch.int64, device=ex.device)
    return gather_groups(mine, group)


# ---------------------------------------------------------------------------- sample sort
def choose_splitters(local: torch.Tensor, group=None, samples_per_rank: int = 4096) -> np.ndarray:
    """Regular sample of the local keys -> all_gather -> P-1 splitters at the global
    sample's quantiles (host array, ascending).  The sample is a strided read of
    `samples_per_rank` keys (with repetition when the shard is smaller); a rank with no
    keys contributes nothing (its sample slots are masked by a gathered count)."""
    world = dist.get_world_size(group)
    n = local.numel()
    dev = local.device
    S = samples_per_rank
    if n:
        idx = (torch.arange(S, device=dev, dtype=torch.int64) * n) // S
        sample = local[idx].contiguous()
    else:
        sample = torch.zeros(S, dtype=torch.int64, device=dev)
    have = torch.tensor([1 if n else 0], dtype=torch.int64, device=dev)
    samples = [torch.empty_like(sample) for _ in range(world)]
    haves = [torch.empty_like(have) for _ in range(world)]
    dist.all_gather(samples, sample, group=group)
    dist.all_gather(haves, have, group=group)
    pool = np.concatenate([s.cpu().numpy() for s, h in zip(samples, haves) if int(h.item())] or
                          [np.zeros(0, np.int64)])
    if len(pool) == 0:
        return np.zeros(world - 1, dtype=np.int64)
    pool.sort()
    m = len(pool)
    return np.array([pool[(i * m) // world] for i in range(1, world)], dtype=np.int64)


def exchange_keys(part: torch.Tensor, counts: List[int], group=None) -> torch.Tensor:
    """All-to-all of the bucket-partitioned keys: segment p (counts[p] keys) goes to rank p.
    Returns this rank's received keys, concatenated in source-rank order."""
    dev = part.device
    send = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    rc = [int(x) for x in recv.tolist()]
    out = torch.empty(sum(rc), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, part[: sum(counts)].contiguous(), rc, list(counts), group=group)
    return out


def join_owner(keys: np.ndarray, nparts: int) -> np.ndarray:
    """Host restatement of nut_hash_partition_i64's part of a key: the top byte of the
    group-by's owner hash, split into nparts ranges: ((owner_hash(k) >> 56) * P) >> 8."""
    def mix(z):
        z = z.astype(np.uint64)
        with np.errstate(over="ignore"):
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

    d = mix(np.asarray(keys, dtype=np.int64).view(np.uint64) ^ np.uint64(0x6A09E667F3BCC908)) >> np.uint64(56)
    return ((d.astype(np.int64) * nparts) >> 8).astype(np.int64)


def exchange_rows(keys: torch.Tensor, rows: torch.Tensor, counts: List[int], group=None):
    """All-to-all of (key, row id) records partitioned by destination rank: segment p
    (counts[p] records) goes to rank p.  Returns the received (keys, rows)."""
    dev = keys.device
    n = sum(counts)
    send = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    rc = [int(x) for x in recv.tolist()]
    pack = torch.stack([keys[:n], rows[:n]], dim=1).contiguous()  # [n, 2]: one record per row
    out = torch.empty((sum(rc), 2), dtype=torch.int64, device=dev)
    dist.all_to_all_single(out, pack, rc, list(counts), group=group)
    return out[:, 0].contiguous(), out[:, 1].contiguous()


def distributed_join(build: torch.Tensor, probe: torch.Tensor, partition: Callable, join: Callable,
                     how: str = "inner", build_row0: int = 0, probe_row0: int = 0, group=None):
    """Multi-GPU hash join (the group-by's key-hash exchange reused):
    both sides are partitioned by part = join_owner(key, P) (`partition(keys, row0, P) ->
    (keys, rows, counts)`, nut_hash_partition_i64 on a GPU), ONE all-to-all per side moves
    (key, global row) records to their owner, and each rank joins what it owns (`join(build
    keys, probe keys, how) -> (probe_idx, build_idx)`, nut_join_i64_into).  Every key's
    build and probe rows meet on one rank, so INNER / LEFT / SEMI / ANTI keep their global
    meaning.  Returns this rank's pairs as GLOBAL (probe row, build row), -1 = no build row;
    each rank's pairs are grouped by the owner's received probe order."""
    world = dist.get_world_size(group)
    bk, br, bc = partition(build, build_row0, world)
    pk, pr, pc = partition(probe, probe_row0, world)
    rbk, rbr = exchange_rows(bk, br, bc, group)
    rpk, rpr = exchange_rows(pk, pr, pc, group)
    pi, bi = join(rbk, rpk, how)
    gp = rpr[pi]
    if rbr.numel() == 0:
        return gp, bi.clone()
    gb = torch.where(bi >= 0, rbr[bi.clamp(min=0)], bi)
    return gp, gb


def distributed_sort(local: torch.Tensor, partition: Callable, sort: Callable, group=None,
                     samples_per_rank: int = 4096) -> torch.Tensor:
    """Multi-GPU ORDER BY k (BASELINE config 5): sample -> splitters ->
    local stable partition into P buckets (`partition(keys, splitters) -> (keys, counts)`,
    nut_partition_i64 on a GPU) -> ONE all-to-all of keys over RCCL -> local radix sort
    (`sort(keys) -> keys`, nut_sort_i64).  Rank r returns the r-th range of the global
    order: every key on rank r is <= every key on rank r+1 (keys equal to a splitter all
    land on the higher rank)."""
    splitters = choose_splitters(local, group, samples_per_rank)
    part, counts = partition(local, splitters)
    recv = exchange_keys(part, counts, group)
    return sort(recv)

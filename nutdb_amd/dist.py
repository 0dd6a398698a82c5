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

import ctypes as C
import weakref
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
def choose_splitters(local: torch.Tensor, group=None, samples_per_rank: int = 4096, with_pool: bool = False):
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
    pool.sort()
    m = len(pool)
    spl = np.array([pool[(i * m) // world] if m else 0 for i in range(1, world)], dtype=np.int64)
    return (spl, pool) if with_pool else spl


INT64_MAX = (1 << 63) - 1


def sort_ranges(splitters, pool, world):
    """Skew-safe key ranges of the sample sort (restatement of csrc/dist.cpp sort_ranges).
    A key k goes to rank #{i : s[i] <= k}, except a key equal to a splitter value v at
    positions a..b: it may sit on ranks a .. b+1 (the ranks in between hold only v), split
    in proportion to how much of v's run in the sorted pooled sample `pool` falls in each
    rank's quantile range.  Returns (e, lo, hi, w): the strictly ascending partition
    splitters (an equal-key bucket is [v, v+1)), each bucket's rank range and weights."""
    pool = np.asarray(pool, dtype=np.int64)
    m = len(pool)
    s = [int(x) for x in splitters]
    vs = []  # [v, a, b]
    for i, v in enumerate(s):
        if vs and vs[-1][0] == v:
            vs[-1][2] = i
        else:
            vs.append([v, i, i])

    def n_e(all_):
        m = 0
        for i, (v, a, b) in enumerate(vs):
            m += 1
            if (all_ or b > a) and v != INT64_MAX and not (i + 1 < len(vs) and vs[i + 1][0] == v + 1):
                m += 1
        return m
    all_ = n_e(True) <= 63
    e, lo, hi, w = [], [0], [0], [[1]]
    for i, (v, a, b) in enumerate(vs):
        e.append(v)
        if all_ or b > a:
            f = int(np.searchsorted(pool, v, "left"))
            l_ = int(np.searchsorted(pool, v, "right"))
            ws = [max(0, min(l_, (t + 1) * m // world) - max(f, t * m // world)) for t in range(a, b + 2)]
            lo.append(a)
            hi.append(b + 1)
            w.append(ws if sum(ws) else [1] * len(ws))
            if v != INT64_MAX and not (i + 1 < len(vs) and vs[i + 1][0] == v + 1):
                e.append(v + 1)
                lo.append(b + 1)
                hi.append(b + 1)
                w.append([1])
        else:
            lo.append(b + 1)
            hi.append(b + 1)
            w.append([1])
    return np.array(e, dtype=np.int64), lo, hi, w


def split_counts(bucket_counts, lo, w, world):
    """Per-destination key counts: bucket j's keys over ranks lo[j] .. by weight w[j]
    (cumulative rounding; bucket order = destination order, so each rank's keys stay
    contiguous in the partitioned array)."""
    out = [0] * world
    for c, a, ws in zip(bucket_counts, lo, w):
        W, acc, prev = sum(ws), 0, 0
        for t, x in enumerate(ws):
            acc += x
            upto = c * acc // W
            out[a + t] += upto - prev
            prev = upto
    return out


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
    skew-safe ranges (sort_ranges) -> local stable partition into their buckets
    (`partition(keys, splitters) -> (keys, counts)`, nut_partition_i64 on a GPU) -> ONE
    all-to-all of keys -> local radix sort (`sort(keys) -> keys`, nut_sort_i64).  Rank r
    returns the r-th range of the global order: every key on rank r is <= every key on
    rank r+1; a key filling several quantiles of the sample is spread over their ranks.
    (Restatement for the gloo tests; the product path is nut_dist_sort_i64.)"""
    world = dist.get_world_size(group)
    splitters, pool = choose_splitters(local, group, samples_per_rank, with_pool=True)
    e, lo, hi, w = sort_ranges(splitters, pool, world)
    part, bcounts = partition(local, e)
    counts = split_counts(bcounts, lo, w, world)
    recv = exchange_keys(part, counts, group)
    return sort(recv)


# ---------------------------------------------------------------------------- nut_dist
class _MemberEx:
    """What Groups needs of an executor: the member's context and device."""

    def __init__(self, ctx, device: torch.device):
        self.ctx = ctx
        self.device = device


class NutDist:
    """The library's own multi-GPU path (include/nutexec.h nut_dist_*): RCCL communicators
    and the partition / all-to-all / merge steps live inside libnutexec.so, so a host
    without torch.distributed (the Rust / C hosts of INTEGRATION.md) drives every GPU of
    the exchange through the C ABI alone.  Three constructors:
      NutDist.create([0, 1, ...])          one process drives several GPUs (ncclCommInitAll)
      NutDist.create_rank(P, r, uid, dev)  one process per GPU (ncclCommInitRank); rank 0
                                           makes `uid` with NutDist.unique_id()
      NutDist.virtual(P, dev)              P ranks on one GPU, exchanges as device copies
    Every call takes one entry per local member (member l = global rank first_rank + l)."""

    def __init__(self, handle: C.c_void_p, devices):
        from ._lib import lib
        self.h = handle
        P, nl, first = C.c_int(), C.c_int(), C.c_int()
        _check(lib.nut_dist_info(self.h, C.byref(P), C.byref(nl), C.byref(first)), "nut_dist_info")
        self.nranks, self.nlocal, self.first_rank = P.value, nl.value, first.value
        self.devices = [torch.device("cuda", d) for d in devices]
        self.members = [_MemberEx(C.c_void_p(lib.nut_dist_ctx(self.h, l)), self.devices[l]) for l in range(self.nlocal)]
        self._results = weakref.WeakSet()  # Groups on member contexts: freed before the members

    @staticmethod
    def unique_id() -> bytes:
        from ._lib import NUT_DIST_ID_BYTES, lib
        buf = C.create_string_buffer(NUT_DIST_ID_BYTES)
        _check(lib.nut_dist_unique_id(buf), "nut_dist_unique_id")
        return buf.raw

    @classmethod
    def create(cls, devices) -> "NutDist":
        from ._lib import lib
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _check(lib.nut_dist_create(len(devices), devs, C.byref(h)), "nut_dist_create")
        return cls(h, list(devices))

    @classmethod
    def create_rank(cls, nranks: int, rank: int, uid: bytes, device: int) -> "NutDist":
        from ._lib import lib
        h = C.c_void_p()
        _check(lib.nut_dist_create_rank(nranks, rank, C.create_string_buffer(uid, len(uid)), device, C.byref(h)),
               "nut_dist_create_rank")
        return cls(h, [device])

    @classmethod
    def virtual(cls, nranks: int, device: int = 0) -> "NutDist":
        from ._lib import lib
        h = C.c_void_p()
        _check(lib.nut_dist_create_virtual(nranks, device, C.byref(h)), "nut_dist_create_virtual")
        return cls(h, [device] * nranks)

    def close(self) -> None:
        from ._lib import lib
        if self.h:
            for g in list(self._results):  # a result must not outlive its member's context
                g.free()
            lib.nut_dist_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def ctx(self, l: int):
        return self.members[l].ctx

    def _ready(self):
        # inputs come from torch's streams; the members run on their own
        for d in set(self.devices):
            torch.cuda.synchronize(d)

    def _copy_out(self, l: int, ptr: int, n: int) -> torch.Tensor:
        from ._lib import lib
        out = torch.empty(n, dtype=torch.int64, device=self.devices[l])
        if n:
            torch.cuda.synchronize(self.devices[l])
            _check(lib.nut_ctx_memcpy(self.members[l].ctx, C.c_void_p(out.data_ptr()), C.c_void_p(ptr), n * 8),
                   "nut_ctx_memcpy")
        return out

    def groupby(self, queries, group_hint: int = 0):
        """nut_dist_groupby: queries[l] = member l's AggQuery / ProgQuery over its shard.
        Returns one entry per member: the global Groups on the member holding rank 0, None
        on the others."""
        from ._lib import NutAggSpec, lib
        from .executor import Groups
        specs = (NutAggSpec * self.nlocal)()
        keep = []
        for l, q in enumerate(queries):
            s = q.to_spec(self.devices[l])
            keep.append(s)
            C.memmove(C.byref(specs[l]), C.byref(s), C.sizeof(NutAggSpec))
        out = (C.c_void_p * self.nlocal)()
        self._ready()
        _check(lib.nut_dist_groupby(self.h, specs, group_hint, out), "nut_dist_groupby")
        res = []
        for l, q in enumerate(queries):
            res.append(Groups(self.members[l], out[l], max(specs[l].nkeys, 1), q.result_types()) if out[l] else None)
            if res[-1] is not None:
                self._results.add(res[-1])
        return res

    def sort_i64(self, cols, copy: bool = True):
        """nut_dist_sort_i64: member l's sorted key range (the r-th of the global order) —
        copied into a tensor, or (copy=False) the member-owned (device address, count),
        valid until the member's next nut_dist call."""
        from ._lib import lib
        ins = (C.c_void_p * self.nlocal)(*[c.data_ptr() if c.numel() else None for c in cols])
        ns = (C.c_uint64 * self.nlocal)(*[c.numel() for c in cols])
        outs = (C.c_void_p * self.nlocal)()
        on = (C.c_uint64 * self.nlocal)()
        self._ready()
        _check(lib.nut_dist_sort_i64(self.h, ins, ns, outs, on), "nut_dist_sort_i64")
        if not copy:
            return [(outs[l], on[l]) for l in range(self.nlocal)]
        return [self._copy_out(l, outs[l], on[l]) for l in range(self.nlocal)]

    def enable_timing(self, on: bool = True) -> None:
        """hipEvent timing of the hot kernels on every member context (nut_ctx_enable_timing)."""
        from ._lib import lib
        for m in self.members:
            _check(lib.nut_ctx_enable_timing(m.ctx, int(on)), "nut_ctx_enable_timing")

    def kernel_time(self, kind: int, l: int = 0):
        """(total ms, launches) of one kernel kind on member l since the last call."""
        from ._lib import lib
        ms, cnt = C.c_double(), C.c_uint64()
        _check(lib.nut_ctx_kernel_time(self.members[l].ctx, kind, C.byref(ms), C.byref(cnt)), "nut_ctx_kernel_time")
        return ms.value, cnt.value

    def sort_stats(self, l: int = 0):
        """(algorithmic bytes, scatter levels) of member l's last local sort."""
        from ._lib import lib
        b, lv = C.c_uint64(), C.c_uint32()
        _check(lib.nut_ctx_sort_stats(self.members[l].ctx, C.byref(b), C.byref(lv)), "nut_ctx_sort_stats")
        return b.value, lv.value

    def filter_i64(self, cols, op, k: int):
        """nut_dist_filter_i64: [(selected values of member l, global offset)]."""
        from ._lib import lib
        from .executor import CMP
        outs = [torch.empty(max(c.numel(), 1), dtype=torch.int64, device=self.devices[l]) for l, c in enumerate(cols)]
        ins = (C.c_void_p * self.nlocal)(*[c.data_ptr() if c.numel() else None for c in cols])
        ns = (C.c_uint64 * self.nlocal)(*[c.numel() for c in cols])
        op_ = (C.c_void_p * self.nlocal)(*[o.data_ptr() for o in outs])
        on = (C.c_uint64 * self.nlocal)()
        off = (C.c_uint64 * self.nlocal)()
        self._ready()
        _check(lib.nut_dist_filter_i64(self.h, ins, ns, CMP[op] if isinstance(op, str) else int(op), int(k), op_, on,
                                       off), "nut_dist_filter_i64")
        return [(outs[l][:on[l]], int(off[l])) for l in range(self.nlocal)]

    def join_i64(self, builds, probes, how: str = "inner", build_row0=None, probe_row0=None, copy: bool = True):
        """nut_dist_join_i64: [(global probe rows, global build rows)] per member (copy=False:
        the member-owned (probe address, build address, pairs))."""
        from ._lib import lib
        from .executor import Executor
        L_ = self.nlocal
        bro = build_row0 if build_row0 is not None else [0] * L_
        pro = probe_row0 if probe_row0 is not None else [0] * L_
        bp = (C.c_void_p * L_)(*[t.data_ptr() if t.numel() else None for t in builds])
        bn = (C.c_uint64 * L_)(*[t.numel() for t in builds])
        pp = (C.c_void_p * L_)(*[t.data_ptr() if t.numel() else None for t in probes])
        pn = (C.c_uint64 * L_)(*[t.numel() for t in probes])
        b0 = (C.c_int64 * L_)(*bro)
        p0 = (C.c_int64 * L_)(*pro)
        po = (C.c_void_p * L_)()
        bo = (C.c_void_p * L_)()
        npairs = (C.c_uint64 * L_)()
        self._ready()
        _check(lib.nut_dist_join_i64(self.h, bp, bn, b0, pp, pn, p0, Executor.JOIN_TYPES[how], po, bo, npairs),
               "nut_dist_join_i64")
        if not copy:
            return [(po[l], bo[l], npairs[l]) for l in range(L_)]
        return [(self._copy_out(l, po[l], npairs[l]), self._copy_out(l, bo[l], npairs[l])) for l in range(L_)]


def _check(status: int, where: str) -> None:
    from ._lib import check
    check(status, where)

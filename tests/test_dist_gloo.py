"""The N>1 group-by exchange on CPU: world_size 2 over gloo.

Each rank pre-aggregates its row shard with the C oracle (standing in for its GPU),
partitions the partial groups by the device owner hash (nutdb_amd.dist.owner_of), runs
the SAME exchange / gather code bench.py runs over RCCL (nutdb_amd.dist), merges its
owned groups, and rank 0 checks the union against a single-process oracle result.
"""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _segments(keys, words, owners, P):
    """column-major segment buffer in nut_groups_partition's layout"""
    width = keys.shape[1] + words.shape[1]
    counts, cols = [], []
    for p in range(P):
        m = owners == p
        counts.append(int(m.sum()))
        block = np.concatenate([keys[m].T, words[m].T.view(np.int64)], axis=0)  # [width, c]
        cols.append(block.reshape(-1))
    buf = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    return torch.from_numpy(np.ascontiguousarray(buf)), counts, width


def _worker(rank, world, port, n, G, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from oracle import oracle as orc
    from nutdb_amd.dist import exchange_partials, gather_groups, owner_of
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = n // world
        key = orc.gen_column(2, 0x51, rows, row0=rank * rows, a=G)
        val = orc.gen_column(4, 0x52, rows, row0=rank * rows)
        aggs = [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,))]
        k, w = orc.groupby([key], aggs, values=[val])
        buf, counts, width = _segments(k, w, owner_of(k[:, 0], None, world), world)
        segs = exchange_partials(buf, counts, width)
        recv = torch.cat(segs, dim=1).numpy()
        # owner merge: SUM of sums, SUM of counts (i64), MIN of mins, MAX of maxes
        mk, mw = orc.groupby([recv[0]], [(0, 0, (0,)), (0, 0, (1,)), (2, 0, (2,)), (3, 0, (3,))],
                             values=[recv[1].view(np.float64), recv[2], recv[3].view(np.float64),
                                     recv[4].view(np.float64)])
        # every received key must be owned by this rank
        assert np.all(owner_of(mk[:, 0], None, world) == rank)
        mine = torch.from_numpy(np.ascontiguousarray(np.concatenate([mk.T, mw.T.view(np.int64)], axis=0)))
        allg = gather_groups(mine)
        if rank == 0:
            q.put(allg.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("G", [7, 1000])
def test_exchange_world2(G, orc):
    n = 400_000
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, G, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    order = np.argsort(got[0], kind="stable")
    got = got[:, order]
    key = orc.gen_column(2, 0x51, n, a=G)
    val = orc.gen_column(4, 0x52, n)
    ok, ow = orc.groupby([key], [(0, 0, (0,)), (1, 0, ()), (2, 0, (0,)), (3, 0, (0,))], values=[val])
    assert np.array_equal(got[0], ok[:, 0])
    s = got[1].view(np.float64)
    assert np.max(np.abs(s - ow[:, 0].view(np.float64)) / np.abs(ow[:, 0].view(np.float64))) <= 1e-12
    assert np.array_equal(got[2], ow[:, 1].view(np.int64))
    assert np.array_equal(got[3], ow[:, 2].view(np.int64))
    assert np.array_equal(got[4], ow[:, 3].view(np.int64))


# ---------------------------------------------------------------------------- sample sort
def _np_partition(keys, splitters):
    """stands in for nut_partition_i64: stable, bucket = #splitters <= key"""
    k = keys.numpy()
    b = np.searchsorted(splitters, k, side="right")
    order = np.argsort(b, kind="stable")
    counts = np.bincount(b, minlength=len(splitters) + 1)
    return torch.from_numpy(np.ascontiguousarray(k[order])), [int(c) for c in counts]


def _sort_keys(orc, kind, rows, row0):
    if kind == "heavy":  # half the rows hold one key (skew-safe splitters)
        k = orc.gen_column(1, 0x50, rows, row0=row0)
        k[(np.arange(rows) + row0) % 2 == 0] = 12345
        return k
    a, b = (0, 0) if kind == 1 else (-3, 7)  # kind 5 (RANGE_I64): heavy duplicates, splitter ties
    return orc.gen_column(kind, 0x50, rows, row0=row0, a=a, b=b)


def _sort_worker(rank, world, port, n, kind, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from oracle import oracle as orc
    from nutdb_amd.dist import distributed_sort, gather_groups
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = n // world
        local = torch.from_numpy(_sort_keys(orc, kind, rows, rank * rows))
        out = distributed_sort(local, _np_partition, lambda t: torch.from_numpy(np.sort(t.numpy())),
                               samples_per_rank=256)
        q.put((rank, len(out)))
        allg = gather_groups(out.view(1, -1))
        if rank == 0:
            q.put(allg.numpy()[0])
    finally:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------- hash join
def _np_hash_partition(keys, row0, P):
    """stands in for nut_hash_partition_i64: (keys, row0 + row, counts) grouped by join_owner"""
    from nutdb_amd.dist import join_owner
    k = keys.numpy()
    o = join_owner(k, P)
    order = np.argsort(o, kind="stable")
    rows = np.arange(len(k), dtype=np.int64) + row0
    return (torch.from_numpy(np.ascontiguousarray(k[order])), torch.from_numpy(rows[order]),
            [int(c) for c in np.bincount(o, minlength=P)])


def _join_tables(world, nb, npr, rank):
    """rank's build / probe shards of one global pair of tables (keys with repeats)"""
    rng = np.random.default_rng(77)
    b = rng.integers(0, nb // 2, nb).astype(np.int64) * 3
    p = rng.integers(-20, nb * 2, npr).astype(np.int64)
    bs, ps = np.array_split(b, world), np.array_split(p, world)
    b0 = sum(len(x) for x in bs[:rank])
    p0 = sum(len(x) for x in ps[:rank])
    return b, p, bs[rank], ps[rank], b0, p0


def _join_worker(rank, world, port, nb, npr, how, q):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from oracle import oracle as orc
    from nutdb_amd.dist import distributed_join, gather_groups, join_owner
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, _, bs, ps, b0, p0 = _join_tables(world, nb, npr, rank)

        def local_join(bk, pk, how_):
            # every received key is owned by this rank
            assert np.all(join_owner(bk.numpy(), world) == rank) and np.all(join_owner(pk.numpy(), world) == rank)
            pi, bi = orc.join_i64(bk.numpy(), pk.numpy(), how_)
            return torch.from_numpy(pi), torch.from_numpy(bi)

        gp, gb = distributed_join(torch.from_numpy(bs), torch.from_numpy(ps), _np_hash_partition, local_join,
                                  how, b0, p0)
        allg = gather_groups(torch.stack([gp, gb]))
        if rank == 0:
            q.put(allg.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,how", [(2, "inner"), (3, "inner"), (2, "left"), (3, "semi"), (2, "anti")])
def test_distributed_join(world, how, orc):
    nb, npr = 20_000, 60_001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_join_worker, args=(r, world, port, nb, npr, how, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    b, p, *_ = _join_tables(world, nb, npr, 0)
    wp, wb = orc.join_i64(b, p, how)
    o = np.lexsort((got[1], got[0]))
    assert np.array_equal(got[0][o], wp) and np.array_equal(got[1][o], wb)


@pytest.mark.parametrize("world,kind", [(2, 1), (3, 1), (2, 5), (2, "heavy"), (3, "heavy")])
def test_sample_sort(world, kind, orc):
    n = 300_000 - (300_000 % world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sort_worker, args=(r, world, port, n, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=240) for _ in range(world + 1)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = [m for m in msgs if not isinstance(m, tuple)][0]
    sizes = dict(m for m in msgs if isinstance(m, tuple))
    want = np.sort(_sort_keys(orc, kind, n, 0))
    assert np.array_equal(got, want)
    if kind != 5:  # (kind 5 has only 7 distinct keys: ranges cannot balance finer than a key)
        assert max(sizes.values()) <= 1.25 * n / world, sizes


def test_sort_ranges_split_heavy_keys():
    """sort_ranges (the restatement of csrc/dist.cpp's): a key filling several sample
    quantiles is spread over their ranks; concatenating the ranks stays sorted."""
    from nutdb_amd.dist import sort_ranges, split_counts
    pool = [1] * 25 + [5] * 70 + [9] * 5  # P = 4: key 5 fills [25, 95) of the pool
    spl = [pool[i * 100 // 4] for i in range(1, 4)]
    assert spl == [5, 5, 5]
    e, lo, hi, w = sort_ranges(spl, pool, 4)
    assert e.tolist() == [5, 6] and lo == [0, 0, 3] and hi == [0, 3, 3]
    assert w[1] == [0, 25, 25, 20]  # v's share of each rank's quantile range
    assert split_counts([250, 700, 50], lo, w, 4) == [250, 250, 250, 250]
    e, lo, hi, w = sort_ranges([1, 2, 9], [0, 1, 2, 9], 4)  # light keys get their own bucket too
    assert e.tolist() == [1, 2, 3, 9, 10] and lo == [0, 0, 1, 2, 2, 3] and hi == [0, 1, 2, 2, 3, 3]
    e, lo, hi, w = sort_ranges([2**63 - 1], [0, 2**63 - 1], 2)
    assert e.tolist() == [2**63 - 1] and lo == [0, 0] and hi == [0, 1]
    s = sorted(np.random.default_rng(1).integers(0, 40, 63).tolist())  # 64 ranks, many repeats
    e, lo, hi, w = sort_ranges(s, s, 64)
    assert len(e) <= 63 and all(np.diff(e) > 0)
    assert all(a <= b for a, b in zip(lo, hi)) and all(h <= l2 for h, l2 in zip(hi, lo[1:]))

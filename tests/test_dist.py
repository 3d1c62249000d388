"""Contig sharding and the region-table exchange (CPU, gloo, world size 2)."""
import os
import socket

import numpy as np
import pytest

from metacov_amd import dist as mdist
from metacov_amd.engine import REGION_STAT_DTYPE


def test_lpt_balances_and_partitions():
    rng = np.random.default_rng(0)
    costs = rng.lognormal(0, 1, size=1000) * 1e6
    for world in (1, 2, 3, 8):
        shards = mdist.lpt_shard(costs, world)
        allc = np.sort(np.concatenate(shards))
        assert np.array_equal(allc, np.arange(1000))
        loads = [costs[s].sum() for s in shards]
        # LPT bound: max load <= 4/3 OPT (+ one item); check against the mean
        assert max(loads) <= costs.sum() / world + costs.max() + 1e-6


def test_select_reads_remap():
    tid = np.array([0, 0, 1, 2, 2, 3], np.int32)
    mask, remap = mdist.select_reads(tid, np.array([1, 3]))
    assert mask.tolist() == [False, False, True, False, False, True]
    assert remap[tid[mask]].tolist() == [0, 1]


def _rows(n, seed):
    rng = np.random.default_rng(seed)
    r = np.zeros(n, REGION_STAT_DTYPE)
    for f in REGION_STAT_DTYPE.names:
        r[f] = rng.integers(0, 1 << 40, size=n)
    r["sumsq"][0] = np.uint64(1 << 63) + np.uint64(5)    # survives the int64 view
    return r


def test_pack_unpack_roundtrip():
    rows = _rows(7, 1)
    idx = np.array([6, 0, 5, 1, 4, 2, 3])
    t = mdist.pack_rows(rows, idx)
    pad = np.full((3, mdist.ROW_WIDTH), -1, np.int64)
    back = mdist.unpack_rows(np.concatenate([t, pad]), 7, REGION_STAT_DTYPE)
    for f in REGION_STAT_DTYPE.names:
        assert np.array_equal(back[f][idx], rows[f])
    with pytest.raises(RuntimeError):
        mdist.unpack_rows(t[:5], 7, REGION_STAT_DTYPE)
    assert np.isnan(mdist.unpack_std(t, 7)).all()
    # numpy's std column (engine.numpy_std) travels with its row
    std = np.array([np.nan, 0.285, np.nan, 1e-300, 3.0, np.nan, 0.2849999999999999])
    t = mdist.pack_rows(rows, idx, std)
    got = mdist.unpack_std(np.concatenate([pad, t]), 7)
    assert np.array_equal(got[idx], std, equal_nan=True)
    # the bench's tables carry no std column
    assert np.array_equal(mdist.unpack_rows(np.delete(t, -2, axis=1), 7, REGION_STAT_DTYPE), back)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_regions, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # each rank owns an LPT shard of the "contigs" (= regions here)
        costs = np.arange(1, n_regions + 1, dtype=np.float64)
        owned = mdist.lpt_shard(costs, world)[rank]
        all_rows = _rows(n_regions, 9)
        table = mdist.pack_rows(all_rows[owned], owned)
        out = mdist.all_gather_table(table, r_max=n_regions)
        rows = mdist.unpack_rows(out, n_regions, REGION_STAT_DTYPE)
        ok = all(np.array_equal(rows[f], all_rows[f]) for f in REGION_STAT_DTYPE.names)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_gloo_all_gather_world2():
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, 11, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def _err_worker(rank, world, port, bad_rank, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        err = OSError("shard unreadable") if rank == bad_rank else None
        try:
            mdist.agree_on_error(err)
            q.put((rank, "none"))
        except mdist.PeerRankError:
            q.put((rank, "peer"))
        except OSError:
            q.put((rank, "own"))
        # everyone is still in step: a later collective completes
        out = mdist.all_gather_table(np.zeros((0, mdist.ROW_WIDTH), np.int64), r_max=1)
        assert out.shape == (world, mdist.ROW_WIDTH)
    finally:
        dist.destroy_process_group()


def test_gloo_error_agreement_world2():
    """One rank's failure (cli.pileup_distributed's per-rank work) reaches
    every rank through one all-reduce: the failing rank re-raises its own
    error, the others raise PeerRankError, none blocks in the table gather."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    for bad in (1, None):
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_err_worker, args=(r, 2, port, bad, q)) for r in range(2)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=120) for _ in ps)
        for p in ps:
            p.join(timeout=60)
        want = [(0, "peer"), (1, "own")] if bad == 1 else [(0, "none"), (1, "none")]
        assert res == want


def _bcast_worker(rank, world, port, fail, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def root_work():   # rank 0 only (the whole-file decode of cli._pileup_shard)
            if fail:
                raise OSError("no valid BGZF block")
            return {"ext": np.arange(5, dtype=np.int64), "names": ("a", "b")}
        try:
            got = mdist.broadcast_result(root_work, rank)
            q.put((rank, "ok", got["ext"].tolist(), got["names"]))
        except mdist.PeerRankError:
            q.put((rank, "peer", None, None))
        except OSError:
            q.put((rank, "own", None, None))
        # still in step afterwards
        mdist.agree_on_error(None)
    finally:
        dist.destroy_process_group()


def test_gloo_broadcast_result_world2():
    """The root's result (the extents table of a BAM without an index)
    reaches every rank; a failure on the root raises there and as
    PeerRankError on the other rank, and nobody blocks."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    for fail in (False, True):
        q = ctx.Queue()
        port = _free_port()
        ps = [ctx.Process(target=_bcast_worker, args=(r, 2, port, fail, q)) for r in range(2)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=120) for _ in ps)
        for p in ps:
            p.join(timeout=60)
        if fail:
            assert res == [(0, "own", None, None), (1, "peer", None, None)]
        else:
            assert res == [(r, "ok", [0, 1, 2, 3, 4], ("a", "b")) for r in (0, 1)]

"""Contig sharding across the GPUs of one node and the region-table exchange.

Depth at a position depends only on the reads of its contig and every
region lies inside one contig (metacov/cli.py:86-91), so contigs are the
shard unit (SURVEY.md §8 e): each rank owns whole contigs, computes their
depth and reduces the regions that lie on them with no data-path
communication.  The only exchange is the final per-region table: one
all-gather of a fixed-size padded int64 table over RCCL ("nccl" backend on
ROCm, xGMI) — KB-scale and latency-bound — after which every rank holds all
rows in input order (rank 0 writes the CSV).
"""
import heapq

import numpy as np

STAT_FIELDS = ("n", "sum", "sumsq", "min", "max", "med_lo", "med_hi", "q23_sum", "q23_cnt")
# + numpy's std near a rounding tie (float64 bits, NaN: none; engine.numpy_std)
# + original region index.  unpack_rows also takes tables without the std
# column (the bench's device rows).
ROW_WIDTH = len(STAT_FIELDS) + 2
_NAN_BITS = np.array([np.nan]).view(np.int64)[0]


def lpt_shard(costs, world):
    """Longest-processing-time greedy: contigs sorted by cost descending,
    each to the currently least-loaded rank.  Returns a list of sorted
    contig-id arrays, one per rank."""
    costs = np.asarray(costs, dtype=np.float64)
    order = np.argsort(-costs, kind="stable")
    heap = [(0.0, r) for r in range(world)]
    owned = [[] for _ in range(world)]
    for c in order:
        load, r = heapq.heappop(heap)
        owned[r].append(int(c))
        heapq.heappush(heap, (load + float(costs[c]), r))
    return [np.array(sorted(o), dtype=np.int64) for o in owned]


def contig_costs(lengths, read_counts):
    """Cost model of K2+K3 per contig: 12 bytes per read + 8 per position
    (depth written once, read once by the region reduction)."""
    return 12.0 * np.asarray(read_counts, np.float64) + 8.0 * np.asarray(lengths, np.float64)


def select_reads(tid, owned):
    """Mask of the reads whose contig this rank owns, and the contig-id
    remap (global tid -> local tid) for the owned contigs."""
    n_contigs = int(max(int(tid.max()) + 1 if len(tid) else 0, int(owned.max()) + 1 if len(owned) else 0))
    remap = np.full(n_contigs, -1, dtype=np.int32)
    remap[owned] = np.arange(len(owned), dtype=np.int32)
    mask = remap[tid] >= 0 if len(tid) else np.zeros(0, bool)
    return mask, remap


def pack_rows(rows, index, std=None):
    """structured stat rows (+ numpy std per row, NaN / None: none) +
    original region index -> int64 [R, ROW_WIDTH]."""
    out = np.empty((len(rows), ROW_WIDTH), dtype=np.int64)
    for k, f in enumerate(STAT_FIELDS):
        out[:, k] = rows[f].astype(np.int64) if f != "sumsq" else rows[f].view(np.int64)
    if std is None:
        out[:, -2] = _NAN_BITS
    else:
        out[:, -2] = np.ascontiguousarray(std, np.float64).view(np.int64)
    out[:, -1] = index
    return out


def _live(table, n_regions):
    table = np.asarray(table)
    table = table[table[:, -1] >= 0]
    idx = table[:, -1]
    if len(np.unique(idx)) != len(idx) or len(idx) != n_regions:
        raise RuntimeError("region table gather lost or duplicated rows (%d of %d)"
                           % (len(idx), n_regions))
    return table, idx


def unpack_rows(table, n_regions, dtype):
    """int64 [*, ROW_WIDTH] (rows with index < 0 are padding) -> structured
    rows in original region order."""
    table, idx = _live(table, n_regions)
    out = np.zeros(n_regions, dtype=dtype)
    for k, f in enumerate(STAT_FIELDS):
        col = table[:, k]
        out[f][idx] = col.view(np.uint64) if f == "sumsq" else col
    return out


def unpack_std(table, n_regions):
    """The numpy-std column of a packed table in original region order
    (float64, NaN where none)."""
    table, idx = _live(table, n_regions)
    out = np.full(n_regions, np.nan)
    out[idx] = np.ascontiguousarray(table[:, -2]).view(np.float64)
    return out


def all_gather_table(local, r_max, group=None, device=None):
    """All-gather a [<= r_max, ROW_WIDTH] int64 table (numpy or torch) from
    every rank; returns the concatenated [world * r_max, ROW_WIDTH] table as
    numpy.  Padding rows carry index -1.  With the nccl (RCCL) backend the
    tensors live on `device`; with gloo on the CPU."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = device if device is not None else torch.device("cpu")
    if isinstance(local, torch.Tensor):
        t = local
    else:
        t = torch.from_numpy(np.ascontiguousarray(local, dtype=np.int64))
    buf = torch.full((r_max, ROW_WIDTH), -1, dtype=torch.int64, device=dev)
    if t.shape[0]:
        buf[:t.shape[0]] = t.to(dev)
    out = torch.empty((world * r_max, ROW_WIDTH), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, buf, group=group)
    return out.cpu().numpy()


class PeerRankError(RuntimeError):
    """Raised on the ranks whose own work succeeded when another rank failed."""


def agree_on_error(err, group=None, device=None):
    """Collective: every rank passes the exception its local work raised (or
    None).  If any rank failed, every rank raises — its own exception, or
    PeerRankError — so no rank is left blocked in a later collective waiting
    for a peer that has already given up."""
    import torch
    import torch.distributed as dist
    dev = device if device is not None else torch.device("cpu")
    flag = torch.tensor([0 if err is None else 1], dtype=torch.int64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.SUM, group=group)
    failed = int(flag.item())
    if err is not None:
        raise err
    if failed:
        raise PeerRankError("%d rank(s) failed; see their logs" % failed)


def broadcast_result(fn, rank, src=0, group=None, device=None):
    """Runs fn() on rank `src` and hands its (picklable) result to every rank
    in one broadcast.  An exception on `src` is raised there and as
    PeerRankError on the other ranks, so no rank waits on a failed root."""
    import torch.distributed as dist
    obj = [None]
    err = None
    if rank == src:
        try:
            obj = [("ok", fn())]
        except BaseException as e:   # every rank learns of it
            err = e
            obj = [("err", "%s: %s" % (type(e).__name__, e))]
    dist.broadcast_object_list(obj, src=src, group=group, device=device)
    if err is not None:
        raise err
    tag, val = obj[0]
    if tag == "err":
        raise PeerRankError("rank %d failed: %s" % (src, val))
    return val

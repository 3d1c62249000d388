"""Benchmark: aligned bases/s into the per-position depth vector (+ per-region
statistics), BASELINE.json metric, on the C3 workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

One step = one pass of the hot path over one batch of reads resident in HBM
(int32 tid, pos, span; SURVEY.md §8 d): the batch is new to the engine every
step, so the step prepares it (the direct path: probe_kernel, then K2 reads
and validates the raw tuples), computes the depth of every contig (K2) with
the whole-contig region statistics folded in, and finalizes the region table
(K3b) [+ for N > 1 the RCCL all-gather of the table].  Inputs are generated on
the GPU before timing (synthetic).

`--gpus N` without torchrun around it starts `torch.distributed.run` with N
ranks as a child process.  Default scaling is strong (BASELINE configs[3]):
ONE C3 workload, contigs LPT-sharded over the ranks; --scaling weak gives
every rank a full C3.  value = all ranks' aligned bases per second.
"""
import argparse
import json
import os
import time

import numpy as np


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks).  Without WORLD_SIZE in the environment, N > 1 starts "
                         "`torch.distributed.run --nproc-per-node N` on this script as a child process")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=["c2", "c3", "c5"],
                    help="c3 (default, BASELINE configs[2]); c2: 1 x 5 Mbp, 10M x 150 bp; "
                         "c5: 10k contigs, 50M lognormal ~10 kbp reads")
    ap.add_argument("--reads", type=int, default=None, help="reads per workload (config default)")
    ap.add_argument("--contigs", type=int, default=None)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong (default, BASELINE configs[3]): ONE workload LPT-sharded by contig over "
                         "the ranks; weak: every rank owns a full workload")
    ap.add_argument("--strong", action="store_true", help="(kept for old command lines: the default)")
    ap.add_argument("--unfused", action="store_true",
                    help="K2 then a separate K3 pass instead of the fused K2 statistics")
    ap.add_argument("--cigar", action="store_true",
                    help="raw-CIGAR input: ~Poisson(--cigar-ops) BAM CIGAR words per read resident "
                         "in HBM; each step runs K1 (CIGAR -> span) + prepare + K2 + K3b")
    ap.add_argument("--cigar-ops", type=float, default=200.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-bases", type=float, default=3.0e9,
                    help="aligned bases in the CPU-baseline sample (~10-20 s on one core)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the contig-parallel CPU baseline (0 = the best of the cgroup CPU "
                         "quota, twice it and the affinity set: SURVEY §8 d's all-cores baseline)")
    ap.add_argument("--cpu-parallel-min-s", type=float, default=2.0,
                    help="the all-cores baseline repeats the whole workload until it has run this long")
    ap.add_argument("--pcie", action="store_true", help="also time host-buffer ingest (H2D)")
    ap.add_argument("--prepare-steps", type=int, default=None,
                    help="steps of the second timed loop, which reuses one explicit prepare's index "
                         "(default: --steps; 0 = skip)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--dump-rows", default=None, metavar="PATH",
                    help="rank 0 saves the (gathered) region rows of the last step, in region "
                         "order, as a .npy (tests compare them with the oracle)")
    ap.add_argument("--exchange-every", type=int, default=8, metavar="G",
                    help="N > 1: the region tables of G consecutive steps leave in one all-gather "
                         "(one collective per step cost the N = 8 share ~20 us of host time per "
                         "step: profiles/r06/r06zg_exchange_cost.txt)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse several ranks on one GPU)")
    return ap.parse_args(argv)


def launch_ranks(args, argv):
    """`bench.py --gpus N` outside torchrun: run N ranks of this script under
    `python -m torch.distributed.run` as a CHILD process (this process never
    imports torch or touches a GPU, so nothing is exec'd over a GPU context)
    and relay rank 0's JSON line.  Returns the exit code."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    line = None
    for raw in p.stdout:                  # stderr passes straight through
        i = raw.find("{\"metric\"")
        if i >= 0:
            line = raw[i:].strip()
        else:
            sys.stderr.write(raw)
    rc = p.wait()
    if line is not None:
        print(line, flush=True)
    return rc if rc else (0 if line is not None else 1)


CONFIGS = {   # name: (reads, contigs, description)
    "c2": (10_000_000, 1, "C2: 1 contig x 5 Mbp, %d x ~150 bp reads, whole-contig stats"),
    "c3": (100_000_000, 1000, "C3 per GPU: %d contigs (~%.2f Gbp), %d x ~150 bp reads, "
                              "whole-contig region stats"),
    "c5": (50_000_000, 10_000, "C5 per GPU: %d contigs (~%.2f Gbp), %d lognormal ~10 kbp reads "
                               "(long-read path), whole-contig region stats"),
}


def config_contigs(cfg, n_reads, n_contigs):
    from metacov_amd import synth
    if cfg == "c2":
        return np.array([5_000_000], np.int64), np.ones(1)
    if cfg == "c5":
        rng = np.random.default_rng(5)
        lengths = rng.integers(50_000, 150_001, size=n_contigs).astype(np.int64)
        return lengths, lengths * rng.lognormal(0.0, 1.0, size=n_contigs)
    return synth.c3_workload(n_reads, n_contigs)


def device_workload(torch, lengths, weights, n_reads, seed, dev, long_reads=False):
    """C3-style pileup intervals generated on the GPU: coordinate-sorted
    int32 (tid, pos, span) with the SURVEY §8(d) span mix (3% soft clips,
    0.5% I, 0.5% D, 0.1% N; filtered records are not part of the stream).
    long_reads: lognormal spans, mean ~10 kbp (C5)."""
    rng = np.random.default_rng(seed)
    counts = rng.multinomial(n_reads, weights / weights.sum())
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    L = torch.from_numpy(lengths).to(dev)
    tid = torch.repeat_interleave(torch.arange(len(lengths), device=dev, dtype=torch.int32),
                                  torch.from_numpy(counts).to(dev))
    u = torch.rand(n_reads, device=dev, generator=g)
    r = torch.rand(n_reads, device=dev, generator=g)
    if long_reads:
        z = torch.randn(n_reads, device=dev, generator=g, dtype=torch.float64)
        span = torch.exp(np.log(10_000) - 0.125 + 0.5 * z).long().clamp_(min=1)
    else:
        span = torch.full((n_reads,), 150, dtype=torch.int64, device=dev)
        span -= ((u < 0.03) * (1 + (r * 29).long()))
        span -= (((u >= 0.03) & (u < 0.035)) * (1 + (r * 5).long()))
        span += (((u >= 0.035) & (u < 0.04)) * (1 + (r * 9).long()))
        span += (((u >= 0.04) & (u < 0.041)) * (50 + (r * 1950).long()))
    Lt = L[tid.long()]
    span = torch.minimum(span, Lt)
    pos = (torch.rand(n_reads, device=dev, generator=g, dtype=torch.float64) *
           (Lt - span + 1).double()).long()
    coff = torch.zeros(len(lengths) + 1, dtype=torch.int64, device=dev)
    coff[1:] = torch.cumsum(L, 0)
    key = coff[tid.long()] + pos
    order = torch.argsort(key)
    del key, u, r
    return (tid[order].contiguous(), pos[order].to(torch.int32).contiguous(),
            span[order].to(torch.int32).contiguous(), counts)


def cpu_baseline(lengths, tid, pos, span, sample_bases, label="C3"):
    """The C restatement of the reference's pileup.classic path (htslib-style
    column walk -> float64 columns -> sort-based stats) on one host core, on
    the first contigs of this workload up to `sample_bases` aligned bases."""
    from oracle import coracle
    per = np.bincount(tid, weights=span.astype(np.float64), minlength=len(lengths))
    k = int(np.searchsorted(np.cumsum(per), sample_bases)) + 1
    k = min(k, len(lengths))
    m = tid < k
    t, p, s = tid[m], pos[m], span[m]
    t0 = time.perf_counter()
    coracle.pileup_classic(t, p, s, np.arange(k, dtype=np.int32), np.zeros(k, np.int64),
                           lengths[:k].astype(np.int64))
    dt = time.perf_counter() - t0
    bases = int(s.astype(np.int64).sum())
    return {"value": bases / dt, "unit": "aligned bases/s", "cores": 1, "kind": "port",
            "sample": "first %d of the rank-0 %s contigs (%d bp, %d reads, %.3g aligned bases), "
                      "whole-contig regions, %.2f s; oracle/oracle.c orc_pileup_classic "
                      "(restated htslib column walk + pileup.classic stats)"
                      % (k, label, int(lengths[:k].sum()), len(t), bases, dt)}


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs the cgroup grants this process (cgroup v2 cpu.max, or v1 CFS
    quota / period), or None when unlimited / unknown.  The GPU box's quota
    (16) is far below its affinity set (256 CPUs)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
        if q != "max":
            return float(q) / float(per)
    except (OSError, ValueError):
        pass
    for d in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        try:
            with open(d + "/cpu.cfs_quota_us") as fh:
                q = int(fh.read())
            with open(d + "/cpu.cfs_period_us") as fh:
                per = int(fh.read())
            if q > 0 and per > 0:
                return q / per
        except (OSError, ValueError):
            pass
    return None


def cpu_thread_counts(explicit=0):
    """Thread counts the all-cores baseline tries: the cgroup quota, twice it
    and the affinity set (or an explicit count); without a readable quota,
    OMP_NUM_THREADS (the box sets it to its CPU share) stands in for it."""
    if explicit:
        return [int(explicit)]
    aff = affinity_cpus()
    q = cpu_quota()
    if q is None:
        try:
            q = float(os.environ.get("OMP_NUM_THREADS", "")) or None
        except ValueError:
            q = None
    base = max(1, int(round(q))) if q else None
    cands = {aff} if base is None else {min(base, aff), min(2 * base, aff), aff}
    return sorted(cands)


def cpu_baseline_parallel(lengths, tid, pos, span, thread_counts, min_s=2.0):
    """The same restatement, contig-parallel over the WHOLE workload (every
    contig; one core would need minutes; the costliest contigs are started
    first), on each of `thread_counts` host threads in turn, each repeated
    until it has run `min_s` seconds (SURVEY.md §8 d: the all-cores CPU
    baseline).  Reports the best; the sweep, the cgroup quota and the
    affinity set are in the record."""
    from oracle import coracle
    k = len(lengths)
    bases = int(span.astype(np.int64).sum())
    sweep = []
    for threads in thread_counts:
        args = (tid, pos, span, np.arange(k, dtype=np.int32), np.zeros(k, np.int64),
                lengths.astype(np.int64), threads)
        reps = 0
        t0 = time.perf_counter()
        while True:
            coracle.pileup_classic_parallel(*args)
            reps += 1
            dt = time.perf_counter() - t0
            if dt >= min_s or reps >= 50:
                break
        sweep.append({"threads": threads, "value": bases * reps / dt, "passes": reps, "seconds": dt})
    best = max(sweep, key=lambda r: r["value"])
    q = cpu_quota()
    return {"value": best["value"], "unit": "aligned bases/s", "cores": best["threads"], "kind": "port",
            "nproc": os.cpu_count(), "cpus_in_affinity": affinity_cpus(), "cpu_quota": q,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "sweep": sweep,
            "sample": "the whole workload (%d contigs, %.3g aligned bases) x %d passes, "
                      "contig-parallel (costliest contig first) on %d threads, %.2f s; best of %s threads"
                      % (k, bases, best["passes"], best["threads"], best["seconds"],
                         "/".join(str(r["threads"]) for r in sweep))}


def cpu_baseline_interval(lengths, tid, pos, span, sample_bases):
    """The simple interval-count CPU path on one core (difference array +
    exact counting-sort statistics: oracle orc_depth_interval +
    orc_region_stats), same sample (BASELINE.md CPU-baseline plan)."""
    from oracle import coracle
    per = np.bincount(tid, weights=span.astype(np.float64), minlength=len(lengths))
    k = min(int(np.searchsorted(np.cumsum(per), sample_bases)) + 1, len(lengths))
    m = tid < k
    t, p, s = tid[m], pos[m], span[m]
    t0 = time.perf_counter()
    d, ext, coff = coracle.depth(lengths[:k], t, p, s, method="interval")
    coracle.region_stats(d, ext, coff, np.arange(k, dtype=np.int32), np.zeros(k, np.int64),
                         lengths[:k].astype(np.int64))
    dt = time.perf_counter() - t0
    bases = int(s.astype(np.int64).sum())
    return {"value": bases / dt, "unit": "aligned bases/s", "cores": 1, "kind": "port",
            "sample": "same %d contigs as cpu_baseline, difference array + counting-sort "
                      "statistics (not the reference algorithm), %.2f s" % (k, dt)}


def kernel_source_id(root):
    """Fingerprint of the K1/K2 sources (kernels.h + engine.hip): a PMC record
    measured on other kernel code is stale and is not reported."""
    import hashlib
    h = hashlib.sha256()
    for f in ("kernels.h", "engine.hip"):
        with open(os.path.join(root, "metacov_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def load_pmc_traffic(root):
    """PMC records of profiles/pmc_depth_kernel.json measured on the current
    kernel sources (scripts/pmc_summary.py stamps each with kernel_source_id)."""
    p = os.path.join(root, "profiles", "pmc_depth_kernel.json")
    if not os.path.exists(p):
        return None
    with open(p) as fh:
        d = json.load(fh)
    sid = kernel_source_id(root)
    d["variants"] = [v for v in d.get("variants", []) if v.get("source_id") == sid]
    return d


def main():
    import sys
    argv = sys.argv[1:]
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    strong = args.scaling == "strong"
    import torch
    import torch.distributed as dist
    from metacov_amd import synth, dist as mdist
    from metacov_amd.engine import CoverageEngine, REGION_STAT_DTYPE

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # ex: the region-table exchange runs (N > 1; or one torchrun rank with
    # MC_BENCH_FORCE_EXCHANGE=1, which exercises the RCCL all-gather path on a
    # one-GPU box: tests/test_gpu_parity.py::test_bench_rccl_exchange_one_rank)
    ex = world > 1 or ("WORLD_SIZE" in os.environ and os.environ.get("MC_BENCH_FORCE_EXCHANGE") == "1")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ex:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")

    if args.prepare_steps is None:
        args.prepare_steps = args.steps
    d_reads, d_contigs, desc = CONFIGS[args.config]
    args.reads = args.reads or d_reads
    args.contigs = args.contigs or d_contigs
    long_reads = args.config == "c5"
    lengths_all, weights_all = config_contigs(args.config, args.reads, args.contigs)
    if strong:
        # one workload, contigs LPT-sharded over the ranks (at N = 1: all of it)
        tid, pos, span, counts = device_workload(torch, lengths_all, weights_all, args.reads,
                                                 args.seed, dev, long_reads)
        owned = mdist.lpt_shard(mdist.contig_costs(lengths_all, counts), world)[rank]
        remap = torch.full((len(lengths_all),), -1, dtype=torch.int32, device=dev)
        remap[torch.from_numpy(owned).to(dev)] = torch.arange(len(owned), dtype=torch.int32,
                                                              device=dev)
        lt = remap[tid.long()]
        keep = lt >= 0
        tid, pos, span = lt[keep].contiguous(), pos[keep].contiguous(), span[keep].contiguous()
        lengths = lengths_all[owned]
        region_index = owned
    else:
        tid, pos, span, _ = device_workload(torch, lengths_all, weights_all, args.reads,
                                            args.seed + 1000 * rank, dev, long_reads)
        lengths = lengths_all
        region_index = np.arange(len(lengths)) + rank * len(lengths)
    n_regions_total = int(len(lengths_all) if strong else len(lengths_all) * world)

    eng = CoverageEngine(local)
    eng.set_contigs(lengths)
    cig_off = cigar = None
    if args.cigar:
        cig_off, cigar = synth.device_cigars(torch, span, args.cigar_ops, args.seed + 7)
        torch.cuda.synchronize()
        eng.add_reads_cigar_device(tid, pos, cig_off, cigar)
    else:
        eng.add_reads(tid, pos, span)
    R = len(lengths)
    rt = np.arange(R, dtype=np.int32)
    rs = np.zeros(R, np.int64)
    re_ = lengths.astype(np.int64)
    r_max = int(n_regions_total if strong else R)
    table = torch.empty((R, 9), dtype=torch.int64, device=dev)
    gathered = None

    xbufs = coll_bufs = gouts = gidx = None
    works = [None, None]   # in-flight all-gathers, one per exchange buffer
    n_calls = [0]
    G = max(1, args.exchange_every)   # steps per all-gather
    last = [None]          # (buffer, slot) the last step wrote; ungathered[0]: its group is not sent yet
    ungathered = [False]
    if ex:
        # two exchange buffers, allocated once: [r_max, 9 stats]; the engine
        # writes a batch's rows straight into the first R of one (no copy per
        # step) while the previous batch's all-gather may still read the other,
        # and the rows' original region indices are gathered once here
        xbufs = [torch.full((G * r_max, 9), -1, dtype=torch.int64, device=dev) for _ in range(2)]
        ibuf = torch.full((r_max, 1), -1, dtype=torch.int64, device=coll_dev)
        ibuf[:R, 0] = torch.from_numpy(np.asarray(region_index, np.int64)).to(coll_dev)
        gidx = torch.empty((world * r_max, 1), dtype=torch.int64, device=coll_dev)
        dist.all_gather_into_tensor(gidx, ibuf)
        coll_bufs = [x if coll_dev == dev else torch.empty((G * r_max, 9), dtype=torch.int64, device=coll_dev)
                     for x in xbufs]
        gouts = [torch.empty((world * G * r_max, 9), dtype=torch.int64, device=coll_dev) for _ in range(2)]

    def step(fresh):
        """One pass of the hot path over the resident batch.  fresh: the
        batch is new to the engine (mc_invalidate first), so the step
        prepares it — the direct path: probe + validating K2 — before K2 and
        K3b; otherwise K2 reuses the index an explicit prepare() built.
        For N > 1 the batch's rows leave in an asynchronous all-gather that
        runs under the next batch's kernels; drain() waits for the last."""
        k = n_calls[0]
        n_calls[0] += 1
        i, slot = (k // G) & 1, k % G
        tbl = table
        if ex:
            if slot == 0 and works[i] is not None:   # this buffer's previous gather must be done
                works[i].wait()
                # RCCL: wait() only orders torch's current stream after the
                # gather; the engine writes the buffer on its own stream, so
                # the host waits for the gather itself (done two groups ago,
                # normally: one event query)
                while coll_dev.type == "cuda" and not works[i].is_completed():
                    time.sleep(0)
                works[i] = None
            tbl = xbufs[i][slot * r_max:slot * r_max + R]
        if args.cigar:   # a fresh raw-CIGAR batch: K1 + prepare run inside this step
            eng.clear_reads()
            eng.add_reads_cigar_device(tid, pos, cig_off, cigar)
        elif fresh:
            eng.invalidate()
        if args.unfused:
            eng.compute_depth()
            eng.region_stats_device(rt, rs, re_, tbl.data_ptr())
        else:
            eng.compute_depth_stats_device(rt, rs, re_, tbl.data_ptr())
        if ex:   # the rows are in the exchange buffer already: one all-gather per G steps
            last[0] = (i, slot)
            ungathered[0] = True
            if slot == G - 1:
                send(i)

    def send(i):
        nonlocal gathered
        if coll_bufs[i] is not xbufs[i]:   # (gloo: through host memory)
            coll_bufs[i].copy_(xbufs[i])
        works[i] = dist.all_gather_into_tensor(gouts[i], coll_bufs[i], async_op=True)
        gathered = gouts[i]
        ungathered[0] = False

    def drain():
        if ex and ungathered[0]:   # a partly filled group (its other slots: an older group's rows)
            send(last[0][0])
        for j, w in enumerate(works):
            if w is not None:
                w.wait()
                works[j] = None

    def sync_all():
        drain()
        torch.cuda.synchronize()
        if ex:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(n_steps, fresh):
        """n_steps steps between barrier + synchronize pairs; kernel times
        from the library's per-call event totals (fused) or per-step queries."""
        sync_all()
        per_step_query = args.unfused or args.cigar
        k2, k3, k1, kp = [], [], [], []
        before = eng.timings()
        t0 = time.perf_counter()
        for _ in range(n_steps):
            step(fresh)
            if per_step_query:
                tm = eng.timings()        # syncs the ctx stream; HIP events around K1 / K2 / K3
                k2.append(tm["depth_ms"])
                k3.append(tm["stats_ms"])
                k1.append(tm["cigar_ms"])
                kp.append(tm["prepare_ms"] if fresh else 0.0)
        sync_all()
        el = time.perf_counter() - t0
        after = eng.timings()
        if not per_step_query:
            calls = max(1, after["fused_calls"] - before["fused_calls"])
            k2 = [(after["fused_depth_ms_total"] - before["fused_depth_ms_total"]) / calls]
            k3 = [(after["fused_stats_ms_total"] - before["fused_stats_ms_total"]) / calls]
            kp = [(after["prepare_ms_total"] - before["prepare_ms_total"]) / max(1, n_steps)]
            k1 = [0.0]
        paths = {"direct": after["direct_batches"] - before["direct_batches"],
                 "full": after["full_prepares"] - before["full_prepares"],
                 "halo_redos": after["halo_redos"] - before["halo_redos"],
                 "halo": after["direct_halo"]}
        return el, [float(np.mean(x)) for x in (k2, k3, k1, kp)], paths

    # ---- the headline: every step is a fresh batch (prepare inside the step)
    for _ in range(args.warmup):
        step(True)
    elapsed, (k2_ms, k3_ms, k1_ms, kp_ms), paths = timed(args.steps, True)
    bases = eng.aligned_bases()
    if args.cigar:   # K1 re-derived exactly the generator's spans
        assert bases == int(span.to(torch.int64).sum()), "K1 spans differ from the generator"
    head_direct = paths["direct"] == args.steps
    # ---- the same batch with the index of one explicit prepare() reused by
    # every step (the reference's BAI analog), reported beside the headline
    elapsed_re, re_k = None, None
    if not args.cigar and args.prepare_steps > 0:
        eng.invalidate()
        eng.prepare()
        step(False)
        elapsed_re, re_k, _ = timed(args.prepare_steps, False)
    # the region-table exchange alone (RCCL all-gather over xGMI), timed apart
    allgather_ms = None
    if ex:
        n_ag = max(5, args.steps)
        sync_all()
        ta = time.perf_counter()
        for _ in range(n_ag):
            dist.all_gather_into_tensor(gouts[0], coll_bufs[0])
        torch.cuda.synchronize()
        allgather_ms = (time.perf_counter() - ta) / n_ag * 1e3
    t_max, t_max_re = elapsed, elapsed_re
    total_bases = bases
    if ex:
        t = torch.tensor([elapsed, elapsed_re or 0.0, allgather_ms], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t[0].item())
        t_max_re = float(t[1].item()) if elapsed_re is not None else None
        allgather_ms = float(t[2].item())
        b = torch.tensor([bases], dtype=torch.int64, device=coll_dev)
        dist.all_reduce(b)
        total_bases = int(b.item())
        # the last step's rows: slot s of every rank's G-step block
        mine = gathered.view(world, G, r_max, 9)[:, last[0][1]].reshape(world * r_max, 9)
        full = torch.cat([mine, gidx], dim=1)   # [world * r_max, 9 stats + region index]
        rows = mdist.unpack_rows(full.cpu().numpy(), n_regions_total, REGION_STAT_DTYPE)
        assert int(rows["sum"].sum()) == total_bases, "gathered region table lost bases"
    else:
        rows = table.cpu().numpy().view(REGION_STAT_DTYPE).reshape(-1)
        if not os.environ.get("MC_BENCH_NOCHECK"):   # set only for deliberately-wrong A/B builds
            assert int(rows["sum"].sum()) == total_bases
    if args.dump_rows and rank == 0:
        np.save(args.dump_rows, rows)

    # roofline of the dominant kernel of the headline step (K2): it reads the
    # raw (tid, pos, span) tuples on the direct path (12 B/read) or the packed
    # read words of a full prepare (4 B/read), and writes 4 B per position
    ext_sum = int(sum(eng.contig_offset(t)[1] for t in range(len(lengths))))
    read_bytes = 12 if head_direct else 4
    k2_bytes = read_bytes * len(tid) + 4 * ext_sum
    achieved = k2_bytes / (k2_ms * 1e-3) / 1e9
    long_path = args.config == "c5"
    variant = "depth_kernel<%s, %s, %s>" % ("false" if args.unfused else "true",
                                             "true" if long_path else "false",
                                             "true" if head_direct else "false")
    pmc = load_pmc_traffic(os.path.dirname(os.path.abspath(__file__)))

    def pmc_for(kernel_name):
        for v in ([] if world > 1 else (pmc or {}).get("variants", [])):   # PMC of the one-GPU workload
            if v.get("reads") == args.reads and v.get("contigs") == args.contigs \
                    and kernel_name in v.get("kernel", ""):
                return v.get("hbm_bytes_per_launch")
        return None
    roofline = {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
                "frac": achieved / 8000.0, "traffic": pmc_for(variant),
                "kernel": "%s (K2)" % variant, "algorithmic_bytes_per_launch": int(k2_bytes),
                "bytes_per_unit": "%d B/read + 4 B/position" % read_bytes}
    if args.cigar and k1_ms > k2_ms:   # K1 streams the CIGAR words: the dominant kernel
        n_words = int(cigar.numel())
        k1_bytes = 4 * n_words + 8 * (len(tid) + 1) + 4 * len(tid)
        achieved_k1 = k1_bytes / (k1_ms * 1e-3) / 1e9
        roofline = {"bound": "hbm", "achieved": achieved_k1, "peak": 8000.0, "unit": "GB/s",
                    "frac": achieved_k1 / 8000.0, "traffic": pmc_for("cigar_span_kernel"),
                    "kernel": "cigar_span_kernel (K1)", "algorithmic_bytes_per_launch": int(k1_bytes),
                    "bytes_per_unit": "4 B/CIGAR word + 12 B/read"}

    if rank == 0:
        cpu = cpu_par = cpu_int = None
        if world == 1 and not args.no_cpu_baseline:
            h = [x.cpu().numpy() for x in (tid, pos, span)]
            cpu = cpu_baseline(lengths, *h, args.cpu_sample_bases, args.config.upper())
            cpu_par = cpu_baseline_parallel(lengths, *h, cpu_thread_counts(args.cpu_threads),
                                            args.cpu_parallel_min_s)
            cpu_int = cpu_baseline_interval(lengths, *h, args.cpu_sample_bases)
            del h
        pcie = None
        if args.pcie and world == 1:
            h = [x.cpu().numpy() for x in (tid, pos, span)]
            e2 = CoverageEngine(local)
            e2.set_contigs(lengths)
            t1 = time.perf_counter()
            e2.add_reads(*h)
            e2.compute_depth_stats(rt, rs, re_)
            pcie = time.perf_counter() - t1
            e2.close()
        value = total_bases * args.steps / t_max
        line = {
            "metric": "aligned bases/sec into per-position depth vector, 1/2/4/8 MI355X",
            "value": value,
            "unit": "aligned bases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32",
            "data": ("synthetic (GPU-generated %s intervals, %s%s)"
                     % (args.config.upper(),
                        "lognormal ~10 kbp spans" if args.config == "c5" else "SURVEY §8d span mix",
                        ", BAM CIGAR words generated on the GPU" if args.cigar else "")),
            "config": {
                "workload": ("one %s workload LPT-sharded by contig over %d GPUs (the whole workload: %s)"
                             % (args.config.upper(), world,
                                (desc % args.reads if args.config == "c2" else
                                 desc % (args.contigs, lengths_all.sum() / 1e9, args.reads))
                                .replace("%s per GPU: " % args.config.upper(), "")))
                            if strong and world > 1 else
                            (desc % args.reads if args.config == "c2" else
                             desc % (args.contigs, lengths_all.sum() / 1e9, args.reads)),
                "config": args.config,
                "contigs_per_gpu": int(len(lengths)),
                "reads_per_gpu": int(len(tid)),
                "aligned_bases_per_step": int(total_bases),
                "regions": n_regions_total,
                "input": ("raw BAM CIGAR words in HBM (%d words, %.1f GB, ~%g ops/read); per step "
                          "K1 CIGAR->span + prepare + K2 + K3b" % (cigar.numel(), cigar.numel() * 4e-9,
                                                                    args.cigar_ops))
                         if args.cigar else
                         "(tid, pos, span) int32 tuples resident in HBM; every step treats them as a "
                         "fresh batch: prepare (%s) + K2 + K3b" % ("direct: probe + validating K2"
                                                                   if head_direct else "full: ingest"),
                "parallelism": ("contig-shard x%d, %s all-gather of region table"
                                % (world, "RCCL" if args.backend == "nccl" else "gloo"))
                               if world > 1 else "single GPU",
            },
            "prepare_path": {"direct_batches": paths["direct"], "full_prepares": paths["full"],
                             "halo_redos": paths["halo_redos"], "chunk_halo_positions": paths["halo"]},
            "kernels_ms": {**({"k1_cigar_span": k1_ms} if args.cigar else {}),
                           "prepare" + ("_probe" if head_direct else "_ingest_index"): kp_ms,
                           "k2_depth" + ("" if args.unfused else "_fused_stats"): k2_ms,
                           ("k3_region_stats" if args.unfused else "k3b_finalize"): k3_ms},
            "fused_fallback_regions": None if args.unfused else eng.fused_fallbacks(),
            "fused_device_recomputes": None if args.unfused else eng.fused_recomputes(),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "cpu_baseline_parallel": cpu_par,
            "cpu_interval_count": cpu_int,
            "world_size": world,
            "ranks_seen": dist.get_world_size() if ex else 1,
            "backend": (args.backend if ex else None),
            "allgather_ms": allgather_ms,   # one all-gather of a G-step group of region tables
            "exchange_every": (G if ex else None),
        }
        if t_max_re is not None:
            line["reused_index"] = {
                "value": total_bases * args.prepare_steps / t_max_re,
                "ms_per_step": t_max_re / args.prepare_steps * 1e3,
                "steps": args.prepare_steps,
                "k2_ms": re_k[0],
                "k3b_ms": re_k[1],
                "step": "one explicit mc_prepare (ingest: chunk index + packed 4 B read words), then "
                        "every step reuses it: K2 (depth_kernel<%s, %s, false>) + K3b"
                        % ("false" if args.unfused else "true", "true" if long_path else "false"),
            }
        if pcie is not None:
            line["host_buffer_end_to_end_s"] = pcie
        print(json.dumps(line), flush=True)
    eng.close()
    if ex:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

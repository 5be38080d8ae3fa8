#!/usr/bin/env python3
"""Benchmark of the BPE merge-training loop and encode pass on MI355X
(BASELINE.json metric "corpus MB/s per merge iter (train) + encode MB/s").

One STEP = one whole training job over the 1 GiB synthetic corpus (splitmix64
seed 2, random_text.txt-shaped, generated in HBM before timing): the one-off
pair counting sort, M merge iterations (count deltas -> argmax -> merge), the
final ids compacted in HBM.  `--steps K` jobs are timed back to back after
`--warmup W` untimed jobs; the merge count does not depend on K.

  N = 1  BASELINE configs[2]: 1 GiB x 8192 merges on one MI355X (the "HBM
         roofline run").  Extra key `train_1024`: the same corpus at 1024
         merges (configs[3] at N = 1, the north-star comparison point).
  N > 1  BASELINE configs[3]: the SAME 1 GiB corpus cut into N contiguous
         shards, one per rank (strong scaling), 1024 merges; per merge a sum
         of count deltas + a gather of edge records over xGMI (P2P mailboxes,
         or RCCL with --xport rccl).  Rank 0 first times the single-GPU job on
         its own device, so the line carries the measured speed-up 1 -> N and
         checks that merges and ids (checksum) equal the single-GPU run.
         Extra key `weak`: N GiB (1 GiB per rank), one job.

value = corpus_MB * merges * K / wall  (MB = 1e6 bytes; whole job, max over ranks)

The line also carries
  roofline        the dominant kernel of the merge loop, the batch scan
                  k_bscan (several merges per scan / apply pair):
                  algorithmic bytes per launch (8 B/candidate + 20 B/occurrence)
                  and its average span from the device wall clock, both over
                  the LAST timed job; the committed rocprofv3 summary and PMC
                  traffic of this same command (profiles/<PROFILE_TAG>_*) beside them;
  roofline_apply  the batch apply k_bapply (table updates, 16 B each), same way;
  roofline_count_pass  the corpus-wide pair-count pass (1 B/token read; the
                  initial u32 ids are written by the counting sort's first
                  pass, k_sort_a, which streams the bytes anyway);
  correctness     merges md5 + position-keyed ids checksum (bpe_gpu_ids_checksum)
                  of the warm-up and the timed jobs: they must agree, else the
                  line carries "error" and the process exits non-zero;
  cpu_baseline    the unmodified reference (oracle/_ref/bpe_ref, 16 pthreads as
                  it hard-codes) on a bounded sample, rank 0 at N = 1 only;
  encode          BASELINE configs[4]: a 10 GiB seed-3 stream through the first
                  32768 merges the trainer learns; ids checksum of the warm and
                  timed runs must agree and n_out + occurrences == bytes.
"""
import argparse
import csv
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)
GIB = 1 << 30
PROFILE_TAG = "r6"     # profiles/<tag>_train_kernel_stats.csv, <tag>_pmc_traffic.json (tools/gpu_profile.sh)


def count_pass_kernel(form):
    """the count pass's kernel from bpe_gpu_stats.count_pass_span"""
    if not form:
        return "k_pair_hist"
    return {2: "k_pair_hist_v", 3: "k_pair_hist_v<skew>", 1: "k_pair_hist_pk", 0: "k_pair_hist_span"}[form // 100]


def cpu_baseline(seed, size, merges):
    """Reference trainer on a bounded sample (first `size` bytes of the same
    corpus).  Falls back to the oracle port (1 thread) if _ref is absent."""
    from llmtokenizer_amd.synth import synth_bytes
    data = synth_bytes(seed, size)
    ref = os.path.join(ROOT, "oracle", "_ref", "bpe_ref")
    with tempfile.TemporaryDirectory() as td:
        inp = os.path.join(td, "c.txt")
        with open(inp, "wb") as f:
            f.write(data)
        if os.path.exists(ref):
            env = dict(os.environ, BPE_REF_MAX_MERGES=str(merges))
            t0 = time.time()
            p = subprocess.run([ref, inp, os.path.join(td, "m"), os.path.join(td, "i")], env=env,
                               capture_output=True, text=True)
            dt = time.time() - t0
            if p.returncode != 0:
                return None
            kind, cores = "reference", 16
        else:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import oracle_lib as O
            t0 = time.time()
            O.train(data, merges, O.FAST)
            dt = time.time() - t0
            kind, cores = "port", 1
    return {"value": round(size / 1e6 * merges / dt, 3), "unit": "corpus MB/s per merge iter",
            "cores": cores, "kind": kind, "s_per_merge": round(dt / merges, 4),
            "sample": f"{size / 2**20:.0f} MiB prefix of the seed-{seed} corpus, {merges} merges, "
                      f"{dt:.1f} s wall incl. load (reference hard-codes 16 pthreads; host nproc={os.cpu_count()})"}


def cpu_encode_baseline(merges, seed, size):
    """CPU encoder with the reference's result (oracle/bpe_oracle.c
    oracle_encode_heap: the replace passes of bpe.c:760-779 replayed smallest
    rank first over a token list, O(n log n), one thread; tests/test_oracle.py
    checks it against the pass-by-pass restatement) on a bounded sample.  The
    pass-by-pass form itself (O(n x merges)) is timed on a 256 KiB slice."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from llmtokenizer_amd.synth import synth_bytes
    data = synth_bytes(seed, size)
    t0 = time.time()
    O.encode_heap(data, merges)
    dt = time.time() - t0
    small = data[: 256 << 10]
    t1 = time.time()
    O.encode(small, merges)
    dt2 = time.time() - t1
    return {"value": round(size / 1e6 / dt, 4), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"{size >> 20} MiB prefix of the seed-{seed} stream through all {len(merges)} merges, "
                      f"smallest-rank-first replay (identical ids), {dt:.1f} s wall",
            "sequential_passes": {"value": round(len(small) / 1e6 / dt2, 4), "unit": "MB/s",
                                  "sample": f"256 KiB prefix, one replace pass per merge as the reference, "
                                            f"{dt2:.1f} s wall"}}


class Ctx:
    """rank / world / torch.distributed plumbing (gloo carries only set-up data,
    barriers and the max over ranks; the per-merge exchange is in libbpe_amd)"""

    def __init__(self, sharded):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # rehearsal of the N-rank flow on a one-GPU box: every rank on this device
        if os.environ.get("BPE_BENCH_DEVICE") is not None:
            self.local = int(os.environ["BPE_BENCH_DEVICE"])
        self.dist = None
        if sharded:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            torch.cuda.set_device(self.local)
            # gloo prints its mesh set-up ("[Gloo] Rank r is connected to ...")
            # on stdout, where the driver reads the one JSON line: send fd 1 to
            # stderr while the group connects, then flush C stdio before restoring
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
                dist.barrier()
            finally:
                try:
                    import ctypes
                    ctypes.CDLL(None).fflush(None)
                except OSError:
                    pass
                os.dup2(saved, 1)
                os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            import torch
            torch.cuda.synchronize()
            self.dist.barrier()

    def allreduce(self, x, op="sum", dtype="float64"):
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=getattr(torch, dtype))
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return t.item()

    def allgather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out


def group_checksum(cx, g):
    """ids checksum of the whole corpus over the ranks' shard groups"""
    s, n = g.ids_checksum(0)
    counts = cx.allgather(n)
    base = sum(counts[:cx.rank])
    s, n = g.ids_checksum(base)
    sums = cx.allgather(s)
    return sum(sums) % (1 << 64), sum(counts)


def timed_jobs(cx, run, k):
    """k back-to-back jobs between barriers + device syncs; max over ranks"""
    cx.barrier()
    t0 = time.perf_counter()
    for _ in range(k):
        run()
    t1 = time.perf_counter()
    cx.barrier()
    return cx.allreduce(t1 - t0, "max")


GATHER_CEILING = os.path.join(ROOT, "profiles", "r5_gather_ceiling.jsonl")  # tools/gather_bench on the MI355X


def gather_ceiling(mode, waves=None):
    """the measured random-access ceiling (tools/gather_bench.hip, committed
    summary): best gathers/s of `mode` over in-flight depth U (and over the
    waves per CU unless `waves` is given), with the configuration it took"""
    if not os.path.exists(GATHER_CEILING):
        return None
    best = None
    with open(GATHER_CEILING) as f:
        for line in f:
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if r.get("mode") != mode or (waves is not None and r.get("waves_per_cu") != waves):
                continue
            if best is None or r["gathers_per_s"] > best["gathers_per_s"]:
                best = r
    return best


def line_rate(achieved, mode, waves, note):
    """roofline.line_rate: random accesses per second of a loop kernel against
    the part's measured ceiling for that access shape"""
    at = gather_ceiling(mode, waves)
    top = gather_ceiling(mode)
    if not at or not top:
        return None
    return {"unit": "random accesses/s", "achieved": float("%.4g" % achieved), "shape": mode,
            "ceiling_at_kernel_occupancy": float("%.4g" % at["gathers_per_s"]),
            "ceiling_config": {"waves_per_cu": at["waves_per_cu"], "in_flight_per_thread": at["U"]},
            "frac": round(achieved / at["gathers_per_s"], 4),
            "ceiling_best": float("%.4g" % top["gathers_per_s"]),
            "ceiling_best_config": {"waves_per_cu": top["waves_per_cu"], "in_flight_per_thread": top["U"]},
            "frac_of_best": round(achieved / top["gathers_per_s"], 4),
            "source": os.path.relpath(GATHER_CEILING, ROOT), "note": note}


def committed_profile(name, sharded=False):
    """rocprof average (ms) of kernel `name` and PMC traffic per launch from
    the committed summaries of this same command (profiles/<tag>_*): the
    single-GPU bench command, or (sharded) the sharded one with one rank"""
    out = {}
    for kind in (("sharded",) if sharded else ("train",)):
        p = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_{kind}_kernel_stats.csv")
        if "avg_ms_rocprof" in out or not os.path.exists(p):
            continue
        with open(p) as f:
            for r in csv.DictReader(f):
                nm = r["Name"].split("(")[0].replace("bpeamd::", "").replace("void ", "").strip()
                if nm.split("<")[0] == name:
                    out["avg_ms_rocprof"] = round(float(r["AverageNs"]) / 1e6, 5)
                    out["rocprof_calls"] = int(r["Calls"])
                    out["rocprof_summary"] = os.path.relpath(p, ROOT)
                    break
    # the same profile's average over the launches >= 6 us only (direct
    # launches queued past a stop exit at once: tools/prof_nonempty.py)
    p = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_{'sharded' if sharded else 'train'}_kernel_nonempty.txt")
    if os.path.exists(p):
        with open(p) as f:
            for line in f.readlines()[1:]:
                parts = line.split()
                if parts and parts[0].split("<")[0] == name:
                    out["avg_ms_rocprof_nonempty"] = round(float(parts[5]) / 1e3, 5)
                    out["rocprof_nonempty_launches"] = int(parts[4])
                    break
    p = os.path.join(ROOT, "profiles", f"{PROFILE_TAG}_pmc_traffic.json")
    if os.path.exists(p):
        with open(p) as f:
            tr = json.load(f)
        # (kernels both commands run carry "@sharded" for the sharded one)
        key = name + "@sharded" if sharded and name + "@sharded" in tr else name
        if key in tr:
            out["traffic"] = tr[key]["traffic_bytes_per_launch"]
            out["traffic_source"] = (os.path.relpath(p, ROOT) + ": FETCH_SIZE x %.1f + WRITE_SIZE, separate "
                                     "--pmc passes of this command" % tr[key]["fetch_correction"])
    return out


def train_single(args, cx, out):
    """N = 1: configs[2] (1 GiB x 8192 merges) + the 1024-merge figure"""
    from llmtokenizer_amd import api
    e = api.Engine(cx.local)
    e.synth(args.seed, args.size)
    merges = args.merges or 8192
    for _ in range(args.warmup):
        e.train(merges)
    ref = None
    if args.warmup:
        ref = (hashlib.md5(e.merges().tobytes()).hexdigest(), e.ids_checksum())
    done = []
    el = timed_jobs(cx, lambda: done.append(e.train(merges)), args.steps)
    got = (hashlib.md5(e.merges().tobytes()).hexdigest(), e.ids_checksum())
    st = e.stats()
    prof = e.kernel_profile()  # the last timed job: bytes per launch and span from one window
    if any(k != merges for k in done):
        out["error"] = f"a job stopped early: {sorted(set(done))} merges"
    if ref is not None and ref != got:
        out["error"] = f"warm-up and timed jobs differ: {ref} vs {got}"
    extra = {}
    if not args.no_extras:
        e.train(1024)  # warm
        t = timed_jobs(cx, lambda: e.train(1024), 1)
        s2 = e.stats()
        extra = {"train_1024": {"value": round(args.size / 1e6 * 1024 / t, 1), "ms": round(t * 1e3, 3),
                                "workload": "configs[3] at N=1: 1 GiB x 1024 merges, one job",
                                "breakdown_ms": {"init": round(s2["ms_init"], 3), "loop": round(s2["ms_train"], 3)},
                                "batches": s2["batches"], "batch_retries": s2["batch_retries"],
                                "ids_checksum": "%016x" % e.ids_checksum(),
                                "merges_md5": hashlib.md5(e.merges().tobytes()).hexdigest()}}
        extra["ingest"] = ingest_rate(e)
        # configs[1]: a 1 MiB random_text.txt-shaped corpus (seed 1), 1024 merges,
        # the reference's static 16-thread tie emulation (tracked iterations)
        c1 = api.Engine(cx.local)
        c1.synth(1, 1 << 20)
        c1.train(1024)
        t = timed_jobs(cx, lambda: c1.train(1024), 1)
        extra["config1"] = {"value": round((1 << 20) / 1e6 * 1024 / t, 1), "ms": round(t * 1e3, 3),
                            "workload": "configs[1]: 1 MiB seed-1 random_text.txt-shaped corpus, 1024 merges, "
                                        "one job (tie order: the reference's static-schedule emulation)",
                            "merges_md5": hashlib.md5(c1.merges().tobytes()).hexdigest()}
        gold = os.path.join(ROOT, "tests", "golden", "synth_s1_1m.json")  # the reference's own merges
        if os.path.exists(gold):
            import numpy as np
            with open(gold) as f:
                gm = np.asarray(json.load(f)["merges"], dtype=np.uint32).reshape(-1, 2)
            extra["config1"]["equals_reference_golden"] = bool(hashlib.md5(gm.tobytes()).hexdigest() ==
                                                               extra["config1"]["merges_md5"])
        c1.close()
        if not args.no_cpu_baseline:
            # the reference on configs[1] itself (64 of the 1024 merges) and
            # on the 1 GiB corpus (4 merges: its per-iteration cost), same host
            extra["config1"]["cpu_baseline"] = cpu_baseline(1, 1 << 20, 64)
            extra["cpu_baseline_1g"] = cpu_baseline(args.seed, GIB, 4)
    e.close()
    return el, merges, st, prof, got, extra


def ingest_rate(e, size=GIB, merges=1024):
    """get_file + strlen into HBM (bpe_gpu_load_fd: pinned double-buffered
    staging, several reader threads, byte presence gathered per chunk) for a
    1 GiB file in the page cache: the PCIe-inclusive rate (never `value`: the
    timed jobs start from resident input).  Then the whole compress() path on
    the same file (bpe.h compress_ex: ingest, training, merges and ids back to
    the host; its engine context kept from a first call) against the ingest
    plus the same training and fetch from resident bytes."""
    import numpy as np
    from llmtokenizer_amd import api
    path = os.path.join(tempfile.gettempdir(), "bpe_bench_ingest.bin")
    try:
        # 1 GiB of uniform printable bytes (random_text.txt-shaped)
        np.random.default_rng(0).integers(32, 127, size, dtype=np.uint8).tofile(path)
        e.load_file(path)  # warm (staging buffers)
        t0 = time.perf_counter()
        n = e.load_file(path)
        t1 = time.perf_counter()
        e.train(merges)
        e.merges(), e.ids()
        t2 = time.perf_counter()
        e.train(merges)
        e.merges(), e.ids()
        t3 = time.perf_counter()
        keep = os.environ.get("BPE_KEEP_CONTEXT")
        os.environ["BPE_KEEP_CONTEXT"] = "1"  # the kept context keeps its HBM pool (bpe_ex.h)
        try:
            api.compress(path, merges)  # (creates the kept context)
            t4 = time.perf_counter()
            api.compress(path, merges)
            t5 = time.perf_counter()
        finally:
            if keep is None:
                os.environ.pop("BPE_KEEP_CONTEXT", None)
            else:
                os.environ["BPE_KEEP_CONTEXT"] = keep
            api.release_engines()
    finally:
        if os.path.exists(path):
            os.remove(path)
    ing, res, comp = t1 - t0, t3 - t2, t5 - t4
    return {"bytes": n, "ms": round(ing * 1e3, 2), "GB/s": round(n / ing / 1e9, 2),
            "note": "file in the page cache -> HBM incl. the NUL scan, PCIe-inclusive; not part of value",
            "compress": {"merges": merges, "ms": round(comp * 1e3, 2),
                         "resident_train_fetch_ms": round(res * 1e3, 2),
                         "ratio_to_ingest_plus_resident": round(comp / (ing + res), 3),
                         "note": "compress_ex(path) = ingest + training + merges and ids to the host, vs the "
                                 "ingest plus the same training and fetch from resident bytes"}}


def train_sharded(args, cx, out):
    """N > 1 (or --sharded): configs[3], one 1 GiB corpus over N ranks"""
    from llmtokenizer_amd import api
    from llmtokenizer_amd import dist as bdist
    merges = args.merges or 1024
    single = None
    if not args.no_extras and cx.world > 1:
        # the 1-GPU reference point, on rank 0's device, same corpus and merges
        if cx.rank == 0:
            e = api.Engine(cx.local)
            e.synth(args.seed, args.size)
            e.train(merges)
            t0 = time.perf_counter()
            e.train(merges)
            t1 = time.perf_counter()
            single = (t1 - t0, hashlib.md5(e.merges().tobytes()).hexdigest(), e.ids_checksum())
            e.close()
        cx.barrier()
    g = bdist.group(cx.local, merges, args.xport)
    lo, hi = bdist.shard_range(args.size, cx.rank, cx.world)
    g.synth(0, args.seed, hi - lo, lo)
    warm = args.warmup
    if cx.world > 1:  # (untimed) a P2P job that fails on any rank moves every rank to RCCL
        g, ok = bdist.first_job(g, cx.local,
                                lambda gg: (gg.train(merges), hashlib.md5(gg.merges().tobytes()).hexdigest()))
        if not ok:
            g.synth(0, args.seed, hi - lo, lo)
            g.train(merges)
        warm -= 1
    for _ in range(max(0, warm)):
        g.train(merges)
    done = []
    el = timed_jobs(cx, lambda: done.append(g.train(merges)), args.steps)
    st = g.stats()
    md5 = hashlib.md5(g.merges().tobytes()).hexdigest()
    digests = cx.allgather(md5)
    csum, n_ids = group_checksum(cx, g)
    prof = g.kernel_profile(0)
    transport = g.transport()
    if any(k != merges for k in done):
        out["error"] = f"a job stopped early: {sorted(set(done))} merges"
    if len(set(digests)) != 1:
        out["error"] = "merges differ across ranks"
    extra = {"merges_identical_across_ranks": len(set(digests)) == 1, "transport": transport,
             "engine_form": ("batches (one delta sum + one record gather per batch)" if st["batches"] else
                             "one merge per exchange")}
    if getattr(g, "fallback_reason", None):
        extra["transport_fallback_reason"] = g.fallback_reason
    if single is not None:
        t1 = single[0]
        extra["single_gpu_1024"] = {"ms": round(t1 * 1e3, 3), "value": round(args.size / 1e6 * merges / t1, 1)}
        extra["speedup_vs_1gpu"] = round(t1 / (el / args.steps), 3)
        same = single[1] == md5 and single[2] == csum
        extra["identical_to_1gpu"] = same
        if not same:
            out["error"] = "sharded merges/ids differ from the single-GPU run"
    if not args.no_extras and cx.world > 1:
        # weak scaling: 1 GiB per rank, one job
        g.synth(0, args.seed, args.size, cx.rank * args.size)
        g.train(merges)
        t = timed_jobs(cx, lambda: g.train(merges), 1)
        extra["weak"] = {"value": round(cx.world * args.size / 1e6 * merges / t, 1), "ms": round(t * 1e3, 3),
                         "workload": f"{cx.world} GiB ({cx.world} x 1 GiB shards), {merges} merges, one job"}
    g.close()
    return el, merges, st, prof, (md5, csum), extra


def encode_bench(args, cx):
    """BASELINE configs[4]: encode a 10 GiB seed-3 stream with the first 32768
    merges the GPU trainer learns on the 1 GiB seed-2 corpus.  Input resident
    in HBM; timed = the whole encode (pair sort + batched merge replay + ids)."""
    from llmtokenizer_amd import api
    tr = api.Engine(cx.local)  # same deterministic merges on every rank
    tr.synth(args.seed, args.size)
    tr.train(args.encode_merges)
    merges = tr.merges()
    tr.close()
    merges_md5 = hashlib.md5(merges.tobytes()).hexdigest()  # (the same on every rank and every N)
    per = 3 << 30  # bytes per shard context (u32 positions)
    total = args.encode_size
    world = cx.world
    if world > 1:
        total = min(total, world * per)  # a rank's share must fit u32 positions
    if world > 1:
        from llmtokenizer_amd import dist as bdist
        lo, hi = bdist.shard_range(total, cx.rank, world)
        g = bdist.group(cx.local, len(merges), args.xport)
        g.synth(0, 3, hi - lo, lo)
    else:
        k = max(1, -(-total // per))
        g = api.ShardGroup(cx.local, local_shards=k)
        step = total // k
        for q in range(k):
            a = q * step
            b = total if q == k - 1 else a + step
            g.synth(q, 3, b - a, a)
    if world > 1:  # warm (pools, graphs); a P2P failure on any rank moves every rank to RCCL
        g, ok = bdist.first_job(g, cx.local, lambda gg: gg.encode(merges))
        if not ok:
            g.synth(0, 3, hi - lo, lo)
            g.encode(merges)
    else:
        g.encode(merges)  # warm (pools, graphs)
    warm = group_checksum(cx, g)
    el = timed_jobs(cx, lambda: g.encode(merges), 1)
    st = g.stats()
    got = group_checksum(cx, g)
    n_out = int(cx.allreduce(st["n_out"], dtype="int64"))
    occ = int(cx.allreduce(st["occurrences"], dtype="int64"))
    w = 2 if 256 + len(merges) <= 65536 else 4
    alg = total + n_out * w  # input bytes + n_out * w
    out = {"metric": "encode MB/s, %g GiB stream through 32k merges" % (total / GIB), "value": round(total / 1e6 / el, 1),
           "unit": "MB/s", "ms": round(el * 1e3, 2), "n_gpus": world, "bytes": total, "merges": len(merges),
           "n_out": n_out, "merges_md5": merges_md5, "ids_checksum": "%016x" % got[0],
           "warm_ids_checksum": "%016x" % warm[0], "shards": g.nshards, "batches": st["iterations"],
           "candidates": int(cx.allreduce(st["candidates"], dtype="int64")), "occurrences": occ,
           "breakdown_ms": {"init": round(st["ms_init"], 2), "replay": round(st["ms_train"], 2)},
           "roofline": {"bound": "hbm", "achieved": round(alg / el / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / el / 1e9 / HBM_PEAK_GBS, 5),
                        "bytes": alg, "note": "whole-job algorithmic bytes (input + n_out*w) / wall"}}
    if getattr(g, "fallback_reason", None):
        out["transport_fallback_reason"] = g.fallback_reason
    errs = []
    if warm != got:
        errs.append("warm and timed encodes differ")
    if n_out + occ != total or got[1] != n_out:
        errs.append(f"n_out {n_out} + occurrences {occ} != bytes {total}")
    if errs:
        out["error"] = "; ".join(errs)
    g.close()
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_encode_baseline(merges, 3, args.cpu_encode_size)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="training jobs timed")
    ap.add_argument("--warmup", type=int, default=1, help="untimed training jobs first")
    ap.add_argument("--merges", type=int, default=None,
                    help="merges per job (default: 8192 at N=1 = configs[2]; 1024 sharded = configs[3])")
    ap.add_argument("--size", type=int, default=GIB, help="corpus bytes (the whole job, all ranks)")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--xport", choices=("p2p", "rccl"), default=None, help="per-merge exchange (N > 1)")
    ap.add_argument("--sharded", action="store_true", help="the sharded path even with one rank")
    ap.add_argument("--no-extras", action="store_true", help="skip the 1024-merge / speed-up / weak legs")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=64 << 20)
    ap.add_argument("--cpu-merges", type=int, default=16)
    ap.add_argument("--no-encode", action="store_true", help="skip the configs[4] encode measurement")
    ap.add_argument("--encode-size", type=int, default=10 << 30)
    ap.add_argument("--encode-merges", type=int, default=32768)
    ap.add_argument("--cpu-encode-size", type=int, default=64 << 20)
    args = ap.parse_args()

    sharded = int(os.environ.get("WORLD_SIZE", "1")) > 1 or args.sharded
    cx = Ctx(sharded)
    out = {}
    if sharded:
        el, merges, st, prof, dig, extra = train_sharded(args, cx, out)
    else:
        el, merges, st, prof, dig, extra = train_single(args, cx, out)
    enc = None if args.no_encode else encode_bench(args, cx)

    if cx.rank != 0:
        return
    k = args.steps
    corpus_mb = args.size / 1e6
    value = corpus_mb * merges * k / el
    name, kms, kbytes, launches = prof
    achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    # count pass: reads the corpus once, 1 B/token (V = 256); the initial ids
    # are written by k_sort_a
    cp_ms = st["ms_count_pass"]
    cp_bytes = args.size
    cp_achieved = cp_bytes / (cp_ms * 1e-3) / 1e9 if cp_ms > 0 else 0.0
    world = cx.world
    if sharded:
        workload = (f"configs[3]: one 1 GiB corpus in {world} contiguous shards (one per rank), "
                    f"{merges} merges per job, {k} jobs timed")
    else:
        workload = f"configs[2]: 1 GiB corpus, {merges} merges per job on one MI355X, {k} jobs timed"
    out.update({
        "metric": "corpus MB/s per merge iter (train), 1 GiB synthetic corpus",
        "value": round(value, 1),
        "unit": "corpus MB/s per merge iter",
        "n_gpus": world,
        "steps": k,
        "warmup": args.warmup,
        "ms_per_step": round(el * 1e3 / max(k, 1), 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (random_text.txt-shaped, splitmix64 seed %d, generated in HBM)" % args.seed,
        "config": {"workload": workload, "corpus_bytes": args.size, "merges_per_job": merges,
                   "step": "one whole training job (count pass + merges + ids compaction)",
                   "parallelism": (f"dp{world}: one training job over {world} contiguous corpus shards, per merge a "
                                   "sum of count deltas + a gather of edge records") if sharded else "single GPU"},
        "correctness": {"merges_md5": dig[0], "ids_checksum": "%016x" % dig[1],
                        "checked": "warm-up job == timed jobs" if not sharded else "ranks agree"},
        "roofline": {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_per_launch": round(kbytes), "avg_ms": round(kms, 5), "launches": launches,
                     "window": "the last timed job (bytes and span from the same launches)",
                     "avg_ms_source": "device wall clock (first block entry to the last block's retired "
                                      "memory operations) inside the timed run",
                     "note": ("batch scan: one random token-window gather per candidate (8 B algorithmic, a "
                              "128-B line moved), bound by the random-line rate" if name == "k_bscan" else
                              "per-merge kernel: dependent random gathers, latency-bound")},
        "roofline_count_pass": {"kernel": count_pass_kernel(st["count_pass_span"]),
                                "bound": "hbm", "achieved": round(cp_achieved, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(cp_achieved / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": cp_bytes, "avg_ms": round(cp_ms, 4),
                                "form": int(st["count_pass_span"]),
                                "note": "histogram of byte-pair rank keys: 1 B/token read, bins in LDS "
                                        "(SURVEY 8(d)); the initial ids are written by k_sort_a; the corpus is "
                                        "read cold (byte presence is gathered at load since round 4; before, "
                                        "that pass left ~1/4 of the corpus in the 256 MB MALL: 0.24-0.25 ms); "
                                        "LDS-conflict bound (DESIGN 4)"},
        "breakdown_ms": {"init": round(st["ms_init"], 3), "loop": round(st["ms_train"], 3),
                         "total_engine": round(st["ms_total"], 3), "per_merge_us": round(st["ms_train"] * 1e3 / merges, 2)},
        "engine": {k2: st[k2] for k2 in ("n_out", "iterations", "distinct_pairs", "merged_buckets",
                                          "rule_ties", "table_grows", "keys", "candidates", "occurrences",
                                          "hot_rebuilds", "hot_mode", "hot_scanned", "relists", "batches",
                                          "batch_dropped", "batch_retries", "table_updates", "spec_hits",
                                          "spec_misses", "select_launches", "keys_skipped", "skip_failed",
                                          "tie_verified", "tie_failed")},
        "batch_end": {k2[4:]: st[k2] for k2 in st if k2.startswith("end_")},
    })
    out.update(extra)
    cp = committed_profile(name, sharded)
    out["roofline"].update({k2: v for k2, v in cp.items() if k2 != "traffic"})
    if "traffic" in cp:
        out["roofline"]["traffic"] = cp["traffic"]
    if "avg_ms_rocprof" in cp:
        out["roofline"]["frac_at_rocprof_avg"] = round(kbytes / (cp["avg_ms_rocprof"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    # the scan's real limit: one random 32-byte token window per candidate
    # (tok_window), 16 waves per CU (one 1024-thread block), against what the
    # part delivers for that access shape
    if launches and kms > 0 and st.get("candidates"):
        lr = line_rate(st["candidates"] / launches / (kms * 1e-3), "window32", 16,
                       "candidates per launch / k_bscan's span: each gathers one random 32-B window of a 4 GiB tok[]")
        if lr:
            out["roofline"]["line_rate"] = lr
    # the batch apply (the pair-table updates): 16 B per update (the key probed,
    # the count read and written), span from the device wall clock like the scan
    nl = st["batches"] + st["batch_retries"]
    if nl and st["ms_apply_span"] > 0:
        ab = 16.0 * st["table_updates"] / nl
        aa = ab / (st["ms_apply_span"] * 1e-3) / 1e9
        ap = committed_profile("k_bapply", sharded)
        out["roofline_apply"] = {"kernel": "k_bapply", "bound": "hbm", "achieved": round(aa, 1), "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": round(aa / HBM_PEAK_GBS, 4), "traffic": ap.get("traffic"),
                                 "bytes_per_launch": round(ab), "avg_ms": round(st["ms_apply_span"], 5), "launches": nl,
                                 "avg_ms_rocprof": ap.get("avg_ms_rocprof"), "rocprof_summary": ap.get("rocprof_summary"),
                                 "note": "16 B per pair-table update (random key probe + count); random-line bound"}
        lr = line_rate(st["table_updates"] / nl / (st["ms_apply_span"] * 1e-3), "atomic_ret", 16,
                       "table updates / k_bapply's span: each a random key probe, then a returning u32 atomic")
        if lr:
            out["roofline_apply"]["line_rate"] = lr
    # the batch select k_bsel: the hot set reduced (16 B per listed key: slot,
    # count, key) beside the previous batch's token rewrite (12 B per
    # occurrence: the id, the end code, the pool entry)
    if st["select_launches"] and st["ms_select_span"] > 0:
        sb = (16.0 * st["hot_scanned"] + 12.0 * st["occurrences"]) / st["select_launches"]
        sa = sb / (st["ms_select_span"] * 1e-3) / 1e9
        sp = committed_profile("k_bsel", sharded)
        out["roofline_select"] = {"kernel": "k_bsel", "bound": "hbm", "achieved": round(sa, 1), "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "frac": round(sa / HBM_PEAK_GBS, 4), "traffic": sp.get("traffic"),
                                  "bytes_per_launch": round(sb), "avg_ms": round(st["ms_select_span"], 5),
                                  "launches": st["select_launches"], "avg_ms_rocprof": sp.get("avg_ms_rocprof"),
                                  "rocprof_summary": sp.get("rocprof_summary"),
                                  "note": "hot-set reduce (16 B/key) + the previous batch's rewrite (12 B per "
                                          "occurrence, one dirtied sector each); device wall clock per launch"}
        # its own random-access rate: the rewrite's paired token stores (the
        # new id at the occurrence, the end code at its end slot) per span
        lr = line_rate(st["occurrences"] / st["select_launches"] / (st["ms_select_span"] * 1e-3), "store_pair", 16,
                       "occurrences rewritten per k_bsel launch / its span (the select's own latency chain "
                       "runs beside the rewrite blocks in the same span)")
        if lr:
            out["roofline_select"]["line_rate"] = lr
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.seed, args.cpu_size, args.cpu_merges)
    if enc is not None:
        out["encode"] = enc
        if "error" in enc:
            out["error"] = (out.get("error", "") + "; encode: " + enc["error"]).lstrip("; ")
    print(json.dumps(out), flush=True)
    if "error" in out:
        print("bench: ERROR " + out["error"], file=sys.stderr, flush=True)
        sys.exit(1)


if __name__ == "__main__":
    main()

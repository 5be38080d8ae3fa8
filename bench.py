#!/usr/bin/env python3
"""Benchmark of the BPE merge-training loop on MI355X (BASELINE.json metric
"corpus MB/s per merge iter").

Workload (BASELINE.json configs[3], one GPU per rank): a 1 GiB synthetic
random_text.txt-shaped corpus (seed 2, generated directly in HBM), trained
for K merge iterations.  One "step" = one merge iteration over the corpus.
The timed region is the WHOLE training job on resident input: the one-off
pair counting sort + K iterations (count deltas -> argmax -> merge), ending
with the final ids compacted in HBM.

value = n_gpus * corpus_MB * K / wall   (MB = 1e6 bytes)

Multi-GPU (torchrun, one rank per GPU): ONE training job over an N GiB
corpus cut into N contiguous 1 GiB shards (weak scaling).  Every merge sums
the shards' count deltas and gathers their 16-word edge records: by default
one push kernel per exchange over xGMI into the peers' IPC-mapped mailboxes
(BPE_XPORT=rccl: RCCL collectives on libbpe_amd.so's own communicator);
torch.distributed/gloo only carries the set-up handles, the barrier and the
max over ranks.  The merges are
checked identical on every rank.  value = N * 1073.7 MB * K / wall.

The JSON line also carries
  roofline     -- the dominant kernel of the loop (k_scan), its average span
                  from the device wall clock inside the timed run, corroborated
                  by HIP event nodes in a second run; algorithmic bytes =
                  8 B/candidate + 20 B/occurrence;
  roofline_count_pass -- the one corpus-wide streaming pass (k_pair_hist),
                  timed with HIP events on the engine's stream;
  cpu_baseline -- the unmodified reference (oracle/_ref/bpe_ref, 16 threads)
                  timed on this host on a bounded sample (rank 0, N=1 only).
"""
import argparse
import csv
import glob
import json
import re
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md)


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
            "cores": cores, "kind": kind,
            "sample": f"{size / 2**20:.0f} MiB prefix of the seed-{seed} corpus, {merges} merges, "
                      f"{dt:.1f} s wall (reference hard-codes 16 pthreads; host nproc={os.cpu_count()})"}


def cpu_encode_baseline(merges, seed, size):
    """Reference-structure encoder (the replace pass applied rank by rank,
    oracle/bpe_oracle.c oracle_encode, one thread) on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    from llmtokenizer_amd.synth import synth_bytes
    data = synth_bytes(seed, size)
    t0 = time.time()
    O.encode(data, merges)
    dt = time.time() - t0
    return {"value": round(size / 1e6 / dt, 4), "unit": "MB/s", "cores": 1, "kind": "port",
            "sample": f"{size >> 10} KiB prefix of the seed-{seed} stream, all {len(merges)} merges as "
                      f"sequential replace passes, {dt:.1f} s wall"}


def encode_bench(args, rank, world, local, dist, barrier):
    """BASELINE configs[4]: encode a 10 GiB seed-3 stream with the first 32768
    merges the GPU trainer learns on the 1 GiB seed-2 corpus.  Input resident
    in HBM; timed = the whole encode (pair sort + batched merge replay + ids)."""
    from llmtokenizer_amd import api
    tr = api.Engine(local)  # same deterministic merges on every rank
    tr.synth(args.seed, args.size)
    tr.train(args.encode_merges)
    merges = tr.merges()
    tr.close()
    import hashlib
    merges_md5 = hashlib.md5(merges.tobytes()).hexdigest()  # (the same on every rank and every N)
    per = 3 << 30  # bytes per shard context (u32 positions)
    total = args.encode_size
    if world > 1:
        # one shard per rank across ranks: a rank's share must fit u32
        # positions (10 GiB over 2 ranks does not; 4 and 8 ranks keep 10 GiB)
        total = min(total, world * per)
    lo, hi = rank * (total // world), (total if rank == world - 1 else (rank + 1) * (total // world))
    if world > 1:
        from llmtokenizer_amd import dist as bdist
        g = bdist.group(local, len(merges))
        g.synth(0, 3, hi - lo, lo)
    else:
        k = max(1, -(-total // per))
        g = api.ShardGroup(local, local_shards=k)
        step = total // k
        for q in range(k):
            a = q * step
            b = total if q == k - 1 else a + step
            g.synth(q, 3, b - a, a)
    g.encode(merges)  # warm (pools, graphs)
    barrier()
    t0 = time.perf_counter()
    g.encode(merges)
    t1 = time.perf_counter()
    barrier()
    el = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    st = g.stats()
    n_out = st["n_out"]
    if dist is not None:
        import torch
        t = torch.tensor([n_out], dtype=torch.int64)
        dist.all_reduce(t)
        n_out = int(t.item())
    w = 2 if 256 + len(merges) <= 65536 else 4
    alg = total + n_out * w  # input bytes + n_out * w
    out = {"metric": "encode MB/s, %g GiB stream through 32k merges" % (total / (1 << 30)), "value": round(total / 1e6 / el, 1),
           "unit": "MB/s", "ms": round(el * 1e3, 2), "n_gpus": world, "bytes": total, "merges": len(merges),
           "n_out": n_out, "merges_md5": merges_md5, "shards": g.nshards, "batches": st["iterations"],
           "candidates": st["candidates"],
           "occurrences": st["occurrences"], "breakdown_ms": {"init": round(st["ms_init"], 2),
                                                             "replay": round(st["ms_train"], 2)},
           "roofline": {"bound": "hbm", "achieved": round(alg / el / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / el / 1e9 / HBM_PEAK_GBS, 5),
                        "bytes": alg, "note": "whole-job algorithmic bytes (input + n_out*w) / wall"}}
    g.close()
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_encode_baseline(merges, 3, args.cpu_encode_size)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1024, help="merge iterations timed")
    ap.add_argument("--warmup", type=int, default=16, help="merge iterations of a throwaway run")
    ap.add_argument("--size", type=int, default=1 << 30, help="corpus bytes per GPU")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-size", type=int, default=64 << 20)
    ap.add_argument("--cpu-merges", type=int, default=16)
    ap.add_argument("--sharded", action="store_true",
                    help="use the sharded path even with one rank")
    ap.add_argument("--no-encode", action="store_true", help="skip the configs[4] encode measurement")
    ap.add_argument("--encode-size", type=int, default=10 << 30)
    ap.add_argument("--encode-merges", type=int, default=32768)
    ap.add_argument("--cpu-encode-size", type=int, default=256 << 10)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N-rank flow on a one-GPU box: every rank on this device
    if os.environ.get("BPE_BENCH_DEVICE") is not None:
        local = int(os.environ["BPE_BENCH_DEVICE"])
    sharded = world > 1 or args.sharded
    dist = None
    if sharded:
        import torch
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        torch.cuda.set_device(local)
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from llmtokenizer_amd import api
    if sharded:
        from llmtokenizer_amd import dist as bdist
        e = bdist.group(local, max(args.steps, args.warmup))
        e.synth(0, args.seed, args.size, offset=rank * args.size)  # resident in HBM before timing
    else:
        e = api.Engine(local)
        e.synth(args.seed, args.size)

    # warmup: a throwaway short run (kernels loaded, graphs captured, pools warm)
    if args.warmup > 0:
        e.train(args.warmup)

    def barrier():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    k = e.train(args.steps)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    same = True
    if dist is not None:
        import hashlib
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        digests = [None] * world
        dist.all_gather_object(digests, hashlib.md5(e.merges().tobytes()).hexdigest())
        same = len(set(digests)) == 1
    st = e.stats()
    transport = e.transport() if sharded else "none"
    name, kms, kbytes, launches = e.kernel_profile()  # live, in-kernel wall clock
    ev_ms, ev_n = 0.0, 0
    if not sharded:
        # corroboration with HIP events: event-record nodes spliced around every
        # k_scan node of a second, shorter run (they add latency, so not in the timed run)
        e.set_profile(True)
        e.train(min(args.steps, 256))
        ev_ms, ev_n = e.event_profile()
        e.set_profile(False)
    if dist is not None:
        dist.barrier()
    e.close()
    enc = None
    if not args.no_encode:
        enc = encode_bench(args, rank, world, local, dist, barrier)

    if rank != 0:
        return
    corpus_mb = args.size / 1e6
    value = world * corpus_mb * k / elapsed
    achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else 0.0
    cp_ms = st["ms_count_pass"]
    cp_name = "k_pair_hist_span" if st["count_pass_span"] else "k_pair_hist"
    # span form: the count pass also writes the initial u32 tokens (fused kernel:
    # algorithmic bytes = 1 B/token read + 4 B/token write)
    cp_bytes = args.size * (5 if st["count_pass_span"] else 1)
    cp_achieved = cp_bytes / (cp_ms * 1e-3) / 1e9 if cp_ms > 0 else 0.0
    out = {
        "metric": "corpus MB/s per merge iter (train), 1 GiB synthetic corpus per GPU",
        "value": round(value, 1),
        "unit": "corpus MB/s per merge iter",
        "n_gpus": world,
        "steps": k,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / max(k, 1), 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic (random_text.txt-shaped, splitmix64 seed %d, generated in HBM)" % args.seed,
        "config": {"workload": "configs[3]: 1 GiB corpus/GPU, %d merges" % args.steps,
                   "corpus_bytes_per_gpu": args.size, "corpus_bytes_total": args.size * world, "merges": k,
                   "parallelism": ("dp%d: one training job, %d contiguous corpus shards, per merge a sum of count "
                                   "deltas + a gather of edge records over %s" %
                                   (world, world, {"p2p": "xGMI P2P mailboxes", "rccl": "RCCL"}.get(transport, transport)))
                   if sharded else "single GPU",
                   "merges_identical_across_ranks": same},
        # dominant kernel of the timed run: k_scan (latency-bound random gathers);
        # algorithmic bytes per launch = 8 B/candidate + 20 B/occurrence
        "roofline": {"kernel": name, "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_per_launch": round(kbytes), "avg_ms": round(kms, 5), "launches": launches,
                     "avg_ms_source": "device wall clock inside the timed run (first block entry to the last block's retired memory operations)",
                     "avg_ms_hip_events": round(ev_ms, 5) if ev_n else None, "hip_event_launches": ev_n,
                     "note": "per-merge kernel is bound by dependent-load latency, not bandwidth; "
                             "event nodes add their own latency to the measured span"},
        # the one corpus-wide streaming pass (pair count over 1 B/token, V = 256)
        "roofline_count_pass": {"kernel": cp_name, "bound": "hbm", "achieved": round(cp_achieved, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(cp_achieved / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": cp_bytes, "avg_ms": round(cp_ms, 4),
                                "note": ("fused count pass + initial tok[] write: 1 B/token read + 4 B/token write"
                                         if st["count_pass_span"] else "1 B/token read")},
        "breakdown_ms": {"init": round(st["ms_init"], 3), "loop": round(st["ms_train"], 3),
                         "total_engine": round(st["ms_total"], 3)},
        "engine": {k2: st[k2] for k2 in ("n_out", "iterations", "distinct_pairs", "merged_buckets",
                                          "tracked_iters", "tie_events", "edge_events", "rule_ties",
                                          "table_grows", "keys", "l1_rescanned", "spec_hits",
                                          "spec_misses")},
    }
    # the committed rocprofv3 --kernel-trace --stats summary of this command
    # (profiles/): its per-launch average includes dispatch and completion
    # signalling, which the in-kernel span (first block entry -> last block
    # exit) does not; both are reported
    prof = sorted(glob.glob(os.path.join(ROOT, "profiles", "r1_v*_train_kernel_stats.csv")),
                  key=lambda p: int(re.search(r"_v(\d+)_", p).group(1)))
    if prof:
        with open(prof[-1]) as f:
            for r in csv.DictReader(f):
                if r["Name"].split("(")[0].replace("bpeamd::", "").replace("void ", "").strip() == name:
                    rp_ms = float(r["AverageNs"]) / 1e6
                    out["roofline"]["avg_ms_rocprof"] = round(rp_ms, 5)
                    out["roofline"]["frac_at_rocprof_avg"] = round(kbytes / (rp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                    out["roofline"]["rocprof_summary"] = os.path.relpath(prof[-1], ROOT)
                    break
    # HBM traffic per launch from the committed rocprofv3 PMC passes
    # (tools/gpu_pmc.sh: FETCH_SIZE and WRITE_SIZE in separate runs)
    pmc = os.path.join(ROOT, "profiles", "r1_pmc_traffic.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            tr = json.load(f)
        if name in tr:
            out["roofline"]["traffic"] = tr[name]["traffic_bytes_per_launch"]
            out["roofline"]["traffic_source"] = ("profiles/r1_pmc_traffic.json (FETCH_SIZE raw, uncalibrated for "
                                                 "4-byte gathers, + WRITE_SIZE; 256-merge run)")
        if cp_name in tr:
            out["roofline_count_pass"]["traffic"] = tr[cp_name]["traffic_bytes_per_launch"]
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args.seed, args.cpu_size, args.cpu_merges)
    if enc is not None:
        out["encode"] = enc
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Benchmark: POA consensus windows/s and global alignments/s on MI355X
(BASELINE.json metric).

Default (`python bench.py`, one GPU): config B, the reference's single-batch
benchmark unit (cudapoa/benchmarks/main.cpp:30-39, single_batch.hpp:82-89): one
step is generate_poa() (H2D of the packed reads + the POA kernel) followed by
get_consensus() (D2H + the per-window result vectors) on a batch of 1024
windows x 32 reads x ~1 kb (std::minstd_rand(seed w) generators,
BatchSize(1100, 32), full alignment, -8/-6/8, int16 scores); windows are added
outside the timed region, as the reference's PauseTiming does.  The same line
carries `secondary` objects for config D (cudaaligner global alignment,
align_all() + sync_alignments() on 100k pairs x 5 kb) and config E (the
multi-batch streaming driver on one GPU's share of the 1M-window job).

Config E (`--config E`, and the default when WORLD_SIZE > 1): the reference's
multi-batch benchmark unit (multi_batch.hpp:64-171, BM_MultiBatchTest): windows
stream through concurrent batches on separate HIP streams fed by host threads
(fill + H2D + kernel + D2H all timed).  A step is E_STEP_WINDOWS windows; the K
timed steps of rank r are its K x 6250 windows, seeds 1 + r*K*6250 ..., streamed
by one process_batches call (K = 20: 125k windows per GPU, the 1M-window job
on 8 GPUs).  Weak scaling; one process per GPU; no collective inside the timed
region; after it, rank 0 gathers every rank's consensus over RCCL.

Prints one JSON line (rank 0) with roofline and cpu_baseline objects.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before libgwamd so both share one HIP runtime)
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
E_STEP_WINDOWS = 6250   # config E: windows per step (20 steps = 125k windows per GPU)
# The N > 1 default workload is config E; its like-for-like N = 1 point is
# `bench.py --config E` (also the secondary.E object of the default N = 1 line,
# whose headline is config B, the reference's single-batch benchmark).
E_ANCHOR = "N=1 like-for-like point: `python bench.py --config E` (= secondary.E of the default --gpus 1 line)"

ALIGNER_CONFIGS = {
    # 100k pairs x 5 kb, ~10% difference; Hirschberg-Myers
    # (create_aligner default) and, separately, full Myers
    "D": dict(pairs=100000, length=5000, algorithm="hirschberg_myers"),
    "D_myers": dict(pairs=100000, length=5000, algorithm="myers"),
    # the reference's other global aligners on the same pairs (secondary rows)
    "D_banded": dict(pairs=100000, length=5000, algorithm="myers_banded"),
    "D_ukkonen": dict(pairs=100000, length=5000, algorithm="ukkonen"),
    # BM_SingleAlignment at its largest size (cudaaligner/benchmarks/main.cpp:33-60,
    # 135-138): one pair, query = generate_random_genome(100000, minstd_rand(1)),
    # target = generate_random_sequence(query, 100000/30 x 3), default aligner
    "D_100k": dict(pairs=1, length=100000, algorithm="hirschberg_myers", recipe="BM_SingleAlignment"),
    # BM_SingleBatchAlignment<AlignerGlobalMyers / MyersBanded> at 65,536 bp
    # (main.cpp:85-124, 140-158): per-pair seeds here, target truncated to 65,536
    "D_myers_64k": dict(pairs=32, length=65536, algorithm="myers", recipe="BM_SingleBatchAlignment"),
    "D_banded_64k": dict(pairs=32, length=65536, algorithm="myers_banded", recipe="BM_SingleBatchAlignment"),
    "D_ukkonen_64k": dict(pairs=32, length=65536, algorithm="ukkonen", recipe="BM_SingleBatchAlignment"),
    # Ukkonen with bands wider than one wave (ukkonen_wide_kernel): 16 kb targets,
    # queries ~1,400 bases shorter (200 substitutions, 100 insertions, 1,500
    # deletions), i.e. ~800-row bands within the aligner's 10 % rule
    "D_ukkonen_wide_16k": dict(pairs=1024, length=16384, algorithm="ukkonen", recipe="length_difference"),
}

# per algorithm: oracle id, dominant kernel
ALIGNER_ALGOS = {
    "hirschberg_myers": (0, "hm_kernel"),
    "myers": (1, "myers_kernel"),
    "myers_banded": (2, "myers_banded_kernel"),
    "ukkonen": (3, "ukkonen_kernel"),
}

CONFIGS = {
    "B": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=False, bw=256, windows=1024),
    "B_banded": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=True, bw=256, windows=1024),
    # MSA mode, 10 kb windows x 16 reads, banded bw 256,
    # BatchSize(10600, 16, 256) -> int32 scores and node ids
    "C": dict(backbone=10000, reads=16, err=500, max_seq=10600, banded=True, bw=256, windows=128, msa=True,
              mem_per_window=400e6),
    # band widths past 256 (the reference accepts any multiple of 128,
    # batch.hpp:85-94): the band kernel with bw / 64 cells per lane
    "B_banded_512": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=True, bw=512, windows=1024),
    "C_512": dict(backbone=10000, reads=16, err=500, max_seq=10600, banded=True, bw=512, windows=128, msa=True,
                  mem_per_window=600e6),
    # shapes the global-memory kernel took until round 5: band widths 384 and
    # 1024 (band kernel, 6 / 16 cells per lane), and full alignment with
    # 32-bit scores (4 kb reads, 16 per window: use32bitScore,
    # cudapoa_limits.hpp:28-53; the LDS kernel's 32-bit pass)
    "B_banded_384": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=True, bw=384, windows=1024),
    # (bw 1,024 runs four windows per CU, so the persistent grid's per-slot
    # scratch for 1,024 slots needs more than 12.5 MB per window; the
    # reference's benchmark gives its batch 90 % of the free memory,
    # single_batch.hpp:43-50)
    "B_banded_1024": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=True, bw=1024, windows=1024,
                          mem_per_window=24e6),
    "F_int32_4k": dict(backbone=4000, reads=16, err=200, max_seq=4400, banded=False, bw=256, windows=128,
                       mem_per_window=300e6),
}
# the config-B generator, seeds 1..1e6, 125k per GPU
STREAM_CONFIGS = {"E": dict(CONFIGS["B"], windows_per_step=E_STEP_WINDOWS)}


def golden_long(recipe, size, algorithm):
    """The tests/golden/aligner_long.json case of a reference benchmark pair, if any."""
    try:
        gl = json.load(open(os.path.join(ROOT, "tests", "golden", "aligner_long.json")))
    except (OSError, ValueError):
        return None
    for c in gl["cases"]:
        if c["recipe"] == recipe and c["size"] == size and c["algorithm"] == algorithm:
            return c
    return None


def aligner_alg_bytes(algorithm, q, t):
    """Algorithmic HBM bytes of one pair (measurement): the
    bit-vector / score state the aligner stores once per pair."""
    Q, T = len(q), len(t)
    if algorithm == "myers_banded":
        # first band of myers_banded_kernel (myers_gpu.cu:749-760): pv, mv, score
        # per band word and target column (config D pairs are accepted on it)
        d = abs(T - Q)
        est = max(1, d + min(T, Q) // 20)
        p = min(T, Q, (est - d) // 2)
        bw = min(1 + 2 * p + d, Q)
        if bw % 32 == 1 and bw != Q:
            bw = min(1 + 2 * (p + 1) + d, Q)
        return ((bw + 31) // 32) * (T + 1) * 12
    if algorithm == "ukkonen":
        # int16 (k, l) band matrix, bw rows x (n + m) columns (ukkonen_gpu.cu:192-197)
        m, n = min(Q, T) + 1, max(Q, T) + 1
        return ((1 + n - m + 200 + 1) // 2) * (n + m) * 2
    # full Myers state: ceil(q/32) words x (t+1) columns x 12 B
    return ((Q + 31) // 32) * (T + 1) * 12


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--config", default=None,
                   choices=sorted(CONFIGS) + sorted(ALIGNER_CONFIGS) + sorted(STREAM_CONFIGS),
                   help="default: B on one GPU (with D and E as secondary objects), E when WORLD_SIZE > 1")
    p.add_argument("--pairs", type=int, default=None, help="override aligner pairs per GPU")
    p.add_argument("--windows", type=int, default=None, help="override windows per GPU (B, C)")
    p.add_argument("--cpu-sample", type=int, default=None, help="windows / pairs in the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-secondary", action="store_true", help="default run: skip the D and E objects")
    p.add_argument("--secondary-steps", type=int, default=3, help="timed steps of the D object")
    p.add_argument("--stream-batches", type=int, default=2, help="E: concurrent batches (streams + host threads)")
    p.add_argument("--stream-batch-windows", type=int, default=4096, help="E: windows per batch")
    p.add_argument("--stream-step-windows", type=int, default=None,
                   help="E: windows per step (default %d; 20 steps = 125k windows per GPU)" % E_STEP_WINDOWS)
    p.add_argument("--secondary-c-steps", type=int, default=3, help="timed steps of the default run's C object")
    p.add_argument("--cpus", type=int, default=None,
                   help="pin each rank to K host CPUs (rank r: the r-th K of its affinity set) before any GPU "
                        "call, to predict a host-bound multi-GPU run on one GPU")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU rehearsal of the multi-rank launch (gloo): config E with stand-in rows instead of the "
                        "GPU engine; prints a line marked dry_run that is not a measurement")
    return p.parse_args()


def affinity_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_threads():
    """Host CPUs this process can use: the CPUs it may run on
    (sched_getaffinity), capped by the cgroup's CPU-time quota (cpu.max) when
    one is set -- more threads than the quota only time-slice the same CPU
    time.  The CPU baseline runs on all of them."""
    n = affinity_cpus()
    q = cgroup_cpu_quota()
    if q:
        n = max(1, min(n, int(q)))
    return n


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (None: unlimited / unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_fields(th, used, value=None):
    """Host facts of a CPU leg; value_per_core = the leg's rate / the threads it
    used, so a reader can scale it to the unthrottled host's core count."""
    f = {"cores": int(used), "threads_requested": th, "nproc": os.cpu_count(),
         "affinity_cpus": affinity_cpus(), "cgroup_cpu_quota": cgroup_cpu_quota(), "cpu_model": cpu_model()}
    if value is not None and used:
        f["value_per_core"] = round(value / int(used), 4)
    return f


def load_traffic(kind, key, n):
    tfile = os.path.join(ROOT, "profiles", "traffic_%s_%s.json" % (kind, key))
    if not os.path.exists(tfile):
        return None, None
    try:
        tf = json.load(open(tfile))
    except (OSError, ValueError):
        return None, None
    if tf.get("windows", tf.get("pairs")) != n:
        return None, None
    # aligner batches run several launches per align_all(): bytes per step
    return tf.get("hbm_bytes_per_step", tf.get("hbm_bytes_per_launch")), tf.get("source")


def load_sq(key):
    """SQ counter summary of the dominant kernel (scripts/pmc_sq.sh), if committed."""
    f = os.path.join(ROOT, "profiles", "sq_%s.json" % key)
    if not os.path.exists(f):
        return None
    try:
        d = json.load(open(f))
    except (OSError, ValueError):
        return None
    d["_file"] = "profiles/sq_%s.json" % key
    return d


def summary_of(line):
    """One config's headline numbers (value, step time, roofline, CPU leg,
    parity) for the compact `summary` object that ends the bench line."""
    if not line:
        return None
    roof = line.get("roofline") or {}
    cpu = line.get("cpu_baseline") or {}
    par = line.get("parity") or {}
    s = {"value": line.get("value"), "unit": line.get("unit"), "ms_per_step": line.get("ms_per_step"),
         "steps": line.get("steps"), "frac": roof.get("frac"), "kernel_ms": roof.get("kernel_ms"),
         "cpu_baseline": cpu.get("value"), "cpu_cores": cpu.get("cores"),
         "bit_exact_vs_oracle": par.get("bit_exact_vs_oracle")}
    if "valu_issue_frac" in roof:
        s["valu_issue_frac"] = roof["valu_issue_frac"]
    return s


class Ctx:
    """One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK /
    WORLD_SIZE); RCCL ("nccl") between the ranks.  dry: gloo on CPU, no GPU."""

    def __init__(self, dry=False):
        self.dry = dry
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if dry:
            if self.world > 1:
                dist.init_process_group("gloo")
            self.dev = None
            self.device = "cpu"
            return
        if self.world > 1:
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local_rank))
        torch.cuda.set_device(self.local_rank)
        self.dev = self.local_rank
        self.device = "cuda"

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def sync(self):
        if not self.dry:
            torch.cuda.synchronize()

    def max_over_ranks(self, v):
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, v):
        t = torch.tensor([v], dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())


def roofline(alg_bytes, kernel_ms, traffic, kernel, source=None, sq=None):
    kernel_s = kernel_ms / 1e3
    achieved = alg_bytes / kernel_s / 1e9
    r = {"bound": "issue", "priced_as": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "kernel": kernel,
         "kernel_ms": round(kernel_ms, 3), "algorithmic_bytes_per_launch": alg_bytes,
         "note": "integer DP; achieved = SURVEY 8(d) algorithmic bytes / kernel time; the kernel is "
                 "instruction-issue / latency bound, measured HBM traffic is in hbm_measured_*"}
    if traffic:
        r["hbm_measured_gbs"] = round(traffic / kernel_s / 1e9, 2)
        r["hbm_measured_frac"] = round(traffic / kernel_s / 1e9 / HBM_PEAK_GBS, 4)
        r["traffic_source"] = source
    if sq:
        # the derived SQ fractions only; the per-counter values stay in the
        # committed profiles/sq_*.json (sq_file), so the line stays short enough
        # for the driver's stdout tail to hold every config's numbers
        r["sq"] = {k: sq[k] for k in ("valu_issue_util", "wait_frac", "active_valu_frac", "salu_per_valu", "source")
                   if k in sq}
        if sq.get("_file"):
            r["sq"]["sq_file"] = sq["_file"]
        if sq.get("valu_issue_util") is not None:
            # the kernels are issue-bound: VALU issue slots used / available (SQ
            # counters of the committed profile, scripts/sq_summary.py)
            r["valu_issue_frac"] = sq["valu_issue_util"]
            r["valu_issue_source"] = sq.get("source")
    return r


# ---------------------------------------------------------------------------
# config D (and D_*): global alignments/s, step = align_all() + sync_alignments()
# ---------------------------------------------------------------------------
def bench_aligner(ctx, key, steps, warmup, args, with_cpu):
    cfg = dict(ALIGNER_CONFIGS[key])
    if args.pairs:
        cfg["pairs"] = args.pairs
    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch

    n, L = cfg["pairs"], cfg["length"]
    t0 = time.time()
    recipe = cfg.get("recipe")
    if recipe == "length_difference":
        qs, ts = synth.pairs(1 + ctx.rank * n, n, L, L, 200, 100, 1500)
        recipe = None
    elif recipe:
        # the reference benchmark's pair: query = the random genome, target =
        # its 10 %-difference copy (L/30 substitutions, insertions, deletions)
        e = L // 30
        muts, genomes = synth.pairs(1 + ctx.rank * n, n, L, L if recipe == "BM_SingleBatchAlignment" else L + e + 1,
                                    e, e, e)
        qs, ts = genomes, muts
    else:
        qs, ts = synth.pairs(1 + ctx.rank * n, n, L, L, 166, 166, 166)
    gen_s = time.time() - t0
    stream = torch.cuda.Stream()
    mq, mt = max(len(q) for q in qs), max(len(t) for t in ts)
    b = CudaAlignerBatch(mq, mt, n, stream=stream, algorithm=cfg["algorithm"])
    for q, t in zip(qs, ts):
        if b.add_alignment(q, t) != 0:
            raise RuntimeError("add_alignment failed")
    for _ in range(warmup):
        b.align_all()
        b.sync_alignments()
    ctx.barrier()
    torch.cuda.synchronize()
    kms = []
    t_start = time.perf_counter()
    for k in range(steps):
        # align_all = H2D + kernel + D2H (aligner_global.cpp:131-159; large
        # batches as two pipelined halves on two streams), sync_alignments =
        # wait + host fill; the aligner's HIP events bracket its kernels
        b.align_all()
        b.sync_alignments()
        kms.append(b.last_kernel_ms())
    torch.cuda.synchronize()
    ctx.barrier()
    wall = time.perf_counter() - t_start
    kernel_ms = float(np.mean(kms))
    wall_max = ctx.max_over_ranks(wall)
    paths, plen = b.raw_paths()
    if ctx.rank != 0:
        return None
    from oracle import oracle
    cells = sum(len(q) * len(t) for q, t in zip(qs, ts))
    alg_bytes = sum(aligner_alg_bytes(cfg["algorithm"], q, t) for q, t in zip(qs, ts))
    k = min(8 if L <= 20000 else 1, n)
    algo = ALIGNER_ALGOS[cfg["algorithm"]][0]
    gold = golden_long(recipe, L, cfg["algorithm"]) if recipe else None
    if gold is not None:
        # the first pair against tests/golden/aligner_long.json (oracle output,
        # make_aligner_long.py): a 100 kb oracle run takes ~40 s
        import hashlib
        p0 = paths[0, :plen[0]][::-1].tobytes()
        ok = int(plen[0]) == gold["path_length"] and hashlib.sha256(p0).hexdigest() == gold["path_sha256"]
        parity = {"pairs_checked": 1, "bit_exact_vs_oracle": bool(ok),
                  "pinned_by": "tests/golden/aligner_long.json: " + gold["name"]}
    else:
        ok = all(paths[i, :plen[i]][::-1].tolist() == oracle.align(qs[i], ts[i], algo, mq) for i in range(k))
        parity = {"pairs_checked": k, "bit_exact_vs_oracle": bool(ok)}
    # size-independent check over every pair: a global alignment consumes the
    # whole query (match/mismatch + deletion) and the whole target (match/
    # mismatch + insertion; cudaaligner.hpp:46-52)
    R = paths.shape[1]
    live = np.arange(R)[None, :] < plen[:, None]
    mm = (((paths == 0) | (paths == 1)) & live).sum(1)
    parity["all_pairs_consume_query_and_target"] = bool(
        np.all(mm + ((paths == 3) & live).sum(1) == np.array([len(q) for q in qs])) and
        np.all(mm + ((paths == 2) & live).sum(1) == np.array([len(t) for t in ts])))
    kb = min(1000, n)
    bases_ok = True
    for i in range(kb):
        p = paths[i, :plen[i]][::-1]
        qi = np.cumsum((p == 0) | (p == 1) | (p == 3)) - 1
        ti = np.cumsum((p == 0) | (p == 1) | (p == 2)) - 1
        qb = np.frombuffer(qs[i], np.uint8)
        tb = np.frombuffer(ts[i], np.uint8)
        m, x = p == 0, p == 1
        bases_ok = bases_ok and bool(np.all(qb[qi[m]] == tb[ti[m]]) and np.all(qb[qi[x]] != tb[ti[x]]))
    parity["pairs_match_states_on_equal_bases"] = {"pairs": kb, "ok": bases_ok}
    if cfg["algorithm"] == "myers_banded":
        # not an invariant of the reference's banded backtrace: its neighbour
        # scores at the band edges (myers_gpu.cu:377-494) can label unequal
        # bases as a match on long pairs; the oracle restatement does the same
        parity["pairs_match_states_on_equal_bases"]["invariant"] = False
    cpu = None
    if with_cpu:  # rank 0, after the timed region, at every GPU count
        th = cpu_threads()
        ns = args.cpu_sample or min(n, max(th * 12, 64) if L <= 20000 else th)
        tc = time.perf_counter()
        cres, used = oracle.align_batch(list(zip(qs[:ns], ts[:ns])), algo, mq, th)
        cpu_s = time.perf_counter() - tc
        match = all(cres[i] == paths[i, :plen[i]][::-1].tolist() for i in range(ns))
        cpu = dict({"value": round(ns / cpu_s, 3), "unit": "alignments/s", "kind": "port",
                    "sample": "first %d pairs of the same workload, oracle/aligner_oracle.cpp (reference-algorithm "
                              "C++ restatement, scalar DP), OpenMP one pair per thread, %.1f s wall" % (ns, cpu_s),
                    "matches_gpu": bool(match)}, **cpu_fields(th, used, ns / cpu_s))
    grid, dev_bytes = b.config()
    traffic, tsrc = load_traffic("aligner", key, n)
    return {
        "metric": "global alignments/sec",
        "value": round(n * ctx.world * steps / wall_max, 3),
        "unit": "alignments/s",
        "n_gpus": ctx.world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(wall_max / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int16" if cfg["algorithm"] == "ukkonen" else "u32 bit-vectors",
        "data": "synthetic (reference genomeutils generators, seeds 1..N)",
        "config": {"workload": "cudaaligner global, %d pairs/GPU x %d bp, ~10%% difference, %s%s"
                               % (n, L, cfg["algorithm"], (", %s recipe" % recipe) if recipe else ""),
                   "config_key": key, "step": "align_all() + sync_alignments() (aligner_global.cpp:131-191)",
                   "pairs_per_gpu": n, "length": L, "algorithm": cfg["algorithm"], "grid": grid,
                   "device_bytes": dev_bytes, "gcups": round(cells / (kernel_ms / 1e3) / 1e9, 3),
                   "kernel_only_alignments_per_s": round(n / (kernel_ms / 1e3), 1),
                   "input_gen_s": round(gen_s, 2), "parallelism": "dp%d (pairs sharded)" % ctx.world},
        "roofline": roofline(alg_bytes, kernel_ms, traffic, ALIGNER_ALGOS[cfg["algorithm"]][1], tsrc,
                             load_sq("aligner_" + key)),
        "cpu_baseline": cpu,
        "parity": parity,
    }


# ---------------------------------------------------------------------------
# configs B, B_banded, C: one resident batch, step = generate_poa() + get_consensus()
# ---------------------------------------------------------------------------
def windows_from_packed(bases, lens):
    raw = bases.tobytes()
    off, out = 0, []
    for w in range(lens.shape[0]):
        win = []
        for r in range(lens.shape[1]):
            k = int(lens[w, r])
            win.append(raw[off:off + k])
            off += k
        out.append(win)
    return out


def bench_poa(ctx, key, steps, warmup, args, with_cpu):
    cfg = dict(CONFIGS[key])
    if args.windows:
        cfg["windows"] = args.windows
    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
    from claragenomicsanalysis_amd.shard import window_range

    first_seed, nwin = window_range(ctx.rank, cfg["windows"])
    t0 = time.time()
    bases, lens = synth.poa_windows_packed(first_seed, nwin, cfg["backbone"], cfg["reads"], cfg["err"], cfg["err"],
                                           cfg["err"])
    windows = windows_from_packed(bases, lens)
    gen_s = time.time() - t0

    stream = torch.cuda.Stream(device=ctx.dev)
    msa = bool(cfg.get("msa", False))
    max_mem = int(nwin * cfg.get("mem_per_window", 12.5e6)) + (2 << 30)
    batch = CudaPoaBatch(cfg["reads"], cfg["max_seq"], max_mem, device_id=ctx.dev, stream=stream,
                         output_type="msa" if msa else "consensus",
                         cuda_banded_alignment=cfg["banded"], alignment_band_width=cfg["bw"])
    if batch.get_capacity()[1] < nwin:
        raise RuntimeError("batch holds %d windows, need %d" % (batch.get_capacity()[1], nwin))
    for w, win in enumerate(windows):
        st, _ = batch.add_poa_group(win)
        if st != 0:
            raise RuntimeError("add_poa_group failed for window %d: %d" % (w, st))
    score_bits, size_bits = batch.get_types()

    def fetch():
        if msa:
            return batch.get_msa()  # Batch::get_msa (D2H + the per-window row vectors)
        return batch.get_consensus_raw()

    for _ in range(warmup):
        batch.generate_poa()
        fetch()
    ctx.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t_start = time.perf_counter()
    for k in range(steps):
        # generate_poa() = H2D of the batch + the kernel (cudapoa_batch.cuh:163-171);
        # the events bracket the kernel on the batch's stream
        batch.upload()
        evs[k][0].record(stream)
        batch.launch()
        evs[k][1].record(stream)
        fetch()  # get_consensus(): blocks, D2H, result vectors
    torch.cuda.synchronize()
    ctx.barrier()
    wall = time.perf_counter() - t_start
    kernel_ms = float(np.mean([a.elapsed_time(e) for a, e in evs]))
    wall_max = ctx.max_over_ranks(wall)

    # outputs + work counters (outside the timed region)
    if msa:
        msa_rows, status = batch.get_msa()
        cons = ["".join(rows) for rows in msa_rows]
        cov = None
    else:
        cons, cov, status = batch.get_consensus()
    cells, final_nodes = batch.get_stats()
    ticks = batch.get_phase_ticks()  # last launch, 100 MHz
    n_ok = int(sum(1 for s in status if s == 0))
    cells_total = int(cells.sum())
    alg_bytes = cells_total * (score_bits // 8) * 2 + 2 * int(lens.sum()) + 3 * int(sum(len(c) for c in cons))

    gather_ms = None
    if ctx.world > 1:  # final consensus gather to rank 0 over RCCL
        from claragenomicsanalysis_amd.shard import gather_consensus
        torch.cuda.synchronize()
        tg = time.perf_counter()
        allc = gather_consensus(cons, max(len(c) for c in cons) if msa else 2 * cfg["max_seq"], device="cuda")
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        if ctx.rank == 0 and len(allc) != nwin * ctx.world:
            raise RuntimeError("gather returned %d strings" % len(allc))
    if ctx.rank != 0:
        return None

    from oracle import oracle
    mn = ((4 if cfg["banded"] else 3) * cfg["max_seq"] + 3) // 4 * 4
    k = min(4, nwin)
    ok = True
    for i in range(k):
        r = oracle.poa_window(windows[i], banded=cfg["banded"], band_width=cfg["bw"], score_bits=score_bits,
                              max_nodes=mn, max_consensus=2 * cfg["max_seq"], max_seqs=cfg["reads"], msa=msa)
        if msa:
            ok = ok and (r.status == status[i] and (r.msa or []) == msa_rows[i])
        else:
            ok = ok and (r.status == status[i] and r.consensus == cons[i] and r.coverage == cov[i])
    parity = {"windows_checked": k, "bit_exact_vs_oracle": bool(ok), "all_windows_status_ok": n_ok == nwin}
    if msa:
        # MSA rows de-gapped are the window's reads (Test_CudapoaGenerateMSA2.cu:125-140)
        parity["all_msa_rows_degap_to_reads"] = bool(all(
            [row.replace("-", "") for row in msa_rows[i]] == [r.decode() for r in windows[i]] for i in range(nwin)))
        parity["pinned_by"] = ("banded + MSA: the reference holds no banded or MSA known-answer vector; parity is "
                               "HIP == IEEE-division oracle restatement (SURVEY 8(c) gap (i)), plus the de-gap "
                               "property above")
    else:
        parity["all_coverage_lengths_match"] = bool(all(len(cov[i]) == len(cons[i]) and len(cons[i]) > 0
                                                        for i in range(nwin)))
        if cfg["banded"]:
            parity["pinned_by"] = ("banded: no reference banded known-answer vector; parity is HIP == IEEE-division "
                                   "oracle restatement (SURVEY 8(c) gap (i))")
    cpu = None
    if with_cpu:  # rank 0, after the timed region, at every GPU count
        th = cpu_threads()
        ns = args.cpu_sample or min(nwin, max(th * (4 if msa else 8), 64))
        tc = time.perf_counter()
        res = oracle.poa_batch(windows[:ns], nthreads=th, banded=cfg["banded"], band_width=cfg["bw"],
                               score_bits=score_bits, max_nodes=mn, max_consensus=2 * cfg["max_seq"],
                               max_seqs=cfg["reads"], msa=msa, coverage=not msa)
        if msa:
            ccons, cst, _, used = res
        else:
            ccons, cst, ccov, _, used = res
        cpu_s = time.perf_counter() - tc
        if msa:
            ccons = ["".join(rows) for rows in ccons]
            match = all(ccons[i] == cons[i] and cst[i] == status[i] for i in range(ns))
        else:
            match = all(ccons[i] == cons[i] and cst[i] == status[i] and list(ccov[i]) == cov[i] for i in range(ns))
        cpu = dict({"value": round(ns / cpu_s, 3), "unit": "windows/s", "kind": "port",
                    "sample": "first %d windows of the same workload, oracle/poa_oracle.cpp (reference-algorithm "
                              "C++ restatement, not SPOA), OpenMP one window per thread, %.1f s wall" % (ns, cpu_s),
                    "matches_gpu": bool(match),
                    "compared": "status, consensus, coverage" if not msa else "status, MSA rows"},
                   **cpu_fields(th, used, ns / cpu_s))
    traffic, tsrc = load_traffic("poa", key, nwin)
    slots, resident = batch.get_grid()
    return {
        "metric": "POA windows/sec (%s)" % ("MSA" if msa else "consensus"),
        "value": round(nwin * ctx.world * steps / wall_max, 3),
        "unit": "windows/s",
        "n_gpus": ctx.world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(wall_max / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int16" if score_bits == 16 else "int32",
        "data": "synthetic (reference genomeutils generators, seeds 1..N)",
        "config": {"workload": "cudapoa %s, %d windows/GPU x %d reads x ~%d bp synthetic ONT, %s"
                               % ("MSA" if msa else "consensus", nwin, cfg["reads"], cfg["backbone"],
                                  "banded bw=%d" % cfg["bw"] if cfg["banded"] else "full alignment"),
                   "config_key": key,
                   "step": "generate_poa() (H2D + kernel) + get_%s() (D2H + result vectors), as BM_SingleBatchTest"
                           % ("msa" if msa else "consensus"),
                   "windows_per_gpu": nwin, "batch_size": [cfg["max_seq"], cfg["reads"]],
                   "scores": [-8, -6, 8], "parallelism": "dp%d (windows sharded, RCCL gather)" % ctx.world,
                   "score_bits": score_bits, "size_bits": size_bits,
                   "kernel_variant": ["", "global", "lds", "band", "band_ad"][batch.kernel_variant()],
                   "grid_slots": slots, "resident_workgroups": resident,
                   "windows_ok": n_ok, "dp_cells_per_step": cells_total,
                   "gcups": round(cells_total / (kernel_ms / 1e3) / 1e9, 3),
                   "kernel_only_windows_per_s": round(nwin / (kernel_ms / 1e3), 1),
                   "mean_final_nodes": round(float(np.mean(final_nodes)), 1),
                   "gather_ms": gather_ms, "input_gen_s": round(gen_s, 2),
                   "phase_ms_mean_per_window": {name: round(float(ticks[:, i].mean()) / 1e5, 3)
                                                for i, name in enumerate(batch.PHASES)}},
        "roofline": roofline(alg_bytes, kernel_ms, traffic, "poa_window_kernel_%s" %
                             ["", "v1", "lds", "band", "band"][batch.kernel_variant()], tsrc, load_sq("poa_" + key)),
        "cpu_baseline": cpu,
        "parity": parity,
    }


# ---------------------------------------------------------------------------
# config E: the multi-batch streaming driver, step = E_STEP_WINDOWS windows
# ---------------------------------------------------------------------------
def busy_union_ms(start, stop):
    """Time during which at least one of the launches [start_i, stop_i) ran."""
    tot, cur_a, cur_b = 0.0, None, None
    for a, b in sorted(zip(start.tolist(), stop.tolist())):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                tot += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        tot += cur_b - cur_a
    return tot


def dry_rows(first_seed, n, width):
    """Dry run stand-in for the GPU engine's output: a deterministic function of
    each window's global seed (status 0, length, bytes, coverage), so rank 0
    can check the gathered rows window by window."""
    seeds = np.arange(first_seed, first_seed + n, dtype=np.int64)
    clen = (1 + seeds % (width - 1)).astype(np.int32)
    col = np.arange(width, dtype=np.int64)[None, :]
    live = col < clen[:, None]
    cons = np.where(live, np.array(list(b"ACGT"), np.uint8)[(seeds[:, None] + col) % 4], 0).astype(np.uint8)
    cov = np.where(live, (seeds[:, None] * 7 + col) % 65521, 0).astype(np.uint16)
    return np.zeros(n, np.int32), clen, cons, cov


def stream_cpu_leg(cfg, first_seed, nwin, ns, gpu=None):
    """CPU baseline of config E: the oracle (OpenMP, one window per thread,
    every usable host CPU) on ns windows spread evenly over the rank's stream,
    regenerated from their seeds (so the dry run times the same work).  gpu =
    (status, clen, cons, cov) of the rank's stream to compare, or None."""
    from claragenomicsanalysis_amd import synth
    from oracle import oracle
    th = cpu_threads()
    sidx = sorted(set(np.linspace(0, nwin - 1, min(ns, nwin)).astype(int).tolist()))
    wins = []
    for i in sidx:
        b1, l1 = synth.poa_windows_packed(first_seed + i, 1, cfg["backbone"], cfg["reads"], cfg["err"], cfg["err"],
                                          cfg["err"])
        wins.append(windows_from_packed(b1, l1)[0])
    tc = time.perf_counter()
    cc, cs, cv, _, cused = oracle.poa_batch(wins, nthreads=th, max_nodes=3 * cfg["max_seq"],
                                            max_consensus=2 * cfg["max_seq"], max_seqs=cfg["reads"], coverage=True)
    cpu_s = time.perf_counter() - tc
    match = None
    if gpu is not None:
        status, clen, cons, cov = gpu
        match = bool(all(cs[j] == status[i] and cc[j] == cons[i, :clen[i]].tobytes().decode() and
                         list(cv[j]) == cov[i, :clen[i]].tolist() for j, i in enumerate(sidx)))
    value = len(sidx) / cpu_s
    return dict({"value": round(value, 3), "unit": "windows/s", "kind": "port",
                 "sample": "%d windows spread evenly over rank 0's stream, oracle/poa_oracle.cpp (reference-algorithm "
                           "C++ restatement, not SPOA), OpenMP one window per thread, %.1f s wall, timed on rank 0 "
                           "after the GPU region" % (len(sidx), cpu_s),
                 "matches_gpu": match, "compared": "status, consensus, coverage"}, **cpu_fields(th, cused, value))


def bench_stream(ctx, key, steps, warmup, args, with_cpu):
    cfg = dict(STREAM_CONFIGS[key])
    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.shard import stream_window_range, gather_rows

    per_step = args.stream_step_windows or cfg["windows_per_step"]
    first_seed, nwin = stream_window_range(ctx.rank, steps, per_step)
    t0 = time.time()
    if ctx.dry:
        bases = np.zeros(0, np.uint8)
        lens = np.zeros((nwin, cfg["reads"]), np.int32)
    else:
        bases, lens = synth.poa_windows_packed(first_seed, nwin, cfg["backbone"], cfg["reads"], cfg["err"],
                                               cfg["err"], cfg["err"])
    gen_s = time.time() - t0
    read_lens = lens.ravel()
    rpw = np.full(nwin, cfg["reads"], np.int64)
    launches = None
    nb_used = per_batch = rounds = mem = None
    if ctx.dry:
        stride = 2 * cfg["max_seq"]
        ctx.barrier()
        t_start = time.perf_counter()
        status, clen, cons, cov = dry_rows(first_seed, nwin, stride)
        ctx.barrier()
        wall = time.perf_counter() - t_start
    else:
        from claragenomicsanalysis_amd.cudapoa import CudaPoaMultiBatch, estimate_max_poas
        # device bytes per batch so that a batch holds stream_batch_windows windows
        # by the reference's own capacity rule (BatchBlock::estimate_max_poas)
        probe = 64 << 30
        per_window = probe / max(1, estimate_max_poas(cfg["max_seq"], cfg["reads"], cfg["bw"], banded=cfg["banded"],
                                                      msa=False, free_device_memory=probe,
                                                      gpu_memory_usage_quota=1.0))
        mem = int(per_window * args.stream_batch_windows) + (64 << 20)
        mb = CudaPoaMultiBatch(cfg["reads"], cfg["max_seq"], num_batches=args.stream_batches, mem_per_batch=mem,
                               device_id=ctx.dev, cuda_banded_alignment=cfg["banded"],
                               alignment_band_width=cfg["bw"])
        stride = mb.stride
        out = (np.zeros(nwin, np.int32), np.zeros(nwin, np.int32), np.zeros((nwin, stride), np.uint8),
               np.zeros((nwin, stride), np.uint16))
        for arr in out:  # touch the pages outside the timed region
            arr.fill(0)
        if warmup > 0:  # untimed pass over this rank's first warmup x step windows
            wn = min(nwin, warmup * per_step)
            nb = int(read_lens[:wn * cfg["reads"]].sum())
            mb.process_packed(bases[:nb], read_lens[:wn * cfg["reads"]], rpw[:wn])
        # HIP events around every kernel launch, on each batch's own stream
        mb.set_launch_timing(True)
        ctx.barrier()
        ctx.sync()
        t_start = time.perf_counter()
        mb.process_packed(bases, read_lens, rpw, out=out)
        ctx.sync()
        ctx.barrier()
        wall = time.perf_counter() - t_start
        launches = mb.launches()
        status, clen, cons, cov = out
        nb_used, per_batch, rounds = mb.info()
    wall_max = ctx.max_over_ranks(wall)
    n_ok = int((status == 0).sum())

    # Final gather: every rank's [len | status | consensus |
    # coverage] rows to rank 0 over RCCL, one dist.gather, rows trimmed to the
    # longest consensus of the job.
    gather_ms = None
    gathered = None
    width = None
    if ctx.world > 1:
        width = int(ctx.max_over_ranks(float(clen.max() if nwin else 0)))
        ctx.sync()
        tg = time.perf_counter()
        rows = np.concatenate([clen.view(np.uint8).reshape(nwin, 4), status.view(np.uint8).reshape(nwin, 4),
                               cons[:, :width], np.ascontiguousarray(cov[:, :width]).view(np.uint8)], axis=1)
        gathered = gather_rows(rows, device=ctx.device)
        ctx.sync()
        gather_ms = (time.perf_counter() - tg) * 1e3
    if ctx.rank != 0:
        return None
    parity = {"all_windows_status_ok": n_ok == nwin}
    if gathered is not None:
        glen = gathered[:, :4].copy().view(np.int32).ravel()
        gst = gathered[:, 4:8].copy().view(np.int32).ravel()
        gcons = gathered[:, 8:8 + width]
        gcov = gathered[:, 8 + width:].copy().view(np.uint16)
        parity["gathered_windows"] = int(gathered.shape[0])
        parity["gathered_bytes"] = int(gathered.nbytes)
        parity["gathered_all_status_ok"] = bool((gst == 0).all() and (glen > 0).all())
        parity["gathered_rank0_rows_equal_local"] = bool(
            np.array_equal(gcons[:nwin], cons[:, :width]) and np.array_equal(gcov[:nwin], cov[:, :width]) and
            np.array_equal(glen[:nwin], clen))
    if ctx.dry:
        if gathered is not None:
            es, el, ec, ev = dry_rows(1, nwin * ctx.world, stride)
            parity["gathered_rows_equal_expected"] = bool(
                np.array_equal(gst, es) and np.array_equal(glen, el) and np.array_equal(gcons, ec[:, :width]) and
                np.array_equal(gcov, ev[:, :width]))
        cpu = stream_cpu_leg(cfg, first_seed, nwin, args.cpu_sample or 16) if with_cpu else None
        return {"metric": "POA windows/sec (consensus)", "value": None, "unit": "windows/s", "dry_run": True,
                "n_gpus": ctx.world, "steps": steps, "warmup": warmup, "ms_per_step": None,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "int16",
                "data": "dry run on CPU (gloo): stand-in rows, no GPU, not a measurement",
                "config": {"workload": "config E rehearsal", "config_key": key, "windows_per_gpu": nwin,
                           "gather_width": width, "gather_ms": gather_ms, "anchor": E_ANCHOR,
                           "parallelism": "dp%d (windows sharded, gloo gather)" % ctx.world},
                "roofline": None, "cpu_baseline": cpu, "parity": parity}

    # oracle check of a sample spread over the rank's stream (windows from every
    # batch round) and, at N > 1, of windows the other ranks computed
    from oracle import oracle
    starts = np.concatenate([[0], np.cumsum(read_lens)])

    def window_reads(i):
        r0 = i * cfg["reads"]
        return [bases[starts[r]:starts[r + 1]].tobytes() for r in range(r0, r0 + cfg["reads"])]

    idx = sorted(set(np.linspace(0, nwin - 1, 12).astype(int).tolist()))
    mn = 3 * cfg["max_seq"]
    rcons, rst, rcov, _, used = oracle.poa_batch([window_reads(i) for i in idx], nthreads=cpu_threads(),
                                                 max_nodes=mn, max_consensus=2 * cfg["max_seq"],
                                                 max_seqs=cfg["reads"], coverage=True)
    ok = all(rst[j] == status[i] and rcons[j] == cons[i, :clen[i]].tobytes().decode() and
             list(rcov[j]) == cov[i, :clen[i]].tolist() for j, i in enumerate(idx))
    parity.update({"windows_checked": len(idx), "bit_exact_vs_oracle": bool(ok)})
    if gathered is not None:
        # two windows of every other rank, regenerated here from their seeds
        gidx = [r * nwin + k for r in range(1, ctx.world) for k in (0, nwin - 1)]
        wins = []
        for g in gidx:
            b1, l1 = synth.poa_windows_packed(1 + g, 1, cfg["backbone"], cfg["reads"], cfg["err"], cfg["err"],
                                              cfg["err"])
            wins.append(windows_from_packed(b1, l1)[0])
        gc, gs, gv, _, _ = oracle.poa_batch(wins, nthreads=cpu_threads(), max_nodes=mn,
                                            max_consensus=2 * cfg["max_seq"], max_seqs=cfg["reads"], coverage=True)
        parity["gathered_other_ranks_checked"] = len(gidx)
        parity["gathered_other_ranks_bit_exact_vs_oracle"] = bool(all(
            gs[j] == gst[g] and gc[j] == gcons[g, :glen[g]].tobytes().decode() and
            list(gv[j]) == gcov[g, :glen[g]].tolist() for j, g in enumerate(gidx)))

    # roofline of the streamed kernels: SURVEY 8(d) priced bytes of every launch
    # (4 B per int16 DP cell + inputs + outputs) over the time the GPU ran at
    # least one of them (the batches' kernels overlap on their two streams)
    cells_total = int(launches["cells"].sum())
    alg_bytes = cells_total * 2 * 2 + 2 * int(read_lens.sum()) + 3 * int(clen.sum())
    busy_ms = busy_union_ms(launches["start_ms"], launches["stop_ms"])
    durations = launches["stop_ms"] - launches["start_ms"]
    # PMC HBM bytes per window of a profiled stream (scripts/summarize_profile.py, config E)
    traffic, tsrc = None, None
    try:
        tf = json.load(open(os.path.join(ROOT, "profiles", "traffic_poa_E.json")))
        traffic, tsrc = int(tf["hbm_bytes_per_window"] * nwin), tf.get("source")
    except (OSError, ValueError, KeyError):
        pass
    roof = roofline(alg_bytes, busy_ms, traffic, "poa_window_kernel_lds", tsrc, load_sq("poa_" + key))
    if traffic:
        roof["traffic_note"] = "PMC bytes per window of a profiled stream x this rank's windows"
    roof.update({"launches": int(len(durations)), "kernel_ms_sum": round(float(durations.sum()), 3),
                 "kernel_busy_ms": round(busy_ms, 3), "kernel_ms_mean_per_launch": round(float(durations.mean()), 3),
                 "windows_per_launch_mean": round(float(launches["windows"].mean()), 1),
                 "timing": "HIP events on each batch's stream around every launch, one clock; kernel_ms = the "
                           "union of the launch intervals (the kernels of the two batches overlap)"})
    cpu = None
    if with_cpu:  # rank 0, after the timed region and the gather, at every GPU count
        cpu = stream_cpu_leg(cfg, first_seed, nwin, args.cpu_sample or max(cpu_threads() * 8, 64),
                             (status, clen, cons, cov))
    total = nwin * ctx.world
    return {
        "metric": "POA windows/sec (consensus)",
        "value": round(total / wall_max, 3),
        "unit": "windows/s",
        "n_gpus": ctx.world, "steps": steps, "warmup": warmup,
        "ms_per_step": round(wall_max / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (reference genomeutils generators, seeds 1 + rank*%d ...)" % nwin,
        "config": {"workload": "cudapoa consensus, multi-batch stream of %d windows/GPU (%d steps x %d) x %d reads "
                               "x ~%d bp synthetic ONT, full alignment (1M-window job at 8 GPUs x 20 steps)"
                               % (nwin, steps, per_step, cfg["reads"], cfg["backbone"]),
                   "config_key": key,
                   "step": "%d windows through MultiBatch::process_batches (fill + H2D + kernel + D2H timed, "
                           "multi_batch.hpp:64-171)" % per_step,
                   "windows_per_gpu": nwin, "windows_total": total, "batches": nb_used,
                   "windows_per_batch": per_batch, "batch_rounds": rounds, "mem_per_batch": mem,
                   "batch_size": [cfg["max_seq"], cfg["reads"]], "scores": [-8, -6, 8],
                   "parallelism": "dp%d (windows sharded, RCCL gather)" % ctx.world,
                   "windows_ok": n_ok, "dp_cells": cells_total, "anchor": E_ANCHOR,
                   "gcups": round(cells_total / (busy_ms / 1e3) / 1e9, 3),
                   "gather_ms": gather_ms, "gather_width": width, "input_gen_s": round(gen_s, 2)},
        "roofline": roof,
        "cpu_baseline": cpu,
        "parity": parity,
    }


RUNNERS = {}
RUNNERS.update({k: bench_poa for k in CONFIGS})
RUNNERS.update({k: bench_aligner for k in ALIGNER_CONFIGS})
RUNNERS.update({k: bench_stream for k in STREAM_CONFIGS})


def free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def relaunch(args):
    """--gpus N > 1 outside torch.distributed.run: start N ranks (one process
    per GPU, the reference's one worker per device, cudamapper/src/main.cu:488-
    513) as a child torch.distributed.run and return its exit code.  Runs
    before anything touches the GPU; the child is a subprocess, not an exec."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr=127.0.0.1", "--master-port=%d" % free_port(), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", str(max(1, cpu_threads() // args.gpus)))
    return subprocess.call(cmd, env=env)


def pin_cpus(k):
    """--cpus K: restrict this rank (and the batch host threads it starts) to
    K CPUs of its affinity set, rank r taking the r-th group of K, so that one
    GPU can rehearse the host share a rank gets at N GPUs (the driver's cgroup
    grants 16 CPUs: 2 per rank at N = 8).  Called before any GPU call."""
    cpus = sorted(os.sched_getaffinity(0))
    r = int(os.environ.get("LOCAL_RANK", "0"))
    pick = cpus[r * k:(r + 1) * k] or cpus[:k]
    os.sched_setaffinity(0, pick)
    os.environ["OMP_NUM_THREADS"] = str(len(pick))
    return pick


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch(args))
    pinned = pin_cpus(args.cpus) if args.cpus else None
    ctx = Ctx(dry=args.dry_run)
    if args.gpus > 1 and ctx.world != args.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (args.gpus, ctx.world))
    default = args.config is None
    key = args.config or ("B" if ctx.world == 1 else "E")
    if ctx.dry and key != "E":
        raise SystemExit("--dry-run rehearses config E only")
    line = RUNNERS[key](ctx, key, args.steps, args.warmup, args, not args.no_cpu)
    if default and ctx.world == 1 and not args.no_secondary and not ctx.dry:
        # the metric's second half, the MSA config and the streaming driver, in the same run
        sec = {}
        sec["D"] = bench_aligner(ctx, "D", max(1, args.secondary_steps), 1, args, not args.no_cpu)
        sec["C"] = bench_poa(ctx, "C", max(1, args.secondary_c_steps), 1, args, not args.no_cpu)
        sec["E"] = bench_stream(ctx, "E", args.steps, min(args.warmup, 1), args, not args.no_cpu)
        if line is not None:
            line["secondary"] = sec
    if ctx.rank == 0 and line is not None:
        if pinned is not None:
            line.setdefault("config", {})["pinned_cpus"] = pinned
        # last key of the line: every config's headline numbers, so a reader of
        # the end of the output (the driver keeps its tail) sees all of them
        summ = {key: summary_of(line)}
        for k, v in (line.get("secondary") or {}).items():
            summ[k] = summary_of(v)
        line["summary"] = summ
        print(json.dumps(line), flush=True)
    if ctx.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

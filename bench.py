"""Benchmark: POA consensus windows/s on MI355X (BASELINE.json configs[1], "B").

Workload: 1024 windows per GPU; window w uses
std::minstd_rand(seed w) -> 1000-base backbone + 31 mutated copies
(generate_random_sequences(bb, 32, rng, 50, 50, 50)), BatchSize(1100, 32),
full alignment, scores -8/-6/8, int16 scores.  A step is one pass of the POA
kernel over the whole resident batch (graph build + NW + add + topsort +
consensus for every window).  Inputs are uploaded before timing.

N GPUs: one process per GPU (torch.distributed, RCCL), each rank runs its own
1024 windows (weak scaling); the consensus strings are gathered to rank 0 over
RCCL once after the timed region.

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

ALIGNER_CONFIGS = {
    # 100k pairs x 5 kb, ~10% difference; Hirschberg-Myers
    # (create_aligner default) and, separately, full Myers
    "D": dict(pairs=100000, length=5000, algorithm="hirschberg_myers"),
    "D_myers": dict(pairs=100000, length=5000, algorithm="myers"),
    # the reference's other global aligners on the same pairs (secondary rows)
    "D_banded": dict(pairs=100000, length=5000, algorithm="myers_banded"),
    "D_ukkonen": dict(pairs=100000, length=5000, algorithm="ukkonen"),
}

# per algorithm: oracle id, dominant kernel
ALIGNER_ALGOS = {
    "hirschberg_myers": (0, "hm_kernel"),
    "myers": (1, "myers_kernel"),
    "myers_banded": (2, "myers_banded_kernel"),
    "ukkonen": (3, "ukkonen_kernel"),
}


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

CONFIGS = {
    # name: (backbone, reads, mut, ins, del, max_seq, banded, band_width, windows per GPU)
    "B": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=False, bw=256, windows=1024),
    "B_banded": dict(backbone=1000, reads=32, err=50, max_seq=1100, banded=True, bw=256, windows=1024),
    # MSA mode, 10 kb windows x 16 reads, banded bw 256,
    # BatchSize(10600, 16, 256) -> int32 scores and node ids
    "C": dict(backbone=10000, reads=16, err=500, max_seq=10600, banded=True, bw=256, windows=128, msa=True,
              mem_per_window=400e6),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--config", default="B", choices=sorted(CONFIGS) + sorted(ALIGNER_CONFIGS))
    p.add_argument("--pairs", type=int, default=None, help="override aligner pairs per GPU")
    p.add_argument("--windows", type=int, default=None, help="override windows per GPU")
    p.add_argument("--cpu-sample", type=int, default=None, help="windows in the CPU baseline sample")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--traffic-file", default=None,
                   help="PMC HBM bytes per launch (default profiles/traffic_poa_<config>.json)")
    return p.parse_args()


def cpu_threads():
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    return os.cpu_count() or 1


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def bench_aligner(args):
    """Global alignments/s on this rank's pairs."""
    cfg = dict(ALIGNER_CONFIGS[args.config])
    if args.pairs:
        cfg["pairs"] = args.pairs
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch

    n, L = cfg["pairs"], cfg["length"]
    t0 = time.time()
    qs, ts = synth.pairs(1 + rank * n, n, L, L, 166, 166, 166)
    gen_s = time.time() - t0
    stream = torch.cuda.Stream()
    b = CudaAlignerBatch(L, L, n, stream=stream, algorithm=cfg["algorithm"])
    for q, t in zip(qs, ts):
        if b.add_alignment(q, t) != 0:
            raise RuntimeError("add_alignment failed")
    b.upload()
    b.synchronize()
    for _ in range(args.warmup):
        b.launch()
    b.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        b.launch()
    ev1.record(stream)
    b.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t_start
    kernel_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)
    t_max = torch.tensor([wall], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    wall_max = float(t_max.item())
    b.download()
    b.synchronize()
    paths, plen = b.raw_paths()
    cells = sum(len(q) * len(t) for q, t in zip(qs, ts))
    alg_bytes = sum(aligner_alg_bytes(cfg["algorithm"], q, t) for q, t in zip(qs, ts))
    out = None
    if rank == 0:
        from oracle import oracle
        k = min(8, n)
        ok = True
        algo = ALIGNER_ALGOS[cfg["algorithm"]][0]
        for i in range(k):
            want = oracle.align(qs[i], ts[i], algo, L)
            got = paths[i, :plen[i]][::-1].tolist()
            ok = ok and got == want
        parity = {"pairs_checked": k, "bit_exact_vs_oracle": bool(ok)}
        # size-independent check over every pair of the workload: a global
        # alignment consumes the whole query (match/mismatch + deletion, i.e.
        # present in query) and the whole target (match/mismatch + insertion,
        # present in target; cudaaligner.hpp:46-52)
        R = paths.shape[1]
        live = np.arange(R)[None, :] < plen[:, None]
        mm = (((paths == 0) | (paths == 1)) & live).sum(1)
        full_ok = bool(np.all(mm + ((paths == 3) & live).sum(1) == np.array([len(q) for q in qs])) and
                       np.all(mm + ((paths == 2) & live).sum(1) == np.array([len(t) for t in ts])))
        parity["all_pairs_consume_query_and_target"] = full_ok
        # and on the first 1000 pairs: match states join equal bases, mismatch states differing ones
        kb = min(1000, n)
        bases_ok = True
        for i in range(kb):
            p = paths[i, :plen[i]][::-1]
            qi = np.cumsum((p == 0) | (p == 1) | (p == 3)) - 1
            ti = np.cumsum((p == 0) | (p == 1) | (p == 2)) - 1
            qb = np.frombuffer(qs[i] if isinstance(qs[i], bytes) else qs[i].encode(), np.uint8)
            tb = np.frombuffer(ts[i] if isinstance(ts[i], bytes) else ts[i].encode(), np.uint8)
            m, x = p == 0, p == 1
            bases_ok = bases_ok and bool(np.all(qb[qi[m]] == tb[ti[m]]) and np.all(qb[qi[x]] != tb[ti[x]]))
        parity["pairs_match_states_on_equal_bases"] = {"pairs": kb, "ok": bases_ok}
        cpu = None
        if not args.no_cpu and world == 1:
            th = cpu_threads()
            ns = args.cpu_sample or min(n, max(th * 4, 16))
            tc = time.perf_counter()
            cres, used = oracle.align_batch(list(zip(qs[:ns], ts[:ns])), algo, L, th)
            cpu_s = time.perf_counter() - tc
            match = all(cres[i] == paths[i, :plen[i]][::-1].tolist() for i in range(ns))
            cpu = {"value": round(ns / cpu_s, 3), "unit": "alignments/s", "cores": int(used), "kind": "port",
                   "nproc": os.cpu_count(), "cpu_model": cpu_model(),
                   "sample": "first %d pairs of the same workload, oracle/aligner_oracle.cpp (reference-algorithm "
                             "C++ restatement, scalar DP), OpenMP one pair per thread, %.1f s wall" % (ns, cpu_s),
                   "matches_gpu": bool(match)}
        kernel_s = kernel_ms / 1e3
        achieved = alg_bytes / kernel_s / 1e9
        grid, dev_bytes = b.config()
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "traffic_aligner_%s.json" % args.config)
        if os.path.exists(tfile):
            try:
                tf = json.load(open(tfile))
                if tf.get("pairs") == n:
                    traffic = tf.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        out = {
            "metric": "global alignments/sec",
            "value": round(n * world * args.steps / wall_max, 3),
            "unit": "alignments/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "int16" if cfg["algorithm"] == "ukkonen" else "u32 bit-vectors",
            "data": "synthetic (reference genomeutils generators, seeds 1..N)",
            "config": {"workload": "cudaaligner global, %d pairs/GPU x %d bp, ~10%% difference, %s"
                                   % (n, L, cfg["algorithm"]),
                       "config_key": args.config, "pairs_per_gpu": n, "length": L,
                       "algorithm": cfg["algorithm"], "grid": grid, "device_bytes": dev_bytes,
                       "gcups": round(cells / kernel_s / 1e9, 3), "input_gen_s": round(gen_s, 2),
                       "parallelism": "dp%d (pairs sharded)" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": ALIGNER_ALGOS[cfg["algorithm"]][1],
                         "kernel_ms": round(kernel_ms, 3), "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.config in ALIGNER_CONFIGS:
        return bench_aligner(args)
    cfg = dict(CONFIGS[args.config])
    if args.windows:
        cfg["windows"] = args.windows
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    torch.cuda.set_device(local_rank)
    dev = local_rank

    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch

    from claragenomicsanalysis_amd.shard import window_range
    first_seed, nwin = window_range(rank, cfg["windows"])
    t0 = time.time()
    bases, lens = synth.poa_windows_packed(first_seed, nwin, cfg["backbone"], cfg["reads"], cfg["err"], cfg["err"],
                                           cfg["err"])
    raw = bases.tobytes()
    gen_s = time.time() - t0

    stream = torch.cuda.Stream(device=dev)
    msa = bool(cfg.get("msa", False))
    max_mem = int(nwin * cfg.get("mem_per_window", 12.5e6)) + (2 << 30)
    batch = CudaPoaBatch(cfg["reads"], cfg["max_seq"], max_mem, device_id=dev, stream=stream,
                         output_type="msa" if msa else "consensus",
                         cuda_banded_alignment=cfg["banded"], alignment_band_width=cfg["bw"])
    if batch.get_capacity()[1] < nwin:
        raise RuntimeError("batch holds %d windows, need %d" % (batch.get_capacity()[1], nwin))
    off = 0
    windows = []
    for w in range(nwin):
        win = []
        for r in range(cfg["reads"]):
            k = int(lens[w, r])
            win.append(raw[off:off + k])
            off += k
        windows.append(win)
        st, _ = batch.add_poa_group(win)
        if st != 0:
            raise RuntimeError("add_poa_group failed for window %d: %d" % (w, st))
    batch.upload()
    batch.synchronize()
    score_bits, size_bits = batch.get_types()

    for _ in range(args.warmup):
        batch.launch()
    batch.synchronize()

    # timed region: barrier + sync on both sides, HIP events on the batch stream
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t_start = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        batch.launch()
    ev1.record(stream)
    batch.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t_start
    kernel_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)

    t_max = torch.tensor([wall], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    wall_max = float(t_max.item())

    # outputs + work counters (outside the timed region)
    if msa:
        msa_rows, status = batch.get_msa()
        cons = ["".join(rows) for rows in msa_rows]  # gathered / counted as output bytes
        cov = None
    else:
        cons, cov, status = batch.get_consensus()
    cells, final_nodes = batch.get_stats()
    ticks = batch.get_phase_ticks()  # last launch, 100 MHz
    n_ok = int(sum(1 for s in status if s == 0))
    sb = score_bits // 8
    cells_total = int(cells.sum())
    alg_bytes = cells_total * sb * 2 + 2 * int(lens.sum()) + 3 * int(sum(len(c) for c in cons))

    # final consensus gather to rank 0 over RCCL
    gather_ms = None
    if world > 1:
        from claragenomicsanalysis_amd.shard import gather_consensus
        torch.cuda.synchronize()
        tg = time.perf_counter()
        allc = gather_consensus(cons, max(len(c) for c in cons) if msa else 2 * cfg["max_seq"], device="cuda")
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
        if rank == 0 and len(allc) != nwin * world:
            raise RuntimeError("gather returned %d strings" % len(allc))

    # parity spot-check and CPU baseline (rank 0, test infrastructure)
    parity = None
    cpu = None
    if rank == 0:
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
        parity = {"windows_checked": k, "bit_exact_vs_oracle": bool(ok)}
        # size-independent checks over every window of the workload
        parity["all_windows_status_ok"] = n_ok == nwin
        if msa:
            # MSA rows de-gapped are the window's reads (Test_CudapoaGenerateMSA2.cu:125-140)
            parity["all_msa_rows_degap_to_reads"] = bool(all(
                [row.replace("-", "") for row in msa_rows[i]] ==
                [r.decode() if isinstance(r, bytes) else r for r in windows[i]] for i in range(nwin)))
        else:
            parity["all_coverage_lengths_match"] = bool(all(len(cov[i]) == len(cons[i]) and len(cons[i]) > 0
                                                            for i in range(nwin)))
        if not args.no_cpu and world == 1:
            th = cpu_threads()
            ns = args.cpu_sample or min(nwin, max(th * (2 if msa else 48), 64 if not msa else 16))
            tc = time.perf_counter()
            ccons, cst, _, used = oracle.poa_batch(windows[:ns], nthreads=th, banded=cfg["banded"],
                                                   band_width=cfg["bw"], score_bits=score_bits, max_nodes=mn,
                                                   max_consensus=2 * cfg["max_seq"], max_seqs=cfg["reads"], msa=msa)
            cpu_s = time.perf_counter() - tc
            if msa:
                ccons = ["".join(rows) for rows in ccons]
            cpu = {"value": round(ns / cpu_s, 3), "unit": "windows/s", "cores": int(used), "kind": "port",
                   "nproc": os.cpu_count(), "cpu_model": cpu_model(),
                   "sample": "first %d windows of the same workload, oracle/poa_oracle.cpp (reference-algorithm "
                             "C++ restatement, not SPOA), OpenMP one window per thread, %.1f s wall" % (ns, cpu_s),
                   "matches_gpu": bool(all(ccons[i] == cons[i] for i in range(ns)))}

    if rank == 0:
        kernel_s = kernel_ms / 1e3
        achieved = alg_bytes / kernel_s / 1e9
        traffic = None
        if args.traffic_file is None:
            args.traffic_file = os.path.join(ROOT, "profiles", "traffic_poa_%s.json" % args.config)
        if os.path.exists(args.traffic_file):
            try:
                tf = json.load(open(args.traffic_file))
                if tf.get("config") == args.config and tf.get("windows") == nwin:
                    traffic = tf.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        total_windows = nwin * world
        out = {
            "metric": "POA windows/sec (%s)" % ("MSA" if msa else "consensus"),
            "value": round(total_windows * args.steps / wall_max, 3),
            "unit": "windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int16" if score_bits == 16 else "int32",
            "data": "synthetic (reference genomeutils generators, seeds 1..N)",
            "config": {"workload": "cudapoa %s, %d windows/GPU x %d reads x ~%d bp synthetic ONT, %s"
                                   % ("MSA" if msa else "consensus", nwin, cfg["reads"], cfg["backbone"],
                                      "banded bw=%d" % cfg["bw"] if cfg["banded"] else "full alignment"),
                       "config_key": args.config, "windows_per_gpu": nwin, "batch_size": [cfg["max_seq"],
                                                                                        cfg["reads"]],
                       "scores": [-8, -6, 8], "parallelism": "dp%d (windows sharded, RCCL gather)" % world,
                       "score_bits": score_bits, "size_bits": size_bits,
                       "kernel_variant": ["", "global", "lds", "band"][batch.kernel_variant()],
                       "windows_ok": n_ok, "dp_cells_per_step": cells_total,
                       "gcups": round(cells_total / kernel_s / 1e9, 3),
                       "mean_final_nodes": round(float(np.mean(final_nodes)), 1),
                       "gather_ms": gather_ms, "input_gen_s": round(gen_s, 2),
                       "phase_ms_mean_per_window": {name: round(float(ticks[:, i].mean()) / 1e5, 3)
                                                    for i, name in enumerate(batch.PHASES)}},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "poa_window_kernel", "kernel_ms": round(kernel_ms, 3),
                         "algorithmic_bytes_per_launch": alg_bytes},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

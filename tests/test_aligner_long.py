"""GPU parity of the aligners past round 2's length limits (queries over
16,384 bases for Hirschberg-Myers, over 8,192 for full and banded Myers,
targets over 65,535): the long-mode kernels (query patterns in HBM, striped
Myers sweeps, target codes in HBM past 131,072 bases, banded chunk state in
HBM for bands wider than LDS) against the aligner oracle and the golden
vectors of tests/golden/aligner_long.json (the reference's own benchmark
recipes, cudaaligner/benchmarks/main.cpp:33-60, :85-124).  The reference has
no length limit (aligner_global_hirschberg_myers.cpp:47-51)."""
import hashlib
import json
import os
import random

import pytest

from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch
from oracle import oracle

pytestmark = pytest.mark.gpu

LONG = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aligner_long.json")))
OALGO = {"hirschberg_myers": oracle.ALIGN_HM, "myers": oracle.ALIGN_MYERS, "myers_banded": oracle.ALIGN_MYERS_BANDED}


def gpu_states(pairs, algorithm, max_q=None, max_t=None, stats=None):
    mq = max_q or max(len(q) for q, _ in pairs)
    mt = max_t or max(len(t) for _, t in pairs)
    b = CudaAlignerBatch(mq, mt, len(pairs), algorithm=algorithm)
    for q, t in pairs:
        assert b.add_alignment(q, t) == 0
    b.align_all()
    b.sync_alignments()
    paths, plen = b.raw_paths()
    if stats is not None:
        stats.update(b.stats())
    return [paths[i, :plen[i]][::-1].tolist() for i in range(len(pairs))], mq


def mutate(rng, s, err):
    q = list(s)
    for _ in range(int(len(s) * err)):
        k, p = rng.randrange(3), rng.randrange(len(q) + 1)
        if k == 0 and p < len(q):
            q[p] = rng.choice("ACGT")
        elif k == 1:
            q.insert(p, rng.choice("ACGT"))
        elif p < len(q):
            del q[p]
    return "".join(q)


def rand_seq(rng, n):
    return "".join(rng.choice("ACGT") for _ in range(n))


@pytest.mark.parametrize("stripe_blocks", ["1", "2"])
def test_hm_striped_sweeps_on_short_pairs(stripe_blocks, monkeypatch):
    # GWAMD_HM_STRIPE_BLOCKS forces the long-mode kernel with stripes of 1 or 2
    # blocks (2,048 / 4,096 rows), so 300 bp - 6 kb pairs cross several stripes
    monkeypatch.setenv("GWAMD_HM_STRIPE_BLOCKS", stripe_blocks)
    rng = random.Random(11 + int(stripe_blocks))
    pairs = []
    for n in (300, 2100, 4500, 6000, 9000):
        t = rand_seq(rng, n)
        pairs.append((mutate(rng, t, 0.1), t))
    pairs.append(("A" * 5000, "C" * 4000))  # no match at all
    got, mq = gpu_states(pairs, "hirschberg_myers")
    for (q, t), g in zip(pairs, got):
        assert g == oracle.align(q, t, oracle.ALIGN_HM, mq), (len(q), len(t))


def test_hm_long_pairs_match_oracle():
    rng = random.Random(21)
    t1 = rand_seq(rng, 20000)
    t2 = rand_seq(rng, 5000)
    t3 = rand_seq(rng, 70000)
    pairs = [(mutate(rng, t1, 0.1), t1),             # query > 16,384
             (mutate(rng, t2, 0.02) + rand_seq(rng, 13000), t2),  # tall query, short target
             (mutate(rng, t3[:30000], 0.05), t3)]     # target > 65,535
    got, mq = gpu_states(pairs, "hirschberg_myers")
    for (q, t), g in zip(pairs, got):
        assert g == oracle.align(q, t, oracle.ALIGN_HM, mq), (len(q), len(t))


@pytest.mark.parametrize("algo", ["myers", "myers_banded"])
def test_myers_long_pairs_match_oracle(algo):
    rng = random.Random(31)
    t1 = rand_seq(rng, 20000)
    t2 = rand_seq(rng, 9000)
    pairs = [(mutate(rng, t1, 0.1), t1), (mutate(rng, t2, 0.03), t2[:3000])]
    got, mq = gpu_states(pairs, algo)
    for (q, t), g in zip(pairs, got):
        assert g == oracle.align(q, t, OALGO[algo], mq), (len(q), len(t))


def test_myers_banded_chunk_state_in_hbm(monkeypatch):
    # a 4 KiB LDS region holds 256 band words; dissimilar 12 kb sequences
    # double the band to the whole query (375 words), so the chunk state of
    # the sweep goes through HBM (the path long queries take when the band
    # outgrows LDS)
    monkeypatch.setenv("GWAMD_BAND_TILE_BYTES", "4096")
    rng = random.Random(41)
    t = rand_seq(rng, 12000)
    pairs = [(mutate(rng, t, 0.45), t), (rand_seq(rng, 11000), t)]
    st = {}
    got, mq = gpu_states(pairs, "myers_banded", stats=st)
    # the sweeps really took the HBM chunk state (not the LDS path)
    assert st["hbm_state_sweeps"] >= len(pairs)
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_MYERS_BANDED, mq)


@pytest.mark.parametrize("waves", ["1", "4", "8", "16"])
def test_myers_banded_two_column_sweep(waves, monkeypatch):
    # bands of several 32-word chunks with their state in LDS run two target
    # columns per wave (one per half wave, each column two chunks behind the
    # previous one; 4 or 8 waves per pair: 8 or 16 columns in flight): target
    # lengths that leave partial last groups, stripes and diagonal bands, up
    # to the whole query (375 words, 12 chunks)
    monkeypatch.setenv("GWAMD_BAND_WAVES", waves)
    rng = random.Random(43)
    t = rand_seq(rng, 12000)
    pairs = [(mutate(rng, t, 0.45), t), (rand_seq(rng, 11000), t[:11001]),
             (mutate(rng, t[:9001], 0.2), t[:9001]), (mutate(rng, t, 0.12), t[:11500])]
    st = {}
    got, mq = gpu_states(pairs, "myers_banded", stats=st)
    assert st["hbm_state_sweeps"] == 0
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_MYERS_BANDED, mq), (len(q), len(tt))


@pytest.mark.parametrize("spec", ["0", "1", "2", "3", "8"])
@pytest.mark.parametrize("waves", ["4", "8"])
def test_myers_banded_run_ahead_sweeps(spec, waves, monkeypatch):
    # band doubling run ahead (few long pairs): launch 1 runs sweeps
    # 0..spec-1 of every pair on their own workgroups (distance only, the last
    # one with its band matrix), launch 2 skips the rejected ones and the
    # stored one and carries on doubling past them. Pairs needing 1 to 5
    # sweeps, and one whose band reaches the whole query early
    monkeypatch.setenv("GWAMD_BAND_SPEC", spec)
    monkeypatch.setenv("GWAMD_BAND_WAVES", waves)
    rng = random.Random(47)
    t = rand_seq(rng, 12000)
    pairs = [(mutate(rng, t, 0.02), t), (mutate(rng, t, 0.12), t[:11500]), (mutate(rng, t, 0.3), t),
             (mutate(rng, t[:9001], 0.2), t[:9001]), (rand_seq(rng, 11000), t[:11001]),
             (mutate(rng, t[:2500], 0.1), t[:2400])]
    got, mq = gpu_states(pairs, "myers_banded")
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_MYERS_BANDED, mq), (spec, len(q), len(tt))


def test_band_spec_checked(monkeypatch):
    monkeypatch.setenv("GWAMD_BAND_SPEC", "9")
    b = CudaAlignerBatch(12000, 12000, 1, algorithm="myers_banded")
    assert b.add_alignment("ACGT" * 3000, "ACGT" * 3000) == 0
    with pytest.raises(ValueError):
        b.align_all()


def test_band_tile_bytes_checked(monkeypatch):
    monkeypatch.setenv("GWAMD_BAND_TILE_BYTES", "4k")
    with pytest.raises(ValueError):
        CudaAlignerBatch(1000, 1000, 1, algorithm="myers_banded")


def _reference_pair(c):
    e = c["size"] // 30
    muts, genomes = synth.pairs(1, 1, c["size"], c["size"] if c["truncate_target"] else c["size"] + e + 1, e, e, e)
    return genomes[0].decode(), muts[0].decode()


@pytest.mark.parametrize("c", LONG["cases"], ids=lambda c: "%s-%s" % (c["recipe"], c["algorithm"]))
def test_reference_benchmark_pairs_golden(c):
    q, t = _reference_pair(c)
    assert (len(q), len(t)) == (c["query_length"], c["target_length"])
    got, _ = gpu_states([(q, t)], c["algorithm"], c["max_query_length"], c["max_target_length"])
    p = got[0]
    assert len(p) == c["path_length"]
    assert [sum(1 for x in p if x == k) for k in range(4)] == c["counts"]
    assert hashlib.sha256(bytes(p)).hexdigest() == c["path_sha256"]


# Ukkonen bands wider than one wave (ukkonen_wide_kernel): the reference runs
# any band with up to 1,024 threads per pair (ukkonen_gpu.cu:213-293); pairs
# whose length differs by up to 10 % of the target at 12 kb and 18 kb need
# 700-1,000 band rows (1 row per thread), a 30 kb one 1,600 (2 rows); at 45 kb
# and 64 kb a ~9-10 % shorter query needs ~2,300 / ~3,300 rows, so each of the
# 1,024 threads holds 3 / 4 rows (64-row edge groups 32-63)
@pytest.mark.parametrize("T", [12000, 18000, 30000, 45000, 64000])
def test_ukkonen_wide_band_matches_oracle(T):
    rng = random.Random(T)
    t = rand_seq(rng, T)
    d = int(T * 0.1) - 3
    q1 = mutate(rng, t, 0.04)[: T - d]              # query shorter by ~10 %
    q2 = mutate(rng, t, 0.08)[: T - d // 2] + "ACGT"
    q3 = t + rand_seq(rng, min(d // 3, 65536 - T))  # query longer (swapped roles)
    pairs = [(q1, t), (q2, t), (q3, t)]
    st = {}
    got, mq = gpu_states(pairs, "ukkonen", max(len(q) for q, _ in pairs), T, stats=st)
    assert st["ukkonen_wide_pairs"] == len(pairs)
    if T >= 45000:
        assert st["ukkonen_max_rows_per_thread"] >= (3 if T < 60000 else 4)
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_UKKONEN, mq), (len(q), len(tt))


def test_ukkonen_narrow_batch_keeps_single_wave_kernel():
    # a 16 kb aligner (wide workspace) whose pairs all have narrow bands runs
    # the single-wave kernel (stats: no wide pairs), same paths as the oracle
    rng = random.Random(5)
    t = rand_seq(rng, 16000)
    pairs = [(mutate(rng, t, 0.05)[:15990], t), (t[:15900], t)]
    st = {}
    got, mq = gpu_states(pairs, "ukkonen", 16000, 16000, stats=st)
    assert st["ukkonen_wide_pairs"] == 0
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_UKKONEN, mq)


@pytest.mark.parametrize("tile", [None, "16384", "24576"])
def test_ukkonen_long_pairs_large_tile(tile, monkeypatch):
    # pairs of 32 kb and more take a backtrace tile of what the CU's LDS has
    # left (up to 48 KiB) filled by direct-to-LDS loads, and the walk decides
    # each 8 x 8 window's moves in parallel: narrow-band pairs of 3-40 kb
    # (single-wave kernel) against the oracle, with the default and two
    # forced tile sizes
    if tile:
        monkeypatch.setenv("GWAMD_UK_TILE_BYTES", tile)
    else:
        monkeypatch.delenv("GWAMD_UK_TILE_BYTES", raising=False)
    rng = random.Random(17)
    t = rand_seq(rng, 40000)
    pairs = [(mutate(rng, t, 0.04)[:39950], t), (t[:39800], t), (mutate(rng, t[:3000], 0.1), t[:3100]),
             (mutate(rng, t[:25000], 0.08), t[:25020]), (rand_seq(rng, 33000)[:32990], t[:33000])]
    pairs = [(q, tt) for q, tt in pairs if abs(len(q) - len(tt)) <= 500]
    st = {}
    got, mq = gpu_states(pairs, "ukkonen", 40000, 40000, stats=st)
    assert st["ukkonen_wide_pairs"] == 0
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_UKKONEN, mq), (len(q), len(tt))


def test_myers_banded_short_launch_on_long_aligner(monkeypatch):
    # an aligner planned for long queries (8 waves per pair) whose batch holds
    # only queries up to 8,192 bases runs that launch with one wave per pair
    # (ADVICE: band waves per launch); same paths as the oracle
    monkeypatch.delenv("GWAMD_BAND_WAVES", raising=False)
    rng = random.Random(53)
    t = rand_seq(rng, 8000)
    pairs = [(mutate(rng, t, 0.1), t), (mutate(rng, t[:5000], 0.2), t[:5000]), (mutate(rng, t[:300], 0.05), t[:320])]
    got, mq = gpu_states(pairs, "myers_banded", 12000, 12000)
    for (q, tt), g in zip(pairs, got):
        assert g == oracle.align(q, tt, oracle.ALIGN_MYERS_BANDED, mq), (len(q), len(tt))

"""GPU parity of the HIP global aligners (through the C ABI via
CudaAlignerBatch) against the aligner oracle and the reference's own KATs."""
import json
import os
import random

import pytest

from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aligner_kat.json")))
ALGOS = [("hirschberg_myers", oracle.ALIGN_HM), ("myers", oracle.ALIGN_MYERS),
         ("myers_banded", oracle.ALIGN_MYERS_BANDED), ("ukkonen", oracle.ALIGN_UKKONEN)]


def run(pairs, max_q=None, max_t=None, algorithm="hirschberg_myers", rc=None):
    mq = max_q if max_q is not None else max(1, max(len(q) for q, _ in pairs))
    mt = max_t if max_t is not None else max(1, max(len(t) for _, t in pairs))
    b = CudaAlignerBatch(mq, mt, len(pairs), algorithm=algorithm)
    for k, (q, t) in enumerate(pairs):
        flags = rc[k] if rc else (False, False)
        assert b.add_alignment(q, t, *flags) == 0
    b.align_all()
    return b, b.get_alignments()


def states(al):
    inv = {"m": 0, "mm": 1, "i": 2, "d": 3}
    return [inv[s] for s in al.alignment]


@pytest.mark.parametrize("case", GOLD["cigar"], ids=lambda c: c["source"])
@pytest.mark.parametrize("algo", ["hirschberg_myers", "myers", "myers_banded", "ukkonen"])
def test_cigar_kats(case, algo):
    if algo != "hirschberg_myers" and algo not in case["algorithms"]:
        pytest.skip("KAT not stated for this aligner")
    pairs = [(p["query"], p["target"]) for p in case["pairs"]]
    _, al = run(pairs, case["max_query_length"], case["max_target_length"], algo)
    assert [a.cigar for a in al] == [p["cigar"] for p in case["pairs"]]
    assert all(a.status == 0 and a.alignment_type == "global" for a in al)


def _rand_pairs(seed, n, lo, hi, err):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        t = "".join(rng.choice("ACGT") for _ in range(rng.randrange(lo, hi + 1)))
        q = list(t)
        for _ in range(int(len(t) * err)):
            k, p = rng.randrange(3), rng.randrange(len(q) + 1)
            if k == 0 and p < len(q):
                q[p] = rng.choice("ACGT")
            elif k == 1:
                q.insert(p, rng.choice("ACGT"))
            elif p < len(q):
                del q[p]
        out.append(("".join(q), t))
    return out


@pytest.mark.parametrize("algo,oalgo", ALGOS)
@pytest.mark.parametrize("lo,hi,err", [(1, 40, 0.2), (50, 200, 0.1), (300, 1200, 0.08), (2000, 4000, 0.05)])
def test_random_pairs_match_oracle(algo, oalgo, lo, hi, err):
    pairs = _rand_pairs(lo * 7 + hi, 24 if hi < 2000 else 6, lo, hi, err)
    mq = max(len(q) for q, _ in pairs)
    mt = max(len(t) for _, t in pairs)
    if algo == "ukkonen":  # |q - t| within 10% of max_target_length (aligner_global_ukkonen.cpp:47-57)
        pairs = [(q, t) for q, t in pairs if abs(len(q) - len(t)) <= int(mt * 0.1)]
    _, al = run(pairs, mq, mt, algo)
    for (q, t), a in zip(pairs, al):
        assert states(a) == oracle.align(q, t, oalgo, mq), (len(q), len(t))


def test_config_d_pairs_match_oracle():
    # SURVEY 8(d) config D shape: 5 kb target, ~10% difference (synthetic generator)
    pairs = synth.aligner_pairs(1, 4, 5000)
    _, al = run(pairs, 5000, 5000)
    for (q, t), a in zip(pairs, al):
        assert states(a) == oracle.align(q, t, oracle.ALIGN_HM, 5000)


def test_unrelated_long_pairs_optimal():
    # Test_AlignerGlobal.cpp:130-134 shape (random 4800 vs 5000, no CIGAR stated)
    rng = random.Random(11)
    pairs = [("".join(rng.choice("ACGT") for _ in range(4800)), "".join(rng.choice("ACGT") for _ in range(5000)))]
    _, al = run(pairs, 5001, 5001)
    q, t = pairs[0]
    st = states(al[0])
    assert st == oracle.align(q, t, oracle.ALIGN_HM, 5001)
    assert sum(1 for s in st if s != 0) == oracle.edit_distance(q, t)


@pytest.mark.parametrize("algo,oalgo", ALGOS)
def test_edge_cases(algo, oalgo):
    pairs = [("", "ACGT"), ("ACGT", ""), ("A", "T"), ("A", "TTTA"), ("G", "ACGTGT"), ("C", "C"),
             ("ACGNNT", "ACGGGT"), ("acgt", "ACGT"), ("NNNN", "ACGT"), ("ACGT" * 20, "TTTT"),
             ("T" * 70, "T" * 69 + "A"), ("", "")]
    if algo == "ukkonen":  # allowed length difference: int(80 * 0.1f) = 8
        pairs = [(q, t) for q, t in pairs if abs(len(q) - len(t)) <= 8]
    _, al = run(pairs, 80, 80, algo)
    for (q, t), a in zip(pairs, al):
        assert states(a) == oracle.align(q, t, oalgo, 80), (q, t)
        assert a.query == q and a.target == t


def test_wide_leaf_in_hbm():
    # a base case (query < 63) over a target segment wider than the LDS leaf
    # (512 columns): query 40 bases vs target 1500
    rng = random.Random(5)
    t = "".join(rng.choice("ACGT") for _ in range(1500))
    q = t[700:740]
    _, al = run([(q, t)], 5000, 5000)
    assert states(al[0]) == oracle.align(q, t, oracle.ALIGN_HM, 5000)


def test_reverse_complement_flags():
    def rc(s):
        return "".join({"A": "T", "T": "A", "C": "G", "G": "C"}.get(c, c) for c in reversed(s))
    pairs = _rand_pairs(3, 4, 100, 300, 0.1)
    flags = [(True, False), (False, True), (True, True), (False, False)]
    _, al = run(pairs, 400, 400, rc=flags)
    for (q, t), (fq, ft), a in zip(pairs, flags, al):
        qq, tt = (rc(q) if fq else q), (rc(t) if ft else t)
        assert a.query == qq and a.target == tt
        assert states(a) == oracle.align(qq, tt, oracle.ALIGN_HM, 400)


def test_add_alignment_status_codes():
    # Test_AlignerGlobal.cpp:58-83
    case = GOLD["add_alignment"]
    b = CudaAlignerBatch(case["max_query_length"], case["max_target_length"], case["max_alignments"])
    for q, t, want in case["calls"]:
        assert b.add_alignment(q, t) == want
    assert b.num_alignments() == case["final_count"]
    b.align_all()
    assert [a.cigar for a in b.get_alignments()] == [oracle.cigar(oracle.align("ATCG", "TACG", 0, 10))] * 5
    b.reset()
    assert b.get_alignments() == []


@pytest.mark.parametrize("max_len,max_n,seq_len,n,ok", [(1000, 100, 10000, 10, False), (1000, 100, 100, 10, True),
                                                        (100, 10, 100, 1000, False)])
def test_various_arguments(max_len, max_n, seq_len, n, ok):
    # test_cudaaligner_bindings.py:84-112
    rng = random.Random(seq_len)
    b = CudaAlignerBatch(max_len, max_len, max_n)
    good = True
    for _ in range(n):
        s = "".join(rng.choice("ACGT") for _ in range(seq_len))
        good &= b.add_alignment(s, s) == 0
    b.align_all()
    assert good is ok


def test_invalid_construction():
    with pytest.raises(RuntimeError):
        CudaAlignerBatch(10, 10, 0)
    with pytest.raises(RuntimeError):
        CudaAlignerBatch(10, 10, 1, alignment_type="local")
    with pytest.raises(ValueError):
        CudaAlignerBatch(10, 10, 1, max_device_memory_allocator_caching_size=-2)


# --- banded Myers / Ukkonen specifics ------------------------------------------

def test_banded_multichunk_and_band_growth():
    # unrelated strings: the band doubles past 1024 rows (several 32-word
    # chunks in the diagonal phase, myers_gpu.cu:597-611) up to the full query;
    # query longer and shorter than the target; Q % 32 == 0 full bands
    rng = random.Random(21)
    pairs = []
    for ql, tl in [(2500, 2600), (2700, 2600), (2048, 2000), (1024, 1100), (64, 64), (96, 130), (3000, 2990)]:
        pairs.append(("".join(rng.choice("ACGT") for _ in range(ql)), "".join(rng.choice("ACGT") for _ in range(tl))))
    _, al = run(pairs, 3000, 3000, "myers_banded")
    for (q, t), a in zip(pairs, al):
        assert states(a) == oracle.align(q, t, oracle.ALIGN_MYERS_BANDED), (len(q), len(t))


@pytest.mark.parametrize("algo,oalgo", [("myers_banded", oracle.ALIGN_MYERS_BANDED), ("ukkonen", oracle.ALIGN_UKKONEN)])
def test_banded_config_d_pairs(algo, oalgo):
    pairs = synth.aligner_pairs(1, 16, 5000)
    _, al = run(pairs, 5000, 5000, algo)
    for (q, t), a in zip(pairs, al):
        st = states(a)
        assert st == oracle.align(q, t, oalgo), (len(q), len(t))
        assert sum(1 for s in st if s != 0) == oracle.edit_distance(q, t)


def test_ukkonen_swapped_and_wide_difference():
    # query longer than target (the kernel swaps and relabels insertions and
    # deletions, ukkonen_gpu.cu:74-79) and length differences near the 10% cap
    rng = random.Random(8)
    pairs = []
    for ql, tl in [(1100, 1000), (1000, 1100), (900, 990), (1090, 1000), (1, 1), (60, 50), (0, 0)]:
        t = "".join(rng.choice("ACGT") for _ in range(tl))
        q = (t[: min(ql, tl)] + "".join(rng.choice("ACGT") for _ in range(max(0, ql - tl))))
        q = "".join(c if rng.random() > 0.05 else rng.choice("ACGT") for c in q)
        pairs.append((q, t))
    _, al = run(pairs, 1100, 1100, "ukkonen")
    for (q, t), a in zip(pairs, al):
        assert states(a) == oracle.align(q, t, oracle.ALIGN_UKKONEN), (len(q), len(t))


def test_ukkonen_add_alignment_status_codes():
    # Test_AlignerGlobal.cpp:58-83 on AlignerGlobalUkkonen(10, 10, 5)
    case = GOLD["add_alignment_ukkonen"]
    b = CudaAlignerBatch(case["max_query_length"], case["max_target_length"], case["max_alignments"],
                         algorithm="ukkonen")
    for q, t, want in case["calls"]:
        assert b.add_alignment(q, t) == want
    assert b.num_alignments() == case["final_count"]
    b.align_all()
    assert [a.cigar for a in b.get_alignments()] == [oracle.cigar(oracle.align("ATCG", "TACG", 3))] * 5


def test_caching_budget_caps_the_workspace():
    # max_device_memory_allocator_caching_size (aligner.hpp:103): the
    # reference serves the aligner's device buffers from a pool of that size;
    # here the workspace gets as many persistent-grid slots as the budget
    # holds after the fixed buffers, and a budget below one slot throws
    from oracle import oracle
    free = CudaAlignerBatch(5000, 5000, 64)
    grid_free, dev_free = free.config()
    slot = (dev_free - 2 * 5000 * 64 - 16 - 2 * 64 * 4 - 10000 * 64 - 16 - 64 * 4) // grid_free
    budget = dev_free - (grid_free - 3) * slot
    b = CudaAlignerBatch(5000, 5000, 64, max_device_memory_allocator_caching_size=budget)
    grid, dev = b.config()
    assert grid == 3 and dev <= budget
    rng = random.Random(3)
    pairs = [("".join(rng.choice("ACGT") for _ in range(rng.randint(1, 5000))),
              "".join(rng.choice("ACGT") for _ in range(rng.randint(1, 5000)))) for _ in range(20)]
    for q, t in pairs:
        assert b.add_alignment(q, t) == 0
    b.align_all()
    for (q, t), a in zip(pairs, b.get_alignments()):
        assert a.cigar == oracle.cigar(oracle.align(q, t, oracle.ALIGN_HM, 5000))
    with pytest.raises(RuntimeError):
        CudaAlignerBatch(5000, 5000, 64, max_device_memory_allocator_caching_size=1 << 20)


@pytest.mark.parametrize("algo", ["hirschberg_myers", "myers", "myers_banded", "ukkonen"])
def test_pipelined_align_all_matches_oracle(algo, monkeypatch):
    # align_all() on a batch of many grids' worth of pairs runs as a pipeline
    # of chunks (copy-in / copy-out streams, two compute streams with half the
    # workspace slots each; GWAMD_ALIGNER_GRID=1: one workgroup per CU, so
    # 1,500 pairs are enough); with 3 and 8 stages (uneven chunks, stages
    # sharing a slot half) every pair equals the oracle and the one-stage run
    # (GWAMD_ALIGNER_PIPELINE=1), and the kernel time is reported
    monkeypatch.setenv("GWAMD_DIAG", "1")
    monkeypatch.setenv("GWAMD_ALIGNER_GRID", "1")
    qs, ts = synth.pairs(77, 1500, 300, 330, 10, 10, 10)
    pairs = list(zip(qs, ts))
    res = {}
    for mode in ("1", "3", "8"):
        monkeypatch.setenv("GWAMD_ALIGNER_PIPELINE", mode)
        b = CudaAlignerBatch(max(len(q) for q in qs), max(len(t) for t in ts), len(pairs), algorithm=algo)
        for q, t in pairs:
            assert b.add_alignment(q, t) == 0
        grid, _ = b.config()
        assert len(pairs) >= 4 * grid
        b.align_all()
        b.sync_alignments()
        assert b.last_kernel_ms() > 0
        res[mode] = [states(a) for a in b.get_alignments()]
    assert res["3"] == res["1"] and res["8"] == res["1"]
    want, _ = oracle.align_batch(pairs, dict(ALGOS)[algo], max(len(q) for q in qs))
    assert res["1"] == want


def test_split_launch_after_pipelined_align_all(monkeypatch):
    # a batch whose last align_all() ran pipelined, then driven
    # through the split C ABI entry points (upload / launch / download) with
    # the same pair count and no manual synchronize: sync_alignments must wait
    # for this launch's download (not the old stages' events) and
    # last_kernel_ms must time this launch
    monkeypatch.setenv("GWAMD_DIAG", "1")
    monkeypatch.setenv("GWAMD_ALIGNER_GRID", "1")
    monkeypatch.setenv("GWAMD_ALIGNER_PIPELINE", "4")
    qs, ts = synth.pairs(91, 1500, 300, 330, 10, 10, 10)
    pairs = list(zip(qs, ts))
    b = CudaAlignerBatch(max(len(q) for q in qs), max(len(t) for t in ts), len(pairs), algorithm="myers")
    for q, t in pairs:
        assert b.add_alignment(q, t) == 0
    b.align_all()
    b.sync_alignments()
    first = [states(a) for a in b.get_alignments()]
    # clear the aligner's host result buffers so stale results cannot pass
    import ctypes as C
    pp, ln, stride = C.c_void_p(), C.c_void_p(), C.c_int32()
    b._lib.gwamd_aligner_get_paths(b._handle, C.byref(pp), C.byref(ln), C.byref(stride))
    C.memset(pp, 0, len(pairs) * stride.value)
    C.memset(ln, 0, len(pairs) * 4)
    b.upload()
    b.launch()
    b.download()
    b.sync_alignments()
    assert b.last_kernel_ms() > 0
    assert [states(a) for a in b.get_alignments()] == first
    want, _ = oracle.align_batch(pairs, oracle.ALIGN_MYERS, max(len(q) for q in qs))
    assert first == want


def test_shared_allocator_pool_caps_aligners():
    # create_default_device_allocator() is a 2 GiB pool
    # (allocator.hpp:297-305) and copies of one allocator share it
    # (shared_ptr<MemoryResource>, allocator.hpp:274-279): two aligners made
    # from one 1 GiB allocator cannot jointly exceed it; the bytes come back
    # when an aligner is destroyed
    import gc
    from claragenomicsanalysis_amd.cudaaligner import DeviceAllocator
    assert DeviceAllocator().capacity == 2 << 30
    pool = DeviceAllocator(1 << 30)
    # 4,000 pairs x 5 kb on all resident slots would take several GiB
    a1 = CudaAlignerBatch(5000, 5000, 4000, allocator=pool)
    grid1, dev1 = a1.config()
    assert 0 < pool.used <= pool.capacity
    assert pool.used == dev1
    try:
        a2 = CudaAlignerBatch(5000, 5000, 4000, allocator=pool)
        grid2, dev2 = a2.config()
        assert pool.used == dev1 + dev2 <= pool.capacity
        del a2
    except RuntimeError:
        pass  # nothing left for the fixed buffers plus one slot
    assert pool.used == dev1
    # the first aligner still aligns correctly on its capped slots
    qs, ts = synth.pairs(5, 40, 5000, 5000, 166, 166, 166)
    for q, t in zip(qs, ts):
        assert a1.add_alignment(q, t) == 0
    a1.align_all()
    a1.sync_alignments()
    want, _ = oracle.align_batch(list(zip(qs, ts)), oracle.ALIGN_HM, 5000)
    assert [states(a) for a in a1.get_alignments()] == want
    del a1
    gc.collect()
    assert pool.used == 0
    # a pool too small for the fixed buffers plus one slot throws
    with pytest.raises(RuntimeError):
        CudaAlignerBatch(5000, 5000, 4000, allocator=DeviceAllocator(1 << 20))

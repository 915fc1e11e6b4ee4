"""GPU parity tests of the level-keyed Kahn sort (topsort_levels in
csrc/poa_wave.hpp, round 6) against the reference's FIFO order
(cudapoa_topsort.cuh:56-85, restated in oracle/poa_oracle.cpp topsort_fast):
the reference's three topological-sort KATs (tests/golden/poa_kat.json, from
Test_CudapoaTopSort.cu), random DAGs through the C-ABI test hook, and whole
windows run with the level sort and with the FIFO sort (GWAMD_TOPSORT=fifo)."""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest

from claragenomicsanalysis_amd import load_library, synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_kat.json")))
MAX_EDGES = 50


def _hook():
    L = load_library()
    f = L.gwamd_internal_topsort_levels
    f.restype = C.c_int
    f.argtypes = [C.c_int] * 4 + [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_void_p]
    return f


def level_sort(outgoing, size_bits=16, threads=128, scratch=64 << 10, hint=None, n_hint=0, want_hint=False,
               prev=None):
    """The device sort of one graph (critical-predecessor hints for the first
    n_hint nodes and the previous order `prev` of the first len(prev) nodes,
    as the kernels keep them between reads; default: the nodes in id order)."""
    n = len(outgoing)
    in_cnt, in_e, out_cnt, out_e = oracle.edges_from_lists(outgoing, n)
    in_e = np.ascontiguousarray(in_e, np.int32)
    out_e = np.ascontiguousarray(out_e, np.int32)
    hi = np.ascontiguousarray(np.arange(n) if hint is None else hint, np.int32)
    order = np.ascontiguousarray(np.arange(n) if prev is None else prev, np.int32)
    res = np.zeros(n, np.int32)
    rc = _hook()(size_bits, n, len(order), n_hint, in_cnt.ctypes.data, in_e.ctypes.data, out_cnt.ctypes.data,
                 out_e.ctypes.data, hi.ctypes.data, order.ctypes.data, threads, scratch, res.ctypes.data)
    if want_hint:
        return rc, res.tolist(), hi.tolist()
    return rc, res.tolist()


@pytest.mark.parametrize("threads", [64, 128, 256])
@pytest.mark.parametrize("case", GOLD["topsort"], ids=lambda c: str(c["answer"]))
def test_topsort_levels_kat(case, threads):
    rc, got = level_sort(case["outgoing"], threads=threads)
    assert rc == 1
    assert got == case["answer"]


def random_dag(rng, n, p_edge, max_out=8, sources=1):
    """A DAG over a random relabelling of 0..n-1: edges go forward in a hidden
    order; out-lists in random slot order (the FIFO order depends on slots)."""
    perm = list(range(n))
    rng.shuffle(perm)
    out = [[] for _ in range(n)]
    indeg = [0] * n
    for i in range(sources, n):
        # at least one predecessor, mostly nearby in the hidden order (POA-like chains)
        k = 1 + (1 if rng.random() < p_edge else 0) + (1 if rng.random() < p_edge / 3 else 0)
        preds = set()
        for _ in range(k):
            j = i - 1 - min(int(rng.expovariate(0.5)), i - 1) if rng.random() < 0.9 else rng.randrange(i)
            preds.add(j)
        for j in preds:
            u, v = perm[j], perm[i]
            if len(out[u]) < max_out and indeg[v] < MAX_EDGES - 1:
                out[u].append(v)
                indeg[v] += 1
    for u in range(n):
        rng.shuffle(out[u])
    return out


@pytest.mark.parametrize("size_bits", [16, 32])
def test_topsort_levels_random_dags(size_bits):
    rng = random.Random(11 + size_bits)
    cases = 0
    for t in range(160):
        n = rng.choice([2, 3, 5, 17, 64, 65, 200, 1000, 3000])
        dag = random_dag(rng, n, rng.choice([0.1, 0.4, 0.8]), sources=rng.choice([1, 1, 2, 5]))
        want = oracle.topsort(dag)
        # hints for a prefix: a random predecessor of each node (the kernels
        # keep the previous read's critical predecessor; any predecessor is a
        # valid first guess), or the node itself (a former source)
        preds = [[] for _ in range(n)]
        for u in range(n):
            for v in dag[u]:
                preds[v].append(u)
        n_hint = rng.randrange(n + 1)
        hint = [rng.choice(preds[v]) if preds[v] and rng.random() < 0.9 else v for v in range(n)]
        # previous order: the FIFO order of the nodes below a random count (a
        # subgraph's sort, as after the previous read), or a random permutation
        n_prev = rng.randrange(1, n + 1)
        if rng.random() < 0.5:
            prev = [v for v in want if v < n_prev]
        else:
            prev = list(range(n_prev))
            rng.shuffle(prev)
        rc, got, c = level_sort(dag, size_bits=size_bits, threads=rng.choice([64, 128, 256]), hint=hint,
                                n_hint=n_hint, want_hint=True, prev=prev)
        assert rc == 1, (t, n)
        assert got == want, (t, n)
        # the returned critical predecessors are deepest predecessors, and a
        # second sort started from them gives the same order
        level = {}
        for v in want:
            level[v] = 1 + max((level[p] for p in preds[v]), default=-1)
        assert all(c[v] == v if not preds[v] else (c[v] in preds[v] and level[c[v]] == level[v] - 1)
                   for v in range(n)), (t, n)
        rc2, got2 = level_sort(dag, size_bits=size_bits, hint=c, n_hint=n)
        assert rc2 == 1 and got2 == want, (t, n)
        cases += 1
    assert cases == 160


def test_topsort_levels_wide_levels_and_sources():
    # many sources (level 0 ordered by id) and wide levels (ranks by parent and slot)
    rng = random.Random(3)
    for t in range(20):
        n = 400
        dag = random_dag(rng, n, 0.9, max_out=20, sources=rng.choice([30, 100]))
        want = oracle.topsort(dag)
        rc, got = level_sort(dag, threads=256)
        assert rc == 1 and got == want, t


def test_topsort_levels_declines_when_scratch_too_small():
    dag = [[i + 1] for i in range(999)] + [[]]
    rc, _ = level_sort(dag, scratch=1024)
    assert rc == 0
    rc, got = level_sort(dag, scratch=16 << 10)
    assert rc == 1 and got == list(range(1000))


def _run(wins, max_seq, max_seqs, banded, out):
    b = CudaPoaBatch(max_seqs, max_seq, 8 << 30, output_type=out, cuda_banded_alignment=banded,
                     alignment_band_width=256)
    for w in wins:
        st, _ = b.add_poa_group(list(w))
        assert st == 0
    b.generate_poa()
    return b


@pytest.mark.parametrize("mode", ["full", "full_msa", "banded", "banded_ad_msa"])
def test_topsort_levels_windows_match_fifo(mode, monkeypatch):
    # every read's sort feeds the next read's rows (banded: the band start of
    # every row is a function of its position), so equal outputs and equal
    # graphs over whole windows pin the order read by read
    banded = mode.startswith("banded")
    msa = mode.endswith("msa")
    if mode == "banded_ad_msa":
        monkeypatch.setenv("GWAMD_BAND_FWD", "ad")
        wins = synth.poa_windows(41, 4, 1500, 8, 75, 75, 75)
        max_seq = 1700
    else:
        wins = synth.poa_windows(29, 6, 600, 20, 30, 30, 30)
        max_seq = 700
    out = "msa" if msa else "consensus"
    res = {}
    for sort in ("levels", "fifo"):
        if sort == "fifo":
            monkeypatch.setenv("GWAMD_TOPSORT", "fifo")
        else:
            monkeypatch.delenv("GWAMD_TOPSORT", raising=False)
        b = _run(wins, max_seq, 20, banded, out)
        res[sort] = (b.get_msa() if msa else b.get_consensus(), b.get_graphs())
        sbits = b.get_types()[0]
    monkeypatch.delenv("GWAMD_TOPSORT", raising=False)
    assert res["levels"][0] == res["fifo"][0]
    ga, gb = res["levels"][1][0], res["fifo"][1][0]
    assert [[(e, g.weight(*e)) for e in g.edges] for g in ga] == [[(e, g.weight(*e)) for e in g.edges] for g in gb]
    for i, w in enumerate(wins):
        mn = ((4 if banded else 3) * max_seq + 3) // 4 * 4
        r = oracle.poa_window(w, banded=banded, band_width=256, msa=msa, score_bits=sbits, max_nodes=mn,
                              max_consensus=2 * max_seq, max_seqs=20)
        if msa:
            got, st = res["levels"][0]
            assert (st[i], got[i]) == (r.status, r.msa), i
        else:
            cons, cov, st = res["levels"][0]
            assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i

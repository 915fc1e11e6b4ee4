"""GPU parity tests of the racon DFS sort used by the MSA output and by
SPOA_ACCURATE batches (topsort_racon_lds / racon_dfs_csr in csrc/poa_wave.hpp)
against the reference's raconTopologicalSortDeviceUtil
(cudapoa_topsort.cuh:94-189, restated in oracle/poa_oracle.cpp topsort_racon),
through the C-ABI test hook: the order, the MSA column of every node
(getNodeIDToMSAPosDevice, cudapoa_generate_msa.cuh:27-45) and the column count,
on final window graphs of the bench shapes (B, C) and of small windows, on
column-structured graphs with large aligned groups and more than 64 list
entries per node, for the round-6 DFS and the round-5 step (v1)."""
import ctypes as C
import random

import numpy as np
import pytest

from claragenomicsanalysis_amd import load_library, synth
from oracle import oracle

pytestmark = pytest.mark.gpu

MAX_EDGES = oracle.MAX_EDGES
MAX_ALN = oracle.MAX_ALIGNMENTS
LDS = 163520  # the band kernel's output scratch at config C


def _hook():
    f = load_library().gwamd_internal_topsort_racon
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int] + [C.c_void_p] * 4 + [C.c_int, C.c_int] + [C.c_void_p] * 3 + [C.c_int,
                                                                                                    C.c_void_p]
    return f


def device_racon(n, ic, ie, ac, al, size_bits=16, scratch=LDS, v1=False, reps=0):
    ic = np.ascontiguousarray(ic, np.uint16)
    ac = np.ascontiguousarray(ac, np.uint16)
    ie = np.ascontiguousarray(ie, np.int32)
    al = np.ascontiguousarray(al, np.int32)
    order = np.zeros(n, np.int32)
    mpos = np.zeros(n, np.int32)
    cols = C.c_int(0)
    ms = C.c_double(0)
    rc = _hook()(size_bits, n, ic.ctypes.data, ie.ctypes.data, ac.ctypes.data, al.ctypes.data, scratch, int(v1),
                 order.ctypes.data, mpos.ctypes.data, C.byref(cols), reps, C.byref(ms))
    return rc, order.tolist(), mpos.tolist(), cols.value, ms.value


def check(graph, size_bits=16, scratch=LDS, v1=False):
    n, ic, ie, ac, al = graph
    ok, want, want_pos, want_cols = oracle.topsort_racon(n, ic, ie, ac, al)
    assert ok
    rc, got, got_pos, cols, _ = device_racon(n, ic, ie, ac, al, size_bits, scratch, v1)
    assert rc == 1
    assert got == want
    assert got_pos == want_pos
    assert cols == want_cols


def window_graph(win, banded=False, score_bits=16, max_nodes=None):
    st, n, ic, ie, ac, al = oracle.poa_window_graph(win, banded=banded, band_width=256, score_bits=score_bits,
                                                    max_nodes=max_nodes)
    assert st == 0
    return n, ic, ie, ac, al


@pytest.fixture(scope="module")
def graph_b():
    return window_graph(synth.poa_windows(1, 1, 1000, 32, 50, 50, 50)[0])


@pytest.fixture(scope="module")
def graph_c():
    win = synth.poa_windows(1, 1, 10000, 16, 500, 500, 500)[0]
    return window_graph(win, banded=True, score_bits=32, max_nodes=40000)


@pytest.mark.parametrize("v1", [False, True], ids=["dfs", "v1"])
def test_racon_window_b(graph_b, v1):
    check(graph_b, v1=v1)


@pytest.mark.parametrize("size_bits", [16, 32])
def test_racon_window_c(graph_c, size_bits):
    check(graph_c, size_bits=size_bits)


def test_racon_small_windows():
    for seed in range(12):
        for win in synth.poa_windows(100 + seed, 2, 120 + 40 * seed, 4 + seed, 6, 6, 6):
            g = window_graph(win)
            check(g)
            check(g, size_bits=32)


def column_graph(rng, ncols, max_group, max_in, span=4, min_group=1):
    """Nodes in columns; edges only from a column to the next `span` ones;
    every column's nodes are mutually aligned (symmetric lists, shuffled),
    ids shuffled so that the outer id loop starts DFSs all over the graph."""
    cols = [list(range(rng.randint(min_group, max_group))) for _ in range(ncols)]
    ids = list(range(sum(len(c) for c in cols)))
    rng.shuffle(ids)
    it = iter(ids)
    cols = [[next(it) for _ in c] for c in cols]
    n = len(ids)
    ins = [[] for _ in range(n)]
    for ci in range(1, ncols):
        for v in cols[ci]:
            cand = [u for cj in range(max(0, ci - span), ci) for u in cols[cj]]
            k = rng.randint(min(max_in, len(cand)) // 2 if min_group > 1 else 1, min(max_in, len(cand)))
            ins[v] = rng.sample(cand, k)
    ic = np.zeros(n, np.uint16)
    ie = np.zeros(n * MAX_EDGES, np.int32)
    ac = np.zeros(n, np.uint16)
    al = np.zeros(n * MAX_ALN, np.int32)
    for v in range(n):
        ic[v] = len(ins[v])
        ie[v * MAX_EDGES:v * MAX_EDGES + len(ins[v])] = ins[v]
    for c in cols:
        for v in c:
            others = [u for u in c if u != v]
            rng.shuffle(others)
            ac[v] = len(others)
            al[v * MAX_ALN:v * MAX_ALN + len(others)] = others
    return n, ic, ie, ac, al


def test_racon_column_graphs():
    rng = random.Random(7)
    for t in range(40):
        g = column_graph(rng, rng.randint(2, 60), rng.randint(1, 6), rng.randint(1, 6))
        check(g)


def test_racon_more_than_64_list_entries():
    # columns of up to 30 aligned nodes with up to 45 predecessors each: list
    # lengths past one wave (the DFS reads a second batch of entries)
    rng = random.Random(11)
    for t in range(6):
        g = column_graph(rng, 12, 31, 45, span=3, min_group=20)
        assert int((g[1].astype(int) + g[3].astype(int)).max()) > 64
        check(g)
        check(g, v1=True)


def test_racon_declines_when_scratch_too_small(graph_b):
    n, ic, ie, ac, al = graph_b
    rc, _, _, _, _ = device_racon(n, ic, ie, ac, al, scratch=n + 64)
    assert rc == 0

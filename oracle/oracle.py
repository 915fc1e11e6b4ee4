"""TEST INFRASTRUCTURE — ctypes wrapper over oracle/build/liboracle.so, the CPU
restatement of the reference algorithms (see poa_oracle.cpp / aligner_oracle.cpp
headers).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module; the product path never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
MAX_EDGES = 50
MAX_ALIGNMENTS = 50

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _p(arr):
    return arr.ctypes.data_as(C.c_void_p) if arr is not None else None


def _declare(L):
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.oracle_poa_window.restype = C.c_int
    L.oracle_poa_window.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                                    vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.oracle_poa_batch.restype = C.c_int
    L.oracle_poa_batch.argtypes = [vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32, i32,
                                   vp, vp, vp, vp, vp, i32, vp]
    L.oracle_set_spoa_accurate.restype = None
    L.oracle_set_spoa_accurate.argtypes = [C.c_int32]
    L.oracle_topsort.restype = None
    L.oracle_topsort.argtypes = [i32, vp, vp, vp, vp]
    L.oracle_poa_window_graph.restype = C.c_int
    L.oracle_poa_window_graph.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, i32, i32, i32, i32, vp, vp, vp, vp, vp]
    L.oracle_topsort_racon.restype = C.c_int
    L.oracle_topsort_racon.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp]
    L.oracle_nw.restype = C.c_int
    L.oracle_nw.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, vp, vp]
    L.oracle_add_alignment.restype = C.c_int
    L.oracle_add_alignment.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp]
    L.oracle_consensus_raw.restype = C.c_int
    L.oracle_consensus_raw.argtypes = [i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i32, vp, vp]
    L.oracle_align.restype = C.c_int
    L.oracle_align.argtypes = [i32, C.c_char_p, i32, C.c_char_p, i32, i32, vp, i32]
    L.oracle_align_batch.restype = C.c_int
    L.oracle_align_batch.argtypes = [i32, i32, vp, vp, vp, i32, vp, vp, i32, i32]
    L.oracle_edit_distance.restype = C.c_int
    L.oracle_edit_distance.argtypes = [C.c_char_p, i32, C.c_char_p, i32]
    L.oracle_query_pattern.restype = C.c_uint32
    L.oracle_myers_banded.restype = C.c_int
    L.oracle_myers_banded.argtypes = [C.c_char_p, i32, C.c_char_p, i32, vp, vp, vp]
    L.oracle_ukkonen.restype = C.c_int
    L.oracle_ukkonen.argtypes = [C.c_char_p, i32, C.c_char_p, i32, i32, vp]
    L.oracle_query_pattern.argtypes = [C.c_char_p, i32, C.c_char, i32, i32]


class WindowResult:
    def __init__(self, status, consensus, coverage, msa, cells, band_cells, final_nodes, graph):
        self.status = status
        self.consensus = consensus
        self.coverage = coverage
        self.msa = msa
        self.cells = cells
        self.band_cells = band_cells
        self.final_nodes = final_nodes
        self.graph = graph


def poa_window(reads, weights=None, gap=-8, mismatch=-6, match=8, banded=False, band_width=256,
               score_bits=16, msa=False, max_nodes=None, max_consensus=None, max_seqs=None,
               want_graph=False, spoa_accurate=False):
    """Run one window through the restatement; reads are bytes/str.  spoa_accurate:
    racon DFS sort after every read (cudapoa_kernels.cuh:324-337)."""
    reads = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
    max_len = max([len(r) for r in reads] + [1])
    if max_nodes is None:
        max_nodes = ((3 * max_len + 3) // 4) * 4 if not banded else ((4 * max_len + 3) // 4) * 4
    if max_consensus is None:
        max_consensus = 2 * max_len
    if max_seqs is None:
        max_seqs = len(reads)
    # the banded DP reads up to a band width past a read's end (values that
    # never reach an output, cudapoa_nw_banded.cuh:123-173): pad accordingly
    seqs = np.frombuffer(b"".join(reads) + b"\0" * (2 * band_width + 64), dtype=np.uint8).copy()
    lens = np.array([len(r) for r in reads], dtype=np.int32)
    if weights is None:
        wts = np.ones(max(len(seqs), 1), dtype=np.int8)
    else:
        wts = np.concatenate([np.asarray(w, dtype=np.int8) for w in weights] + [np.zeros(16, np.int8)])
    cons = np.zeros(max_consensus + 1, dtype=np.uint8)
    cov = np.zeros(max_consensus + 1, dtype=np.uint16)
    clen = np.zeros(1, dtype=np.int32)
    msa_buf = np.zeros(max(len(reads), 1) * max_consensus, dtype=np.uint8) if msa else None
    cells = np.zeros(2, dtype=np.int64)
    fnodes = np.zeros(1, dtype=np.int32)
    gb = gc = ge = gw = None
    if want_graph:
        gb = np.zeros(max_nodes, dtype=np.uint8)
        gc = np.zeros(max_nodes, dtype=np.int32)
        ge = np.zeros(max_nodes * MAX_EDGES, dtype=np.int32)
        gw = np.zeros(max_nodes * MAX_EDGES, dtype=np.int32)
    lib().oracle_set_spoa_accurate(int(bool(spoa_accurate)))
    try:
        st = lib().oracle_poa_window(_p(seqs), _p(lens), _p(wts), len(reads), gap, mismatch, match, int(banded),
                                     band_width, score_bits, int(msa), max_nodes, max_consensus, max_seqs,
                                     _p(cons), _p(cov), _p(clen), _p(msa_buf), _p(cells), _p(fnodes),
                                     _p(gb), _p(gc), _p(ge), _p(gw))
    finally:
        lib().oracle_set_spoa_accurate(0)
    n = int(clen[0])
    # latin-1: lossless for any byte (windows may hold non-ASCII bases); ASCII as before
    consensus = bytes(cons[:n]).decode("latin-1") if st == 0 and not msa else ""
    coverage = cov[:n].tolist() if st == 0 and not msa else []
    rows = None
    if msa and st == 0:
        rows = []
        for s in range(len(reads)):
            row = bytes(msa_buf[s * max_consensus:(s + 1) * max_consensus])
            rows.append(row.split(b"\0", 1)[0].decode("latin-1"))
    graph = None
    if want_graph:
        nn = int(fnodes[0])
        graph = {"bases": bytes(gb[:nn]).decode(errors="replace"),
                 "in": [[(int(ge[v * MAX_EDGES + e]), int(gw[v * MAX_EDGES + e])) for e in range(int(gc[v]))]
                        for v in range(nn)]}
    return WindowResult(st, consensus, coverage, rows, int(cells[0]), int(cells[1]), int(fnodes[0]), graph)


def poa_batch(windows, nthreads=0, gap=-8, mismatch=-6, match=8, banded=False, band_width=256, score_bits=16,
              max_nodes=None, max_consensus=None, max_seqs=None, msa=False, spoa_accurate=False, coverage=False):
    """Run many windows (list of lists of bytes) on all host cores (OpenMP).
    Returns (consensus list, status array, cells array, threads used); with
    msa=True the first element is the list of MSA row lists instead; with
    coverage=True (consensus only) the coverage lists are returned after the
    status array: (consensus, status, coverage, cells, threads)."""
    flat = []
    lens = []
    first = []
    nseq = []
    for w in windows:
        first.append(len(lens))
        nseq.append(len(w))
        for r in w:
            r = r.encode() if isinstance(r, str) else bytes(r)
            flat.append(r)
            lens.append(len(r))
    max_len = max(lens + [1])
    if max_nodes is None:
        max_nodes = ((3 * max_len + 3) // 4) * 4
    if max_consensus is None:
        max_consensus = 2 * max_len
    if max_seqs is None:
        max_seqs = max(nseq + [1])
    seqs = np.frombuffer(b"".join(flat) + b"\0" * (2 * band_width + 64), dtype=np.uint8).copy()
    lens_a = np.array(lens, dtype=np.int32)
    offs = np.zeros(len(lens), dtype=np.int64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(lens_a[:-1])
    first_a = np.array(first, dtype=np.int32)
    nseq_a = np.array(nseq, dtype=np.int32)
    nw = len(windows)
    cons = np.zeros(nw * max_consensus, dtype=np.uint8)
    cov = np.zeros(nw * max_consensus, dtype=np.uint16)
    clen = np.zeros(nw, dtype=np.int32)
    status = np.zeros(nw, dtype=np.uint8)
    cells = np.zeros(nw, dtype=np.int64)
    msa_buf = np.zeros(nw * max_seqs * max_consensus, dtype=np.uint8) if msa else None
    lib().oracle_set_spoa_accurate(int(bool(spoa_accurate)))
    try:
        used = lib().oracle_poa_batch(_p(seqs), _p(offs), _p(lens_a), _p(first_a), _p(nseq_a), nw, gap, mismatch,
                                      match, int(banded), band_width, score_bits, max_nodes, max_consensus,
                                      max_seqs, nthreads, _p(cons), _p(cov), _p(clen), _p(status), _p(cells),
                                      int(msa), _p(msa_buf))
    finally:
        lib().oracle_set_spoa_accurate(0)
    if msa:
        rows = []
        for i in range(nw):
            base = i * max_seqs * max_consensus
            win = []
            if status[i] == 0:
                for s in range(nseq[i]):
                    row = bytes(msa_buf[base + s * max_consensus:base + (s + 1) * max_consensus])
                    win.append(row.split(b"\0", 1)[0].decode())
            rows.append(win)
        return rows, status, cells, used
    out = [bytes(cons[i * max_consensus:i * max_consensus + clen[i]]).decode() for i in range(nw)]
    if coverage:
        covs = [cov[i * max_consensus:i * max_consensus + clen[i]].tolist() for i in range(nw)]
        return out, status, covs, cells, used
    return out, status, cells, used


# ---- single-kernel known-answer hooks ------------------------------------------

def topsort(outgoing):
    n = len(outgoing)
    in_cnt = np.zeros(n, np.uint16)
    out_cnt = np.zeros(n, np.uint16)
    out_e = np.zeros(n * MAX_EDGES, np.int32)
    for i, outs in enumerate(outgoing):
        out_cnt[i] = len(outs)
        for j, o in enumerate(outs):
            in_cnt[o] += 1
            out_e[i * MAX_EDGES + j] = o
    res = np.zeros(n, np.int32)
    lib().oracle_topsort(n, _p(in_cnt), _p(out_e), _p(out_cnt), _p(res))
    return res.tolist()


def poa_window_graph(reads, gap=-8, mismatch=-6, match=8, banded=False, band_width=256, score_bits=16,
                     max_nodes=None, max_consensus=None):
    """The final graph of one window with its aligned-node lists: (status, n,
    in_cnt, in_e, aln_cnt, aln), edges and aligned nodes in slot order
    (MAX_EDGES / MAX_ALIGNMENTS slots per node)."""
    reads = [r.encode() if isinstance(r, str) else bytes(r) for r in reads]
    max_len = max([len(r) for r in reads] + [1])
    if max_nodes is None:
        max_nodes = ((3 * max_len + 3) // 4) * 4 if not banded else ((4 * max_len + 3) // 4) * 4
    if max_consensus is None:
        max_consensus = 2 * max_len
    seqs = np.frombuffer(b"".join(reads) + b"\0" * (2 * band_width + 64), dtype=np.uint8).copy()
    lens = np.array([len(r) for r in reads], dtype=np.int32)
    wts = np.ones(max(len(seqs), 1), dtype=np.int8)
    nn = np.zeros(1, np.int32)
    in_cnt = np.zeros(max_nodes, np.uint16)
    aln_cnt = np.zeros(max_nodes, np.uint16)
    in_e = np.zeros(max_nodes * MAX_EDGES, np.int32)
    aln = np.zeros(max_nodes * MAX_ALIGNMENTS, np.int32)
    st = lib().oracle_poa_window_graph(_p(seqs), _p(lens), _p(wts), len(reads), gap, mismatch, match, int(banded),
                                       band_width, score_bits, max_nodes, max_consensus, _p(nn), _p(in_cnt),
                                       _p(in_e), _p(aln_cnt), _p(aln))
    n = int(nn[0])
    return (st, n, in_cnt[:n].copy(), in_e[:n * MAX_EDGES].copy(), aln_cnt[:n].copy(),
            aln[:n * MAX_ALIGNMENTS].copy())


def topsort_racon(n, in_cnt, in_e, aln_cnt, aln):
    """racon DFS sort (cudapoa_topsort.cuh:94-189) of a graph in slot arrays:
    (ok, order, node -> MSA column, column count)."""
    in_cnt = np.ascontiguousarray(in_cnt, np.uint16)
    aln_cnt = np.ascontiguousarray(aln_cnt, np.uint16)
    in_e = np.ascontiguousarray(in_e, np.int32)
    aln = np.ascontiguousarray(aln, np.int32)
    order = np.zeros(max(n, 1), np.int32)
    mpos = np.zeros(max(n, 1), np.int32)
    cols = np.zeros(1, np.int32)
    ok = lib().oracle_topsort_racon(n, _p(in_cnt), _p(in_e), _p(aln_cnt), _p(aln), _p(order), _p(mpos), _p(cols))
    return ok == 1, order[:n].tolist(), mpos[:n].tolist(), int(cols[0])


def edges_from_lists(outgoing, n):
    """BasicGraph::get_edges (reference cudapoa/tests/basic_graph.hpp:70-85)."""
    in_cnt = np.zeros(n, np.uint16)
    out_cnt = np.zeros(n, np.uint16)
    in_e = np.zeros(n * MAX_EDGES, np.int32)
    out_e = np.zeros(n * MAX_EDGES, np.int32)
    for i, outs in enumerate(outgoing):
        out_cnt[i] = len(outs)
        for j, o in enumerate(outs):
            in_e[o * MAX_EDGES + int(in_cnt[o])] = i
            in_cnt[o] += 1
            out_e[i * MAX_EDGES + j] = o
    return in_cnt, in_e, out_cnt, out_e


def nw(nodes, sorted_graph, outgoing, read, gap=-8, mismatch=-6, match=8):
    n = len(nodes)
    in_cnt, in_e, out_cnt, _ = edges_from_lists(outgoing, n)
    bases = np.frombuffer(nodes.encode(), np.uint8).copy()
    srt = np.array(sorted_graph, np.int32)
    pos = np.zeros(n, np.int32)
    for p, v in enumerate(sorted_graph):
        pos[v] = p
    rd = np.frombuffer(read.encode() + b"\0" * 8, np.uint8).copy()
    ag = np.zeros(n + len(read) + 4, np.int32)
    ar = np.zeros(n + len(read) + 4, np.int32)
    k = lib().oracle_nw(n, _p(bases), _p(srt), _p(pos), _p(in_cnt), _p(in_e), _p(out_cnt), _p(rd), len(read),
                        gap, mismatch, match, _p(ag), _p(ar))
    return ag[:k].tolist(), ar[:k].tolist()


def add_alignment(nodes, edges, aligned, coverage, read, graph, readpos, max_nodes=3072, weights=None):
    n = len(nodes)
    in_cnt, in_e, out_cnt, out_e = (np.zeros(max_nodes, np.uint16), np.zeros(max_nodes * MAX_EDGES, np.int32),
                                    np.zeros(max_nodes, np.uint16), np.zeros(max_nodes * MAX_EDGES, np.int32))
    a, b, c, d = edges_from_lists(edges, n)
    in_cnt[:n], in_e[:n * MAX_EDGES], out_cnt[:n], out_e[:n * MAX_EDGES] = a, b, c, d
    bases = np.zeros(max_nodes, np.uint8)
    bases[:n] = np.frombuffer(nodes.encode(), np.uint8)
    in_w = np.zeros(max_nodes * MAX_EDGES, np.uint16)
    aln_cnt = np.zeros(max_nodes, np.uint16)
    aln = np.zeros(max_nodes * MAX_EDGES, np.int32)
    for i, al in enumerate(aligned):
        for j, x in enumerate(al):
            aln[i * MAX_EDGES + j] = x
            aln_cnt[i] += 1
    cov = np.zeros(max_nodes, np.uint16)
    cov[:len(coverage)] = coverage
    ncount = np.array([n], np.int32)
    ag = np.array(graph, np.int32)
    ar = np.array(readpos, np.int32)
    rd = np.frombuffer(read.encode() + b"\0" * 8, np.uint8).copy()
    w = np.zeros(len(read) + 8, np.int8) if weights is None else np.asarray(weights + [0] * 8, np.int8)
    st = lib().oracle_add_alignment(max_nodes, _p(ncount), _p(bases), _p(in_cnt), _p(in_e), _p(in_w), _p(out_cnt),
                                    _p(out_e), _p(aln_cnt), _p(aln), _p(cov), _p(ag), _p(ar), len(graph), _p(rd),
                                    _p(w))
    nn = int(ncount[0])
    outs = [[int(out_e[v * MAX_EDGES + e]) for e in range(int(out_cnt[v]))] for v in range(nn)]
    return st, outs


def consensus_raw(nodes, sorted_graph, aligned, outgoing, coverage, weights, max_cons=2048):
    """generateConsensusTestKernel input construction as in the reference test
    (Test_CudapoaGenerateConsensus.cu:30-75, 160-240): the incoming weight of
    edge i->o is written at slot index i of node o (the test's own indexing)."""
    n = len(nodes)
    in_cnt, in_e, out_cnt, out_e = edges_from_lists(outgoing, n)
    in_w = np.zeros(n * MAX_EDGES, np.uint16)
    for i, outs in enumerate(outgoing):
        for j, o in enumerate(outs):
            in_w[o * MAX_EDGES + i] = weights[i][j]
    bases = np.frombuffer(nodes.encode(), np.uint8).copy()
    srt = np.array(sorted_graph, np.int32)
    pos = np.zeros(n, np.int32)
    for p, v in enumerate(sorted_graph):
        pos[v] = p
    aln_cnt = np.zeros(n, np.uint16)
    aln = np.zeros(n * MAX_EDGES, np.int32)
    for i, al in enumerate(aligned):
        for j, x in enumerate(al):
            aln[i * MAX_EDGES + j] = x
            aln_cnt[i] += 1
    cov = np.array(coverage, np.uint16)
    cons = np.zeros(max_cons + 1, np.uint8)
    ccov = np.zeros(max_cons + 1, np.uint16)
    st = lib().oracle_consensus_raw(n, _p(bases), _p(srt), _p(pos), _p(in_cnt), _p(in_e), _p(in_w), _p(out_cnt),
                                    _p(out_e), _p(aln_cnt), _p(aln), _p(cov), max_cons, _p(cons), _p(ccov))
    return st, bytes(cons).split(b"\0", 1)[0].decode()


# ---------------------------------------------------------------------------
# cudaaligner restatement (oracle/aligner_oracle.cpp)
ALIGN_HM, ALIGN_MYERS, ALIGN_MYERS_BANDED, ALIGN_UKKONEN = 0, 1, 2, 3
UKKONEN_P = 100  # aligner_global_ukkonen.cpp:29
_CIGAR = {0: "M", 1: "M", 2: "I", 3: "D"}


def _b(s):
    return s.encode() if isinstance(s, str) else bytes(s)


def align(query, target, algo=ALIGN_HM, max_query_length=None):
    """Alignment states (AlignmentState values, start -> end) of query vs target."""
    q, t = _b(query), _b(target)
    mq = len(q) if max_query_length is None else max_query_length
    cap = len(q) + len(t) + 8
    buf = np.zeros(cap, np.int8)
    n = lib().oracle_align(algo, q, len(q), t, len(t), mq, _p(buf), cap)
    if n < 0:
        raise RuntimeError("oracle path buffer too small")
    return buf[:n][::-1].tolist()


def cigar(states):
    """AlignmentImpl::convert_to_cigar (alignment_impl.cpp:47-73)."""
    if not states:
        return ""
    out, last, cnt = [], _CIGAR[states[0]], 0
    for s in states:
        c = _CIGAR[s]
        if c == last:
            cnt += 1
        else:
            out.append("%d%s" % (cnt, last))
            last, cnt = c, 1
    out.append("%d%s" % (cnt, last))
    return "".join(out)


def format_alignment(query, target, states):
    """AlignmentImpl::format_alignment (alignment_impl.cpp:75-112): (query, pairing, target)."""
    q, t = (query.decode() if isinstance(query, bytes) else query), (target.decode() if isinstance(target, bytes)
                                                                    else target)
    qs, ps, ts, qi, ti = [], [], [], 0, 0
    for s in states:
        if s in (0, 1):
            ts.append(t[ti]); qs.append(q[qi]); ps.append("|" if s == 0 else "x"); ti += 1; qi += 1
        elif s == 3:
            ts.append("-"); qs.append(q[qi]); ps.append(" "); qi += 1
        else:
            ts.append(t[ti]); qs.append("-"); ps.append(" "); ti += 1
    return "".join(qs), "".join(ps), "".join(ts)


def edit_distance(query, target):
    q, t = _b(query), _b(target)
    return lib().oracle_edit_distance(q, len(q), t, len(t))


def myers_banded(query, target):
    """Banded Myers: (states start -> end, accepted band width, tries)."""
    q, t = _b(query), _b(target)
    buf = np.zeros(len(q) + len(t) + 8, np.int8)
    bw, tries = C.c_int(0), C.c_int(0)
    n = lib().oracle_myers_banded(q, len(q), t, len(t), _p(buf), C.byref(bw), C.byref(tries))
    return buf[:n][::-1].tolist(), bw.value, tries.value


def ukkonen(query, target, p=UKKONEN_P):
    """Ukkonen banded NW with band parameter p: states start -> end."""
    q, t = _b(query), _b(target)
    buf = np.zeros(len(q) + len(t) + 8, np.int8)
    n = lib().oracle_ukkonen(q, len(q), t, len(t), int(p), _p(buf))
    return buf[:n][::-1].tolist()


def query_pattern(query, x, word, reverse=False):
    q = _b(query)
    return lib().oracle_query_pattern(q, len(q), _b(x), word, int(reverse))


def align_batch(pairs, algo=ALIGN_HM, max_query_length=None, nthreads=0):
    """All pairs (query, target) with OpenMP; returns (list of state lists, threads used)."""
    n = len(pairs)
    blobs, off, lens = [], np.zeros(2 * n, np.int64), np.zeros(2 * n, np.int32)
    pos = 0
    for i, (q, t) in enumerate(pairs):
        for k, s in enumerate((_b(q), _b(t))):
            off[2 * i + k] = pos
            lens[2 * i + k] = len(s)
            blobs.append(s)
            pos += len(s)
    seqs = np.frombuffer(b"".join(blobs) + b"\0", np.uint8).copy()
    mq = int(max(lens[0::2])) if max_query_length is None and n else (max_query_length or 0)
    stride = int(lens.max()) * 2 + 8 if n else 8
    paths = np.zeros(n * stride, np.int8)
    plen = np.zeros(n, np.int32)
    used = lib().oracle_align_batch(algo, n, _p(seqs), _p(off), _p(lens), mq, _p(paths), _p(plen), stride, nthreads)
    out = [paths[i * stride:i * stride + plen[i]][::-1].tolist() for i in range(n)]
    return out, used

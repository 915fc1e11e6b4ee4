"""GPU parity for caller-supplied base weights (Entry.weights, the path racon
feeds base qualities through).

Reference semantics this pins:
- weights are copied per base, or set to 1 when the caller passes none
  (cudapoa_batch.cuh:515-531), and negative weights throw
  (cudapoa_batch.cuh:524-528);
- the backbone's edge i-1 -> i weighs w[i-1] + w[i], node 0's first slot w[0]
  (cudapoa_kernels.cuh:180,195), and the weight pointer advances by each
  read's length (cudapoa_kernels.cuh:218);
- addAlignmentToGraph adds prev_weight + w[pos] to an existing edge, or
  creates the edge with that weight, in u16 arithmetic
  (cudapoa_add_alignment.cuh:86,104,221-249,273), so heavy windows wrap.

Every kernel family runs on the same weighted windows (LDS full kernel,
banded row-parallel and anti-diagonal passes, the global-memory v1 kernel),
consensus and MSA, and the final graphs (edge weights included) are compared
bit for bit with the oracle (oracle/poa_oracle.cpp, weights argument).
"""
import numpy as np
import pytest

from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
from oracle import oracle

pytestmark = pytest.mark.gpu
MEM = 8 << 30


def _weights_for(wins, seed, lo=0, hi=60, none_every=0):
    """Phred-like per-base weights; with none_every=k every k-th read gets
    None (default all-ones weights, mixed with explicit ones in one window)."""
    rng = np.random.default_rng(seed)
    out = []
    for w in wins:
        ww = []
        for j, r in enumerate(w):
            if none_every and j % none_every == 1:
                ww.append(None)
            else:
                ww.append(rng.integers(lo, hi + 1, size=len(r), dtype=np.int8))
        out.append(ww)
    return out


def _oracle_weights(ww, w):
    return [np.ones(len(r), np.int8) if x is None else x for x, r in zip(ww, w)]


def _run(wins, wts, max_seq, max_seqs, banded, bw, out):
    b = CudaPoaBatch(max_seqs, max_seq, MEM, output_type=out, cuda_banded_alignment=banded,
                     alignment_band_width=bw)
    for w, ww in zip(wins, wts):
        st, _ = b.add_poa_group(list(w), weights=ww)
        assert st == 0
    b.generate_poa()
    return b


def _check(b, wins, wts, max_seq, max_seqs, banded, bw, out, tag):
    msa = out == "msa"
    sbits = b.get_types()[0]
    got = b.get_msa() if msa else b.get_consensus()
    graphs, gst = b.get_graphs()
    mn = ((4 if banded else 3) * max_seq + 3) // 4 * 4
    for i, (w, ww) in enumerate(zip(wins, wts)):
        r = oracle.poa_window(w, weights=_oracle_weights(ww, w), banded=banded, band_width=bw, msa=msa,
                              score_bits=sbits, max_nodes=mn, max_consensus=2 * max_seq, max_seqs=max_seqs,
                              want_graph=True)
        if msa:
            assert (got[1][i], got[0][i]) == (r.status, r.msa), (tag, i)
        else:
            cons, cov, st = got
            assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (tag, i)
        g = graphs[i]
        expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
        assert {(u, v): g.weight(u, v) for (u, v) in g.edges} == expect, (tag, i)
    return graphs


# (mode, env, expected kernel_variant): 2 = LDS full kernel, 3 = band kernel
# row-parallel pass, 4 = band kernel anti-diagonal pass, 1 = global-memory v1
KERNELS = {
    "lds": ({}, False, 2),
    "band_row": ({"GWAMD_BAND_FWD": "row"}, True, 3),
    "band_ad": ({"GWAMD_BAND_FWD": "ad"}, True, 4),
    "v1_full": ({"GWAMD_POA_KERNEL": "v1"}, False, 1),
    "v1_band": ({"GWAMD_POA_KERNEL": "v1"}, True, 1),
}


def _env(monkeypatch, env):
    for k in ("GWAMD_POA_KERNEL", "GWAMD_BAND_FWD"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)


@pytest.mark.parametrize("kernel", list(KERNELS))
@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_weighted_windows_match_oracle(kernel, out, monkeypatch):
    env, banded, variant = KERNELS[kernel]
    _env(monkeypatch, env)
    wins = synth.poa_windows(1701, 6, 600, 12, 30, 30, 30)
    wins += synth.poa_windows(1711, 3, 150, 20, 10, 10, 10)
    wins.append([b"ACGTACGTTA", b"", b"A", b"ACGTTCGTTA", b"ACGAACGTTA"])  # empty / one-base reads
    wts = _weights_for(wins, 5)
    # one window mixing None (all-ones) with explicit weights
    wins += synth.poa_windows(1721, 2, 400, 10, 20, 20, 20)
    wts += _weights_for(wins[-2:], 6, none_every=3)
    max_seq, max_seqs = 700, 20
    b = _run(wins, wts, max_seq, max_seqs, banded, 256, out)
    assert b.kernel_variant() == variant
    graphs = _check(b, wins, wts, max_seq, max_seqs, banded, 256, out, kernel)
    # the weights are observable: the same windows with default weights give
    # other edge weights
    b1 = _run(wins[:1], [None], max_seq, max_seqs, banded, 256, out)
    g1, _ = b1.get_graphs()
    assert {e: g1[0].weight(*e) for e in g1[0].edges} != {e: graphs[0].weight(*e) for e in graphs[0].edges}


@pytest.mark.parametrize("kernel", ["lds", "band_row", "band_ad", "v1_full"])
def test_edge_weight_u16_wrap(kernel, monkeypatch):
    # >= 300 reads of weight 127: an edge shared by every read collects
    # 300 x 254 > 65,535 and wraps in the reference's u16 arithmetic
    env, banded, variant = KERNELS[kernel]
    _env(monkeypatch, env)
    wins = synth.poa_windows(1801, 1, 80, 320, 2, 2, 2)
    wts = [[np.full(len(r), 127, np.int8) for r in wins[0]]]
    b = _run(wins, wts, 128, 320, banded, 128, "consensus")
    assert b.kernel_variant() == variant
    graphs = _check(b, wins, wts, 128, 320, banded, 128, "consensus", kernel)
    # some edge really wrapped: each read adds 127 + 127 to (len - 1) edges
    # and weights only grow, so without a wrap the stored weights would sum
    # to exactly that total
    total = sum((len(r) - 1) * 254 for r in wins[0] if len(r) > 0)
    assert sum(graphs[0].weight(*e) for e in graphs[0].edges) < total


def test_weighted_windows_config_b_shape():
    # config B's shape (BatchSize(1100, 32), full alignment, LDS kernel),
    # phred-like weights on every read
    wins = synth.poa_windows(1901, 16, 1000, 32, 50, 50, 50)
    wts = _weights_for(wins, 7, lo=1, hi=60)
    b = _run(wins, wts, 1100, 32, False, 256, "consensus")
    assert b.kernel_variant() == 2
    _check(b, wins, wts, 1100, 32, False, 256, "consensus", "B")


def test_weighted_windows_int32_lds():
    # 32-bit scores (max_sequence_size 1,600 >= 1,490, use32bitScore) on the
    # LDS kernel's 32-bit pass, weights on every read, consensus and graphs
    wins = synth.poa_windows(1951, 6, 1200, 12, 60, 60, 60)
    wts = _weights_for(wins, 9, lo=0, hi=60, none_every=4)
    b = _run(wins, wts, 1600, 12, False, 256, "consensus")
    assert b.kernel_variant() == 2 and b.get_types()[0] == 32
    _check(b, wins, wts, 1600, 12, False, 256, "consensus", "lds32")


def test_negative_weights_raise():
    # cudapoa_batch.cuh:524-528: throw_on_negative -> std::invalid_argument
    b = CudaPoaBatch(4, 128, MEM, alignment_band_width=128)
    with pytest.raises(ValueError):
        b.add_poa_group(["ACGT", "ACGA"], weights=[np.array([1, 2, 3, 4], np.int8),
                                                  np.array([1, -1, 3, 4], np.int8)])

"""GPU parity tests for the POA path: the HIP kernels (through the C ABI of
libgwamd.so) against the CPU restatement (oracle/) and the reference KATs.
Bit-exact: consensus strings, coverage vectors, MSA rows, graphs, statuses."""
import json
import os

import pytest

from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_kat.json")))
MEM = 8 << 30


def _batch(name):
    return [b for b in GOLD["batch"] if b["name"] == name][0]


def run_gpu(windows, max_seq, max_seqs, banded=False, bw=None, output_type="consensus", mem=MEM, **kw):
    if bw is None:  # BatchSize requires band width <= max_sequence_size (batch.hpp:126)
        bw = 256 if max_seq >= 256 else 128
    b = CudaPoaBatch(max_seqs, max_seq, mem, output_type=output_type, cuda_banded_alignment=banded,
                     alignment_band_width=bw, **kw)
    for w in windows:
        st, seq_st = b.add_poa_group(list(w))
        assert st == 0
    b.generate_poa()
    return b


def run_oracle(w, max_seq, max_seqs, banded=False, bw=256, msa=False, score_bits=16, **kw):
    mn = kw.get("max_nodes", ((4 if banded else 3) * max_seq + 3) // 4 * 4)
    return oracle.poa_window(w, banded=banded, band_width=bw, msa=msa, score_bits=score_bits,
                             max_nodes=mn, max_consensus=kw.get("max_consensus", 2 * max_seq), max_seqs=max_seqs,
                             want_graph=kw.get("want_graph", False), spoa_accurate=kw.get("spoa_accurate", False))


def test_kat_all_A():
    case = _batch("all_A_1023x3")
    b = run_gpu(case["windows"], 1024, 10)
    cons, cov, st = b.get_consensus()
    assert st == [0]
    assert cons == case["consensus"]


def test_kat_python_graph():
    case = _batch("py_graph")
    b = run_gpu(case["windows"], 1024, 10)
    graphs, st = b.get_graphs()
    assert st == [0]
    assert graphs[0].number_of_nodes() == 10
    assert graphs[0].number_of_edges() == 11


def test_kat_python_seed2():
    case = _batch("py_complex_seed2")
    b = run_gpu(case["windows"], 1024, 1000)
    cons, cov, st = b.get_consensus()
    assert st == [0]
    assert cons[0] == case["consensus"][0]


def test_kat_python_simple():
    case = _batch("py_simple")
    for banded in (False, True):
        b = run_gpu(case["windows"], 1024, 10, banded=banded)
        cons, cov, st = b.get_consensus()
        assert len(cons) == 2 and b.total_poas == 2
        for w, c, v, s in zip(case["windows"], cons, cov, st):
            r = run_oracle(w, 1024, 10, banded=banded)
            assert (s, c, v) == (r.status, r.consensus, r.coverage)


@pytest.mark.parametrize("L,nreads,nwin,err", [(60, 6, 32, 5), (300, 12, 24, 20), (1000, 32, 8, 50)])
def test_full_parity_synthetic(L, nreads, nwin, err):
    wins = synth.poa_windows(7, nwin, L, nreads, err, err, err)
    max_seq = max(L + err + 8, 128)
    b = run_gpu(wins, max_seq, nreads)
    cons, cov, st = b.get_consensus()
    cells, _ = b.get_stats()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, nreads)
        assert st[i] == r.status, i
        assert cons[i] == r.consensus, i
        assert cov[i] == r.coverage, i
        assert cells[i] == r.cells, i


def test_full_parity_int32_scores():
    # max_sequence_size large enough that use32bitScore selects int32
    wins = synth.poa_windows(11, 6, 400, 10, 20, 20, 20)
    b = run_gpu(wins, 4200, 10)
    assert b.get_types()[0] == 32
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 4200, 10)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage)


@pytest.mark.parametrize("bw", [128, 256, 512])
def test_banded_parity_synthetic(bw):
    wins = synth.poa_windows(21, 12, 600, 10, 30, 30, 30)
    max_seq = 700
    b = run_gpu(wins, max_seq, 10, banded=True, bw=bw)
    sbits = b.get_types()[0]
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 10, banded=True, bw=bw, score_bits=sbits)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


@pytest.mark.parametrize("variant", ["band", "v1"])
@pytest.mark.parametrize("bw", [384, 640, 768, 896, 1024])
def test_banded_other_widths(bw, variant, monkeypatch):
    # every other band width the reference accepts up to 1,024 (multiples of
    # 128, batch.hpp:85-94): the LDS band kernel with bw / 64 cells per lane
    # (poa_band_c<CPL>.hip), and the global-memory kernel on the same windows;
    # the windows include reads much shorter than the band, empty and
    # one-base reads and a 60-read window (nodes with many predecessors)
    if variant == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(23, 6, 1000, 12, 40, 40, 40)
    wins += synth.poa_windows(29, 2, 200, 8, 10, 10, 10)
    wins.append([b"ACGTTGCA" * 20, b"ACGTTGCA" * 120, b"", b"A", b"GGGG" * 100, b"ACGTTGCA" * 20])
    wins += synth.poa_windows(31, 1, 300, 60, 30, 30, 30)
    max_seq = 1100
    b = run_gpu(wins, max_seq, 60, banded=True, bw=bw)
    assert b.kernel_variant() == (1 if variant == "v1" else 3)
    sbits = b.get_types()[0]
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 60, banded=True, bw=bw, score_bits=sbits)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (bw, variant, i)


@pytest.mark.parametrize("bw", [384, 1024])
@pytest.mark.parametrize("spoa", [False, True])
def test_banded_wide_msa_int32(bw, spoa, monkeypatch):
    # wide bands with 32-bit scores (max_sequence_size 6000), MSA output and
    # SPOA_ACCURATE, on the band kernel, against the oracle
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(733, 4, 1500, 8, 75, 75, 75)
    b = run_gpu(wins, 6000, 8, banded=True, bw=bw, output_type="msa", spoa_accurate=spoa)
    assert b.kernel_variant() == 3 and b.get_types()[0] == 32
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 6000, 8, banded=True, bw=bw, msa=True, score_bits=32, spoa_accurate=spoa)
        assert (st[i], msa[i]) == (r.status, r.msa), (bw, spoa, i)


@pytest.mark.parametrize("variant", ["lds", "v1"])
def test_full_int32_long_reads(variant, monkeypatch):
    # full alignment with 32-bit scores (4 kb reads: use32bitScore,
    # cudapoa_limits.hpp:28-53): the LDS kernel's 32-bit pass
    # (nw_forward_lds_w, 16 columns per lane on 8 waves) and the global-memory
    # kernel on the same windows
    if variant == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(27, 3, 4000, 6, 150, 150, 150)
    b = run_gpu(wins, 4400, 6, mem=8 << 30)
    assert b.get_types()[0] == 32 and b.kernel_variant() == (1 if variant == "v1" else 2)
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 4400, 6, score_bits=32)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


# 32-bit scores on the LDS kernel at every (columns per lane, waves) shape the
# plan uses; windows whose reads are longer than one sweep (NW * 64 * CPL
# columns), hit span and sweep boundaries, or are empty / one base, plus a
# 40-read window (many predecessors; rows read from beyond the ring go
# through the HBM spill rows), consensus and MSA
@pytest.mark.parametrize("shape", ["8,1", "8,2", "8,4", "8,8", "16,8"])
@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_full_int32_lds_shapes(shape, out, monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    monkeypatch.setenv("GWAMD_DIAG", "1")
    monkeypatch.setenv("GWAMD_POA_LDS_SHAPE", shape)
    max_seq = 2200
    wins = synth.poa_windows(811, 3, 1500, 10, 60, 60, 60)
    wins += synth.poa_windows(821, 2, 500, 40, 25, 25, 25)
    wins.append([b"ACGT" * 256, b"ACGT" * 256 + b"A", b"", b"ACGTTGCA" * 64, b"ACGTTGCA" * 64 + b"G",
                 b"ACGT" * 128, b"C" * 2100, b"ACGTTGCA" * 257])
    msa = out == "msa"
    b = run_gpu(wins, max_seq, 40, output_type=out)
    assert b.get_types()[0] == 32 and b.kernel_variant() == 2
    got = b.get_msa() if msa else b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 40, msa=msa, score_bits=32)
        if msa:
            assert (got[1][i], got[0][i]) == (r.status, r.msa), (shape, i)
        else:
            assert (got[2][i], got[0][i], got[1][i]) == (r.status, r.consensus, r.coverage), (shape, i)


def test_msa_parity_synthetic():
    wins = synth.poa_windows(31, 8, 300, 8, 15, 15, 15)
    b = run_gpu(wins, 400, 8, output_type="msa")
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 400, 8, msa=True)
        assert st[i] == r.status
        assert msa[i] == r.msa
        # de-gapped rows equal the inputs (Test_CudapoaGenerateMSA2.cu:125-140)
        assert [row.replace("-", "") for row in msa[i]] == [x.decode() for x in w]


def test_banded_msa_parity():
    wins = synth.poa_windows(41, 4, 500, 6, 25, 25, 25)
    b = run_gpu(wins, 600, 6, banded=True, output_type="msa")
    sbits = b.get_types()[0]
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 600, 6, banded=True, msa=True, score_bits=sbits)
        assert (st[i], msa[i]) == (r.status, r.msa)


def test_graph_parity():
    wins = synth.poa_windows(51, 4, 200, 6, 10, 10, 10)
    b = run_gpu(wins, 300, 6)
    graphs, st = b.get_graphs()
    for i, w in enumerate(wins):
        r = run_oracle(w, 300, 6, want_graph=True)
        g = graphs[i]
        expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
        got = {(u, v): g.weight(u, v) for (u, v) in g.edges}
        assert got == expect
        assert "".join(g.label(v) for v in range(r.final_nodes)) == r.graph["bases"]


def test_single_read_and_status_codes():
    b = CudaPoaBatch(4, 128, MEM, alignment_band_width=128)
    st, seq_st = b.add_poa_group(["ACGTACGT"])
    assert (st, seq_st) == (0, [0])
    st, seq_st = b.add_poa_group(["A" * 129, "ACGT", "ACGA", "ACGG", "ACGC", "ACGT"])
    assert st == 0
    # too long (not added); four added; exceeded_maximum_sequences_per_poa (cudapoa_batch.cuh:490-510)
    assert seq_st == [2, 0, 0, 0, 0, 3]
    b.generate_poa()
    cons, cov, st = b.get_consensus()
    assert cons[0] == "ACGTACGT" and cov[0] == [1] * 8 and st[0] == 0
    r = oracle.poa_window([b"ACGT", b"ACGA", b"ACGG", b"ACGC"], max_nodes=384, max_consensus=256)
    assert (st[1], cons[1], cov[1]) == (r.status, r.consensus, r.coverage)


def test_node_limit_error_matches_oracle():
    # tiny node capacity forces node_count_exceeded_maximum_graph_size
    wins = synth.poa_windows(61, 3, 100, 8, 20, 20, 20)
    b = CudaPoaBatch(8, 130, MEM, max_nodes_per_window=140, alignment_band_width=128)
    for w in wins:
        b.add_poa_group(list(w))
    b.generate_poa()
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = oracle.poa_window(w, max_nodes=140, max_consensus=260, max_seqs=8)
        assert (st[i], cons[i]) == (r.status, r.consensus)
    assert any(s == 4 for s in st)


def test_output_type_unavailable_and_reset():
    b = CudaPoaBatch(4, 128, MEM, output_type="consensus", alignment_band_width=128)
    b.add_poa_group(["ACGT", "ACGT"])
    b.generate_poa()
    with pytest.raises(RuntimeError):
        b.get_msa()
    assert b.total_poas == 1
    b.reset()
    assert b.total_poas == 0


def test_zero_memory_throws():
    with pytest.raises(RuntimeError):
        CudaPoaBatch(5, 1024, 0)


@pytest.mark.parametrize("variant", ["v1", "lds"])
def test_kernel_variants_agree_with_oracle(variant, monkeypatch):
    # the global-memory kernel and the LDS-resident kernel give identical outputs
    if variant == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(71, 12, 700, 16, 40, 40, 40)
    b = run_gpu(wins, 800, 16)
    assert b.kernel_variant() == (1 if variant == "v1" else 2)
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 800, 16)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


def test_lds_kernel_empty_and_tiny_reads():
    wins = [[b"ACGTACGTAC", b"", b"ACG", b"A", b"ACGTTCGTAC"], [b"GATTACA", b"GATTACA", b"TTT"]]
    b = run_gpu(wins, 128, 8)
    assert b.kernel_variant() == 2
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 128, 8)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


@pytest.mark.parametrize("shape", ["8,1", "16,1", "24,1", "32,1", "8,2", "8,3", "8,4", "16,4", "4,4"])
def test_lds_forward_shapes(shape, monkeypatch):
    # every (columns per lane, waves per window) forward-pass shape; reads
    # longer than one sweep (NW*64*CPL columns) take several sweeps, and span /
    # sweep boundaries (512, 513, 1024, 1025 columns) are hit exactly
    monkeypatch.setenv("GWAMD_POA_LDS_SHAPE", shape)
    max_seq = 1100
    wins = synth.poa_windows(301, 4, 1040, 12, 25, 25, 25)
    wins.append([b"ACGT" * 256, b"ACGT" * 256 + b"A", b"", b"ACGTTGCA" * 64, b"ACGTTGCA" * 64 + b"G",
                 b"ACGT" * 128, b"C" * 1100])
    b = run_gpu(wins, max_seq, 12)
    assert b.kernel_variant() == 2
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 12)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (shape, i)


def test_lds_msa_multiwave(monkeypatch):
    monkeypatch.setenv("GWAMD_POA_LDS_SHAPE", "8,3")
    wins = synth.poa_windows(411, 4, 900, 10, 40, 40, 40)
    b = run_gpu(wins, 1000, 10, output_type="msa")
    assert b.kernel_variant() == 2
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 1000, 10, msa=True)
        assert st[i] == r.status and msa[i] == r.msa, i


def test_config_c_msa_10kb_banded_int32():
    # SURVEY.md 8(d) config C shape: BatchSize(10600, 16, 256), banded, MSA,
    # 10 kb backbone with 500/500/500 mutations -> int32 scores and node ids
    wins = synth.poa_windows(1, 2, 10000, 16, 500, 500, 500)
    b = run_gpu(wins, 10600, 16, banded=True, bw=256, output_type="msa", mem=16 << 30)
    assert b.get_types() == (32, 32)
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 10600, 16, banded=True, bw=256, msa=True, score_bits=32)
        assert st[i] == r.status == 0
        assert msa[i] == r.msa, i


@pytest.mark.parametrize("variant", ["v1", "band"])
@pytest.mark.parametrize("bw", [128, 256, 512])
def test_banded_kernel_variants(variant, bw, monkeypatch):
    # the banded kernel (codes + LDS ring) and the global-memory kernel agree
    # with the oracle, including reads much shorter than the band (every row
    # starts at column 0), reads longer than the graph (gradient > 1), empty
    # and single-base reads
    if variant == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(501, 6, 700, 10, 35, 35, 35)
    wins += synth.poa_windows(601, 3, 90, 8, 6, 6, 6)
    wins.append([b"ACGTTGCA" * 20, b"ACGTTGCA" * 80, b"", b"A", b"ACGTTGCA" * 40 + b"T" * 100,
                 b"GGGG" * 100, b"ACGTTGCA" * 20])
    wins.append([b"A" * 600, b"C" * 600, b"A" * 300 + b"C" * 300, b"ACGT"])
    b = run_gpu(wins, 800, 10, banded=True, bw=bw)
    assert b.kernel_variant() in ((1,) if variant == "v1" else (3, 4))
    sbits = b.get_types()[0]
    cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 800, 10, banded=True, bw=bw, score_bits=sbits)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (variant, bw, i)


@pytest.mark.parametrize("bw", [512])
def test_banded_512_msa_int32_and_spoa(bw, monkeypatch):
    # band width 512: the LDS band kernel with 8 cells per lane (row-parallel
    # pass; predecessor band shifts of 4 take the element-wise fetch), int32
    # scores, MSA and SPOA_ACCURATE, against the oracle
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(711, 4, 1500, 8, 75, 75, 75)
    for spoa in (False, True):
        b = run_gpu(wins, 6000, 8, banded=True, bw=bw, output_type="msa", spoa_accurate=spoa)
        assert b.kernel_variant() == 3 and b.get_types()[0] == 32
        msa, st = b.get_msa()
        for i, w in enumerate(wins):
            r = run_oracle(w, 6000, 8, banded=True, bw=bw, msa=True, score_bits=32, spoa_accurate=spoa)
            assert (st[i], msa[i]) == (r.status, r.msa), (spoa, i)


def test_banded_kernel_msa_graph_int32(monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(701, 5, 900, 9, 45, 45, 45)
    b = run_gpu(wins, 4200, 9, banded=True, bw=256, output_type="msa")
    assert b.kernel_variant() in (3, 4) and b.get_types()[0] == 32
    msa, st = b.get_msa()
    for i, w in enumerate(wins):
        r = run_oracle(w, 4200, 9, banded=True, bw=256, msa=True, score_bits=32)
        assert (st[i], msa[i]) == (r.status, r.msa), i


def _band_ad_windows(seed):
    # uneven windows: long and short reads (gradient above and below 1), reads
    # shorter than the band (every row starts at column 0), empty and one-base
    # reads, repeats (many equal-score ties), and a 60-read window whose graph
    # has nodes with many predecessors
    wins = synth.poa_windows(seed, 4, 700, 10, 35, 35, 35)
    wins += synth.poa_windows(seed + 100, 2, 1500, 6, 120, 120, 120)
    wins += synth.poa_windows(seed + 200, 2, 90, 8, 6, 6, 6)
    wins.append([b"ACGTTGCA" * 20, b"ACGTTGCA" * 80, b"", b"A", b"ACGTTGCA" * 40 + b"T" * 100,
                 b"GGGG" * 100, b"ACGTTGCA" * 20])
    wins.append([b"A" * 600, b"C" * 600, b"A" * 300 + b"C" * 300, b"ACGT"])
    wins += synth.poa_windows(seed + 300, 1, 300, 60, 30, 30, 30)
    return wins


# Anti-diagonal forward pass of the banded kernel (poa_band_ad.hpp; default
# for large windows, forced here with GWAMD_BAND_FWD=ad) against the oracle
# and the row-parallel pass, 16- and 32-bit scores, both band widths,
# consensus and MSA output, SPOA_ACCURATE sorts.
@pytest.mark.parametrize("bw", [128, 256])
@pytest.mark.parametrize("max_seq", [1700, 4200])
@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_band_anti_diagonal(bw, max_seq, out, monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = _band_ad_windows(1301)
    msa = out == "msa"
    res = {}
    for fwd in ("ad", "row"):
        monkeypatch.setenv("GWAMD_BAND_FWD", fwd)
        b = run_gpu(wins, max_seq, 60, banded=True, bw=bw, output_type=out)
        assert b.kernel_variant() == (4 if fwd == "ad" else 3)
        res[fwd] = b.get_msa() if msa else b.get_consensus()
        res[fwd + "_cells"] = b.get_stats()[0]
        sbits = b.get_types()[0]
    monkeypatch.delenv("GWAMD_BAND_FWD", raising=False)
    assert res["ad"] == res["row"]
    assert list(res["ad_cells"]) == list(res["row_cells"])
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 60, banded=True, bw=bw, msa=msa, score_bits=sbits)
        if msa:
            assert (res["ad"][1][i], res["ad"][0][i]) == (r.status, r.msa), i
        else:
            cons, cov, st = res["ad"]
            assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_band_anti_diagonal_spoa_graph(out, monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    monkeypatch.setenv("GWAMD_BAND_FWD", "ad")
    wins = synth.poa_windows(1401, 6, 400, 20, 20, 20, 20)
    b = run_gpu(wins, 1000, 20, banded=True, bw=256, output_type=out, spoa_accurate=True)
    assert b.kernel_variant() == 4
    sbits = b.get_types()[0]
    graphs, gst = b.get_graphs()
    got = b.get_msa() if out == "msa" else b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, 1000, 20, banded=True, bw=256, msa=(out == "msa"), score_bits=sbits,
                       want_graph=True, spoa_accurate=True)
        if out == "msa":
            assert (got[1][i], got[0][i]) == (r.status, r.msa), i
        else:
            assert (got[2][i], got[0][i], got[1][i]) == (r.status, r.consensus, r.coverage), i
        g = graphs[i]
        assert {(u, v): g.weight(u, v) for (u, v) in g.edges} == \
            {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}, i


@pytest.mark.parametrize("variant", ["v1", "fast"])
@pytest.mark.parametrize("banded", [False, True])
@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_spoa_accurate(variant, banded, out, monkeypatch):
    # SPOA_ACCURATE (cudapoa_kernels.cuh:324-337): racon DFS sort after every
    # read, on every kernel; these windows include ones whose output differs
    # from the default Kahn-order build, so the mode is observable
    if variant == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    wins = synth.poa_windows(100, 16, 300, 20, 60, 60, 60)
    b = run_gpu(wins, 400, 20, banded=banded, bw=256, output_type=out, spoa_accurate=True)
    assert b.kernel_variant() in ((1,) if variant == "v1" else ((3, 4) if banded else (2,)))
    sbits = b.get_types()[0]
    if out == "msa":
        got, st = b.get_msa()
    else:
        cons, cov, st = b.get_consensus()
        got = list(zip(cons, cov))
    differ = 0
    for i, w in enumerate(wins):
        r = run_oracle(w, 400, 20, banded=banded, bw=256, msa=(out == "msa"), score_bits=sbits, spoa_accurate=True)
        k = run_oracle(w, 400, 20, banded=banded, bw=256, msa=(out == "msa"), score_bits=sbits)
        want = r.msa if out == "msa" else (r.consensus, r.coverage)
        assert (st[i], got[i]) == (r.status, want), i
        differ += (k.msa if out == "msa" else (k.consensus, k.coverage)) != want
    assert differ > 0


@pytest.mark.parametrize("banded", [False, True])
def test_serialize_graph_case(banded):
    # Test_CudapoaSerializeGraph.cpp:58-90: 500 reads generated from a 50 bp
    # backbone with minstd_rand(1) (10 / 5 / 10 mutations), MSA output,
    # BatchSize(1024, 500); the final graph equals the oracle's, edge weights
    # included, and serialises to one DOT line per node label and per edge
    wins = synth.poa_windows(1, 1, 50, 500, 10, 5, 10)
    b = run_gpu(wins, 1024, 500, banded=banded, bw=256, output_type="msa")
    graphs, st = b.get_graphs()
    r = run_oracle(wins[0], 1024, 500, banded=banded, bw=256, msa=True, want_graph=True)
    assert st == [r.status] == [0]
    g = graphs[0]
    expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
    assert {(u, v): g.weight(u, v) for (u, v) in g.edges} == expect
    assert "".join(g.label(v) for v in range(r.final_nodes)) == r.graph["bases"]
    msa, mst = b.get_msa()
    assert (mst[0], msa[0]) == (r.status, oracle.poa_window(wins[0], banded=banded, msa=True, max_nodes=(4 if banded else 3) * 1024,
                                                            max_consensus=2048, max_seqs=500).msa)


# Persistent grid and launch order (poa_batch.cpp plan_launch_order): with
# GWAMD_POA_SLOTS the batch gets fewer scratch slots than windows, so every
# workgroup dequeues several windows (heaviest first) and reuses its slot's
# scratch; GWAMD_LAUNCH_ORDER_CUS plans the snake order for a 2-CU device, so
# batches far smaller than the real CU count run reordered.  Every output stays
# bit-exact per window, and a second generate (dequeue counter reset) repeats it.
@pytest.mark.parametrize("mode", ["full", "full_msa", "banded", "banded_msa", "banded_ad", "banded_ad_msa", "v1",
                                  "full_spoa"])
@pytest.mark.parametrize("grid", ["slots3", "cus2", "slots5_cus2"])
def test_persistent_grid_and_launch_order(mode, grid, monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    # banded_ad: the anti-diagonal forward pass (helper waves, progress words,
    # ring) on a persistent grid whose workgroups reuse their slot across windows
    if "_ad" in mode:
        monkeypatch.setenv("GWAMD_BAND_FWD", "ad")
    else:
        monkeypatch.delenv("GWAMD_BAND_FWD", raising=False)
    if "slots" in grid:
        monkeypatch.setenv("GWAMD_POA_SLOTS", grid.split("_")[0][5:])
    else:
        monkeypatch.delenv("GWAMD_POA_SLOTS", raising=False)
    if "cus" in grid:
        monkeypatch.setenv("GWAMD_LAUNCH_ORDER_CUS", "2")
    else:
        monkeypatch.delenv("GWAMD_LAUNCH_ORDER_CUS", raising=False)
    if mode == "v1":
        monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    banded = mode.startswith("banded")
    msa = mode.endswith("msa")
    # windows of very different cost, so the heaviest-first order is not the window order
    wins = synth.poa_windows(901, 6, 120, 6, 8, 8, 8)
    wins += synth.poa_windows(911, 5, 500, 10, 25, 25, 25)
    wins += synth.poa_windows(921, 6, 250, 4, 12, 12, 12)
    wins.append([b"ACGT", b"ACGA"])
    wins.append([b"GATTACA" * 40] + [b"GATTACA" * 40 + b"T"] * 7)
    max_seq = 600
    b = run_gpu(wins, max_seq, 10, banded=banded, bw=256, output_type="msa" if msa else "consensus",
                spoa_accurate=(mode == "full_spoa"))
    slots, resident = b.get_grid()
    if mode == "v1":
        assert resident == 0 and b.kernel_variant() == 1
    elif "_ad" in mode:
        assert b.kernel_variant() == 4
    else:
        assert b.kernel_variant() in ((3, 4) if banded else (2,))
        if "slots" in grid:
            assert slots < len(wins)
    sbits = b.get_types()[0]
    for rep in range(2):
        if rep:
            b.generate_poa()
        if msa:
            got, st = b.get_msa()
        else:
            cons, cov, st = b.get_consensus()
            got = list(zip(cons, cov))
        graphs, gst = b.get_graphs()
        for i, w in enumerate(wins):
            r = run_oracle(w, max_seq, 10, banded=banded, bw=256, msa=msa, score_bits=sbits, want_graph=True,
                           spoa_accurate=(mode == "full_spoa"))
            want = r.msa if msa else (r.consensus, r.coverage)
            assert (st[i], got[i]) == (r.status, want), (mode, grid, rep, i)
            expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
            assert {(u, v): graphs[i].weight(u, v) for (u, v) in graphs[i].edges} == expect, (mode, grid, rep, i)


# Traceback move-window walk: pointer doubling and the scalar walk, over
# strip windows along the path (16 x 8 default, 32 x 4) and 16 x 8 rectangles
# (GWAMD_TB_WALK=default | scalar | rect | scalar_rect | strip32 |
# scalar_strip32) give identical
# alignments, so identical outputs, on the full-mode LDS kernel and the banded
# kernel (row-parallel and anti-diagonal forward), consensus and MSA, against
# the oracle; the windows include repeats, empty/one-base reads and reads
# shorter than the band.
@pytest.mark.parametrize("mode", ["full", "band_row", "band_ad"])
@pytest.mark.parametrize("out", ["consensus", "msa"])
def test_traceback_walk_modes(mode, out, monkeypatch):
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    banded = mode != "full"
    if banded:
        monkeypatch.setenv("GWAMD_BAND_FWD", "ad" if mode == "band_ad" else "row")
    wins = _band_ad_windows(1501)
    # full mode: the LDS kernel's shape (config B's 1,100-base windows)
    ms = 1700 if banded else 1100
    wins = [w for w in wins if max(len(r) for r in w) < ms - 60]
    msa = out == "msa"
    res = {}
    for walk in ("rank", "scalar", "rect", "scalar_rect", "strip32", "scalar_strip32"):
        monkeypatch.setenv("GWAMD_TB_WALK", walk)
        b = run_gpu(wins, ms, 60, banded=banded, bw=256, output_type=out)
        assert b.kernel_variant() == {"full": 2, "band_row": 3, "band_ad": 4}[mode]
        res[walk] = b.get_msa() if msa else b.get_consensus()
        sbits = b.get_types()[0]
    monkeypatch.delenv("GWAMD_TB_WALK", raising=False)
    monkeypatch.delenv("GWAMD_BAND_FWD", raising=False)
    assert res["rank"] == res["scalar"]
    assert res["rank"] == res["rect"]
    assert res["rank"] == res["scalar_rect"]
    assert res["rank"] == res["strip32"]
    assert res["rank"] == res["scalar_strip32"]
    for i, w in enumerate(wins):
        r = run_oracle(w, ms, 60, banded=banded, bw=256, msa=msa, score_bits=sbits)
        if msa:
            assert (res["rank"][1][i], res["rank"][0][i]) == (r.status, r.msa), i
        else:
            cons, cov, st = res["rank"]
            assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), i


# Kahn sort ring of queued info words (topsort_lds kMode 2, graphs whose
# words do not all fit LDS): GWAMD_TOPSORT_RING=1 forces it with a 4-entry
# ring; these windows queue 5-6 nodes at once (oracle graphs), so pops run
# past the ring and must fall back to the node words (a pop read a
# slot the branch-free pop had overwritten).  Forced in the LDS kernel only:
# the band kernel runs the same topsort_lds code without the runtime flag (it
# cost that kernel's register allocation).
@pytest.mark.parametrize("mode", ["full", "full_msa"])
def test_topsort_queue_ring(mode, monkeypatch):
    monkeypatch.setenv("GWAMD_TOPSORT_RING", "1")
    monkeypatch.setenv("GWAMD_TOPSORT", "fifo")  # the FIFO sort (the default is the level sort)
    banded = mode.startswith("banded")
    msa = mode.endswith("msa")
    wins = synth.poa_windows(7, 6, 300, 32, 40, 40, 40)
    max_seq = 400
    b = run_gpu(wins, max_seq, 32, banded=banded, output_type="msa" if msa else "consensus")
    sbits = b.get_types()[0]
    if msa:
        got, st = b.get_msa()
    else:
        cons, cov, st = b.get_consensus()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 32, banded=banded, msa=msa, score_bits=sbits)
        assert st[i] == r.status, i
        if msa:
            assert got[i] == r.msa, i
        else:
            assert (cons[i], cov[i]) == (r.consensus, r.coverage), i


@pytest.mark.parametrize("fwd", ["v2", "v1"])
def test_marked_rows_multi_source_fwd2(fwd, monkeypatch):
    # Pins the round-4 workaround of a ROCm 7.2 miscompile ("A
    # backend miscompile worked around"): rows marked for the general path
    # (sources, non-ACGT bases, far predecessors) read the virtual row 0 or the
    # ring through their own loader.  These windows are built to have several
    # source nodes (reads that start with bases the graph does not have, so
    # the alignment inserts them before the first node) and non-ACGT bases (N,
    # lower case), and run on the LDS kernel with the default scores, for
    # which the row-program forward pass (fwd2) is selected; GWAMD_POA_FWD=v1
    # (diagnostic) runs the round-3 pass on the same windows.  Both must equal
    # the oracle; the oracle's graphs show the windows really have >= 2 sources.
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    if fwd == "v1":
        monkeypatch.setenv("GWAMD_DIAG", "1")
        monkeypatch.setenv("GWAMD_POA_FWD", "v1")
    else:
        monkeypatch.delenv("GWAMD_POA_FWD", raising=False)
    import random
    rng = random.Random(5)
    wins = []
    for k in range(12):
        bb = "".join(rng.choice("ACGT") for _ in range(300 + 40 * k))
        reads = [bb]
        for j in range(10):
            r = list(bb[rng.randrange(0, 20):len(bb) - rng.randrange(0, 20)])
            for _ in range(12):
                p = rng.randrange(len(r))
                r[p] = rng.choice("ACGTN" if j % 3 == 0 else "ACGT")
            head = "".join(rng.choice("ACGT") for _ in range(rng.randrange(3, 30))) if j % 2 == 0 else ""
            reads.append((head + "".join(r)).encode())
        reads[0] = reads[0].encode()
        if k % 4 == 3:
            reads[3] = reads[3].lower()  # lower-case bases are not ACGT either
        wins.append(reads)
    b = run_gpu(wins, 900, 12)
    assert b.kernel_variant() == 2
    cons, cov, st = b.get_consensus()
    multi = 0
    for i, w in enumerate(wins):
        r = run_oracle(w, 900, 12, want_graph=True)
        assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (fwd, i)
        multi += sum(1 for ins in r.graph["in"] if not ins) >= 2
    assert multi >= 10


@pytest.mark.parametrize("shape", ["fwd2", "v1", "int32"])
def test_non_ascii_bases_compared_whole(shape, monkeypatch):
    # The LDS kernel's row records keep 7 bits of the base (bit 7 is the
    # general-path flag); 0x7f stands for 0x7f and every byte >= 0x80, and
    # the forward passes read those rows' base back from the graph, because
    # the reference compares whole bytes (0xc1 is not 'A').  Reads carry such
    # bytes; the graphs (edges and weights: the alignments decide them) must
    # equal the oracle's on the 16-bit row-program pass, the round-3 pass and
    # the 32-bit pass.
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    monkeypatch.delenv("GWAMD_POA_FWD", raising=False)
    if shape == "v1":
        monkeypatch.setenv("GWAMD_POA_FWD", "v1")
    import random
    rng = random.Random(9)
    odd = [0xc1, 0xc3, 0xc7, 0xd4, 0x7f, 0xe1, 0x81]
    wins = []
    for k in range(8):
        bb = bytearray(rng.choice(b"ACGT") for _ in range(250 + 30 * k))
        for _ in range(len(bb) // 12):
            bb[rng.randrange(len(bb))] = rng.choice(odd)
        reads = [bytes(bb)]
        for j in range(9):
            r = bytearray(bb[rng.randrange(0, 10):len(bb) - rng.randrange(0, 10)])
            for _ in range(10):
                r[rng.randrange(len(r))] = rng.choice(odd if j % 2 else b"ACGT")
            reads.append(bytes(r))
        wins.append(reads)
    max_seq = 1600 if shape == "int32" else 600
    b = run_gpu(wins, max_seq, 10)
    sbits = b.get_types()[0]
    assert b.kernel_variant() == 2 and sbits == (32 if shape == "int32" else 16)
    graphs, _ = b.get_graphs()
    for i, w in enumerate(wins):
        r = run_oracle(w, max_seq, 10, score_bits=sbits, want_graph=True)
        g = graphs[i]
        expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
        assert {(u, v): g.weight(u, v) for (u, v) in g.edges} == expect, (shape, i)


@pytest.mark.parametrize("spoa", [False, True])
def test_full_int32_persistent_grid(spoa, monkeypatch):
    # the 32-bit LDS kernel on a persistent grid of 3 slots (workgroups reuse
    # their slot's scratch across windows, heaviest first), two generates,
    # SPOA_ACCURATE on and off, final graphs against the oracle
    monkeypatch.delenv("GWAMD_POA_KERNEL", raising=False)
    monkeypatch.setenv("GWAMD_DIAG", "1")
    monkeypatch.setenv("GWAMD_POA_SLOTS", "3")
    wins = synth.poa_windows(841, 4, 900, 8, 40, 40, 40)
    wins += synth.poa_windows(851, 4, 200, 6, 10, 10, 10)
    b = run_gpu(wins, 1600, 8, spoa_accurate=spoa)
    slots, _ = b.get_grid()
    assert b.get_types()[0] == 32 and b.kernel_variant() == 2 and slots < len(wins)
    for rep in range(2):
        if rep:
            b.generate_poa()
        cons, cov, st = b.get_consensus()
        graphs, gst = b.get_graphs()
        for i, w in enumerate(wins):
            r = run_oracle(w, 1600, 8, score_bits=32, want_graph=True, spoa_accurate=spoa)
            assert (st[i], cons[i], cov[i]) == (r.status, r.consensus, r.coverage), (rep, i)
            expect = {(src, v): wt for v, ins in enumerate(r.graph["in"]) for (src, wt) in ins}
            assert {(u, v): graphs[i].weight(u, v) for (u, v) in graphs[i].edges} == expect, (rep, i)

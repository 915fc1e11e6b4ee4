"""Overlap alignment (cudamapper/src/main.cu:48-175), PAF output
(cudamapper/src/cudamapper_utils.cpp:30-112) and the FASTA reader
(common/io/src/kseqpp_fasta_parser.cpp:31-72) over include/gwamd_cudamapper.h.

CPU: the PAF text against a restatement of print_paf's format string, the
reader's filtering/ordering, and argument validation (it fails before touching
the GPU).  GPU: every CIGAR equals the aligner oracle's on the same region,
with the target reverse-complemented for '-' overlaps."""
import random

import pytest

from claragenomicsanalysis_amd import cudamapper as cm

COMP = {"A": "T", "T": "A", "C": "G", "G": "C"}


def rc(s):
    return "".join(COMP.get(c, c) for c in reversed(s))


def paf_line(o, cigar, qname, qlen, tname, tlen, k):
    # cudamapper_utils.cpp:74-96 ("%s\t%lu\t%i\t%i\t%c\t%s\t%lu\t%i\t%i\t%i\t%ld\t%i" + "\tcg:Z:%s")
    span = max(abs(o.target_start - o.target_end), abs(o.query_start - o.query_end))
    s = "%s\t%d\t%d\t%d\t%s\t%s\t%d\t%d\t%d\t%d\t%d\t%d" % (qname, qlen, o.query_start, o.query_end, o.strand,
                                                          tname, tlen, o.target_start, o.target_end,
                                                          o.num_residues * k, span, 255)
    if cigar is not None:
        s += "\tcg:Z:" + cigar
    return s + "\n"


def test_paf_format_matches_print_paf():
    rng = random.Random(5)
    q = [("read_q%d" % i, rng.randint(100, 900)) for i in range(5)]
    t = [("read_t%d" % i, rng.randint(100, 900)) for i in range(4)]
    ovs, cig = [], []
    for i in range(20):
        qi, ti = rng.randrange(5), rng.randrange(4)
        qs = rng.randrange(q[qi][1] // 2)
        ts = rng.randrange(t[ti][1] // 2)
        ovs.append(cm.Overlap(qi, ti, qs, rng.randint(qs, q[qi][1]), ts, rng.randint(ts, t[ti][1]),
                              rng.choice("+-"), rng.randrange(100)))
        cig.append("%dM%dI" % (rng.randrange(1, 99), rng.randrange(1, 9)))
    for k in (15, 1):
        got = cm.format_paf(ovs, cig, q, t, k)
        assert got == "".join(paf_line(o, c, q[o.query_read_id][0], q[o.query_read_id][1],
                                       t[o.target_read_id][0], t[o.target_read_id][1], k)
                              for o, c in zip(ovs, cig))
        got = cm.format_paf(ovs, None, q, t, k)
        assert got == "".join(paf_line(o, None, q[o.query_read_id][0], q[o.query_read_id][1],
                                       t[o.target_read_id][0], t[o.target_read_id][1], k) for o in ovs)
    assert cm.format_paf([], None, q, t, 15) == ""


def test_paf_rejects_mismatched_cigars_and_ids():
    q, t = [("q", 10)], [("t", 10)]
    with pytest.raises(ValueError):
        cm.format_paf([cm.Overlap(0, 0, 0, 5, 0, 5)], ["5M", "1M"], q, t, 15)
    with pytest.raises(ValueError):
        cm.format_paf([cm.Overlap(0, 3, 0, 5, 0, 5)], None, q, t, 15)
    with pytest.raises(ValueError):
        cm.format_paf([cm.Overlap(0, 0, 0, 5, 0, 5, "x")], None, q, t, 15)


def test_read_fasta(tmp_path):
    p = tmp_path / "r.fa"
    recs = [("r%d" % i, "ACGT" * (i + 1) + "A" * i) for i in range(12)]
    with open(p, "w") as f:
        for n, s in recs:
            f.write(">%s some description\n" % n)
            for k in range(0, len(s), 7):
                f.write(s[k:k + 7] + "\n")
    assert cm.read_fasta(p, shuffle=False) == recs
    assert cm.read_fasta(p, min_sequence_length=30, shuffle=False) == [r for r in recs if len(r[1]) >= 30]
    sh = cm.read_fasta(p)
    assert sorted(sh) == sorted(recs) and sh != recs  # a permutation, deterministic
    assert cm.read_fasta(p) == sh
    fq = tmp_path / "r.fq"
    with open(fq, "w") as f:
        for n, s in recs[:3]:
            f.write("@%s\n%s\n+\n%s\n" % (n, s, "@" * len(s)))
    assert cm.read_fasta(fq, shuffle=False) == recs[:3]
    with pytest.raises(ValueError):
        cm.read_fasta(tmp_path / "missing.fa")
    (tmp_path / "empty.fa").write_text("")
    with pytest.raises(ValueError):
        cm.read_fasta(tmp_path / "empty.fa")


def test_align_overlaps_validation():
    q, t = ["ACGTACGTAC"], ["ACGTACGTAC"]
    assert cm.align_overlaps([], q, t) == []
    with pytest.raises(ValueError):  # query range past the read
        cm.align_overlaps([cm.Overlap(0, 0, 0, 11, 0, 5)], q, t)
    with pytest.raises(ValueError):  # start after end
        cm.align_overlaps([cm.Overlap(0, 0, 6, 5, 0, 5)], q, t)
    with pytest.raises(ValueError):  # unknown read id
        cm.align_overlaps([cm.Overlap(0, 1, 0, 5, 0, 5)], q, t)


def _mutate(rng, s, err):
    out = []
    for c in s:
        r = rng.random()
        if r < err / 3:
            continue
        if r < 2 * err / 3:
            out.append(rng.choice("ACGT"))
        elif r < err:
            out.append(c)
            out.append(rng.choice("ACGT"))
        else:
            out.append(c)
    return "".join(out)


def _dataset(seed, nreads, nov, lo, hi):
    rng = random.Random(seed)
    targets = ["".join(rng.choice("ACGT") for _ in range(rng.randint(lo, hi))) for _ in range(nreads)]
    queries, ovs = [], []
    for i in range(nov):
        ti = rng.randrange(nreads)
        t = targets[ti]
        ts = rng.randrange(len(t) // 3)
        te = rng.randint(ts + len(t) // 2, len(t))
        strand = rng.choice("+-")
        region = t[ts:te] if strand == "+" else rc(t[ts:te])
        pre = "".join(rng.choice("ACGT") for _ in range(rng.randrange(50)))
        body = _mutate(rng, region, 0.08)
        queries.append(pre + body + "".join(rng.choice("ACGT") for _ in range(rng.randrange(50))))
        ovs.append(cm.Overlap(i, ti, len(pre), len(pre) + len(body), ts, te, strand, rng.randrange(200)))
    return queries, targets, ovs


@pytest.mark.gpu
@pytest.mark.parametrize("engines", [1, 3])
def test_align_overlaps_matches_oracle(engines):
    from oracle import oracle
    queries, targets, ovs = _dataset(11 + engines, 6, 40, 300, 2500)
    cigars = cm.align_overlaps(ovs, queries, targets, num_alignment_engines=engines)
    assert len(cigars) == len(ovs)
    mq = max(o.query_end - o.query_start for o in ovs)
    for o, c in zip(ovs, cigars):
        qr = queries[o.query_read_id][o.query_start:o.query_end]
        tr = targets[o.target_read_id][o.target_start:o.target_end]
        if o.strand == "-":
            tr = rc(tr)
        assert c == oracle.cigar(oracle.align(qr, tr, oracle.ALIGN_HM, mq))
    paf = cm.format_paf(ovs, cigars, [("q%d" % i, s) for i, s in enumerate(queries)],
                        [("t%d" % i, s) for i, s in enumerate(targets)], 15)
    assert paf.count("\tcg:Z:") == len(ovs)


@pytest.mark.gpu
def test_align_overlaps_more_engines_than_overlaps():
    # the reference's batch size would be 0 here (and its engines would spin);
    # this build aligns at least one overlap per batch
    from oracle import oracle
    queries, targets, ovs = _dataset(7, 2, 2, 200, 400)
    cigars = cm.align_overlaps(ovs, queries, targets, num_alignment_engines=4)
    mq = max(o.query_end - o.query_start for o in ovs)
    for o, c in zip(ovs, cigars):
        tr = targets[o.target_read_id][o.target_start:o.target_end]
        qr = queries[o.query_read_id][o.query_start:o.query_end]
        assert c == oracle.cigar(oracle.align(qr, rc(tr) if o.strand == "-" else tr, oracle.ALIGN_HM, mq))


@pytest.mark.gpu
def test_align_overlaps_long_overlap_gets_its_cigar():
    # an overlap longer than 16,384 query / 65,535 target bases (round 2's
    # limits) takes the long-mode Hirschberg-Myers kernel (striped sweeps,
    # patterns in HBM) and gets the same CIGAR as the oracle, like the
    # reference's cudamapper -a (main.cu:48-122), which has no length limit
    from oracle import oracle
    queries, targets, ovs = _dataset(23, 3, 6, 300, 1500)
    rng = random.Random(5)
    big_t = "".join(rng.choice("ACGT") for _ in range(70000))
    big_q = _mutate(rng, big_t[:20000], 0.03)
    targets.append(big_t)
    queries.append(big_q)
    ovs.append(cm.Overlap(len(queries) - 1, len(targets) - 1, 0, len(big_q), 0, len(big_t), "+", 10))
    cigars = cm.align_overlaps(ovs, queries, targets, num_alignment_engines=2)
    mq = max(o.query_end - o.query_start for o in ovs)
    for o, c in zip(ovs, cigars):
        qr = queries[o.query_read_id][o.query_start:o.query_end]
        tr = targets[o.target_read_id][o.target_start:o.target_end]
        assert c and c == oracle.cigar(oracle.align(qr, rc(tr) if o.strand == "-" else tr, oracle.ALIGN_HM, mq))
    paf = cm.format_paf(ovs, cigars, [("q%d" % i, s) for i, s in enumerate(queries)],
                        [("t%d" % i, s) for i, s in enumerate(targets)], 15)
    assert all("cg:Z:" in ln for ln in paf.splitlines())

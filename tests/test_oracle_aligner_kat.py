"""The aligner oracle against the reference's own known answers
(tests/golden/aligner_kat.json) and size-independent properties; CPU only."""
import json
import os
import random

import pytest

from oracle import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aligner_kat.json")))


@pytest.mark.parametrize("case", GOLD["cigar"], ids=lambda c: c["source"])
def test_cigar_kats(case):
    for p in case["pairs"]:
        hm = oracle.align(p["query"], p["target"], oracle.ALIGN_HM, case["max_query_length"])
        assert oracle.cigar(hm) == p["cigar"], p
        if "myers" in case["algorithms"]:
            assert oracle.cigar(oracle.align(p["query"], p["target"], oracle.ALIGN_MYERS)) == p["cigar"], p


@pytest.mark.parametrize("case", GOLD["patterns"], ids=lambda c: "%d%s%d" % (c["word"], c["letter"], c["reverse"]))
def test_query_pattern_kats(case):
    assert oracle.query_pattern(case["query"], case["letter"], case["word"], case["reverse"]) == case["value"]


@pytest.mark.parametrize("case", GOLD["distances"], ids=range(len(GOLD["distances"])))
def test_distance_kats(case):
    assert oracle.edit_distance(case["query"], case["target"]) == case["distance"]


def _cost(q, t, states):
    qi = ti = cost = 0
    for s in states:
        if s in (0, 1):
            assert (s == 0) == (q[qi] == "ACTG"[(ord(t[ti]) >> 1) & 3])
            cost += s
            qi += 1
            ti += 1
        elif s == 2:
            cost += 1
            ti += 1
        else:
            cost += 1
            qi += 1
    assert qi == len(q) and ti == len(t)
    return cost


def _mutate(rng, s, n):
    s = list(s)
    for _ in range(n):
        k = rng.randrange(3)
        p = rng.randrange(len(s) + 1)
        if k == 0 and p < len(s):
            s[p] = rng.choice("ACGT")
        elif k == 1:
            s.insert(p, rng.choice("ACGT"))
        elif p < len(s):
            del s[p]
    return "".join(s)


@pytest.mark.parametrize("seed", range(6))
def test_hirschberg_path_is_optimal(seed):
    # Hirschberg-Myers recursion (query >= 63 splits): the path consumes both
    # strings and its cost is the edit distance
    rng = random.Random(seed)
    t = "".join(rng.choice("ACGT") for _ in range(rng.randrange(100, 700)))
    q = _mutate(rng, t, len(t) // 8)
    for algo in (oracle.ALIGN_HM, oracle.ALIGN_MYERS):
        st = oracle.align(q, t, algo, max(len(q), len(t)))
        assert _cost(q, t, st) == oracle.edit_distance(q, t)


def test_hm_small_workspace_splits_more():
    # with a tiny max_query_length the full-Myers base case is skipped more
    # often (workspace (T+1)*words <= ceil(maxQ/4)*64); result stays optimal
    rng = random.Random(7)
    t = "".join(rng.choice("ACGT") for _ in range(300))
    q = _mutate(rng, t, 30)
    a = oracle.align(q, t, oracle.ALIGN_HM, 4)
    assert _cost(q, t, a) == oracle.edit_distance(q, t)


def test_empty_inputs():
    assert oracle.align("", "ACGT") == [2, 2, 2, 2]
    assert oracle.align("ACG", "") == [3, 3, 3]
    assert oracle.align("", "") == []
    assert oracle.cigar([]) == ""


def test_format_alignment():
    st = oracle.align("ACTGA", "GCTAG", oracle.ALIGN_HM, 6)
    q, p, t = oracle.format_alignment("ACTGA", "GCTAG", st)
    assert len(q) == len(p) == len(t) == len(st)
    assert q.replace("-", "") == "ACTGA" and t.replace("-", "") == "GCTAG"

"""Pins the CPU restatement (oracle/) against the reference's own known-answer
vectors for the POA path (tests/golden/poa_kat.json, see make_golden.py)."""
import json
import os

import pytest

from oracle import oracle

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "poa_kat.json")))


@pytest.mark.parametrize("case", GOLD["topsort"], ids=lambda c: str(c["answer"]))
def test_topsort_kat(case):
    # Test_CudapoaTopSort.cu:37-58
    assert oracle.topsort(case["outgoing"]) == case["answer"]


@pytest.mark.parametrize("case", GOLD["nw"], ids=lambda c: c["read"])
def test_nw_kat(case):
    # Test_CudapoaNW.cu:76-180
    ag, ar = oracle.nw(case["nodes"], case["sorted"], case["outgoing"], case["read"])
    assert ag == case["graph"]
    assert ar == case["readpos"]


@pytest.mark.parametrize("case", GOLD["add_alignment"], ids=lambda c: c["read"])
def test_add_alignment_kat(case):
    # Test_CudapoaAddAlignment.cu:104-224
    st, outs = oracle.add_alignment(case["nodes"], case["edges"], case["aligned"], case["coverage"],
                                    case["read"], case["graph"], case["readpos"])
    assert st == 0
    assert outs == case["answer"]


@pytest.mark.parametrize("case", GOLD["consensus"], ids=lambda c: c["answer"])
def test_consensus_kat(case):
    # Test_CudapoaGenerateConsensus.cu:77-156 (raw kernel output, reversed)
    st, cons = oracle.consensus_raw(case["nodes"], case["sorted"], case["aligned"], case["outgoing"],
                                    case["coverage"], case["weights"])
    assert st == 0
    assert cons == case["answer"]


def _batch(name):
    return [b for b in GOLD["batch"] if b["name"] == name][0]


def test_all_A_batch():
    # Test_CudapoaBatch.cu:151-203
    case = _batch("all_A_1023x3")
    r = oracle.poa_window(case["windows"][0], max_nodes=3072, max_consensus=2048)
    assert r.status == 0
    assert r.consensus == case["consensus"][0]


def test_python_graph_shape():
    # pygenomeworks test_cudapoa_bindings.py:95-120
    case = _batch("py_graph")
    r = oracle.poa_window(case["windows"][0], max_nodes=3072, max_consensus=2048, want_graph=True)
    assert r.status == 0
    assert r.final_nodes == case["graph_nodes"][0]
    assert sum(len(e) for e in r.graph["in"]) == case["graph_edges"][0]


def test_python_complex_seed2():
    # pygenomeworks test_cudapoa_bindings.py:122-146
    case = _batch("py_complex_seed2")
    r = oracle.poa_window(case["windows"][0], max_nodes=3072, max_consensus=2048, max_seqs=1000)
    assert r.status == 0
    assert r.consensus == case["consensus"][0]


def test_python_simple_two_windows():
    case = _batch("py_simple")
    outs = [oracle.poa_window(w, max_nodes=3072, max_consensus=2048) for w in case["windows"]]
    assert len(outs) == case["n_consensus"]
    assert all(o.status == 0 and len(o.consensus) > 0 for o in outs)

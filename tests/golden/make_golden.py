"""Writes the known-answer fixtures the reference's own tests hold for the POA
path into tests/golden/poa_kat.json.

Every vector below is data (inputs and expected outputs) transcribed from the
cited reference test file; no reference source is reproduced.  Re-run with
``python tests/golden/make_golden.py`` (needs no GPU and no reference tree).
"""
import json
import os
import random

HERE = os.path.dirname(os.path.abspath(__file__))


def topsort_cases():
    # cudapoa/tests/Test_CudapoaTopSort.cu:43-56  (outgoing edge lists, answer)
    return [
        {"outgoing": [[], [], [3], [1], [0, 1], [0, 2]], "answer": [4, 5, 0, 2, 3, 1]},
        {"outgoing": [[1, 3], [2, 3], [3, 4, 5], [4, 5], [5], []], "answer": [0, 1, 2, 3, 4, 5]},
        {"outgoing": [[], [], [3], [1], [0, 1, 7], [0, 2], [4], [5]], "answer": [6, 4, 7, 5, 0, 2, 3, 1]},
    ]


def nw_cases():
    # cudapoa/tests/Test_CudapoaNW.cu:92-177 (nodes, sorted graph, outgoing edges,
    # read; expected reversed alignment_graph / alignment_read); scores -8/-6/8
    return [
        {"nodes": "AAAA", "sorted": [0, 1, 2, 3], "outgoing": [[1], [2], [3], []], "read": "AATA",
         "graph": [3, 2, 1, 0], "readpos": [3, 2, 1, 0]},
        {"nodes": "ATCG", "sorted": [0, 1, 2, 3], "outgoing": [[1], [2], [3], []], "read": "ATCGA",
         "graph": [-1, 3, 2, 1, 0], "readpos": [4, 3, 2, 1, 0]},
        {"nodes": "AACGC", "sorted": [0, 4, 1, 2, 3], "outgoing": [[1, 4], [2], [3], [], [2]], "read": "ATCG",
         "graph": [3, 2, 1, 0], "readpos": [3, 2, 1, 0]},
        {"nodes": "ATTGA", "sorted": [0, 1, 2, 3, 4], "outgoing": [[1], [2], [3], [4], []], "read": "AA",
         "graph": [4, 3, 2, 1, 0], "readpos": [1, -1, -1, -1, 0]},
        {"nodes": "ATGTACA", "sorted": [0, 5, 1, 6, 2, 3, 4],
         "outgoing": [[1, 5], [2], [3], [4], [], [6], [3]], "read": "ACTTA",
         "graph": [4, 3, 6, 5, 0], "readpos": [4, 3, 2, 1, 0]},
    ]


def add_alignment_cases():
    # cudapoa/tests/Test_CudapoaAddAlignment.cu:104-222.  Graph edges are given
    # in the test's (incoming-looking) orientation and loaded through
    # BasicGraph::get_edges (basic_graph.hpp:70-85); "answer" is the expected
    # edge structure in the same orientation.  Base weights are never copied
    # into the kernel buffer by the test harness (basic member left empty), so
    # the weights are all zero (Test_CudapoaAddAlignment.cu:30-98).
    return [
        {"nodes": "AAAA", "edges": [[], [0], [1], [2]], "aligned": [[], [], [], []], "coverage": [1, 1, 1, 1],
         "read": "AATA", "graph": [0, 1, 2, 3], "readpos": [0, 1, 2, 3],
         "answer": [[], [0], [1], [2, 4], [1]]},
        {"nodes": "ATCG", "edges": [[], [0], [1], [2]], "aligned": [[], [], [], []], "coverage": [1, 1, 1, 1],
         "read": "ATCGA", "graph": [0, 1, 2, 3, -1], "readpos": [0, 1, 2, 3, 4],
         "answer": [[], [0], [1], [2], [3]]},
        {"nodes": "AACGC", "edges": [[], [0], [1, 4], [2], [0]], "aligned": [[], [], [], []],
         "coverage": [2, 1, 2, 2, 1], "read": "ATCG", "graph": [0, 4, 2, 3], "readpos": [0, 1, 2, 3],
         "answer": [[], [0], [1, 4, 5], [2], [0], [0]]},
        {"nodes": "ATTGA", "edges": [[], [0], [1], [2], [3]], "aligned": [[], [], [], []],
         "coverage": [1, 1, 1, 1, 1], "read": "AA", "graph": [0, 1, 2, 3, 4], "readpos": [0, -1, -1, -1, 1],
         "answer": [[], [0], [1], [2], [3, 0]]},
        {"nodes": "ATGTACA", "edges": [[], [0], [1], [2, 6], [3], [0], [5]], "aligned": [[], [], [], []],
         "coverage": [2, 1, 1, 2, 2, 1, 1], "read": "ACTTA", "graph": [0, 5, 6, 3, 4],
         "readpos": [0, 1, 2, 3, 4], "answer": [[], [0], [1], [2, 6, 7], [3], [0], [5], [5]]},
    ]


def consensus_cases():
    # cudapoa/tests/Test_CudapoaGenerateConsensus.cu:77-154 (nodes, sorted graph,
    # node alignments, outgoing edges, node coverage, outgoing edge weights;
    # expected raw kernel output, i.e. the consensus written backwards).
    return [
        {"nodes": "AAAAT", "sorted": [0, 1, 2, 4, 3], "aligned": [[], [], [4], [], [2]],
         "outgoing": [[1], [2, 4], [3], [], [3]], "coverage": [2, 2, 1, 2, 1],
         "weights": [[5], [4, 3], [2], [], [1]], "answer": "ATAA"},
        {"nodes": "ATCGA", "sorted": [0, 1, 2, 3, 4], "aligned": [[], [], [], [], []],
         "outgoing": [[1], [2], [3], [4], []], "coverage": [1, 1, 1, 1, 1],
         "weights": [[4], [3], [2], [1], []], "answer": "AGCTA"},
        {"nodes": "AACGCT", "sorted": [0, 1, 4, 5, 2, 3], "aligned": [[], [4, 5], [], [], [1, 5], [1, 4]],
         "outgoing": [[1, 4, 5], [2], [3], [], [2], [2]], "coverage": [3, 1, 3, 3, 1, 1],
         "weights": [[7, 6, 5], [4], [3], [], [2], [1]], "answer": "GCCA"},
        {"nodes": "ATTGA", "sorted": [0, 1, 2, 3, 4], "aligned": [[], [], [], [], []],
         "outgoing": [[1, 4], [2], [3], [4], []], "coverage": [2, 1, 1, 1, 2],
         "weights": [[5, 4], [3], [2], [1], []], "answer": "AGTTA"},
        {"nodes": "ATGTACAT", "sorted": [0, 1, 5, 2, 6, 7, 3, 4],
         "aligned": [[], [5], [6, 7], [], [], [1], [2, 7], [2, 6]],
         "outgoing": [[1, 5], [2], [3], [4], [], [6, 7], [3], [3]], "coverage": [3, 1, 1, 3, 3, 2, 1, 1],
         "weights": [[9, 8], [7], [6], [5], [], [4, 3], [2], [1]], "answer": "ATTCA"},
    ]


def batch_cases():
    out = []
    # cudapoa/tests/Test_CudapoaBatch.cu:151-203: three identical 1023-base
    # all-A reads, BatchSize(1024, 10) -> consensus equals the read.
    out.append({"name": "all_A_1023x3", "max_seq": 1024, "max_seqs_per_poa": 10,
                "windows": [["A" * 1023] * 3], "consensus": ["A" * 1023]})
    # pygenomeworks/test/test_cudapoa_bindings.py:95-120: three reads -> graph of
    # 10 nodes and 11 edges.
    out.append({"name": "py_graph", "max_seq": 1024, "max_seqs_per_poa": 10,
                "windows": [["ACTGACTG", "ACTTACTG", "ACTCACTG"]], "graph_nodes": [10], "graph_edges": [11]})
    # test_cudapoa_bindings.py:122-146: random.seed(2), 100 reads of 500 bases at
    # a 2% substitution rate; the consensus must equal the reference string.
    random.seed(2)
    read_len = 500
    ref = ''.join([random.choice(['A', 'C', 'G', 'T']) for _ in range(read_len)])
    reads = []
    for _ in range(100):
        reads.append(''.join([r if random.random() > 0.02 else random.choice(['A', 'C', 'G', 'T']) for r in ref]))
    out.append({"name": "py_complex_seed2", "max_seq": 1024, "max_seqs_per_poa": 1000,
                "windows": [reads], "consensus": [ref]})
    # test_cudapoa_bindings.py:19-37: two small groups -> two consensus strings.
    out.append({"name": "py_simple", "max_seq": 1024, "max_seqs_per_poa": 10,
                "windows": [["ACTGACTG", "ACTTACTG", "ACGGACTG", "ATCGACTG"],
                            ["ACTGAC", "ACTTAC", "ACGGAC", "ATCGAC"]], "n_consensus": 2})
    return out


def main():
    data = {
        "source": "GenomeWorks 0.5.0 reference tests (see make_golden.py for file:line)",
        "scores": {"gap": -8, "mismatch": -6, "match": 8},
        "topsort": topsort_cases(),
        "nw": nw_cases(),
        "add_alignment": add_alignment_cases(),
        "consensus": consensus_cases(),
        "batch": batch_cases(),
    }
    with open(os.path.join(HERE, "poa_kat.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("wrote poa_kat.json")


if __name__ == "__main__":
    main()

"""Writes the known-answer fixtures the reference's own tests hold for the
cudaaligner path into tests/golden/aligner_kat.json.

Vectors are data transcribed from the cited reference test files (inputs and
expected outputs); the edit distances of the fixed pairs are recomputed here
with a plain-Python naive NW (the reference test's own yardstick,
Test_MyersAlgorithm.cpp:28-61 vs needleman_wunsch_cpu.cpp:100-119).
Re-run with ``python tests/golden/make_aligner_golden.py``.
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def cigar_cases():
    out = []
    # cudaaligner/tests/Test_AlignerGlobal.cpp:95-141: each test case is one
    # aligner with max lengths = longest string in the case + 1 (:170-186)
    groups = [
        [("AAAA", "TTAT", "4M")],
        [("ATAAAAAAAA", "AAAAAAAAA", "1M1D8M")],
        [("AAAAAAAAA", "ATAAAAAAAA", "1M1I8M")],
        [("ACTGA", "GCTAG", "3M1D1M1I")],
        [("ACTGA", "GCTAG", "3M1D1M1I"), ("ACTG", "ACTG", "4M"), ("A", "T", "1M")],
    ]
    six = [("AAAA", "TTAT", "4M"), ("ATAAAAAAAA", "AAAAAAAAA", "1M1D8M"), ("AAAAAAAAA", "ATAAAAAAAA", "1M1I8M"),
           ("ACTGA", "GCTAG", "3M1D1M1I"), ("ACTGA", "GCTAG", "3M1D1M1I"), ("ACTG", "ACTG", "4M"), ("A", "T", "1M")]
    groups.append(six * 4)
    for gi, g in enumerate(groups):
        ms = max(max(len(q), len(t)) for q, t, _ in g) + 1
        out.append({"source": "Test_AlignerGlobal.cpp case %d" % (gi + 1), "max_query_length": ms,
                    "max_target_length": ms, "pairs": [{"query": q, "target": t, "cigar": c} for q, t, c in g],
                    "algorithms": ["default", "hirschberg_myers", "myers", "myers_banded", "ukkonen"]})
    # pygenomeworks/test/test_cudaaligner_bindings.py:28-31 (the xfail case is omitted)
    for q, t, c in [("AAAAAAA", "TTTTTTT", "7M"), ("AAATC", "TACGTTTT", "3M1I2M2I"), ("TACGTA", "ACATAC", "1D5M1I"),
                    ("TGCA", "ATACGCT", "1I1M2I3M")]:
        out.append({"source": "test_cudaaligner_bindings.py:28-31", "max_query_length": len(q),
                    "max_target_length": len(t), "pairs": [{"query": q, "target": t, "cigar": c}],
                    "algorithms": ["default"]})
    return out


def formatted_cases():
    # cudaaligner/tests/Test_AlignmentImpl.cpp:54-127: query, target, the
    # AlignmentState sequence (0 match, 1 mismatch, 2 insertion, 3 deletion;
    # cudaaligner.hpp:46-52), the formatted triple and the CIGAR
    M, X, I, D = 0, 1, 2, 3
    return [
        {"query": "AAAA", "target": "TTATG", "states": [X, X, M, X, I],
         "formatted": ["AAAA-", "xx|x ", "TTATG"], "cigar": "4M1I"},
        {"query": "CGATAATG", "target": "CATAA", "states": [D, X, M, M, M, M, D, D],
         "formatted": ["CGATAATG", " x||||  ", "-CATAA--"], "cigar": "1D5M2D"},
        {"query": "GTTAG", "target": "AAGTCTAGAA", "states": [I, I, M, M, I, M, M, M, I, I],
         "formatted": ["--GT-TAG--", "  || |||  ", "AAGTCTAGAA"], "cigar": "2I2M1I3M2I"},
        {"query": "GTTACA", "target": "GATTCA", "states": [M, I, M, M, D, M, M],
         "formatted": ["G-TTACA", "| || ||", "GATT-CA"], "cigar": "1M1I2M1D2M"},
    ]


def pattern_cases():
    # cudaaligner/tests/Test_HirschbergMyers.cu:93-140 (A=0, C=1, T=2, G=3; +4 reverse)
    q = "AACCGGTTACGTACGT" "AAACCCGGGTTTACGT" "AAACCCGGGTTTACG"
    w = {
        (0, 0): "00010000000001110001000100000011", (0, 1): "00100000001110000010001000001100",
        (0, 2): "10001110000000001000100011000000", (0, 3): "01000001110000000100010000110000",
        (1, 0): "001000000000111", (1, 1): "010000000111000", (1, 2): "000111000000000", (1, 3): "100000111000000",
        (0, 4): "01110000000001000111000000000100", (0, 5): "00001110000000100000111000000010",
        (0, 6): "10000000001110001000000000111000", (0, 7): "00000001110000010000000111000001",
        (1, 4): "110000001000100", (1, 5): "001100000100010", (1, 6): "000000110001000", (1, 7): "000011000010001",
    }
    letters = "ACTG"
    return [{"query": q, "word": k[0], "letter": letters[k[1] % 4], "reverse": k[1] >= 4, "value": int(v, 2)}
            for k, v in sorted(w.items())]


def naive_nw(t, q):
    m, n = len(q), len(t)
    prev = list(range(n + 1))
    for i in range(1, m + 1):
        cur = [i] + [0] * n
        for j in range(1, n + 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (0 if q[i - 1] == t[j - 1] else 1))
        prev = cur
    return prev[n]


def distance_cases():
    # cudaaligner/tests/cudaaligner_test_cases.cpp:38-80 (the fixed pairs)
    pairs = [
        ("AAAAAAAAAA", "CGTCGTCGTC"), ("AATAATAATA", "CGTCGTCGTC"), ("AATAATAATA", ""), ("", "CGTCGTCGTC"),
        ("AATAATAATA", "C"), ("CGTCGTCGTC", "CGTCGTCGTC"),
        ("CGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGT", "AGTCGTCGTCCGTAATCGTCCGTCGTCGTCGA"),
        ("CGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTC", "AGTCGTCGTCCGTAATCGTCCGTCGTCGTCGTA"),
        ("GTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTCGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTCGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTC",
         "GTCGTCGTCCGTCGTCGTCCGTCGTCGTCGAAAACGTCGTCCGTCGTCGTCCGTCGTCGAAAACGTCGTCGTCCGTAGTCGTCCGACGTCGTCGTC"),
        ("GTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTCGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTCGTCGTCGTCCGTCGTCGTCCGTCGTCGTCGTC",
         "A" * 96),
    ]
    return [{"target": t, "query": q, "distance": naive_nw(t, q)} for t, q in pairs]


def ukkonen_cases():
    # cudaaligner/tests/Test_NeedlemanWunschImplementation.cpp:40-91: (target,
    # query, p); the reference checks the banded score matrix against the naive
    # one inside the band and the CPU and GPU Ukkonen backtraces against each
    # other (:194-206, :280-286).  The distance is the naive NW's.
    pairs = [("ACTG", "ACTG", 0), ("ACTG", "ATCG", 3), ("ACTG", "ATG", 2), ("ACTG", "", 0), ("ACTGGTCA", "ACTG", 4),
             ("ACTG", "BDEF", 4)]
    return [{"target": t, "query": q, "p": p, "distance": naive_nw(t, q)} for t, q, p in pairs]


def add_cases():
    # cudaaligner/tests/Test_AlignerGlobal.cpp:58-83: aligner(10, 10, 5)
    return {"max_query_length": 10, "max_target_length": 10, "max_alignments": 5,
            "calls": [["ATCG", "TACG", 0], ["ATCG", "TACG", 0], ["ATCG", "TACG", 0],
                      ["ATCGATTACGC", "TACGTACGGA", 3], ["ATCGATTACG", "ATACGTAGCGA", 3],
                      ["ATCG", "TACG", 0], ["ATCG", "TACG", 0], ["ATCG", "TACG", 2]],
            "final_count": 5}


def add_cases_ukkonen():
    # Test_AlignerGlobal.cpp:58-83 runs on AlignerGlobalUkkonen(10, 10, 5): the
    # length-difference check (|q - t| > int(10 * 0.1f) = 1 ->
    # exceeded_max_alignment_difference, aligner_global_ukkonen.cpp:47-57)
    # comes before the length checks; the two over-long pairs differ by 1.
    c = add_cases()
    c["calls"] = c["calls"] + [["ACG", "ACGTA", 4]]
    return c


def main():
    data = {"cigar": cigar_cases(), "patterns": pattern_cases(), "distances": distance_cases(),
            "add_alignment": add_cases(), "ukkonen": ukkonen_cases(), "add_alignment_ukkonen": add_cases_ukkonen(),
            "formatted": formatted_cases()}
    with open(os.path.join(HERE, "aligner_kat.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("wrote", os.path.join(HERE, "aligner_kat.json"))


if __name__ == "__main__":
    main()

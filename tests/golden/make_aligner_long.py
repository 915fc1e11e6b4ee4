"""Golden vectors for long pairs (the reference's own benchmark recipes,
cudaaligner/benchmarks/main.cpp:33-60 and :85-124), computed by the aligner
oracle (oracle/aligner_oracle.cpp).  Each case stores the generator recipe,
the path length, a SHA-256 of the AlignmentState bytes (start -> end) and of
the CIGAR, and the match / mismatch / insertion / deletion counts, so a GPU
test can check a 100 kb alignment bit for bit without the oracle's runtime.

    python tests/golden/make_aligner_long.py   (writes tests/golden/aligner_long.json)
"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from claragenomicsanalysis_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402

ALGO = {"hirschberg_myers": oracle.ALIGN_HM, "myers": oracle.ALIGN_MYERS, "myers_banded": oracle.ALIGN_MYERS_BANDED,
        "ukkonen": oracle.ALIGN_UKKONEN}


def reference_pair(size, truncate):
    """minstd_rand(1); genome_1 = generate_random_genome(size); genome_2 =
    generate_random_sequence(genome_1, size/30, size/30, size/30), truncated to
    size for BM_SingleBatchAlignment (main.cpp:109-115); query = genome_1,
    target = genome_2 (add_alignment(genome_1, genome_2))."""
    e = size // 30
    muts, genomes = synth.pairs(1, 1, size, size if truncate else size + e + 1, e, e, e)
    return genomes[0].decode(), muts[0].decode()


def digest(path):
    b = bytes(int(x) for x in path)
    return hashlib.sha256(b).hexdigest()


def case(name, recipe, size, truncate, algo):
    q, t = reference_pair(size, truncate)
    t0 = time.time()
    p = oracle.align(q, t, ALGO[algo], len(q))
    dt = time.time() - t0
    cg = oracle.cigar(p)
    print("%-45s %-16s q=%d t=%d path=%d %.1fs" % (name, algo, len(q), len(t), len(p), dt), flush=True)
    return {"name": name, "recipe": recipe, "size": size, "truncate_target": truncate, "algorithm": algo,
            "query_length": len(q), "target_length": len(t), "max_query_length": len(q),
            "max_target_length": len(t), "path_length": len(p), "path_sha256": digest(p),
            "cigar_sha256": hashlib.sha256(cg.encode()).hexdigest(),
            "counts": [sum(1 for x in p if x == k) for k in range(4)]}


def main():
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "aligner_long.json")
    # cases already in the file are kept (the 100 kb Hirschberg-Myers oracle run is slow)
    have = {}
    if os.path.exists(out):
        for c in json.load(open(out))["cases"]:
            have[(c["recipe"], c["size"], c["algorithm"])] = c
    want = [("BM_SingleAlignment 100000 (main.cpp:33-60)", "BM_SingleAlignment", 100000, False, "hirschberg_myers")]
    for algo in ("hirschberg_myers", "myers", "myers_banded", "ukkonen"):
        want.append(("BM_SingleBatchAlignment 65536, first pair (main.cpp:85-124)", "BM_SingleBatchAlignment",
                     65536, True, algo))
    # Ukkonen at the 16,384 BM_SingleBatchAlignment size (512 x 4^k).  The
    # recipe's pairs have equal lengths, so the band is ~101 rows and the
    # single-wave kernel runs; the aligner only *sizes* its workspace for the
    # 920-row band a 10 % length difference would need.  The wide kernel's
    # 1-4 rows per thread are covered by test_ukkonen_wide_band_matches_oracle.
    want.append(("BM_SingleBatchAlignment 16384, first pair (main.cpp:85-124)", "BM_SingleBatchAlignment",
                 16384, True, "ukkonen"))
    cases = [have.get((w[1], w[2], w[4])) or case(*w) for w in want]
    json.dump({"generator": "tests/golden/make_aligner_long.py", "oracle": "oracle/aligner_oracle.cpp",
               "cases": cases}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

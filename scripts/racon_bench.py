"""Timing of the racon DFS sort (topsort_racon_lds, csrc/poa_wave.hpp) in
isolation: one wave sorting the final graph of a config-B or config-C window
(oracle graphs with their aligned-node lists) in the band kernel's LDS
budget, round-6 DFS against the round-5 step (v1).

  python scripts/racon_bench.py [B|C] [reps]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from claragenomicsanalysis_amd import synth  # noqa: E402
from oracle import oracle  # noqa: E402
from test_poa_racon import LDS, device_racon, window_graph  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    if cfg == "C":
        g = window_graph(synth.poa_windows(1, 1, 10000, 16, 500, 500, 500)[0], banded=True, score_bits=32,
                         max_nodes=40000)
    else:
        g = window_graph(synth.poa_windows(1, 1, 1000, 32, 50, 50, 50)[0])
    n, ic, ie, ac, al = g
    ok, want, want_pos, want_cols = oracle.topsort_racon(n, ic, ie, ac, al)
    lists = int(ic.sum()) + int(ac.sum())
    need = ((n + 15) & ~15) + 4 * n + ((2 * lists + 15) & ~15) + 2 * 4096
    print("%s: n=%d list entries=%d CSR bytes=%d of %d" % (cfg, n, lists, need, LDS))
    for v1 in (False, True):
        rc, got, pos, cols, ms = device_racon(n, ic, ie, ac, al, size_bits=16, v1=v1, reps=reps)
        print("  %-4s rc=%d exact=%s %.3f ms per sort, %.0f ns per node" % (
            "v1" if v1 else "dfs", rc, got == want and pos == want_pos and cols == want_cols, ms, ms * 1e6 / n))


if __name__ == "__main__":
    main()

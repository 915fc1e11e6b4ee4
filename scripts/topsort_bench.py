"""Timing of the level-keyed Kahn sort (topsort_levels, csrc/poa_wave.hpp) in
isolation: one workgroup sorting the final graph of a config-B or config-C
window (oracle graphs, in-edges in slot order), with the previous order of all
but the last read's nodes and the critical-predecessor hints of a first sort,
as in the kernels.  Prints the mean time per sort and, with a
GWAMD_TOPSORT_PROFILE build (GWAMD_LIBRARY), the section cycles per sort.

  python scripts/topsort_bench.py [B|C] [reps] [threads]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from claragenomicsanalysis_amd import load_library, synth  # noqa: E402
from oracle import oracle  # noqa: E402

SECTIONS = ("init", "reset", "in-order pass", "anchor rounds", "final + checks", "count sort + slots + table",
            "runs", "outputs")


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    thr = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if cfg == "C":
        win = synth.poa_windows(1, 1, 10000, 16, 500, 500, 500)[0]
        r = oracle.poa_window(win, banded=True, band_width=256, score_bits=32, msa=True, want_graph=True)
        threads, scratch, bits = 256, 163520 - 64, 32
    else:
        win = synth.poa_windows(1, 1, 1000, 32, 50, 50, 50)[0]
        r = oracle.poa_window(win, want_graph=True)
        threads, scratch, bits = 128, 38000, 16
    if thr:
        threads = thr
    n = r.final_nodes
    ins = r.graph["in"]
    outgoing = [[] for _ in range(n)]
    for v in range(n):
        for (u, _w) in ins[v]:
            outgoing[u].append(v)
    want = oracle.topsort(outgoing)
    n_prev = max(1, n - len(win[-1]) // 3)  # the last read added about a third of its length
    prev = [v for v in want if v < n_prev]
    in_cnt, in_e, out_cnt, out_e = oracle.edges_from_lists(outgoing, n)
    in_e = np.ascontiguousarray(in_e, np.int32)
    out_e = np.ascontiguousarray(out_e, np.int32)
    order = np.ascontiguousarray(prev, np.int32)
    L = load_library()
    f = L.gwamd_internal_topsort_levels_timed
    f.restype = C.c_int
    f.argtypes = [C.c_int] * 4 + [C.c_void_p] * 6 + [C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                                     C.c_void_p]
    for label, n_hint in (("no hints", 0), ("hints", n_prev)):
        hint = np.ascontiguousarray(np.arange(n), np.int32)
        if n_hint:
            # hints of a first sort (the kernels keep c(v) of the previous read's sort)
            res = np.zeros(n, np.int32)
            ms = C.c_double()
            f(bits, n, len(order), 0, in_cnt.ctypes.data, in_e.ctypes.data, out_cnt.ctypes.data, out_e.ctypes.data,
              hint.ctypes.data, order.ctypes.data, threads, scratch, res.ctypes.data, 0, C.byref(ms), None)
        res = np.zeros(n, np.int32)
        ms = C.c_double()
        prof = np.zeros(10, np.uint64)
        hint_in = hint.copy()
        rc = f(bits, n, len(order), n_hint, in_cnt.ctypes.data, in_e.ctypes.data, out_cnt.ctypes.data,
               out_e.ctypes.data, hint_in.ctypes.data, order.ctypes.data, threads, scratch, res.ctypes.data, reps,
               C.byref(ms), prof.ctypes.data)
        ok = rc == 1 and res.tolist() == want
        print("%s %s: n=%d threads=%d rc=%d order_ok=%s %.1f us per sort" % (cfg, label, n, threads, rc, ok,
                                                                          ms.value * 1e3))
        if prof.any():
            rounds = int(prof[7]) // 1000000000
            prof[7] = int(prof[7]) % 1000000000
            for name, v in zip(SECTIONS, prof[:8]):
                print("   %-28s %9.0f cycles" % (name, float(v) / (reps + 0)))
            print("   jump rounds per sort %.1f, anchors %.0f, iterations %.1f" % (rounds / reps, prof[8] / reps,
                                                                               prof[9] / reps))


if __name__ == "__main__":
    main()

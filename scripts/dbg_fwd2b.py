"""Diagnostic (GPU): first graph difference between the LDS kernel and the
oracle for window 0 of the config-B-like set after n reads."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
from oracle import oracle

wins = synth.poa_windows(7, 8, 1000, 32, 50, 50, 50)
max_seq = 1058
w = wins[0]
for n in (30, 31):
    sub = list(w[:n])
    b = CudaPoaBatch(n, max_seq, 2 << 30)
    assert b.add_poa_group(sub)[0] == 0
    b.generate_poa()
    gs, st = b.get_graphs()
    g = gs[0]
    r = oracle.poa_window(sub, max_nodes=(3 * max_seq + 3) // 4 * 4, max_consensus=2 * max_seq, max_seqs=n,
                          want_graph=True)
    og = r.graph
    nn = len(og["bases"])
    print("n=%d oracle nodes %d gpu nodes %d" % (n, nn, g.number_of_nodes()), flush=True)
    for v in range(nn):
        gin = sorted((u, wt) for (u, x), wt in g._weights.items() if x == v)
        oin = sorted(og["in"][v])
        lab = g.nodes[v] if v in g.nodes else None
        if gin != oin:
            print("  first differing node", v, "oracle in", oin, "gpu in", gin, flush=True)
            break
    print("  read len", len(sub[-1]), flush=True)

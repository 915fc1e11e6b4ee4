"""Diagnostic (GPU): which LDS-kernel shapes / forward passes disagree with the
oracle on config-B-like windows, and after how many reads (round-4 forward
pass bring-up)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
from oracle import oracle

MEM = 2 << 30
wins = synth.poa_windows(7, 8, 1000, 32, 50, 50, 50)
max_seq = 1058


def run(ws, nreads):
    b = CudaPoaBatch(nreads, max_seq, MEM)
    for w in ws:
        assert b.add_poa_group(list(w))[0] == 0
    b.generate_poa()
    return b.get_consensus()


def orc(w, nreads):
    return oracle.poa_window(w, max_nodes=(3 * max_seq + 3) // 4 * 4, max_consensus=2 * max_seq, max_seqs=nreads)


ref = [orc(w, 32) for w in wins]
os.environ["GWAMD_DIAG"] = "1"
cases = [("v2 8x2", {}), ("v2 16x1", {"GWAMD_POA_LDS_SHAPE": "16,1"}),
                  ("v2 8x1", {"GWAMD_POA_LDS_SHAPE": "8,1"}), ("v1 8x2", {"GWAMD_POA_FWD": "v1"})]
if os.environ.get("DBG_QUICK"):
    cases = cases[:1]
if os.environ.get("DBG_SET"):
    cases = [("v2 dbg=%s" % x, {"GWAMD_FWD2_DBG": x}) for x in os.environ["DBG_SET"].split(",")]
for name, env in cases:
    for k in ("GWAMD_POA_LDS_SHAPE", "GWAMD_POA_FWD", "GWAMD_FWD2_DBG"):
        os.environ.pop(k, None)
    os.environ.update(env)
    cons, cov, st = run(wins, 32)
    bad = [i for i in range(len(wins)) if (cons[i], cov[i], st[i]) != (ref[i].consensus, ref[i].coverage, ref[i].status)]
    print(name, "mismatching windows:", bad, flush=True)
    for i in bad[:2]:
        print("  w%d status %s/%s len %d/%d" % (i, st[i], ref[i].status, len(cons[i]), len(ref[i].consensus)), flush=True)
for k in ("GWAMD_POA_LDS_SHAPE", "GWAMD_POA_FWD"):
    os.environ.pop(k, None)
# first read count at which window 0 diverges (default shape)
for n in ([] if os.environ.get("DBG_QUICK") else range(2, 33)):
    sub = [w[:n] for w in wins[:1]]
    cons, cov, st = run(sub, n)
    r = orc(sub[0], n)
    if (cons[0], cov[0], st[0]) != (r.consensus, r.coverage, r.status):
        print("window 0 diverges at", n, "reads; lengths", [len(x) for x in sub[0]][-3:], flush=True)
        break
else:
    print("window 0 never diverges")

"""Time the parts of config D's step on one GPU: H2D upload, kernel, D2H
download and the host fill of sync_alignments (each synchronised on its own,
so the parts do not overlap here)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from claragenomicsanalysis_amd import synth  # noqa: E402
from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch  # noqa: E402

n, L = int(sys.argv[1]) if len(sys.argv) > 1 else 100000, 5000
algo = sys.argv[2] if len(sys.argv) > 2 else "hirschberg_myers"
qs, ts = synth.pairs(1, n, L, L, 166, 166, 166)
stream = torch.cuda.Stream()
b = CudaAlignerBatch(max(len(q) for q in qs), max(len(t) for t in ts), n, stream=stream, algorithm=algo)
for q, t in zip(qs, ts):
    b.add_alignment(q, t)
b.align_all()
b.sync_alignments()
for rep in range(3):
    t = [time.perf_counter()]
    b.upload(); stream.synchronize(); t.append(time.perf_counter())
    b.launch(); stream.synchronize(); t.append(time.perf_counter())
    b.download(); stream.synchronize(); t.append(time.perf_counter())
    b.sync_alignments(); t.append(time.perf_counter())
    d = [round((t[i + 1] - t[i]) * 1e3, 2) for i in range(4)]
    print("upload %.2f kernel %.2f download %.2f fill %.2f ms" % tuple(d), flush=True)

"""Aligner phase counters (diagnostic build, make alnprof):
python scripts/aln_prof.py [pairs] [algorithm] -> cycles per phase per alignment
(hirschberg_myers: split levels / frontier / base cases; myers: score matrix /
backtrace)."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["GWAMD_DIAG"] = "1"
os.environ["GWAMD_LIBRARY"] = os.path.join(ROOT, "claragenomicsanalysis_amd", "lib", "alnprof", "libgwamd.so")
import torch  # noqa: E402,F401  (HIP runtime first)
from claragenomicsanalysis_amd import synth  # noqa: E402
from claragenomicsanalysis_amd._lib import load_library  # noqa: E402
from claragenomicsanalysis_amd.cudaaligner import CudaAlignerBatch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
algo = sys.argv[2] if len(sys.argv) > 2 else "hirschberg_myers"
L = 5000
qs, ts = synth.pairs(1, n, L, L, 166, 166, 166)
b = CudaAlignerBatch(L, L, n, algorithm=algo)
for q, t in zip(qs, ts):
    b.add_alignment(q, t)
b.upload()
b.synchronize()
lib = load_library()
lib.gwamd_internal_aln_prof.argtypes = [C.c_void_p, C.c_int]
buf = (C.c_ulonglong * 8)()
b.launch()
b.synchronize()
lib.gwamd_internal_aln_prof(buf, 1)
t0 = time.perf_counter()
b.launch()
b.synchronize()
dt = time.perf_counter() - t0
lib.gwamd_internal_aln_prof(buf, 1)
v = list(buf)
print("pairs", n, "algorithm", algo, "grid", b.config()[0], "wall_ms", round(dt * 1e3, 1))
if algo == "myers":
    names = ["score_matrix", "backtrace", "-", "total", "column_blocks", "backtrace_steps"]
    for k, nm in enumerate(names):
        if nm != "-":
            print("%-18s %14.0f per pair" % (nm, v[k] / n))
    print("cycles per column-block: %.1f" % (v[0] / max(v[4], 1)))
    print("cycles per backtrace step: %.1f" % (v[1] / max(v[5], 1)))
else:
    names = ["split_levels", "frontier", "base_cases", "total", "big_col_blocks", "leaf_cols", "leaves"]
    for k, nm in enumerate(names):
        print("%-18s %14.0f per pair" % (nm, v[k] / n))
    print("cycles per sweep column-block: %.1f" % ((v[0] + v[1]) / max(v[4], 1)))
    print("cycles per leaf column: %.1f" % (v[2] / max(v[5], 1)))

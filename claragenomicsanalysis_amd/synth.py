"""Synthetic ONT-like windows and alignment pairs (reference generators,
genomeutils.hpp:26-126, restated in csrc/synth.cpp)."""
import ctypes as C

import numpy as np

from ._lib import load_library


def _decl(L):
    if getattr(L, "_synth_declared", False):
        return
    L.gwamd_synth_poa_windows.restype = C.c_int64
    L.gwamd_synth_poa_windows.argtypes = [C.c_int32] * 7 + [C.c_void_p, C.c_int64, C.c_void_p]
    L.gwamd_synth_pairs.restype = C.c_int32
    L.gwamd_synth_pairs.argtypes = [C.c_int32] * 7 + [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
    L._synth_declared = True


def poa_windows_packed(first_seed, n, backbone_len, num_reads, max_mut, max_ins, max_del):
    """Returns (bases uint8[total], lens int32[n, num_reads])."""
    L = load_library()
    _decl(L)
    cap = int(n) * num_reads * (backbone_len + max_ins + 1) + 16
    bases = np.zeros(cap, np.uint8)
    lens = np.zeros((n, num_reads), np.int32)
    tot = L.gwamd_synth_poa_windows(first_seed, n, backbone_len, num_reads, max_mut, max_ins, max_del,
                                    bases.ctypes.data, cap, lens.ctypes.data)
    if tot < 0:
        raise RuntimeError("synthetic buffer too small")
    return bases[:tot], lens


def poa_windows(first_seed, n, backbone_len, num_reads, max_mut, max_ins, max_del):
    """Returns a list of windows, each a list of read byte strings."""
    bases, lens = poa_windows_packed(first_seed, n, backbone_len, num_reads, max_mut, max_ins, max_del)
    out, off = [], 0
    raw = bases.tobytes()
    for w in range(n):
        win = []
        for r in range(num_reads):
            k = int(lens[w, r])
            win.append(raw[off:off + k])
            off += k
        out.append(win)
    return out


def pairs(first_seed, n, target_len, query_cap, max_mut, max_ins, max_del):
    """Returns (queries, targets) lists of byte strings."""
    L = load_library()
    _decl(L)
    stride = max(target_len + max_ins + 1, query_cap)
    q = np.zeros(n * stride, np.uint8)
    t = np.zeros(n * stride, np.uint8)
    ql = np.zeros(n, np.int32)
    tl = np.zeros(n, np.int32)
    rc = L.gwamd_synth_pairs(first_seed, n, target_len, query_cap, max_mut, max_ins, max_del, q.ctypes.data,
                             t.ctypes.data, stride, ql.ctypes.data, tl.ctypes.data)
    if rc != 0:
        raise RuntimeError("synthetic pair buffer too small")
    qs = [q[i * stride:i * stride + ql[i]].tobytes() for i in range(n)]
    ts = [t[i * stride:i * stride + tl[i]].tobytes() for i in range(n)]
    return qs, ts


def aligner_pairs(first_seed, n, length=5000, errors=166):
    """per pair i, minstd_rand(first_seed + i); target =
    generate_random_genome(length); query = generate_random_sequence(target,
    errors, errors, errors) truncated to length (cudaaligner/benchmarks/main.cpp:109-115).
    Returns a list of (query, target) str pairs."""
    qs, ts = pairs(first_seed, n, length, length, errors, errors, errors)
    return [(q.decode(), t.decode()) for q, t in zip(qs, ts)]

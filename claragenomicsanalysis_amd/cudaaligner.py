"""Python API for the MI355X global aligner; mirrors pygenomeworks'
``genomeworks.cudaaligner`` (pygenomeworks/genomeworks/cudaaligner/cudaaligner.pyx:28-270):
``CudaAlignerBatch`` with the same constructor arguments and defaults, and
``CudaAlignment`` result objects.  Everything runs through the C ABI of
libgwamd.so (include/gwamd_cudaaligner.h).
"""
import ctypes as C

import numpy as np

from ._lib import load_library, last_error

# StatusType (cudaaligner.hpp:27-35)
STATUS_NAMES = ["success", "uninitialized", "exceeded_max_alignments", "exceeded_max_length",
                "exceeded_max_alignment_difference", "generic_error"]
SUCCESS, UNINITIALIZED, EXCEEDED_MAX_ALIGNMENTS, EXCEEDED_MAX_LENGTH = 0, 1, 2, 3
# AlignmentState (cudaaligner.hpp:45-52)
MATCH, MISMATCH, INSERTION, DELETION = 0, 1, 2, 3
_STATE_STR = {MATCH: "m", MISMATCH: "mm", INSERTION: "i", DELETION: "d"}
ALGORITHMS = {"hirschberg_myers": 0, "myers": 1, "myers_banded": 2, "ukkonen": 3}


def _declare(L):
    vp, i8, i32, i64 = C.c_void_p, C.c_int8, C.c_int32, C.c_int64
    P = C.POINTER
    L.gwamd_aligner_create.restype = i32
    L.gwamd_aligner_create.argtypes = [P(vp), i32, i32, i32, i32, i32, vp, i32, i64]
    L.gwamd_aligner_destroy.restype = None
    L.gwamd_aligner_destroy.argtypes = [vp]
    L.gwamd_aligner_add_alignment.restype = i32
    L.gwamd_aligner_add_alignment.argtypes = [vp, C.c_char_p, i32, C.c_char_p, i32, i32, i32]
    for name in ("gwamd_aligner_align_all", "gwamd_aligner_sync_alignments", "gwamd_aligner_num_alignments",
                 "gwamd_aligner_upload", "gwamd_aligner_launch", "gwamd_aligner_download",
                 "gwamd_aligner_synchronize"):
        getattr(L, name).restype = i32
        getattr(L, name).argtypes = [vp]
    L.gwamd_aligner_get_alignment.restype = i32
    L.gwamd_aligner_get_alignment.argtypes = [vp, i32, vp, i32, P(i32)]
    L.gwamd_aligner_get_sequences.restype = i32
    L.gwamd_aligner_get_sequences.argtypes = [vp, i32, P(vp), P(i32), P(vp), P(i32)]
    L.gwamd_aligner_get_cigar.restype = i32
    L.gwamd_aligner_get_cigar.argtypes = [vp, i32, C.c_char_p, i32]
    L.gwamd_aligner_reset.restype = None
    L.gwamd_aligner_reset.argtypes = [vp]
    L.gwamd_aligner_get_paths.restype = i32
    L.gwamd_aligner_get_paths.argtypes = [vp, P(vp), P(vp), P(i32)]
    L.gwamd_aligner_get_config.restype = i32
    L.gwamd_aligner_get_config.argtypes = [vp, P(i32), P(i64)]
    L.gwamd_aligner_max_lengths.restype = i32
    L.gwamd_aligner_max_lengths.argtypes = [i32, P(i32), P(i32)]
    L.gwamd_aligner_pair_fits.restype = i32
    L.gwamd_aligner_pair_fits.argtypes = [i32, i32, i32]
    L.gwamd_aligner_last_kernel_ms.restype = i32
    L.gwamd_aligner_last_kernel_ms.argtypes = [vp, P(C.c_double)]
    L.gwamd_aligner_get_stats.restype = i32
    L.gwamd_aligner_get_stats.argtypes = [vp, P(i64), P(i64), P(i64)]
    L.gwamd_device_allocator_create.restype = i32
    L.gwamd_device_allocator_create.argtypes = [P(vp), i64]
    L.gwamd_device_allocator_destroy.restype = None
    L.gwamd_device_allocator_destroy.argtypes = [vp]
    for name in ("gwamd_device_allocator_capacity", "gwamd_device_allocator_used"):
        getattr(L, name).restype = i64
        getattr(L, name).argtypes = [vp]
    L.gwamd_device_allocator_default_size.restype = i64
    L.gwamd_device_allocator_default_size.argtypes = []
    L.gwamd_aligner_create_with_allocator.restype = i32
    L.gwamd_aligner_create_with_allocator.argtypes = [P(vp), i32, i32, i32, i32, i32, vp, i32, vp]
    del i8


def max_lengths(algorithm="hirschberg_myers"):
    """(max query length, max target length) this implementation's aligner
    accepts (the reference has no limits; CudaAlignerBatch raises
    ValueError above them, include/gwamd_cudaaligner.h)."""
    from . import load_library
    L = load_library()
    _declare(L)
    q, t = C.c_int32(), C.c_int32()
    _check(L.gwamd_aligner_max_lengths(ALGORITHMS[algorithm], C.byref(q), C.byref(t)))
    return q.value, t.value


def status_to_str(status):
    """cudaaligner.pyx:28-44."""
    if 0 <= status < len(STATUS_NAMES):
        return STATUS_NAMES[status]
    raise RuntimeError("Unknown error status : %s" % status)


def _check(rc):
    if rc < 0:
        msg = last_error()
        if rc == -1:
            raise ValueError(msg)
        raise RuntimeError(msg)
    return rc


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    if hasattr(stream, "cuda_stream"):  # torch.cuda.Stream
        return stream.cuda_stream
    if hasattr(stream, "stream"):
        return stream.stream
    raise RuntimeError("Type for stream option must be a HIP stream handle")


class CudaAlignment:
    """One alignment (cudaaligner.pyx:47-118)."""

    def __init__(self, query, target, cigar, alignment_type, status, alignment, format_alignment):
        self.query = query
        self.target = target
        self.cigar = cigar
        self.alignment_type = alignment_type
        self.status = status
        self.alignment = [_STATE_STR[s] for s in alignment]
        self.format_alignment = format_alignment

    def __str__(self):
        return "{}\n{}\n{}\n".format(self.format_alignment[0], self.format_alignment[1], self.format_alignment[2])


def _format(query, target, states):
    # AlignmentImpl::format_alignment (alignment_impl.cpp:75-112)
    qs, ps, ts, qi, ti = [], [], [], 0, 0
    for s in states:
        if s == MATCH or s == MISMATCH:
            ts.append(target[ti]); qs.append(query[qi]); ps.append("|" if s == MATCH else "x"); ti += 1; qi += 1
        elif s == DELETION:
            ts.append("-"); qs.append(query[qi]); ps.append(" "); qi += 1
        else:
            ts.append(target[ti]); qs.append("-"); ps.append(" "); ti += 1
    return ["".join(qs), "".join(ps), "".join(ts)]


class DeviceAllocator:
    """The C++ API's DefaultDeviceAllocator (create_default_device_allocator,
    allocator.hpp:297-305): a device-memory pool of max_caching_size bytes
    (default 2 GiB, -1 = all available) shared by every aligner created with
    it (pass it as CudaAlignerBatch(..., allocator=...))."""

    def __init__(self, max_caching_size=None):
        self._lib = load_library()
        if max_caching_size is None:
            max_caching_size = self._lib.gwamd_device_allocator_default_size()
        self._handle = C.c_void_p()
        _check(self._lib.gwamd_device_allocator_create(C.byref(self._handle), int(max_caching_size)))

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            self._lib.gwamd_device_allocator_destroy(h)
            self._handle = None

    @property
    def capacity(self):
        return int(self._lib.gwamd_device_allocator_capacity(self._handle))

    @property
    def used(self):
        """Device bytes reserved by the live aligners created with this pool."""
        return int(self._lib.gwamd_device_allocator_used(self._handle))


class CudaAlignerBatch:
    """Python API for MI355X sequence-to-sequence global alignment
    (cudaaligner.pyx:121-270).  ``algorithm`` (an extension) selects the
    full-matrix Myers aligner instead of the default Hirschberg + Myers."""

    def __init__(self, max_query_length, max_target_length, max_alignments, alignment_type="global", stream=None,
                 device_id=0, max_device_memory_allocator_caching_size=-1, algorithm="hirschberg_myers",
                 *args, allocator=None, **kwargs):
        if alignment_type != "global":
            raise RuntimeError("Unknown alignment_type provided. Must be global.")
        if algorithm not in ALGORITHMS:
            raise RuntimeError("Unknown algorithm %r" % (algorithm,))
        self._lib = load_library()
        self._handle = C.c_void_p()
        self.stream = stream
        if allocator is not None:
            # create_aligner(..., DefaultDeviceAllocator, stream, device_id) (aligner.hpp:90)
            _check(self._lib.gwamd_aligner_create_with_allocator(
                C.byref(self._handle), int(max_query_length), int(max_target_length), int(max_alignments), 0,
                ALGORITHMS[algorithm], _stream_handle(stream), int(device_id), allocator._handle))
            self._allocator = allocator
        else:
            _check(self._lib.gwamd_aligner_create(C.byref(self._handle), int(max_query_length),
                                                  int(max_target_length), int(max_alignments), 0,
                                                  ALGORITHMS[algorithm], _stream_handle(stream), int(device_id),
                                                  int(max_device_memory_allocator_caching_size)))
        self._synced = False

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            self._lib.gwamd_aligner_destroy(h)
            self._handle = None

    def add_alignment(self, query, target, reverse_complement_query=False, reverse_complement_target=False):
        """cudaaligner.pyx:194-208; returns the StatusType."""
        q = query.encode() if isinstance(query, str) else bytes(query)
        t = target.encode() if isinstance(target, str) else bytes(target)
        return _check(self._lib.gwamd_aligner_add_alignment(self._handle, q, len(q), t, len(t),
                                                            int(bool(reverse_complement_query)),
                                                            int(bool(reverse_complement_target))))

    def align_all(self):
        _check(self._lib.gwamd_aligner_align_all(self._handle))
        self._synced = False

    def sync_alignments(self):
        """Aligner::sync_alignments (aligner.hpp:58): waits for align_all and
        fills the alignments' states (aligner_global.cpp:161-191)."""
        _check(self._lib.gwamd_aligner_sync_alignments(self._handle))
        self._synced = True

    def num_alignments(self):
        return self._lib.gwamd_aligner_num_alignments(self._handle)

    def get_alignments(self):
        """Syncs, then returns CudaAlignment objects in insertion order (cudaaligner.pyx:215-260)."""
        n = self.num_alignments()
        if n and not self._synced:
            _check(self._lib.gwamd_aligner_sync_alignments(self._handle))
            self._synced = True
        out = []
        for i in range(n):
            st = C.c_int32()
            ln = _check(self._lib.gwamd_aligner_get_alignment(self._handle, i, None, 0, C.byref(st)))
            buf = np.zeros(max(ln, 1), np.int8)
            _check(self._lib.gwamd_aligner_get_alignment(self._handle, i, buf.ctypes.data, ln, C.byref(st)))
            states = buf[:ln].tolist()
            cl = _check(self._lib.gwamd_aligner_get_cigar(self._handle, i, None, 0))
            cb = C.create_string_buffer(cl + 1)
            _check(self._lib.gwamd_aligner_get_cigar(self._handle, i, cb, cl + 1))
            q, t = self._pair(i)
            out.append(CudaAlignment(q, t, cb.value.decode(), "global", st.value, states, _format(q, t, states)))
        return out

    def _pair(self, i):
        # the sequences as stored by add_alignment (reverse-complemented if asked)
        qp, ql, tp, tl = C.c_void_p(), C.c_int32(), C.c_void_p(), C.c_int32()
        _check(self._lib.gwamd_aligner_get_sequences(self._handle, i, C.byref(qp), C.byref(ql), C.byref(tp),
                                                     C.byref(tl)))
        q = C.string_at(qp, ql.value).decode() if ql.value else ""
        t = C.string_at(tp, tl.value).decode() if tl.value else ""
        return q, t

    def reset(self):
        self._lib.gwamd_aligner_reset(self._handle)
        self._synced = False

    # --- bench.py helpers --------------------------------------------------
    def upload(self):
        _check(self._lib.gwamd_aligner_upload(self._handle))

    def launch(self):
        _check(self._lib.gwamd_aligner_launch(self._handle))

    def download(self):
        _check(self._lib.gwamd_aligner_download(self._handle))

    def synchronize(self):
        _check(self._lib.gwamd_aligner_synchronize(self._handle))

    def raw_paths(self):
        """(paths int8 [n, stride] emitted end -> start, lengths int32 [n]) after download + synchronize."""
        n = self.num_alignments()
        p, ln, stride = C.c_void_p(), C.c_void_p(), C.c_int32()
        self._lib.gwamd_aligner_get_paths(self._handle, C.byref(p), C.byref(ln), C.byref(stride))
        paths = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int8)), shape=(max(n, 1) * stride.value,))
        lens = np.ctypeslib.as_array(C.cast(ln, C.POINTER(C.c_int32)), shape=(max(n, 1),))
        return paths[:n * stride.value].reshape(n, stride.value).copy(), lens[:n].copy()

    def last_kernel_ms(self):
        """Kernel time of the last align_all() (ms, union of its launches;
        gwamd_aligner_last_kernel_ms)."""
        v = C.c_double()
        _check(self._lib.gwamd_aligner_last_kernel_ms(self._handle, C.byref(v)))
        return v.value

    def stats(self):
        """Path counters accumulated over this aligner's launches
        (gwamd_aligner_get_stats)."""
        v, w, r = C.c_int64(), C.c_int64(), C.c_int64()
        _check(self._lib.gwamd_aligner_get_stats(self._handle, C.byref(v), C.byref(w), C.byref(r)))
        return {"hbm_state_sweeps": v.value, "ukkonen_wide_pairs": w.value, "ukkonen_max_rows_per_thread": r.value}

    def config(self):
        g, b = C.c_int32(), C.c_int64()
        self._lib.gwamd_aligner_get_config(self._handle, C.byref(g), C.byref(b))
        return g.value, b.value

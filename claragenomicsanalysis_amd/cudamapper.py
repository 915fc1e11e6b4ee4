"""Overlap alignment and PAF output of cudamapper over the C ABI
(include/gwamd_cudamapper.h; reference cudamapper/src/main.cu:48-175 and
cudamapper/src/cudamapper_utils.cpp:30-112).

Overlaps are aligned with the MI355X global aligner (Hirschberg-Myers, the
aligner create_aligner returns); a Reverse ('-') overlap aligns the query
region against the reverse complement of the target region.
"""
import ctypes as C

from ._lib import load_library, last_error


class Overlap(C.Structure):
    """cudamapper::Overlap (cudamapper/include/.../types.hpp:68-89)."""
    _fields_ = [("query_read_id", C.c_uint32), ("target_read_id", C.c_uint32),
                ("query_start", C.c_uint32), ("target_start", C.c_uint32),
                ("query_end", C.c_uint32), ("target_end", C.c_uint32),
                ("relative_strand", C.c_ubyte), ("num_residues", C.c_uint32),
                ("overlap_complete", C.c_uint8)]

    def __init__(self, query_read_id, target_read_id, query_start, query_end, target_start, target_end,
                 strand="+", num_residues=0, overlap_complete=False):
        s = strand.encode() if isinstance(strand, str) else bytes([strand])
        super().__init__(query_read_id, target_read_id, query_start, target_start, query_end, target_end,
                         s[0], num_residues, int(bool(overlap_complete)))

    @property
    def strand(self):
        return chr(self.relative_strand)


def _declare(L):
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    P = C.POINTER
    L.gwamd_align_overlaps.restype = i32
    L.gwamd_align_overlaps.argtypes = [C.c_char_p, vp, i32, C.c_char_p, vp, i32, vp, i32, i32, i32, P(vp)]
    L.gwamd_format_paf.restype = i32
    L.gwamd_format_paf.argtypes = [C.c_char_p, vp, vp, i32, C.c_char_p, vp, vp, i32, vp, i32, vp, i32, P(vp)]
    L.gwamd_read_fasta.restype = i32
    L.gwamd_read_fasta.argtypes = [C.c_char_p, C.c_uint32, i32, P(vp), P(vp)]
    L.gwamd_text_list_create.restype = i32
    L.gwamd_text_list_create.argtypes = [vp, vp, i32, P(vp)]
    L.gwamd_text_list_size.restype = i32
    L.gwamd_text_list_size.argtypes = [vp]
    L.gwamd_text_list_get.restype = i32
    L.gwamd_text_list_get.argtypes = [vp, i32, P(C.c_void_p), P(i64)]
    L.gwamd_text_list_free.restype = None
    L.gwamd_text_list_free.argtypes = [vp]


def _check(rc):
    if rc == -1:
        raise ValueError(last_error())
    if rc < 0:
        raise RuntimeError(last_error())
    return rc


def _pack(items):
    data = [x.encode() if isinstance(x, str) else bytes(x) for x in items]
    offs = (C.c_int64 * (len(data) + 1))()
    for i, d in enumerate(data):
        offs[i + 1] = offs[i] + len(d)
    return b"".join(data), offs


def _overlap_array(overlaps):
    arr = (Overlap * max(len(overlaps), 1))()
    for i, o in enumerate(overlaps):
        arr[i] = o if isinstance(o, Overlap) else Overlap(*o)
    return arr


def _take(L, handle):
    try:
        out = []
        for i in range(L.gwamd_text_list_size(handle)):
            p, n = C.c_void_p(), C.c_int64()
            _check(L.gwamd_text_list_get(handle, i, C.byref(p), C.byref(n)))
            out.append(C.string_at(p, n.value).decode())
        return out
    finally:
        L.gwamd_text_list_free(handle)


def align_overlaps(overlaps, query_reads, target_reads, num_alignment_engines=1, device_id=0):
    """CIGAR of every overlap (align_overlaps, main.cu:125-175).

    query_reads / target_reads: sequences indexed by the overlaps' read ids."""
    L = load_library()
    qb, qo = _pack(query_reads)
    tb, to = _pack(target_reads)
    arr = _overlap_array(overlaps)
    h = C.c_void_p()
    _check(L.gwamd_align_overlaps(qb, qo, len(query_reads), tb, to, len(target_reads), arr, len(overlaps),
                                  num_alignment_engines, device_id, C.byref(h)))
    return _take(L, h)


def format_paf(overlaps, cigars, query_reads, target_reads, kmer_size):
    """PAF text of print_paf (cudamapper_utils.cpp:30-112).

    query_reads / target_reads: (name, sequence or length) per read id; cigars
    may be None or empty (no cg:Z: tag)."""
    L = load_library()
    qn, qno = _pack([r[0] for r in query_reads])
    tn, tno = _pack([r[0] for r in target_reads])
    qlen = (C.c_int64 * max(len(query_reads), 1))(*[r[1] if isinstance(r[1], int) else len(r[1])
                                                    for r in query_reads])
    tlen = (C.c_int64 * max(len(target_reads), 1))(*[r[1] if isinstance(r[1], int) else len(r[1])
                                                     for r in target_reads])
    arr = _overlap_array(overlaps)
    cig = None
    if cigars:
        data = [c.encode() if isinstance(c, str) else bytes(c) for c in cigars]
        ptrs = (C.c_char_p * len(data))(*data)
        lens = (C.c_int64 * len(data))(*[len(d) for d in data])
        cig = C.c_void_p()
        _check(L.gwamd_text_list_create(ptrs, lens, len(data), C.byref(cig)))
    h = C.c_void_p()
    try:
        _check(L.gwamd_format_paf(qn, qno, qlen, len(query_reads), tn, tno, tlen, len(target_reads), arr,
                                  len(overlaps), cig, kmer_size, C.byref(h)))
    finally:
        if cig is not None:
            L.gwamd_text_list_free(cig)
    return _take(L, h)[0]


def read_fasta(path, min_sequence_length=0, shuffle=True):
    """(name, sequence) records as io::create_kseq_fasta_parser holds them
    (kseqpp_fasta_parser.cpp:31-72): shorter records dropped, shuffled with
    std::mt19937(0) unless shuffle is False."""
    L = load_library()
    n, s = C.c_void_p(), C.c_void_p()
    _check(L.gwamd_read_fasta(str(path).encode(), int(min_sequence_length), int(bool(shuffle)), C.byref(n),
                              C.byref(s)))
    return list(zip(_take(L, n), _take(L, s)))

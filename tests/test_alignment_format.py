"""The product AlignmentImpl (csrc/aligner_batch.cpp, through the C ABI
gwamd_alignment_format / gwamd_alignment_cigar) against the formatted
alignments and CIGARs of cudaaligner/tests/Test_AlignmentImpl.cpp:54-168
(transcribed into tests/golden/aligner_kat.json).  Host-only: no device work."""
import ctypes as C
import json
import os

import numpy as np
import pytest

from claragenomicsanalysis_amd._lib import load_library

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "aligner_kat.json")))


def _lib():
    L = load_library()
    L.gwamd_alignment_format.restype = C.c_int32
    L.gwamd_alignment_format.argtypes = [C.c_char_p, C.c_int32, C.c_char_p, C.c_int32, C.c_void_p, C.c_int32,
                                         C.c_int32, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32,
                                         C.POINTER(C.c_int32)]
    L.gwamd_alignment_cigar.restype = C.c_int32
    L.gwamd_alignment_cigar.argtypes = [C.c_void_p, C.c_int32, C.c_char_p, C.c_int32]
    return L


def format_alignment(query, target, states, line=-1):
    L = _lib()
    st = np.asarray(states, np.int8)
    cap = len(states) + 1
    bufs = [C.create_string_buffer(cap) for _ in range(3)]
    lb = C.c_int32()
    n = L.gwamd_alignment_format(query.encode(), len(query), target.encode(), len(target), st.ctypes.data,
                                 len(st), line, bufs[0], bufs[1], bufs[2], cap, C.byref(lb))
    assert n == len(states)
    return [b.value.decode() for b in bufs], lb.value


def cigar(states):
    L = _lib()
    st = np.asarray(states, np.int8)
    buf = C.create_string_buffer(4 * len(states) + 8)
    n = L.gwamd_alignment_cigar(st.ctypes.data, len(st), buf, len(buf))
    return buf.value.decode()[:n]


@pytest.mark.parametrize("case", range(len(GOLD["formatted"])))
def test_format_alignment_kat(case):
    c = GOLD["formatted"][case]
    rows, lb = format_alignment(c["query"], c["target"], c["states"])
    assert rows == c["formatted"]
    assert lb == 0  # maximal_line_length < 0 -> no line breaks (alignment_impl.cpp:80)
    rows80, lb80 = format_alignment(c["query"], c["target"], c["states"], line=80)  # the default (alignment.hpp:85)
    assert rows80 == c["formatted"] and lb80 == 80


@pytest.mark.parametrize("case", range(len(GOLD["formatted"])))
def test_convert_to_cigar_kat(case):
    c = GOLD["formatted"][case]
    assert cigar(c["states"]) == c["cigar"]


def test_format_line_length_and_empty():
    c = GOLD["formatted"][0]
    rows, lb = format_alignment(c["query"], c["target"], c["states"], line=2)
    assert rows == c["formatted"] and lb == 2
    assert cigar([]) == ""

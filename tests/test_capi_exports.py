"""CPU-side checks of the drop-in boundary: libgwamd.so loads without a GPU
and exports every entry point declared in include/*.h."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "claragenomicsanalysis_amd", "lib", "libgwamd.so")


def declared_symbols():
    names = set()
    inc = os.path.join(ROOT, "include")
    for fn in os.listdir(inc):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(inc, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(gwamd_[a-z0-9_]+)\s*\(", text):
            names.add(m.group(1))
    return names


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "claragenomicsanalysis_amd", "csrc")])
    return LIB


def test_library_loads_without_gpu(built):
    from claragenomicsanalysis_amd import load_library
    L = load_library()
    assert L.gwamd_last_error() is not None


def test_every_declared_symbol_is_exported(built):
    out = subprocess.check_output(["nm", "-D", "--defined-only", built]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = sorted(declared_symbols() - exported)
    assert not missing, missing
    assert len(declared_symbols()) >= 15


def test_batch_size_mirrors_reference():
    # BatchSize(1100, 32): batch.hpp:74-95
    from claragenomicsanalysis_amd.cudapoa import BatchSize
    bs = BatchSize.make(1100, 32)
    assert (bs.max_sequence_size, bs.max_consensus_size, bs.max_nodes_per_window,
            bs.max_nodes_per_window_banded, bs.alignment_band_width, bs.max_sequences_per_poa) == \
        (1100, 2200, 3300, 4400, 256, 32)
    bs = BatchSize.make(1024, 10, 200)  # band width rounded up to 128 multiple
    assert bs.alignment_band_width == 256


def test_batch_size_validation_throws():
    from claragenomicsanalysis_amd.cudapoa import BatchSize
    with pytest.raises(ValueError):
        BatchSize.make_full(100, 50, 300, 400, 128, 10)   # consensus < seq
    with pytest.raises(ValueError):
        BatchSize.make_full(100, 200, 300, 400, 256, 10)  # band > seq
    with pytest.raises(ValueError):
        BatchSize.make(-1, 10)


def test_synthetic_generator_is_deterministic():
    from claragenomicsanalysis_amd import synth
    a = synth.poa_windows(1, 2, 300, 4, 10, 10, 10)
    b = synth.poa_windows(1, 2, 300, 4, 10, 10, 10)
    assert a == b
    assert a[0][0] != a[1][0]
    assert len(a[0][0]) == 300


def test_aligner_length_limits_are_queryable(built):
    # this implementation's limits (the reference has none): documented in
    # include/gwamd_cudaaligner.h, INTEGRATION.md and DESIGN.md.  The
    # reference's own benchmarks run 100 kb (BM_SingleAlignment) and 65,536 bp
    # batches for every aligner (cudaaligner/benchmarks/main.cpp:135-158).
    from claragenomicsanalysis_amd.cudaaligner import max_lengths
    assert max_lengths("hirschberg_myers") == (1 << 24, 1 << 24)
    assert max_lengths("myers") == (1 << 24, 1 << 24)  # and the pair's matrix within one 32 GiB slot
    assert max_lengths("myers_banded") == (65536, 65536)
    q, t = max_lengths("ukkonen")
    assert q == 65535 and 8000 < t < 8300

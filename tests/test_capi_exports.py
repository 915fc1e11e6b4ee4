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
    # Ukkonen: bands up to 4,096 rows (ukkonen_wide_kernel), the reference
    # benchmark's 65,536 bp (main.cpp:140-143)
    assert max_lengths("ukkonen") == (65536, 65536)


def test_tuning_env_ignored_without_diag_switch(built, monkeypatch):
    # the GWAMD_* tuning variables change the kernel plan
    # only with GWAMD_DIAG=1, so a drop-in user's environment cannot
    import ctypes as C
    from claragenomicsanalysis_amd import load_library
    L = load_library()

    def tuning():
        v = [C.c_int32() for _ in range(4)]
        assert L.gwamd_poa_env_tuning(*[C.byref(x) for x in v]) == 0
        return tuple(x.value for x in v)

    monkeypatch.setenv("GWAMD_TB_WALK", "scalar")
    monkeypatch.setenv("GWAMD_BAND_FWD", "row")
    monkeypatch.setenv("GWAMD_POA_KERNEL", "v1")
    monkeypatch.setenv("GWAMD_TOPSORT_RING", "1")
    monkeypatch.delenv("GWAMD_DIAG", raising=False)
    assert tuning() == (3, 0, 0, 0)  # defaults: pointer doubling over strips, plan decides
    monkeypatch.setenv("GWAMD_DIAG", "0")
    assert tuning() == (3, 0, 0, 0)
    monkeypatch.setenv("GWAMD_DIAG", "1")
    assert tuning() == (2, 2, 1, 1)


def test_aligner_pair_fits(built):
    # the two limits of max_lengths are not jointly valid for full Myers
    # (one pair's matrix must fit a 32 GiB slot): pair_fits says which are
    from claragenomicsanalysis_amd import load_library
    from claragenomicsanalysis_amd.cudaaligner import ALGORITHMS
    L = load_library()
    fits = lambda a, q, t: L.gwamd_aligner_pair_fits(ALGORITHMS[a], q, t)
    assert fits("myers", 65536, 65536) == 1
    assert fits("myers", 1 << 24, 1 << 24) == 0
    assert fits("myers", 1 << 24, 5000) == 1
    assert fits("hirschberg_myers", 1 << 24, 1 << 24) == 1
    assert fits("myers_banded", 65536, 65536) == 1
    assert fits("myers_banded", 65537, 100) == 0
    assert fits("ukkonen", 5000, 5000) == 1
    assert fits("ukkonen", 18432, 18432) == 1
    assert fits("ukkonen", 65536, 65536) == 1
    assert fits("ukkonen", 65537, 100) == 0
    assert L.gwamd_aligner_pair_fits(ALGORITHMS["myers"], -1, 5) < 0

"""The cudapoa command-line tool (claragenomicsanalysis_amd/lib/cudapoa, built from
csrc/cudapoa_main.cpp; reference cudapoa/src/main.cpp + application_parameters.cpp).

CPU tests cover option validation (it fails before touching the GPU); GPU tests
run the tool on windows written in the cudapoa and FASTA formats and compare
every consensus / MSA row with the oracle."""
import os
import subprocess

import pytest

from claragenomicsanalysis_amd import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "claragenomicsanalysis_amd", "lib", "cudapoa")


def _run(args, timeout=120):
    if not os.path.exists(CLI):
        pytest.fail("cudapoa tool not built: run make -C claragenomicsanalysis_amd/csrc")
    return subprocess.run([CLI] + args, capture_output=True, text=True, timeout=timeout)


def _write_cudapoa(path, windows):
    with open(path, "w") as f:
        for w in windows:
            f.write(f"{len(w)}\n")
            for s in w:
                f.write(s.decode() if isinstance(s, bytes) else s)
                f.write("\n")


def _write_fasta(path, reads):
    with open(path, "w") as f:
        for i, s in enumerate(reads):
            s = s.decode() if isinstance(s, bytes) else s
            f.write(f">read{i}\n")
            for k in range(0, len(s), 60):  # multi-line records
                f.write(s[k:k + 60] + "\n")


def test_help_exits_zero():
    r = _run(["-h"])
    assert r.returncode == 0
    assert "--band-width" in r.stderr and "--gpu-mem-alloc" in r.stderr


@pytest.mark.parametrize("args,msg", [
    (["-R", "1.5"], "gpu-mem-alloc"),
    (["-m", "-1"], "match score"),
    (["-n", "2"], "mismatch score"),
    (["-g", "3"], "gap score"),
    (["-M", "0"], "max-groups"),
])
def test_invalid_options(tmp_path, args, msg):
    p = tmp_path / "w.txt"
    _write_cudapoa(p, [["ACGT", "ACGT"]])
    r = _run(["-i", str(p)] + args)
    assert r.returncode != 0
    assert msg in r.stderr


def test_input_rules(tmp_path):
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    _write_cudapoa(a, [["ACGT"]])
    _write_cudapoa(b, [["ACGT"]])
    r = _run(["-i", str(a), "-i", str(b)])  # two cudapoa files: rejected
    assert r.returncode != 0 and "Invalid input" in r.stderr
    r = _run([])
    assert r.returncode != 0
    r = _run(["-i", str(tmp_path / "missing.txt")])
    assert r.returncode != 0 and "Invalid input file" in r.stderr


def _oracle_consensus(w, banded, bw=256):
    from oracle import oracle
    max_seq = max(len(s) for s in w)
    res = oracle.poa_window(w, banded=banded, band_width=bw, max_nodes=((4 if banded else 3) * max_seq + 3) // 4 * 4,
                            max_consensus=2 * max_seq, max_seqs=len(w))
    assert res.status == 0
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("banded", [True, False])
def test_cudapoa_file_consensus(tmp_path, banded):
    wins = synth.poa_windows(101, 10, 700, 8, 30, 30, 30)
    p = tmp_path / "windows.txt"
    _write_cudapoa(p, wins)
    args = ["-i", str(p)] + ([] if banded else ["-f"])
    r = _run(args)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")[:-1]
    assert len(lines) == len(wins)
    # one batch here, so the printed order is the input order (main.cpp:200-280)
    assert lines == [_oracle_consensus(w, banded).consensus for w in wins]


@pytest.mark.gpu
def test_cudapoa_print_order_follows_batch_bins(tmp_path):
    # main.cpp:189-289: windows are binned by get_multi_batch_sizes (utils.cu:24-138)
    # and printed batch by batch in each batch's group order.  A small memory
    # quota (-R) puts windows of different sizes into different capacity bins,
    # so the printed order differs from the input order; the expected order
    # comes from the same binning (C ABI) at the device's free memory.
    from claragenomicsanalysis_amd.cudapoa import get_multi_batch_sizes
    from claragenomicsanalysis_amd._lib import load_library
    import ctypes as C
    shapes = [(200, 4, 8), (2500, 6, 100), (900, 8, 40)]
    wins = []
    for k in range(3):
        for j, (L, n, e) in enumerate(shapes):
            wins += synth.poa_windows(131 + 10 * k + j, 1, L, n, e, e, e)
    quota = 0.002
    free, total = C.c_size_t(), C.c_size_t()
    hip = C.CDLL("libamdhip64.so")
    load_library()
    assert hip.hipMemGetInfo(C.byref(free), C.byref(total)) == 0
    groups = [[s.decode() for s in w] for w in wins]
    plans = [get_multi_batch_sizes(groups, banded_alignment=True, msa_flag=False, band_width=256,
                                   gpu_memory_usage_quota=quota, free_device_memory=int(free.value * f))
             for f in (0.95, 1.0, 1.05)]
    assert plans[0][1] == plans[1][1] == plans[2][1], "binning not stable around the free memory; adjust sizes"
    order = [g for batch in plans[1][1] for g in batch]
    assert order != list(range(len(wins))) and sorted(order) == list(range(len(wins)))
    p = tmp_path / "windows.txt"
    _write_cudapoa(p, wins)
    r = _run(["-i", str(p), "-R", str(quota)])
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")[:-1]
    assert lines == [_oracle_consensus(wins[g], True).consensus for g in order]


@pytest.mark.gpu
def test_max_groups_repeats_windows(tmp_path):
    wins = synth.poa_windows(103, 3, 400, 6, 20, 20, 20)
    p = tmp_path / "windows.txt"
    _write_cudapoa(p, wins)
    r = _run(["-i", str(p), "-M", "7"])
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")[:-1]
    assert len(lines) == 7
    assert lines == [_oracle_consensus(wins[i % 3], True).consensus for i in range(7)]


@pytest.mark.gpu
def test_fasta_msa_and_dot(tmp_path):
    wins = synth.poa_windows(107, 2, 500, 5, 25, 25, 25)
    paths = []
    for i, w in enumerate(wins):
        paths.append(tmp_path / f"w{i}.fa")
        _write_fasta(paths[-1], w)
    dot = tmp_path / "g.dot"
    args = []
    for p in paths:
        args += ["-i", str(p)]
    r = _run(args + ["-a", "-d", str(dot)])
    assert r.returncode == 0, r.stderr
    rows = r.stdout.split("\n")[:-1]
    from oracle import oracle
    expect = []
    for w in wins:
        max_seq = max(len(s) for s in w)
        res = oracle.poa_window(w, banded=True, band_width=256, msa=True, max_nodes=(4 * max_seq + 3) // 4 * 4,
                                max_consensus=2 * max_seq, max_seqs=len(w))
        expect += [m.decode() if isinstance(m, bytes) else m for m in res.msa]
    assert rows == expect  # one batch: windows in input order, rows in read order
    text = dot.read_text()
    assert text.count("digraph") == len(wins)

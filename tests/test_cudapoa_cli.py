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
    # windows are printed in get_multi_batch_sizes bin order (main.cpp:200-280)
    assert sorted(lines) == sorted(_oracle_consensus(w, banded).consensus for w in wins)


@pytest.mark.gpu
def test_max_groups_repeats_windows(tmp_path):
    wins = synth.poa_windows(103, 3, 400, 6, 20, 20, 20)
    p = tmp_path / "windows.txt"
    _write_cudapoa(p, wins)
    r = _run(["-i", str(p), "-M", "7"])
    assert r.returncode == 0, r.stderr
    lines = r.stdout.split("\n")[:-1]
    assert len(lines) == 7
    assert sorted(lines) == sorted(_oracle_consensus(wins[i % 3], True).consensus for i in range(7))


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
    assert sorted(rows) == sorted(expect)
    text = dot.read_text()
    assert text.count("digraph") == len(wins)

"""GPU tests of the concurrent multi-batch driver (reference
cudapoa/benchmarks/multi_batch.hpp:30-215; C++ MultiBatch in
csrc/poa_multibatch.cpp, called through the C ABI gwamd_poa_multibatch_*):
windows stream through several batches on their own streams and host threads,
and every window's consensus, coverage and status equal the oracle's."""
import os

import numpy as np
import pytest

from claragenomicsanalysis_amd import synth
from claragenomicsanalysis_amd.cudapoa import CudaPoaMultiBatch, estimate_max_poas, multibatch_file_assembly
from oracle import oracle

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "sample-golden-value.txt")


def mem_for(max_seq, reads, windows):
    """Device bytes per batch that give `windows` windows by the reference's
    capacity rule (BatchBlock::estimate_max_poas)."""
    probe = 64 << 30
    per = probe / estimate_max_poas(max_seq, reads, 256, banded=False, msa=False, free_device_memory=probe,
                                    gpu_memory_usage_quota=1.0)
    return int(per * windows) + (1 << 20)


def test_multibatch_many_rounds_bit_exact():
    # 240 windows of mixed size through 3 batches of ~40 windows: every batch
    # is refilled several times, windows are handed out in order under the mutex
    wins = synth.poa_windows(1001, 120, 180, 8, 9, 9, 9)
    wins += synth.poa_windows(2001, 80, 260, 6, 12, 12, 12)
    wins += synth.poa_windows(3001, 40, 60, 10, 4, 4, 4)
    wins.insert(17, [b"ACGT"])
    wins.insert(50, [b"GATTACA" * 30] * 3)
    mb = CudaPoaMultiBatch(10, 300, num_batches=3, mem_per_batch=mem_for(300, 10, 40))
    cons, cov, st = mb.process(wins)
    nb, per_batch, rounds = mb.info()
    assert nb == 3 and rounds >= len(wins) // per_batch and rounds > 3
    rc, rst, rcov, _, _ = oracle.poa_batch(wins, max_nodes=900, max_consensus=600, max_seqs=10, coverage=True)
    for i in range(len(wins)):
        assert (st[i], cons[i], cov[i]) == (int(rst[i]), rc[i], rcov[i]), i
    # a second pass over the same windows through the same batches is identical
    cons2, cov2, st2 = mb.process(wins)
    assert (cons2, cov2, st2) == (cons, cov, st)


def test_multibatch_config_b_shape_sample():
    # config-B-shaped windows (1 kb x 32 reads) in batches of ~300 windows, two
    # batches on two streams; all statuses ok, a sample spread over every batch
    # round bit-exact against the oracle
    n = 1500
    bases, lens = synth.poa_windows_packed(1, n, 1000, 32, 50, 50, 50)
    mb = CudaPoaMultiBatch(32, 1100, num_batches=2, mem_per_batch=mem_for(1100, 32, 300))
    status, clen, cons, cov = mb.process_packed(bases, lens.ravel(), np.full(n, 32))
    nb, per_batch, rounds = mb.info()
    assert rounds >= 5
    assert (status == 0).all() and (clen > 0).all()
    idx = np.linspace(0, n - 1, 10).astype(int)
    starts = np.concatenate([[0], np.cumsum(lens.ravel())])
    samp = [[bases[starts[r]:starts[r + 1]].tobytes() for r in range(i * 32, i * 32 + 32)] for i in idx]
    rc, rst, rcov, _, _ = oracle.poa_batch(samp, max_nodes=3300, max_consensus=2200, max_seqs=32, coverage=True)
    for j, i in enumerate(idx):
        assert rst[j] == status[i]
        assert rc[j] == cons[i, :clen[i]].tobytes().decode(), i
        assert rcov[j] == cov[i, :clen[i]].tolist(), i


def test_multibatch_overlong_window_is_skipped_not_stale():
    # a window whose longest read needs more score-matrix memory than a whole
    # batch has (reserve_buf fails on an empty batch, cudapoa_batch.cuh:542-564)
    # fits no batch; the reference's loop stops every thread there.  Here the
    # window gets exceeded_maximum_sequence_size (its read is longer than the
    # batch's 300), the rest are processed, and output arrays reused from an
    # earlier call never keep stale rows.
    wins = synth.poa_windows(4001, 30, 150, 6, 6, 6, 6)
    wins.insert(11, [b"ACGT" * 7500, b"ACGT" * 99])
    mb = CudaPoaMultiBatch(8, 300, num_batches=2, mem_per_batch=mem_for(300, 8, 7))
    flat = [r for w in wins for r in w]
    bases = np.frombuffer(b"".join(flat), np.uint8)
    lens = np.array([len(r) for r in flat], np.int32)
    rpw = [len(w) for w in wins]
    n = len(wins)
    stale = (np.full(n, 0, np.int32), np.full(n, 77, np.int32), np.full((n, mb.stride), 65, np.uint8),
             np.full((n, mb.stride), 9, np.uint16))
    mb.set_launch_timing(True)
    status, clen, cons, cov = mb.process_packed(bases, lens, rpw, out=stale)
    assert mb.skipped() == 1
    assert status[11] == 2 and clen[11] == 0  # exceeded_maximum_sequence_size
    rest = [w for i, w in enumerate(wins) if i != 11]
    rc, rst, rcov, _, _ = oracle.poa_batch(rest, max_nodes=900, max_consensus=600, max_seqs=8, coverage=True)
    j = 0
    for i in range(n):
        if i == 11:
            continue
        assert status[i] == rst[j] and cons[i, :clen[i]].tobytes().decode() == rc[j], i
        assert cov[i, :clen[i]].tolist() == rcov[j], i
        j += 1
    # launch records: every processed window is in exactly one launch, on one clock
    L = mb.launches()
    assert int(L["windows"].sum()) == n - 1
    assert (L["stop_ms"] >= L["start_ms"]).all() and (L["cells"] > 0).all()
    assert set(L["batch"].tolist()) <= {0, 1}


def test_multibatch_rejects_inconsistent_inputs():
    mb = CudaPoaMultiBatch(4, 300, num_batches=1, mem_per_batch=mem_for(300, 4, 4))
    with pytest.raises(ValueError):
        mb.process_packed(np.zeros(10, np.uint8), np.array([5, 5], np.int32), [3])
    with pytest.raises(ValueError):
        mb.process_packed(np.zeros(9, np.uint8), np.array([5, 5], np.int32), [2])
    with pytest.raises(ValueError):
        mb.process_packed(np.zeros(10, np.uint8), np.array([5, 5], np.int32), [-1, 3])


@pytest.mark.skipif(not os.environ.get("GWAMD_SAMPLE_WINDOWS"),
                    reason="cudapoa/data/sample-windows.txt is not in the reference snapshot "
                           "(.MISSING_LARGE_BLOBS); set GWAMD_SAMPLE_WINDOWS to a copy to run")
@pytest.mark.parametrize("batches", [2, 4])
def test_end2end_golden_assembly(batches):
    # Test_CudapoaBatchEnd2End.cu:33-85: MultiBatch(batches, sample-windows.txt),
    # process_batches(), assembly() == sample-golden-value.txt
    want = open(GOLDEN).read().strip()
    assert multibatch_file_assembly(os.environ["GWAMD_SAMPLE_WINDOWS"], batches) == want

"""Host-side cudapoa utilities (no GPU): window file formats and
get_multi_batch_sizes binning (cudapoa/include/.../utils.hpp:48-175,
cudapoa/src/utils.cu:24-138), checked against a restatement of the reference's
binning loop over the library's own estimate_max_poas."""
import random

import pytest

from claragenomicsanalysis_amd import cudapoa


def ref_binning(groups, free, banded=True, msa=False, bw=256, bins=None, quota=0.9):
    # utils.cu:36-137, with BatchBlock::estimate_max_poas from the library
    n = len(groups)
    max_len = [max(len(r) for r in g) for g in groups]
    max_poas = [cudapoa.estimate_max_poas(max_len[i], len(groups[i]), bw, banded, msa, free, quota)
                for i in range(n)]
    bins = bins or [1 << j for j in range(20)]
    nb = len(bins)
    freq, blen, bnr, blist = [0] * nb, [0] * nb, [0] * nb, [[] for _ in range(nb)]
    for i in range(n):
        cur = max_len[i] * len(groups[i])
        for j in range(nb):
            if max_poas[i] <= bins[j] or j == nb - 1:
                freq[j] += 1
                blist[j].append(i)
                if blen[j] * bnr[j] < cur:
                    blen[j], bnr[j] = max_len[i], len(groups[i])
                break
    sizes, per = [], []
    for j in range(nb):
        if freq[j] > 0:
            sizes.append((blen[j], bnr[j]))
            per.append(list(blist[j]))
            for k in range(j + 1, nb):
                if freq[k] > 0:
                    if bins[j] >= freq[k]:
                        per[-1].extend(blist[k])
                        freq[k] = 0
                    else:
                        break
    return sizes, per


def _groups(seed, n):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        L = rng.choice([300, 600, 1000, 2000, 5000, 12000])
        out.append(["A" * rng.randint(L // 2, L)] + ["C" * rng.randint(1, L)] * rng.randint(1, 40))
    return out


@pytest.mark.parametrize("free_gb", [1, 16, 200])
@pytest.mark.parametrize("banded,msa", [(True, False), (False, False), (True, True)])
def test_multi_batch_sizes_match_reference_binning(free_gb, banded, msa):
    groups = _groups(free_gb * 7 + banded + 2 * msa, 60)
    free = free_gb << 30
    got = cudapoa.get_multi_batch_sizes(groups, banded, msa, free_device_memory=free)
    assert got == ref_binning(groups, free, banded, msa)
    # every group lands in exactly one batch
    assert sorted(g for b in got[1] for g in b) == list(range(len(groups)))


def test_multi_batch_sizes_custom_bins():
    groups = _groups(5, 40)
    bins = [2, 8, 32, 128, 512]
    got = cudapoa.get_multi_batch_sizes(groups, bins_capacity=bins, free_device_memory=4 << 30)
    assert got == ref_binning(groups, 4 << 30, bins=bins)


def test_estimate_max_poas_monotone():
    small = cudapoa.estimate_max_poas(1000, 32, free_device_memory=64 << 30)
    big = cudapoa.estimate_max_poas(10000, 32, free_device_memory=64 << 30)
    assert small > big > 0
    assert cudapoa.estimate_max_poas(1000, 32, free_device_memory=128 << 30) >= 2 * small - 1


def test_parse_cudapoa_file_and_resize(tmp_path):
    p = tmp_path / "w.txt"
    p.write_text("2\nACGT\nACGA\n3\nTTT\nTTA\nTTG\n1\nGG\n")
    w = cudapoa.parse_cudapoa_file(str(p))
    assert w == [["ACGT", "ACGA"], ["TTT", "TTA", "TTG"], ["GG"]]
    assert cudapoa.parse_cudapoa_file(str(p), 2) == w[:2]
    # fewer windows than asked: repeated in order (utils.hpp:68-86)
    assert cudapoa.parse_cudapoa_file(str(p), 5) == w + w[:2]


def test_parse_fasta_files(tmp_path):
    a = tmp_path / "a.fa"
    a.write_text(">r1\nACGT\nAC\n>r2 desc\nGGG\n")
    b = tmp_path / "b.fa"
    b.write_text(">x\nTTTT\n")
    assert cudapoa.parse_fasta_files([str(a), str(b)]) == [["ACGTAC", "GGG"], ["TTTT"]]


@pytest.mark.gpu
def test_multi_batch_sizes_on_device_and_batches_run():
    # free device memory queried (hipMemGetInfo, utils.cu:40-44); every group
    # lands in exactly one batch, and a batch created with its size takes its
    # groups and runs.  As in the reference, a merged bin keeps the batch size
    # of its own largest group (utils.cu:111-130), so a group merged from
    # another bin may bring more reads than max_sequences_per_poa: those reads
    # get exceeded_maximum_sequences_per_poa (3) and are dropped
    from claragenomicsanalysis_amd import synth
    from claragenomicsanalysis_amd.cudapoa import CudaPoaBatch
    groups = synth.poa_windows(5, 6, 300, 6, 15, 15, 15) + synth.poa_windows(9, 4, 1500, 4, 60, 60, 60)
    sizes, per_batch = cudapoa.get_multi_batch_sizes(groups, gpu_memory_usage_quota=0.5)
    assert sorted(i for b in per_batch for i in b) == list(range(len(groups)))
    for (max_seq, max_reads), ids in zip(sizes, per_batch):
        if not ids:
            continue
        b = CudaPoaBatch(max_reads, max_seq, 2 << 30, cuda_banded_alignment=True)
        for i in ids:
            st, seq_st = b.add_poa_group(list(groups[i]))
            assert st == 0
            assert seq_st == [0 if k < max_reads else 3 for k in range(len(groups[i]))]
        b.generate_poa()
        _, _, st = b.get_consensus()
        assert all(s == 0 for s in st)

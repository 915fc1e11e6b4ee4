"""Python API for MI355X batched POA; mirrors pygenomeworks'
``genomeworks.cudapoa.CudaPoaBatch`` (pygenomeworks/genomeworks/cudapoa/cudapoa.pyx:19-320):
same constructor arguments and defaults, same methods and return shapes.
Everything runs through the C ABI of libgwamd.so (include/gwamd_cudapoa.h).
"""
import ctypes as C

import numpy as np

from ._lib import load_library, last_error

MAX_EDGES = 50

# StatusType (cudapoa.hpp:26-38)
STATUS_NAMES = ["success", "exceeded_maximum_poas", "exceeded_maximum_sequence_size",
                "exceeded_maximum_sequences_per_poa", "node_count_exceeded_maximum_graph_size",
                "edge_count_exceeded_maximum_graph_size", "seq_len_exceeded_maximum_nodes_per_window",
                "loop_count_exceeded_upper_bound", "output_type_unavailable", "generic_error"]
SUCCESS = 0
OUTPUT_TYPE_UNAVAILABLE = 8
CONSENSUS = 0x1
MSA = 0x2


def status_to_str(status):
    """cudapoa.pyx:19-40."""
    if 0 <= int(status) < len(STATUS_NAMES):
        return STATUS_NAMES[int(status)]
    raise RuntimeError("Unknown error status : " + str(status))


class BatchSize(C.Structure):
    """cudapoa::BatchSize (batch.hpp:53-129)."""
    _fields_ = [(n, C.c_int32) for n in (
        "max_sequence_size", "max_consensus_size", "max_nodes_per_window", "max_nodes_per_window_banded",
        "max_matrix_graph_dimension", "max_matrix_graph_dimension_banded", "max_matrix_sequence_dimension",
        "alignment_band_width", "max_sequences_per_poa")]

    @classmethod
    def make(cls, max_seq_sz=1024, max_seq_per_poa=100, band_width=256):
        bs = cls()
        _check(load_library().gwamd_poa_batch_size_init(C.byref(bs), max_seq_sz, max_seq_per_poa, band_width))
        return bs

    @classmethod
    def make_full(cls, max_seq_sz, max_consensus_sz, max_nodes_per_w, max_nodes_per_w_banded, band_width,
                  max_seq_per_poa):
        bs = cls()
        _check(load_library().gwamd_poa_batch_size_init_full(C.byref(bs), max_seq_sz, max_consensus_sz,
                                                             max_nodes_per_w, max_nodes_per_w_banded, band_width,
                                                             max_seq_per_poa))
        return bs


def _check(rc):
    if rc == -1:
        raise ValueError(last_error())
    if rc < 0:
        raise RuntimeError(last_error())
    return rc


class DiGraph:
    """Minimal directed graph returned by get_graphs (the reference returns a
    networkx.DiGraph, cudapoa.pyx:268-288; networkx is not a dependency here)."""

    def __init__(self):
        self._succ = {}
        self._labels = {}
        self._weights = {}

    def add_edge(self, u, v, weight=0):
        self._succ.setdefault(u, set())
        self._succ.setdefault(v, set())
        if v not in self._succ[u]:
            self._succ[u].add(v)
            self._weights[(u, v)] = weight

    def add_node(self, n, label=None):
        self._succ.setdefault(n, set())
        if label is not None:
            self._labels[n] = label

    @property
    def nodes(self):
        return sorted(self._succ)

    @property
    def edges(self):
        return sorted(self._weights)

    def number_of_nodes(self):
        return len(self._succ)

    def number_of_edges(self):
        return len(self._weights)

    def label(self, n):
        return self._labels.get(n, "")

    def weight(self, u, v):
        return self._weights[(u, v)]


class CudaPoaBatch:
    """Python API for MI355X partial order alignment (cudapoa.pyx:60-320)."""

    def __init__(self, max_sequences_per_poa, max_sequence_size, max_gpu_mem, output_type="consensus",
                 device_id=0, stream=None, gap_score=-8, mismatch_score=-6, match_score=8,
                 cuda_banded_alignment=False, alignment_band_width=256, max_consensus_size=None,
                 max_nodes_per_window=None, max_nodes_per_window_banded=None, spoa_accurate=None, *args, **kwargs):
        self._lib = load_library()
        self._handle = C.c_void_p()
        if stream is None:
            st = None
        elif isinstance(stream, int):
            st = stream
        elif hasattr(stream, "cuda_stream"):  # torch.cuda.Stream
            st = stream.cuda_stream
        elif hasattr(stream, "stream"):
            st = stream.stream
        else:
            raise RuntimeError("Type for stream option must be a HIP stream handle")
        if output_type == "consensus":
            output_mask = CONSENSUS
        elif output_type == "msa":
            output_mask = MSA
        elif output_type in ("both", "consensus+msa"):
            output_mask = CONSENSUS | MSA
        else:
            raise RuntimeError("Unknown output_type provided. Must be consensus/msa.")
        self.output_type = output_type
        mx_cons = 2 * max_sequence_size if max_consensus_size is None else max_consensus_size
        mx_nodes = 3 * max_sequence_size if max_nodes_per_window is None else max_nodes_per_window
        mx_nodes_b = 4 * max_sequence_size if max_nodes_per_window_banded is None else max_nodes_per_window_banded
        self.batch_size = BatchSize.make_full(max_sequence_size, mx_cons, mx_nodes, mx_nodes_b,
                                              alignment_band_width, max_sequences_per_poa)
        _check(self._lib.gwamd_poa_create_batch(C.byref(self._handle), device_id, st, int(max_gpu_mem),
                                                output_mask, C.byref(self.batch_size), gap_score, mismatch_score,
                                                match_score, int(bool(cuda_banded_alignment))))
        if spoa_accurate is not None:  # None: GWAMD_SPOA_ACCURATE decides (reference: build option)
            self.set_spoa_accurate(spoa_accurate)

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            self._lib.gwamd_poa_destroy_batch(h)
            self._handle = None

    def add_poa_group(self, poa, weights=None):
        """cudapoa.pyx:147-178; returns (status, per-sequence status list)."""
        if not isinstance(poa, list):
            poa = [poa]
        if len(poa) < 1:
            raise RuntimeError("At least one sequence must be present in POA group")
        n = len(poa)
        data = [s.encode() if isinstance(s, str) else bytes(s) for s in poa]
        seqs = (C.c_char_p * n)(*data)
        lens = (C.c_int32 * n)(*[len(d) for d in data])
        wptrs = None
        keep = []
        if weights is not None:
            wptrs = (C.c_void_p * n)()
            for i, w in enumerate(weights):
                if w is None:
                    wptrs[i] = None
                else:
                    a = np.ascontiguousarray(w, dtype=np.int8)
                    keep.append(a)
                    wptrs[i] = a.ctypes.data
        seq_status = (C.c_int32 * n)()
        rc = _check(self._lib.gwamd_poa_add_poa_group(self._handle, seqs, wptrs, lens, n, seq_status))
        return rc, list(seq_status)

    @property
    def total_poas(self):
        return self._lib.gwamd_poa_get_total_poas(self._handle)

    @property
    def batch_id(self):
        return self._lib.gwamd_poa_batch_id(self._handle)

    def generate_poa(self):
        _check(self._lib.gwamd_poa_generate_poa(self._handle))

    # split form of generate_poa used by bench.py
    def upload(self):
        _check(self._lib.gwamd_poa_upload(self._handle))

    def launch(self):
        _check(self._lib.gwamd_poa_launch(self._handle))

    def synchronize(self):
        _check(self._lib.gwamd_poa_synchronize(self._handle))

    def get_consensus(self):
        """cudapoa.pyx:226-245: (consensus list, coverage list, status list)."""
        n = self.total_poas
        status = (C.c_int32 * max(n, 1))()
        lens = (C.c_int32 * max(n, 1))()
        cbase, vbase, stride = C.c_void_p(), C.c_void_p(), C.c_int32()
        rc = _check(self._lib.gwamd_poa_get_consensus(self._handle, status, lens, C.byref(cbase), C.byref(vbase),
                                                      C.byref(stride)))
        if rc == OUTPUT_TYPE_UNAVAILABLE:
            raise RuntimeError("Output type not requested during batch initialization")
        cons, covs = [], []
        for i in range(n):
            L = lens[i]
            if L > 0:
                cons.append(C.string_at(cbase.value + i * stride.value, L).decode())
                buf = (C.c_uint16 * L).from_address(vbase.value + 2 * i * stride.value)
                covs.append(list(buf))
            else:
                cons.append("")
                covs.append([])
        return cons, covs, [status[i] for i in range(n)]

    def get_consensus_raw(self):
        """Batch::get_consensus (D2H + the C++ result vectors) without building
        Python strings: returns (status int32[n], lengths int32[n], consensus
        base address, coverage base address, stride).  The buffers stay valid
        until the next generate_poa / reset."""
        n = self.total_poas
        status = np.zeros(max(n, 1), np.int32)
        lens = np.zeros(max(n, 1), np.int32)
        cbase, vbase, stride = C.c_void_p(), C.c_void_p(), C.c_int32()
        rc = _check(self._lib.gwamd_poa_get_consensus(
            self._handle, status.ctypes.data_as(C.POINTER(C.c_int32)), lens.ctypes.data_as(C.POINTER(C.c_int32)),
            C.byref(cbase), C.byref(vbase), C.byref(stride)))
        if rc == OUTPUT_TYPE_UNAVAILABLE:
            raise RuntimeError("Output type not requested during batch initialization")
        return status[:n], lens[:n], cbase.value, vbase.value, stride.value

    def get_msa(self):
        """cudapoa.pyx:207-224: (list of per-window MSA row lists, status list)."""
        n = self.total_poas
        status = (C.c_int32 * max(n, 1))()
        rows = (C.c_int32 * max(n, 1))()
        base, rstride, mseq = C.c_void_p(), C.c_int32(), C.c_int32()
        rc = _check(self._lib.gwamd_poa_get_msa(self._handle, status, rows, C.byref(base), C.byref(rstride),
                                                C.byref(mseq)))
        if rc == OUTPUT_TYPE_UNAVAILABLE:
            raise RuntimeError("Output type not requested during batch initialization")
        out = []
        for i in range(n):
            msa = []
            for s in range(rows[i]):
                msa.append(C.string_at(base.value + (i * mseq.value + s) * rstride.value).decode())
            out.append(msa)
        return out, [status[i] for i in range(n)]

    def get_graphs(self):
        """cudapoa.pyx:247-288: (list of DiGraph, status list)."""
        n = self.total_poas
        status = (C.c_int32 * max(n, 1))()
        nodes = (C.c_int32 * max(n, 1))()
        b, cnt, ie, iw = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        mn = C.c_int32()
        _check(self._lib.gwamd_poa_get_graphs(self._handle, status, nodes, C.byref(b), C.byref(cnt), C.byref(ie),
                                              C.byref(iw), C.byref(mn)))
        graphs = []
        M = mn.value
        for w in range(n):
            g = DiGraph()
            if status[w] == SUCCESS:
                nn = nodes[w]
                labels = C.string_at(b.value + w * M, nn)
                counts = np.ctypeslib.as_array((C.c_uint16 * (nn or 1)).from_address(cnt.value + 2 * w * M))
                edges = np.ctypeslib.as_array((C.c_int32 * (nn * MAX_EDGES or 1)).from_address(
                    ie.value + 4 * w * M * MAX_EDGES))
                wts = np.ctypeslib.as_array((C.c_uint16 * (nn * MAX_EDGES or 1)).from_address(
                    iw.value + 2 * w * M * MAX_EDGES))
                for v in range(nn):
                    for e in range(int(counts[v])):
                        g.add_edge(int(edges[v * MAX_EDGES + e]), v, weight=int(wts[v * MAX_EDGES + e]))
                for v in g.nodes:
                    g.add_node(v, chr(labels[v]) if v < nn else "")
            graphs.append(g)
        return graphs, [status[i] for i in range(n)]

    def get_stats(self):
        """Per-window DP cell counts and final node counts of the last run."""
        n = self.total_poas
        cells = np.zeros(max(n, 1), np.int64)
        fn = np.zeros(max(n, 1), np.int32)
        _check(self._lib.gwamd_poa_get_stats(self._handle, cells.ctypes.data_as(C.POINTER(C.c_int64)),
                                             fn.ctypes.data_as(C.POINTER(C.c_int32))))
        return cells[:n], fn[:n]

    PHASES = ("backbone", "forward", "traceback", "add", "topsort", "output", "rowprog", "total")

    def get_phase_ticks(self):
        """Per-window in-kernel phase timers (s_memrealtime ticks at 100 MHz), shape (n, 8)."""
        n = self.total_poas
        out = np.zeros((max(n, 1), len(self.PHASES)), np.int64)
        _check(self._lib.gwamd_poa_get_phase_ticks(self._handle, out.ctypes.data_as(C.POINTER(C.c_int64))))
        return out[:n]

    def get_types(self):
        """(score bits, size bits) chosen by create_batch (cudapoa_limits.hpp:28-53)."""
        sb, zb = C.c_int32(), C.c_int32()
        self._lib.gwamd_poa_get_types(self._handle, C.byref(sb), C.byref(zb))
        return sb.value, zb.value


    def kernel_variant(self):
        """1: global-memory kernel, 2: LDS-resident kernel (full), 3: banded kernel,
        4: banded kernel with the anti-diagonal forward pass (poa_band_ad.hpp)."""
        sb, zb = C.c_int32(), C.c_int32()
        return self._lib.gwamd_poa_get_types(self._handle, C.byref(sb), C.byref(zb))

    def set_spoa_accurate(self, on=True):
        """SPOA_ACCURATE mode (cudapoa_kernels.cuh:324-337): racon DFS sort after every read.
        Returns the previous setting."""
        return bool(self._lib.gwamd_poa_set_spoa_accurate(self._handle, int(bool(on))))

    def get_capacity(self):
        nb, mp = C.c_int64(), C.c_int32()
        self._lib.gwamd_poa_get_capacity(self._handle, C.byref(nb), C.byref(mp))
        return nb.value, mp.value

    def get_grid(self):
        """(scratch slots, resident workgroups on the device) of the persistent
        grid; resident 0 means the global-memory kernel (one workgroup per window)."""
        sl, rs = C.c_int32(), C.c_int32()
        self._lib.gwamd_poa_get_grid(self._handle, C.byref(sl), C.byref(rs))
        return sl.value, rs.value

    def reset(self):
        self._lib.gwamd_poa_reset(self._handle)


class CudaPoaMultiBatch:
    """Concurrent multi-batch driver (reference cudapoa/benchmarks/multi_batch.hpp:30-215):
    num_batches batches, each on its own HIP stream and host thread, fed windows
    in order under a mutex; consensus output.  mem_per_batch 0 takes 0.9 x free
    device memory / num_batches, as the reference does."""

    def __init__(self, max_sequences_per_poa, max_sequence_size, num_batches=2, mem_per_batch=0, device_id=0,
                 gap_score=-8, mismatch_score=-6, match_score=8, cuda_banded_alignment=False,
                 alignment_band_width=256, max_consensus_size=None):
        self._lib = load_library()
        _declare_multibatch(self._lib)
        self._handle = C.c_void_p()
        mx_cons = 2 * max_sequence_size if max_consensus_size is None else max_consensus_size
        self.batch_size = BatchSize.make_full(max_sequence_size, mx_cons, 3 * max_sequence_size,
                                              4 * max_sequence_size, alignment_band_width, max_sequences_per_poa)
        self.stride = mx_cons
        _check(self._lib.gwamd_poa_multibatch_create(C.byref(self._handle), device_id, num_batches,
                                                     int(mem_per_batch), CONSENSUS, C.byref(self.batch_size),
                                                     gap_score, mismatch_score, match_score,
                                                     int(bool(cuda_banded_alignment))))

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            self._lib.gwamd_poa_multibatch_destroy(h)
            self._handle = None

    def process_packed(self, bases, read_lens, reads_per_window, out=None):
        """bases: uint8 array of all reads back to back; read_lens: int32 per read;
        reads_per_window: reads of each window, in order.  Returns (status, lengths,
        consensus uint8[n, stride], coverage uint16[n, stride]); pass `out` (a tuple
        from an earlier call of the same size) to reuse the output arrays."""
        read_lens = np.ascontiguousarray(read_lens, dtype=np.int32).ravel()
        rpw = np.asarray(reads_per_window, dtype=np.int64).ravel()
        n = len(rpw)
        if (rpw < 0).any() or (read_lens < 0).any():
            raise ValueError("negative read count or read length")
        first = np.zeros(n + 1, np.int64)
        np.cumsum(rpw, out=first[1:])
        if first[-1] != len(read_lens):
            raise ValueError("reads_per_window sums to %d, but %d read lengths were given"
                             % (int(first[-1]), len(read_lens)))
        off = np.zeros(len(read_lens), np.int64)
        if len(read_lens) > 1:
            np.cumsum(read_lens[:-1], out=off[1:])
        bases = np.ascontiguousarray(bases, dtype=np.uint8).ravel()
        if int(read_lens.sum(dtype=np.int64)) > len(bases):
            raise ValueError("read lengths sum to %d bases, but only %d were given"
                             % (int(read_lens.sum(dtype=np.int64)), len(bases)))
        if out is None:
            out = (np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros((n, self.stride), np.uint8),
                   np.zeros((n, self.stride), np.uint16))
        status, lens, cons, cov = out
        self._inputs = (bases, read_lens, first, off)
        _check(self._lib.gwamd_poa_multibatch_process(
            self._handle, bases.ctypes.data, off.ctypes.data, read_lens.ctypes.data, first.ctypes.data, n,
            status.ctypes.data, lens.ctypes.data, cons.ctypes.data, cov.ctypes.data, self.stride))
        return out

    def process(self, windows):
        """windows: list of lists of reads (str/bytes).  Returns (consensus, coverage, status) lists."""
        data = [[r.encode() if isinstance(r, str) else bytes(r) for r in w] for w in windows]
        flat = b"".join(b"".join(w) for w in data)
        lens = np.array([len(r) for w in data for r in w], np.int32)
        rpw = [len(w) for w in data]
        status, ln, cons, cov = self.process_packed(np.frombuffer(flat, np.uint8), lens, rpw)
        cs = [cons[i, :ln[i]].tobytes().decode() for i in range(len(data))]
        cv = [cov[i, :ln[i]].tolist() for i in range(len(data))]
        return cs, cv, status.tolist()

    def set_launch_timing(self, on=True):
        """Record HIP events around every kernel launch of the next process calls
        (bench.py config E roofline).  Returns the previous setting."""
        return bool(self._lib.gwamd_poa_multibatch_set_launch_timing(self._handle, int(bool(on))))

    def launches(self):
        """Kernel launches of the last process (launch timing on), sorted by start:
        dict of arrays start_ms, stop_ms (ms after the call began, one clock for
        all streams), cells (DP cells), windows, batch."""
        n = self._lib.gwamd_poa_multibatch_launches(self._handle, None, None, None, None, None, 0)
        out = {"start_ms": np.zeros(n, np.float32), "stop_ms": np.zeros(n, np.float32),
               "cells": np.zeros(n, np.int64), "windows": np.zeros(n, np.int32), "batch": np.zeros(n, np.int32)}
        self._lib.gwamd_poa_multibatch_launches(self._handle, out["start_ms"].ctypes.data, out["stop_ms"].ctypes.data,
                                                out["cells"].ctypes.data, out["windows"].ctypes.data,
                                                out["batch"].ctypes.data, n)
        return out

    def skipped(self):
        """Windows of the last process that fit no empty batch (they carry their
        add_poa_group status, e.g. exceeded_maximum_sequence_size)."""
        return int(self._lib.gwamd_poa_multibatch_skipped(self._handle))

    def info(self):
        """(batches, the most windows one batch took, generate_poa calls) of the last process."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        self._lib.gwamd_poa_multibatch_info(self._handle, C.byref(a), C.byref(b), C.byref(c))
        return a.value, b.value, c.value


def multibatch_file_assembly(filename, num_batches=2, total_windows=-1):
    """MultiBatch(num_batches, filename, total_windows).process_batches().assembly()
    (Test_CudapoaBatchEnd2End.cu:55-69)."""
    L = load_library()
    _declare_multibatch(L)
    n = C.c_int64()
    _check(L.gwamd_poa_multibatch_run_file(str(filename).encode(), num_batches, total_windows, None, 0, C.byref(n)))
    buf = C.create_string_buffer(n.value + 1)
    _check(L.gwamd_poa_multibatch_run_file(str(filename).encode(), num_batches, total_windows, buf, n.value,
                                           C.byref(n)))
    return buf.raw[:n.value].decode()


def _declare_multibatch(L):
    if getattr(L, "_mb_declared", False):
        return
    vp, i8, i16, i32, i64, sz = C.c_void_p, C.c_int8, C.c_int16, C.c_int32, C.c_int64, C.c_size_t
    P = C.POINTER
    L.gwamd_poa_multibatch_create.restype = i32
    L.gwamd_poa_multibatch_create.argtypes = [P(vp), i32, i32, sz, i8, vp, i16, i16, i16, i32]
    L.gwamd_poa_multibatch_destroy.restype = None
    L.gwamd_poa_multibatch_destroy.argtypes = [vp]
    L.gwamd_poa_multibatch_process.restype = i32
    L.gwamd_poa_multibatch_process.argtypes = [vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, i32]
    L.gwamd_poa_multibatch_info.restype = i32
    L.gwamd_poa_multibatch_info.argtypes = [vp, P(i32), P(i32), P(i32)]
    L.gwamd_poa_multibatch_set_launch_timing.restype = i32
    L.gwamd_poa_multibatch_set_launch_timing.argtypes = [vp, i32]
    L.gwamd_poa_multibatch_launches.restype = i32
    L.gwamd_poa_multibatch_launches.argtypes = [vp, vp, vp, vp, vp, vp, i32]
    L.gwamd_poa_multibatch_skipped.restype = i32
    L.gwamd_poa_multibatch_skipped.argtypes = [vp]
    L.gwamd_poa_multibatch_run_file.restype = i32
    L.gwamd_poa_multibatch_run_file.argtypes = [C.c_char_p, i32, i32, vp, i64, P(i64)]
    L._mb_declared = True


# --- window batching (cudapoa/include/.../utils.hpp:48-66, cudapoa/src/utils.cu:24-138) ---

def _declare_utils(L):
    i32, i64, u64, f32, vp = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_void_p
    L.gwamd_poa_estimate_max_poas.restype = i64
    L.gwamd_poa_estimate_max_poas.argtypes = [i32, i32, i32, i32, i32, u64, f32, i32, i32, i32]
    L.gwamd_poa_get_multi_batch_sizes.restype = i32
    L.gwamd_poa_get_multi_batch_sizes.argtypes = [vp, vp, i32, u64, i32, i32, i32, vp, i32, f32, i32, i32, i32,
                                                  vp, vp, vp, vp, vp]


def estimate_max_poas(max_sequence_size, max_sequences_per_poa, band_width=256, banded=True, msa=False,
                      free_device_memory=0, gpu_memory_usage_quota=0.9, mismatch=-6, gap=-8, match=8):
    """BatchBlock::estimate_max_poas (allocate_block.hpp:364-401); free_device_memory 0
    queries the current device."""
    L = load_library()
    _declare_utils(L)
    r = L.gwamd_poa_estimate_max_poas(int(max_sequence_size), int(max_sequences_per_poa), int(band_width),
                                      int(bool(banded)), int(bool(msa)), int(free_device_memory),
                                      float(gpu_memory_usage_quota), int(mismatch), int(gap), int(match))
    _check(int(r) if r < 0 else 0)
    return int(r)


def get_multi_batch_sizes(groups, banded_alignment=True, msa_flag=False, band_width=256, bins_capacity=None,
                          gpu_memory_usage_quota=0.9, mismatch_score=-6, gap_score=-8, match_score=8,
                          free_device_memory=0):
    """Bins POA groups (lists of reads) into batch sizes, as the reference's
    get_multi_batch_sizes.  Returns (list of (max_sequence_size,
    max_sequences_per_poa), list of group-index lists per batch)."""
    L = load_library()
    _declare_utils(L)
    n = len(groups)
    ml = np.array([max([len(r) for r in g] + [0]) for g in groups], np.int32)
    nr = np.array([len(g) for g in groups], np.int32)
    bins = np.array(bins_capacity, np.int32) if bins_capacity is not None else None
    nb = np.zeros(1, np.int32)
    bmax = np.zeros(max(n, 1), np.int32)
    bnr = np.zeros(max(n, 1), np.int32)
    gb = np.full(max(n, 1), -1, np.int32)
    gr = np.zeros(max(n, 1), np.int32)
    _check(L.gwamd_poa_get_multi_batch_sizes(
        ml.ctypes.data, nr.ctypes.data, n, int(free_device_memory), int(bool(banded_alignment)), int(bool(msa_flag)),
        int(band_width), bins.ctypes.data if bins is not None else None, len(bins) if bins is not None else 0,
        float(gpu_memory_usage_quota), int(mismatch_score), int(gap_score), int(match_score),
        nb.ctypes.data, bmax.ctypes.data, bnr.ctypes.data, gb.ctypes.data, gr.ctypes.data))
    k = int(nb[0])
    sizes = [(int(bmax[b]), int(bnr[b])) for b in range(k)]
    per_batch = [[] for _ in range(k)]
    for g in sorted(range(n), key=lambda g: (gb[g], gr[g])):
        per_batch[int(gb[g])].append(g)
    return sizes, per_batch


def parse_cudapoa_file(filename, total_windows=-1):
    """cudapoa window format (utils.hpp:88-132): a count line, then that many reads."""
    windows, left = [], 0
    with open(filename) as f:
        for line in f:
            line = line.rstrip("\n")
            if left == 0:
                left = int(line.split()[0]) if line.split() else 0
                windows.append([])
            else:
                windows[-1].append(line)
                left -= 1
    return resize_windows(windows, total_windows)


def parse_fasta_files(paths, total_windows=-1):
    """One window per FASTA file, its records in file order (utils.hpp:142-157)."""
    windows = []
    for p in paths:
        recs = []
        with open(p) as f:
            for line in f:
                line = line.rstrip("\r\n")
                if line.startswith(">"):
                    recs.append("")
                elif recs:
                    recs[-1] += line
        windows.append(recs)
    return resize_windows(windows, total_windows)


def resize_windows(windows, total_windows):
    """Truncate or cyclically repeat to total_windows; -1 keeps all (utils.hpp:68-86)."""
    if total_windows is None or total_windows < 0:
        return windows
    if len(windows) > total_windows:
        return windows[:total_windows]
    read = len(windows)
    while len(windows) < total_windows:
        windows.append(windows[len(windows) - read])
    return windows

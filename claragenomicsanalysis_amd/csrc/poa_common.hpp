// Shared host/device definitions for the MI355X POA path.
//
// Layout summary (DESIGN.md "Data layout in HBM"): every per-window buffer is a
// fixed-capacity slot of one batch-wide allocation, window w at offset
// w * capacity.  Graph adjacency keeps the reference's fixed 50-slot lists
// (cudapoa_structs.cuh:17-21) so edge/alignment overflow errors fire at exactly
// the same point as in the reference.
#pragma once

#include <cstdint>

namespace gwamd
{
namespace poa
{

constexpr int kMaxEdges      = 50; // CUDAPOA_MAX_NODE_EDGES (cudapoa_structs.cuh:18)
constexpr int kMaxAlignments = 50; // CUDAPOA_MAX_NODE_ALIGNMENTS (cudapoa_structs.cuh:21)
constexpr int kBandPad       = 8;  // CUDAPOA_BANDED_MATRIX_RIGHT_PADDING (cudapoa_structs.cuh:27)
constexpr int kWave          = 64; // CDNA wavefront
constexpr int kCellsPerLane  = 8;  // full-mode DP: 8 consecutive columns per lane
constexpr int kChunk         = kWave * kCellsPerLane; // 512 columns per wave pass
constexpr int kAdRing        = 128; // LDS ring rows of the banded anti-diagonal pass (poa_band_ad.hpp)
constexpr int kAdSpillDist   = kAdRing - kWave + 1; // successor distance that needs a spill row there
// banded kernel (poa_band.hip): LDS ring rows (power of two) and traceback
// tile rows per cells-per-lane value.  Band widths past 512 take a 32-row
// tile and, at 1,024, an 8-row ring, so four windows share a CU (one wave per
// SIMD) instead of two; the host plan (plan_band_kernel) sizes the LDS image
// from the same two functions
constexpr int band_ring_rows(int cpl) { return cpl >= 16 ? 8 : 16; }
constexpr int band_tile_rows(int cpl) { return cpl >= 10 ? 32 : 64; }
constexpr int kReadGuard     = 64;  // banded kernel: LDS bytes in front of the staged read
constexpr int kAdMaxWaves    = 4;   // waves of a banded workgroup running the anti-diagonal pass
constexpr int kColShift      = 7;  // column j of a full-mode score row lives at index j + 7,
                                   // so each lane's 8 cells are one 16-B aligned group

// StatusType (cudapoa.hpp:26-38); values are ABI.
enum Status : uint8_t
{
    kSuccess               = 0,
    kExceededMaxPoas       = 1,
    kExceededMaxSeqSize    = 2,
    kExceededMaxSeqsPerPoa = 3,
    kNodeCountExceeded     = 4,
    kEdgeCountExceeded     = 5,
    kSeqLenExceededNodes   = 6,
    kLoopCountExceeded     = 7,
    kOutputTypeUnavailable = 8,
    kGenericError          = 9,
};

// One window of the packed input batch.
struct WindowDesc
{
    int32_t first_seq; // index of the window's first read in seq_len / seq_off
    int32_t num_seqs;
};

// Capacities, identical for every window of a batch.
struct Dims
{
    int32_t max_nodes;     // graph node capacity (BatchSize max_nodes_per_window[_banded])
    int32_t max_seqs;      // reads per window
    int32_t max_seq_len;   // BatchSize max_sequence_size
    int32_t max_consensus; // BatchSize max_consensus_size
    int32_t score_stride;  // ScoreT elements per score row
    int32_t score_rows;    // rows per window score matrix (max_nodes + 1)
    int32_t aln_cap;       // traceback buffer capacity
    int32_t band_width;    // banded mode only
    int32_t want_consensus; // MSA kernels also emit the consensus when set
    int32_t spoa_accurate;  // per-read racon DFS sort instead of Kahn (SPOA_ACCURATE builds)
    // LDS-resident kernel (full alignment, 16-bit scores): layout of the
    // per-workgroup LDS image and of the per-window HBM side buffers
    int32_t lds_kernel;     // 1: launch the LDS-resident kernel
    int32_t lds_bytes;      // dynamic LDS per workgroup
    int32_t lds_ring_off;   // E-domain score rows ring (int16)
    int32_t lds_ring_rows;  // power of two
    int32_t lds_sh_off;     // small shared region (layout: kSh* below)
    int32_t lds_rec_off;    // per-row program (u32 per row)
    int32_t lds_xl_off;     // predecessor lists (u16)
    int32_t lds_xl_cap;
    int32_t lds_cpl;        // forward pass: columns per lane
    int32_t lds_waves;      // forward pass: waves per window
    int32_t code_stride;    // bytes per traceback-code row
    int64_t aux_stride;     // bytes per window of the HBM side buffer:
    int32_t aux_carry_off;  //   codes [score_rows x code_stride] | per-row span carries (int16)
    // banded kernel (lds_kernel == 3): LDS work region size; the HBM side
    // buffer holds codes [score_rows x band_width] | row records a, b (u32) |
    // column-0 values (i32) | row flags (u8) | predecessor lists (i32)
    int32_t lds_work_bytes;
    int32_t aux_reca_off;
    int32_t aux_recb_off;
    int32_t aux_col0_off;
    int32_t aux_flag_off;
    int32_t aux_xl_off;
    int32_t aux_xl_cap;
    int32_t aux_bx_off;     //   | per-256-row-block predecessor-list offsets (i32)
    int32_t aux_recc_off;   //   | row records c (u32)
    int32_t aux_rece_off;   //   | row records e (u32)
    int32_t band_ad;        // banded kernel: waves of the anti-diagonal forward pass (0: row-parallel pass)
    int32_t tb_rank;        // traceback move windows (TbWin): bit 0 pointer-doubling walk, bit 1 strips, bit 2 32 x 4 strips
    int32_t diag;           // diagnostic switches (GWAMD_DIAG=1 only): bit 0 Kahn sort queued words in a ring,
                            // bit 1 LDS kernel on the round-3 forward pass, bit 2 FIFO Kahn sort,
                            // bit 3 round-5 racon DFS step for the MSA
};

// LDS bytes of the pointer-doubling traceback walk (walk_window_ranked)
constexpr int kTbRankBytes = 7 * 144 + 128 * 4;

// Small shared region of the LDS kernel (kShBytes(waves) at Dims::lds_sh_off):
// control ints, per-wave channel progress, the end-row slot, the per-span
// boundary column ([waves][ring rows] int16) and the span-to-span carry
// channels ([waves-1][kChanRows] tagged words).
constexpr int kShProg    = 16;
constexpr int kShEnd     = 32;
constexpr int kShBnd     = 64;
constexpr int kShChan    = 128;
constexpr int kChanRows  = 64;
constexpr int kMaxWaves  = 4;
constexpr int kShBytes(int waves) { return kShChan + (waves - 1) * kChanRows * 4; }
// ... of the 32-bit pass (nw_forward_lds_w): end row, progress words (one per
// wave, up to 8), the carries of the ring rows per wave, then the channels
// ([waves-1][kChanRows] 64-bit words: row | carry << 32)
constexpr int kShEndW   = 32;
constexpr int kShProgW  = 64;
constexpr int kShBndW   = 128; // [8 waves][8 ring rows] int32
constexpr int kShChanW  = 384;
constexpr int kMaxRingW = 8;
constexpr int kShBytesW(int waves) { return kShChanW + (waves - 1) * kChanRows * 8; }

constexpr int kTileRows = 128; // traceback tile (codes) rows
constexpr int kTileCols = 128; // traceback tile columns (bytes)
constexpr int kTileXlMin = 512; // predecessor-list entries staged with a tile (at least)

// Device pointers of one batch (all batch-wide; per-window slots are derived
// in-kernel).  SizeT-typed arrays are passed as void* and cast in the kernel.
struct Buffers
{
    // input
    const uint8_t* seqs;
    const int8_t* wts;
    const int32_t* seq_len;
    const int64_t* seq_off;
    const WindowDesc* windows;
    const int32_t* order; // window of each queue position (nullptr: position i is window i)
    int32_t num_windows;
    // Persistent grid (LDS and banded kernels): workgroup i first runs queue
    // position i, then dequeues num_slots + atomicAdd(head, 1) until the queue
    // is empty.  head == nullptr: one window per workgroup.  The per-window
    // scratch of the forward pass and traceback (spill rows, codes, row
    // records, alignment path, consensus scores) is indexed by workgroup
    // ("slot"), the graph and the outputs by window.
    int32_t* head;
    int32_t num_slots;
    // graph scratch
    uint8_t* base;
    uint16_t* in_cnt;
    uint16_t* out_cnt;
    uint16_t* aln_cnt;
    uint16_t* node_cov;
    uint16_t* in_w;
    void* in_e;
    void* out_e;
    void* aln;
    void* sorted;
    void* pos;
    void* ag;
    void* ar;
    void* scores;       // v1: score matrix; LDS kernel: E-domain spill rows
    uint8_t* codes;     // LDS kernel: traceback codes, one byte per cell
    // consensus / topsort / msa scratch
    int32_t* cscore;
    void* cpred;
    uint16_t* edge_cov;     // msa: read ids per outgoing edge
    uint16_t* edge_cov_cnt; // msa
    void* seq_begin;        // msa
    // outputs
    uint8_t* cons;      // max_consensus per window; consensus in host order
    uint16_t* cov;      // max_consensus per window
    int32_t* cons_len;  // per window
    uint8_t* status;    // per window, consensus output
    uint8_t* msa_status; // per window, MSA output
    uint8_t* msa;       // max_seqs * max_consensus per window
    int32_t* msa_len;   // per window
    int32_t* final_nodes;
    int64_t* cells;     // per window: sum over reads of (|V|+1)*(|r|+1) (or band cells)
    int64_t* phase;     // per window kPhases counters of s_memrealtime ticks (100 MHz)
};

// Phase counters written per window (diagnostics, bench.py "phases").
enum Phase
{
    kPhBackbone = 0,
    kPhForward,
    kPhTraceback,
    kPhAdd,
    kPhTopsort,
    kPhOutput,
    kPhRowProg, // read staging + row program (LDS kernel)
    kPhTotal,
    kPhases
};

struct Scores
{
    int32_t gap, mismatch, match;
};

} // namespace poa
} // namespace gwamd

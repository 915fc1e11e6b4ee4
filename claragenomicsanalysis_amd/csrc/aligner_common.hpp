// Shared host/device definitions for the MI355X global aligner
// (cudaaligner: AlignerGlobalHirschbergMyers, AlignerGlobalMyers).
//
// Batch layout (same packing as the reference, aligner_global.cpp:33-116):
// pair i's query at seqs + 2*i*stride, its target at seqs + (2*i+1)*stride;
// lengths[2i], lengths[2i+1]; path i (int8 AlignmentState, emitted end ->
// start, reversed on the host) at paths + i*max_path_length; path_len[i].
#pragma once

#include <cstdint>

namespace gwamd
{
namespace aln
{

constexpr int kWave       = 64;
constexpr int kWordBits   = 32;  // Myers word (hirschbergmyers::WordType, uint32_t)
constexpr int kStackSize  = 64;  // hirschberg_myers_stackbuffer_size (aligner_global_hirschberg_myers.cpp:29)
constexpr int kFullMyers  = 63;  // hirschberg_myers_switch_to_myers_size (:30)
constexpr int kMaxChunks  = 4;   // Myers block = 64 lanes x 32 bits; up to 4 blocks per sweep
constexpr int kLeafCols   = 128; // base-case columns kept in LDS (larger leaves use HBM)
constexpr int kSplitLds   = 512; // split segments up to this many columns keep their scores in LDS
constexpr int kLeafColBytes = 20; // per column: pv u64, mv u64, score i32
constexpr int kChunkWords  = 32;  // banded Myers: one reference warp of 32 words per step (myers_gpu.cu:35)
constexpr int kUkChunks    = 8;   // Ukkonen: band rows k held 64 per chunk, up to 512 (one wave)
constexpr int kUkWideChunks = 4;  // wider bands: rows per thread of a workgroup of up to 1,024 (4,096 rows)
constexpr int kUkTileRows  = 64;  //   backtrace tile: band rows x
constexpr int kUkTileCols  = 128; //   anti-diagonal columns (int16, 16 KiB)
constexpr int kUkkonenP    = 100; // aligner_global_ukkonen.cpp:29
constexpr int32_t kSpecUnknown = -2147483647 - 1; // spec_ed: sweep not run ahead
constexpr int16_t kUkMax   = 32766; // numeric_limits<int16_t>::max() - 1 (ukkonen_gpu.cu:75)

// AlignmentState (cudaaligner.hpp:46-52)
enum State : int8_t
{
    kMatch     = 0,
    kMismatch  = 1,
    kInsertion = 2,
    kDeletion  = 3,
};

struct Args
{
    const char* seqs;
    const int32_t* lens;
    int32_t stride;          // max(max_query_length, max_target_length)
    int8_t* paths;
    int32_t* path_len;
    int32_t max_path_length; // ceil4(maxQ + maxT) (aligner_global.cpp:32-37)
    int32_t n;
    int32_t max_query_length;
    int64_t max_matrix_elems; // ceil(maxQ/4) * 64: the reference's pv/mv matrix capacity
    // global workspace, one slot per resident workgroup
    uint8_t* ws;
    int64_t ws_slot_bytes;
    int64_t ws_front_off;    // Hirschberg-Myers: frontier of the breadth-first recursion in the slot
    int32_t front_cap;       //   entries per frontier buffer (two buffers, then one u16 split column each)
    int64_t ws_leaf_off;     //   per-lane base cases: columns (pv, mv, score) then paths
    int32_t leaf_cols;       //   column capacity (target + one per segment)
    int64_t ws_split_off;    //   split scores of segments too wide for LDS (forward, reverse)
    int64_t ws_pat_off;      //   long mode: query patterns
    int64_t ws_hbuf_off;     //   long mode: striped sweeps' per-column hand-over deltas
    int64_t ws_tcod_off;     //   long mode: target letter codes when they do not fit LDS (-1: in LDS)
    int32_t long_mode;       // queries / targets past the LDS-resident limits (see aligner_batch.cpp)
    int32_t stripe_blocks;   // long mode: 64-word blocks per stripe of a tall sweep (kMaxChunks)
    // LDS layout (bytes)
    int32_t lds_target_off;
    int32_t lds_pat_off;     // [pat_words][8] u32: forward A C T G, reverse A C T G
    int32_t lds_scratch_off;
    int32_t lds_stack_off;
    int32_t lds_bytes;
    int32_t pat_words;       // ceil(max_query_length / 32)
    int32_t scratch_bytes;
    // banded aligners (aligner_banded.hip)
    int32_t lds_seq2_off;    // Ukkonen: the longer sequence
    int32_t lds_tile_off;    // backtrace staging tile
    int32_t tile_bytes;
    int32_t ukkonen_p;       // AlignerGlobalUkkonen::ukkonen_p_ (aligner_global_ukkonen.cpp:29)
    int32_t uk_threads;      // Ukkonen: > 0 runs ukkonen_wide_kernel with this many threads per pair
    int32_t lds_edge_off;    //   its 64-row-group edge values (2 x 2 x kUkWideChunks*16 int)
    int32_t band_waves;      // banded Myers: waves per pair (1, 4, 8 or 16; myers_banded_kernel<NWV>)
    // banded Myers band doubling run ahead (few long pairs): launch 1
    // (spec_phase 1) runs sweeps 0..spec_sweeps-1 of every pair on their own
    // workgroups (distance only; the last one also stores its band matrix in
    // the pair's slot) into spec_ed[pair * spec_sweeps + k]; launch 2
    // (spec_phase 2) skips the sweeps those distances reject and the stored
    // last one; spec_phase 0: the plain loop
    int32_t spec_phase;
    int32_t spec_sweeps;
    int32_t* spec_ed;
    // path counters, accumulated over the aligner's launches (gwamd_aligner_get_stats):
    // [0] banded Myers sweeps whose chunk state went through HBM, [1] pairs
    // aligned by ukkonen_wide_kernel, [2] the most band rows one thread of
    // ukkonen_wide_kernel held (64-bit: long-lived aligners do not wrap)
    unsigned long long* stats;
};

} // namespace aln
} // namespace gwamd

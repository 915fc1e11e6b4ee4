// MI355X (gfx950) banded POA kernel: one window per 64-lane workgroup.
//
// Banded mode of the reference (cudapoa_nw_banded.cuh:28-487, driven by
// generatePOAKernel, cudapoa_kernels.cuh:66-359) with the reference's flat
// band layout reproduced value for value ("banded kernel"):
//
//   * a row of the band holds F(r, idx), idx 0 .. bw+7, for columns
//     band_start(r) + idx; idx 0 is the column-0 value when band_start is 0,
//     else min_score_value; idx bw+1 .. bw+7 are min_score_value (row 0:
//     idx*gap); get_score() reads minv beyond idx bw (:107-121) while the DP's
//     get_scores() reads the padding (:123-173) -- both are kept apart;
//   * the per-read row program (base, predecessor distances, band start,
//     sink/spill flags) is built lane-parallel into HBM and streamed into
//     registers 64 rows at a time;
//   * each lane owns CPL = bw/64 consecutive band cells; predecessor r-1 comes
//     from registers (DPP wave shifts for band shifts of 0 or one lane),
//     others from a 16-row LDS ring or, when farther back, from HBM spill
//     rows; the horizontal closure is an exact max-prefix in the E domain;
//   * instead of the score matrix, one traceback code per cell is written
//     (direction + first matching predecessor slot, the reference's tie order
//     with get_score() semantics); the traceback walks codes from 64-row LDS
//     tiles.  Cells outside the band (only reached through layout corner
//     cases) are evaluated exactly from spill rows: every row holding a value
//     that an out-of-band comparison could match is spilled;
//   * addAlignmentToGraph and the Kahn sort reuse the wave-parallel LDS
//     versions (poa_wave.hpp) with the sequential restatements as fallback.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "poa_wave.hpp"

namespace gwamd
{
namespace poa
{

#ifndef GWAMD_BAND_ADD_AU
#define GWAMD_BAND_ADD_AU 4
#endif
// read positions per lane and pass of the add (one wave per SIMD: registers to spare)
constexpr int kBandAddAU = GWAMD_BAND_ADD_AU;
constexpr uint32_t kNpEsc = 63;

// rec_a: base (8) | np (6; 63 = escape: read the graph) | sink (1) | spill (1) | band_start/4 (16)
// rec_b: bit 31 clear: distance to pred 0 | distance to pred 1 << 16 (both < 32768);
//        bit 31 set: offset of the row's predecessor list in xl (np >= 5 or far predecessors)
// rec_c: distance to pred 2 | distance to pred 3 << 16 (np 3-4, inline)
__device__ __forceinline__ int ra_base(uint32_t a) { return int(a & 0xffu); }
__device__ __forceinline__ int ra_np(uint32_t a) { return int((a >> 8) & 63u); }
__device__ __forceinline__ bool ra_sink(uint32_t a) { return (a >> 14) & 1u; }
__device__ __forceinline__ bool ra_spill(uint32_t a) { return (a >> 15) & 1u; }
__device__ __forceinline__ int ra_bs(uint32_t a) { return int(a >> 16) << 2; }

// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt and lgkmcnt left at their maxima)
__device__ __forceinline__ void vm_drain()
{
    __builtin_amdgcn_s_waitcnt(0x0F70);
}

// Inclusive max-scan over the wave on sign-flipped values (x ^ 0x80000000
// orders like x and 0 is the identity), so every step is one v_max_u32 with a
// DPP source (row_shr 1/2/4/8, row_bcast 15/31; missing sources read 0).
__device__ __forceinline__ uint32_t wave_incl_maxu_dpp(uint32_t v)
{
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x111, 0xf, 0xf, true)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x112, 0xf, 0xf, true)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x114, 0xf, 0xf, true)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x118, 0xf, 0xf, true)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x142, 0xa, 0xf, false)));
    v = max(v, uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x143, 0xc, 0xf, false)));
    return v;
}

template <typename ScoreT>
__device__ __forceinline__ int trunc_score(int v)
{
    return int(ScoreT(v));
}

struct BandAux
{
    uint8_t* codes;  // [score_rows][bw]
    uint32_t* reca;  // [score_rows]
    uint32_t* recb;  // [score_rows]
    uint32_t* recc;  // [score_rows] distances to predecessors 2 and 3 (rows with 3-4 inline predecessors)
    uint32_t* rece;  // [score_rows] band shifts / 4 of inline predecessors 0-3 (bytes; clamped to 255)
    int32_t* col0;   // [score_rows] F(r, 0) of rows with band_start 0
    uint8_t* flags;  // [score_rows] bit 0: row stored in the spill rows
    int32_t* xl;     // [xl_cap] predecessor rows of rows with np >= 3 (or far)
    int32_t* bx;     // [score_rows / 256 + 2] xl offset of the first listed row of each 256-row block
    int xl_cap;
};

// Diagnostic counters (-DGWAMD_BAND_PROFILE builds only; stored over the
// phase slots, see the kernel epilogue).
struct BandProf
{
    uint64_t v[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#ifdef GWAMD_BAND_PROFILE
    __device__ void add(int i, uint64_t x) { v[i] += x; }
    __device__ static uint64_t now() { return __builtin_amdgcn_s_memtime(); }
#else
    __device__ void add(int, uint64_t) {}
    __device__ static uint64_t now() { return 0; }
#endif
};
enum
{
    kBpRows = 0,     // forward rows
    kBpMulti,        // forward rows with two or more predecessors
    kBpStageCyc,     // forward cycles spent staging blocks
    kBpFwdCyc,       // forward cycles
    kBpSteps,        // traceback steps
    kBpTileCyc,      // traceback cycles spent staging tiles
    kBpTbCyc,        // traceback cycles
    kBpFlushCyc,     // traceback cycles in path flushes
    kBpRefill,       // traceback move-window refills
    kBpSlow,         // traceback steps through the general (non-window) step
    kBpAddSeq,       // reads added by the sequential add (parallel add declined)
    kBpAdBlocks,     // anti-diagonal pass: row blocks
    kBpAdSetup,      // anti-diagonal pass: cycles in block setup (records, slots, dispatch)
    kBpAdLoop,       // anti-diagonal pass: cycles in the step loops
    kBpAdSteps,      // anti-diagonal pass: steps
};

__device__ __forceinline__ BandAux as_global(BandAux X)
{
    X.codes = glb(X.codes);
    X.reca  = glb(X.reca);
    X.recb  = glb(X.recb);
    X.recc  = glb(X.recc);
    X.rece  = glb(X.rece);
    X.col0  = glb(X.col0);
    X.flags = glb(X.flags);
    X.xl    = glb(X.xl);
    X.bx    = glb(X.bx);
    return X;
}

constexpr int kStageRows = 256;  // forward pass: row records staged in LDS per block
constexpr int kStageXl   = 1024; // predecessor-list entries staged per block

// k-th predecessor row of row r (0 = the virtual row 0) and the predecessor count
template <typename SizeT>
__device__ __forceinline__ int band_pred2(WinGraph<SizeT> g, BandAux X, int r, uint32_t a, uint32_t b,
                                          uint32_t c, int k)
{
    X = as_global(X);
    g = as_global(g);
    const int np = ra_np(a);
    if (np == 0)
        return 0;
    if (np == int(kNpEsc))
        return pred_row(g, int(g.sorted[r - 1]), k);
    if (b >> 31)
        return int(X.xl[(b & 0x7fffffffu) + uint32_t(k)]);
    const uint32_t w = k < 2 ? b : c;
    return r - int((k & 1) ? (w >> 16) : (w & 0xffffu));
}

// The aux arrays with global-typed pointers (see WinGraphG).
struct BandAuxG
{
    GWAMD_GLB uint8_t* codes;
    GWAMD_GLB const uint32_t* reca;
    GWAMD_GLB const uint32_t* recb;
    GWAMD_GLB const uint32_t* recc;
    GWAMD_GLB int32_t* col0;
    GWAMD_GLB uint8_t* flags;
    GWAMD_GLB const int32_t* xl;
};

__device__ __forceinline__ BandAuxG typed_aux(const BandAux& X)
{
    BandAuxG t;
    t.codes = (GWAMD_GLB uint8_t*)(X.codes);
    t.reca  = (GWAMD_GLB const uint32_t*)(X.reca);
    t.recb  = (GWAMD_GLB const uint32_t*)(X.recb);
    t.recc  = (GWAMD_GLB const uint32_t*)(X.recc);
    t.col0  = (GWAMD_GLB int32_t*)(X.col0);
    t.flags = (GWAMD_GLB uint8_t*)(X.flags);
    t.xl    = (GWAMD_GLB const int32_t*)(X.xl);
    return t;
}

template <typename SizeT>
__device__ __forceinline__ int band_pred2(const WinGraphG<SizeT>& g, const BandAuxG& X, int r, uint32_t a, uint32_t b,
                                          uint32_t c, int k)
{
    const int np = ra_np(a);
    if (np == 0)
        return 0;
    if (np == int(kNpEsc))
        return pred_row(g, int(g.sorted[r - 1]), k);
    if (b >> 31)
        return int(X.xl[(b & 0x7fffffffu) + uint32_t(k)]);
    const uint32_t w = k < 2 ? b : c;
    return r - int((k & 1) ? (w >> 16) : (w & 0xffffu));
}

template <typename SizeT>
__device__ __forceinline__ int band_np2(const WinGraphG<SizeT>& g, int r, uint32_t a, uint32_t b)
{
    const int np = ra_np(a);
    return np == int(kNpEsc) ? int(g.in_cnt[int(g.sorted[r - 1])]) : np;
}

template <typename SizeT>
__device__ __forceinline__ int band_np2(WinGraph<SizeT> g, int r, uint32_t a, uint32_t b)
{
    g = as_global(g);
    const int np = ra_np(a);
    return np == int(kNpEsc) ? int(g.in_cnt[int(g.sorted[r - 1])]) : np;
}

// Row program of rows 1..V (after every topological sort).  Loads are batched
// kRP rows per lane for memory-level parallelism; spill flags (a successor
// reads the row from spill_dist or more rows later) are collected as LDS bytes
// from the successor's side and folded into rec_a in a second pass; far flags
// (a successor far_dist or more rows later: the anti-diagonal pass reads the
// row from HBM) become bit 1 of X.flags.
template <typename SizeT>
__device__ __forceinline__ int band_row_program(WinGraph<SizeT> g, int V, const Band& B, BandAux X, int lane,
                                 GWAMD_LDS uint8_t* flags, int spill_dist, int far_dist)
{
    X = as_global(X);
    g = as_global(g);
    constexpr int kRP = 4;
    GWAMD_LDS uint8_t* far = flags + ((V + 2 + 15) & ~15);
    for (int r = lane; r <= V + 1; r += kWave)
        flags[r] = 0, far[r] = 0;
    wave_sync();
    auto mark = [&](int p, int dist) {
        if (dist >= spill_dist)
            flags[p] = 1;
        if (dist >= far_dist)
            far[p] = 1;
    };
    int xbase = 0;
    int npmax = 0; // largest predecessor count (returned, wave-uniform)
    static_assert(kRP * kWave == kStageRows, "one row-program pass per staged block");
    for (int r0 = 1; r0 <= V; r0 += kRP * kWave)
    {
        if (lane == 0)
            X.bx[(r0 - 1) / kStageRows] = xbase;
        int node[kRP], np[kRP], base[kRP], oc[kRP], e0[kRP], e1[kRP], p0[kRP], p1[kRP];
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            const int r = min(r0 + u * kWave + lane, V);
            node[u]     = int(g.sorted[r - 1]);
        }
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            np[u]   = int(g.in_cnt[node[u]]);
            base[u] = int(g.base[node[u]]);
            oc[u]   = int(g.out_cnt[node[u]]);
            e0[u]   = int(g.in_e[node[u] * kMaxEdges]);
            e1[u]   = int(g.in_e[node[u] * kMaxEdges + 1]);
        }
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            p0[u] = int(g.pos[np[u] >= 1 ? e0[u] : 0]) + 1;
            p1[u] = int(g.pos[np[u] >= 2 ? e1[u] : 0]) + 1;
        }
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            const int r      = r0 + u * kWave + lane;
            const bool valid = r <= V;
            const int n      = valid ? np[u] : 0;
            npmax            = max(npmax, n);
            int p2 = 0, p3 = 0;
            if (n >= 3 && n <= 4)
            {
                p2 = pred_row(g, node[u], 2);
                p3 = n == 4 ? pred_row(g, node[u], 3) : r;
            }
            bool near2 = n <= 4 && (n < 1 || r - p0[u] < 32768) && (n < 2 || r - p1[u] < 32768) &&
                         (n < 3 || (r - p2 < 32768 && r - p3 < 32768));
            if (B.bw > 1016 && near2 && valid)
            {
                // rec_e holds band shifts / 4 clamped to 255, which stands for
                // "cuts every group" only while bw + 4 <= 1,020: rows of wider
                // bands with a shift that large list their predecessors instead
                const int bsr = B.start(r);
                auto big      = [&](int pk) { return bsr - (pk == 0 ? 0 : B.start(pk)) >= 1020; };
                if ((n == 0 && big(0)) || (n >= 1 && big(p0[u])) || (n >= 2 && big(p1[u])) ||
                    (n >= 3 && big(p2)) || (n >= 4 && big(p3)))
                    near2 = false;
            }
            const int listed = near2 ? 0 : n;
            int total        = 0;
            const int excl   = wave_excl_sum(listed, lane, total);
            if (valid)
            {
                uint32_t a = uint32_t(base[u]) | (uint32_t(oc[u] == 0 ? 1 : 0) << 14) |
                             (uint32_t(B.start(r) >> 2) << 16);
                uint32_t bw = 0;
                if (near2)
                {
                    a |= uint32_t(n) << 8;
                    if (n >= 1)
                    {
                        bw = uint32_t(r - p0[u]);
                        mark(p0[u], r - p0[u]);
                    }
                    if (n >= 2)
                    {
                        bw |= uint32_t(r - p1[u]) << 16;
                        mark(p1[u], r - p1[u]);
                    }
                    if (n >= 3)
                    {
                        X.recc[r] = uint32_t(r - p2) | (uint32_t(r - p3) << 16);
                        mark(p2, r - p2);
                        if (n == 4)
                            mark(p3, r - p3);
                    }
                }
                else
                {
                    const int off  = xbase + excl;
                    const bool fit = off + n <= X.xl_cap;
                    for (int k = 0; k < n; k++)
                    {
                        const int pk = k == 0 ? p0[u] : (k == 1 ? p1[u] : pred_row(g, node[u], k));
                        if (fit)
                            X.xl[off + k] = pk;
                        mark(pk, r - pk);
                    }
                    a |= (fit ? uint32_t(n) : kNpEsc) << 8;
                    bw = 0x80000000u | uint32_t(off);
                }
                if (near2)
                {
                    // band shifts of the inline predecessors (/4, clamped: >= bw+4 cuts every group)
                    const int bsr = B.start(r);
                    auto sh4      = [&](int pk) { return uint32_t(min((bsr - (pk == 0 ? 0 : B.start(pk))) >> 2, 255)); };
                    uint32_t ew   = n == 0 ? sh4(0) : 0u;
                    if (n >= 1)
                        ew |= sh4(p0[u]);
                    if (n >= 2)
                        ew |= sh4(p1[u]) << 8;
                    if (n >= 3)
                        ew |= sh4(p2) << 16;
                    if (n >= 4)
                        ew |= sh4(p3) << 24;
                    X.rece[r] = ew;
                }
                X.reca[r]  = a;
                X.recb[r]  = bw;
            }
            xbase += total;
        }
    }
    if (lane == 0)
        X.bx[(V + kStageRows - 1) / kStageRows] = xbase;
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    // X.flags bit 0 is set by the forward pass for the rows it spills
    for (int r = lane + 1; r <= V; r += kWave)
    {
        if (flags[r])
            X.reca[r] |= 1u << 15;
        X.flags[r] = far[r] ? 2 : 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return uniform(wave_max(npmax));
}

// Predecessor values F(p, d + CPL*lane + c), c = 0..CPL (flat get_scores()
// reads, :123-173).  Lanes whose groups are cut read clamped garbage.
typedef int v4i_t __attribute__((ext_vector_type(4)));
typedef int v2i_t __attribute__((ext_vector_type(2)));

// q points at an aligned group of CPL cells; F[0] is the element before it
#define GWAMD_BAND_LOAD_ROW(NAME, AS)                                                                        \
    template <typename ScoreT, int CPL>                                                                      \
    __device__ __forceinline__ void NAME(AS const ScoreT* q, int(&F)[CPL + 1])                               \
    {                                                                                                        \
        F[0] = int(q[-1]);                                                                                   \
        if constexpr (sizeof(ScoreT) == 4 && CPL == 4)                                                       \
        {                                                                                                    \
            const v4i_t v = *reinterpret_cast<AS const v4i_t*>(q);                                          \
            F[1] = v.x, F[2] = v.y, F[3] = v.z, F[4] = v.w;                                         \
        }                                                                                                    \
        else if constexpr (sizeof(ScoreT) == 2 && CPL == 4)                                                  \
        {                                                                                                    \
            const v2i_t v = *reinterpret_cast<AS const v2i_t*>(q);                                          \
            F[1] = int(int16_t(v.x & 0xffff)), F[2] = v.x >> 16;                                             \
            F[3] = int(int16_t(v.y & 0xffff)), F[4] = v.y >> 16;                             \
        }                                                                                                    \
        else                                                                                                 \
        {                                                                                                    \
            _Pragma("unroll") for (int c = 0; c < CPL; c++) F[c + 1] = int(q[c]);                            \
        }                                                                                                    \
    }
GWAMD_BAND_LOAD_ROW(band_load_lds, GWAMD_LDS)
GWAMD_BAND_LOAD_ROW(band_load_glb, )
#undef GWAMD_BAND_LOAD_ROW

template <typename ScoreT, int CPL>
__device__ __forceinline__ void band_fetch(int p, int d, int r, const int (&Hp)[CPL], int prevF0,
                                           GWAMD_LDS ScoreT* ring, const ScoreT* spill, int rowsz, int gap, int minv,
                                           int lane, int (&F)[CPL + 1])
{
    constexpr int kBandRing = band_ring_rows(CPL);
    if (p == 0)
    {
#pragma unroll
        for (int c = 0; c <= CPL; c++)
            F[c] = (d + CPL * lane + c) * gap;
        return;
    }
    if (p == r - 1 && d == 0)
    {
        F[0] = __builtin_amdgcn_update_dpp(prevF0, Hp[CPL - 1], 0x138, 0xf, 0xf, false); // wave_shr:1
#pragma unroll
        for (int c = 1; c <= CPL; c++)
            F[c] = Hp[c - 1];
        return;
    }
    if (p == r - 1 && d == CPL)
    {
        F[0] = Hp[CPL - 1];
#pragma unroll
        for (int c = 1; c <= CPL; c++)
            F[c] = __builtin_amdgcn_update_dpp(minv, Hp[c - 1], 0x130, 0xf, 0xf, false); // wave_shl:1
        return;
    }
    if (CPL > 4 && (d % CPL) != 0)
    {
        // band shift not a multiple of the lane's CPL cells (CPL 8: shifts are
        // multiples of 4): element-wise loads from position d + CPL*(lane+1) - 1
        const int pos = min(d + CPL * (lane + 1), rowsz - CPL);
        if (r - p < kBandRing)
        {
            const GWAMD_LDS ScoreT* q = ring + (p & (kBandRing - 1)) * rowsz + pos;
#pragma unroll
            for (int c = 0; c <= CPL; c++)
                F[c] = int(q[c - 1]);
        }
        else
        {
            const ScoreT* q = spill + size_t(p) * rowsz + pos;
#pragma unroll
            for (int c = 0; c <= CPL; c++)
                F[c] = int(q[c - 1]);
            vm_drain();
        }
        return;
    }
    const int gmax = rowsz / CPL - 1;
    const int gi   = min(d / CPL + lane + 1, gmax);
    if (r - p < kBandRing)
        band_load_lds<ScoreT, CPL>(ring + (p & (kBandRing - 1)) * rowsz + gi * CPL, F);
    else
    {
        band_load_glb<ScoreT, CPL>(spill + size_t(p) * rowsz + gi * CPL, F);
        vm_drain(); // rare path: keep its loads from forcing waits where the paths join
    }
}

// Forward pass over rows 1..V.  Returns the end row (first sink with the
// strictly greatest get_score(row, L), :349-365).
//
// Rows with at most one predecessor that is not listed (the common case) take
// a straight path: one predecessor fetch, the closure and the codes without
// predecessor loops.  Row records and read bytes are software-pipelined: the
// record of row r+2 and the read bytes of row r+1 are requested while row r is
// computed.
// Band widths 128 / 256 / 512 (CPL 2, 4, 8) keep their read bytes in one
// integer; the wider classes (CPL 6, 10, 12, 14, 16: band widths 384 - 1,024,
// any multiple of 128 the reference accepts, batch.hpp:85-94) in CPL/2
// 16-bit pieces (band starts are multiples of 4, CPL*lane is even).
template <int CPL>
struct ReadPieces
{
    uint32_t h[CPL / 2];
};
template <int CPL>
using ReadBytesT = typename std::conditional<
    (CPL == 2 || CPL == 4), uint32_t,
    typename std::conditional<(CPL == 8), uint64_t, ReadPieces<CPL>>::type>::type;

template <typename ScoreT, int CPL>
__device__ __forceinline__ ReadBytesT<CPL> band_read_bytes(GWAMD_LDS const uint8_t* read, int bs, int lane)
{
    if constexpr (CPL == 8)
    {
        // band starts are multiples of 4: two aligned 4-byte reads
        const GWAMD_LDS uint32_t* p = reinterpret_cast<GWAMD_LDS const uint32_t*>(read + bs + 8 * lane);
        return uint64_t(p[0]) | (uint64_t(p[1]) << 32);
    }
    else if constexpr (CPL == 4)
        return *reinterpret_cast<GWAMD_LDS const uint32_t*>(read + bs + 4 * lane);
    else if constexpr (CPL == 2)
        return uint32_t(*reinterpret_cast<GWAMD_LDS const uint16_t*>(read + bs + 2 * lane));
    else
    {
        ReadPieces<CPL> r;
        const GWAMD_LDS uint16_t* p = reinterpret_cast<GWAMD_LDS const uint16_t*>(read + bs + CPL * lane);
#pragma unroll
        for (int k = 0; k < CPL / 2; k++)
            r.h[k] = p[k];
        return r;
    }
}

// read byte c of a lane's CPL bytes
template <int CPL>
__device__ __forceinline__ int band_read_byte(const ReadBytesT<CPL>& rb, int c)
{
    if constexpr (CPL == 2 || CPL == 4 || CPL == 8)
        return int((rb >> (8 * c)) & 0xffu);
    else
        return int((rb.h[c / 2] >> (8 * (c & 1))) & 0xffu);
}

// Out of line (round 6): with the level sort and the multi-wave graph update
// in the kernel, the inlined pass's register allocation cost B_banded's
// forward 52 -> 64 ms per window; its own function keeps its own allocation,
// as band_forward_ad's does
template <typename ScoreT, typename SizeT, int CPL>
__device__ __noinline__ int band_forward(WinGraph<SizeT> g, BandAux X, int V, GWAMD_LDS const uint8_t* read, int L,
                            const Band& B, const Scores sc, GWAMD_LDS ScoreT* ring, GWAMD_LDS uint32_t* stage,
                            ScoreT* spill, int rowsz, int lane, BandProf& bp)
{
    constexpr int kBandRing = band_ring_rows(CPL);
    X = as_global(X);
    g = as_global(g);
    const uint64_t f_t0 = BandProf::now();
    const int gap  = sc.gap;
    const int bw   = B.bw;
    const int minv = int(band_min_value<ScoreT>(sc));
    // an out-of-band traceback comparison matches only values minv - match,
    // minv - mismatch, minv - gap: rows holding a value <= the largest of them
    // are spilled so the slow path can read them
    const int Tmax = max(max(minv - sc.match, minv - sc.mismatch), minv - gap);
    // ring padding (idx bw+1 ..) is never overwritten by row stores
    for (int k = lane; k < kBandRing * rowsz; k += kWave)
        if (k % rowsz >= bw + CPL)
            ring[k] = ScoreT(minv);
    int egap[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++)
        egap[c] = (CPL * lane + c + 1) * gap;
    // row 0 as the "previous row" of row 1: F(0, idx) = idx * gap
    int Hp[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++)
        Hp[c] = (CPL * lane + c + 1) * gap;
    int prevF0 = 0;
    int bsv    = 0; // lane k < kBandRing: band start of the row in ring slot k
    int best = INT_MIN, end_row = 0;
    wave_sync();

    GWAMD_LDS uint32_t* srec = stage;
    GWAMD_LDS int32_t* sxl   = (GWAMD_LDS int32_t*)(stage + 4 * kStageRows);
    for (int r0 = 1; r0 <= V; r0 += kStageRows)
    {
        const int rend = min(V, r0 + kStageRows - 1);
        const uint64_t st0 = BandProf::now();
        // one wait per block: records and the block's predecessor lists
        uint32_t av[kStageRows / kWave], bv[kStageRows / kWave], cv[kStageRows / kWave],
            ev[kStageRows / kWave];
#pragma unroll
        for (int u = 0; u < kStageRows / kWave; u++)
        {
            const int rr = r0 + u * kWave + lane;
            av[u]        = rr <= V ? X.reca[rr] : 0u;
            bv[u]        = rr <= V ? X.recb[rr] : 0u;
            cv[u]        = rr <= V ? X.recc[rr] : 0u;
            ev[u]        = rr <= V ? X.rece[rr] : 0u;
        }
        const int xs  = uniform(X.bx[(r0 - 1) / kStageRows]);
        const int xe  = uniform(X.bx[(r0 - 1) / kStageRows + 1]);
        const int nxs = min(xe - xs, kStageXl);
        int xv[kStageXl / kWave];
#pragma unroll
        for (int u = 0; u < kStageXl / kWave; u++)
        {
            const int k = u * kWave + lane;
            xv[u]       = k < nxs ? X.xl[xs + k] : 0;
        }
#pragma unroll
        for (int u = 0; u < kStageRows / kWave; u++)
        {
            srec[4 * (u * kWave + lane)]     = av[u];
            srec[4 * (u * kWave + lane) + 1] = bv[u];
            srec[4 * (u * kWave + lane) + 2] = cv[u];
            srec[4 * (u * kWave + lane) + 3] = ev[u];
        }
#pragma unroll
        for (int u = 0; u < kStageXl / kWave; u++)
            sxl[u * kWave + lane] = xv[u];
        wave_sync();

        uint32_t a   = uint32_t(uniform(int(srec[0])));
        uint32_t b   = uint32_t(uniform(int(srec[1])));
        uint32_t c2  = uint32_t(uniform(int(srec[2])));
        uint32_t e2  = uint32_t(uniform(int(srec[3])));
        const int q1 = min(1, rend - r0);
        uint32_t a1  = uint32_t(uniform(int(srec[4 * q1])));
        uint32_t b1  = uint32_t(uniform(int(srec[4 * q1 + 1])));
        uint32_t c1  = uint32_t(uniform(int(srec[4 * q1 + 2])));
        uint32_t e1  = uint32_t(uniform(int(srec[4 * q1 + 3])));
        ReadBytesT<CPL> rbw = band_read_bytes<ScoreT, CPL>(read, ra_bs(a), lane);
        bp.add(kBpStageCyc, BandProf::now() - st0);
        bp.add(kBpRows, uint64_t(rend - r0 + 1));
        for (int r = r0; r <= rend; r++)
        {
            // prefetch: record of row r+2, read bytes of row r+1
            const int q2       = min(r + 2, rend) - r0;
            const uint32_t va2 = srec[4 * q2];
            const uint32_t vb2 = srec[4 * q2 + 1];
            const uint32_t vc2 = srec[4 * q2 + 2];
            const uint32_t ve2 = srec[4 * q2 + 3];
            const ReadBytesT<CPL> rbn = band_read_bytes<ScoreT, CPL>(read, ra_bs(a1), lane);

            const int bs = ra_bs(a);
            const int gb = ra_base(a);
            const int f  = ra_np(a);
            int sig[CPL];
#pragma unroll
            for (int c = 0; c < CPL; c++)
                sig[c] = (band_read_byte<CPL>(rbw, c) == gb) ? sc.match : sc.mismatch;

            int v[CPL];
            int carry;
            int H[CPL];
            int code[CPL];
            auto closure = [&]() {
                // E domain: E(t) = H(t) - (t+1)*gap, E(-1) = carry; the
                // prefix maximum runs on sign-flipped values
                constexpr uint32_t kFlip = 0x80000000u;
                uint32_t m[CPL];
                uint32_t run = lane == 0 ? (uint32_t(carry) ^ kFlip) : 0u;
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    run  = max(run, uint32_t(v[c] - egap[c]) ^ kFlip);
                    m[c] = run;
                }
                const uint32_t incl = wave_incl_maxu_dpp(run);
                const uint32_t excl = uint32_t(__builtin_amdgcn_update_dpp(0, int(incl), 0x138, 0xf, 0xf, true));
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    H[c] = trunc_score<ScoreT>(int(max(m[c], excl) ^ kFlip) + egap[c]);
            };
            auto horiz = [&](bool (&found)[CPL]) {
                int left = __builtin_amdgcn_update_dpp(carry, H[CPL - 1], 0x138, 0xf, 0xf, false);
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    if (!found[c] && left + gap == H[c])
                        code[c] = 2, found[c] = true;
                    left = H[c];
                }
            };

            // rows with 1..4 inline predecessors (distances in rec_b, rec_c) and
            // sources: predecessor values stay in registers, one pass each
            auto rowk = [&](auto npc) {
                constexpr int NP = decltype(npc)::value;
                int d[NP];
                int F[NP][CPL + 1];
#pragma unroll
                for (int k = 0; k < NP; k++)
                {
                    // distance (rec_b / rec_c) and band shift / 4 (rec_e, byte k)
                    const uint32_t w = k < 2 ? b : c2;
                    const int p      = f == 0 ? 0 : r - int((k & 1) ? (w >> 16) : (w & 0xffffu));
                    const int dk     = int((e2 >> (8 * k)) & 0xffu) << 2;
                    d[k]             = dk;
                    band_fetch<ScoreT, CPL>(p, dk, r, Hp, prevF0, ring, spill, rowsz, gap, minv, lane, F[k]);
                    // get_scores() reads the padding up to idx bw+7 (minv, except
                    // row 0) and cut groups read minv; get_score() sees minv
                    // beyond idx bw.  Rows >= 1 shifted by <= 4 need neither.
                    if (p == 0 || dk > 4)
                    {
                        int val[CPL];
#pragma unroll
                        for (int c = 0; c < CPL; c++)
                        {
                            const int t    = CPL * lane + c;
                            const bool cut = (t & ~3) + dk >= bw + 4;
                            const int vl   = trunc_score<ScoreT>(max(F[k][c] + sig[c], F[k][c + 1] + gap));
                            val[c]         = cut ? minv : vl;
                        }
#pragma unroll
                        for (int i = 0; i <= CPL; i++)
                            F[k][i] = (dk + CPL * lane + i > bw) ? minv : F[k][i];
                        // fold the cut values in through a sentinel pair: the
                        // value pass below recomputes from G, so keep val here
#pragma unroll
                        for (int c = 0; c < CPL; c++)
                            v[c] = k == 0 ? val[c] : max(v[c], val[c]);
                    }
                    else
                    {
#pragma unroll
                        for (int c = 0; c < CPL; c++)
                        {
                            const int vl = trunc_score<ScoreT>(max(F[k][c] + sig[c], F[k][c + 1] + gap));
                            v[c]         = k == 0 ? vl : max(v[c], vl);
                        }
                    }
                }
                // column 0 (:219-245): F(r, 0) is the column-0 value when the
                // band starts at 0, else the minv initialize_band writes at idx 0
                // (with band start 0 every shift is 0, so G(p, 0) = F(p, 0))
                carry = minv;
                if (bs == 0)
                {
                    int c0max = INT_MIN;
#pragma unroll
                    for (int k = 0; k < NP; k++)
                        c0max = max(c0max, __builtin_amdgcn_readlane(F[k][0], 0));
                    carry = f == 0 ? gap : trunc_score<ScoreT>(c0max + gap);
                }
                closure();
                // first diagonal slot, else first vertical slot (:367-477)
                bool found[CPL];
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    int dsl = -1, vsl = -1;
#pragma unroll
                    for (int k = NP - 1; k >= 0; k--)
                    {
                        dsl = (F[k][c] + sig[c] == H[c]) ? k : dsl;
                        vsl = (F[k][c + 1] + gap == H[c]) ? k : vsl;
                    }
                    code[c]  = dsl >= 0 ? (dsl << 2) : (vsl >= 0 ? ((vsl << 2) | 1) : 3);
                    found[c] = dsl >= 0 || vsl >= 0;
                }
                horiz(found);
            };
            const bool inl = f <= 4 && !(b >> 31);
            bp.add(kBpMulti, f >= 2 ? 1 : 0);
            if (inl && f <= 1)
                rowk(std::integral_constant<int, 1>{});
            else if (inl && f == 2)
                rowk(std::integral_constant<int, 2>{});
            else if (inl && f == 3)
                rowk(std::integral_constant<int, 3>{});
            else if (inl && f == 4)
                rowk(std::integral_constant<int, 4>{});
            else
            {
                const int np  = band_np2<SizeT>(g, r, a, b);
                const int npp = np == 0 ? 1 : np;
                // k-th predecessor row, predecessor lists from the staged block
                auto pred = [&](int k) -> int {
                    if (f == 0)
                        return 0;
                    if (f == int(kNpEsc))
                    {
                        const int pr = uniform(pred_row(g, int(g.sorted[r - 1]), k));
                        vm_drain();
                        return pr;
                    }
                    if (b >> 31)
                    {
                        const int rel = int(b & 0x7fffffffu) - xs + k;
                        if (rel < nxs)
                            return uniform(int(sxl[rel]));
                        const int pr = uniform(int(X.xl[int(b & 0x7fffffffu) + k]));
                        vm_drain();
                        return pr;
                    }
                    const uint32_t w = k < 2 ? b : c2;
                    return r - int((k & 1) ? (w >> 16) : (w & 0xffffu));
                };
                auto pbs = [&](int p) -> int {
                    return p == 0 ? 0
                                  : (r - p < kBandRing ? __builtin_amdgcn_readlane(bsv, p & (kBandRing - 1))
                                                       : B.start(p));
                };
                int F0[CPL + 1], F1[CPL + 1];
                int d0 = 0, d1 = 0;
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    v[c] = kNeg;
                int c0max = INT_MIN;
                for (int k = 0; k < npp; k++)
                {
                    const int p = pred(k);
                    const int d = bs - pbs(p);
                    int Fk[CPL + 1];
                    band_fetch<ScoreT, CPL>(p, d, r, Hp, prevF0, ring, spill, rowsz, gap, minv, lane, Fk);
#pragma unroll
                    for (int c = 0; c < CPL; c++)
                    {
                        const int t    = CPL * lane + c;
                        const bool cut = (t & ~3) + d >= bw + 4;
                        const int val  = cut ? minv : trunc_score<ScoreT>(max(Fk[c] + sig[c], Fk[c + 1] + gap));
                        v[c]           = max(v[c], val);
                    }
                    c0max = max(c0max, __builtin_amdgcn_readlane(Fk[0], 0));
                    if (k == 0)
                    {
#pragma unroll
                        for (int c = 0; c <= CPL; c++)
                            F0[c] = Fk[c];
                        d0 = d;
                    }
                    else if (k == 1)
                    {
#pragma unroll
                        for (int c = 0; c <= CPL; c++)
                            F1[c] = Fk[c];
                        d1 = d;
                    }
                }
                const int col0 = np == 0 ? gap : trunc_score<ScoreT>(c0max + gap);
                carry          = bs == 0 ? col0 : minv;
                closure();
                // codes (:367-477 with get_score(): minv beyond idx bw)
                bool found[CPL];
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    code[c] = 3, found[c] = false;
                for (int pass = 0; pass < 2; pass++)
                {
                    for (int k = 0; k < npp; k++)
                    {
                        int Fk[CPL + 1];
                        int d;
                        if (k == 0)
                        {
#pragma unroll
                            for (int c = 0; c <= CPL; c++)
                                Fk[c] = F0[c];
                            d = d0;
                        }
                        else if (k == 1)
                        {
#pragma unroll
                            for (int c = 0; c <= CPL; c++)
                                Fk[c] = F1[c];
                            d = d1;
                        }
                        else
                        {
                            const int p = pred(k);
                            d           = bs - pbs(p);
                            band_fetch<ScoreT, CPL>(p, d, r, Hp, prevF0, ring, spill, rowsz, gap, minv, lane, Fk);
                        }
#pragma unroll
                        for (int c = 0; c < CPL; c++)
                        {
                            const int t = CPL * lane + c;
                            if (pass == 0)
                            {
                                const int gA = (d + t > bw) ? minv : Fk[c];
                                if (!found[c] && gA + sig[c] == H[c])
                                    code[c] = k << 2, found[c] = true;
                            }
                            else
                            {
                                const int gB = (d + t + 1 > bw) ? minv : Fk[c + 1];
                                if (!found[c] && gB + gap == H[c])
                                    code[c] = (k << 2) | 1, found[c] = true;
                            }
                        }
                    }
                }
                horiz(found);
            }

            // store codes (one byte per cell)
            {
                uint8_t* crow = X.codes + size_t(r) * bw + CPL * lane;
                if constexpr (CPL == 8)
                {
                    uint64_t w8 = 0;
#pragma unroll
                    for (int c = 0; c < 8; c++)
                        w8 |= uint64_t(uint8_t(code[c % CPL])) << (8 * c);
                    *reinterpret_cast<uint64_t*>(crow) = w8;
                }
                else if constexpr (CPL == 4)
                {
                    const uint32_t w4 = uint32_t(code[0]) | (uint32_t(code[1]) << 8) | (uint32_t(code[2]) << 16) |
                                        (uint32_t(code[3]) << 24);
                    *reinterpret_cast<uint32_t*>(crow) = w4;
                }
                else if constexpr (CPL == 2)
                {
                    const uint16_t w2 = uint16_t(code[0] | (code[1 % CPL] << 8));
                    *reinterpret_cast<uint16_t*>(crow) = w2;
                }
                else if constexpr (CPL % 4 == 0)
                {
                    // CPL 12, 16: 4-byte aligned (bw and CPL*lane are multiples of 4)
#pragma unroll
                    for (int k = 0; k < CPL / 4; k++)
                        reinterpret_cast<uint32_t*>(crow)[k] =
                            uint32_t(code[4 * k]) | (uint32_t(code[4 * k + 1]) << 8) |
                            (uint32_t(code[4 * k + 2]) << 16) | (uint32_t(code[4 * k + 3]) << 24);
                }
                else
                {
                    // CPL 6, 10, 14: 2-byte aligned pieces
#pragma unroll
                    for (int k = 0; k < CPL / 2; k++)
                        reinterpret_cast<uint16_t*>(crow)[k] = uint16_t(code[2 * k] | (code[2 * k + 1] << 8));
                }
            }
            // end cell candidates (sinks in topological order, strict >)
            if (ra_sink(a))
            {
                int sval;
                if (L >= bs + 1 && L <= bs + bw)
                {
                    const int t = L - bs - 1;
                    int hv      = H[0];
#pragma unroll
                    for (int c = 1; c < CPL; c++)
                        hv = (t % CPL == c) ? H[c] : hv;
                    sval = __builtin_amdgcn_readlane(hv, t / CPL);
                }
                else if (L == bs)
                    sval = carry;
                else
                    sval = minv;
                if (best < sval)
                    best = sval, end_row = r;
            }
            // (columns past L included: spilling more rows only costs stores)
            int hmin = H[0];
#pragma unroll
            for (int c = 1; c < CPL; c++)
                hmin = min(hmin, H[c]);
            const bool tflag = __builtin_amdgcn_ballot_w64(hmin <= Tmax) != 0;
            // ring row: position idx + CPL - 1
            GWAMD_LDS ScoreT* rrow = ring + (r & (kBandRing - 1)) * rowsz;
            if constexpr (CPL == 4 && sizeof(ScoreT) == 4)
            {
                v4i_t q = {H[0], H[1 % CPL], H[2 % CPL], H[3 % CPL]};
                *reinterpret_cast<GWAMD_LDS v4i_t*>(rrow + CPL * (lane + 1)) = q;
            }
            else if constexpr (CPL == 4 && sizeof(ScoreT) == 2)
            {
                v2i_t q = {int((H[0] & 0xffff) | (H[1 % CPL] << 16)), int((H[2 % CPL] & 0xffff) | (H[3 % CPL] << 16))};
                *reinterpret_cast<GWAMD_LDS v2i_t*>(rrow + CPL * (lane + 1)) = q;
            }
            else
            {
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    rrow[CPL * (lane + 1) + c] = ScoreT(H[c]);
            }
            if (lane == 0)
                rrow[CPL - 1] = ScoreT(carry);
            bsv = lane == (r & (kBandRing - 1)) ? bs : bsv;
            if (ra_spill(a) || tflag)
            {
                ScoreT* srow = spill + size_t(r) * rowsz;
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    srow[CPL * (lane + 1) + c] = ScoreT(H[c]);
                const int pg = rowsz / CPL - (kWave + 1); // padding groups
                if (lane < pg)
                {
#pragma unroll
                    for (int c = 0; c < CPL; c++)
                        srow[CPL * (kWave + 1 + lane) + c] = ScoreT(minv);
                }
                if (lane == 0)
                {
                    srow[CPL - 1] = ScoreT(carry);
                    X.flags[r]    = 1;
                }
            }
            if (bs == 0 && lane == 0)
                X.col0[r] = carry;
            wave_sync();
#pragma unroll
            for (int c = 0; c < CPL; c++)
                Hp[c] = H[c];
            prevF0 = carry;
            a      = a1;
            b      = b1;
            c2     = c1;
            e2     = e1;
            rbw    = rbn;
            a1     = uint32_t(uniform(int(va2)));
            b1     = uint32_t(uniform(int(vb2)));
            c1     = uint32_t(uniform(int(vc2)));
            e1     = uint32_t(uniform(int(ve2)));
        }
        wave_sync(); // the staging buffers are rewritten by the next block
    }
    bp.add(kBpFwdCyc, BandProf::now() - f_t0);
    return end_row;
}

#include "poa_band_ad.hpp"

// get_score(row, col) semantics for the out-of-band traceback step.  Sets
// known = false for an in-band value that was not stored: such a value is
// not one of the T values, so no comparison with minv can match it.
template <typename ScoreT, int CPL>
__device__ int band_get_slow(int p, int col, const Band& B, BandAux X, const ScoreT* spill, int rowsz,
                             int gap, int minv, bool& known)
{
    X = as_global(X);
    known = true;
    if (p == 0)
        return (col >= 0 && col <= B.bw) ? col * gap : minv;
    const int bsp = B.start(p);
    if (col == 0)
        return bsp == 0 ? int(X.col0[p]) : minv;
    if (col < bsp || col > bsp + B.bw)
        return minv;
    const int idx = col - bsp;
    if (idx == 0)
        return minv;
    if (X.flags[p] & 1)
        return int(spill[size_t(p) * rowsz + idx + CPL - 1]);
    known = false;
    return 0;
}

// Traceback from (end_row, L) over the codes (:367-477).  Writes the reversed
// alignment into ag / ar and returns its length, -1 at the loop bound.
template <typename ScoreT, typename SizeT, int CPL>
__device__ __forceinline__ int band_traceback(WinGraph<SizeT> g, BandAux X, int V, const uint8_t* read, int L,
                              int end_row, const Band& B, const Scores sc, const ScoreT* spill, int rowsz,
                              GWAMD_LDS uint8_t* tile, SizeT* ag, SizeT* ar, int aln_cap,
                              int lane, BandProf& bp, bool rank, int tbmode)
{
    constexpr int kBandTile = band_tile_rows(CPL);
    X = as_global(X);
    spill = glb(spill);
    ag    = glb(ag);
    ar    = glb(ar);
    g = as_global(g);
    const uint64_t t_t0 = BandProf::now();
    const int bw    = B.bw;
    const int gap   = sc.gap;
    const int minv  = int(band_min_value<ScoreT>(sc));
    V               = uniform(V);
    L               = uniform(L);
    int i           = uniform(end_row), j = L;
    int prev_i = 0, prev_j = 0;
    int ti0 = INT_MIN / 2;
    uint32_t ta = 0, tb = 0, tcw = 0; // row records of the tile rows, lane k: row ti0 + k
    static_assert(kBandTile <= kWave, "tile records are held one per lane (lanes past the tile: unused)");
    // per-row move-decode info of the tile rows, after the code tile
    GWAMD_LDS v4i_t* rowinfo = reinterpret_cast<GWAMD_LDS v4i_t*>(tile + kBandTile * bw);
    int n = 0, loops = 0;
    const int bound = L + V + 2;
    int eg = 0, er = 0;
    auto flush = [&](int upto) {
        const int base = (upto - 1) & ~(kWave - 1);
        const int k    = base + lane;
        if (k < upto && k < aln_cap)
        {
            ag[k] = SizeT(eg > 0 ? int(g.sorted[eg - 1]) : -1);
            ar[k] = SizeT(er);
        }
    };
    bool bad = false;
    // code tile: kBandTile rows of bw = 64*CPL code bytes from row ti0 on, and
    // their row records one per lane
    auto load_tile = [&](int ii) {
        const uint64_t tt0 = BandProf::now();
        ti0 = max(1, ii - (kBandTile - 1));
        wave_sync();
        // 4*CPL 16-B pieces per lane, all loads of a chunk issued before its
        // first store waits (band widths past 512: chunks of 16 pieces, so the
        // staging stays within 64 VGPRs)
        constexpr int kPer    = kBandTile * CPL / 16;
        constexpr int kPerRow = 4 * CPL; // 16-B pieces per code row
        constexpr int kCh     = kPer > 32 ? (kPer % 16 == 0 ? 16 : 8) : kPer;
        static_assert(kPer % kCh == 0, "whole chunks");
        {
            const int rr = min(ti0 + lane, V); // one record per lane (rows past the tile: unused)
            ta           = X.reca[rr];
            tb           = X.recb[rr];
            tcw          = X.recc[rr];
        }
        for (int u0 = 0; u0 < kPer; u0 += kCh)
        {
            v4i_t q[kCh];
#pragma unroll
            for (int u = 0; u < kCh; u++)
            {
                const int t  = (u0 + u) * kWave + lane;
                const int rr = min(ti0 + t / kPerRow, V); // rows past V: never read
                q[u]         = *reinterpret_cast<const v4i_t*>(X.codes + size_t(rr) * bw + (t % kPerRow) * 16);
            }
#pragma unroll
            for (int u = 0; u < kCh; u++)
            {
                const int t = (u0 + u) * kWave + lane;
                *reinterpret_cast<GWAMD_LDS v4i_t*>(tile + (t / kPerRow) * bw + (t % kPerRow) * 16) = q[u];
            }
        }
        {
            // per tile row (lane k: row ti0 + k), what a move decode needs:
            // band start | no-predecessor flag (bit 30) | listed or escaped
            // predecessors (bit 31), and the inline distances of slots 0-3
            const int f       = ra_np(ta);
            const bool listed = f == int(kNpEsc) || (tb >> 31);
            v4i_t info;
            info.x = int(uint32_t(ra_bs(ta)) | (f == 0 ? (1u << 30) : 0u) | (listed ? (1u << 31) : 0u));
            info.y = int(tb);
            info.z = int(tcw);
            info.w = 0;
            rowinfo[lane] = info;
        }
        wave_sync();
        bp.add(kBpTileCyc, BandProf::now() - tt0);
    };
    // Move window (TbWin, poa_wave.hpp): the moves of 128 cells decoded in
    // one lane-parallel pass, two cells per lane, packed (row << 16 |
    // column); the walk then takes them instead of one LDS round trip and
    // its decoding per step.  Cells whose move needs more than the tile and
    // the inline predecessor distances (row 0, column 0, outside the band,
    // listed or escaped predecessor rows, no move) are kSlow and go through
    // the general step.
    constexpr uint32_t kSlow = 0xffffffffu;
    const bool win_ok       = V < 65535 && L < 65535;
    TbWin G;
    G.init(tbmode, i, L, kBandTile);
    uint32_t wpk0 = kSlow, wpk1 = kSlow;
    // branch-free: the row's info from the LDS table, then its code byte
    auto decode_cell = [&](int t) -> uint32_t {
        const int r      = G.row(t);
        const int c      = G.col(t);
        const int k      = min(max(r - ti0, 0), kBandTile - 1);
        const v4i_t info = rowinfo[k];
        const uint32_t x = uint32_t(info.x);
        const int bs     = int(x & 0x3fffffffu);
        const int idx    = c - bs - 1;
        const bool ok    = r >= 1 && c >= 1 && r >= ti0 && r < ti0 + kBandTile && uint32_t(idx) < uint32_t(bw);
        const int code   = int(tile[k * bw + min(max(idx, 0), bw - 1)]);
        const int dir    = code & 3;
        const int slot   = code >> 2;
        const uint32_t w = uint32_t(slot < 2 ? info.y : info.z);
        const int p      = (x & (1u << 30)) ? 0 : r - int((slot & 1) ? (w >> 16) : (w & 0xffffu));
        const uint32_t mv = dir == 2 ? ((uint32_t(r) << 16) | uint32_t(c - 1))
                                     : ((uint32_t(p) << 16) | uint32_t(dir == 0 ? c - 1 : c));
        const bool slow = !ok || dir == 3 || (dir != 2 && (x >> 31) != 0);
        return slow ? kSlow : mv;
    };
    while (!(i == 0 && j == 0) && loops < bound)
    {
        i      = uniform(i);
        j      = uniform(j);
        prev_i = uniform(prev_i);
        prev_j = uniform(prev_j);
        ti0    = uniform(ti0);
        G.wi0   = uniform(G.wi0);
        G.wj0   = uniform(G.wj0);
        G.slope = uniform(G.slope);
        G.next  = uniform(G.next);
        n      = uniform(n);
        loops  = uniform(loops);
        if (win_ok && i >= 1 && j >= 1)
        {
            if (G.index(i, j) < 0)
            {
                G.refill(i, j);
                // the tile must hold the window's rows (those >= 1)
                if (i < ti0 || i >= ti0 + kBandTile || (i - G.row_span() < ti0 && ti0 > 1))
                    load_tile(i);
                wpk0 = decode_cell(lane);
                wpk1 = decode_cell(lane + kWave);
                bp.add(kBpRefill, 1);
            }
            // walk the window: every value here is wave-uniform (SGPRs)
            int ci = i, cj = j, cn = n, cl = loops;
            if (rank)
                walk_window_ranked<1>(wpk0, wpk1, G, ci, cj, cn, cl, bound, lane, eg, er,
                                      tile + kBandTile * bw + kWave * 16 + 512, flush);
            else
            while (true)
            {
                const int idx     = G.index(ci, cj);
                const uint32_t nx = uint32_t(idx < kWave ? __builtin_amdgcn_readlane(int(wpk0), idx)
                                                         : __builtin_amdgcn_readlane(int(wpk1), idx - kWave));
                if (nx == kSlow)
                    break;
                const int pi = int(nx >> 16), pj = int(nx & 0xffffu);
                cl++;
                if (lane == (cn & (kWave - 1)))
                {
                    eg = ci == pi ? -1 : ci;
                    er = cj == pj ? -1 : cj - 1;
                }
                cn++;
                if ((cn & (kWave - 1)) == 0)
                    flush(cn);
                ci = pi;
                cj = pj;
                if ((ci == 0 && cj == 0) || cl >= bound || ci < 1 || cj < 1 || G.index(ci, cj) < 0)
                    break;
            }
            if (cl != loops)
            {
                G.follow(ci, cj);
                prev_i = i = ci;
                prev_j = j = cj;
                n      = cn;
                loops  = cl;
                continue;
            }
        }
        loops++;
        bp.add(kBpSlow, 1);
        bool found = false;
        int pi = 0, pj = 0;
        if (i == 0)
        {
            const int sij = (j <= bw) ? j * gap : minv;
            const int lft = (j - 1 >= 0 && j - 1 <= bw) ? (j - 1) * gap : minv;
            if (sij == lft + gap)
                pi = 0, pj = j - 1, found = true;
        }
        else
        {
            if (i < ti0 || i >= ti0 + kBandTile)
                load_tile(i);
            const uint32_t a = __builtin_amdgcn_readlane(ta, i - ti0);
            const uint32_t b = __builtin_amdgcn_readlane(tb, i - ti0);
            const uint32_t c = __builtin_amdgcn_readlane(tcw, i - ti0);
            const int bs     = ra_bs(a);
            if (j == 0)
            {
                // column 0: vertical moves only (get(i, -1) is minv)
                const int sij = bs == 0 ? int(X.col0[i]) : minv;
                const int np  = band_np2<SizeT>(g, i, a, b);
                const int npp = np == 0 ? 1 : np;
                for (int k = 0; k < npp && !found; k++)
                {
                    const int p   = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, c, k);
                    const int f0  = p == 0 ? 0 : (B.start(p) == 0 ? int(X.col0[p]) : minv);
                    if (sij == f0 + gap)
                        pi = p, pj = 0, found = true;
                }
                if (!found && sij == minv + gap)
                {
                    bad = true; // column -1: outside anything this build reproduces
                    break;
                }
            }
            else if (j >= bs + 1 && j <= bs + bw)
            {
                const int code = uniform(int(tile[(i - ti0) * bw + (j - bs - 1)]));
                const int dir  = code & 3;
                if (dir == 2)
                    pi = i, pj = j - 1, found = true;
                else if (dir != 3)
                {
                    const int f = ra_np(a);
                    if (f == 0)
                        pi = 0;
                    else if (f != int(kNpEsc) && !(b >> 31))
                    {
                        const int k      = code >> 2;
                        const uint32_t w = k < 2 ? b : c;
                        pi               = i - int((k & 1) ? (w >> 16) : (w & 0xffffu));
                    }
                    else
                    {
                        pi = uniform(band_pred2<SizeT>(g, X, i, a, b, c, code >> 2));
                        vm_drain();
                    }
                    pj           = dir == 0 ? j - 1 : j;
                    found        = true;
                }
            }
            else
            {
                // outside the band: get_score(i, j) is minv
                const int sij  = minv;
                const int cost = (ra_base(a) == int(read[j - 1])) ? sc.match : sc.mismatch;
                const int np   = band_np2<SizeT>(g, i, a, b);
                const int npp  = np == 0 ? 1 : np;
                for (int k = 0; k < npp && !found; k++)
                {
                    const int p = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, c, k);
                    bool kn;
                    const int gv = band_get_slow<ScoreT, CPL>(p, j - 1, B, X, spill, rowsz, gap, minv, kn);
                    if (kn && sij == gv + cost)
                        pi = p, pj = j - 1, found = true;
                }
                for (int k = 0; k < npp && !found; k++)
                {
                    const int p = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, c, k);
                    bool kn;
                    const int gv = band_get_slow<ScoreT, CPL>(p, j, B, X, spill, rowsz, gap, minv, kn);
                    if (kn && sij == gv + gap)
                        pi = p, pj = j, found = true;
                }
                if (!found)
                {
                    bool kn;
                    const int gv = band_get_slow<ScoreT, CPL>(i, j - 1, B, X, spill, rowsz, gap, minv, kn);
                    if (kn && sij == gv + gap)
                        pi = i, pj = j - 1, found = true;
                }
            }
        }
        if (found)
            prev_i = pi, prev_j = pj;
        if (lane == (n & (kWave - 1)))
        {
            eg = i == prev_i ? -1 : i;
            er = j == prev_j ? -1 : j - 1;
        }
        n++;
        if ((n & (kWave - 1)) == 0)
        {
            const uint64_t ft0 = BandProf::now();
            flush(n);
            bp.add(kBpFlushCyc, BandProf::now() - ft0);
        }
        i = prev_i;
        j = prev_j;
    }
    bp.add(kBpSteps, uint64_t(n));
    bp.add(kBpTbCyc, BandProf::now() - t_t0);
    if ((n & (kWave - 1)) != 0)
        flush(n);
    wave_sync();
    if (bad || loops >= bound || n > aln_cap)
        return -1;
    return n;
}

// Per-window pointers of the banded kernel (graph by window, scratch by slot).
template <typename ScoreT, typename SizeT>
__device__ __forceinline__ void band_window_ptrs(const Buffers& b, const Dims& d, int w, size_t slot, int rowsz,
                                                 WinGraph<SizeT>& g, BandAux& X, ScoreT*& spill)
{
    const size_t mn = size_t(d.max_nodes);
    g.base      = b.base + w * mn;
    g.in_cnt    = b.in_cnt + w * mn;
    g.out_cnt   = b.out_cnt + w * mn;
    g.aln_cnt   = b.aln_cnt + w * mn;
    g.cov       = b.node_cov + w * mn;
    g.in_w      = b.in_w + w * mn * kMaxEdges;
    g.in_e      = static_cast<SizeT*>(b.in_e) + w * mn * kMaxEdges;
    g.out_e     = static_cast<SizeT*>(b.out_e) + w * mn * kMaxEdges;
    g.aln       = static_cast<SizeT*>(b.aln) + w * mn * kMaxAlignments;
    g.sorted    = static_cast<SizeT*>(b.sorted) + w * mn;
    g.pos       = static_cast<SizeT*>(b.pos) + w * mn;
    g.max_nodes = d.max_nodes;
    spill       = static_cast<ScoreT*>(b.scores) + slot * d.score_rows * size_t(rowsz);
    uint8_t* aux = b.codes + slot * size_t(d.aux_stride);
    X.codes  = aux;
    X.reca   = reinterpret_cast<uint32_t*>(aux + d.aux_reca_off);
    X.recb   = reinterpret_cast<uint32_t*>(aux + d.aux_recb_off);
    X.recc   = reinterpret_cast<uint32_t*>(aux + d.aux_recc_off);
    X.rece   = reinterpret_cast<uint32_t*>(aux + d.aux_rece_off);
    X.col0   = reinterpret_cast<int32_t*>(aux + d.aux_col0_off);
    X.flags  = aux + d.aux_flag_off;
    X.xl     = reinterpret_cast<int32_t*>(aux + d.aux_xl_off);
    X.bx     = reinterpret_cast<int32_t*>(aux + d.aux_bx_off);
    X.xl_cap = d.aux_xl_cap;
}

// LDS bytes and layout of the graph update's scratch in the work region
__device__ __forceinline__ int band_add_bytes(int L, int V)
{
    const int ls = (L + 16 + 15) & ~15;
    return 5 * ls + ((2 * (V + L + 16) + 15) & ~15) + 2 * ls;
}

__device__ __forceinline__ AddScratch band_add_scratch(GWAMD_LDS uint8_t* work, GWAMD_LDS uint8_t* shb, int L, int V)
{
    const int ls   = (L + 16 + 15) & ~15;
    const int hoff = 5 * ls + ((2 * (V + L + 16) + 15) & ~15);
    AddScratch AX;
    AX.gid   = (GWAMD_LDS uint16_t*)(work);
    AX.curr  = (GWAMD_LDS uint16_t*)(work + 2 * ls);
    AX.kind  = work + 4 * ls;
    AX.owner = (GWAMD_LDS uint16_t*)(work + 5 * ls);
    AX.hit   = work + hoff;
    AX.ohit  = work + hoff + ls;
    AX.sh    = (GWAMD_LDS int*)(shb);
    return AX;
}

// One window per workgroup.  Wave 0 runs the whole window; with the
// anti-diagonal pass (d.band_ad) the workgroup has kAdMaxWaves waves and waves
// 1.. only join the forward passes: wave 0 posts each pass in sh_job and both
// sides meet at two barriers around it (sh_job[0] < 0: no more passes).
template <typename ScoreT, typename SizeT, bool MSA, int CPL>
__global__ void __launch_bounds__(kWave * kAdMaxWaves) poa_window_kernel_band(Buffers b, Dims d, Scores sc)
{
    constexpr int kBandRing = band_ring_rows(CPL);
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int sh_status;
    __shared__ int sh_len;
    __shared__ AdShared ad_sh;
    __shared__ int sh_job[8]; // window, V, L, gradient bits, job kind (0 forward pass, 1 topological sort:
                              // window, node count, hint count, previous node count; 2 graph update:
                              // window, node count, alignment length, L, -, read index, V)

    __shared__ int sh_next;
    if (int(blockIdx.x) >= b.num_windows)
        return;
    const int lane    = int(threadIdx.x) % kWave;
    const int wave    = int(threadIdx.x) / kWave;
    const int nw      = int(blockDim.x) / kWave;
    const size_t slot = blockIdx.x; // scratch slot (grid <= slots)
    GWAMD_LDS AdShared* adsh = (GWAMD_LDS AdShared*)(&ad_sh);

    uint8_t* lread          = lds + kReadGuard; // guard: the anti-diagonal pass reads read[c-1] for c >= -63
    GWAMD_LDS uint8_t* work = (GWAMD_LDS uint8_t*)(lds) + d.lds_ring_off;
    GWAMD_LDS ScoreT* ring  = (GWAMD_LDS ScoreT*)(work);
    GWAMD_LDS uint8_t* shb  = (GWAMD_LDS uint8_t*)(lds) + d.lds_sh_off;
    GWAMD_LDS uint8_t* tile = work;
    const int rowsz          = d.score_stride;
    // row-record staging after the ring (planned by poa_batch.cpp)
    GWAMD_LDS uint32_t* stage = (GWAMD_LDS uint32_t*)(work + ((kBandRing * rowsz * int(sizeof(ScoreT)) + 15) & ~15));

    if (wave > 0)
    {
        // helper waves: forward passes posted by wave 0
        while (true)
        {
            __syncthreads(); // pass posted
            const int w = sh_job[0];
            if (w < 0)
                break;
            WinGraph<SizeT> g;
            BandAux X;
            ScoreT* spill;
            band_window_ptrs<ScoreT, SizeT>(b, d, w, slot, rowsz, g, X, spill);
            if (sh_job[4] == 1)
            {
                // the level-keyed Kahn sort of this read (every wave)
                topsort_levels<SizeT>(g, sh_job[1], sh_job[3], (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off,
                                      int(threadIdx.x), int(blockDim.x),
                                      static_cast<SizeT*>(b.cpred) + slot * size_t(d.max_nodes) * 4, sh_job[2]);
                __syncthreads(); // pass done
                continue;
            }
            if (sh_job[4] == 2)
            {
                // the order-free passes of the graph update (every wave)
                const WindowDesc wd = b.windows[w];
                const int s         = sh_job[5];
                const int L         = sh_job[3];
                const int V         = sh_job[6];
                int nc              = sh_job[1];
                const size_t mn     = size_t(d.max_nodes);
                uint16_t* ecov      = MSA ? b.edge_cov + w * mn * kMaxEdges * d.max_seqs : nullptr;
                uint16_t* ecovc     = MSA ? b.edge_cov_cnt + w * mn * kMaxEdges : nullptr;
                SizeT* seq_begin    = MSA ? static_cast<SizeT*>(b.seq_begin) + size_t(w) * d.max_seqs : nullptr;
                AddScratch AX       = band_add_scratch(work, shb, L, V);
                add_alignment_parallel_batched<SizeT, MSA, kBandAddAU>(
                    g, nc, static_cast<SizeT*>(b.ag) + slot * d.aln_cap, static_cast<SizeT*>(b.ar) + slot * d.aln_cap,
                    sh_job[2], L, lread, b.wts + b.seq_off[wd.first_seq + s], s, ecov, ecovc, seq_begin, d.max_seqs,
                    AX, lane, nullptr, wave, nw);
                __syncthreads(); // pass done
                continue;
            }
            Band B;
            B.bw         = d.band_width;
            B.stride     = d.band_width + kBandPad;
            B.max_column = sh_job[2] + 1;
            B.gradient   = __int_as_float(sh_job[3]);
            BandProf bp;
            if constexpr (CPL <= 4) // the anti-diagonal pass serves band widths 128 and 256
                band_forward_ad<ScoreT, SizeT, CPL>(g, X, sh_job[1], (GWAMD_LDS const uint8_t*)(lread), sh_job[2], B,
                                                    sc, ring, spill, rowsz, d.score_rows, lane, wave, nw, adsh, bp);
            __syncthreads(); // pass done
        }
        return;
    }

    for (int idx = blockIdx.x; idx < b.num_windows;)
    {
    const int w     = b.order ? b.order[idx] : idx;
    const size_t mn = size_t(d.max_nodes);
    WinGraph<SizeT> g;
    BandAux X;
    ScoreT* spill;
    band_window_ptrs<ScoreT, SizeT>(b, d, w, slot, rowsz, g, X, spill);
    SizeT* ag        = static_cast<SizeT*>(b.ag) + slot * d.aln_cap;
    SizeT* ar        = static_cast<SizeT*>(b.ar) + slot * d.aln_cap;
    int32_t* cscore  = b.cscore + slot * mn;
    SizeT* cpred     = static_cast<SizeT*>(b.cpred) + slot * mn * 4;
    uint16_t* ecov   = MSA ? b.edge_cov + w * mn * kMaxEdges * d.max_seqs : nullptr;
    uint16_t* ecovc  = MSA ? b.edge_cov_cnt + w * mn * kMaxEdges : nullptr;
    SizeT* seq_begin = MSA ? static_cast<SizeT*>(b.seq_begin) + size_t(w) * d.max_seqs : nullptr;

    PhaseTimer ph;
    BandProf bp;
    uint64_t tsprof[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}; // topsort sections (GWAMD_TOPSORT_PROFILE builds)
    uint64_t addprof[8] = {0, 0, 0, 0, 0, 0, 0, 0}; // add sections (GWAMD_ADD_PROFILE builds)
    const WindowDesc wd = b.windows[w];
    const int nseq      = wd.num_seqs;
    int status          = kSuccess;
    int64_t cells       = 0;
    int node_count      = 0;
    int lv_hint         = 0; // nodes whose critical predecessor of the last level sort is in cpred

    if (nseq > 0)
    {
        const int len0      = b.seq_len[wd.first_seq];
        const uint8_t* seq0 = b.seqs + b.seq_off[wd.first_seq];
        const int8_t* w0    = b.wts + b.seq_off[wd.first_seq];
        build_backbone<SizeT, MSA>(g, seq0, w0, len0, lane, ecov, ecovc, seq_begin, d.max_seqs);
        node_count = len0;
        ph.lap<kPhBackbone>();
        for (int s = 1; s < nseq; s++)
        {
            if (node_count >= d.max_nodes) // cudapoa_kernels.cuh:222-227
            {
                status = kNodeCountExceeded;
                break;
            }
            const int L           = b.seq_len[wd.first_seq + s];
            const int64_t off     = b.seq_off[wd.first_seq + s];
            const uint8_t* read_g = b.seqs + off;
            const int8_t* wts_g   = b.wts + off;
            // staged read, zero padded past the band's last column
            const int padded = (L + d.band_width + 32 + 15) & ~15;
            for (int j = lane; j < padded; j += kWave)
                lread[j] = j < L ? read_g[j] : 0;
            const int V = node_count;
            Band B;
            B.bw         = d.band_width;
            B.stride     = d.band_width + kBandPad;
            B.max_column = L + 1;
            B.gradient   = float(L + 1) / float(V + 1); // cudapoa_nw_banded.cuh:206
            // spill rows for successors kBandRing or more rows later: enough for
            // both forward passes (kAdSpillDist > kBandRing)
            const int npmax = band_row_program<SizeT>(g, V, B, X, lane, work, kBandRing, kAdSpillDist);
            wave_sync();
            ph.lap<kPhRowProg>();
            cells += int64_t(V + 1) * (d.band_width + kBandPad);
            int end_row;
            if (CPL <= 4 && d.band_ad && npmax <= kAdMaxSlots)
            {
              if constexpr (CPL <= 4)
              {
                band_ad_init<ScoreT, CPL>(ring, rowsz, d.band_width, int(band_min_value<ScoreT>(sc)), V, adsh, lane);
                if (nw > 1)
                {
                    if (lane == 0)
                    {
                        sh_job[0] = w;
                        sh_job[1] = V;
                        sh_job[2] = L;
                        sh_job[3] = __float_as_int(B.gradient);
                        sh_job[4] = 0;
                    }
                    __syncthreads(); // pass posted
                }
                band_forward_ad<ScoreT, SizeT, CPL>(g, X, V, (GWAMD_LDS const uint8_t*)(lread), L, B, sc, ring, spill,
                                                    rowsz, d.score_rows, lane, 0, nw, adsh, bp);
                if (nw > 1)
                    __syncthreads(); // pass done
                end_row = uniform(band_ad_end_row(adsh, nw));
                if (uniform(__hip_atomic_load(&adsh->stalled, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
                {
                    status = kGenericError; // a progress wait ran out: the scores are not trustworthy
                    break;
                }
              }
            }
            else
                end_row = band_forward<ScoreT, SizeT, CPL>(g, X, V, (GWAMD_LDS const uint8_t*)(lread), L, B, sc, ring,
                                                           stage, spill, rowsz, lane, bp);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ph.lap<kPhForward>();
            const int alen = band_traceback<ScoreT, SizeT, CPL>(g, X, V, lread, L, end_row, B, sc, spill, rowsz, tile,
                                                                ag, ar, d.aln_cap, lane, bp, (d.tb_rank & 1) != 0,
                                                                d.tb_rank);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ph.lap<kPhTraceback>();
            if (alen == -1)
            {
                status = kLoopCountExceeded;
                break;
            }
            int nc = node_count;
            int rc = -1;
            if (band_add_bytes(L, V) <= d.lds_work_bytes)
            {
                // add-alignment scratch in the work region, sized for this read;
                // with helper waves the order-free passes run on all of them
                AddScratch AX = band_add_scratch(work, shb, L, V);
                if (nw > 1)
                {
                    if (lane == 0)
                    {
                        sh_job[0] = w;
                        sh_job[1] = nc;
                        sh_job[2] = alen;
                        sh_job[3] = L;
                        sh_job[4] = 2;
                        sh_job[5] = s;
                        sh_job[6] = V;
                    }
                    __syncthreads(); // pass posted
                }
                rc = add_alignment_parallel_batched<SizeT, MSA, kBandAddAU>(g, nc, ag, ar, alen, L, lread, wts_g, s,
                                                                           ecov, ecovc, seq_begin, d.max_seqs, AX,
                                                                           lane, addprof, 0, nw);
                if (nw > 1)
                    __syncthreads(); // pass done
            }
            if (rc < 0)
            {
                bp.add(kBpAddSeq, 1);
                if (lane == 0)
                {
                    sh_status = add_alignment<SizeT, MSA>(g, nc, ag, ar, alen, read_g, wts_g, s, ecov, ecovc,
                                                          seq_begin, d.max_seqs);
                    sh_len    = nc;
                }
                wave_sync();
                rc = sh_status;
                nc = sh_len;
            }
            ph.lap<kPhAdd>();
            rc = uniform(rc); // wave-uniform: the sort below runs scalar control flow
            nc = uniform(nc);
            bool lv_done = false;
            if (rc == kSuccess && !d.spoa_accurate && !(d.diag & 4))
            {
                // level-keyed Kahn sort on every wave of the workgroup
                // (GWAMD_TOPSORT=fifo, Dims::diag bit 2, keeps the FIFO below)
                if (nw > 1)
                {
                    if (lane == 0)
                    {
                        sh_job[0] = w;
                        sh_job[1] = nc;
                        sh_job[2] = lv_hint;
                        sh_job[3] = V;
                        sh_job[4] = 1;
                    }
                    __syncthreads(); // pass posted
                }
                lv_done = topsort_levels<SizeT>(g, nc, V, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, int(threadIdx.x),
                                                int(blockDim.x), cpred, lv_hint,
#ifdef GWAMD_TOPSORT_PROFILE
                                                tsprof
#else
                                                nullptr
#endif
                );
                if (nw > 1)
                    __syncthreads(); // pass done
                lv_done = uniform(lv_done ? 1 : 0) != 0;
            }
            lv_hint = lv_done ? nc : 0; // cpred holds c(v) of this sort for the next one
            if (rc == kSuccess && !lv_done)
            {
                if (d.spoa_accurate)
                    rc = topsort_racon_wave<SizeT>(g, nc, cscore, cpred, 4 * d.max_nodes, lane,
                                                   (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off);
                // (no ring-forcing diagnostic here: that runtime flag doubled
                // this kernel's SGPR spill reloads, 6,364 -> 13,364, and slowed
                // config C's forward pass 64 -> 79 ms per window; the ring mode
                // is the same topsort_lds code, tested through the LDS kernel)
                else if (!topsort_lds<SizeT>(g, nc, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, (GWAMD_LDS int*)(shb),
                                             lane, tsprof) &&
                         !topsort_lds_big<SizeT>(g, nc, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, lane))
                {
                    if (lane == 0)
                        topsort_kahn<SizeT>(g, nc, cscore);
                    wave_sync();
                }
            }
            ph.lap<kPhTopsort>();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            status     = uniform(rc);
            node_count = uniform(nc);
            if (status != kSuccess)
                break;
        }
    }

    uint64_t oprof[3] = {0, 0, 0}; // output sections (GWAMD_OUTPUT_PROFILE builds)
    finish_window<SizeT, MSA>(b, d, w, lane, g, status, nseq, node_count, cscore, cpred, ecov, ecovc, seq_begin,
                              sh_len, sh_status, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, oprof);
    ph.lap<kPhOutput>();
    if (lane == 0)
    {
        if (b.phase)
        {
            ph.store(b.phase + size_t(w) * kPhases);
#ifdef GWAMD_ADD_PROFILE
            // add sections over all 8 slots (ticks): gid fill, kinds, new ids,
            // node claims, group claims, edge existence, writes 1, writes 2
            for (int k = 0; k < 8; k++)
                b.phase[size_t(w) * kPhases + k] = int64_t(addprof[k]);
#endif
#ifdef GWAMD_OUTPUT_PROFILE
            // output sections over the backbone / add / rowprog slots (ticks):
            // consensus, racon sort + column map, MSA rows
            b.phase[size_t(w) * kPhases + kPhBackbone] = int64_t(oprof[0]);
            b.phase[size_t(w) * kPhases + kPhAdd]      = int64_t(oprof[1]);
            b.phase[size_t(w) * kPhases + kPhRowProg]  = int64_t(oprof[2]);
#endif
#ifdef GWAMD_TOPSORT_PROFILE
            // level sort sections (s_memtime cycles / 1000 in every phase slot,
            // in order: init, reset, in-order pass, anchor rounds, final pass +
            // checks, counting sort + slots, runs + outputs; the total slot
            // holds the anchor count)
            for (int k = 0; k < 7; k++)
                b.phase[size_t(w) * kPhases + k] = int64_t(tsprof[k] / 1000);
            b.phase[size_t(w) * kPhases + kPhTotal] = int64_t(tsprof[7] / 1000);
#endif
#ifdef GWAMD_BAND_PROFILE
            // counters over the phase slots (read raw: value = phase_ms * 1e5)
            // backbone: traceback tile-staging cycles, add: sequential adds,
            // topsort: move-window refills, output: forward cycles, rowprog:
            // traceback steps, total: traceback cycles
            int64_t* ph8 = b.phase + size_t(w) * kPhases;
#ifdef GWAMD_BAND_PROFILE_AD
            if (d.band_ad)
#else
            if (false)
#endif
            {
                // anti-diagonal pass: general-step blocks, blocks, setup cycles,
                // forward cycles, step-loop cycles, steps
                ph8[kPhBackbone] = int64_t(bp.v[kBpMulti]);
                ph8[kPhAdd]      = int64_t(bp.v[kBpAdBlocks]);
                ph8[kPhTopsort]  = int64_t(bp.v[kBpAdSetup]);
                ph8[kPhOutput]   = int64_t(bp.v[kBpFwdCyc]);
                ph8[kPhRowProg]  = int64_t(bp.v[kBpAdLoop]);
                ph8[kPhTotal]    = int64_t(bp.v[kBpAdSteps]);
            }
            else
            {
            ph8[kPhBackbone] = int64_t(bp.v[kBpTileCyc]);
            ph8[kPhAdd]      = int64_t(bp.v[kBpAddSeq]); // reads added by the sequential add
            ph8[kPhTopsort]  = int64_t(bp.v[kBpRefill]);
            ph8[kPhOutput]   = int64_t(bp.v[kBpFwdCyc]);
            ph8[kPhRowProg]  = int64_t(bp.v[kBpSteps]);
            ph8[kPhTotal]    = int64_t(bp.v[kBpTbCyc]);
            }
#endif
        }
        b.final_nodes[w] = node_count;
        b.cells[w]       = cells;
    }
    if (b.head == nullptr)
        break;
    // next queue position; the LDS image is rewritten by the next window
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane == 0)
        sh_next = b.num_slots + atomicAdd(b.head, 1);
    wave_sync();
    idx = uniform(sh_next);
    }
    if (nw > 1)
    {
        if (lane == 0)
            sh_job[0] = -1;
        __syncthreads(); // release the helper waves
    }
}

} // namespace poa
} // namespace gwamd

// Launch and occupancy entry points of one band-width class: poa_band.hip is
// compiled once per cells-per-lane value (poa_band_c2/c4/c8.hip define
// GWAMD_BAND_TU_CPL) so the three instantiation sets build in parallel;
// poa_band_dispatch.cpp picks the one the plan needs.
#ifndef GWAMD_BAND_TU_CPL
#error "poa_band.hip is built through poa_band_c<CPL>.hip (CPL 2, 4, 6, 8, 10, 12, 14, 16)"
#endif
#define GWAMD_BAND_CAT2(a, b) a##b
#define GWAMD_BAND_CAT(a, b) GWAMD_BAND_CAT2(a, b)

extern "C" hipError_t GWAMD_BAND_CAT(gwamd_internal_poa_band_launch_cpl, GWAMD_BAND_TU_CPL)(
    const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d, const gwamd::poa::Scores* sc, int score_bits,
    int size_bits, int msa, hipStream_t stream)
{
    using namespace gwamd::poa;
    constexpr int CPL = GWAMD_BAND_TU_CPL;
    const dim3 grid(b->head ? b->num_slots : b->num_windows), blk(kWave * (d->band_ad ? d->band_ad : 1));
    const size_t lb = size_t(d->lds_bytes);
#define GWAMD_BAND_LAUNCH(ST, ZT, MS)                                                                           \
    {                                                                                                         \
        auto kfn = poa_window_kernel_band<ST, ZT, MS, CPL>;                                                   \
        if (lb > 65536)                                                                                       \
        {                                                                                                     \
            hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),                            \
                                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lb));          \
            if (e != hipSuccess)                                                                              \
                return e;                                                                                     \
        }                                                                                                     \
        hipLaunchKernelGGL(kfn, grid, blk, lb, stream, *b, *d, *sc);                                          \
        return hipGetLastError();                                                                             \
    }
#define GWAMD_BAND_MSA(ST, ZT)              \
    if (msa)                                \
        GWAMD_BAND_LAUNCH(ST, ZT, true)     \
    GWAMD_BAND_LAUNCH(ST, ZT, false)
    if (d->lds_cpl != CPL)
        return hipErrorInvalidConfiguration;
    if (score_bits == 16)
    {
        GWAMD_BAND_MSA(int16_t, int16_t)
    }
    if (size_bits == 16)
    {
        GWAMD_BAND_MSA(int32_t, int16_t)
    }
    GWAMD_BAND_MSA(int32_t, int32_t)
#undef GWAMD_BAND_MSA
#undef GWAMD_BAND_LAUNCH
}

// Resident workgroups per CU of the planned banded kernel (persistent grid).
extern "C" int GWAMD_BAND_CAT(gwamd_internal_poa_band_blocks_per_cu_cpl, GWAMD_BAND_TU_CPL)(
    const gwamd::poa::Dims* d, int score_bits, int size_bits, int msa)
{
    using namespace gwamd::poa;
    constexpr int CPL = GWAMD_BAND_TU_CPL;
    const size_t lb = size_t(d->lds_bytes);
#define GWAMD_BAND_OCC(ST, ZT, MS)                                                                              \
    {                                                                                                         \
        auto kfn = poa_window_kernel_band<ST, ZT, MS, CPL>;                                                   \
        if (lb > 65536 && hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),                             \
                                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lb)) != hipSuccess) \
            return 0;                                                                                         \
        int n = 0;                                                                                            \
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kfn, kWave * (d->band_ad ? d->band_ad : 1), lb) !=      \
            hipSuccess)                                                                                       \
            return 0;                                                                                         \
        return n;                                                                                             \
    }
#define GWAMD_BAND_OCC_MSA(ST, ZT)         \
    if (msa)                               \
        GWAMD_BAND_OCC(ST, ZT, true)       \
    GWAMD_BAND_OCC(ST, ZT, false)
    if (d->lds_cpl != CPL)
        return 0;
    if (score_bits == 16)
    {
        GWAMD_BAND_OCC_MSA(int16_t, int16_t)
    }
    if (size_bits == 16)
    {
        GWAMD_BAND_OCC_MSA(int32_t, int16_t)
    }
    GWAMD_BAND_OCC_MSA(int32_t, int32_t)
#undef GWAMD_BAND_OCC_MSA
#undef GWAMD_BAND_OCC
}
#undef GWAMD_BAND_CAT
#undef GWAMD_BAND_CAT2

// MI355X (gfx950) POA kernels: one POA window per 64-lane workgroup.
//
// Per window and per read s >= 1 (reference generatePOAKernel,
// cudapoa_kernels.cuh:66-359):
//   1. the read is staged in LDS;
//   2. the DP over the graph rows in topological order runs wave-parallel:
//      each lane owns 8 consecutive columns (one 16-B group of the score row),
//      the diagonal/vertical maxima over all predecessors are formed in
//      registers, and the horizontal gap closure is an exact max-prefix scan
//      across the wave (H[j] - j*gap is a running maximum), replacing the
//      reference's __any_sync fix-point loop (cudapoa_nw.cuh:265-310);
//   3. traceback, addAlignmentToGraph and the Kahn topological sort run on
//      lane 0 with the reference's tie order;
// then the heaviest-bundle consensus (or the racon sort + MSA) is generated in
// the same launch (reference runs them as separate kernels).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "poa_wave.hpp"

namespace gwamd
{
namespace poa
{

// ---------------------------------------------------------------------------
template <typename ScoreT, typename SizeT, bool BANDED, bool MSA>
__global__ void __launch_bounds__(kWave) poa_window_kernel(Buffers b, Dims d, Scores sc)
{
    extern __shared__ __align__(16) uint8_t lds_read[];
    __shared__ int sh_alen;
    __shared__ int sh_status;
    __shared__ int sh_len;

    const int w = b.order ? b.order[blockIdx.x] : int(blockIdx.x);
    if (w >= b.num_windows)
        return;
    const int lane = threadIdx.x;

    const size_t mn = size_t(d.max_nodes);
    WinGraph<SizeT> g;
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

    SizeT* ag        = static_cast<SizeT*>(b.ag) + size_t(w) * d.aln_cap;
    SizeT* ar        = static_cast<SizeT*>(b.ar) + size_t(w) * d.aln_cap;
    ScoreT* S        = static_cast<ScoreT*>(b.scores) + size_t(w) * d.score_rows * size_t(d.score_stride);
    int32_t* cscore  = b.cscore + w * mn;
    SizeT* cpred     = static_cast<SizeT*>(b.cpred) + w * mn * 4; // also the racon stack
    uint16_t* ecov   = MSA ? b.edge_cov + w * mn * kMaxEdges * d.max_seqs : nullptr;
    uint16_t* ecovc  = MSA ? b.edge_cov_cnt + w * mn * kMaxEdges : nullptr;
    SizeT* seq_begin = MSA ? static_cast<SizeT*>(b.seq_begin) + size_t(w) * d.max_seqs : nullptr;

    PhaseTimer ph;
    const WindowDesc wd = b.windows[w];
    const int nseq      = wd.num_seqs;
    int status          = kSuccess;
    int64_t cells       = 0;
    int node_count      = 0;

    if (nseq > 0)
    {
        const int len0 = b.seq_len[wd.first_seq];
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
            const int L             = b.seq_len[wd.first_seq + s];
            const int64_t off       = b.seq_off[wd.first_seq + s];
            const uint8_t* read_g   = b.seqs + off;
            const int8_t* wts_g     = b.wts + off;
            // stage read in LDS (padded with zeros to a 16-B multiple)
            const int padded = (L + 16 + 15) & ~15;
            for (int j = lane; j < padded; j += kWave)
                lds_read[j] = j < L ? read_g[j] : 0;
            __syncthreads();
            const int V = node_count;
            int alen;
            if (BANDED)
            {
                Band B;
                B.bw         = d.band_width;
                B.stride     = d.band_width + kBandPad;
                B.max_column = L + 1;
                B.gradient   = float(L + 1) / float(V + 1);
                cells += int64_t(V + 1) * (d.band_width + kBandPad);
                nw_forward_banded<ScoreT, SizeT>(g, V, lds_read, L, S, B, sc, lane);
                __syncthreads();
                ph.lap<kPhForward>();
                if (lane == 0)
                    sh_alen = traceback_banded<ScoreT, SizeT>(g, V, lds_read, L, S, B, sc, ag, ar, d.aln_cap);
            }
            else
            {
                cells += int64_t(V + 1) * (L + 1);
                nw_forward_full<ScoreT, SizeT>(g, V, lds_read, L, S, d.score_stride, sc, lane);
                __syncthreads();
                ph.lap<kPhForward>();
                if (lane == 0)
                    sh_alen = traceback_full<ScoreT, SizeT>(g, V, lds_read, L, S, d.score_stride, sc, ag, ar,
                                                            d.aln_cap);
            }
            __syncthreads();
            ph.lap<kPhTraceback>();
            alen = sh_alen;
            if (alen == -1)
            {
                status = kLoopCountExceeded;
                break;
            }
            if (lane == 0)
            {
                int nc     = node_count;
                uint8_t rc = add_alignment<SizeT, MSA>(g, nc, ag, ar, alen, read_g, wts_g, s, ecov, ecovc, seq_begin,
                                                       d.max_seqs);
                ph.lap<kPhAdd>();
                rc = uniform(rc); // wave-uniform: the sort below runs scalar control flow
                nc = uniform(nc);
                if (rc == kSuccess)
                {
                    if (d.spoa_accurate) // cudapoa_kernels.cuh:324-337
                    {
                        if (!topsort_racon<SizeT>(g, nc, cscore, cpred, 4 * d.max_nodes))
                            rc = kGenericError;
                    }
                    else
                        topsort_kahn<SizeT>(g, nc, cscore);
                }
                ph.lap<kPhTopsort>();
                sh_status = rc;
                sh_len    = nc;
            }
            __syncthreads();
            status     = uniform(sh_status); // LDS values: tell the compiler they are wave-uniform
            node_count = uniform(sh_len);
            if (status != kSuccess)
                break;
        }
    }

    finish_window<SizeT, MSA>(b, d, w, lane, g, status, nseq, node_count, cscore, cpred, ecov, ecovc, seq_begin,
                              sh_len, sh_status);
    ph.lap<kPhOutput>();
    if (lane == 0)
    {
        if (b.phase)
            ph.store(b.phase + size_t(w) * kPhases);
        b.final_nodes[w] = node_count;
        b.cells[w]       = cells;
    }
}


// ===========================================================================
// LDS-resident kernel (full alignment, 16-bit scores and node ids).
//
// Differences from poa_window_kernel, same results:
//  * scores are kept in the E domain, E[i][j] = H[i][j] - j*gap, so the
//    horizontal gap closure is a plain prefix maximum and row 0 is all zeros;
//  * only the last kRing rows live in LDS (a ring); a row is also written to
//    HBM ("spilled") only if a later row reads it from farther back than the
//    ring (measured predecessor distances are <= 10 rows);
//  * instead of the score matrix the forward pass writes one traceback code
//    per cell (direction + predecessor slot, chosen with the reference's tie
//    order, cudapoa_nw.cuh:361-443), and the traceback walks those codes from
//    128x128 tiles staged in LDS;
//  * the per-read row program (base, predecessor rows, sink/spill flags) is
//    built in LDS once per read, so the row loop touches HBM only for the
//    code stores.
// ===========================================================================

constexpr uint32_t kRecEscape = 63; // np field: predecessor rows read from the graph in HBM


struct RowProg
{
    const uint32_t* rec;
    const uint16_t* xl;
    int ring_mask;
};

// k-th predecessor row of row r (0 = the virtual row 0)
template <typename SizeT>
__device__ __forceinline__ int prog_pred(const RowProg& P, WinGraph<SizeT> g, int r, uint32_t rec, int k)
{
    g = as_global(g);
    const int np = (rec >> 8) & 63;
    if (np == 0)
        return 0; // source node: the virtual row 0
    if (np == 1)
        return r - int(rec >> 16);
    if (np == int(kRecEscape))
    {
        uint32_t t = uint32_t(pred_row(g, int(g.sorted[r - 1]), k));
        asm volatile("" : "+v"(t)); // wait here, not where the paths join
        return int(t);
    }
    return int(P.xl[(rec >> 16) + k]);
}

template <typename SizeT>
__device__ __forceinline__ int prog_np(WinGraph<SizeT> g, int r, uint32_t rec)
{
    g = as_global(g);
    const int np = (rec >> 8) & 63;
    return np == int(kRecEscape) ? int(g.in_cnt[int(g.sorted[r - 1])]) : np;
}

// Row program for rows 1..V (built after every topological sort).  The graph
// lives in HBM, so the loads are batched for memory-level parallelism: each
// lane takes kRP rows per pass and every dependent level (node, its counts,
// its first two predecessors' node ids, their rows) is issued for all of them
// before the next level waits.  A row spills when a successor reads it from
// ring_rows or more rows later; that is marked from the successor's side
// (row s, predecessor row p: s - p >= ring_rows) into byte flags in `flags`
// (V + 2 bytes of free LDS), so no out-edge lists are read.
// The base of forward-pass row r from its record (build_row_program): bits
// 0-6, or the graph's own byte when they hold 0x7f, which stands for 0x7f and
// for every byte >= 0x80 (the reference compares whole bytes, and bit 7 of
// the record is the general-path flag)
template <typename SizeT>
__device__ __forceinline__ int row_base(WinGraph<SizeT> g, uint32_t rec, int r)
{
    const int b = int(rec & 0x7fu);
    return b == 0x7f ? uniform(int(g.base[g.sorted[r - 1]])) : b;
}

template <typename SizeT>
__device__ void build_row_program(WinGraph<SizeT> g, int V, uint32_t* rec, uint16_t* xl, int xl_cap,
                                  int ring_rows, int lane, GWAMD_LDS uint8_t* flags)
{
    g = as_global(g);
    constexpr int kRP = 4;
    for (int r = lane; r <= V + 1; r += kWave)
        flags[r] = 0;
    wave_sync();
    int xbase = 0;
    for (int r0 = 1; r0 <= V; r0 += kRP * kWave)
    {
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
            // slots beyond in_cnt hold stale ids: clamp to a valid node
            p0[u] = int(g.pos[np[u] >= 1 ? e0[u] : 0]) + 1;
            p1[u] = int(g.pos[np[u] >= 2 ? e1[u] : 0]) + 1;
        }
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            const int r      = r0 + u * kWave + lane;
            const bool valid = r <= V;
            const int n      = valid ? np[u] : 0;
            int total        = 0;
            const int excl   = wave_excl_sum(n >= 2 ? n : 0, lane, total);
            if (valid)
            {
                // bits 0-6: the base, 0x7f standing for 0x7f and for every
                // byte >= 0x80 (the forward passes read such rows' base back
                // from the graph, row_base); bit 7: the forward pass must take
                // its general path (nw_forward_lds_v2): a source, a
                // predecessor beyond the ring, an escaped list or a base
                // other than ACGT
                const uint32_t ub = uint32_t(base[u]);
                uint32_t v        = (ub >= 0x7fu ? 0x7fu : ub) | (uint32_t(oc[u] == 0 ? 1 : 0) << 14);
                bool slow = n == 0 || !((ub & 0xc0u) == 0x40u && ((0x10008aull >> (ub & 0x3fu)) & 1u));
                if (n == 1)
                {
                    v |= (1u << 8) | (uint32_t(r - p0[u]) << 16);
                    if (r - p0[u] >= ring_rows)
                    {
                        flags[p0[u]] = 1;
                        slow         = true;
                    }
                }
                else if (n >= 2)
                {
                    const int off  = xbase + excl;
                    const bool fit = off + n <= xl_cap;
                    for (int k = 0; k < n; k++)
                    {
                        const int pk = k == 0 ? p0[u] : (k == 1 ? p1[u] : pred_row(g, node[u], k));
                        if (fit)
                            xl[off + k] = uint16_t(pk);
                        if (r - pk >= ring_rows)
                        {
                            flags[pk] = 1;
                            slow      = true;
                        }
                    }
                    v |= fit ? (uint32_t(n) << 8) | (uint32_t(off) << 16) : (kRecEscape << 8);
                    slow = slow || !fit;
                }
                rec[r] = v | (slow ? 0x80u : 0u);
            }
            xbase += total;
        }
    }
    wave_sync();
    for (int r = lane + 1; r <= V; r += kWave)
        if (flags[r])
            rec[r] |= 1u << 15;
    wave_sync();
}

// ---------------------------------------------------------------------------
// Packed 16-bit forward pass.  E values are int16 (the E-domain bounds of a
// window that selects 16-bit scores fit: cudapoa_limits.hpp:28-53), two cells
// per 32-bit register, so the diagonal/vertical/max work runs on v_pk_*
// instructions.  Cells beyond the read may wrap; they only feed cells further
// right, never a cell <= L.
typedef short pk_s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short pk_u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(pk_s16x2, a),
                                                                  __builtin_bit_cast(pk_s16x2, b)));
}
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(pk_u16x2, a) + __builtin_bit_cast(pk_u16x2, b));
}
// min/mad against 0/1 constants are rewritten by the compiler into per-half
// compare + select sequences; the callers pass the constants through
// opaque_u32() so the packed forms survive.
__device__ __forceinline__ uint32_t pk_sub(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(pk_u16x2, a) - __builtin_bit_cast(pk_u16x2, b));
}
__device__ __forceinline__ uint32_t pk_min_u(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(pk_u16x2, a),
                                                                  __builtin_bit_cast(pk_u16x2, b)));
}
__device__ __forceinline__ uint32_t pk_mad(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(pk_u16x2, a) * __builtin_bit_cast(pk_u16x2, b) +
                                            __builtin_bit_cast(pk_u16x2, c));
}
__device__ __forceinline__ uint32_t opaque_u32(uint32_t v)
{
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ uint32_t pk_bcast(int v) { return (uint32_t(uint16_t(v)) * 0x10001u); }
// (lo, max(hi, lo)): one v_pk_max_i16 with op_sel_hi selecting src1's low half
__device__ __forceinline__ uint32_t pk_max_lo_into_hi(uint32_t a)
{
    const pk_s16x2 v = __builtin_bit_cast(pk_s16x2, a);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(v, __builtin_shufflevector(v, v, 0, 0)));
}
// max(a, (c.hi, c.hi)): the carry of the previous register pair, via op_sel
__device__ __forceinline__ uint32_t pk_max_hi_carry(uint32_t a, uint32_t c)
{
    const pk_s16x2 v = __builtin_bit_cast(pk_s16x2, c);
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(pk_s16x2, a),
                                                                  __builtin_shufflevector(v, v, 1, 1)));
}

// Global loads on the rare far-predecessor paths are waited for inside their
// branch: a value still in flight where the paths join makes the compiler wait
// for vmcnt(0) on the common path too, i.e. for every code/spill store the
// wave has issued (HBM store latency on each row).
__device__ __forceinline__ void settle_vm1(uint32_t& v) { asm volatile("" : "+v"(v)); }
template <int NR>
__device__ __forceinline__ void settle_vm(uint32_t (&P)[NR], uint32_t& prev)
{
#pragma unroll
    for (int i = 0; i < NR; i++)
        settle_vm1(P[i]);
    settle_vm1(prev);
}

// loads the packed E values of predecessor row p (NR registers) and E_p[jb]
template <int NR>
__device__ __forceinline__ void load_pred_pk(const int16_t* ring, int ring_stride, int ring_mask, const int16_t* spill,
                                             int stride, int r, int p, int jb, uint32_t (&P)[NR], uint32_t& prev)
{
    const int16_t* lrow = ring + (p & ring_mask) * ring_stride + jb + kColShift;
#pragma unroll
    for (int q = 0; q < NR / 4; q++)
    {
        const uint4 v = *reinterpret_cast<const uint4*>(lrow + 1 + 8 * q);
        P[4 * q] = v.x, P[4 * q + 1] = v.y, P[4 * q + 2] = v.z, P[4 * q + 3] = v.w;
    }
    prev = uint32_t(uint16_t(lrow[0]));
    if (p == 0)
    {
#pragma unroll
        for (int i = 0; i < NR; i++)
            P[i] = 0;
        prev = 0;
    }
    else if (r - p > ring_mask)
    {
        const int16_t* grow = spill + size_t(p) * stride + jb + kColShift;
#pragma unroll
        for (int q = 0; q < NR / 4; q++)
        {
            const uint4 v = *reinterpret_cast<const uint4*>(grow + 1 + 8 * q);
            P[4 * q] = v.x, P[4 * q + 1] = v.y, P[4 * q + 2] = v.z, P[4 * q + 3] = v.w;
        }
        prev = uint32_t(uint16_t(grow[0]));
        settle_vm<NR>(P, prev);
    }
}

// diagonal sources E_p[j-1] for the lane's cells: element 2i-1 and 2i
template <int NR>
__device__ __forceinline__ void diag_src(const uint32_t (&P)[NR], uint32_t prev, uint32_t (&Dg)[NR])
{
    Dg[0] = __builtin_amdgcn_alignbyte(P[0], prev << 16, 2);
#pragma unroll
    for (int i = 1; i < NR; i++)
        Dg[i] = __builtin_amdgcn_alignbyte(P[i], P[i - 1], 2);
}

// Diagnostic build only (-DGWAMD_FWD_PROFILE): shader-clock cycles of the
// forward pass sections, stored in place of the backbone/add/topsort/output
// phase slots.
#ifdef GWAMD_FWD_PROFILE
struct FwdProf
{
    uint64_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t m    = 0;
    __device__ void start() { m = __builtin_amdgcn_s_memtime(); }
    template <int I>
    __device__ void lap()
    {
        const uint64_t x = __builtin_amdgcn_s_memtime();
        t[I] += x - m;
        m = x;
    }
};
#define GWAMD_FP_START(fp) fp.start()
#define GWAMD_FP_LAP(fp, I) fp.template lap<I>()
#else
struct FwdProf
{
};
#define GWAMD_FP_START(fp)
#define GWAMD_FP_LAP(fp, I)
#endif

// Lane-parallel predecessor rows of row rr: lane k < n holds the row of
// predecessor slot k.  A source row gets the virtual row 0 as its single
// predecessor (n = 1, row 0), which gives the same column-0 value (gap) and
// the same scores as the reference's source-node case.
template <typename SizeT>
__device__ __forceinline__ int row_preds(const RowProg& P, WinGraph<SizeT> g, int rr, uint32_t rec, int lane,
                                         int& n)
{
    g = as_global(g);
    n      = int((rec >> 8) & 63);
    int pv = 0;
    if (n == int(kRecEscape))
    {
        const int node = uniform(int(g.sorted[rr - 1]));
        n              = uniform(int(g.in_cnt[node]));
        uint32_t t     = lane < n ? uint32_t(pred_row(g, node, lane)) : 0u;
        settle_vm1(t);
        pv = int(t);
    }
    else if (n >= 2)
        pv = lane < n ? int(P.xl[(rec >> 16) + lane]) : 0;
    else if (n == 1)
        pv = rr - int(rec >> 16);
    if (n == 0)
        n = 1;
    return pv;
}

// Forward pass of one read, split over NW waves of the workgroup: wave q owns
// the span of 64*CPL columns starting at cb = q*64*CPL (CPL cells per lane),
// and one sweep covers the read.  The waves are decoupled, not in lockstep:
// wave q needs from wave q-1 only the carry of each row (E_r[cb], the maximum
// over every column left of its span), which wave q-1 posts into a tagged
// LDS channel as soon as its row scan is done; wave q computes its own cells
// of the row before it waits for that word.  The column-0 value of a row is
// the maximum of its predecessors' column-0 values, which lane 0 of wave 0
// loads anyway as the diagonal source of column 1.  The diagonal source of a
// span's first column for predecessor row p is the carry the wave received
// for row p (kept per wave in `bnd`, and in the spill row for far rows).
// The predecessor row r-1 (the common case in Kahn order) comes from
// registers; row r+1's predecessor list and row r+2's record are loaded while
// row r is computed.
template <int NR>
__device__ __forceinline__ void load_row_pk(const int16_t* p, uint32_t (&P)[NR], uint32_t& prev)
{
    if constexpr (NR % 4 == 0)
    {
#pragma unroll
        for (int q = 0; q < NR / 4; q++)
        {
            const uint4 v = *reinterpret_cast<const uint4*>(p + 1 + 8 * q);
            P[4 * q] = v.x, P[4 * q + 1] = v.y, P[4 * q + 2] = v.z, P[4 * q + 3] = v.w;
        }
    }
    else
    {
        static_assert(NR == 2, "4 or a multiple of 8 cells per lane");
        const uint2 v = *reinterpret_cast<const uint2*>(p + 1);
        P[0] = v.x, P[1] = v.y;
    }
    prev = uint32_t(uint16_t(p[0]));
}

template <int CPL, int NW, typename SizeT>
__device__ int nw_forward_lds_pk(WinGraph<SizeT> g, const RowProg& P, int V, const uint8_t* read, int L,
                                 int16_t* ring, int ring_stride, int16_t* spill, int stride, uint8_t* codes,
                                 int code_stride, const Scores sc, GWAMD_LDS uint8_t* shb, int16_t* carry_hbm,
                                 int tid, FwdProf& fp)
{
    g = as_global(g);
    constexpr int NR    = CPL / 2;
    constexpr int kSpan = kWave * CPL;
    const int lane      = tid & (kWave - 1);
    const int wave      = uniform(tid / kWave);
    V                   = uniform(V);
    L                   = uniform(L);
    const int gap       = sc.gap;
    const int s_eq      = sc.match - gap;
    const int s_ne      = sc.mismatch - gap;
    const uint32_t gap2 = pk_bcast(gap);
    const uint32_t one2 = opaque_u32(0x00010001u);
    const uint32_t two2 = opaque_u32(0x00020002u);
    // wave-uniform (an SGPR): P arrives through a flat pointer, and a value
    // first used inside the row loop made the compiler wait for vmcnt(0) --
    // every outstanding code / spill store -- at the top of every row
    const int mask      = uniform(P.ring_mask);
    GWAMD_LDS int* prog          = (GWAMD_LDS int*)(shb + kShProg);
    GWAMD_LDS int16_t* bnd       = (GWAMD_LDS int16_t*)(shb + kShBnd) + wave * (mask + 1);
    GWAMD_LDS uint32_t* chan     = (GWAMD_LDS uint32_t*)(shb + kShChan);
    volatile GWAMD_LDS uint32_t* chan_in  = chan + (wave - 1) * kChanRows; // wave > 0
    volatile GWAMD_LDS uint32_t* chan_out = chan + wave * kChanRows;       // wave < NW-1
    volatile GWAMD_LDS int* prog_v        = prog;
    // owner of the last column (L-1): span, lane, cell
    const int jl        = L > 0 ? L - 1 : 0;
    const int own_span  = jl / kSpan;
    const int own_lane  = (jl % kSpan) / CPL;
    const int own_c     = jl % CPL;
    const int nspan     = max(1, (L + kSpan - 1) / kSpan);
    const int nsweep    = (nspan + NW - 1) / NW;
    int best_row        = 0;
    int best_val        = INT_MIN;
    for (int sweep = 0; sweep < nsweep; sweep++)
    {
    if (sweep > 0)
    {
        // channels restart empty; the previous sweep's carries are in HBM
        __syncthreads();
        for (int t = tid; t < (kShChan - kShProg) / 4 + (NW - 1) * kChanRows; t += kWave * NW)
            reinterpret_cast<GWAMD_LDS int*>(shb + kShProg)[t] = 0;
        __syncthreads();
    }
    const int span      = sweep * NW + wave;
    const int cb        = span * kSpan;
    const bool first    = span == 0;                // holds column 0
    const bool wact     = cb < L || first;
    const bool feed     = wave + 1 < NW && cb + kSpan < L;  // next span, same sweep
    const bool to_hbm   = wave == NW - 1 && cb + kSpan < L; // next span, next sweep
    const bool from_hbm = wave == 0 && sweep > 0;
    const bool owner    = span == own_span;
    const int jb        = cb + lane * CPL;
    const bool active   = jb < L;
    const int ja        = active ? jb : 0; // address used by inactive lanes
    if (wact && V >= 1)
    {
        // per-read substitution profiles for A, C, G, T
        uint32_t sig_acgt[4][NR];
#pragma unroll
        for (int i = 0; i < NR; i++)
        {
            const int c0 = int(read[ja + 2 * i]), c1 = int(read[ja + 2 * i + 1]);
            const char bases[4] = {'A', 'C', 'G', 'T'};
#pragma unroll
            for (int b = 0; b < 4; b++)
                sig_acgt[b][i] = uint32_t(uint16_t(c0 == bases[b] ? s_eq : s_ne)) |
                                 (uint32_t(uint16_t(c1 == bases[b] ? s_eq : s_ne)) << 16);
        }
        uint32_t Eprev[NR]; // final E of row r-1 (row 0: zeros)
#pragma unroll
        for (int i = 0; i < NR; i++)
            Eprev[i] = 0;
        int cin_prev = 0;
        int hbm_c    = 0; // carries of 64 rows from the previous sweep, one per lane
        // software pipeline: predecessor rows of
        // rows r and r+1, records of rows r+1 and r+2; row r issues the loads
        // of row r+2's predecessors and row r+3's record
        uint32_t rec_c = uniform(int(P.rec[1]));
        uint32_t rec_a = uniform(int(P.rec[min(2, V)]));
        uint32_t rec_b = uniform(int(P.rec[min(3, V)]));
        int np_c, np_a = 1;
        int pv_c       = row_preds<SizeT>(P, g, 1, rec_c, lane, np_c);
        int pv_a       = V >= 2 ? row_preds<SizeT>(P, g, 2, rec_a, lane, np_a) : 0;
        uint8_t* crow  = codes + code_stride;
        int16_t* srow  = spill + stride;
        for (int r = 1; r <= V; r++, crow += code_stride, srow += stride)
        {
            GWAMD_FP_START(fp);
            int np_b = 1, pv_b = 0;
            if (r + 2 <= V)
                pv_b = row_preds<SizeT>(P, g, r + 2, rec_b, lane, np_b);
            const uint32_t rec_bb = P.rec[min(r + 3, V)];
            GWAMD_FP_LAP(fp, 4);

            const uint32_t rec = rec_c;
            const int np       = np_c;
            const int pv       = pv_c;
            const int base     = row_base<SizeT>(g, rec, r); // bit 7: general-path flag (build_row_program)
            const bool spill_r = (rec >> 15) & 1;
            int16_t* row       = ring + (r & mask) * ring_stride;
            const bool anyfar  = __builtin_amdgcn_ballot_w64(lane < np && pv != 0 && r - pv > mask) != 0;
            uint32_t sig[NR];
            // 'A' 'C' 'G' 'T' are bits 1, 3, 7, 20 of 0x40..0x7f; (base >> 1) & 3
            // gives A 0, C 1, T 2, G 3 (branch-free, a few scalar ops)
            const uint32_t ub = uint32_t(base);
            if ((ub & 0xc0u) == 0x40u && ((0x10008aull >> (ub & 0x3fu)) & 1u))
            {
                // bitwise selects (a select between the profile arrays would
                // index them dynamically, i.e. through scratch)
                const uint32_t bcode = (ub >> 1) & 3u;
                const uint32_t m1    = opaque_u32(((bcode ^ (bcode >> 1)) & 1u) ? ~0u : 0u); // C or T
                const uint32_t m2    = opaque_u32((bcode >> 1) ? ~0u : 0u);                  // G or T
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    const uint32_t lo = (sig_acgt[1][i] & m1) | (sig_acgt[0][i] & ~m1);
                    const uint32_t hi = (sig_acgt[3][i] & m1) | (sig_acgt[2][i] & ~m1);
                    sig[i]            = (hi & m2) | (lo & ~m2);
                }
            }
            else
            {
                const uint32_t* rw = reinterpret_cast<const uint32_t*>(read + ja);
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    const uint32_t wv = rw[i / 2] >> ((i & 1) * 16);
                    const int ch0 = int(wv & 0xff), ch1 = int((wv >> 8) & 0xff);
                    sig[i]        = uint32_t(uint16_t(ch0 == base ? s_eq : s_ne)) |
                             (uint32_t(uint16_t(ch1 == base ? s_eq : s_ne)) << 16);
                }
            }
            GWAMD_FP_LAP(fp, 5);
            // E values of predecessor row p for the lane's cells, and E_p[jb]
            auto load_pred = [&](int p, uint32_t(&Q)[NR], uint32_t& qprev) {
                if (p == r - 1)
                {
#pragma unroll
                    for (int i = 0; i < NR; i++)
                        Q[i] = Eprev[i];
                    qprev = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(uint16_t(cin_prev))),
                                                                 int(Eprev[NR - 1] >> 16), 0x138, 0xf, 0xf, false));
                }
                else if (p == 0)
                {
#pragma unroll
                    for (int i = 0; i < NR; i++)
                        Q[i] = 0;
                    qprev = 0;
                }
                else if (anyfar && r - p > mask)
                {
                    load_row_pk<NR>(spill + size_t(p) * stride + ja + kColShift, Q, qprev);
                    settle_vm<NR>(Q, qprev);
                }
                else
                {
                    load_row_pk<NR>(ring + (p & mask) * ring_stride + ja + kColShift, Q, qprev);
                    {
                        const uint32_t bv = uint32_t(uint16_t(bnd[p & mask]));
                        if (lane == 0 && cb > 0)
                            qprev = bv;
                    }
                }
            };
            uint32_t dg[NR], vt[NR], kd[NR], kv[NR], E[NR];
            int c0v, c0kv = 0;
            {
                uint32_t Pv[NR], prev;
                load_pred(__builtin_amdgcn_readfirstlane(pv), Pv, prev);
                c0v = int(int16_t(prev)); // wave 0, lane 0: E_p[0]
                diag_src<NR>(Pv, prev, dg);
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    dg[i] = pk_add(dg[i], sig[i]);
                    vt[i] = pk_add(Pv[i], gap2);
                }
            }
            GWAMD_FP_LAP(fp, 6);
            // in-lane prefix maximum: per register pair max(diag, vertical),
            // then its low half into its high half, then the previous pair's
            // high half into both (op_sel forms, no shifts or permutes)
            auto prefix = [&]() {
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    const uint32_t s = pk_max_lo_into_hi(pk_max(dg[i], vt[i]));
                    E[i]             = i == 0 ? s : pk_max_hi_carry(s, E[i - 1]);
                }
            };
            if (np > 1)
            {
                // rows with several predecessors track the first maximising
                // slot of each cell, pre-scaled to the code layout: kd = 4 *
                // slot, kv = 4 * slot + 1 (codes: 0 diagonal, 1 vertical,
                // 2 horizontal, + slot << 2)
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    kd[i] = 0;
                    kv[i] = one2;
                }
                for (int k = 1; k < np; k++)
                {
                    uint32_t Q[NR], qprev, dq[NR];
                    load_pred(__builtin_amdgcn_readlane(pv, k), Q, qprev);
                    {
                        // column 0: first maximising predecessor slot
                        const int pe = int(int16_t(qprev));
                        c0kv         = pe > c0v ? k : c0kv;
                        c0v          = max(c0v, pe);
                    }
                    diag_src<NR>(Q, qprev, dq);
                    const uint32_t kk4 = pk_bcast(4 * k);
                    const uint32_t kk1 = pk_bcast(4 * k + 1);
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        // running maxima with the first maximising predecessor slot
                        const uint32_t d  = pk_add(dq[i], sig[i]);
                        const uint32_t nd = pk_max(dg[i], d);
                        kd[i]             = pk_mad(pk_min_u(pk_sub(nd, dg[i]), one2), pk_sub(kk4, kd[i]), kd[i]);
                        dg[i]             = nd;
                        const uint32_t v  = pk_add(Q[i], gap2);
                        const uint32_t nv = pk_max(vt[i], v);
                        kv[i]             = pk_mad(pk_min_u(pk_sub(nv, vt[i]), one2), pk_sub(kk1, kv[i]), kv[i]);
                        vt[i]             = nv;
                    }
                }
                prefix();
            }
            else
                prefix();
            const int m    = active ? int(int16_t(E[NR - 1] >> 16)) : kNeg;
            GWAMD_FP_LAP(fp, 0);
            const int incl = wave_incl_max_dpp(m);
            const int excl = __builtin_amdgcn_update_dpp(kNeg, incl, 0x138, 0xf, 0xf, false);
            const int wtot = __builtin_amdgcn_readlane(incl, kWave - 1);
            int cin;
            if (first)
            {
                cin           = __builtin_amdgcn_readfirstlane(c0v) + gap; // column 0
                const int c0k = __builtin_amdgcn_readfirstlane(c0kv);
                if (lane == 0)
                {
                    row[kColShift]  = int16_t(cin);
                    crow[kColShift] = uint8_t(1 | (c0k << 2));
                    if (spill_r)
                        srow[kColShift] = int16_t(cin);
                }
            }
            else
            {
                if (from_hbm)
                {
                    // carry of this row from the previous sweep's last span
                    if (((r - 1) & (kWave - 1)) == 0)
                    {
                        const int x = r + lane;
                        uint32_t hc = x <= V ? uint32_t(int(carry_hbm[x])) : 0u;
                        settle_vm1(hc); // wait here, once per 64 rows, not at every row's readlane
                        hbm_c = int(hc);
                    }
                    cin = int(int16_t(__builtin_amdgcn_readlane(hbm_c, (r - 1) & (kWave - 1))));
                }
                else
                {
                    // carry of this row from the previous span
                    uint32_t w = uint32_t(uniform(int(chan_in[r & (kChanRows - 1)])));
                    while ((w >> 16) != (uint32_t(r) & 0xffffu))
                    {
                        __builtin_amdgcn_s_sleep(1);
                        w = uint32_t(uniform(int(chan_in[r & (kChanRows - 1)])));
                    }
                    cin = int(int16_t(w & 0xffffu));
                    if ((r & 7) == 0 && lane == 0)
                        prog_v[wave] = r;
                }
                if (lane == 0)
                {
                    bnd[r & mask] = int16_t(cin);
                    if (spill_r)
                        srow[cb + kColShift] = int16_t(cin); // same value as the previous span's last cell
                }
            }
            GWAMD_FP_LAP(fp, 1);
            if (feed)
            {
                // flow control: the consumer must have taken row r-kChanRows+32
                if ((r & 31) == 0 && r >= kChanRows)
                {
                    while (uniform(prog_v[wave + 1]) < r - 32)
                        __builtin_amdgcn_s_sleep(1);
                }
                if (lane == 0)
                    chan_out[r & (kChanRows - 1)] = (uint32_t(r) << 16) | uint32_t(uint16_t(max(cin, wtot)));
            }
            if (to_hbm && lane == 0)
                carry_hbm[r] = int16_t(max(cin, wtot));
            GWAMD_FP_LAP(fp, 2);
            const uint32_t b2v = pk_bcast(max(excl, cin));
#pragma unroll
            for (int i = 0; i < NR; i++)
                E[i] = pk_max(E[i], b2v);
            if (active)
            {
                // codes: 0 diagonal, 1 vertical, 2 horizontal (+ slot << 2)
                uint32_t code[NR];
                if (np > 1)
                {
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        const uint32_t a   = pk_min_u(pk_sub(E[i], dg[i]), one2); // 0: diagonal match
                        const uint32_t bb  = pk_min_u(pk_sub(E[i], vt[i]), one2); // 0: vertical match
                        const uint32_t cvh = pk_mad(bb, pk_sub(two2, kv[i]), kv[i]); // vertical or horizontal
                        code[i]            = pk_mad(a, pk_sub(cvh, kd[i]), kd[i]);
                    }
                }
                else
                {
                    // one predecessor (slot 0): a * (1 + bb)
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        const uint32_t a  = pk_min_u(pk_sub(E[i], dg[i]), one2);
                        const uint32_t bb = pk_min_u(pk_sub(E[i], vt[i]), one2);
                        code[i]           = pk_mad(a, bb, a);
                    }
                }
                if constexpr (NR % 4 == 0)
                {
#pragma unroll
                    for (int q = 0; q < NR / 4; q++)
                    {
                        const uint4 ev = make_uint4(E[4 * q], E[4 * q + 1], E[4 * q + 2], E[4 * q + 3]);
                        *reinterpret_cast<uint4*>(row + jb + kColShift + 1 + 8 * q) = ev;
                        if (spill_r)
                            *reinterpret_cast<uint4*>(srow + jb + kColShift + 1 + 8 * q) = ev;
                        const uint32_t w0 = __builtin_amdgcn_perm(code[4 * q + 1], code[4 * q], 0x06040200u);
                        const uint32_t w1 = __builtin_amdgcn_perm(code[4 * q + 3], code[4 * q + 2], 0x06040200u);
                        __builtin_nontemporal_store(uint64_t(w0) | (uint64_t(w1) << 32),
                                                    reinterpret_cast<uint64_t*>(crow + jb + kColShift + 1 + 8 * q));
                    }
                }
                else
                {
                    // 4 cells per lane: 8-byte E stores, one 4-byte code word
                    const uint2 ev = make_uint2(E[0], E[1]);
                    *reinterpret_cast<uint2*>(row + jb + kColShift + 1) = ev;
                    if (spill_r)
                        *reinterpret_cast<uint2*>(srow + jb + kColShift + 1) = ev;
                    __builtin_nontemporal_store(__builtin_amdgcn_perm(code[1], code[0], 0x06040200u),
                                                reinterpret_cast<uint32_t*>(crow + jb + kColShift + 1));
                }
            }
            if ((rec & (1u << 14)) && owner)
            {
                // sink row: E at the last column (column 0 for an empty read)
                int endv = cin;
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    if (2 * i == own_c)
                        endv = int(int16_t(E[i] & 0xffff));
                    if (2 * i + 1 == own_c)
                        endv = int(int16_t(E[i] >> 16));
                }
                const int v = L == 0 ? cin : __builtin_amdgcn_readlane(endv, own_lane);
                if (best_val < v)
                    best_val = v, best_row = r;
            }
#pragma unroll
            for (int i = 0; i < NR; i++)
                Eprev[i] = E[i];
            cin_prev = cin;
            rec_c    = rec_a;
            np_c     = np_a;
            pv_c     = pv_a;
            rec_a    = rec_b;
            np_a     = np_b;
            pv_a     = pv_b;
            rec_b    = uniform(int(rec_bb));
            GWAMD_FP_LAP(fp, 3);
        }
    }
    } // sweeps
    if (nsweep > 1 || NW > 1)
    {
        // publish the end row from the wave that owns the last column
        GWAMD_LDS int* endp = (GWAMD_LDS int*)(shb + kShEnd);
        if (wave == own_span % NW && lane == 0)
            *endp = best_row;
        __syncthreads();
        best_row = uniform(*endp);
    }
    return best_row;
}

// Traceback over the code matrix, run by one wave (lane-uniform walk; code
// tiles of 128 rows x 128 columns staged in LDS).  The tile code and the row
// record are loaded together, so a step waits for at most two LDS round trips
// (code/record, then a predecessor list).  Emitted pairs (node id or -1, read
// position or -1; reversed, as the reference's traceback,
// cudapoa_nw.cuh:361-452) are collected one per lane and stored 64 at a time;
// rows become node ids at the store.
template <typename SizeT>
__device__ int traceback_codes(WinGraph<SizeT> g, const RowProg& P, int V, int L, int end_row,
                               const uint8_t* codes_f, int code_stride, uint8_t* tile_f, SizeT* ag_f, SizeT* ar_f,
                               int aln_cap, int lane, bool rank, int tbmode)
{
    g = as_global(g);
    // typed pointers: this function is called, not inlined (lds_of)
    const GWAMD_GLB uint8_t* codes = glb_of(codes_f);
    GWAMD_LDS uint8_t* tile        = lds_of(tile_f);
    GWAMD_GLB SizeT* ag            = glb_of(ag_f);
    GWAMD_GLB SizeT* ar            = glb_of(ar_f);
    const GWAMD_LDS uint32_t* prec = lds_of(P.rec);
    const GWAMD_LDS uint16_t* pxl  = lds_of(P.xl);

    V       = uniform(V);
    L       = uniform(L);
    int i   = uniform(end_row), j = L;
    int ti0 = INT_MIN / 2, tj0 = INT_MIN / 2;
    int n = 0, loops = 0;
    const int bound = L + V + 2;
    int eg = 0, er = 0; // lane (n & 63) holds pair n until it is stored
    auto flush = [&](int upto) {
        // pairs [upto & ~63, upto) are held by lanes 0 .. (upto-1) & 63
        const int base = (upto - 1) & ~(kWave - 1);
        const int k    = base + lane;
        if (k < upto && k < aln_cap)
        {
            ag[k] = SizeT(eg > 0 ? int(g.sorted[eg - 1]) : -1);
            ar[k] = SizeT(er);
        }
    };
    auto load_tile = [&](int ii, int cj) {
        ti0 = max(0, ii - (kTileRows - 1));
        tj0 = max(0, cj - (kTileCols - 16)) & ~15;
        wave_sync();
        // 16 loads per lane, issued 8 at a time before any is waited for
        constexpr int kPer = kTileRows * (kTileCols / 16) / kWave;
        constexpr int kB   = 8;
#pragma unroll
        for (int b0 = 0; b0 < kPer; b0 += kB)
        {
            u32x4 v[kB];
#pragma unroll
            for (int u = 0; u < kB; u++)
            {
                const int t   = (b0 + u) * kWave + lane;
                const int tr  = t / (kTileCols / 16);
                const int tc  = (t % (kTileCols / 16)) * 16;
                const int rr  = ti0 + tr;
                const bool ok = rr <= V && tj0 + tc + 16 <= code_stride;
                v[u] = *reinterpret_cast<const GWAMD_GLB u32x4*>(codes + size_t(ok ? rr : 0) * code_stride +
                                                                 (ok ? tj0 + tc : 0));
                v[u] = ok ? v[u] : u32x4{0, 0, 0, 0};
            }
#pragma unroll
            for (int u = 0; u < kB; u++)
            {
                const int t  = (b0 + u) * kWave + lane;
                const int tr = t / (kTileCols / 16);
                const int tc = (t % (kTileCols / 16)) * 16;
                *reinterpret_cast<GWAMD_LDS u32x4*>(tile + tr * kTileCols + tc) = v[u];
            }
        }
        wave_sync();
    };
    // Move window (TbWin, as in the banded traceback, poa_band.hip): the moves
    // of 128 cells decoded in one lane-parallel pass, two cells per lane,
    // packed (row << 16 | column), then walked.  Cells outside the tile or
    // with escaped predecessor lists are kSlow and take the general step.
    constexpr uint32_t kSlow = 0xffffffffu;
    const bool win_ok        = V < 65535 && L < 65535;
    TbWin G;
    G.init(tbmode, i, L, kTileRows);
    uint32_t wpk0 = kSlow, wpk1 = kSlow;
    auto decode_cell = [&](int t) -> uint32_t {
        const int r  = G.row(t);
        const int c  = G.col(t);
        const int cj = c + kColShift;
        uint32_t res = kSlow;
        if (r >= 1 && c >= 0 && r >= ti0 && r < ti0 + kTileRows && cj >= tj0 && cj < tj0 + kTileCols)
        {
            const int code     = int(tile[(r - ti0) * kTileCols + (cj - tj0)]);
            const uint32_t rec = prec[r];
            const int dir      = code & 3;
            const int np       = int((rec >> 8) & 63);
            const int pj       = dir == 1 ? c : c - 1;
            if (pj < 0)
                res = kSlow;
            else if (dir == 2)
                res = (uint32_t(r) << 16) | uint32_t(pj);
            else if (np != int(kRecEscape))
            {
                const int p = np == 0 ? 0 : (np == 1 ? r - int(rec >> 16) : int(pxl[(rec >> 16) + (code >> 2)]));
                res         = (uint32_t(p) << 16) | uint32_t(pj);
            }
        }
        return res;
    };
    while (!(i == 0 && j == 0) && loops < bound)
    {
        i     = uniform(i);
        j     = uniform(j);
        n     = uniform(n);
        loops = uniform(loops);
        ti0   = uniform(ti0);
        tj0   = uniform(tj0);
        G.wi0   = uniform(G.wi0);
        G.wj0   = uniform(G.wj0);
        G.slope = uniform(G.slope);
        G.next  = uniform(G.next);
        if (win_ok && i >= 1)
        {
            if (G.index(i, j) < 0)
            {
                G.refill(i, j);
                const int cj = j + kColShift;
                if (i < ti0 || i >= ti0 + kTileRows || cj < tj0 || cj >= tj0 + kTileCols ||
                    (i - G.row_span() < ti0 && ti0 > 0) || (cj - G.col_span() < tj0 && tj0 > 0))
                    load_tile(i, cj);
                wpk0  = decode_cell(lane);
                wpk1  = decode_cell(lane + kWave);
            }
            // walk the window: every value here is wave-uniform (SGPRs)
            int ci = i, cj = j, cn = n, cl = loops;
            if (rank)
                walk_window_ranked<0>(wpk0, wpk1, G, ci, cj, cn, cl, bound, lane, eg, er,
                                      tile + kTileRows * kTileCols, flush);
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
                if ((ci == 0 && cj == 0) || cl >= bound || ci < 1 || G.index(ci, cj) < 0)
                    break;
            }
            if (cl != loops)
            {
                G.follow(ci, cj);
                i     = ci;
                j     = cj;
                n     = cn;
                loops = cl;
                continue;
            }
        }
        loops++;
        int pi, pj;
        if (i == 0)
        {
            pi = 0;
            pj = j - 1;
        }
        else
        {
            const int cj = j + kColShift;
            if (i < ti0 || i >= ti0 + kTileRows || cj < tj0 || cj >= tj0 + kTileCols)
                load_tile(i, cj);
            const int code_v   = int(tile[(i - ti0) * kTileCols + (cj - tj0)]);
            const int rec_v    = int(prec[i]);
            const int code     = uniform(code_v);
            const uint32_t rec = uint32_t(uniform(rec_v));
            const int dir      = code & 3;
            if (dir == 2)
            {
                pi = i;
                pj = j - 1;
            }
            else
            {
                const int np = int((rec >> 8) & 63), k = code >> 2;
                pi = np == 0 ? 0
                             : (np == 1 ? i - int(rec >> 16)
                                        : (np == int(kRecEscape) ? uniform(pred_row(g, int(g.sorted[i - 1]), k))
                                                                 : uniform(int(pxl[(rec >> 16) + k]))));
                pj = dir == 0 ? j - 1 : j;
            }
        }
        if (lane == (n & (kWave - 1)))
        {
            eg = i == pi ? -1 : i;
            er = j == pj ? -1 : j - 1;
        }
        n++;
        if ((n & (kWave - 1)) == 0)
            flush(n);
        i = pi;
        j = pj;
    }
    if ((n & (kWave - 1)) != 0)
        flush(n);
    wave_sync();
    if (loops >= bound || n > aln_cap)
        return -1;
    return n;
}

#include "poa_fwd2.hpp"
#include "poa_fwd_w.hpp"

// LDS-resident POA kernel: one workgroup of NW waves per window.  The forward
// pass, the traceback tile loads and the level-keyed topological sort use
// every wave; the serial phases (graph update, consensus, MSA) run on wave 0
// while the other waves wait at the next barrier.  W: 32-bit scores (nw_forward_lds_w, the
// reference's use32bitScore batches), else 16-bit.  Two waves per window
// (config B: four windows per CU, two waves per SIMD) need the kernel within
// 256 registers; it is (252 with the per-kernel level sort instance), and a
// second launch bound of 2 to force it costs config B 4% (the traceback
// phase 5.8 -> 8.1 ms per window, same traceback code), so it is not set.
template <bool MSA, int CPL, int NW, bool W>
__global__ void __launch_bounds__(kWave * NW, W ? (NW >= 8 ? 2 : 1) : (NW >= 4 ? 2 : 1))
    poa_window_kernel_lds(Buffers b, Dims d, Scores sc)
{
    using SizeT  = int16_t;
    using RowT   = typename std::conditional<W, int32_t, int16_t>::type; // E-domain row element
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int sh_status;
    __shared__ int sh_len;

    __shared__ int sh_next;
    if (int(blockIdx.x) >= b.num_windows)
        return;
    const int tid      = threadIdx.x;
    const int lane     = tid & (kWave - 1);
    const int wave     = uniform(tid / kWave);
    constexpr int kThr = kWave * NW;
    const size_t slot  = blockIdx.x; // scratch slot (grid <= slots)

    uint8_t* lread   = lds;
    RowT* ring       = reinterpret_cast<RowT*>(lds + d.lds_ring_off);
    uint8_t* tile    = lds + d.lds_ring_off; // traceback tiles reuse the ring
    const int rstride = d.score_stride;      // ring / spill row stride (elements)
    GWAMD_LDS uint8_t* shb = (GWAMD_LDS uint8_t*)(lds) + d.lds_sh_off;
    AddScratch AX;
    {
        // add-alignment scratch lives in the ring region (free between reads)
        GWAMD_LDS uint8_t* a = (GWAMD_LDS uint8_t*)(lds) + d.lds_ring_off;
        const int ms         = (d.max_seq_len + 16) & ~15;
        AX.gid               = (GWAMD_LDS uint16_t*)(a);
        AX.curr              = (GWAMD_LDS uint16_t*)(a + 2 * ms);
        AX.kind              = a + 4 * ms;
        AX.owner             = (GWAMD_LDS uint16_t*)(a + 5 * ms);
        AX.sh                = (GWAMD_LDS int*)(shb);
    }

    for (int idx = blockIdx.x; idx < b.num_windows;)
    {
    const int w     = b.order ? b.order[idx] : idx;
    const size_t mn = size_t(d.max_nodes);
    WinGraph<SizeT> g;
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

    SizeT* ag        = static_cast<SizeT*>(b.ag) + slot * d.aln_cap;
    SizeT* ar        = static_cast<SizeT*>(b.ar) + slot * d.aln_cap;
    RowT* spill      = static_cast<RowT*>(b.scores) + slot * d.score_rows * size_t(rstride);
    uint8_t* codes   = b.codes + slot * size_t(d.aux_stride);
    uint32_t* rec    = reinterpret_cast<uint32_t*>(lds + d.lds_rec_off);
    uint16_t* xl     = reinterpret_cast<uint16_t*>(lds + d.lds_xl_off);
    RowT* carry      = reinterpret_cast<RowT*>(codes + d.aux_carry_off);
    RowProg P{rec, xl, d.lds_ring_rows - 1};
    int32_t* cscore  = b.cscore + slot * mn;
    SizeT* cpred     = static_cast<SizeT*>(b.cpred) + slot * mn * 4;
    uint16_t* ecov   = MSA ? b.edge_cov + w * mn * kMaxEdges * d.max_seqs : nullptr;
    uint16_t* ecovc  = MSA ? b.edge_cov_cnt + w * mn * kMaxEdges : nullptr;
    SizeT* seq_begin = MSA ? static_cast<SizeT*>(b.seq_begin) + size_t(w) * d.max_seqs : nullptr;

    PhaseTimer ph;
    FwdProf fp;
    // round-4 forward pass unless the scores do not fit its byte table (or
    // Dims::diag bit 1, GWAMD_POA_FWD=v1 under GWAMD_DIAG, asks for round 3's)
#ifdef GWAMD_FWD_PROFILE
    const bool use_v2 = false;
#else
    const bool use_v2 = !W && fwd2_ok(sc) && !(d.diag & 2);
#endif
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
        if (wave == 0)
            build_backbone<SizeT, MSA>(g, seq0, w0, len0, lane, ecov, ecovc, seq_begin, d.max_seqs);
        node_count = len0;
        ph.lap<kPhBackbone>();
        for (int s = 1; s < nseq; s++)
        {
            if (node_count >= d.max_nodes)
            {
                status = kNodeCountExceeded;
                break;
            }
            const int L           = b.seq_len[wd.first_seq + s];
            const int64_t off     = b.seq_off[wd.first_seq + s];
            const uint8_t* read_g = b.seqs + off;
            const int8_t* wts_g   = b.wts + off;
            const int padded      = (L + 32 + 15) & ~15;
            for (int j = tid; j < padded; j += kThr)
                lread[j] = j < L ? read_g[j] : 0;
            const int V = node_count;
            if (wave == 0) // spill flags in the ring region (free until the forward pass)
                build_row_program<SizeT>(g, V, rec, xl, d.lds_xl_cap, d.lds_ring_rows, lane,
                                         (GWAMD_LDS uint8_t*)(lds) + d.lds_ring_off);
            if (NW > 1)
            {
                // forward-pass channels and progress words start empty
                constexpr int kP = W ? kShProgW : kShProg;
                constexpr int kB = W ? kShBytesW(NW) : kShBytes(NW);
                for (int t = tid; t < (kB - kP) / 4; t += kThr)
                    reinterpret_cast<GWAMD_LDS int*>(shb + kP)[t] = 0;
            }
            __syncthreads();
            ph.lap<kPhRowProg>();
            cells += int64_t(V + 1) * (L + 1);
            int end_row;
            // (the diagnostic 24- and 32-column shapes keep the round-3 pass)
            if constexpr (W)
                end_row = nw_forward_lds_w<CPL, NW, SizeT>(g, P, V, lread, L, ring, rstride, spill, rstride, codes,
                                                           d.code_stride, sc, shb, carry, tid);
            else if constexpr (CPL <= 16)
                end_row = use_v2 ? nw_forward_lds_v2<CPL, NW, SizeT>(g, P, V, lread, L, ring, rstride, spill, rstride,
                                                                     codes, d.code_stride, sc, shb, carry, tid,
                                                                     d.lds_xl_cap)
                                 : nw_forward_lds_pk<CPL, NW, SizeT>(g, P, V, lread, L, ring, rstride, spill, rstride,
                                                                     codes, d.code_stride, sc, shb, carry, tid, fp);
            else
                end_row = nw_forward_lds_pk<CPL, NW, SizeT>(g, P, V, lread, L, ring, rstride, spill, rstride, codes,
                                                            d.code_stride, sc, shb, carry, tid, fp);
            __syncthreads();
            ph.lap<kPhForward>();
            if (wave == 0)
            {
                const int alen_w = traceback_codes<SizeT>(g, P, V, L, end_row, codes, d.code_stride, tile, ag, ar,
                                                          d.aln_cap, lane, (d.tb_rank & 1) != 0,
                                                          d.tb_rank);
                if (lane == 0)
                    sh_len = alen_w;
            }
            __syncthreads();
            const int alen = uniform(sh_len);
            __syncthreads();
            ph.lap<kPhTraceback>();
            if (alen == -1)
            {
                status = kLoopCountExceeded;
                break;
            }
            if (wave == 0)
            {
                int nc = node_count;
                int rc = add_alignment_parallel<SizeT, MSA>(g, nc, ag, ar, alen, L, lread, wts_g, s, ecov, ecovc,
                                                             seq_begin, d.max_seqs, AX, lane);
                if (rc < 0)
                {
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
                if (lane == 0)
                {
                    sh_status = rc;
                    sh_len    = nc;
                }
            }
            __syncthreads();
            int rc       = uniform(sh_status);
            int nc       = uniform(sh_len);
            bool lv_done = false;
            __syncthreads(); // sh_* are rewritten below
            // level-keyed Kahn sort on every wave of the workgroup
            // (GWAMD_TOPSORT=fifo, Dims::diag bit 2, keeps the FIFO below)
            if (rc == kSuccess && !d.spoa_accurate && !(d.diag & 4))
                lv_done = topsort_levels<SizeT, NW>(g, nc, V, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, tid, kThr,
                                                    cpred, lv_hint);
            lv_hint = lv_done ? nc : 0; // cpred holds c(v) of this sort for the next one
            if (wave == 0)
            {
                if (rc == kSuccess && !lv_done)
                {
                    if (d.spoa_accurate)
                        rc = topsort_racon_wave<SizeT>(g, nc, cscore, cpred, 4 * d.max_nodes, lane,
                                                       (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off);
                    // scratch: the read and the ring (both free after the add)
                    else if (!topsort_lds<SizeT>(g, nc, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, AX.sh, lane, nullptr,
                                                       (d.diag & 1) != 0) &&
                             !topsort_lds_big<SizeT>(g, nc, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, lane))
                    {
                        if (lane == 0)
                            topsort_kahn<SizeT>(g, nc, cscore);
                        wave_sync();
                    }
                }
                ph.lap<kPhTopsort>();
                wave_sync();
                if (lane == 0)
                {
                    sh_status = rc;
                    sh_len    = nc;
                }
            }
            __syncthreads();
            status     = uniform(sh_status); // LDS values: tell the compiler they are wave-uniform
            node_count = uniform(sh_len);
            __syncthreads(); // sh_* are rewritten by the next read
            if (status != kSuccess)
                break;
        }
    }
    if (wave == 0)
    {
        finish_window<SizeT, MSA>(b, d, w, lane, g, status, nseq, node_count, cscore, cpred, ecov, ecovc, seq_begin,
                                  sh_len, sh_status, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off);
        ph.lap<kPhOutput>();
        if (lane == 0)
        {
            if (b.phase)
            {
                ph.store(b.phase + size_t(w) * kPhases);
#ifdef GWAMD_FWD_PROFILE
                // cycles / 1000 so the 100 MHz tick scaling reads as kcycles*1e-5
                const int slot[8] = {kPhBackbone, kPhAdd, kPhTopsort, kPhOutput, kPhForward, kPhTraceback, kPhRowProg,
                                     kPhTotal};
                for (int i = 0; i < 8; i++)
                    b.phase[size_t(w) * kPhases + slot[i]] = int64_t(fp.t[i]);
#endif
            }
            b.final_nodes[w] = node_count;
            b.cells[w]       = cells;
        }
    }
#if defined(GWAMD_FWD_PROFILE) && defined(GWAMD_FWD_PROFILE_WAVE)
    // diagnostic: another wave's section timers replace wave 0's
    __syncthreads();
    if (wave == GWAMD_FWD_PROFILE_WAVE && lane == 0 && b.phase)
    {
        const int slot[8] = {kPhBackbone, kPhAdd, kPhTopsort, kPhOutput, kPhForward, kPhTraceback, kPhRowProg,
                             kPhTotal};
        for (int i = 0; i < 8; i++)
            b.phase[size_t(w) * kPhases + slot[i]] = int64_t(fp.t[i]);
    }
#endif
    if (b.head == nullptr)
        break;
    // next queue position; the LDS image is rewritten by the next window
    __syncthreads();
    if (tid == 0)
        sh_next = b.num_slots + atomicAdd(b.head, 1);
    __syncthreads();
    idx = uniform(sh_next);
    }
}

// Test hook: the level-keyed Kahn sort (topsort_levels) of one graph by one
// workgroup, for the known-answer and random-DAG tests against the FIFO sort.
template <typename SizeT>
__global__ void __launch_bounds__(1024) topsort_levels_test_kernel(WinGraph<SizeT> g, int n, int n_prev, int scratch,
                                                                   SizeT* hint, int n_hint, int* ok, uint64_t* prof)
{
    extern __shared__ __align__(16) uint8_t lds[];
#ifdef GWAMD_TOPSORT_PROFILE
    uint64_t p[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    const bool r = topsort_levels<SizeT>(g, n, n_prev, (GWAMD_LDS uint8_t*)(lds), scratch, int(threadIdx.x),
                                         int(blockDim.x), hint, n_hint, p);
    if (threadIdx.x == 0 && prof)
        for (int k = 0; k < 10; k++)
            prof[k] += p[k];
#else
    const bool r = topsort_levels<SizeT>(g, n, n_prev, (GWAMD_LDS uint8_t*)(lds), scratch, int(threadIdx.x),
                                         int(blockDim.x), hint, n_hint);
    (void)prof;
#endif
    if (threadIdx.x == 0)
        *ok = r ? 1 : 0;
}

template <typename SizeT>
int topsort_levels_test(int n, int n_prev, int n_hint, const uint16_t* in_cnt, const int32_t* in_e,
                        const uint16_t* out_cnt, const int32_t* out_e, int32_t* hint, const int32_t* order_prev,
                        int threads, int scratch, int32_t* sorted, int reps = 0, double* ms = nullptr,
                        uint64_t* prof_out = nullptr)
{
    const size_t ne = size_t(n) * kMaxEdges;
    std::vector<SizeT> ie(ne), oe(ne), hi(n, SizeT(0));
    for (size_t i = 0; i < ne; i++)
    {
        ie[i] = SizeT(in_e[i]);
        oe[i] = SizeT(out_e[i]);
    }
    for (int v = 0; hint && v < n; v++)
        hi[v] = SizeT(hint[v]);
    uint16_t *d_ic = nullptr, *d_oc = nullptr;
    SizeT *d_ie = nullptr, *d_oe = nullptr, *d_sorted = nullptr, *d_pos = nullptr, *d_hint = nullptr;
    int* d_ok   = nullptr;
    uint64_t* d_prof = nullptr;
    int ok      = 0;
    auto fin    = [&](int r) {
        (void)hipFree(d_ic);
        (void)hipFree(d_oc);
        (void)hipFree(d_ie);
        (void)hipFree(d_oe);
        (void)hipFree(d_sorted);
        (void)hipFree(d_pos);
        (void)hipFree(d_hint);
        (void)hipFree(d_ok);
        (void)hipFree(d_prof);
        return r;
    };
    if (n <= 0 || threads < 64 || threads > 1024 || threads % 64 || scratch < 0 || scratch > 163840 ||
        (n_hint > 0 && !hint) || n_prev < 0 || n_prev > n || (n_prev > 0 && !order_prev))
        return -2;
    // the previous order: a permutation of the first n_prev nodes
    std::vector<SizeT> so(n, SizeT(0));
    {
        std::vector<char> seen(n_prev, 0);
        for (int q = 0; q < n_prev; q++)
        {
            const int v = order_prev[q];
            if (v < 0 || v >= n_prev || seen[v])
                return -2;
            seen[v] = 1;
            so[q]   = SizeT(v);
        }
    }
    if (hipMalloc(&d_ic, n * 2) || hipMalloc(&d_oc, n * 2) || hipMalloc(&d_ie, ne * sizeof(SizeT)) ||
        hipMalloc(&d_oe, ne * sizeof(SizeT)) || hipMalloc(&d_sorted, n * sizeof(SizeT)) ||
        hipMalloc(&d_pos, n * sizeof(SizeT)) || hipMalloc(&d_hint, n * sizeof(SizeT)) ||
        hipMalloc(&d_ok, sizeof(int)) || hipMalloc(&d_prof, 10 * sizeof(uint64_t)) ||
        hipMemset(d_prof, 0, 10 * sizeof(uint64_t)))
        return fin(-1);
    if (hipMemcpy(d_ic, in_cnt, n * 2, hipMemcpyHostToDevice) || hipMemcpy(d_oc, out_cnt, n * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(d_ie, ie.data(), ne * sizeof(SizeT), hipMemcpyHostToDevice) ||
        hipMemcpy(d_oe, oe.data(), ne * sizeof(SizeT), hipMemcpyHostToDevice) ||
        hipMemcpy(d_hint, hi.data(), n * sizeof(SizeT), hipMemcpyHostToDevice) ||
        hipMemcpy(d_sorted, so.data(), n * sizeof(SizeT), hipMemcpyHostToDevice))
        return fin(-1);
    WinGraph<SizeT> g{};
    g.in_cnt    = d_ic;
    g.out_cnt   = d_oc;
    g.in_e      = d_ie;
    g.out_e     = d_oe;
    g.sorted    = d_sorted;
    g.pos       = d_pos;
    g.max_nodes = n;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topsort_levels_test_kernel<SizeT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, scratch))
        return fin(-1);
    hipLaunchKernelGGL(topsort_levels_test_kernel<SizeT>, dim3(1), dim3(threads), size_t(scratch), 0, g, n, n_prev,
                       scratch, d_hint, n_hint, d_ok, nullptr);
    if (hipGetLastError() || hipDeviceSynchronize() || hipMemcpy(&ok, d_ok, sizeof(int), hipMemcpyDeviceToHost))
        return fin(-1);
    if (reps > 0)
    {
        // timing mode: the same sort `reps` times (the graph, previous order and
        // hints are inputs only; the outputs are rewritten identically)
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) || hipEventCreate(&e1))
            return fin(-1);
        (void)hipEventRecord(e0, 0);
        for (int k = 0; k < reps; k++)
        {
            if (hipMemcpy(d_sorted, so.data(), n * sizeof(SizeT), hipMemcpyHostToDevice))
                return fin(-1);
            hipLaunchKernelGGL(topsort_levels_test_kernel<SizeT>, dim3(1), dim3(threads), size_t(scratch), 0, g, n,
                               n_prev, scratch, d_hint, n_hint, d_ok, d_prof);
        }
        (void)hipEventRecord(e1, 0);
        float t = 0.f;
        if (hipEventSynchronize(e1) || hipEventElapsedTime(&t, e0, e1))
            return fin(-1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (ms)
            *ms = double(t) / reps;
        if (prof_out && hipMemcpy(prof_out, d_prof, 10 * sizeof(uint64_t), hipMemcpyDeviceToHost))
            return fin(-1);
    }
    std::vector<SizeT> s(n);
    if (hipMemcpy(s.data(), d_sorted, n * sizeof(SizeT), hipMemcpyDeviceToHost) ||
        hipMemcpy(hi.data(), d_hint, n * sizeof(SizeT), hipMemcpyDeviceToHost))
        return fin(-1);
    for (int q = 0; q < n; q++)
        sorted[q] = int32_t(s[q]);
    for (int v = 0; hint && v < n; v++)
        hint[v] = int32_t(hi[v]);
    return fin(ok);
}

// Test hook: the racon DFS sort (topsort_racon_lds) of one graph by one wave,
// with the group heads in HBM (heads != nullptr: racon_dfs_csr) or the
// round-5 step (heads == nullptr).
template <typename SizeT>
__global__ void __launch_bounds__(64) topsort_racon_test_kernel(WinGraph<SizeT> g, int n, int scratch, int32_t* heads,
                                                               SizeT* mpos, int* out)
{
    extern __shared__ __align__(16) uint8_t lds[];
    // a static word first, as in the kernels: the dynamic scratch then does
    // not start at LDS address 0 (a null scratch pointer means "no scratch")
    __shared__ int keep[4];
    if (threadIdx.x < 4)
        keep[threadIdx.x] = n;
    __syncthreads();
    int cols     = 0;
    const bool r = topsort_racon_lds<SizeT>(g, n, (GWAMD_LDS uint8_t*)(lds), scratch, int(threadIdx.x), mpos, &cols,
                                            heads);
    if (threadIdx.x == 0)
    {
        out[0] = r && keep[3] == n ? 1 : 0;
        out[1] = cols;
    }
}

template <typename SizeT>
int topsort_racon_test(int n, const uint16_t* in_cnt, const int32_t* in_e, const uint16_t* aln_cnt,
                       const int32_t* aln, int scratch, int v1, int32_t* sorted, int32_t* mpos, int* ncols, int reps,
                       double* ms)
{
    if (n <= 0 || n > 65535 || scratch < 0 || scratch > 163840 - 64)
        return -2;
    const size_t ne = size_t(n) * kMaxEdges, na = size_t(n) * kMaxAlignments;
    std::vector<SizeT> ie(ne), al(na);
    for (size_t i = 0; i < ne; i++)
        ie[i] = SizeT(in_e[i]);
    for (size_t i = 0; i < na; i++)
        al[i] = SizeT(aln[i]);
    uint16_t *d_ic = nullptr, *d_ac = nullptr;
    SizeT *d_ie = nullptr, *d_al = nullptr, *d_sorted = nullptr, *d_pos = nullptr, *d_mpos = nullptr;
    int32_t* d_heads = nullptr;
    int* d_out       = nullptr;
    auto fin         = [&](int r) {
        (void)hipFree(d_ic);
        (void)hipFree(d_ac);
        (void)hipFree(d_ie);
        (void)hipFree(d_al);
        (void)hipFree(d_sorted);
        (void)hipFree(d_pos);
        (void)hipFree(d_mpos);
        (void)hipFree(d_heads);
        (void)hipFree(d_out);
        return r;
    };
    if (hipMalloc(&d_ic, n * 2) || hipMalloc(&d_ac, n * 2) || hipMalloc(&d_ie, ne * sizeof(SizeT)) ||
        hipMalloc(&d_al, na * sizeof(SizeT)) || hipMalloc(&d_sorted, n * sizeof(SizeT)) ||
        hipMalloc(&d_pos, n * sizeof(SizeT)) || hipMalloc(&d_mpos, n * sizeof(SizeT)) ||
        hipMalloc(&d_heads, n * sizeof(int32_t)) || hipMalloc(&d_out, 2 * sizeof(int)))
        return fin(-1);
    if (hipMemcpy(d_ic, in_cnt, n * 2, hipMemcpyHostToDevice) || hipMemcpy(d_ac, aln_cnt, n * 2, hipMemcpyHostToDevice) ||
        hipMemcpy(d_ie, ie.data(), ne * sizeof(SizeT), hipMemcpyHostToDevice) ||
        hipMemcpy(d_al, al.data(), na * sizeof(SizeT), hipMemcpyHostToDevice) ||
        hipMemset(d_sorted, 0xff, n * sizeof(SizeT)) || hipMemset(d_mpos, 0xff, n * sizeof(SizeT)))
        return fin(-1);
    WinGraph<SizeT> g{};
    g.in_cnt    = d_ic;
    g.aln_cnt   = d_ac;
    g.in_e      = d_ie;
    g.aln       = d_al;
    g.sorted    = d_sorted;
    g.pos       = d_pos;
    g.max_nodes = n;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&topsort_racon_test_kernel<SizeT>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, scratch))
        return fin(-1);
    int32_t* hp = v1 ? nullptr : d_heads;
    hipLaunchKernelGGL(topsort_racon_test_kernel<SizeT>, dim3(1), dim3(64), size_t(scratch), 0, g, n, scratch, hp,
                       d_mpos, d_out);
    int out[2] = {0, 0};
    if (hipGetLastError() || hipDeviceSynchronize() || hipMemcpy(out, d_out, sizeof(out), hipMemcpyDeviceToHost))
        return fin(-1);
    if (reps > 0)
    {
        hipEvent_t e0, e1;
        if (hipEventCreate(&e0) || hipEventCreate(&e1))
            return fin(-1);
        (void)hipEventRecord(e0, 0);
        for (int k = 0; k < reps; k++)
            hipLaunchKernelGGL(topsort_racon_test_kernel<SizeT>, dim3(1), dim3(64), size_t(scratch), 0, g, n,
                               scratch, hp, d_mpos, d_out);
        (void)hipEventRecord(e1, 0);
        float t = 0.f;
        if (hipEventSynchronize(e1) || hipEventElapsedTime(&t, e0, e1))
            return fin(-1);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        if (ms)
            *ms = double(t) / reps;
    }
    std::vector<SizeT> s(n), mp(n);
    if (hipMemcpy(s.data(), d_sorted, n * sizeof(SizeT), hipMemcpyDeviceToHost) ||
        hipMemcpy(mp.data(), d_mpos, n * sizeof(SizeT), hipMemcpyDeviceToHost))
        return fin(-1);
    for (int q = 0; q < n; q++)
    {
        sorted[q] = int32_t(s[q]);
        if (mpos)
            mpos[q] = int32_t(mp[q]);
    }
    if (ncols)
        *ncols = out[1];
    return fin(out[0]);
}

} // namespace poa
} // namespace gwamd

// Test hook (tests/test_poa_topsort.py, scripts/racon_bench.py): the racon
// DFS sort (cudapoa_topsort.cuh:94-189) of one graph given as fixed-slot
// in-edge and aligned-node arrays (kMaxEdges / kMaxAlignments slots), by one
// wave with `scratch` bytes of LDS; v1 selects the round-5 DFS step.  Writes
// the order, the MSA column of every node and the column count.  Returns 1
// when the LDS sort ran, 0 when it declined (the kernels then run the HBM
// sort), negative on a HIP error or bad arguments.  reps > 0: that many more
// sorts, *ms = the mean time per sort.
extern "C" int gwamd_internal_topsort_racon(int size_bits, int n, const uint16_t* in_cnt, const int32_t* in_e,
                                            const uint16_t* aln_cnt, const int32_t* aln, int scratch, int v1,
                                            int32_t* sorted, int32_t* mpos, int* ncols, int reps, double* ms)
{
    if (size_bits == 16)
        return gwamd::poa::topsort_racon_test<int16_t>(n, in_cnt, in_e, aln_cnt, aln, scratch, v1, sorted, mpos,
                                                       ncols, reps, ms);
    return gwamd::poa::topsort_racon_test<int32_t>(n, in_cnt, in_e, aln_cnt, aln, scratch, v1, sorted, mpos, ncols,
                                                   reps, ms);
}

// Test hook (tests/test_poa_topsort.py): topsort_levels of one graph given as
// the reference's fixed-slot edge arrays (kMaxEdges slots per node), with the
// previous read's order of the first n_prev nodes (order_prev: a permutation
// of 0..n_prev-1, may be null when n_prev is 0) and critical-predecessor
// hints for the first n_hint nodes (hint may be null when n_hint is 0; it
// receives the final c(v)).  Returns 1 when the level sort produced sorted[],
// 0 when it declined (the kernels then run the FIFO sort), negative on a HIP
// error or bad arguments.
// Timing mode of the same hook (scripts/topsort_bench.py): after the checked
// run, `reps` more sorts; *ms gets the mean time per sort (HIP events around
// launches of one workgroup, copies of the previous order included) and
// prof[10] the section cycles, anchors and iterations of GWAMD_TOPSORT_PROFILE
// builds.
extern "C" int gwamd_internal_topsort_levels_timed(int size_bits, int n, int n_prev, int n_hint,
                                                   const uint16_t* in_cnt, const int32_t* in_e,
                                                   const uint16_t* out_cnt, const int32_t* out_e, int32_t* hint,
                                                   const int32_t* order_prev, int threads, int scratch,
                                                   int32_t* sorted, int reps, double* ms, uint64_t* prof)
{
    if (size_bits == 16)
        return gwamd::poa::topsort_levels_test<int16_t>(n, n_prev, n_hint, in_cnt, in_e, out_cnt, out_e, hint,
                                                        order_prev, threads, scratch, sorted, reps, ms, prof);
    return gwamd::poa::topsort_levels_test<int32_t>(n, n_prev, n_hint, in_cnt, in_e, out_cnt, out_e, hint, order_prev,
                                                    threads, scratch, sorted, reps, ms, prof);
}

extern "C" int gwamd_internal_topsort_levels(int size_bits, int n, int n_prev, int n_hint, const uint16_t* in_cnt,
                                             const int32_t* in_e, const uint16_t* out_cnt, const int32_t* out_e,
                                             int32_t* hint, const int32_t* order_prev, int threads, int scratch,
                                             int32_t* sorted)
{
    if (size_bits == 16)
        return gwamd::poa::topsort_levels_test<int16_t>(n, n_prev, n_hint, in_cnt, in_e, out_cnt, out_e, hint,
                                                        order_prev, threads, scratch, sorted);
    return gwamd::poa::topsort_levels_test<int32_t>(n, n_prev, n_hint, in_cnt, in_e, out_cnt, out_e, hint, order_prev,
                                                    threads, scratch, sorted);
}

// ---------------------------------------------------------------------------
extern "C" hipError_t gwamd_internal_poa_band_launch(const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d,
                                                     const gwamd::poa::Scores* sc, int score_bits, int size_bits,
                                                     int msa, hipStream_t stream); // poa_band.hip
extern "C" int gwamd_internal_poa_band_blocks_per_cu(const gwamd::poa::Dims* d, int score_bits, int size_bits,
                                                     int msa); // poa_band.hip

namespace
{
template <typename K>
int blocks_per_cu(K kfn, int threads, size_t lds)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kfn, threads, lds) != hipSuccess)
        return 0;
    return n;
}
} // namespace

// Workgroups of the planned LDS or banded kernel that are resident on one CU
// at once (the persistent grid is this times the CU count); 0 for the v1
// kernel, which runs one workgroup per window.
extern "C" int gwamd_internal_poa_blocks_per_cu(const gwamd::poa::Dims* d, int score_bits, int size_bits, int banded,
                                                int msa)
{
    using namespace gwamd::poa;
    if (d->lds_kernel == 3 && banded)
        return gwamd_internal_poa_band_blocks_per_cu(d, score_bits, size_bits, msa);
    if (d->lds_kernel != 1 || banded || size_bits != 16 || (score_bits != 16 && score_bits != 32))
        return 0;
    const size_t lb = size_t(d->lds_bytes);
#define GWAMD_LDS_OCC_W(CPL, NW, WD)                                                                          \
    if (d->lds_cpl == CPL && d->lds_waves == NW && (score_bits == 32) == WD)                                   \
    {                                                                                                          \
        auto kt = poa_window_kernel_lds<true, CPL, NW, WD>;                                                    \
        auto kf = poa_window_kernel_lds<false, CPL, NW, WD>;                                                   \
        if (lb > 65536 &&                                                                                      \
            (hipFuncSetAttribute(reinterpret_cast<const void*>(msa ? kt : kf),                                 \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, int(lb)) != hipSuccess))          \
            return 0;                                                                                          \
        return msa ? blocks_per_cu(kt, kWave * NW, lb) : blocks_per_cu(kf, kWave * NW, lb);                    \
    }
#define GWAMD_LDS_OCC(CPL, NW) GWAMD_LDS_OCC_W(CPL, NW, false)
    // 32-bit scores: (columns per lane, waves) planned by poa_batch.cpp
    GWAMD_LDS_OCC_W(8, 1, true)
    GWAMD_LDS_OCC_W(8, 2, true)
    GWAMD_LDS_OCC_W(8, 4, true)
    GWAMD_LDS_OCC_W(8, 8, true)
    GWAMD_LDS_OCC_W(16, 8, true)
    GWAMD_LDS_OCC(8, 1)
    GWAMD_LDS_OCC(16, 1)
    GWAMD_LDS_OCC(24, 1)
    GWAMD_LDS_OCC(32, 1)
    GWAMD_LDS_OCC(8, 2)
    GWAMD_LDS_OCC(8, 3)
    GWAMD_LDS_OCC(8, 4)
    GWAMD_LDS_OCC(16, 4)
    GWAMD_LDS_OCC(4, 4)
#undef GWAMD_LDS_OCC
#undef GWAMD_LDS_OCC_W
    return 0;
}

// Internal launch ABI used by the C++ batch (poa_batch.cpp).
extern "C" hipError_t gwamd_internal_poa_launch(const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d,
                                       const gwamd::poa::Scores* sc, int score_bits, int size_bits, int banded,
                                       int msa, hipStream_t stream)
{
    using namespace gwamd::poa;
    if (b->num_windows <= 0)
        return hipSuccess;
    dim3 grid(b->num_windows), block(kWave);
    if (d->lds_kernel && b->head)
        grid = dim3(b->num_slots); // persistent grid: one workgroup per scratch slot
    if (d->lds_kernel == 3 && banded)
        return gwamd_internal_poa_band_launch(b, d, sc, score_bits, size_bits, msa, stream);
    if (d->lds_kernel == 1 && !banded && size_bits == 16 && (score_bits == 16 || score_bits == 32))
    {
        const size_t lb = size_t(d->lds_bytes);
#define GWAMD_LDS_LAUNCH_W(CPL, NW, WD)                                                                        \
    if (d->lds_cpl == CPL && d->lds_waves == NW && (score_bits == 32) == WD)                                   \
    {                                                                                                          \
        const dim3 blk(kWave * NW);                                                                            \
        auto kt = poa_window_kernel_lds<true, CPL, NW, WD>;                                                    \
        auto kf = poa_window_kernel_lds<false, CPL, NW, WD>;                                                   \
        if (lb > 65536)                                                                                        \
        {                                                                                                      \
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(msa ? kt : kf),             \
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, int(lb));     \
            if (e != hipSuccess)                                                                               \
                return e;                                                                                      \
        }                                                                                                      \
        if (msa)                                                                                               \
            hipLaunchKernelGGL(kt, grid, blk, lb, stream, *b, *d, *sc);                                        \
        else                                                                                                   \
            hipLaunchKernelGGL(kf, grid, blk, lb, stream, *b, *d, *sc);                                        \
        return hipGetLastError();                                                                              \
    }
#define GWAMD_LDS_LAUNCH(CPL, NW) GWAMD_LDS_LAUNCH_W(CPL, NW, false)
        // (columns per lane, waves per window) pairs planned by poa_batch.cpp
        GWAMD_LDS_LAUNCH_W(8, 1, true)
        GWAMD_LDS_LAUNCH_W(8, 2, true)
        GWAMD_LDS_LAUNCH_W(8, 4, true)
        GWAMD_LDS_LAUNCH_W(8, 8, true)
        GWAMD_LDS_LAUNCH_W(16, 8, true)
        GWAMD_LDS_LAUNCH(8, 1)
        GWAMD_LDS_LAUNCH(16, 1)
        GWAMD_LDS_LAUNCH(24, 1)
        GWAMD_LDS_LAUNCH(32, 1)
        GWAMD_LDS_LAUNCH(8, 2)
        GWAMD_LDS_LAUNCH(8, 3)
        GWAMD_LDS_LAUNCH(8, 4)
        GWAMD_LDS_LAUNCH(16, 4)
        GWAMD_LDS_LAUNCH(4, 4)
        return hipErrorInvalidConfiguration;
#undef GWAMD_LDS_LAUNCH
#undef GWAMD_LDS_LAUNCH_W
    }
    const int lds_bytes = (d->max_seq_len > d->band_width + kBandPad ? d->max_seq_len : d->band_width + kBandPad) + 32;
    const size_t lds    = size_t((lds_bytes + 15) & ~15);
#define GWAMD_LAUNCH(ST, ZT, BD, MS)                                                                          \
    hipLaunchKernelGGL((poa_window_kernel<ST, ZT, BD, MS>), grid, block, lds, stream, *b, *d, *sc);           \
    return hipGetLastError();
#define GWAMD_DISPATCH_MODE(ST, ZT)           \
    if (banded)                               \
    {                                         \
        if (msa)                              \
        {                                     \
            GWAMD_LAUNCH(ST, ZT, true, true)  \
        }                                     \
        GWAMD_LAUNCH(ST, ZT, true, false)     \
    }                                         \
    if (msa)                                  \
    {                                         \
        GWAMD_LAUNCH(ST, ZT, false, true)     \
    }                                         \
    GWAMD_LAUNCH(ST, ZT, false, false)
    if (score_bits == 16)
    {
        GWAMD_DISPATCH_MODE(int16_t, int16_t)
    }
    if (size_bits == 16)
    {
        GWAMD_DISPATCH_MODE(int32_t, int16_t)
    }
    GWAMD_DISPATCH_MODE(int32_t, int32_t)
#undef GWAMD_DISPATCH_MODE
#undef GWAMD_LAUNCH
}

// MI355X global aligners: Hirschberg + Myers (the default of create_aligner,
// cudaaligner/src/hirschberg_myers_gpu.cu) and full Myers with backtrace
// (AlignerGlobalMyers, cudaaligner/src/myers_gpu.cu:95-375).
//
// One wave per pair; a persistent grid walks the pairs with a static stride.
// The Myers bit-vector state of a query segment lives in registers: lane l of
// block c holds query word 64c + l (32 rows), a block is 2048 rows, and the
// multi-word addition and the one-bit shift of the recurrence cross lanes with
// ballot masks (carry lookahead on the 64-bit generate/propagate masks) and
// the lane-bit extraction below.  Any exact Myers implementation gives the
// edit-distance matrix bit for bit, so the results depend only on the tie
// rules, which follow the reference:
//   * target split: minimum of fwd(t) + rev(T-t), ties to the 32-lane /
//     shfl_down order (hirschberg_myers_gpu.cu:450-474),
//   * backtrace: insertion, then deletion, then diagonal (:118-160),
//   * base cases and their order, the 64-entry stack and its overflow
//     behaviour, the full-Myers switch condition with the reference's
//     workspace capacity (:569-638, aligner_global_hirschberg_myers.cpp:51-54).
#include <hip/hip_runtime.h>

#include "aligner_common.hpp"
#include "aligner_device.hpp"

#include <climits>
#include <type_traits>

#ifdef GWAMD_ALN_PROFILE
// Diagnostic build only: cycle counters per phase of hm_kernel, summed over
// waves ([0] reverse sweeps, [1] forward sweeps, [2] base cases, [3] total,
// [4] sweep columns x blocks, [5] base-case columns, [6] base cases).
__device__ unsigned long long gwamd_aln_prof[8];
#define GWAMD_PROF_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define GWAMD_PROF_ADD(acc, v) acc += __builtin_amdgcn_s_memtime() - v
#else
#define GWAMD_PROF_T0(v)
#define GWAMD_PROF_ADD(acc, v)
#endif

namespace gwamd
{
namespace aln
{

// One column of the block-wise Myers recurrence for block c.  hin is the
// horizontal delta entering the block's first row; returns the delta leaving
// its last row (row `hb` of lane `ll` for the segment's last block).
struct MyersBlock
{
    uint32_t pv, mv;
    uint32_t e[4];
    uint64_t act; // lanes holding segment words
};

// own (optional): each lane's delta at its own word's last row (bit own_hb),
// i.e. the per-word score update of the full-matrix variant (myers_gpu.cu:356).
template <bool OWN = false>
__device__ __forceinline__ int myers_block_step(MyersBlock& B, int code, int hin, bool last, int ll, int hb, int lane,
                                                uint32_t hisel, uint32_t lane0bit, int own_hb = 31,
                                                int* own = nullptr)
{
    // select the pattern of this column's letter (code is wave-uniform)
    const uint32_t lo = (code & 1) ? B.e[1] : B.e[0];
    const uint32_t hi = (code & 1) ? B.e[3] : B.e[2];
    uint32_t eq       = (code & 2) ? hi : lo;
    const uint32_t xv = eq | B.mv;
    if (hin < 0)
        eq |= lane0bit;
    // (eq & pv) + pv over the whole block: carry lookahead on ballot masks
    const uint32_t a = eq & B.pv;
    uint32_t s;
    const bool ov     = __builtin_add_overflow(a, B.pv, &s);
    const uint64_t G  = __builtin_amdgcn_ballot_w64(ov) & B.act;
    const uint64_t P  = __builtin_amdgcn_ballot_w64(s == 0xffffffffu) & B.act;
    const uint64_t GP = G | P;
    const uint64_t C  = ((GP + G) ^ GP ^ G);
    s += mask_bit(C, hisel, lane);
    const uint32_t xh = (s ^ B.pv) | eq;
    uint32_t ph       = B.mv | ~(xh | B.pv);
    uint32_t mh       = B.pv & xh;
    if constexpr (OWN)
        *own = int((ph >> own_hb) & 1u) - int((mh >> own_hb) & 1u);
    int hout;
    const uint64_t PH = __builtin_amdgcn_ballot_w64((ph >> 31) != 0u);
    const uint64_t MH = __builtin_amdgcn_ballot_w64((mh >> 31) != 0u);
    if (last)
    {
        const uint32_t phl = uniu(__builtin_amdgcn_readlane(int(ph), ll));
        const uint32_t mhl = uniu(__builtin_amdgcn_readlane(int(mh), ll));
        hout               = int((phl >> hb) & 1u) - int((mhl >> hb) & 1u);
    }
    else
        hout = int((PH >> 63) & 1u) - int((MH >> 63) & 1u);
    ph = (ph << 1) | mask_bit(PH << 1, hisel, lane);
    mh = (mh << 1) | mask_bit(MH << 1, hisel, lane);
    if (hin > 0)
        ph |= lane0bit;
    if (hin < 0)
        mh |= lane0bit;
    B.pv = mh | ~(xv | ph);
    B.mv = ph & xv;
    return hout;
}

// Myers sweep of query rows [qb, qe) (reversed: rows qe-1 down to qb) over the
// target columns [tb, te) (reversed: te-1 down to tb); on_col(t, D(m, t)) for
// t = 0..T (myers_compute_scores with full_score_matrix = false, :272-370).
template <typename OnCol>
__device__ void myers_sweep(const GWAMD_LDS uint32_t* pat, int pat_words, int Q, int qb, int qe, bool rev,
                            const GWAMD_LDS uint8_t* tgt, int tb, int te, int lane, OnCol&& on_col)
{
    const int m      = qe - qb;
    const int nwords = (m + kWordBits - 1) / kWordBits;
    const int nch    = uni((nwords + kWave - 1) / kWave);
    const int off    = rev ? Q - qe : qb;
    const int pbase  = rev ? 4 : 0;
    const int lw     = nwords - 1;
    const int lc     = lw / kWave;
    const int ll     = lw % kWave;
    const int hb     = (m - 1) % kWordBits;
    const uint32_t hisel    = lane >= 32 ? 1u : 0u;
    const uint32_t lane0bit = lane == 0 ? 1u : 0u;
    MyersBlock B[kMaxChunks];
#pragma unroll
    for (int c = 0; c < kMaxChunks; c++)
    {
        const int w      = c * kWave + lane;
        const bool valid = c < nch && w < nwords;
#pragma unroll
        for (int L = 0; L < 4; L++)
            B[c].e[L] = valid ? seg_pattern(pat, pat_words, off, w, pbase + L) : 0u;
        B[c].pv  = ~0u;
        B[c].mv  = 0u;
        B[c].act = __builtin_amdgcn_ballot_w64(valid);
    }
    const int T = te - tb;
    int score   = m;
    on_col(0, score);
    int tv = 0;
    for (int t = 1; t <= T; t++)
    {
        const int tl = (t - 1) & (kWave - 1);
        if (tl == 0)
        {
            // next 64 target characters, one per lane
            const int idx = t - 1 + lane;
            tv            = idx < T ? int(tgt[rev ? te - 1 - idx : tb + idx]) : 0;
        }
        const int code = letter(uni(__builtin_amdgcn_readlane(tv, tl)));
        int h          = 1; // top row 0, 1, 2, ...: +1 into the first block
#pragma unroll
        for (int c = 0; c < kMaxChunks; c++)
        {
            if (c < nch)
                h = myers_block_step(B[c], code, h, c == lc, ll, hb, lane, hisel, lane0bit);
        }
        score += h;
        on_col(t, score);
    }
}

// Branch-free variant of myers_block_step: no data-dependent branches, so the
// two independent sweeps of a split interleave in one instruction stream.
__device__ __forceinline__ int block_step_bf(MyersBlock& B, int code, int hin, bool last, int ll, int hb, int lane,
                                             uint32_t hisel, uint32_t lane0bit)
{
    const uint32_t lo  = (code & 1) ? B.e[1] : B.e[0];
    const uint32_t hi  = (code & 1) ? B.e[3] : B.e[2];
    const uint32_t neg = hin < 0 ? lane0bit : 0u;
    const uint32_t pos = hin > 0 ? lane0bit : 0u;
    uint32_t eq        = (code & 2) ? hi : lo;
    const uint32_t xv  = eq | B.mv;
    eq |= neg;
    uint32_t s;
    const bool ov     = __builtin_add_overflow(eq & B.pv, B.pv, &s);
    const uint64_t G  = __builtin_amdgcn_ballot_w64(ov) & B.act;
    const uint64_t P  = __builtin_amdgcn_ballot_w64(s == 0xffffffffu) & B.act;
    const uint64_t GP = G | P;
    s += mask_bit((GP + G) ^ GP ^ G, hisel, lane);
    const uint32_t xh  = (s ^ B.pv) | eq;
    uint32_t ph        = B.mv | ~(xh | B.pv);
    uint32_t mh        = B.pv & xh;
    const uint64_t PH  = __builtin_amdgcn_ballot_w64((ph >> 31) != 0u);
    const uint64_t MH  = __builtin_amdgcn_ballot_w64((mh >> 31) != 0u);
    const uint32_t phl = uniu(__builtin_amdgcn_readlane(int(ph), ll));
    const uint32_t mhl = uniu(__builtin_amdgcn_readlane(int(mh), ll));
    const int h_last   = int((phl >> hb) & 1u) - int((mhl >> hb) & 1u);
    const int h_full   = int((PH >> 63) & 1u) - int((MH >> 63) & 1u);
    ph                 = (ph << 1) | mask_bit(PH << 1, hisel, lane) | pos;
    mh                 = (mh << 1) | mask_bit(MH << 1, hisel, lane) | neg;
    B.pv               = mh | ~(xv | ph);
    B.mv               = ph & xv;
    return last ? h_last : h_full;
}

// Myers state of one half of a split (rows [qb, qe), forward or reversed)
template <int N>
struct HalfSweep
{
    MyersBlock B[N];
    int lc, ll, hb, score;
    // m rows starting at row `off` of the forward (rev: reversed) query
    template <typename PatPtr>
    __device__ void init_rows(PatPtr pat, int pat_words, int off, int m, bool rev, int lane)
    {
        const int nwords = (m + kWordBits - 1) / kWordBits;
        const int pbase  = rev ? 4 : 0;
        const int lw     = nwords - 1;
        lc               = lw / kWave;
        ll               = lw % kWave;
        hb               = (m - 1) % kWordBits;
        score            = m;
#pragma unroll
        for (int c = 0; c < N; c++)
        {
            const int w      = c * kWave + lane;
            const bool valid = w < nwords;
#pragma unroll
            for (int L = 0; L < 4; L++)
                B[c].e[L] = valid ? seg_pattern(pat, pat_words, off, w, pbase + L) : 0u;
            B[c].pv  = ~0u;
            B[c].mv  = 0u;
            B[c].act = __builtin_amdgcn_ballot_w64(valid);
        }
    }
    template <typename PatPtr>
    __device__ void init(PatPtr pat, int pat_words, int Q, int qb, int qe, bool rev, int lane)
    {
        init_rows(pat, pat_words, rev ? Q - qe : qb, qe - qb, rev, lane);
    }
    // one column; hin enters the first row, returns the delta leaving the last
    __device__ __forceinline__ int step_in(int code, int hin, int lane, uint32_t hisel, uint32_t lane0bit)
    {
        int h = hin, hl = 0;
#pragma unroll
        for (int c = 0; c < N; c++)
        {
            h  = block_step_bf(B[c], code, h, c == lc, ll, hb, lane, hisel, lane0bit);
            hl = c == lc ? h : hl;
        }
        return hl;
    }
    __device__ __forceinline__ void step(int code, int lane, uint32_t hisel, uint32_t lane0bit)
    {
        score += step_in(code, 1, lane, hisel, lane0bit); // top row 0, 1, 2, ...: +1 into the first block
    }
};

// Both sweeps of a Hirschberg split in one pass over the target segment
// (hirschberg_myers_compute_target_mid_warp, hirschberg_myers_gpu.cu:411-475):
// fw[t] = D(q[qb, qm), target[tb, tb + t)), rv[t] = D(q[qm, qe) reversed,
// target[te - t, te) reversed), t = 0..Ts.  N: 64-word blocks of the larger
// half.
template <int N, typename PatPtr, typename TcPtr, typename Buf>
__device__ void split_sweep(PatPtr pat, int pat_words, int Q, int qb, int qm, int qe,
                            TcPtr tcod, int tb, int te, int lane, Buf fw, Buf rv)
{
    const uint32_t hisel    = lane >= 32 ? 1u : 0u;
    const uint32_t lane0bit = lane == 0 ? 1u : 0u;
    HalfSweep<N> F, R;
    F.init(pat, pat_words, Q, qb, qm, false, lane);
    R.init(pat, pat_words, Q, qm, qe, true, lane);
    const int Ts = te - tb;
    for (int t0 = 0; t0 <= Ts; t0 += kWave)
    {
        // letter codes of the next 64 columns, one per lane
        const int tt = t0 + lane;
        const bool in = tt >= 1 && tt <= Ts;
        const int cf  = in ? code_at(tcod, tb + tt - 1) : 0;
        const int cr  = in ? code_at(tcod, te - tt) : 0;
        const int cnt = min(kWave, Ts + 1 - t0);
        uint32_t bf = F.score, br = R.score; // lane x: column t0 + x
        for (int x = t0 == 0 ? 1 : 0; x < cnt; x++)
        {
            F.step(uni(__builtin_amdgcn_readlane(cf, x)), lane, hisel, lane0bit);
            R.step(uni(__builtin_amdgcn_readlane(cr, x)), lane, hisel, lane0bit);
            bf = lane == x ? uint32_t(F.score) : bf;
            br = lane == x ? uint32_t(R.score) : br;
        }
        if (lane < cnt)
        {
            fw[t0 + lane] = bf;
            rv[t0 + lane] = br;
        }
    }
}

// One half of a split too tall for one register-resident sweep (more than
// kMaxChunks blocks, queries over 16,384 bases): stripes of kMaxChunks blocks
// from the half's first row down; the horizontal delta leaving a stripe's last
// row at every column reaches the next stripe through hbuf (one int8 per
// column, written and read back by the same lane).  out[t] = D(m, t) of the
// half (forward, or reversed rows and columns), t = 0..Ts: the same values as
// one tall sweep, since the Myers column recurrence is exact.
template <typename PatPtr, typename TcPtr, typename Buf>
__device__ void half_sweep_striped(PatPtr pat, int pat_words, int Q, int qb, int qe, bool rev,
                                   TcPtr tcod, int tb, int te, int lane, Buf out, int8_t* hbuf,
                                   int stripe_blocks)
{
    const int m        = qe - qb;
    const int off0     = rev ? Q - qe : qb;
    const int rows_per = stripe_blocks * kWave * kWordBits; // stripe_blocks <= kMaxChunks
    const int Ts       = te - tb;
    const uint32_t hisel    = lane >= 32 ? 1u : 0u;
    const uint32_t lane0bit = lane == 0 ? 1u : 0u;
    for (int r0 = 0; r0 < m; r0 += rows_per)
    {
        const int ms     = min(rows_per, m - r0);
        const bool first = r0 == 0;
        const bool last  = r0 + ms == m;
        HalfSweep<kMaxChunks> H;
        H.init_rows(pat, pat_words, off0 + r0, ms, rev, lane);
        int score = m; // D(m, 0); only the last stripe's deltas reach row m
        for (int t0 = 0; t0 <= Ts; t0 += kWave)
        {
            const int tt  = t0 + lane;
            const bool in = tt >= 1 && tt <= Ts;
            const int cd  = in ? code_at(tcod, rev ? te - tt : tb + tt - 1) : 0;
            const int hv  = (!first && in) ? int(hbuf[tt]) : 1; // first stripe: the top row's +1
            const int cnt = min(kWave, Ts + 1 - t0);
            int ho        = 0;
            uint32_t bo   = uint32_t(score);
            for (int x = t0 == 0 ? 1 : 0; x < cnt; x++)
            {
                const int h = H.step_in(uni(__builtin_amdgcn_readlane(cd, x)), uni(__builtin_amdgcn_readlane(hv, x)),
                                        lane, hisel, lane0bit);
                score += h;
                ho = lane == x ? h : ho;
                bo = lane == x ? uint32_t(score) : bo;
            }
            if (!last && in)
                hbuf[tt] = int8_t(ho);
            if (last && lane < cnt)
                out[t0 + lane] = bo;
        }
        __threadfence_block();
        wave_sync();
    }
}

// Split column: minimum of fw[t] + rv[Ts - t]; ties to the smallest 5-bit-
// reversed t, then the smallest t (the reference's 32-lane striding and
// shfl_down tree, hirschberg_myers_gpu.cu:450-474).
template <typename Buf>
__device__ int split_argmin(Buf fw, Buf rv, int Ts, int lane)
{
    uint64_t best = ~uint64_t(0);
    for (int t = lane; t <= Ts; t += kWave)
    {
        const uint32_t sum = uint32_t(fw[t]) + uint32_t(rv[Ts - t]);
        const uint32_t key = __builtin_bitreverse32(uint32_t(t) & 31u) >> 27;
        const uint64_t v   = (uint64_t(sum) << 40) | (uint64_t(key) << 32) | uint32_t(t);
        best               = v < best ? v : best;
    }
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1)
    {
        const uint64_t o = __shfl_xor(best, d);
        best             = o < best ? o : best;
    }
    return uni(int(uint32_t(best)));
}

template <typename PatPtr, typename TcPtr, typename Buf>
__device__ void run_split(int nblk, PatPtr pat, int pat_words, int Q, int qb, int qm, int qe,
                          TcPtr tcod, int tb, int te, int lane, Buf fw, Buf rv)
{
    switch (nblk)
    {
    case 1: split_sweep<1>(pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fw, rv); break;
    case 2: split_sweep<2>(pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fw, rv); break;
    case 3: split_sweep<3>(pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fw, rv); break;
    default: split_sweep<4>(pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fw, rv); break;
    }
}

// ---------------------------------------------------------------------------
// Hirschberg + Myers, breadth first.
//
// The reference recursion (hirschberg_myers, :569-638) pops segments from a
// LIFO stack, so it visits the recursion tree depth first and emits the base
// cases from the last (rightmost) to the first.  A segment's split column
// depends only on its own ranges, so the tree can be built level by level
// instead: the frontier is the in-order list of the current segments; every
// level computes the split column of each segment that is not a base case and
// replaces it by its two halves; when only base cases are left they are
// emitted from the last to the first, which is the reference's output order.
// The stack never holds more than the recursion depth + 1 <= 16 entries for
// queries of up to 16384 bases, so the reference's 64-entry overflow case
// cannot occur and is not modelled.
//
// Building the tree by levels lets the many short segments of the deep levels
// share a wave: a "pack" puts the forward and reverse halves of several
// segments side by side in the lanes of one Myers block (one lane group per
// half, one 32-row word per lane), with the carry look-ahead and the one-bit
// shift cut at the group boundaries and the target letter read per lane.

// frontier entry: query rows [qb, qe), target columns [tb, te)
__device__ __forceinline__ uint4 seg_pack(int qb, int qe, int tb, int te)
{
    return make_uint4(uint32_t(qb), uint32_t(qe), uint32_t(tb), uint32_t(te));
}

// base case kinds (:577-611): 1 no target, 2 no query, 3 one query base,
// 4 full Myers; 0: split
__device__ __forceinline__ int base_kind(int m, int Ts, int64_t max_elems)
{
    if (Ts == 0)
        return 1;
    if (m == 0)
        return 2;
    if (m == 1)
        return 3;
    const int nw = (m + kWordBits - 1) / kWordBits;
    if (m < kFullMyers && int64_t(Ts + 1) * nw <= max_elems)
        return 4;
    return 0;
}

// One packed segment: rows [qb, qe) split at qm, target [tb, te); its split
// scores at buffer offset boff (Ts + 1 entries each), frontier entry f.
struct PackSeg
{
    int32_t qb, qm, qe, tb, te, f, boff, pad;
};

// Both sweeps of up to 32 small segments in one pass: lane group F of a
// segment holds the words of rows [qb, qm) (forward), group R those of rows
// [qm, qe) of the reversed query.  fw / rv + boff receive the scores of
// columns 0..Ts as split_sweep does for one segment.
template <typename PatPtr, typename TcPtr, typename Buf>
__device__ void packed_split_sweep(PatPtr pat, int pat_words, int Q,
                                   const GWAMD_LDS PackSeg* segs, int nseg, TcPtr tcod, int lane,
                                   Buf fw, Buf rv)
{
    // this lane's group
    int g_ts = -1, g_tb = 0, g_te = 0, g_w = 0, g_m = 0, g_boff = 0, g_off = 0;
    bool g_rev = false, is_start = false, is_last = false;
    int lo = 0, tmax = 0;
    for (int s = 0; s < nseg; s++)
    {
        const int qb = segs[s].qb, qm = segs[s].qm, qe = segs[s].qe, tb = segs[s].tb, te = segs[s].te;
        const int mf = qm - qb, mr = qe - qm;
        const int wf = (mf + kWordBits - 1) / kWordBits, wr = (mr + kWordBits - 1) / kWordBits;
        tmax = max(tmax, te - tb);
        if (lane >= lo && lane < lo + wf)
        {
            g_ts = te - tb, g_tb = tb, g_te = te, g_w = lane - lo, g_m = mf, g_boff = segs[s].boff;
            g_rev = false, g_off = qb, is_start = lane == lo, is_last = lane == lo + wf - 1;
        }
        else if (lane >= lo + wf && lane < lo + wf + wr)
        {
            g_ts = te - tb, g_tb = tb, g_te = te, g_w = lane - lo - wf, g_m = mr, g_boff = segs[s].boff;
            g_rev = true, g_off = Q - qe, is_start = lane == lo + wf, is_last = lane == lo + wf + wr - 1;
        }
        lo += wf + wr;
    }
    const bool valid  = g_ts >= 0;
    const uint64_t act = __builtin_amdgcn_ballot_w64(valid);
    // carries and shifted bits stop at group boundaries
    const uint64_t cut = act & ~__builtin_amdgcn_ballot_w64(is_last);
    const uint32_t start_bit = is_start ? 1u : 0u;
    const uint32_t hisel     = lane >= 32 ? 1u : 0u;
    uint32_t e[4];
#pragma unroll
    for (int L = 0; L < 4; L++)
        e[L] = valid ? seg_pattern(pat, pat_words, g_off, g_w, (g_rev ? 4 : 0) + L) : 0u;
    uint32_t pv = ~0u, mv = 0u;
    const int hb = (g_m - 1) & (kWordBits - 1);
    int score    = g_m;
    Buf out      = g_rev ? rv : fw;
    if (is_last)
        out[g_boff] = score;
    // the letter of column t for this lane, read one column ahead
    auto code_of = [&](int t) -> int {
        if (!valid || t > g_ts)
            return 0;
        return code_at(tcod, g_rev ? g_te - t : g_tb + t - 1);
    };
    int code = code_of(1);
    tmax     = uni(tmax);
    for (int t = 1; t <= tmax; t++)
    {
        const int next = code_of(t + 1);
        const uint32_t l2 = (code & 1) ? e[1] : e[0];
        const uint32_t h2 = (code & 1) ? e[3] : e[2];
        const uint32_t eq = (code & 2) ? h2 : l2;
        const uint32_t xv = eq | mv;
        uint32_t sum;
        const bool ov     = __builtin_add_overflow(eq & pv, pv, &sum);
        const uint64_t G  = __builtin_amdgcn_ballot_w64(ov) & cut;
        const uint64_t P  = __builtin_amdgcn_ballot_w64(sum == 0xffffffffu) & cut;
        const uint64_t GP = G | P;
        sum += mask_bit((GP + G) ^ GP ^ G, hisel, lane);
        const uint32_t xh = (sum ^ pv) | eq;
        uint32_t ph       = mv | ~(xh | pv);
        uint32_t mh       = pv & xh;
        score += int((ph >> hb) & 1u) - int((mh >> hb) & 1u);
        const uint64_t PH = __builtin_amdgcn_ballot_w64((ph >> 31) != 0u) & cut;
        const uint64_t MH = __builtin_amdgcn_ballot_w64((mh >> 31) != 0u) & cut;
        // the top row enters every group with +1 (:327-331)
        ph = (ph << 1) | mask_bit(PH << 1, hisel, lane) | start_bit;
        mh = (mh << 1) | mask_bit(MH << 1, hisel, lane);
        pv = mh | ~(xv | ph);
        mv = ph & xv;
        if (is_last && t <= g_ts)
            out[g_boff + t] = score;
        code = next;
    }
}

// Base case of one frontier entry, emitted at path + len (end -> start).
template <typename LeafFn>
__device__ int emit_base(int kind, int qb, int qe, int tb, int te, const char* q, const char* tg, int8_t* path,
                         int lane, LeafFn&& leaf)
{
    const int m  = qe - qb;
    const int Ts = te - tb;
    if (kind == 1)
    {
        for (int k = lane; k < m; k += kWave)
            path[k] = kDeletion;
        return m;
    }
    if (kind == 2)
    {
        for (int k = lane; k < Ts; k += kWave)
            path[k] = kInsertion;
        return Ts;
    }
    if (kind == 3)
    {
        // last target position equal to the query character (:477-508)
        const char c = q[qb];
        int found    = -1;
        for (int k0 = 0; k0 < Ts && found < 0; k0 += kWave)
        {
            const int k       = k0 + lane;
            const bool hit    = k < Ts && tg[te - 1 - k] == c; // raw characters
            const uint64_t hm = __builtin_amdgcn_ballot_w64(hit);
            if (hm != 0)
                found = k0 + __builtin_ctzll(hm);
        }
        for (int k = lane; k < Ts; k += kWave)
        {
            int8_t st = k == found ? kMatch : kInsertion;
            if (found < 0 && k == Ts - 1)
                st = kMismatch;
            path[k] = st;
        }
        return Ts;
    }
    return leaf(qb, qe, tb, te, path);
}

// Full-Myers base case of a segment shorter than 63 rows (one 64-bit word;
// hirschberg_myers_compute_path / append_myers_backtrace, :372-392,
// :100-160), run by ONE lane (each lane of the wave takes one base case of
// the frontier), with the column state in the lane's own stretch of the slot
// and the path (end -> start) in its own stretch of path scratch.
template <typename PatPtr, typename TcPtr>
__device__ int leaf_lane(PatPtr pat, int pat_words, int qb, int qe,
                         TcPtr tcod, int tb, int te, uint64_t* lpv, uint64_t* lmv, int32_t* lsc,
                         int8_t* path)
{
    const int m         = qe - qb;
    const int T         = te - tb;
    const uint64_t full = (uint64_t(1) << m) - 1;
    uint64_t e[4];
    {
        const int k  = qb >> 5;
        const int sh = qb & 31;
#pragma unroll
        for (int L = 0; L < 4; L++)
        {
            const uint64_t w0 = k < pat_words ? pat[k * 8 + L] : 0u;
            const uint64_t w1 = k + 1 < pat_words ? pat[(k + 1) * 8 + L] : 0u;
            const uint64_t w2 = k + 2 < pat_words ? pat[(k + 2) * 8 + L] : 0u;
            uint64_t r        = (w0 | (w1 << 32)) >> sh;
            if (sh != 0)
                r |= w2 << (64 - sh);
            e[L] = r & full;
        }
    }
    uint64_t pv = full, mv = 0;
    int score   = m;
    lpv[0]      = pv;
    lmv[0]      = mv;
    lsc[0]      = score;
    for (int t = 1; t <= T; t++)
    {
        const int code    = code_at(tcod, tb + t - 1);
        const uint64_t lo = (code & 1) ? e[1] : e[0];
        const uint64_t hi = (code & 1) ? e[3] : e[2];
        const uint64_t eq = (code & 2) ? hi : lo;
        const uint64_t xv = eq | mv;
        const uint64_t xh = (((eq & pv) + pv) ^ pv) | eq;
        uint64_t ph       = mv | ~(xh | pv);
        uint64_t mh       = pv & xh;
        score += int((ph >> (m - 1)) & 1u) - int((mh >> (m - 1)) & 1u);
        ph     = (ph << 1) | 1u;
        mh     = mh << 1;
        pv     = (mh | ~(xv | ph)) & full;
        mv     = (ph & xv) & full;
        lpv[t] = pv;
        lmv[t] = mv;
        lsc[t] = score;
    }
    // D(i, j) = D(m, j) - sum of vertical deltas of rows i+1..m
    auto D = [&](int i, int j) -> int {
        if (i == 0)
            return j;
        const uint64_t hm = full & ~((uint64_t(1) << i) - 1);
        return lsc[j] - __builtin_popcountll(lpv[j] & hm) + __builtin_popcountll(lmv[j] & hm);
    };
    int i = m, j = T, pos = 0;
    int s = D(i, j);
    while (i > 0 && j > 0)
    {
        const int above = D(i - 1, j);
        const int diag  = D(i - 1, j - 1);
        const int left  = D(i, j - 1);
        int8_t r;
        if (left + 1 == s) // insertion, then deletion, then diagonal (:118-160)
        {
            r = kInsertion;
            s = left;
            --j;
        }
        else if (above + 1 == s)
        {
            r = kDeletion;
            s = above;
            --i;
        }
        else
        {
            r = diag == s ? kMatch : kMismatch;
            s = diag;
            --i;
            --j;
        }
        path[pos++] = r;
    }
    for (int k = 0; k < i; k++)
        path[pos + k] = kDeletion;
    pos += i;
    for (int k = 0; k < j; k++)
        path[pos + k] = kInsertion;
    return pos + j;
}

// ---------------------------------------------------------------------------
// Hirschberg + Myers (hirschberg_myers, :569-638), one wave per pair.
// LONG (queries over 16,384 or targets over 65,535 bases): query patterns in
// the HBM slot instead of LDS, 32-bit split scores, and halves taller than
// kMaxChunks blocks swept in stripes (half_sweep_striped).
// 4 waves per SIMD: 120 VGPRs instead of 152 (3 waves), no VGPR spills; the
// LDS image (~9.4 KB at 5 kb pairs) allows 17 workgroups per CU.  Measured
// (gpurun_out/r4l): 243.6k -> 261.6k alignments/s on config D; 5 waves per
// SIMD (96 VGPRs, spills) 202k.
template <bool LONG>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4))) hm_kernel(Args a)
{
    using SC = typename std::conditional<LONG, uint32_t, uint16_t>::type; // split score
    using PatPtr = typename std::conditional<LONG, const uint32_t*, const GWAMD_LDS uint32_t*>::type;
    // target letter codes: LDS; in long mode a generic pointer, to LDS when the
    // target's codes fit it (a.ws_tcod_off < 0), else to the HBM slot
    using TcW = typename std::conditional<LONG, uint32_t*, GWAMD_LDS uint32_t*>::type;
    extern __shared__ __align__(16) uint8_t lds[];
    const int lane                  = threadIdx.x;
    GWAMD_LDS uint8_t* base         = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint8_t* scratch      = base + a.lds_scratch_off;
    // split scores of segments up to kSplitLds columns (wider ones in HBM)
    GWAMD_LDS SC* fwl               = (GWAMD_LDS SC*)(scratch);
    GWAMD_LDS SC* rvl               = fwl + kSplitLds;
    GWAMD_LDS PackSeg* pack         = (GWAMD_LDS PackSeg*)(base + a.lds_stack_off);
    uint8_t* ws                     = a.ws + size_t(blockIdx.x) * size_t(a.ws_slot_bytes);
    // (global-typed: the split sweeps are called, not inlined, and a flat
    // store there makes every LDS wait of the sweep wait for it)
    GWAMD_GLB SC* fwg = (GWAMD_GLB SC*)(ws + a.ws_split_off);
    GWAMD_GLB SC* rvg = fwg + (a.stride + 1 + kWave);
    int8_t* hbuf  = reinterpret_cast<int8_t*>(ws + a.ws_hbuf_off); // LONG: stripe hand-over
    uint32_t* patw = reinterpret_cast<uint32_t*>(ws + a.ws_pat_off); // LONG: query patterns
    PatPtr pat;
    TcW tcod;
    if constexpr (LONG)
    {
        pat  = patw;
        tcod = a.ws_tcod_off >= 0 ? reinterpret_cast<uint32_t*>(ws + a.ws_tcod_off)
                                  : (uint32_t*)((GWAMD_LDS uint32_t*)(base + a.lds_target_off));
    }
    else
    {
        pat  = (GWAMD_LDS uint32_t*)(base + a.lds_pat_off);
        tcod = (GWAMD_LDS uint32_t*)(base + a.lds_target_off);
    }
    // the two frontier buffers by select, not through an array of pointers
    // (which would leave their accesses flat)
    uint4* const front0 = reinterpret_cast<uint4*>(ws + a.ws_front_off);
    uint4* const front1 = front0 + a.front_cap;
    auto front          = [&](int c) { return c ? front1 : front0; };
    int32_t* spl  = reinterpret_cast<int32_t*>(front1 + a.front_cap); // split column per entry
    // per-lane base cases: column state (pv, mv, score) and paths; (path
    // offset, length) per frontier entry
    uint64_t* lcol_pv = reinterpret_cast<uint64_t*>(ws + a.ws_leaf_off);
    uint64_t* lcol_mv = lcol_pv + a.leaf_cols;
    int32_t* lcol_sc  = reinterpret_cast<int32_t*>(lcol_mv + a.leaf_cols);
    int2* lmeta       = reinterpret_cast<int2*>(lcol_sc + ((a.leaf_cols + 3) & ~1));
    int8_t* lpath     = reinterpret_cast<int8_t*>(lmeta + a.front_cap);
#ifdef GWAMD_ALN_PROFILE
    uint64_t pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

    for (int idx = blockIdx.x; idx < a.n; idx += gridDim.x)
    {
        GWAMD_PROF_T0(t_all);
        const char* q  = a.seqs + size_t(2 * idx) * a.stride;
        const char* tg = a.seqs + size_t(2 * idx + 1) * a.stride;
        const int Q    = uni(a.lens[2 * idx]);
        const int T    = uni(a.lens[2 * idx + 1]);
        int8_t* path   = a.paths + size_t(idx) * a.max_path_length;
        pack_target(tcod, tg, T, lane);
        if constexpr (LONG)
            build_patterns(patw, q, Q, lane); // read back after the fence below
        else
            build_patterns((GWAMD_LDS uint32_t*)(base + a.lds_pat_off), q, Q, lane);
        const int pat_words = (Q + kWordBits - 1) / kWordBits;
        if (lane == 0)
            front(0)[0] = seg_pack(0, Q, 0, T);
        __threadfence_block();
        wave_sync();
        int cur = 0, nf = 1;
        while (true)
        {
            // 1. split columns of this level's non-base segments
            GWAMD_PROF_T0(t_rev);
            int nsplit = 0, npk = 0, lanes_used = 0, boff = 0;
            auto flush = [&]() {
                if (npk == 0)
                    return;
                wave_sync();
                packed_split_sweep(pat, pat_words, Q, pack, npk, tcod, lane, fwg, rvg);
                __threadfence_block();
                wave_sync();
                for (int s = 0; s < npk; s++)
                {
                    const int Ts = uni(pack[s].te) - uni(pack[s].tb);
                    const int bo = uni(pack[s].boff);
                    const int bt = split_argmin(fwg + bo, rvg + bo, Ts, lane);
                    if (lane == 0)
                        spl[uni(pack[s].f)] = bt;
                }
                wave_sync();
                npk = 0, lanes_used = 0, boff = 0;
            };
            for (int f = 0; f < nf; f++)
            {
                const uint4 v  = front(cur)[f];
                const int qb   = uni(int(v.x)), qe = uni(int(v.y));
                const int tb   = uni(int(v.z)), te = uni(int(v.w));
                const int m    = qe - qb;
                const int Ts   = te - tb;
                if (base_kind(m, Ts, a.max_matrix_elems) != 0)
                    continue;
                nsplit++;
                const int qm = qb + m / 2;
                const int wf = (qm - qb + kWordBits - 1) / kWordBits;
                const int wr = (qe - qm + kWordBits - 1) / kWordBits;
                if (wf + wr <= kWave)
                {
                    if (lanes_used + wf + wr > kWave || npk == 32 || boff + Ts + 1 > a.stride + 1 + kWave)
                        flush();
                    if (lane == 0)
                    {
                        GWAMD_LDS PackSeg* ps = pack + npk;
                        ps->qb = qb, ps->qm = qm, ps->qe = qe, ps->tb = tb, ps->te = te, ps->f = f, ps->boff = boff;
                    }
                    npk++;
                    lanes_used += wf + wr;
                    boff += Ts + 1;
                    continue;
                }
                // a segment too large to share a block: both sweeps over
                // 1..4 blocks of 64 words (split_sweep)
                const int nblk = uni(((max(wf, wr)) + kWave - 1) / kWave);
#ifdef GWAMD_ALN_PROFILE
                pr[4] += uint64_t(Ts) * nblk;
#endif
                int bt;
                if (LONG && nblk > a.stripe_blocks)
                {
                    // halves over 8,192 rows (stripe_blocks = kMaxChunks; fewer
                    // in the parity tests): one striped sweep per half
                    half_sweep_striped(pat, pat_words, Q, qb, qm, false, tcod, tb, te, lane, fwg, hbuf, a.stripe_blocks);
                    half_sweep_striped(pat, pat_words, Q, qm, qe, true, tcod, tb, te, lane, rvg, hbuf, a.stripe_blocks);
                    bt = split_argmin(fwg, rvg, Ts, lane);
                }
                else if (Ts + 1 <= kSplitLds)
                {
                    run_split(nblk, pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fwl, rvl);
                    wave_sync();
                    bt = split_argmin(fwl, rvl, Ts, lane);
                }
                else
                {
                    run_split(nblk, pat, pat_words, Q, qb, qm, qe, tcod, tb, te, lane, fwg, rvg);
                    __threadfence_block();
                    wave_sync();
                    bt = split_argmin(fwg, rvg, Ts, lane);
                }
                if (lane == 0)
                    spl[f] = bt;
                wave_sync();
            }
            flush();
            __threadfence_block();
            wave_sync();
            GWAMD_PROF_ADD(pr[0], t_rev);
            if (nsplit == 0)
                break;
            // 2. next frontier: each split segment becomes its two halves, in order
            GWAMD_PROF_T0(t_fwd);
            int nn = 0;
            for (int f0 = 0; f0 < nf; f0 += kWave)
            {
                const int f      = f0 + lane;
                const bool in    = f < nf;
                const uint4 v    = in ? front(cur)[f] : make_uint4(0, 0, 0, 0);
                const int qb     = int(v.x), qe = int(v.y);
                const int tb     = int(v.z), te = int(v.w);
                const bool split = in && base_kind(qe - qb, te - tb, a.max_matrix_elems) == 0;
                const int cnt    = in ? (split ? 2 : 1) : 0;
                // exclusive prefix sum of cnt over the lanes
                int x = cnt;
#pragma unroll
                for (int d = 1; d < kWave; d <<= 1)
                {
                    const int y = __shfl_up(x, d);
                    x += lane >= d ? y : 0;
                }
                const int pos = nn + x - cnt;
                if (in)
                {
                    if (split)
                    {
                        const int qm = qb + (qe - qb) / 2;
                        const int tm = tb + int(spl[f]);
                        front(cur ^ 1)[pos]     = seg_pack(qb, qm, tb, tm);
                        front(cur ^ 1)[pos + 1] = seg_pack(qm, qe, tm, te);
                    }
                    else
                        front(cur ^ 1)[pos] = v;
                }
                nn += uni(__shfl(x, kWave - 1));
            }
            __threadfence_block();
            wave_sync();
            cur ^= 1;
            nf = nn;
            GWAMD_PROF_ADD(pr[1], t_fwd);
        }
        // 3. base cases.  The full-Myers ones (all but a few) are computed
        // one per lane, their paths into scratch; then every base case is
        // emitted from the last segment to the first.
        GWAMD_PROF_T0(t_leaf);
        {
            int coff = 0, poff = 0;
            for (int f0 = 0; f0 < nf; f0 += kWave)
            {
                const int f   = f0 + lane;
                const bool in = f < nf;
                const uint4 v = in ? front(cur)[f] : make_uint4(0, 0, 0, 0);
                const int qb = int(v.x), qe = int(v.y);
                const int tb = int(v.z), te = int(v.w);
                const bool full_myers = in && base_kind(qe - qb, te - tb, a.max_matrix_elems) == 4;
                // scratch stretches: columns 0..Ts, path up to m + Ts states
                int cc = full_myers ? te - tb + 1 : 0, pc = full_myers ? qe - qb + te - tb : 0;
                int xc = cc, xp = pc;
#pragma unroll
                for (int d = 1; d < kWave; d <<= 1)
                {
                    const int yc = __shfl_up(xc, d), yp = __shfl_up(xp, d);
                    xc += lane >= d ? yc : 0;
                    xp += lane >= d ? yp : 0;
                }
                const int mc = coff + xc - cc, mp = poff + xp - pc;
#ifdef GWAMD_ALN_PROFILE
                pr[5] += uni(__shfl(xc, kWave - 1));
                pr[6] += __builtin_popcountll(__builtin_amdgcn_ballot_w64(full_myers));
#endif
                if (full_myers)
                {
                    const int n = leaf_lane(pat, pat_words, qb, qe, tcod, tb, te, lcol_pv + mc, lcol_mv + mc,
                                            lcol_sc + mc, lpath + mp);
                    lmeta[f] = make_int2(mp, n);
                }
                coff += uni(__shfl(xc, kWave - 1));
                poff += uni(__shfl(xp, kWave - 1));
            }
        }
        __threadfence_block();
        wave_sync();
        int len = 0;
        for (int f = nf - 1; f >= 0; f--)
        {
            const uint4 v = front(cur)[f];
            const int qb  = uni(int(v.x)), qe = uni(int(v.y));
            const int tb  = uni(int(v.z)), te = uni(int(v.w));
            const int kind = base_kind(qe - qb, te - tb, a.max_matrix_elems);
            if (kind == 4)
            {
                const int2 md = lmeta[f];
                const int mp  = uni(md.x), n = uni(md.y);
                for (int k = lane; k < n; k += kWave)
                    path[len + k] = lpath[mp + k];
                len += n;
            }
            else
                len += emit_base(kind, qb, qe, tb, te, q, tg, path + len, lane,
                                 [&](int, int, int, int, int8_t*) -> int { return 0; });
        }
        wave_sync();
        GWAMD_PROF_ADD(pr[2], t_leaf);
        if (lane == 0)
            a.path_len[idx] = len;
        wave_sync();
        GWAMD_PROF_ADD(pr[3], t_all);
    }
#ifdef GWAMD_ALN_PROFILE
    if (lane == 0)
        for (int k = 0; k < 8; k++)
            atomicAdd(&gwamd_aln_prof[k], (unsigned long long)pr[k]);
#endif
}

// ---------------------------------------------------------------------------
// Full Myers (myers_compute_score_matrix_kernel + myers_backtrace,
// myers_gpu.cu:95-375): per (word, column) pv, mv and the score of the word's
// last row in the workgroup's HBM slot, then the backtrace on the wave.
// Queries over kMaxChunks blocks (8,192 bases) are swept in stripes of
// kMaxChunks blocks, top to bottom, each over all columns; the horizontal
// delta leaving a stripe's last row at every column reaches the next stripe
// through a per-column int8 buffer in the slot (written and read back by the
// same lane).  LONG: query patterns in the slot, target letter codes through
// a generic pointer (LDS, or the slot for targets too long for LDS).
constexpr int kTbW = 4;  // full-Myers backtrace tile: words
constexpr int kTbC = 64; // and columns (12 B per entry in LDS)

template <bool LONG>
__global__ void __launch_bounds__(kWave) myers_kernel(Args a)
{
    using PatPtr = typename std::conditional<LONG, const uint32_t*, const GWAMD_LDS uint32_t*>::type;
    using TcW    = typename std::conditional<LONG, uint32_t*, GWAMD_LDS uint32_t*>::type;
    extern __shared__ __align__(16) uint8_t lds[];
    const int lane          = threadIdx.x;
    GWAMD_LDS uint8_t* base = (GWAMD_LDS uint8_t*)(lds);
    uint8_t* ws             = a.ws + size_t(blockIdx.x) * size_t(a.ws_slot_bytes);
    int8_t* hbuf            = reinterpret_cast<int8_t*>(ws + a.ws_hbuf_off);
    uint32_t* patw          = reinterpret_cast<uint32_t*>(ws + a.ws_pat_off);
    PatPtr pat;
    TcW tcod;
    if constexpr (LONG)
    {
        pat  = patw;
        tcod = a.ws_tcod_off >= 0 ? reinterpret_cast<uint32_t*>(ws + a.ws_tcod_off)
                                  : (uint32_t*)((GWAMD_LDS uint32_t*)(base + a.lds_target_off));
    }
    else
    {
        pat  = (GWAMD_LDS uint32_t*)(base + a.lds_pat_off);
        tcod = (GWAMD_LDS uint32_t*)(base + a.lds_target_off);
    }
    const int stripe_words = kMaxChunks * kWave;
#ifdef GWAMD_ALN_PROFILE
    // [0] forward (score matrix) cycles, [1] backtrace cycles, [3] total,
    // [4] column-blocks, [5] backtrace steps
    uint64_t pr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

    for (int idx = blockIdx.x; idx < a.n; idx += gridDim.x)
    {
        GWAMD_PROF_T0(t_all);
        const char* q  = a.seqs + size_t(2 * idx) * a.stride;
        const char* tg = a.seqs + size_t(2 * idx + 1) * a.stride;
        const int Q    = uni(a.lens[2 * idx]);
        const int T    = uni(a.lens[2 * idx + 1]);
        int8_t* path   = a.paths + size_t(idx) * a.max_path_length;
        pack_target(tcod, tg, T, lane);
        if constexpr (LONG)
            build_patterns(patw, q, Q, lane);
        else
            build_patterns((GWAMD_LDS uint32_t*)(base + a.lds_pat_off), q, Q, lane);
        const int nw = (Q + kWordBits - 1) / kWordBits;
        __threadfence_block();
        wave_sync();
        // (word, column) entry t * nwp + w; the row stride is padded to whole
        // 128-B lines and the pad words are stored too, so every line a
        // column writes is written whole by one store (no partial lines for
        // the L2 to fill from HBM)
        const int nwp = (nw + 31) & ~31;
        uint32_t* wpv = reinterpret_cast<uint32_t*>(ws);
        uint32_t* wmv = wpv + size_t(nwp) * (T + 1);
        int32_t* wsc  = reinterpret_cast<int32_t*>(wmv + size_t(nwp) * (T + 1));
        GWAMD_PROF_T0(t_fwd);
        const uint32_t hisel    = lane >= 32 ? 1u : 0u;
        const uint32_t lane0bit = lane == 0 ? 1u : 0u;
        const int gl            = nw - 1;               // last word of the query
        const int ghb           = (Q - 1) % kWordBits;  // its last row
        for (int w0 = 0; w0 < nw; w0 += stripe_words)
        {
            const int sw            = min(stripe_words, nw - w0);
            const bool first        = w0 == 0;
            const bool last_stripe  = w0 + sw == nw;
            const int nch           = uni((sw + kWave - 1) / kWave);
            const int lw            = sw - 1;
            const int lc            = lw / kWave;
            const int ll            = lw % kWave;
            const int hb            = last_stripe ? ghb : kWordBits - 1;
            const int wend          = last_stripe ? nwp : w0 + sw; // stored words (incl. the pad)
            MyersBlock B[kMaxChunks];
            int score[kMaxChunks];
#pragma unroll
            for (int c = 0; c < kMaxChunks; c++)
            {
                const int w      = w0 + c * kWave + lane;
                const bool valid = c < nch && w < w0 + sw;
#pragma unroll
                for (int L = 0; L < 4; L++)
                    B[c].e[L] = valid ? seg_pattern(pat, nw, 0, w, L) : 0u;
                B[c].pv  = ~0u;
                B[c].mv  = 0u;
                B[c].act = __builtin_amdgcn_ballot_w64(valid);
                score[c] = min((w + 1) * kWordBits, Q); // myers_gpu.cu:341
                if (c < nch && w < wend)
                {
                    wpv[w] = ~0u;
                    wmv[w] = 0u;
                    wsc[w] = score[c];
                }
            }
            int tv = 0, hv = 1, ho = 0;
            for (int t = 1; t <= T; t++)
            {
                const int tl = (t - 1) & (kWave - 1);
                if (tl == 0)
                {
                    // next 64 columns: letter codes and the deltas entering the stripe
                    const int x = t + lane;
                    tv          = x <= T ? code_at(tcod, x - 1) : 0;
                    hv          = (!first && x <= T) ? int(hbuf[x]) : 1; // first stripe: the top row's +1
                }
                const int code = uni(__builtin_amdgcn_readlane(tv, tl));
                int h          = uni(__builtin_amdgcn_readlane(hv, tl));
#pragma unroll
                for (int c = 0; c < kMaxChunks; c++)
                {
                    if (c < nch)
                    {
                        const int w = w0 + c * kWave + lane;
                        int own     = 0;
                        h = myers_block_step<true>(B[c], code, h, c == lc, ll, hb, lane, hisel, lane0bit,
                                                   w == gl ? ghb : 31, &own);
                        score[c] += own;
                        if (w < wend)
                        {
                            wpv[size_t(t) * nwp + w] = B[c].pv;
                            wmv[size_t(t) * nwp + w] = B[c].mv;
                            wsc[size_t(t) * nwp + w] = score[c];
                        }
                    }
                }
                if (!last_stripe)
                {
                    // the delta leaving this stripe's last row, for the next stripe
                    ho = lane == tl ? h : ho;
                    if (tl == kWave - 1 || t == T)
                    {
                        const int x = t - tl + lane;
                        if (x <= T)
                            hbuf[x] = int8_t(ho);
                    }
                }
            }
            __threadfence_block();
            wave_sync();
        }
        __threadfence_block();
        wave_sync();
        GWAMD_PROF_ADD(pr[0], t_fwd);
#ifdef GWAMD_ALN_PROFILE
        pr[4] += uint64_t(T) * uint64_t((nw + kWave - 1) / kWave);
#endif
        GWAMD_PROF_T0(t_bt);
        // backtrace (myers_backtrace, myers_gpu.cu:181-245).  The walk's
        // windows read words (i-9)/32 .. (i-1)/32 of columns j-8 .. j; a tile
        // of kTbW words x kTbC columns ending at the current cell is staged in
        // LDS with one round of lane-parallel loads and refilled when a window
        // leaves it (about every 55 steps), so a step costs LDS reads, not HBM
        // latency.
        const uint32_t last_mask = (Q % kWordBits) != 0 ? (1u << (Q % kWordBits)) - 1u : ~0u;
        GWAMD_LDS uint32_t* tpv  = (GWAMD_LDS uint32_t*)(base + a.lds_scratch_off);
        GWAMD_LDS uint32_t* tmv  = tpv + kTbW * kTbC;
        GWAMD_LDS int32_t* tsc   = (GWAMD_LDS int32_t*)(tmv + kTbW * kTbC);
        int tw0 = 0, tc0 = 0;
        auto refill = [&](int i, int j) {
            tw0 = max(0, (i - 1) / kWordBits - (kTbW - 1));
            tc0 = max(0, j - (kTbC - 1));
            wave_sync(); // the previous tile's readers are done
#pragma unroll
            for (int e0 = 0; e0 < kTbW * kTbC; e0 += kWave)
            {
                const int e = e0 + lane;
                const int c = tc0 + e / kTbW, w = tw0 + e % kTbW;
                if (c <= j && w < nw)
                {
                    const size_t o = size_t(c) * nwp + w;
                    tpv[e]         = wpv[o];
                    tmv[e]         = wmv[o];
                    tsc[e]         = wsc[o];
                }
            }
            wave_sync();
        };
        int i = Q, j = T, pos = 0;
        // the walk in 8 x 8 windows (as ukkonen_kernel): lane 8a + b takes
        // cell (i0 - a, j0 - b), computes its value from the tile (row 0 is
        // j) and, from its three neighbours (ds_bpermute), its move, which
        // depends on the cell alone (its value is the walk's running score);
        // the walk follows next-lane links until the window's last row or
        // column, i = 0 or j = 0, and the visited lanes store their moves at
        // their rank (a + b grows by 1 or 2 per step)
        {
            const int wa = lane >> 3, wb = lane & 7;
            if (i > 0 && j > 0)
                refill(i, j);
            while (i > 0 && j > 0)
            {
                if ((max(i - 9, 1) - 1) / kWordBits < tw0 || max(j - 8, 0) < tc0)
                    refill(i, j);
                const int ci = i - wa, cj = j - wb;
                int v        = cj;
                if (ci > 0)
                {
                    const int wi  = (ci - 1) / kWordBits;
                    const int bi  = (ci - 1) % kWordBits;
                    uint32_t mask = (~1u) << bi;
                    if (wi == nw - 1)
                        mask &= last_mask;
                    const int e = min(max((cj - tc0) * kTbW + (wi - tw0), 0), kTbW * kTbC - 1);
                    v           = tsc[e] - __builtin_popcount(mask & tpv[e]) + __builtin_popcount(mask & tmv[e]);
                }
                const int up      = __builtin_amdgcn_ds_bpermute(4 * (lane + 8), v);
                const int dg      = __builtin_amdgcn_ds_bpermute(4 * (lane + 9), v);
                const int lf      = __builtin_amdgcn_ds_bpermute(4 * (lane + 1), v);
                const bool mv_ins = lf + 1 == v;
                const bool mv_del = !mv_ins && up + 1 == v;
                const int r       = mv_ins ? int(kInsertion) : (mv_del ? int(kDeletion) : (dg == v ? int(kMatch) : int(kMismatch)));
                const bool term   = wa == 7 || wb == 7 || ci <= 0 || cj <= 0;
                const int nxt     = term ? lane : lane + (mv_ins ? 1 : (mv_del ? 8 : 9));
                uint64_t visited  = 0;
                uint32_t sums     = 0;
                int o = 0, steps = 0;
                while (true)
                {
                    const int nx = uni(__builtin_amdgcn_readlane(nxt, o));
                    if (nx == o)
                        break;
                    visited |= 1ull << o;
                    sums |= 1u << ((o >> 3) + (o & 7));
                    ++steps;
                    o = nx;
                }
                if ((visited >> lane) & 1ull)
                    path[pos + __builtin_popcount(sums & ((1u << (wa + wb)) - 1u))] = int8_t(r);
                pos += steps;
                i -= o >> 3;
                j -= o & 7;
            }
        }
        for (int k = lane; k < i; k += kWave)
            path[pos + k] = kDeletion;
        pos += i;
        for (int k = lane; k < j; k += kWave)
            path[pos + k] = kInsertion;
        pos += j;
        GWAMD_PROF_ADD(pr[1], t_bt);
#ifdef GWAMD_ALN_PROFILE
        pr[5] += uint64_t(pos);
#endif
        if (lane == 0)
            a.path_len[idx] = pos;
        wave_sync();
        GWAMD_PROF_ADD(pr[3], t_all);
    }
#ifdef GWAMD_ALN_PROFILE
    if (lane == 0)
        for (int k = 0; k < 8; k++)
            atomicAdd(&gwamd_aln_prof[k], (unsigned long long)pr[k]);
#endif
}

} // namespace aln
} // namespace gwamd

extern "C" hipError_t gwamd_internal_align_launch(const gwamd::aln::Args* a, int algo, int grid, hipStream_t stream)
{
    using namespace gwamd::aln;
    if (a->n <= 0)
        return hipSuccess;
    if (algo == 0 && a->long_mode)
        hipLaunchKernelGGL(hm_kernel<true>, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    else if (algo == 0)
        hipLaunchKernelGGL(hm_kernel<false>, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    else if (a->long_mode)
        hipLaunchKernelGGL(myers_kernel<true>, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    else
        hipLaunchKernelGGL(myers_kernel<false>, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    return hipGetLastError();
}

extern "C" hipError_t gwamd_internal_align_occupancy(int algo, int lds_bytes, int* blocks_per_cu)
{
    using namespace gwamd::aln;
    if (algo == 0)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, hm_kernel<false>, kWave, size_t(lds_bytes));
    if (algo == 100)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, hm_kernel<true>, kWave, size_t(lds_bytes));
    if (algo == 101)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, myers_kernel<true>, kWave,
                                                            size_t(lds_bytes));
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, myers_kernel<false>, kWave, size_t(lds_bytes));
}

#ifdef GWAMD_ALN_PROFILE
// Diagnostic build only: read (and optionally clear) the hm_kernel counters.
extern "C" int gwamd_internal_aln_prof(unsigned long long* out8, int reset)
{
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(gwamd_aln_prof), 8 * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    if (reset)
    {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(gwamd_aln_prof), z, sizeof(z)) != hipSuccess)
            return -1;
    }
    return 0;
}
#endif

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

#include "poa_wave.hpp"

namespace gwamd
{
namespace poa
{

constexpr int kBandRing  = 16; // LDS ring rows (power of two)
constexpr int kBandTile  = 64; // traceback tile rows
constexpr uint32_t kNpEsc = 63;

// rec_a: base (8) | np (6; 63 = escape: read the graph) | sink (1) | spill (1) | band_start/4 (16)
// rec_b: bit 31 clear: distance to pred 0 | distance to pred 1 << 16 (both < 32768);
//        bit 31 set: offset of the row's predecessor list in xl (np >= 3 or far predecessors)
__device__ __forceinline__ int ra_base(uint32_t a) { return int(a & 0xffu); }
__device__ __forceinline__ int ra_np(uint32_t a) { return int((a >> 8) & 63u); }
__device__ __forceinline__ bool ra_sink(uint32_t a) { return (a >> 14) & 1u; }
__device__ __forceinline__ bool ra_spill(uint32_t a) { return (a >> 15) & 1u; }
__device__ __forceinline__ int ra_bs(uint32_t a) { return int(a >> 16) << 2; }

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
    int32_t* col0;   // [score_rows] F(r, 0) of rows with band_start 0
    uint8_t* flags;  // [score_rows] bit 0: row stored in the spill rows
    int32_t* xl;     // [xl_cap] predecessor rows of rows with np >= 3 (or far)
    int xl_cap;
};

// k-th predecessor row of row r (0 = the virtual row 0) and the predecessor count
template <typename SizeT>
__device__ __forceinline__ int band_pred2(const WinGraph<SizeT>& g, const BandAux& X, int r, uint32_t a, uint32_t b,
                                          int k)
{
    const int np = ra_np(a);
    if (np == 0)
        return 0;
    if (np == int(kNpEsc))
        return pred_row(g, int(g.sorted[r - 1]), k);
    if (b >> 31)
        return int(X.xl[(b & 0x7fffffffu) + uint32_t(k)]);
    return r - int(k == 0 ? (b & 0xffffu) : (b >> 16));
}

template <typename SizeT>
__device__ __forceinline__ int band_np2(const WinGraph<SizeT>& g, int r, uint32_t a, uint32_t b)
{
    const int np = ra_np(a);
    return np == int(kNpEsc) ? int(g.in_cnt[int(g.sorted[r - 1])]) : np;
}

// Row program of rows 1..V (after every topological sort).  Loads are batched
// kRP rows per lane for memory-level parallelism; spill flags (a successor
// reads the row from kBandRing or more rows later) are collected as LDS bytes
// from the successor's side and folded into rec_a in a second pass.
template <typename SizeT>
__device__ void band_row_program(const WinGraph<SizeT>& g, int V, const Band& B, const BandAux& X, int lane,
                                 GWAMD_LDS uint8_t* flags)
{
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
            p0[u] = int(g.pos[np[u] >= 1 ? e0[u] : 0]) + 1;
            p1[u] = int(g.pos[np[u] >= 2 ? e1[u] : 0]) + 1;
        }
#pragma unroll
        for (int u = 0; u < kRP; u++)
        {
            const int r      = r0 + u * kWave + lane;
            const bool valid = r <= V;
            const int n      = valid ? np[u] : 0;
            const bool near2 = n <= 2 && (n < 1 || r - p0[u] < 32768) && (n < 2 || r - p1[u] < 32768);
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
                        if (r - p0[u] >= kBandRing)
                            flags[p0[u]] = 1;
                    }
                    if (n >= 2)
                    {
                        bw |= uint32_t(r - p1[u]) << 16;
                        if (r - p1[u] >= kBandRing)
                            flags[p1[u]] = 1;
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
                        if (r - pk >= kBandRing)
                            flags[pk] = 1;
                    }
                    a |= (fit ? uint32_t(n) : kNpEsc) << 8;
                    bw = 0x80000000u | uint32_t(off);
                }
                X.reca[r] = a;
                X.recb[r] = bw;
            }
            xbase += total;
        }
    }
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    for (int r = lane + 1; r <= V; r += kWave)
        if (flags[r])
            X.reca[r] |= 1u << 15;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Predecessor values F(p, d + CPL*lane + c), c = 0..CPL (flat get_scores()
// reads, :123-173).  Lanes whose groups are cut read clamped garbage.
template <typename ScoreT, int CPL>
__device__ __forceinline__ void band_fetch(int p, int d, int r, const int (&Hp)[CPL], int prevF0, const ScoreT* ring,
                                           const ScoreT* spill, int rowsz, int gap, int minv, int lane,
                                           int (&F)[CPL + 1])
{
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
    const ScoreT* row = (r - p < kBandRing) ? ring + (p & (kBandRing - 1)) * rowsz : spill + size_t(p) * rowsz;
    const int gmax    = rowsz / CPL - 1;
    const int gi      = min(d / CPL + lane + 1, gmax);
    const ScoreT* q   = row + gi * CPL;
    F[0]              = int(q[-1]);
#pragma unroll
    for (int c = 0; c < CPL; c++)
        F[c + 1] = int(q[c]);
}

// Forward pass over rows 1..V.  Returns the end row (first sink with the
// strictly greatest get_score(row, L), :349-365).
template <typename ScoreT, typename SizeT, int CPL>
__device__ int band_forward(const WinGraph<SizeT>& g, const BandAux& X, int V, const uint8_t* read, int L,
                            const Band& B, const Scores sc, ScoreT* ring, ScoreT* spill, int rowsz, int lane)
{
    const int gap  = sc.gap;
    const int bw   = B.bw;
    const int minv = int(band_min_value<ScoreT>(sc));
    const int T0 = minv - sc.match, T1 = minv - sc.mismatch, T2 = minv - gap;
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
    int prevF0 = 0, prev_bs = 0;
    int best = INT_MIN, end_row = 0;
    const int minv_s = minv;
    wave_sync();

    uint32_t ca = 0, cb = 0, na = 0, nb = 0;
    if (1 + lane <= V)
        ca = X.reca[1 + lane], cb = X.recb[1 + lane];
    if (65 + lane <= V)
        na = X.reca[65 + lane], nb = X.recb[65 + lane];
    for (int r0 = 1; r0 <= V; r0 += kWave)
    {
        const int rend = min(V, r0 + kWave - 1);
        for (int r = r0; r <= rend; r++)
        {
            const uint32_t a = __builtin_amdgcn_readlane(ca, r - r0);
            const uint32_t b = __builtin_amdgcn_readlane(cb, r - r0);
            const int bs     = ra_bs(a);
            const int gb     = ra_base(a);
            const int np  = band_np2<SizeT>(g, r, a, b);
            const int npp = np == 0 ? 1 : np;
            // read bases of this lane's cells: columns bs+1+t read read[bs+t]
            int sig[CPL];
            {
                const uint8_t* rp = read + bs + CPL * lane;
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    sig[c] = (int(rp[c]) == gb) ? sc.match : sc.mismatch;
            }
            int F0[CPL + 1], F1[CPL + 1];
            int d0 = 0, d1 = 0, p0 = 0, p1 = 0;
            int v[CPL];
#pragma unroll
            for (int c = 0; c < CPL; c++)
                v[c] = kNeg;
            int c0max = INT_MIN;
            for (int k = 0; k < npp; k++)
            {
                const int p  = np == 0 ? 0 : uniform(band_pred2<SizeT>(g, X, r, a, b, k));
                const int pb = (p == r - 1) ? prev_bs : (p == 0 ? 0 : B.start(p));
                const int d  = bs - pb;
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
                    d0 = d, p0 = p;
                }
                else if (k == 1)
                {
#pragma unroll
                    for (int c = 0; c <= CPL; c++)
                        F1[c] = Fk[c];
                    d1 = d, p1 = p;
                }
            }
            // column 0 (:219-245): F(r, 0) is the column-0 value when the band
            // starts at 0, else the minv initialize_band writes at index 0
            const int col0 = np == 0 ? gap : trunc_score<ScoreT>(c0max + gap);
            const int carry = bs == 0 ? col0 : minv;
            // horizontal closure, E domain: E(t) = H(t) - (t+1)*gap, E(-1) = carry
            int m[CPL];
            int run = lane == 0 ? carry : kNeg;
#pragma unroll
            for (int c = 0; c < CPL; c++)
            {
                run  = max(run, v[c] - egap[c]);
                m[c] = run;
            }
            const int incl = wave_incl_max_dpp(run);
            const int excl = __builtin_amdgcn_update_dpp(kNeg, incl, 0x138, 0xf, 0xf, false);
            int H[CPL];
#pragma unroll
            for (int c = 0; c < CPL; c++)
                H[c] = trunc_score<ScoreT>(max(m[c], excl) + egap[c]);
            // traceback codes (:367-477 with get_score(): minv beyond idx bw)
            const int vlim = L - bs - 1; // cells t <= vlim are columns <= L
            int code[CPL];
            bool found[CPL];
#pragma unroll
            for (int c = 0; c < CPL; c++)
                code[c] = 3, found[c] = false;
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
                    const int p  = uniform(band_pred2<SizeT>(g, X, r, a, b, k));
                    const int pb = (p == r - 1) ? prev_bs : (p == 0 ? 0 : B.start(p));
                    d            = bs - pb;
                    band_fetch<ScoreT, CPL>(p, d, r, Hp, prevF0, ring, spill, rowsz, gap, minv, lane, Fk);
                }
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    const int t  = CPL * lane + c;
                    const int gA = (d + t > bw) ? minv : Fk[c];
                    if (!found[c] && gA + sig[c] == H[c])
                        code[c] = k << 2, found[c] = true;
                }
            }
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
                    const int p  = uniform(band_pred2<SizeT>(g, X, r, a, b, k));
                    const int pb = (p == r - 1) ? prev_bs : (p == 0 ? 0 : B.start(p));
                    d            = bs - pb;
                    band_fetch<ScoreT, CPL>(p, d, r, Hp, prevF0, ring, spill, rowsz, gap, minv, lane, Fk);
                }
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    const int t  = CPL * lane + c;
                    const int gB = (d + t + 1 > bw) ? minv : Fk[c + 1];
                    if (!found[c] && gB + gap == H[c])
                        code[c] = (k << 2) | 1, found[c] = true;
                }
            }
            {
                int left = __builtin_amdgcn_update_dpp(carry, H[CPL - 1], 0x138, 0xf, 0xf, false);
#pragma unroll
                for (int c = 0; c < CPL; c++)
                {
                    if (!found[c] && left + gap == H[c])
                        code[c] = 2, found[c] = true;
                    left = H[c];
                }
            }
            // store codes (one byte per cell)
            {
                uint8_t* crow = X.codes + size_t(r) * bw + CPL * lane;
                if (CPL == 4)
                {
                    const uint32_t w4 = uint32_t(code[0]) | (uint32_t(code[1 % CPL]) << 8) |
                                        (uint32_t(code[2 % CPL]) << 16) | (uint32_t(code[3 % CPL]) << 24);
                    *reinterpret_cast<uint32_t*>(crow) = w4;
                }
                else
                {
#pragma unroll
                    for (int c = 0; c < CPL; c++)
                        crow[c] = uint8_t(code[c]);
                }
            }
            // end cell candidates (sinks in topological order, strict >)
            if (ra_sink(a))
            {
                int sval;
                if (L >= bs + 1 && L <= bs + bw)
                {
                    const int t  = L - bs - 1;
                    int hv       = H[0];
#pragma unroll
                    for (int c = 1; c < CPL; c++)
                        hv = (t % CPL == c) ? H[c] : hv;
                    sval = __builtin_amdgcn_readlane(hv, t / CPL);
                }
                else if (L == bs)
                    sval = carry;
                else
                    sval = minv_s;
                if (best < sval)
                    best = sval, end_row = r;
            }
            // rows an out-of-band traceback comparison could match (T values)
            bool tv = false;
#pragma unroll
            for (int c = 0; c < CPL; c++)
            {
                const int t = CPL * lane + c;
                tv |= t <= vlim && (H[c] == T0 || H[c] == T1 || H[c] == T2);
            }
            const bool tflag = __builtin_amdgcn_ballot_w64(tv) != 0;
            // ring row: position idx + CPL - 1
            ScoreT* rrow = ring + (r & (kBandRing - 1)) * rowsz;
            if (CPL == 4 && sizeof(ScoreT) == 4)
            {
                *reinterpret_cast<int4*>(rrow + CPL * (lane + 1)) = make_int4(H[0], H[1 % CPL], H[2 % CPL], H[3 % CPL]);
            }
            else
            {
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    rrow[CPL * (lane + 1) + c] = ScoreT(H[c]);
            }
            if (lane == 0)
                rrow[CPL - 1] = ScoreT(carry);
            if (ra_spill(a) || tflag)
            {
                ScoreT* srow = spill + size_t(r) * rowsz;
#pragma unroll
                for (int c = 0; c < CPL; c++)
                    srow[CPL * (lane + 1) + c] = ScoreT(H[c]);
                if (lane == 0)
                    srow[CPL - 1] = ScoreT(carry);
                const int pg = rowsz / CPL - (kWave + 1); // padding groups
                if (lane < pg)
                {
#pragma unroll
                    for (int c = 0; c < CPL; c++)
                        srow[CPL * (kWave + 1 + lane) + c] = ScoreT(minv);
                }
            }
            if (lane == 0)
            {
                X.flags[r] = uint8_t(tflag ? 1 : 0);
                if (bs == 0)
                    X.col0[r] = carry;
            }
            wave_sync();
#pragma unroll
            for (int c = 0; c < CPL; c++)
                Hp[c] = H[c];
            prevF0  = carry;
            prev_bs = bs;
        }
        ca = na, cb = nb;
        na = nb = 0;
        if (r0 + 2 * kWave + lane <= V)
            na = X.reca[r0 + 2 * kWave + lane], nb = X.recb[r0 + 2 * kWave + lane];
    }


    return end_row;
}

// get_score(row, col) semantics for the out-of-band traceback step.  Sets
// known = false for an in-band value that was not stored: such a value is
// not one of the T values, so no comparison with minv can match it.
template <typename ScoreT, int CPL>
__device__ int band_get_slow(int p, int col, const Band& B, const BandAux& X, const ScoreT* spill, int rowsz,
                             int gap, int minv, bool& known)
{
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
__device__ int band_traceback(const WinGraph<SizeT>& g, const BandAux& X, int V, const uint8_t* read, int L,
                              int end_row, const Band& B, const Scores sc, const ScoreT* spill, int rowsz,
                              uint8_t* tile, uint32_t* trec, SizeT* ag, SizeT* ar, int aln_cap,
                              int lane)
{
    const int bw    = B.bw;
    const int gap   = sc.gap;
    const int minv  = int(band_min_value<ScoreT>(sc));
    V               = uniform(V);
    L               = uniform(L);
    int i           = uniform(end_row), j = L;
    int prev_i = 0, prev_j = 0;
    int ti0 = INT_MIN / 2;
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
    while (!(i == 0 && j == 0) && loops < bound)
    {
        loops++;
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
            {
                ti0 = max(1, i - (kBandTile - 1));
                wave_sync();
                constexpr int kPer = kBandTile * 256 / 16 / kWave; // bw <= 256
                const int per_row  = bw / 16;
#pragma unroll
                for (int u = 0; u < kPer; u++)
                {
                    const int t   = u * kWave + lane;
                    const int tr  = t / per_row;
                    const int tc  = (t % per_row) * 16;
                    const int rr  = ti0 + tr;
                    const bool ok = tr < kBandTile && rr <= V;
                    uint4 q       = ok ? *reinterpret_cast<const uint4*>(X.codes + size_t(rr) * bw + tc)
                                       : make_uint4(0, 0, 0, 0);
                    if (tr < kBandTile)
                        *reinterpret_cast<uint4*>(tile + tr * bw + tc) = q;
                }
                {
                    const int rr = ti0 + lane;
                    if (lane < kBandTile)
                    {
                        trec[2 * lane]     = rr <= V ? X.reca[rr] : 0u;
                        trec[2 * lane + 1] = rr <= V ? X.recb[rr] : 0u;
                    }
                }
                wave_sync();
            }
            const uint32_t a = uint32_t(uniform(int(trec[2 * (i - ti0)])));
            const uint32_t b = uint32_t(uniform(int(trec[2 * (i - ti0) + 1])));
            const int bs     = ra_bs(a);
            if (j == 0)
            {
                // column 0: vertical moves only (get(i, -1) is minv)
                const int sij = bs == 0 ? int(X.col0[i]) : minv;
                const int np  = band_np2<SizeT>(g, i, a, b);
                const int npp = np == 0 ? 1 : np;
                for (int k = 0; k < npp && !found; k++)
                {
                    const int p   = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, k);
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
                    const int np = band_np2<SizeT>(g, i, a, b);
                    pi           = np == 0 ? 0 : uniform(band_pred2<SizeT>(g, X, i, a, b, code >> 2));
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
                    const int p = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, k);
                    bool kn;
                    const int gv = band_get_slow<ScoreT, CPL>(p, j - 1, B, X, spill, rowsz, gap, minv, kn);
                    if (kn && sij == gv + cost)
                        pi = p, pj = j - 1, found = true;
                }
                for (int k = 0; k < npp && !found; k++)
                {
                    const int p = np == 0 ? 0 : band_pred2<SizeT>(g, X, i, a, b, k);
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
            flush(n);
        i = prev_i;
        j = prev_j;
    }
    if ((n & (kWave - 1)) != 0)
        flush(n);
    wave_sync();
    if (bad || loops >= bound || n > aln_cap)
        return -1;
    return n;
}

template <typename ScoreT, typename SizeT, bool MSA, int CPL>
__global__ void __launch_bounds__(kWave) poa_window_kernel_band(Buffers b, Dims d, Scores sc)
{
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int sh_status;
    __shared__ int sh_len;

    const int w = blockIdx.x;
    if (w >= b.num_windows)
        return;
    const int lane = threadIdx.x;

    uint8_t* lread          = lds;
    GWAMD_LDS uint8_t* work = (GWAMD_LDS uint8_t*)(lds) + d.lds_ring_off;
    ScoreT* ring            = reinterpret_cast<ScoreT*>(lds + d.lds_ring_off);
    GWAMD_LDS uint8_t* shb  = (GWAMD_LDS uint8_t*)(lds) + d.lds_sh_off;
    uint8_t* tile           = lds + d.lds_ring_off;
    uint32_t* trec          = reinterpret_cast<uint32_t*>(tile + kBandTile * d.band_width);
    const int rowsz          = d.score_stride;

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
    ScoreT* spill    = static_cast<ScoreT*>(b.scores) + size_t(w) * d.score_rows * size_t(rowsz);
    uint8_t* aux     = b.codes + size_t(w) * size_t(d.aux_stride);
    BandAux X;
    X.codes          = aux;
    X.reca           = reinterpret_cast<uint32_t*>(aux + d.aux_reca_off);
    X.recb           = reinterpret_cast<uint32_t*>(aux + d.aux_recb_off);
    X.col0           = reinterpret_cast<int32_t*>(aux + d.aux_col0_off);
    X.flags          = aux + d.aux_flag_off;
    X.xl             = reinterpret_cast<int32_t*>(aux + d.aux_xl_off);
    X.xl_cap         = d.aux_xl_cap;
    int32_t* cscore  = b.cscore + w * mn;
    SizeT* cpred     = static_cast<SizeT*>(b.cpred) + w * mn * 4;
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
            band_row_program<SizeT>(g, V, B, X, lane, work);
            wave_sync();
            ph.lap<kPhRowProg>();
            cells += int64_t(V + 1) * (d.band_width + kBandPad);
            const int end_row =
                band_forward<ScoreT, SizeT, CPL>(g, X, V, lread, L, B, sc, ring, spill, rowsz, lane);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            ph.lap<kPhForward>();
            const int alen = band_traceback<ScoreT, SizeT, CPL>(g, X, V, lread, L, end_row, B, sc, spill, rowsz, tile,
                                                                trec, ag, ar, d.aln_cap, lane);
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
            {
                // add-alignment scratch in the work region, sized for this read
                auto a16             = [](int v) { return (v + 15) & ~15; };
                const int ls         = a16(L + 16);
                const int need       = 5 * ls + 2 * (V + L + 16) + 16;
                if (need <= d.lds_work_bytes)
                {
                    AddScratch AX;
                    AX.gid   = (GWAMD_LDS uint16_t*)(work);
                    AX.curr  = (GWAMD_LDS uint16_t*)(work + 2 * ls);
                    AX.kind  = work + 4 * ls;
                    AX.owner = (GWAMD_LDS uint16_t*)(work + 5 * ls);
                    AX.sh    = (GWAMD_LDS int*)(shb);
                    rc = add_alignment_parallel<SizeT, MSA>(g, nc, ag, ar, alen, L, lread, wts_g, s, ecov, ecovc,
                                                            seq_begin, d.max_seqs, AX, lane);
                }
            }
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
            if (rc == kSuccess)
            {
                if (!topsort_lds<SizeT>(g, nc, (GWAMD_LDS uint8_t*)(lds), d.lds_sh_off, (GWAMD_LDS int*)(shb),
                                        lane))
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

} // namespace poa
} // namespace gwamd

// Launch of the banded kernel (called by gwamd_internal_poa_launch).
extern "C" hipError_t gwamd_internal_poa_band_launch(const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d,
                                                     const gwamd::poa::Scores* sc, int score_bits, int size_bits,
                                                     int msa, hipStream_t stream)
{
    using namespace gwamd::poa;
    const dim3 grid(b->num_windows), blk(kWave);
    const size_t lb = size_t(d->lds_bytes);
#define GWAMD_BAND_LAUNCH(ST, ZT, MS, CPL)                                                                      \
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
#define GWAMD_BAND_CPL(ST, ZT, MS)          \
    if (d->lds_cpl == 4)                    \
        GWAMD_BAND_LAUNCH(ST, ZT, MS, 4)    \
    if (d->lds_cpl == 2)                    \
        GWAMD_BAND_LAUNCH(ST, ZT, MS, 2)    \
    return hipErrorInvalidConfiguration;
#define GWAMD_BAND_MSA(ST, ZT)              \
    if (msa)                                \
    {                                       \
        GWAMD_BAND_CPL(ST, ZT, true)        \
    }                                       \
    GWAMD_BAND_CPL(ST, ZT, false)
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
#undef GWAMD_BAND_CPL
#undef GWAMD_BAND_LAUNCH
}

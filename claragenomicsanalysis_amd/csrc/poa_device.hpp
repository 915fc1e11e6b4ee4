// Device-side building blocks of the POA kernels (shared by the global-memory
// kernel and the LDS-resident kernel in poa_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "poa_common.hpp"

namespace gwamd
{
namespace poa
{

constexpr int32_t kNeg = -(1 << 29); // "minus infinity" for int32 DP temporaries

template <typename SizeT>
struct WinGraph
{
    uint8_t* base;
    uint16_t* in_cnt;
    uint16_t* out_cnt;
    uint16_t* aln_cnt;
    uint16_t* cov;
    uint16_t* in_w;
    SizeT* in_e;
    SizeT* out_e;
    SizeT* aln;
    SizeT* sorted;
    SizeT* pos;
    int32_t max_nodes;
};

// Pointers reached through structs (WinGraph, Buffers fields copied into
// locals) lose their address space when a struct is passed to a call that is
// not inlined; flat accesses then count in both vmcnt and lgkmcnt, so every
// LDS wait also waits for outstanding global stores.  as_global() re-asserts
// the global space (an addrspacecast the compiler propagates).
template <typename T>
__device__ __forceinline__ T* glb(T* p)
{
    return (T*)((__attribute__((address_space(1))) T*)(p));
}

template <typename SizeT>
__device__ __forceinline__ WinGraph<SizeT> as_global(WinGraph<SizeT> g)
{
    g.base    = glb(g.base);
    g.in_cnt  = glb(g.in_cnt);
    g.out_cnt = glb(g.out_cnt);
    g.aln_cnt = glb(g.aln_cnt);
    g.cov     = glb(g.cov);
    g.in_w    = glb(g.in_w);
    g.in_e    = glb(g.in_e);
    g.out_e   = glb(g.out_e);
    g.aln     = glb(g.aln);
    g.sorted  = glb(g.sorted);
    g.pos     = glb(g.pos);
    return g;
}

__device__ __forceinline__ uint64_t now_ticks()
{
    return __builtin_amdgcn_s_memrealtime();
}

// Ordering point for code run by a single wave (LDS and global accesses of one
// wave complete in issue order; this only stops the compiler from moving
// memory operations across it).
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int uniform(int x)
{
    return __builtin_amdgcn_readfirstlane(x);
}

// Exclusive max-scan across the 64 lanes (lane 0 gets kNeg).
__device__ __forceinline__ int wave_excl_max(int v, int lane)
{
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1)
    {
        int t = __shfl_up(v, d, kWave);
        if (lane >= d)
            v = max(v, t);
    }
    int e = __shfl_up(v, 1, kWave);
    return lane == 0 ? kNeg : e;
}

__device__ __forceinline__ int wave_max(int v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1)
        v = max(v, __shfl_xor(v, d, kWave));
    return v;
}

// Row of the score matrix for predecessor slot p of node (cudapoa_nw.cuh:103).
template <typename SizeT>
__device__ __forceinline__ int pred_row(WinGraph<SizeT> g, int node, int p)
{
    g = as_global(g);
    return int(g.pos[int(g.in_e[node * kMaxEdges + p])]) + 1;
}

// The graph with global-typed pointers, for functions kept out of line (their
// struct arguments arrive with flat pointers, and a flat access counts against
// the LDS wait counter too): the anti-diagonal banded pass.
#ifndef GWAMD_GLB
#define GWAMD_GLB __attribute__((address_space(1)))
#endif
template <typename SizeT>
struct WinGraphG
{
    GWAMD_GLB const uint16_t* in_cnt;
    GWAMD_GLB const SizeT* in_e;
    GWAMD_GLB const SizeT* sorted;
    GWAMD_GLB const SizeT* pos;
};

template <typename SizeT>
__device__ __forceinline__ WinGraphG<SizeT> typed_graph(WinGraph<SizeT> g)
{
    WinGraphG<SizeT> t;
    t.in_cnt = (GWAMD_GLB const uint16_t*)(g.in_cnt);
    t.in_e   = (GWAMD_GLB const SizeT*)(g.in_e);
    t.sorted = (GWAMD_GLB const SizeT*)(g.sorted);
    t.pos    = (GWAMD_GLB const SizeT*)(g.pos);
    return t;
}

template <typename SizeT>
__device__ __forceinline__ int pred_row(const WinGraphG<SizeT>& g, int node, int p)
{
    return int(g.pos[int(g.in_e[node * kMaxEdges + p])]) + 1;
}

// ---------------------------------------------------------------------------
// Backbone from read 0 (cudapoa_kernels.cuh:171-209), lane-parallel.
template <typename SizeT, bool MSA>
__device__ void build_backbone(WinGraph<SizeT> g, const uint8_t* seq, const int8_t* w, int len, int lane,
                               uint16_t* ecov, uint16_t* ecov_cnt, SizeT* seq_begin, int max_seqs)
{
    g = as_global(g);
    if (lane == 0)
    {
        g.base[0]    = seq[0];
        g.sorted[0]  = 0;
        g.in_cnt[0]  = 0;
        g.aln_cnt[0] = 0;
        g.pos[0]     = 0;
        g.in_w[0]    = uint16_t(int(w[0]));
        g.cov[0]     = 1;
        if (MSA)
            seq_begin[0] = 0;
    }
    for (int n = 1 + lane; n < len; n += kWave)
    {
        g.base[n]                    = seq[n];
        g.sorted[n]                  = SizeT(n);
        g.out_e[(n - 1) * kMaxEdges] = SizeT(n);
        g.out_cnt[n - 1]             = 1;
        g.in_e[n * kMaxEdges]        = SizeT(n - 1);
        g.in_w[n * kMaxEdges]        = uint16_t(int(w[n - 1]) + int(w[n]));
        g.in_cnt[n]                  = 1;
        g.aln_cnt[n]                 = 0;
        g.pos[n]                     = SizeT(n);
        g.cov[n]                     = 1;
        if (MSA)
        {
            ecov[size_t(n - 1) * kMaxEdges * max_seqs] = 0;
            ecov_cnt[(n - 1) * kMaxEdges]              = 1;
        }
    }
    wave_sync();
    if (lane == 0 && len >= 1)
        g.out_cnt[len - 1] = 0; // written last, as in the reference (:179 then loop)
    wave_sync();
}

// ---------------------------------------------------------------------------
// Full-matrix NW forward pass (cudapoa_nw.cuh:165-327).  Rows are stored with
// column j at index j + kColShift; lanes whose 8 columns all lie beyond the
// read are masked (those cells never feed a valid cell).
template <typename ScoreT>
struct Pack8;
template <>
struct Pack8<int16_t>
{
    __device__ static void load(const int16_t* p, int (&v)[8])
    {
        uint4 q = *reinterpret_cast<const uint4*>(p);
        v[0]    = int(int16_t(q.x & 0xffff));
        v[1]    = int(int16_t(q.x >> 16));
        v[2]    = int(int16_t(q.y & 0xffff));
        v[3]    = int(int16_t(q.y >> 16));
        v[4]    = int(int16_t(q.z & 0xffff));
        v[5]    = int(int16_t(q.z >> 16));
        v[6]    = int(int16_t(q.w & 0xffff));
        v[7]    = int(int16_t(q.w >> 16));
    }
    __device__ static void store(int16_t* p, const int (&v)[8])
    {
        uint4 q;
        q.x = (uint32_t(uint16_t(v[0]))) | (uint32_t(uint16_t(v[1])) << 16);
        q.y = (uint32_t(uint16_t(v[2]))) | (uint32_t(uint16_t(v[3])) << 16);
        q.z = (uint32_t(uint16_t(v[4]))) | (uint32_t(uint16_t(v[5])) << 16);
        q.w = (uint32_t(uint16_t(v[6]))) | (uint32_t(uint16_t(v[7])) << 16);
        *reinterpret_cast<uint4*>(p) = q;
    }
};
template <>
struct Pack8<int32_t>
{
    __device__ static void load(const int32_t* p, int (&v)[8])
    {
        int4 a = *reinterpret_cast<const int4*>(p);
        int4 b = *reinterpret_cast<const int4*>(p + 4);
        v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w;
        v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
    }
    __device__ static void store(int32_t* p, const int (&v)[8])
    {
        *reinterpret_cast<int4*>(p)     = make_int4(v[0], v[1], v[2], v[3]);
        *reinterpret_cast<int4*>(p + 4) = make_int4(v[4], v[5], v[6], v[7]);
    }
};

template <typename ScoreT, typename SizeT>
__device__ void nw_forward_full(WinGraph<SizeT> g, int V, const uint8_t* read, int L, ScoreT* S, int stride,
                                const Scores sc, int lane)
{
    g = as_global(g);
    const int gap = sc.gap;
    // row 0: H[0][j] = j * gap (cudapoa_nw.cuh:176-179)
    for (int j = lane; j <= L; j += kWave)
        S[j + kColShift] = ScoreT(j * gap);

    for (int r = 1; r <= V; r++)
    {
        const int node = uniform(int(g.sorted[r - 1]));
        const int np   = uniform(int(g.in_cnt[node]));
        const int gb   = uniform(int(g.base[node]));
        ScoreT* row    = S + size_t(r) * stride + kColShift;
        // column 0 (:187-210)
        int c0;
        if (np == 0)
            c0 = gap;
        else
        {
            c0 = kNeg;
            for (int p = 0; p < np; p++)
            {
                int pr = uniform(pred_row(g, node, p));
                c0     = max(c0, int(S[size_t(pr) * stride + kColShift]));
            }
            c0 += gap;
        }
        if (lane == 0)
            row[0] = ScoreT(c0);

        int carry = c0; // E-domain carry: E[j] = H[j] - j*gap; E[0] = H[0]
        for (int cb = 0; cb < L; cb += kChunk)
        {
            const int jb     = cb + lane * kCellsPerLane; // lane cells: columns jb+1 .. jb+8
            const bool active = jb < L;
            int D[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                D[k] = kNeg;
            if (active)
            {
                const uint2 rc = *reinterpret_cast<const uint2*>(read + jb);
                int sig[8];
#pragma unroll
                for (int k = 0; k < 8; k++)
                {
                    uint32_t ch = ((k < 4 ? rc.x : rc.y) >> (8 * (k & 3))) & 0xff;
                    sig[k]      = (int(ch) == gb) ? sc.match : sc.mismatch;
                }
                const int npp = np == 0 ? 1 : np;
                for (int p = 0; p < npp; p++)
                {
                    const int pr    = np == 0 ? 0 : uniform(pred_row(g, node, p));
                    const ScoreT* P = S + size_t(pr) * stride + kColShift;
                    int cur[8];
                    Pack8<ScoreT>::load(P + jb + 1, cur); // columns jb+1..jb+8 (16-B aligned)
                    int prev = int(P[jb]);                // column jb
#pragma unroll
                    for (int k = 0; k < 8; k++)
                    {
                        D[k] = max(D[k], max(prev + sig[k], cur[k] + gap));
                        prev = cur[k];
                    }
                }
            }
            // horizontal closure as a running maximum in the E domain
            int E[8];
            int m = kNeg;
#pragma unroll
            for (int k = 0; k < 8; k++)
            {
                int e = D[k] - (jb + k + 1) * gap;
                m     = max(m, e);
                E[k]  = m;
            }
            const int below = max(wave_excl_max(m, lane), carry);
            if (active)
            {
                int H[8];
#pragma unroll
                for (int k = 0; k < 8; k++)
                    H[k] = max(E[k], below) + (jb + k + 1) * gap;
                Pack8<ScoreT>::store(row + jb + 1, H);
            }
            carry = max(carry, wave_max(m));
        }
    }
}

// Traceback (cudapoa_nw.cuh:329-462), lane 0 only.  Writes the reversed
// alignment and returns its length, or -1 at the loop bound.
template <typename ScoreT, typename SizeT>
__device__ int traceback_full(WinGraph<SizeT> g, int V, const uint8_t* read, int L, const ScoreT* S,
                              int stride, const Scores sc, SizeT* ag, SizeT* ar, int aln_cap)
{
    g = as_global(g);
    auto H = [&](int i, int j) { return int(S[size_t(i) * stride + kColShift + j]); };
    int i = 0, j = L;
    int best = INT_MIN;
    for (int idx = 1; idx <= V; idx++)
    {
        if (g.out_cnt[int(g.sorted[idx - 1])] == 0)
        {
            int s = H(idx, j);
            if (best < s)
            {
                best = s;
                i    = idx;
            }
        }
    }
    int prev_i = 0, prev_j = 0, n = 0, loops = 0;
    const int bound = L + V + 2;
    while (!(i == 0 && j == 0) && loops < bound)
    {
        loops++;
        const int sij = H(i, j);
        bool found    = false;
        int node      = 0, np = 0;
        if (i != 0)
        {
            node = int(g.sorted[i - 1]);
            np   = int(g.in_cnt[node]);
        }
        if (i != 0 && j != 0)
        {
            const int cost = (g.base[node] == read[j - 1]) ? sc.match : sc.mismatch;
            int pi         = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H(pi, j - 1) + cost)
            {
                prev_i = pi, prev_j = j - 1, found = true;
            }
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H(pi, j - 1) + cost)
                    prev_i = pi, prev_j = j - 1, found = true;
            }
        }
        if (!found && i != 0)
        {
            int pi = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H(pi, j) + sc.gap)
                prev_i = pi, prev_j = j, found = true;
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H(pi, j) + sc.gap)
                    prev_i = pi, prev_j = j, found = true;
            }
        }
        if (!found && j != 0 && sij == H(i, j - 1) + sc.gap)
            prev_i = i, prev_j = j - 1, found = true;
        if (n < aln_cap)
        {
            ag[n] = SizeT(i == prev_i ? -1 : int(g.sorted[i - 1]));
            ar[n] = SizeT(j == prev_j ? -1 : j - 1);
        }
        n++;
        i = prev_i;
        j = prev_j;
    }
    if (loops >= bound || n > aln_cap)
        return -1;
    return n;
}

// ---------------------------------------------------------------------------
// Banded NW (cudapoa_nw_banded.cuh:28-487).  The flat row layout (stride
// bw + 8, column c at index c - band_start, column 0 written at band_start but
// read from index 0) is reproduced exactly; see DESIGN.md.
struct Band
{
    int bw, stride, max_column;
    float gradient;
    __device__ int start(int row) const
    {
        int s = int(float(row) * gradient) - bw / 2;
        s     = max(s, 0);
        if (s + bw > max_column)
            s = max_column - bw + 4;
        s = max(s, 0);
        return s - (s % 4);
    }
};

template <typename ScoreT>
__device__ __forceinline__ ScoreT band_get(const ScoreT* S, const Band& B, int row, int col, ScoreT minv)
{
    int bs = B.start(row);
    if ((col > bs + B.bw || col < bs) && col != 0)
        return minv;
    int idx = (col == 0) ? 0 : col - bs;
    return S[int64_t(row) * B.stride + idx];
}

template <typename ScoreT>
__device__ __forceinline__ void band_set(ScoreT* S, const Band& B, int row, int col, ScoreT v)
{
    int bs  = B.start(row);
    int idx = (col == 0) ? bs : col - bs;
    S[int64_t(row) * B.stride + idx] = v;
}

template <typename ScoreT>
__device__ __forceinline__ ScoreT score_min()
{
    return sizeof(ScoreT) == 2 ? ScoreT(INT16_MIN) : ScoreT(INT32_MIN);
}

template <typename ScoreT>
__device__ __forceinline__ ScoreT band_min_value(const Scores sc)
{
    // cudapoa_nw_banded.cuh:197
    int a = min(min(sc.gap, sc.mismatch), -sc.match) - 1;
    return ScoreT(2 * (a < 0 ? -a : a) + int(score_min<ScoreT>()));
}

template <typename ScoreT, typename SizeT>
__device__ void nw_forward_banded(WinGraph<SizeT> g, int V, const uint8_t* read, int L, ScoreT* S,
                                  const Band& B, const Scores sc, int lane)
{
    g = as_global(g);
    const ScoreT minv = band_min_value<ScoreT>(sc);
    const int gap     = sc.gap;
    // horizontal boundary (:212-216)
    for (int j = lane; j < B.stride; j += kWave)
        band_set(S, B, 0, j, ScoreT(j * gap));
    __syncthreads();
    // vertical boundary (:219-245): serial over rows (reads earlier rows' col 0)
    if (lane == 0)
    {
        for (int r = 0; r < V; r++)
        {
            band_set(S, B, 0, 0, ScoreT(0));
            int node = int(g.sorted[r]);
            int np   = int(g.in_cnt[node]);
            if (np == 0)
                band_set(S, B, r + 1, 0, ScoreT(gap));
            else
            {
                int pen = int(score_min<ScoreT>());
                for (int p = 0; p < np; p++)
                    pen = max(pen, int(band_get(S, B, pred_row(g, node, p), 0, minv)));
                band_set(S, B, r + 1, 0, ScoreT(pen + gap));
            }
        }
    }
    __syncthreads();
    for (int r = 1; r <= V; r++)
    {
        const int node = uniform(int(g.sorted[r - 1]));
        const int np   = uniform(int(g.in_cnt[node]));
        const int gb   = uniform(int(g.base[node]));
        const int bs   = B.start(r);
        ScoreT* row    = S + int64_t(r) * B.stride;
        // initialize_band (:90-105)
        if (lane == 0)
            row[(bs == 0) ? 1 : 0] = minv;
        if (lane < kBandPad)
            row[B.bw + lane] = minv;
        __syncthreads();
        int carry = int(band_get(S, B, r, 0, minv));
        // 64 lanes x 4 cells = 256 columns per pass (reference: 32 x 4 per pass;
        // the closure is exact so the pass width does not change any cell)
        for (int base_pos = bs; base_pos < bs + B.bw; base_pos += kWave * 4)
        {
            const int rp      = base_pos + lane * 4;
            const bool active = rp < bs + B.bw;
            int v[4];
            if (active)
            {
                int prof[4];
#pragma unroll
                for (int c = 0; c < 4; c++)
                    prof[c] = (int(read[rp + c]) == gb) ? sc.match : sc.mismatch;
                const int npp = np == 0 ? 1 : np;
                for (int p = 0; p < npp; p++)
                {
                    const int pr  = np == 0 ? 0 : uniform(pred_row(g, node, p));
                    const int pbs = B.start(pr);
                    const int pbe = pbs + B.bw + 4;
                    int t[4];
                    if ((rp + 1 > pbe || rp + 1 < pbs) && rp + 1 != 0)
                    {
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            t[c] = int(minv);
                    }
                    else
                    {
                        const int idx   = (rp == 0) ? 0 : rp - pbs;
                        const ScoreT* q = S + int64_t(pr) * B.stride + idx;
                        t[0]            = int(ScoreT(max(int(q[0]) + prof[0], int(q[1]) + gap)));
                        t[1]            = int(ScoreT(max(int(q[1]) + prof[1], int(q[2]) + gap)));
                        t[2]            = int(ScoreT(max(int(q[2]) + prof[2], int(q[3]) + gap)));
                        t[3]            = int(ScoreT(max(int(q[3]) + prof[3], int(q[4]) + gap)));
                    }
                    if (p == 0)
                    {
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            v[c] = t[c];
                    }
                    else
                    {
#pragma unroll
                        for (int c = 0; c < 4; c++)
                            v[c] = max(v[c], t[c]);
                    }
                }
            }
            else
            {
#pragma unroll
                for (int c = 0; c < 4; c++)
                    v[c] = kNeg;
            }
            int E[4];
            int m = kNeg;
#pragma unroll
            for (int c = 0; c < 4; c++)
            {
                int e = v[c] - (rp + c + 1) * gap;
                m     = max(m, e);
                E[c]  = m;
            }
            const int below = max(wave_excl_max(m, lane), carry - (base_pos)*gap);
            int H[4];
#pragma unroll
            for (int c = 0; c < 4; c++)
                H[c] = max(E[c], below) + (rp + c + 1) * gap;
            if (active)
            {
                ScoreT* dst = row + (rp + 1 - bs);
#pragma unroll
                for (int c = 0; c < 4; c++)
                    dst[c] = ScoreT(H[c]);
            }
            // carry = H at the pass's last column (lane 63's 4th cell)
            carry = __shfl(H[3], kWave - 1, kWave);
            carry = int(ScoreT(carry));
        }
        __syncthreads();
    }
}

template <typename ScoreT, typename SizeT>
__device__ int traceback_banded(WinGraph<SizeT> g, int V, const uint8_t* read, int L, const ScoreT* S,
                                const Band& B, const Scores sc, SizeT* ag, SizeT* ar, int aln_cap)
{
    g = as_global(g);
    const ScoreT minv = band_min_value<ScoreT>(sc);
    auto H            = [&](int i, int j) { return int(band_get(S, B, i, j, minv)); };
    int i = 0, j = L;
    int best = int(score_min<ScoreT>());
    for (int idx = 1; idx <= V; idx++)
    {
        if (g.out_cnt[int(g.sorted[idx - 1])] == 0)
        {
            int s = H(idx, j);
            if (best < s)
                best = s, i = idx;
        }
    }
    int prev_i = 0, prev_j = 0, n = 0, loops = 0;
    const int bound = L + V + 2;
    while (!(i == 0 && j == 0) && loops < bound)
    {
        loops++;
        const int sij = H(i, j);
        bool found    = false;
        int node = 0, np = 0;
        if (i != 0)
        {
            node = int(g.sorted[i - 1]);
            np   = int(g.in_cnt[node]);
        }
        if (i != 0 && j != 0)
        {
            const int cost = (g.base[node] == read[j - 1]) ? sc.match : sc.mismatch;
            int pi         = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H(pi, j - 1) + cost)
                prev_i = pi, prev_j = j - 1, found = true;
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H(pi, j - 1) + cost)
                    prev_i = pi, prev_j = j - 1, found = true;
            }
        }
        if (!found && i != 0)
        {
            int pi = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H(pi, j) + sc.gap)
                prev_i = pi, prev_j = j, found = true;
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H(pi, j) + sc.gap)
                    prev_i = pi, prev_j = j, found = true;
            }
        }
        if (!found && sij == H(i, j - 1) + sc.gap)
            prev_i = i, prev_j = j - 1, found = true;
        if (n < aln_cap)
        {
            ag[n] = SizeT(i == prev_i ? -1 : int(g.sorted[i - 1]));
            ar[n] = SizeT(j == prev_j ? -1 : j - 1);
        }
        n++;
        i = prev_i;
        j = prev_j;
    }
    if (loops >= bound || n > aln_cap)
        return -1;
    return n;
}

// ---------------------------------------------------------------------------
// addAlignmentToGraph (cudapoa_add_alignment.cuh:59-279), lane 0.
template <typename SizeT, bool MSA>
__device__ uint8_t add_alignment(WinGraph<SizeT> g, int& node_count, const SizeT* ag, const SizeT* ar, int alen,
                                 const uint8_t* read, const int8_t* w, int s, uint16_t* ecov, uint16_t* ecov_cnt,
                                 SizeT* seq_begin, int max_seqs)
{
    g = as_global(g);
    int head = -1, curr = -1;
    uint16_t prev_w = 0;
    int nc          = node_count;
    for (int k = alen - 1; k >= 0; k--)
    {
        const int rp = int(ar[k]);
        if (rp == -1)
            continue;
        const int8_t nw  = w[rp];
        const uint8_t rb = read[rp];
        const int gid    = int(ag[k]);
        bool fresh       = false;
        if (gid == -1)
        {
            curr = nc++;
            if (nc >= g.max_nodes)
            {
                node_count = nc;
                return kNodeCountExceeded;
            }
            fresh = true;
        }
        else if (g.base[gid] == rb)
        {
            curr = gid;
        }
        else
        {
            const int na = int(g.aln_cnt[gid]);
            int hit      = -1;
            for (int n = 0; n < na; n++)
            {
                int aid = int(g.aln[gid * kMaxAlignments + n]);
                if (g.base[aid] == rb)
                {
                    hit = aid;
                    break;
                }
            }
            if (hit != -1)
                curr = hit;
            else
            {
                curr = nc++;
                if (nc >= g.max_nodes)
                {
                    node_count = nc;
                    return kNodeCountExceeded;
                }
                g.base[curr]    = rb;
                g.out_cnt[curr] = 0;
                g.in_cnt[curr]  = 0;
                g.aln_cnt[curr] = 0;
                g.cov[curr]     = 0;
                int cnt         = 0;
                for (int n = 0; n < na; n++)
                {
                    int aid                                  = int(g.aln[gid * kMaxAlignments + n]);
                    int ac                                   = int(g.aln_cnt[aid]);
                    g.aln[aid * kMaxAlignments + ac]         = SizeT(curr);
                    g.aln_cnt[aid]                           = uint16_t(ac + 1);
                    g.aln[curr * kMaxAlignments + cnt]       = SizeT(aid);
                    cnt++;
                }
                g.aln[gid * kMaxAlignments + na]   = SizeT(curr);
                g.aln_cnt[gid]                     = uint16_t(na + 1);
                g.aln[curr * kMaxAlignments + cnt] = SizeT(gid);
                cnt++;
                g.aln_cnt[curr] = uint16_t(cnt);
            }
        }
        if (fresh)
        {
            g.base[curr]    = rb;
            g.out_cnt[curr] = 0;
            g.in_cnt[curr]  = 0;
            g.aln_cnt[curr] = 0;
            g.cov[curr]     = 0;
        }
        if (MSA && rp == 0)
            seq_begin[s] = SizeT(curr);
        if (head != -1)
        {
            bool exists  = false;
            const int ic = int(g.in_cnt[curr]);
            for (int e = 0; e < ic; e++)
            {
                if (int(g.in_e[curr * kMaxEdges + e]) == head)
                {
                    exists = true;
                    g.in_w[curr * kMaxEdges + e] =
                        uint16_t(int(g.in_w[curr * kMaxEdges + e]) + (int(prev_w) + int(nw)));
                }
            }
            if (!exists)
            {
                g.in_e[curr * kMaxEdges + ic] = SizeT(head);
                g.in_w[curr * kMaxEdges + ic] = uint16_t(int(prev_w) + int(nw));
                g.in_cnt[curr]                = uint16_t(ic + 1);
                const int oc                  = int(g.out_cnt[head]);
                g.out_e[head * kMaxEdges + oc] = SizeT(curr);
                if (MSA)
                {
                    ecov_cnt[head * kMaxEdges + oc]                       = 1;
                    ecov[size_t(head * kMaxEdges + oc) * max_seqs]        = uint16_t(s);
                }
                g.out_cnt[head] = uint16_t(oc + 1);
                if (oc + 1 >= kMaxEdges || ic + 1 >= kMaxEdges)
                {
                    node_count = nc;
                    return kEdgeCountExceeded;
                }
            }
            else if (MSA)
            {
                const int oc = int(g.out_cnt[head]);
                for (int e = 0; e < oc; e++)
                {
                    if (int(g.out_e[head * kMaxEdges + e]) == curr)
                    {
                        int c                                                  = int(ecov_cnt[head * kMaxEdges + e]);
                        ecov[size_t(head * kMaxEdges + e) * max_seqs + c]      = uint16_t(s);
                        ecov_cnt[head * kMaxEdges + e]                         = uint16_t(c + 1);
                        break;
                    }
                }
            }
        }
        head = curr;
        g.cov[head]++;
        prev_w = uint16_t(int(nw));
    }
    node_count = nc;
    return kSuccess;
}

// Kahn topological sort (cudapoa_topsort.cuh:38-88), lane 0.
template <typename SizeT>
__device__ void topsort_kahn(WinGraph<SizeT> g, int n, int32_t* local)
{
    g = as_global(g);
    int k = 0;
    for (int v = 0; v < n; v++)
    {
        local[v] = g.in_cnt[v];
        if (local[v] == 0)
        {
            g.pos[v]      = SizeT(k);
            g.sorted[k++] = SizeT(v);
        }
    }
    for (int q = 0; q < k; q++)
    {
        const int v  = int(g.sorted[q]);
        const int oc = int(g.out_cnt[v]);
        for (int e = 0; e < oc; e++)
        {
            const int o = int(g.out_e[v * kMaxEdges + e]);
            if (--local[o] == 0)
            {
                g.pos[o]      = SizeT(k);
                g.sorted[k++] = SizeT(o);
            }
        }
    }
}

// racon/SPOA DFS sort (cudapoa_topsort.cuh:94-189), lane 0.  marks packs
// node_marks (bits 0-1) and check_aligned_nodes (bit 2).
template <typename SizeT>
__device__ bool topsort_racon(WinGraph<SizeT> g, int n, int32_t* marks, SizeT* stack, int stack_cap)
{
    g = as_global(g);
    for (int i = 0; i < g.max_nodes; i++)
        marks[i] = 4; // mark 0, check = true
    int top = -1, k = 0;
    for (int v = 0; v < n; v++)
    {
        if ((marks[v] & 3) != 0)
            continue;
        stack[++top] = SizeT(v);
        while (top != -1)
        {
            const int id = int(stack[top]);
            bool valid   = true;
            if ((marks[id] & 3) != 2)
            {
                for (int e = 0; e < int(g.in_cnt[id]); e++)
                {
                    int b = int(g.in_e[id * kMaxEdges + e]);
                    if ((marks[b] & 3) != 2)
                    {
                        if (top + 1 >= stack_cap)
                            return false;
                        stack[++top] = SizeT(b);
                        valid        = false;
                    }
                }
                if (marks[id] & 4)
                {
                    for (int a = 0; a < int(g.aln_cnt[id]); a++)
                    {
                        int aid = int(g.aln[id * kMaxAlignments + a]);
                        if ((marks[aid] & 3) != 2)
                        {
                            if (top + 1 >= stack_cap)
                                return false;
                            stack[++top] = SizeT(aid);
                            marks[aid] &= 3; // check = false
                            valid = false;
                        }
                    }
                }
                if (valid)
                {
                    marks[id] = (marks[id] & 4) | 2;
                    if (marks[id] & 4)
                    {
                        g.sorted[k] = SizeT(id);
                        g.pos[id]   = SizeT(k);
                        k++;
                        for (int a = 0; a < int(g.aln_cnt[id]); a++)
                        {
                            int aid     = int(g.aln[id * kMaxAlignments + a]);
                            g.sorted[k] = SizeT(aid);
                            g.pos[aid]  = SizeT(k);
                            k++;
                        }
                    }
                }
                else
                    marks[id] = (marks[id] & 4) | 1;
            }
            if (valid)
                top--;
        }
    }
    return true;
}

// Heaviest bundle (cudapoa_generate_consensus.cuh:28-276), lane 0.  Writes the
// consensus backwards (as the reference kernel) and returns its length or -status.
template <typename SizeT>
__device__ int branch_completion(WinGraph<SizeT> g, int n, int max_pos, int32_t* score, SizeT* pred)
{
    g = as_global(g);
    int node = int(g.sorted[max_pos]);
    for (int oe = 0; oe < int(g.out_cnt[node]); oe++)
    {
        const int o = int(g.out_e[node * kMaxEdges + oe]);
        for (int ie = 0; ie < int(g.in_cnt[o]); ie++)
        {
            int id = int(g.in_e[o * kMaxEdges + ie]);
            if (id != node)
                score[id] = -1;
        }
    }
    int max_score = 0, max_id = 0;
    for (int r = max_pos + 1; r < n; r++)
    {
        node       = int(g.sorted[r]);
        pred[node] = SizeT(-1);
        int s      = -1;
        for (int e = 0; e < int(g.in_cnt[node]); e++)
        {
            const int b = int(g.in_e[node * kMaxEdges + e]);
            if (score[b] == -1)
                continue;
            const int w = int(g.in_w[node * kMaxEdges + e]);
            if (s < w || (s == w && score[int(pred[node])] <= score[b]))
            {
                s          = w;
                pred[node] = SizeT(b);
            }
        }
        if (int(pred[node]) != -1)
            s += score[int(pred[node])];
        if (max_score <= s)
            max_score = s, max_id = node;
        score[node] = s;
    }
    return max_id;
}

template <typename SizeT>
__device__ int consensus_raw(WinGraph<SizeT> g, int n, int32_t* score, SizeT* pred, uint8_t* cons,
                             uint16_t* cov, int max_cons)
{
    g = as_global(g);
    for (int i = 0; i < n; i++)
    {
        pred[i]  = SizeT(-1);
        score[i] = -1;
    }
    int max_id = 0, max_score = -1;
    for (int r = 0; r < n; r++)
    {
        const int node = int(g.sorted[r]);
        int s          = score[node];
        for (int e = 0; e < int(g.in_cnt[node]); e++)
        {
            const int w = int(g.in_w[node * kMaxEdges + e]);
            const int b = int(g.in_e[node * kMaxEdges + e]);
            if (s < w || (s == w && score[int(pred[node])] <= score[b]))
            {
                s          = w;
                pred[node] = SizeT(b);
            }
        }
        if (int(pred[node]) != -1)
            s += score[int(pred[node])];
        if (max_score <= s)
            max_id = node, max_score = s;
        score[node] = s;
    }
    int loops = 0;
    if (g.out_cnt[max_id] != 0)
    {
        while (g.out_cnt[max_id] != 0 && loops < n)
        {
            max_id = branch_completion(g, n, int(g.pos[max_id]), score, pred);
            loops++;
        }
    }
    if (loops >= n)
        return -int(kLoopCountExceeded);
    auto node_cov = [&](int id) {
        uint16_t c = g.cov[id];
        for (int a = 0; a < int(g.aln_cnt[id]); a++)
            c = uint16_t(c + g.cov[int(g.aln[id * kMaxAlignments + a])]);
        return c;
    };
    int cpos = 0, count = 0;
    while (int(pred[max_id]) != -1)
    {
        cons[cpos] = g.base[max_id];
        cov[cpos]  = node_cov(max_id);
        max_id     = int(pred[max_id]);
        cpos       = min(cpos + 1, max_cons - 1);
        count++;
    }
    cons[cpos] = g.base[max_id];
    cov[cpos]  = node_cov(max_id);
    if (count >= max_cons - 1)
        return -int(kExceededMaxSeqSize);
    return cpos + 1;
}

} // namespace poa
} // namespace gwamd

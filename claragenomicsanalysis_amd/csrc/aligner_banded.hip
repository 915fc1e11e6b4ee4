// MI355X banded global aligners:
//   * banded Myers (AlignerGlobalMyersBanded, cudaaligner/src/myers_gpu.cu:377-780)
//   * Ukkonen banded NW (AlignerGlobalUkkonen, cudaaligner/src/ukkonen_gpu.cu:59-329)
//
// One wave per pair; a persistent grid walks the pairs with a static stride
// and each workgroup owns one HBM workspace slot.  Both aligners keep the
// reference's band matrices in HBM exactly (column-major, same index maps),
// because their backtraces read the band through the reference's own index
// arithmetic, including its behaviour at the band edges; what is MI355X-
// specific is how the band is filled and walked:
//
// banded Myers: the 32 words of a band chunk (the reference's warp) sit in
//   lanes 0..31; the 1024-bit addition of a Myers step is a carry-lookahead
//   on ballot masks, the one-bit shifts across words are ballots as well, and
//   the chunk state stays in registers from column to column (the reference
//   reloads it from HBM).  Only the column stores go to HBM.
// Ukkonen: band row k of the (k, l) matrix is lane k % 64 of chunk k / 64;
//   the anti-diagonal sweep keeps the last two l columns in registers and
//   takes the k +- 1 neighbours with DPP wave shifts, so a column costs one
//   coalesced 2-byte store per cell and no LDS round trip.
//
// Both backtraces stage the part of the band they are about to read in an
// LDS tile (refilled with coalesced dword loads when the walk leaves it) and
// emit the path 64 steps at a time.
#include <hip/hip_runtime.h>

#include "aligner_common.hpp"
#include "aligner_device.hpp"

namespace gwamd
{
namespace aln
{

namespace
{

__device__ __forceinline__ uint64_t ballot(bool b) { return __builtin_amdgcn_ballot_w64(b); }
__device__ __forceinline__ uint32_t bit_of(uint32_t m, int lane) { return __builtin_amdgcn_ubfe(m, uint32_t(lane & 31), 1u); }

// (~1u) << b as the reference's GPU evaluates it (PTX shl: counts >= 32 give 0)
__device__ __forceinline__ uint32_t shl_ptx(uint32_t x, int b) { return (b < 0 || b >= 32) ? 0u : (x << b); }

// Path emission: 64 states buffered one per lane, stored 64 at a time.
struct PathWriter
{
    int8_t* path;
    int cap;
    int pos = 0;
    int buf = 0;
    bool overflow = false;
    __device__ void put(int8_t r, int lane)
    {
        if (lane == (pos & 63))
            buf = r;
        if ((pos & 63) == 63)
            flush_full(lane);
        ++pos;
    }
    __device__ void flush_full(int lane)
    {
        const int at = (pos & ~63) + lane;
        if (at < cap)
            path[at] = int8_t(buf);
        else
            overflow = true;
    }
    __device__ void finish(int lane)
    {
        const int at = (pos & ~63) + lane;
        if (lane < (pos & 63))
        {
            if (at < cap)
                path[at] = int8_t(buf);
        }
        overflow = overflow || pos > cap;
    }
    // n copies of r (lane-parallel), after finish()
    __device__ void fill(int8_t r, int n, int lane)
    {
        for (int k = lane; k < n; k += kWave)
            if (pos + k < cap)
                path[pos + k] = r;
        pos += n;
        overflow = overflow || pos > cap;
    }
};

// One Myers step over a chunk of up to 32 words in lanes 0..31
// (myers_advance_block, myers_gpu.cu:95-125).  act: the chunk's lanes; hin
// enters lane 0 only; returns each lane's delta at its bit `hbit`.
__device__ __forceinline__ int chunk_step(uint32_t& pv, uint32_t& mv, uint32_t eq, int hin, uint32_t hbit,
                                          uint64_t act, int lane)
{
    const uint32_t lane0 = lane == 0 ? 1u : 0u;
    const uint32_t xv    = eq | mv;
    if (hin < 0)
        eq |= lane0;
    uint32_t s;
    const bool ov     = __builtin_add_overflow(eq & pv, pv, &s);
    const uint64_t G  = ballot(ov) & act;
    const uint64_t P  = ballot(s == 0xffffffffu) & act;
    const uint64_t GP = G | P;
    s += bit_of(uint32_t((GP + G) ^ GP ^ G), lane); // carry into this word
    const uint32_t xh = (s ^ pv) | eq;
    uint32_t ph       = mv | ~(xh | pv);
    uint32_t mh       = pv & xh;
    const int out     = int((ph & hbit) != 0u) - int((mh & hbit) != 0u);
    const uint32_t PH = uint32_t(ballot((ph >> 31) != 0u));
    const uint32_t MH = uint32_t(ballot((mh >> 31) != 0u));
    ph                = (ph << 1) | bit_of(PH << 1, lane);
    mh                = (mh << 1) | bit_of(MH << 1, lane);
    if (hin < 0)
        mh |= lane0;
    if (hin > 0)
        ph |= lane0;
    pv = mh | ~(xv | ph);
    mv = ph & xv;
    return out;
}

} // namespace

// ---------------------------------------------------------------------------
// Banded Myers (myers_banded_kernel, myers_gpu.cu:706-780)
__global__ void __launch_bounds__(kWave) myers_banded_kernel(Args a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    const int lane          = threadIdx.x;
    GWAMD_LDS uint8_t* base = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint8_t* tgt  = base + a.lds_target_off;
    GWAMD_LDS uint32_t* pat = (GWAMD_LDS uint32_t*)(base + a.lds_pat_off);
    const int TL            = a.tile_bytes / 12; // tile elements per array
    GWAMD_LDS uint32_t* tpv = (GWAMD_LDS uint32_t*)(base + a.lds_tile_off);
    GWAMD_LDS uint32_t* tmv = tpv + TL;
    GWAMD_LDS int32_t* tsc  = (GWAMD_LDS int32_t*)(tmv + TL);
    uint8_t* ws             = a.ws + size_t(blockIdx.x) * size_t(a.ws_slot_bytes);
    const bool chunk_lane   = lane < kChunkWords;

    for (int idx = blockIdx.x; idx < a.n; idx += gridDim.x)
    {
        const char* q  = a.seqs + size_t(2 * idx) * a.stride;
        const char* tg = a.seqs + size_t(2 * idx + 1) * a.stride;
        const int Q    = uni(a.lens[2 * idx]);
        const int T    = uni(a.lens[2 * idx + 1]);
        PathWriter pw{a.paths + size_t(idx) * a.max_path_length, a.max_path_length};
        if (Q == 0 || T == 0)
        {
            // the reference asserts non-empty sequences; the only path
            pw.fill(kDeletion, Q, lane);
            pw.fill(kInsertion, T, lane);
            if (lane == 0)
                a.path_len[idx] = pw.overflow ? -1 : pw.pos;
            continue;
        }
        for (int k = lane; k < T; k += kWave)
            tgt[k] = uint8_t(tg[k]);
        build_patterns(pat, q, Q, lane);
        wave_sync();
        const int nwq  = (Q + kWordBits - 1) / kWordBits;
        const int dlen = Q > T ? Q - T : T - Q;
        int est        = max(1, dlen + min(T, Q) / 20); // initial_distance_guess_factor (:36, :749)
        int bw = 0, nwb = 0, db = 0, de = 0;
        uint32_t* wpv = nullptr;
        uint32_t* wmv = nullptr;
        int32_t* wsc  = nullptr;
        while (true)
        {
            int p = min(min(T, Q), (est - dlen) / 2);
            bw    = min(1 + 2 * p + dlen, Q);
            if (bw % kWordBits == 1 && bw != Q) // at least two bits in the last word
            {
                p += 1;
                bw = min(1 + 2 * p + dlen, Q);
            }
            nwb           = (bw + kWordBits - 1) / kWordBits;
            const int nch = uni((nwb + kChunkWords - 1) / kChunkWords);
            wpv           = reinterpret_cast<uint32_t*>(ws);
            wmv           = wpv + size_t(nwb) * (T + 1);
            wsc           = reinterpret_cast<int32_t*>(wmv + size_t(nwb) * (T + 1));
            if (bw >= Q)
                db = de = T + 1;
            else
            {
                db = Q < T ? T - Q + p + 2 : p + 2;
                de = Q < T ? Q - p + 1 : Q - (Q - T) - p + 1;
            }
            const int lastw      = nwb - 1;
            const int top_last   = bw - lastw * kWordBits; // rows of the last word
            uint32_t pv[kBandChunks], mv[kBandChunks];
            int sc[kBandChunks];
            uint64_t act[kBandChunks];
#pragma unroll
            for (int c = 0; c < kBandChunks; c++)
            {
                const int w  = c * kChunkWords + lane;
                const bool v = chunk_lane && c < nch && w < nwb;
                act[c]       = ballot(v);
                pv[c]        = ~0u;
                mv[c]        = 0u;
                sc[c]        = min((w + 1) * kWordBits, bw);
                if (v)
                {
                    wpv[w] = ~0u;
                    wmv[w] = 0u;
                    wsc[w] = sc[c];
                }
            }
            int tv = 0;
            for (int t = 1; t <= T; t++)
            {
                const int tl = (t - 1) & (kWave - 1);
                if (tl == 0)
                {
                    const int x = t - 1 + lane;
                    tv          = x < T ? int(tgt[x]) : 0;
                }
                const int code  = letter(uni(__builtin_amdgcn_readlane(tv, tl)));
                const bool diag = t >= db && t < de;
                if (!diag)
                {
                    // horizontal stripe (myers_compute_scores_horizontal_band_impl, :496-538)
                    const int po = t >= de ? Q - bw : 0;
                    int carry    = 1; // worst case for the band's top row
#pragma unroll
                    for (int c = 0; c < kBandChunks; c++)
                    {
                        if (c < nch)
                        {
                            const int w         = c * kChunkWords + lane;
                            const uint32_t eq   = seg_pattern(pat, nwq, po, w, code);
                            const uint32_t hbit = 1u << (w == lastw ? top_last - 1 : kWordBits - 1);
                            const int out       = chunk_step(pv[c], mv[c], eq, carry, hbit, act[c], lane);
                            sc[c] += out;
                            if ((act[c] >> lane) & 1u)
                            {
                                const size_t o = size_t(t) * nwb + w;
                                wpv[o]         = pv[c];
                                wmv[o]         = mv[c];
                                wsc[o]         = sc[c];
                            }
                            carry = uni(__builtin_amdgcn_readlane(out, kChunkWords - 1));
                        }
                    }
                }
                else
                {
                    // diagonal band (myers_compute_scores_diagonal_band_impl, :540-614)
                    const int po   = t - db + 1;
                    int carry_down = 1;
#pragma unroll
                    for (int c = 0; c < kBandChunks; c++)
                    {
                        if (c < nch)
                        {
                            const int w = c * kChunkWords + lane;
                            // shift the previous column down one row across the chunk
                            const uint32_t PB = uint32_t(ballot(pv[c] & 1u) & act[c]);
                            const uint32_t MB = uint32_t(ballot(mv[c] & 1u) & act[c]);
                            uint32_t p2       = (pv[c] >> 1) | (bit_of(PB >> 1, lane) << 31);
                            uint32_t m2       = (mv[c] >> 1) | (bit_of(MB >> 1, lane) << 31);
                            if (c + 1 < kBandChunks && c + 1 < nch)
                            {
                                // word 31 takes bit 0 of the next chunk's first word (:567-573)
                                const uint32_t np = uint32_t(ballot(pv[c + 1] & 1u)) & 1u;
                                const uint32_t nm = uint32_t(ballot(mv[c + 1] & 1u)) & 1u;
                                if (lane == kChunkWords - 1)
                                {
                                    p2 |= np << 31;
                                    m2 |= nm << 31;
                                }
                            }
                            const uint32_t crb = 1u << (w == lastw ? top_last - 2 : kWordBits - 2);
                            const uint32_t cdb = crb << 1;
                            const uint32_t eq  = seg_pattern(pat, nwq, po, w, code);
                            if (w == lastw)
                            {
                                // no left neighbour for the new bottom row: assume +1
                                p2 |= cdb;
                                m2 &= ~cdb;
                            }
                            const int right = chunk_step(p2, m2, eq, carry_down, crb, act[c], lane);
                            const int down  = int((p2 & cdb) != 0u) - int((m2 & cdb) != 0u);
                            pv[c]           = p2;
                            mv[c]           = m2;
                            sc[c] += right + down;
                            if ((act[c] >> lane) & 1u)
                            {
                                const size_t o = size_t(t) * nwb + w;
                                wpv[o]         = p2;
                                wmv[o]         = m2;
                                wsc[o]         = sc[c];
                            }
                            carry_down = uni(__builtin_amdgcn_readlane(down, kChunkWords - 1));
                        }
                    }
                }
            }
            // edit distance of the band: the last word's tracked row at column T
            int ed = 0;
#pragma unroll
            for (int c = 0; c < kBandChunks; c++)
                if (c == lastw / kChunkWords)
                    ed = uni(__builtin_amdgcn_readlane(sc[c], lastw % kChunkWords));
            if (ed <= est || bw == Q)
                break;
            est *= 2;
        }
        __threadfence_block();
        wave_sync();

        // backtrace (myers_backtrace_banded, :377-494) over an LDS tile of the
        // flat band arrays
        const int64_t total = int64_t(nwb) * (T + 1);
        int64_t tb          = -1; // flat index of tile element 0
        int64_t te          = -1;
        auto refill = [&](int jcol) {
            const int64_t hi = min<int64_t>(total, int64_t(nwb) * (jcol + 1));
            int64_t lo       = max<int64_t>(0, hi - TL);
            wave_sync();
            for (int64_t e = lane; e < hi - lo; e += kWave)
            {
                tpv[e] = wpv[lo + e];
                tmv[e] = wmv[lo + e];
                tsc[e] = wsc[lo + e];
            }
            wave_sync();
            tb = lo;
            te = hi;
        };
        const uint32_t lem = (bw % kWordBits) != 0 ? (1u << (bw % kWordBits)) - 1u : ~0u;
        auto gms           = [&](int i, int j) -> int {
            const int wi    = (i - 1) / kWordBits;
            const int bi    = (i - 1) % kWordBits;
            const int64_t o = int64_t(wi) + int64_t(nwb) * j;
            if (o < 0 || o >= total)
                return 0; // outside the band matrix (the oracle does the same)
            int s;
            uint32_t p, n;
            if (o >= tb && o < te)
            {
                s = tsc[o - tb];
                p = tpv[o - tb];
                n = tmv[o - tb];
            }
            else
            {
                s = wsc[o];
                p = wpv[o];
                n = wmv[o];
            }
            uint32_t mask = shl_ptx(~1u, bi);
            if (wi == nwb - 1)
                mask &= lem;
            return uni(s - __builtin_popcount(mask & uniu(p)) + __builtin_popcount(mask & uniu(n)));
        };
        int i = bw, j = T;
        refill(j);
        // start from the band's last word: the reference reads word
        // band_width / 32 (:393), one past the band when band_width % 32 == 0
        int s = uni(wsc[int64_t((bw - 1) / kWordBits) + int64_t(nwb) * j]);
        auto ensure = [&](int jj) {
            if (int64_t(nwb) * (jj - 1) < tb)
                refill(jj);
        };
        auto choose = [&](int left, int above, int diag, int di_left, int di_above, int di_diag, int dj_diag) {
            int8_t r;
            if (left + 1 == s)
            {
                r = kInsertion;
                s = left;
                i += di_left;
                --j;
            }
            else if (above + 1 == s)
            {
                r = kDeletion;
                s = above;
                i += di_above;
            }
            else
            {
                r = diag == s ? kMatch : kMismatch;
                s = diag;
                i += di_diag;
                j += dj_diag;
            }
            pw.put(r, lane);
        };
        while (j >= de)
        {
            ensure(j);
            const int above = i <= 1 ? j : gms(i - 1, j);
            const int dg    = i <= 1 ? j - 1 : gms(i - 1, j - 1);
            const int left  = gms(i, j - 1);
            choose(left, above, dg, 0, -1, -1, -1);
        }
        while (j >= db)
        {
            ensure(j);
            const int above = i <= 1 ? j : gms(i - 1, j);
            const int dg    = i <= 0 ? j - 1 : gms(i, j - 1);
            const int left  = gms(i + 1, j - 1);
            choose(left, above, dg, +1, -1, 0, -1);
        }
        while (i > 0 && j > 0)
        {
            ensure(j);
            const int above = i == 1 ? j : gms(i - 1, j);
            const int dg    = i == 1 ? j - 1 : gms(i - 1, j - 1);
            const int left  = gms(i, j - 1);
            choose(left, above, dg, 0, -1, -1, -1);
        }
        pw.finish(lane);
        pw.fill(kDeletion, max(i, 0), lane);
        pw.fill(kInsertion, max(j, 0), lane);
        if (lane == 0)
            a.path_len[idx] = pw.overflow ? -1 : pw.pos;
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// Ukkonen (ukkonen_compute_score_matrix + ukkonen_backtrace_kernel,
// ukkonen_gpu.cu:59-249)
namespace
{

__device__ __forceinline__ int dpp_from_lower(int v) // lane i <- lane i-1 (wave_shr:1)
{
    return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ int dpp_from_upper(int v) // lane i <- lane i+1 (wave_shl:1)
{
    return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false);
}

} // namespace

__global__ void __launch_bounds__(kWave) ukkonen_kernel(Args a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    const int lane          = threadIdx.x;
    GWAMD_LDS uint8_t* base = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint8_t* sA   = base + a.lds_target_off; // along i (the shorter sequence)
    GWAMD_LDS uint8_t* sB   = base + a.lds_seq2_off;   // along j
    const int TE            = (a.tile_bytes / 4) * 2;  // tile elements (int16), even
    GWAMD_LDS int16_t* tile = (GWAMD_LDS int16_t*)(base + a.lds_tile_off);
    int16_t* S              = reinterpret_cast<int16_t*>(a.ws + size_t(blockIdx.x) * size_t(a.ws_slot_bytes));
    const int p             = a.ukkonen_p;
    constexpr int M         = kUkMax;

    for (int idx = blockIdx.x; idx < a.n; idx += gridDim.x)
    {
        const int Q = uni(a.lens[2 * idx]);
        const int T = uni(a.lens[2 * idx + 1]);
        const char* qs = a.seqs + size_t(2 * idx) * a.stride;
        const char* ts = a.seqs + size_t(2 * idx + 1) * a.stride;
        int m = Q + 1, n = T + 1;
        int8_t ins = kInsertion, del = kDeletion;
        const bool swp = m > n;
        if (swp)
        {
            m   = T + 1;
            n   = Q + 1;
            ins = kDeletion;
            del = kInsertion;
        }
        const char* A = swp ? ts : qs;
        const char* B = swp ? qs : ts;
        for (int k = lane; k < m - 1; k += kWave)
            sA[k] = uint8_t(A[k]);
        for (int k = lane; k < n - 1; k += kWave)
            sB[k] = uint8_t(B[k]);
        wave_sync();
        const int bw        = (1 + n - m + 2 * p + 1) / 2;
        const int cols      = n + m;
        const int kmax_odd  = (n - m + 2 * p - 1) / 2 + 1;
        const int kmax_even = (n - m + 2 * p) / 2 + 1;
        const int nck       = uni((bw + kWave - 1) / kWave);

        // anti-diagonal sweep (ukkonen_init_score_matrix + compute_score_matrix_{even,odd})
        int V1[kUkChunks], V2[kUkChunks], V0[kUkChunks];
#pragma unroll
        for (int c = 0; c < kUkChunks; c++)
        {
            V1[c] = M;
            V2[c] = M;
        }
        for (int l = 0; l < cols; l++)
        {
            const bool even = ((l - p) & 1) == 0;
            const int kmax  = even ? kmax_even : kmax_odd;
#pragma unroll
            for (int c = 0; c < kUkChunks; c++)
            {
                if (c < nck)
                {
                    const int k    = c * kWave + lane;
                    const int j    = k - (p + l) / 2 + l;
                    const int i    = l - j;
                    const int d    = even ? 2 * k : 2 * k + 1; // diagonal + p
                    const int lmin = d >= p ? d - p : p - d;
                    const int lmax = d <= p ? 2 * (m - p + d) + lmin : 2 * min(m, n - d + p) + lmin;
                    const bool cmp = k < kmax && k < bw && l >= lmin + 1 && l < lmax;
                    // k - 1 and k + 1 of column l - 1
                    int lo = dpp_from_lower(V1[c]);
                    int hi = dpp_from_upper(V1[c]);
                    if (c > 0)
                    {
                        const int x = __builtin_amdgcn_readlane(V1[c > 0 ? c - 1 : 0], kWave - 1);
                        if (lane == 0)
                            lo = x;
                    }
                    if (c + 1 < kUkChunks && c + 1 < nck)
                    {
                        const int x = __builtin_amdgcn_readlane(V1[c + 1 < kUkChunks ? c + 1 : c], 0);
                        if (lane == kWave - 1)
                            hi = x;
                    }
                    const int ii  = cmp ? i - 1 : 0;
                    const int jj  = cmp ? j - 1 : 0;
                    const int ca  = sA[ii];
                    const int cb  = sB[jj];
                    const int dgv = l < 2 ? M : V2[c] + (ca == cb ? 0 : 1);
                    int left, above;
                    if (even)
                    {
                        left  = k - 1 < 0 ? M : lo + 1;
                        above = V1[c] + 1;
                    }
                    else
                    {
                        left  = V1[c] + 1;
                        above = k + 1 >= bw ? M : hi + 1;
                    }
                    const int init = i == 0 ? j : (j == 0 ? i : M);
                    const int v    = cmp ? min(dgv, min(left, above)) : init;
                    V0[c]          = int(int16_t(v));
                    if (k < bw)
                        S[size_t(k) + size_t(bw) * l] = int16_t(v);
                }
            }
#pragma unroll
            for (int c = 0; c < kUkChunks; c++)
            {
                V2[c] = V1[c];
                V1[c] = V0[c];
            }
        }
        __threadfence_block();
        wave_sync();

        // backtrace over an LDS tile of the flat matrix
        const int64_t total = int64_t(bw) * cols;
        int64_t tb = -1, te = -1;
        auto refill = [&](int lcol) {
            // flat range ending with column lcol, aligned to dwords
            const int64_t hi = min<int64_t>(total, int64_t(bw) * (lcol + 1));
            const int64_t lo = max<int64_t>(0, hi - TE) & ~int64_t(1);
            const int64_t nd = (hi - lo + 1) / 2;
            const uint32_t* src = reinterpret_cast<const uint32_t*>(S + lo);
            GWAMD_LDS uint32_t* dst = (GWAMD_LDS uint32_t*)tile;
            wave_sync();
            for (int64_t e = lane; e < nd; e += kWave)
                dst[e] = src[e];
            wave_sync();
            tb = lo;
            te = min<int64_t>(lo + 2 * nd, total);
        };
        auto val = [&](int i, int j) -> int {
            const int k = (j - i + p) / 2;
            const int l = j + i;
            if (k < 0 || k >= bw || l < 0 || l >= cols)
                return M;
            const int64_t o = int64_t(k) + int64_t(bw) * l;
            return uni(o >= tb && o < te ? int(tile[o - tb]) : int(S[o]));
        };
        PathWriter pw{a.paths + size_t(idx) * a.max_path_length, a.max_path_length};
        int i = m - 1, j = n - 1;
        refill(i + j);
        int s = val(i, j);
        while (i > 0 && j > 0)
        {
            if (int64_t(bw) * (i + j - 2) < tb)
                refill(i + j);
            const int above = val(i - 1, j);
            const int dg    = val(i - 1, j - 1);
            const int left  = val(i, j - 1);
            int8_t r;
            if (left + 1 == s)
            {
                r = ins;
                s = left;
                --j;
            }
            else if (above + 1 == s)
            {
                r = del;
                s = above;
                --i;
            }
            else
            {
                r = dg == s ? kMatch : kMismatch;
                s = dg;
                --i;
                --j;
            }
            pw.put(r, lane);
        }
        pw.finish(lane);
        pw.fill(del, i, lane);
        pw.fill(ins, j, lane);
        if (lane == 0)
            a.path_len[idx] = pw.overflow ? -1 : pw.pos;
        wave_sync();
    }
}

} // namespace aln
} // namespace gwamd

extern "C" hipError_t gwamd_internal_banded_launch(const gwamd::aln::Args* a, int algo, int grid, hipStream_t stream)
{
    using namespace gwamd::aln;
    if (a->n <= 0)
        return hipSuccess;
    if (algo == 2)
        hipLaunchKernelGGL(myers_banded_kernel, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    else
        hipLaunchKernelGGL(ukkonen_kernel, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    return hipGetLastError();
}

extern "C" hipError_t gwamd_internal_banded_occupancy(int algo, int lds_bytes, int* blocks_per_cu)
{
    using namespace gwamd::aln;
    if (algo == 2)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, myers_banded_kernel, kWave,
                                                            size_t(lds_bytes));
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, ukkonen_kernel, kWave, size_t(lds_bytes));
}

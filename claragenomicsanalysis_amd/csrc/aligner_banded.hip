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
#include <type_traits>
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

// chunk_step on two independent 32-word chunks at once, one in each half of
// the wave (lanes 0..31 and 32..63; act covers both).  hin is per lane (the
// carry into its half's lane 0); the carry-lookahead and the one-bit shifts
// stop at the half boundary, so each half computes exactly what chunk_step
// computes for it alone.
__device__ __forceinline__ int chunk_step2(uint32_t& pv, uint32_t& mv, uint32_t eq, int hin, uint32_t hbit,
                                           uint64_t act, int lane)
{
    constexpr uint64_t kLo = 0xffffffffull;
    const uint32_t first   = (lane & 31) == 0 ? 1u : 0u;
    const uint32_t xv      = eq | mv;
    if (hin < 0)
        eq |= first;
    uint32_t s;
    const bool ov     = __builtin_add_overflow(eq & pv, pv, &s);
    const uint64_t G  = ballot(ov) & act;
    const uint64_t P  = ballot(s == 0xffffffffu) & act;
    const uint64_t GP = G | P;
    const uint64_t cs = (((GP & kLo) + (G & kLo)) & kLo) | ((GP & ~kLo) + (G & ~kLo));
    s += uint32_t((cs ^ GP ^ G) >> lane) & 1u; // carry into this word
    const uint32_t xh = (s ^ pv) | eq;
    uint32_t ph       = mv | ~(xh | pv);
    uint32_t mh       = pv & xh;
    const int out     = int((ph & hbit) != 0u) - int((mh & hbit) != 0u);
    const uint64_t PH = (ballot((ph >> 31) != 0u) << 1) & ~(1ull << 32);
    const uint64_t MH = (ballot((mh >> 31) != 0u) << 1) & ~(1ull << 32);
    ph                = (ph << 1) | (uint32_t(PH >> lane) & 1u);
    mh                = (mh << 1) | (uint32_t(MH >> lane) & 1u);
    if (hin < 0)
        mh |= first;
    if (hin > 0)
        ph |= first;
    pv = mh | ~(xv | ph);
    mv = ph & xv;
    return out;
}

} // namespace

// ---------------------------------------------------------------------------
// Banded Myers (myers_banded_kernel, myers_gpu.cu:706-780)
//
// LDS: query patterns letter-major (patL[L * pat_words + k], conflict-free
// for lanes reading consecutive words), the target as 2-bit letter codes
// (16 per word), and one 4 KiB region that holds the per-chunk state of
// bands wider than one chunk during the sweep and the backtrace tile after it.

// Band entry of the flat column-major band matrix (entry = word + nwb *
// column, the reference's index map): pv, mv and the score of the word's
// tracked row, one 16-byte load or store.
struct BandEntry
{
    uint32_t pv, mv;
    int32_t sc, pad;
};

namespace
{

// LDS copies of a band entry (field-wise: address-space-qualified struct
// assignment does not compile)
__device__ __forceinline__ BandEntry lds_get(const GWAMD_LDS BandEntry* p)
{
    BandEntry e;
    e.pv  = p->pv;
    e.mv  = p->mv;
    e.sc  = p->sc;
    e.pad = 0;
    return e;
}
__device__ __forceinline__ void lds_put(GWAMD_LDS BandEntry* p, const BandEntry& e)
{
    p->pv  = e.pv;
    p->mv  = e.mv;
    p->sc  = e.sc;
    p->pad = 0;
}

// HBM copies of a band entry: one 16-byte global load / store
typedef uint32_t be_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ BandEntry glb_get(const GWAMD_GLB BandEntry* p)
{
    const be_u32x4 v = *(const GWAMD_GLB be_u32x4*)(p);
    return BandEntry{v.x, v.y, int32_t(v.z), 0};
}
__device__ __forceinline__ void glb_put(GWAMD_GLB BandEntry* p, const BandEntry& e)
{
    *(GWAMD_GLB be_u32x4*)(p) = be_u32x4{e.pv, e.mv, uint32_t(e.sc), 0u};
}

__device__ void build_patterns_lm(GWAMD_LDS uint32_t* patL, int pat_words, const char* q, int Q, int lane)
{
    const int nw          = (Q + kWordBits - 1) / kWordBits;
    const char letters[4] = {'A', 'C', 'T', 'G'};
    for (int k = lane; k < nw; k += kWave)
    {
        uint32_t f[4] = {0, 0, 0, 0};
        const int lim = min(Q - k * kWordBits, kWordBits);
        for (int i = 0; i < lim; i++)
        {
            const char c = q[k * kWordBits + i];
#pragma unroll
            for (int L = 0; L < 4; L++)
                f[L] |= (c == letters[L] ? 1u : 0u) << i;
        }
#pragma unroll
        for (int L = 0; L < 4; L++)
            patL[L * pat_words + k] = f[L];
    }
}

// get_query_pattern (myers_gpu.cu:140-171) on the letter-major patterns; both
// words are read unconditionally (clamped) so the two loads overlap
__device__ __forceinline__ uint32_t band_pattern(const GWAMD_LDS uint32_t* patL, int pat_words, int nwq, int off,
                                                 int w, int L)
{
    const int k  = (off >> 5) + w;
    const int sh = off & 31;
    const GWAMD_LDS uint32_t* row = patL + L * pat_words;
    uint32_t lo  = row[min(k, nwq - 1)];
    uint32_t hi  = row[min(k + 1, nwq - 1)];
    lo           = k < nwq ? lo : 0u;
    hi           = k + 1 < nwq ? hi : 0u;
    return sh != 0 ? (lo >> sh) | (hi << (32 - sh)) : lo;
}

} // namespace

// LDS-only workgroup barrier for the multi-wave sweep: the waves exchange
// band chunks through LDS only, so the step barrier waits for the LDS queue
// and not for the band matrix's HBM stores (a workgroup fence would)
__device__ __forceinline__ void lds_barrier()
{
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// NWV waves per pair: wave 0 does everything; waves 1..NWV-1 join the sweeps of
// bands of several chunks whose state fits LDS (2 * NWV target columns in
// flight, see sweep_multi).  Compiled for 5 waves per SIMD (96 VGPRs, a few
// bytes of scratch): with the window backtrace the one-wave kernel needs 100,
// and 4 resident waves per SIMD instead of 5 cost D_banded 830k -> 751k
// alignments/s
template <int NWV>
__global__ void __launch_bounds__(kWave * NWV) __attribute__((amdgpu_waves_per_eu(5))) myers_banded_kernel(Args a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    __shared__ int ed_slot;
    const int lane           = threadIdx.x & (kWave - 1);
    const int wv             = threadIdx.x / kWave;
    GWAMD_LDS uint8_t* base  = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint32_t* tcod = (GWAMD_LDS uint32_t*)(base + a.lds_target_off);
    GWAMD_LDS uint32_t* patL = (GWAMD_LDS uint32_t*)(base + a.lds_pat_off);
    GWAMD_LDS BandEntry* reg = (GWAMD_LDS BandEntry*)(base + a.lds_tile_off); // chunk state / tile
    const int TLE            = a.tile_bytes / int(sizeof(BandEntry));
    const int pw_stride      = a.pat_words;
    // band doubling run ahead (Args::spec_phase): launch 1 takes (pair,
    // sweep) items, launch 2 one pair per workgroup (slot = pair)
    const int K              = a.spec_sweeps;
    const int n_items        = a.spec_phase == 1 ? a.n * K : a.n;

    for (int item = blockIdx.x; item < n_items; item += gridDim.x)
    {
        const int idx = a.spec_phase == 1 ? item / K : item;
        const int ks  = a.spec_phase == 1 ? item - idx * K : 0; // launch 1: this item's sweep
        // global-typed: flat stores would hold every LDS wait of the sweep behind them
        GWAMD_GLB BandEntry* E =
            (GWAMD_GLB BandEntry*)(a.ws + size_t(a.spec_phase == 1 ? idx : int(blockIdx.x)) * size_t(a.ws_slot_bytes));
        // launch 1 stores the band matrix of its last sweep only
        const bool st_on = a.spec_phase != 1 || ks == K - 1;
        const char* q  = a.seqs + size_t(2 * idx) * a.stride;
        const char* tg = a.seqs + size_t(2 * idx + 1) * a.stride;
        const int Q    = uni(a.lens[2 * idx]);
        const int T    = uni(a.lens[2 * idx + 1]);
        PathWriter pw{a.paths + size_t(idx) * a.max_path_length, a.max_path_length};
        if (Q == 0 || T == 0)
        {
            if (a.spec_phase == 1)
                continue;
            // the reference asserts non-empty sequences; the only path
            if (wv == 0)
            {
                pw.fill(kDeletion, Q, lane);
                pw.fill(kInsertion, T, lane);
                if (lane == 0)
                    a.path_len[idx] = pw.overflow ? -1 : pw.pos;
            }
            continue;
        }
        if (wv == 0)
        {
            wave_sync();
            pack_target(tcod, tg, T, lane);
            build_patterns_lm(patL, pw_stride, q, Q, lane);
            wave_sync();
        }
        const int nwq  = (Q + kWordBits - 1) / kWordBits;
        const int dlen = Q > T ? Q - T : T - Q;
        int est        = max(1, dlen + min(T, Q) / 20); // initial_distance_guess_factor (:36, :749)
        int bw = 0, nwb = 0, db = 0, de = 0;
        // letter code of target column t (1-based)
        auto code_of = [&](int t) -> int {
            const uint32_t w = uniu(tcod[(t - 1) >> 4]);
            return int((w >> (2 * ((t - 1) & 15))) & 3u);
        };
        int kk = 0; // sweep number of this est
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
            if (bw >= Q)
                db = de = T + 1;
            else
            {
                db = Q < T ? T - Q + p + 2 : p + 2;
                de = Q < T ? Q - p + 1 : Q - (Q - T) - p + 1;
            }
            const int lastw    = nwb - 1;
            const int top_last = bw - lastw * kWordBits; // rows of the last word (>= 2 when banded)
            // pattern offset of column t: 0 (top stripe), t - db + 1 (diagonal
            // band), Q - bw (bottom stripe)
            auto col_off = [&](int t) { return t < db ? 0 : (t < de ? t - db + 1 : Q - bw); };
            int ed       = 0;
            if (a.spec_phase == 1 && kk < ks)
            {
                // launch 1: on to this item's sweep, unless the doubling
                // loop would have stopped at the full band already
                if (bw >= Q)
                {
                    if (threadIdx.x == 0)
                        a.spec_ed[item] = kSpecUnknown;
                    break;
                }
                est *= 2;
                ++kk;
                continue;
            }
            if (a.spec_phase == 1 && nwb > TLE && !st_on)
            {
                // a sweep with its chunk state in HBM needs its stores (the
                // host does not run ahead such batches)
                if (threadIdx.x == 0)
                    a.spec_ed[item] = kSpecUnknown;
                break;
            }
            if (a.spec_phase == 2 && kk < K)
            {
                const int ek = a.spec_ed[idx * K + kk];
                if (ek != kSpecUnknown)
                {
                    if (!(ek <= est || bw == Q))
                    {
                        est *= 2; // launch 1's distance rejects this band
                        ++kk;
                        continue;
                    }
                    if (kk == K - 1)
                        break; // accepted, and its band matrix is in this pair's slot
                }
            }
            // all NWV waves: several chunks with their state in LDS; half
            // wave g runs columns g + 1, g + 1 + G, ... (G = 2 * NWV), column
            // g + 1 + G q starting at step 2 g + q P and its chunk c at the
            // step after chunk c-1 (it needs chunks c and c+1 of the previous
            // column, which started at least 2 steps earlier, and its own
            // chunk c-1); P = max(2 G, nch), so the columns follow each
            // other without draining the pipeline between groups of G
            // columns; one LDS barrier per step
            auto sweep_multi = [&]() -> int {
                lds_barrier(); // this pair's target and patterns (wave 0), previous backtrace done
                for (int w = int(threadIdx.x); w < nwb; w += kWave * NWV)
                {
                    const BandEntry e0{~0u, 0u, min((w + 1) * kWordBits, bw), 0};
                    lds_put(reg + w, e0);
                    if (st_on)
                        glb_put(E + (w), e0);
                }
                lds_barrier();
                constexpr int G = 2 * NWV;
                const int g     = 2 * wv + (lane >> 5);
                const int hl    = lane & 31;
                const int P     = max(2 * G, nch);
                // the last column's last chunk
                const int nst   = 2 * ((T - 1) % G) + ((T - 1) / G) * P + nch;
                int carry       = 1; // +1 into the band's top row
                int c           = -2 * g; // chunk of the half wave's column at this step
                int tt          = 1 + g;  // the half wave's column
                for (int st = 0; st < nst; st++)
                {
                    const bool hcol = tt <= T;
                    const int tc    = min(tt, T);
                    const int code  = int((tcod[(tc - 1) >> 4] >> (2 * ((tc - 1) & 15))) & 3u);
                    const int off   = col_off(tc);
                    const bool diag = tc >= db && tc < de;
                    carry           = c == 0 ? 1 : carry;
                    {
                        const bool cin     = hcol && c >= 0 && c < nch;
                        const int w        = c * kChunkWords + hl;
                        const bool valid   = cin && w < nwb;
                        const uint64_t act = ballot(valid);
                        const int wr       = valid ? w : 0;
                        const BandEntry e  = lds_get(reg + wr);
                        uint32_t pv = e.pv, mv = e.mv;
                        int sc            = e.sc;
                        const uint32_t eq = band_pattern(patL, pw_stride, nwq, off, wr, code);
                        const bool last   = w == lastw;
                        uint32_t hb;
                        if (diag)
                        {
                            const uint64_t PB = ((ballot(pv & 1u) & act) >> 1) & ~(1ull << 31);
                            const uint64_t MB = ((ballot(mv & 1u) & act) >> 1) & ~(1ull << 31);
                            pv                = (pv >> 1) | ((uint32_t(PB >> lane) & 1u) << 31);
                            mv                = (mv >> 1) | ((uint32_t(MB >> lane) & 1u) << 31);
                            if (hl == kChunkWords - 1 && cin && c + 1 < nch)
                            {
                                const BandEntry nx = lds_get(reg + (c + 1) * kChunkWords);
                                pv |= (nx.pv & 1u) << 31;
                                mv |= (nx.mv & 1u) << 31;
                            }
                            hb = last ? 1u << max(top_last - 2, 0) : 0x40000000u;
                            if (last)
                            {
                                pv |= hb << 1;
                                mv &= ~(hb << 1);
                            }
                        }
                        else
                            hb = last ? 1u << (top_last - 1) : 0x80000000u;
                        const int r    = chunk_step2(pv, mv, eq, carry, hb, act, lane);
                        const int down = int((pv & (hb << 1)) != 0u) - int((mv & (hb << 1)) != 0u);
                        const int hout = diag ? down : r;
                        sc += diag ? r + down : r;
                        const int c0 = __builtin_amdgcn_readlane(hout, kChunkWords - 1);
                        const int c1 = __builtin_amdgcn_readlane(hout, kWave - 1);
                        carry        = cin ? ((lane >> 5) ? c1 : c0) : carry;
                        if (valid)
                        {
                            const BandEntry o{pv, mv, sc, 0};
                            lds_put(reg + w, o);
                            if (st_on)
                                glb_put(E + (size_t(tt) * nwb + w), o);
                        }
                        lds_barrier();
                    }
                    // next step: the next chunk, or the half wave's next column
                    if (++c == P)
                    {
                        c = 0;
                        tt += G;
                    }
                }
                __syncthreads(); // every wave's band-matrix stores before wave 0's backtrace
                return uni(lds_get(reg + lastw).sc);
            };
            if (NWV > 1 && nch > 1 && nwb <= TLE)
                ed = sweep_multi();
            else if (wv != 0)
                ;
            else if (nch == 1)
            {
                // one chunk: the band's words live in lanes 0..nwb-1 for the whole sweep
                const bool act_l   = lane < nwb;
                const uint64_t act = ballot(act_l);
                const bool is_last = lane == lastw;
                const uint32_t hbH = is_last ? 1u << (top_last - 1) : 0x80000000u;
                const uint32_t crb = is_last ? 1u << max(top_last - 2, 0) : 0x40000000u;
                const uint32_t cdb = crb << 1;
                uint32_t pv = ~0u, mv = 0u;
                int sc      = min((lane + 1) * kWordBits, bw);
                if (act_l && st_on)
                    glb_put(E + (lane), BandEntry{pv, mv, sc, 0});
                uint32_t eqn = band_pattern(patL, pw_stride, nwq, col_off(1), lane, code_of(1));
                for (int t = 1; t <= T; t++)
                {
                    const uint32_t eq = eqn;
                    if (t < T) // next column's pattern word, in flight during this one
                        eqn = band_pattern(patL, pw_stride, nwq, col_off(t + 1), lane, code_of(t + 1));
                    if (t < db || t >= de)
                    {
                        // horizontal stripe (myers_compute_scores_horizontal_band_impl, :496-538)
                        sc += chunk_step(pv, mv, eq, 1, hbH, act, lane);
                    }
                    else
                    {
                        // diagonal band (myers_compute_scores_diagonal_band_impl, :540-614):
                        // the previous column moves up one row; the new bottom row
                        // has no left neighbour and is assumed +1
                        const uint32_t PB = uint32_t(ballot(pv & 1u) & act);
                        const uint32_t MB = uint32_t(ballot(mv & 1u) & act);
                        uint32_t p2       = (pv >> 1) | (bit_of(PB >> 1, lane) << 31);
                        uint32_t m2       = (mv >> 1) | (bit_of(MB >> 1, lane) << 31);
                        if (is_last)
                        {
                            p2 |= cdb;
                            m2 &= ~cdb;
                        }
                        const int right = chunk_step(p2, m2, eq, 1, crb, act, lane);
                        const int down  = int((p2 & cdb) != 0u) - int((m2 & cdb) != 0u);
                        pv              = p2;
                        mv              = m2;
                        sc += right + down;
                    }
                    if (act_l && st_on)
                        glb_put(E + (size_t(t) * nwb + lane), BandEntry{pv, mv, sc, 0});
                }
                ed = uni(__builtin_amdgcn_readlane(sc, lastw));
            }
            else
            {
                // wider bands: chunk c (words 32c..32c+31) in lanes 0..31 in turn,
                // its state in LDS between columns; bands wider than the LDS
                // region (long queries) read the previous column's state back
                // from the band matrix in HBM, with a workgroup fence per column
                // (two instantiations: with the state in LDS the sweep never
                // loads from the band matrix, so its stores need no waits)
                auto sweep = [&](auto lds_tag) -> int {
                constexpr bool lds_state = decltype(lds_tag)::value;
                for (int w = lane; w < nwb; w += kWave)
                {
                    const BandEntry e0{~0u, 0u, min((w + 1) * kWordBits, bw), 0};
                    if constexpr (lds_state)
                        lds_put(reg + w, e0);
                    if (st_on || !lds_state)
                        glb_put(E + (w), e0);
                }
                __threadfence_block();
                wave_sync();
                if constexpr (lds_state)
                {
                    // two columns per pass: half hf = lane / 32 runs column
                    // t0 + hf, the second half two chunks behind the first (its
                    // chunk c needs chunks c and c+1 of column t0 and its own
                    // chunk c-1), so a column's nch dependent chunk steps are
                    // shared by two columns (nch + 2 steps per pair of columns)
                    const int hf = lane >> 5;
                    const int hl = lane & 31;
                    for (int t0 = 1; t0 <= T; t0 += 2)
                    {
                        const int tt    = t0 + hf; // this half's column
                        const bool hcol = tt <= T;
                        const int tc    = min(tt, T);
                        const int code  = int((tcod[(tc - 1) >> 4] >> (2 * ((tc - 1) & 15))) & 3u);
                        const int off   = col_off(tc);
                        const bool diag = tc >= db && tc < de;
                        int carry       = 1; // +1 into the band's top row
                        for (int st = 0; st < nch + 2; st++)
                        {
                            const int c        = st - 2 * hf;
                            const bool cin     = hcol && c >= 0 && c < nch;
                            const int w        = c * kChunkWords + hl;
                            const bool valid   = cin && w < nwb;
                            const uint64_t act = ballot(valid);
                            const int wr       = valid ? w : 0;
                            const BandEntry e  = lds_get(reg + wr);
                            uint32_t pv = e.pv, mv = e.mv;
                            int sc            = e.sc;
                            const uint32_t eq = band_pattern(patL, pw_stride, nwq, off, wr, code);
                            const bool last   = w == lastw;
                            uint32_t hb;
                            if (diag)
                            {
                                // the previous column moves up one row; word 31
                                // takes bit 0 of the next chunk's first word
                                const uint64_t PB = ((ballot(pv & 1u) & act) >> 1) & ~(1ull << 31);
                                const uint64_t MB = ((ballot(mv & 1u) & act) >> 1) & ~(1ull << 31);
                                pv                = (pv >> 1) | ((uint32_t(PB >> lane) & 1u) << 31);
                                mv                = (mv >> 1) | ((uint32_t(MB >> lane) & 1u) << 31);
                                if (hl == kChunkWords - 1 && cin && c + 1 < nch)
                                {
                                    const BandEntry nx = lds_get(reg + (c + 1) * kChunkWords);
                                    pv |= (nx.pv & 1u) << 31;
                                    mv |= (nx.mv & 1u) << 31;
                                }
                                hb = last ? 1u << max(top_last - 2, 0) : 0x40000000u;
                                if (last)
                                {
                                    pv |= hb << 1;
                                    mv &= ~(hb << 1);
                                }
                            }
                            else
                                hb = last ? 1u << (top_last - 1) : 0x80000000u;
                            const int r    = chunk_step2(pv, mv, eq, carry, hb, act, lane);
                            const int down = int((pv & (hb << 1)) != 0u) - int((mv & (hb << 1)) != 0u);
                            const int hout = diag ? down : r;
                            sc += diag ? r + down : r;
                            // chunk hand-over within each half (:527-532, :605-611)
                            const int c0 = __builtin_amdgcn_readlane(hout, kChunkWords - 1);
                            const int c1 = __builtin_amdgcn_readlane(hout, kWave - 1);
                            carry        = cin ? (hf ? c1 : c0) : carry;
                            if (valid)
                            {
                                const BandEntry o{pv, mv, sc, 0};
                                lds_put(reg + w, o);
                                if (st_on)
                                    glb_put(E + (size_t(tt) * nwb + w), o);
                            }
                        }
                    }
                    __threadfence_block();
                    wave_sync();
                    return uni(lds_get(reg + lastw).sc);
                }
                for (int t = 1; t <= T; t++)
                {
                    const int code  = code_of(t);
                    const int off   = col_off(t);
                    const bool diag = t >= db && t < de;
                    int carry       = 1; // +1 into the band's top row
                    for (int c = 0; c < nch; c++)
                    {
                        const int w        = c * kChunkWords + lane;
                        const bool valid   = lane < kChunkWords && w < nwb;
                        const uint64_t act = ballot(valid);
                        BandEntry e;
                        if constexpr (lds_state)
                            e = lds_get(reg + (valid ? w : 0));
                        else
                            e = glb_get(E + (size_t(t - 1) * nwb + (valid ? w : 0)));
                        uint32_t pv = e.pv, mv = e.mv;
                        int sc            = e.sc;
                        const uint32_t eq = band_pattern(patL, pw_stride, nwq, off, w, code);
                        const bool last   = w == lastw;
                        int hout;
                        if (!diag)
                        {
                            const uint32_t hb = last ? 1u << (top_last - 1) : 0x80000000u;
                            hout              = chunk_step(pv, mv, eq, carry, hb, act, lane);
                            sc += hout;
                        }
                        else
                        {
                            const uint32_t PB = uint32_t(ballot(pv & 1u) & act);
                            const uint32_t MB = uint32_t(ballot(mv & 1u) & act);
                            uint32_t p2       = (pv >> 1) | (bit_of(PB >> 1, lane) << 31);
                            uint32_t m2       = (mv >> 1) | (bit_of(MB >> 1, lane) << 31);
                            if (c + 1 < nch)
                            {
                                // word 31 takes bit 0 of the next chunk's first word,
                                // still the previous column's (:567-573)
                                BandEntry nx;
                                if constexpr (lds_state)
                                    nx = lds_get(reg + (c + 1) * kChunkWords);
                                else
                                    nx = glb_get(E + (size_t(t - 1) * nwb + (c + 1) * kChunkWords));
                                if (lane == kChunkWords - 1)
                                {
                                    p2 |= (nx.pv & 1u) << 31;
                                    m2 |= (nx.mv & 1u) << 31;
                                }
                            }
                            const uint32_t crb = last ? 1u << max(top_last - 2, 0) : 0x40000000u;
                            const uint32_t cdb = crb << 1;
                            if (last)
                            {
                                p2 |= cdb;
                                m2 &= ~cdb;
                            }
                            const int right = chunk_step(p2, m2, eq, carry, crb, act, lane);
                            hout            = int((p2 & cdb) != 0u) - int((m2 & cdb) != 0u);
                            pv              = p2;
                            mv              = m2;
                            sc += right + hout;
                        }
                        // chunk hand-over: horizontal delta (stripes) or vertical
                        // delta (diagonal band) of the chunk's last word (:527-532, :605-611)
                        carry = uni(__builtin_amdgcn_readlane(hout, kChunkWords - 1));
                        if (valid)
                        {
                            const BandEntry o{pv, mv, sc, 0};
                            if constexpr (lds_state)
                                lds_put(reg + w, o);
                            if (st_on || !lds_state)
                                glb_put(E + (size_t(t) * nwb + w), o);
                        }
                    }
                    if constexpr (!lds_state)
                    {
                        // this column's entries before the next column reads them
                        __threadfence_block();
                        wave_sync();
                    }
                }
                __threadfence_block();
                wave_sync();
                if constexpr (lds_state)
                    return uni(lds_get(reg + lastw).sc);
                else
                    return uni(glb_get(E + (size_t(T) * nwb + lastw)).sc);
                };
                if (nwb <= TLE)
                    ed = sweep(std::true_type{});
                else
                {
                    if (lane == 0)
                        atomicAdd(a.stats, 1ull);
                    ed = sweep(std::false_type{});
                }
            }
            if constexpr (NWV > 1)
            {
                if (!(nch > 1 && nwb <= TLE))
                {
                    // wave 0's distance to every wave (the band loop is uniform)
                    if (threadIdx.x == 0)
                        ed_slot = ed;
                    __syncthreads();
                    ed = uni(ed_slot);
                    __syncthreads();
                }
            }
            if (a.spec_phase == 1)
            {
                if (threadIdx.x == 0)
                    a.spec_ed[item] = ed;
                break;
            }
            if (ed <= est || bw == Q)
                break;
            est *= 2;
            ++kk;
        }
        if (a.spec_phase == 1)
        {
            // the next item's target and patterns (wave 0) wait for every wave
            __syncthreads();
            continue;
        }
        if (wv != 0)
            continue; // the backtrace is wave 0's
        __threadfence_block();
        wave_sync();
#ifdef GWAMD_ALN_NO_BACKTRACE // timing experiment only: forward sweep alone
        if (lane == 0)
            a.path_len[idx] = 0;
        continue;
#endif

        // backtrace (myers_backtrace_banded, :377-494): the three neighbour
        // scores of a step are evaluated by lanes 0..2 (get_myers_score,
        // :173-185) from an LDS tile of the band.  One-wave kernel (short
        // pairs, many resident): whole columns j-1..j and below, a flat range
        // of contiguous entries (coalesced refills), or HBM when two columns
        // do not fit.  Multi-wave kernels (long pairs, few resident): KW words
        // x KC columns around the walk (a step reads words (i - 2) / 32 ..
        // i / 32 of columns j - 1 and j, and the word index changes once every
        // 32 rows, so a few words over many columns last ~KC steps), refilled
        // when the walk leaves it.  Words outside [0, nwb) (the flat index
        // map aliases word nwb onto the next column) read HBM
        constexpr bool kRect = NWV > 1;
        const int64_t total  = int64_t(nwb) * (T + 1);
        const bool use_tile  = !kRect && 2 * nwb <= TLE;
        int64_t tb = 0, te = 0; // flat tile: entries [tb, te)
        auto refill_flat = [&](int jcol) {
            const int64_t hi = min<int64_t>(total, int64_t(nwb) * (jcol + 1));
            const int64_t lo = max<int64_t>(0, hi - TLE);
            const int nr     = int(hi - lo);
            wave_sync();
            // 8 entries per lane in flight before the first LDS store waits
            // (a loop of single loads waited one HBM latency per 64 entries)
            for (int e0 = 0; e0 < nr; e0 += 8 * kWave)
            {
                BandEntry v[8];
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e = e0 + u * kWave + lane;
                    if (e < nr)
                        v[u] = glb_get(E + (lo + e));
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e = e0 + u * kWave + lane;
                    if (e < nr)
                        lds_put(reg + e, v[u]);
                }
            }
            wave_sync();
            tb = lo;
            te = hi;
        };
        const int kwb = TLE >= 1024 ? 4 : 2; // rectangular tile: KW = 16 or 4 words
        const int KW  = 1 << kwb;
        const int KC  = TLE >> kwb;
        int w0 = INT_MIN / 2, c0 = INT_MIN / 2;
        auto refill = [&](int wc, int jc) {
            w0          = wc - 1;
            c0          = jc - KC + 1;
            const int n = KW * KC;
            wave_sync();
            // 8 entries per lane in flight before the first LDS store waits
            for (int e0 = 0; e0 < n; e0 += 8 * kWave)
            {
                BandEntry v[8];
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e   = e0 + u * kWave + lane;
                    const int w   = w0 + (e & (KW - 1));
                    const int col = c0 + (e >> kwb);
                    if (e < n && w >= 0 && w < nwb && col >= 0 && col <= T)
                        v[u] = glb_get(E + (int64_t(w) + int64_t(nwb) * col));
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e = e0 + u * kWave + lane;
                    if (e < n)
                        lds_put(reg + e, v[u]);
                }
            }
            wave_sync();
        };
        const uint32_t lem = (bw % kWordBits) != 0 ? (1u << (bw % kWordBits)) - 1u : ~0u;
        const int bl       = min(lane, 2);
        int i = bw, j = T;
        if (use_tile)
            refill_flat(j);
        // start from the band's last word: the reference reads word
        // band_width / 32 (:393), one past the band when band_width % 32 == 0
        int s = uni(glb_get(E + (int64_t((bw - 1) / kWordBits) + int64_t(nwb) * j)).sc);
        // score of band cell (gi, gj) (get_myers_score, :173-185) on this
        // lane, without the callers' boundary cases: 0 outside the flat range
        auto band_val = [&](int gi, int gj) -> int {
            const int wi    = (gi - 1) / kWordBits;
            const int bi    = (gi - 1) % kWordBits;
            const int64_t o = int64_t(wi) + int64_t(nwb) * gj;
            const bool inr  = o >= 0 && o < total;
            BandEntry e{0u, 0u, 0, 0};
            const unsigned ww = unsigned(wi - w0), cc = unsigned(gj - c0);
            if (kRect ? (inr && wi < nwb && ww < unsigned(KW) && cc < unsigned(KC)) : (o >= tb && o < te))
                e = kRect ? lds_get(reg + ((cc << kwb) + ww)) : lds_get(reg + (o - tb));
            else if (inr)
                e = glb_get(E + (o));
            uint32_t mask = shl_ptx(~1u, bi);
            if (wi == nwb - 1)
                mask &= lem;
            const int v = e.sc - __builtin_popcount(mask & e.pv) + __builtin_popcount(mask & e.mv);
            return inr ? v : 0;
        };
        // Window walk.  A step's move depends on its cell (i, j) and the
        // running score s; for cells with i >= 1 s is the cell's own score
        // whichever neighbour the walk arrived from (the boundary cases of
        // :173-185 only apply to rows <= 0), so lane 8(a + 4) + b takes cell
        // (i0 + a, j0 - b), a in [-4, 3], computes its score, its three
        // neighbours' (ds_bpermute, with the per-role boundary cases) and its
        // move, and the walk follows next-lane links (one v_readlane per step,
        // the step's rank kept in its lane) until a cell at the window's edge, a row
        // <= 0 or the end of the loop; the visited lanes store their moves at
        // their ranks.  Rows <= 0 take the per-step code below with the
        // running score.  Tiles must hold the window (10 rows, 9 columns).
        const bool win = kRect || (use_tile && TLE >= 10 * nwb);
        const int wr = lane >> 3, wcl = lane & 7;
        while (j > 0 && (i > 0 || j >= db))
        {
            if constexpr (kRect)
            {
                if ((i - 6) / kWordBits < w0 || (i + 3) / kWordBits >= w0 + KW || j - 8 < c0 || j > c0 + KC - 1)
                    refill((i - 1) / kWordBits, j);
            }
            else if (use_tile && int64_t(nwb) * max(j - (win ? 8 : 1), 0) < tb)
                refill_flat(j);
            if (win && i >= 1)
            {
                const int i0 = i, j0 = j;
                const int r  = i0 + wr - 4, c = j0 - wcl;
                const int ph = c >= de ? 3 : (c >= db ? 2 : 1);
                const int v  = band_val(r, c);
                const int la = lane - 8;                        // (r - 1, c)
                const int ld = ph == 2 ? lane + 1 : lane - 7;   // (r, c - 1) / (r - 1, c - 1)
                const int ll = ph == 2 ? lane + 9 : lane + 1;   // (r + 1, c - 1) / (r, c - 1)
                const int va = __builtin_amdgcn_ds_bpermute(4 * (la & 63), v);
                const int vd = __builtin_amdgcn_ds_bpermute(4 * (ld & 63), v);
                const int vl = __builtin_amdgcn_ds_bpermute(4 * (ll & 63), v);
                const int above = r <= 1 ? c : va;
                const int dg    = (ph == 2 ? r <= 0 : r <= 1) ? c - 1 : vd;
                const int left  = vl;
                const bool mins = left + 1 == v;
                const bool mdel = !mins && above + 1 == v;
                const int mr    = mins ? int(kInsertion) : (mdel ? int(kDeletion) : (dg == v ? int(kMatch) : int(kMismatch)));
                const int chosen = mins ? left : (mdel ? above : dg);
                const bool term  = wr == 0 || wr == 7 || wcl == 7 || r <= 0 || !(c > 0 && (r > 0 || c >= db));
                const int nxt    = term ? lane : (mins ? ll : (mdel ? la : ld));
                uint64_t visited = 0;
                int rank = 0, o = 32, last = 32, steps = 0;
                while (true)
                {
                    const int nx = uni(__builtin_amdgcn_readlane(nxt, o));
                    if (nx == o)
                        break;
                    rank = lane == o ? steps : rank;
                    visited |= 1ull << o;
                    last = o;
                    ++steps;
                    o = nx;
                }
                if (((visited >> lane) & 1ull) && pw.pos + rank < pw.cap)
                    pw.path[pw.pos + rank] = int8_t(mr);
                pw.pos += steps;
                if (steps > 0)
                {
                    s = uni(__builtin_amdgcn_readlane(chosen, last));
                    i = i0 + (o >> 3) - 4;
                    j = j0 - (o & 7);
                    continue;
                }
            }
            const int phase = j >= de ? 3 : (j >= db ? 2 : 1);
            // lane 0: above, lane 1: diagonal, lane 2: left
            int gi, gj, spv;
            bool special;
            if (bl == 0)
            {
                gi      = i - 1;
                gj      = j;
                special = i <= 1;
                spv     = j;
            }
            else if (bl == 1)
            {
                gi      = phase == 2 ? i : i - 1;
                gj      = j - 1;
                special = phase == 2 ? i <= 0 : i <= 1;
                spv     = j - 1;
            }
            else
            {
                gi      = phase == 2 ? i + 1 : i;
                gj      = j - 1;
                special = false;
                spv     = 0;
            }
            const int v     = special ? spv : band_val(gi, gj);
            const int above = uni(__builtin_amdgcn_readlane(v, 0));
            const int dg    = uni(__builtin_amdgcn_readlane(v, 1));
            const int left  = uni(__builtin_amdgcn_readlane(v, 2));
            int8_t r;
            if (left + 1 == s)
            {
                r = kInsertion;
                s = left;
                if (phase == 2)
                    ++i;
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
                r = dg == s ? kMatch : kMismatch;
                s = dg;
                if (phase != 2)
                    --i;
                --j;
            }
            if (lane == 0 && pw.pos < pw.cap)
                pw.path[pw.pos] = r;
            pw.pos++;
        }
        pw.overflow = pw.overflow || pw.pos > pw.cap;
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

// One column of the anti-diagonal sweep for NCK live 64-row chunks; PAR is
// the column's parity class (0: (l - p) even, 1: odd). Lane k of chunk c is
// band row k = c * 64 + lane; its cell is (i, j) = (h - k, k + l - h) with
// h = (p + l) / 2 (ukkonen_gpu.cu:96-133).
template <int NCK, int PAR>
__device__ __forceinline__ void uk_column(const GWAMD_LDS uint8_t* sA, const GWAMD_LDS uint8_t* sB,
                                          int16_t* Sl, int l, int p, int bw, int lane,
                                          const int (&lo_lim)[2][NCK], const int (&hi_lim)[2][NCK],
                                          int (&V1)[NCK], int (&V2)[NCK])
{
    constexpr int M = kUkMax;
    const int h     = (p + l) >> 1;
    int V0[NCK];
#pragma unroll
    for (int c = 0; c < NCK; c++)
    {
        const int k = c * kWave + lane;
        const int i = h - k;
        const int j = l - i;
        // lo_lim = lmin + 1 (or INT_MAX for rows past kmax / bw), hi_lim = lmax
        const bool cmp = l >= lo_lim[PAR][c] && l < hi_lim[PAR][c];
        int lo         = dpp_from_lower(V1[c]);
        int hi         = dpp_from_upper(V1[c]);
        if (c > 0)
        {
            const int x = __builtin_amdgcn_readlane(V1[c > 0 ? c - 1 : 0], kWave - 1);
            if (lane == 0)
                lo = x;
        }
        if (c + 1 < NCK)
        {
            const int x = __builtin_amdgcn_readlane(V1[c + 1 < NCK ? c + 1 : c], 0);
            if (lane == kWave - 1)
                hi = x;
        }
        const int ii  = cmp ? i - 1 : 0;
        const int jj  = cmp ? j - 1 : 0;
        const int ca  = sA[ii];
        const int cb  = sB[jj];
        const int dgv = l < 2 ? M : V2[c] + (ca == cb ? 0 : 1);
        int left, above;
        if (PAR == 0)
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
        if (c + 1 < NCK || k < bw)
            Sl[k] = int16_t(v);
    }
#pragma unroll
    for (int c = 0; c < NCK; c++)
    {
        V2[c] = V1[c];
        V1[c] = V0[c];
    }
}

// The whole sweep (ukkonen_init_score_matrix + compute_score_matrix_{even,odd})
// specialised on the number of live chunks: the per-row diagonal limits of
// both parities are computed once, and columns run in (even, odd) pairs so
// the parity is a compile-time constant in each body.
template <int NCK>
__device__ void uk_sweep(const GWAMD_LDS uint8_t* sA, const GWAMD_LDS uint8_t* sB, int16_t* S, int m, int n,
                         int p, int bw, int lane)
{
    constexpr int M     = kUkMax;
    const int cols      = n + m;
    const int kmax_odd  = (n - m + 2 * p - 1) / 2 + 1;
    const int kmax_even = (n - m + 2 * p) / 2 + 1;
    int lo_lim[2][NCK], hi_lim[2][NCK];
#pragma unroll
    for (int c = 0; c < NCK; c++)
    {
        const int k = c * kWave + lane;
#pragma unroll
        for (int par = 0; par < 2; par++)
        {
            const int d    = par ? 2 * k + 1 : 2 * k; // diagonal + p
            const int lmin = d >= p ? d - p : p - d;
            const int lmax = d <= p ? 2 * (m - p + d) + lmin : 2 * min(m, n - d + p) + lmin;
            const bool ok  = k < (par ? kmax_odd : kmax_even) && k < bw;
            lo_lim[par][c] = ok ? lmin + 1 : 0x7fffffff;
            hi_lim[par][c] = lmax;
        }
    }
    int V1[NCK], V2[NCK];
#pragma unroll
    for (int c = 0; c < NCK; c++)
    {
        V1[c] = M;
        V2[c] = M;
    }
    int l = 0;
    if (cols > 0 && ((l - p) & 1) != 0)
    {
        uk_column<NCK, 1>(sA, sB, S, l, p, bw, lane, lo_lim, hi_lim, V1, V2);
        l++;
    }
    for (; l + 1 < cols; l += 2)
    {
        uk_column<NCK, 0>(sA, sB, S + size_t(bw) * l, l, p, bw, lane, lo_lim, hi_lim, V1, V2);
        uk_column<NCK, 1>(sA, sB, S + size_t(bw) * (l + 1), l + 1, p, bw, lane, lo_lim, hi_lim, V1, V2);
    }
    if (l < cols)
        uk_column<NCK, 0>(sA, sB, S + size_t(bw) * l, l, p, bw, lane, lo_lim, hi_lim, V1, V2);
}

} // namespace

__global__ void __launch_bounds__(kWave) ukkonen_kernel(Args a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    const int lane          = threadIdx.x;
    GWAMD_LDS uint8_t* base = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint8_t* sA   = base + a.lds_target_off; // along i (the shorter sequence)
    GWAMD_LDS uint8_t* sB   = base + a.lds_seq2_off;   // along j
    // tiles of 16 KiB and more (long pairs, one workgroup per CU) are filled
    // by direct-to-LDS loads (global_load_lds_dwordx4: every piece in flight
    // at once, no staging registers), whose last 64-lane chunk may write up
    // to 1 KiB past the range: those tiles keep 1 KiB spare
    const bool tdirect      = a.tile_bytes >= 16384;
    const int TE8           = tdirect ? ((a.tile_bytes - 1024) / 2) & ~511
                                      : ((a.tile_bytes / 2) - 8) & ~7; // tile range (int16 elements); + 7 for alignment
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
        const int bw   = (1 + n - m + 2 * p + 1) / 2;
        const int cols = n + m;
        const int nck  = uni((bw + kWave - 1) / kWave);

        // anti-diagonal sweep (ukkonen_init_score_matrix + compute_score_matrix_{even,odd})
        static_assert(kUkChunks == 8, "uk_sweep dispatch covers 1..8 chunks");
        switch (nck)
        {
        case 1: uk_sweep<1>(sA, sB, S, m, n, p, bw, lane); break;
        case 2: uk_sweep<2>(sA, sB, S, m, n, p, bw, lane); break;
        case 3: uk_sweep<3>(sA, sB, S, m, n, p, bw, lane); break;
        case 4: uk_sweep<4>(sA, sB, S, m, n, p, bw, lane); break;
        case 5: uk_sweep<5>(sA, sB, S, m, n, p, bw, lane); break;
        case 6: uk_sweep<6>(sA, sB, S, m, n, p, bw, lane); break;
        case 7: uk_sweep<7>(sA, sB, S, m, n, p, bw, lane); break;
        default: uk_sweep<8>(sA, sB, S, m, n, p, bw, lane); break;
        }
        __threadfence_block();
        wave_sync();
#ifdef GWAMD_ALN_NO_BACKTRACE
        if (lane == 0)
            a.path_len[idx] = 0;
        continue;
#endif

        // backtrace over an LDS tile of the flat matrix
        const int64_t total = int64_t(bw) * cols;
        int64_t tb = -1, te = -1;
        auto refill = [&](int lcol) {
            // flat range ending with column lcol, in 16-byte pieces (8
            // elements) from an aligned start, 8 pieces per lane in flight
            // before the first LDS store waits (a loop of single dword loads
            // waited one HBM latency per 64 dwords, the bulk of a long pair's
            // backtrace)
            const int64_t hi = min<int64_t>(total, int64_t(bw) * (lcol + 1));
            const int64_t lo = max<int64_t>(0, hi - TE8) & ~int64_t(7);
            const int np16   = int((hi - lo + 7) / 8);
            const be_u32x4* src = reinterpret_cast<const be_u32x4*>(S + lo);
            GWAMD_LDS be_u32x4* dst = (GWAMD_LDS be_u32x4*)tile;
            wave_sync();
            if (tdirect)
            {
                // lane r of chunk e0 writes piece e0 + r (lanes past the range
                // reload its last piece into the spare kilobyte)
                for (int e0 = 0; e0 < np16; e0 += kWave)
                    __builtin_amdgcn_global_load_lds(src + min(e0 + lane, np16 - 1), (GWAMD_LDS void*)(dst + e0), 16, 0,
                                                     0);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            else
            for (int e0 = 0; e0 < np16; e0 += 8 * kWave)
            {
                be_u32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e = e0 + u * kWave + lane;
                    if (e < np16)
                        v[u] = src[e];
                }
#pragma unroll
                for (int u = 0; u < 8; u++)
                {
                    const int e = e0 + u * kWave + lane;
                    if (e < np16)
                        dst[e] = v[u];
                }
            }
            wave_sync();
            tb = lo;
            te = min<int64_t>(lo + 8 * int64_t(np16), total);
        };
        auto val = [&](int i, int j) -> int {
            const int k = (j - i + p) / 2;
            const int l = j + i;
            if (k < 0 || k >= bw || l < 0 || l >= cols)
                return M;
            const int64_t o = int64_t(k) + int64_t(bw) * l;
            return o >= tb && o < te ? int(tile[o - tb]) : int(S[o]);
        };
        PathWriter pw{a.paths + size_t(idx) * a.max_path_length, a.max_path_length};
        int i = m - 1, j = n - 1;
        refill(i + j);
        int s = uni(val(i, j));
        // neighbours above (i-1, j), diagonal (i-1, j-1) and left (i, j-1).
        // The move out of a cell depends on that cell alone (its value is the
        // walk's running score), so when the tile holds >= 16 columns lane
        // 8a + b takes cell (i0 - a, j0 - b) of an 8 x 8 window at the walk's
        // position (i0, j0) and decides that cell's move from its neighbours
        // (three ds_bpermute reads); the walk then only follows next-lane
        // links (one v_readlane per step) until it reaches the window's last
        // row or column, i = 0 or j = 0, and the visited lanes store their
        // moves at their rank on the path (a + b grows by 1 or 2 per step, so
        // the rank is the number of visited cells with a smaller a + b).
        // Otherwise lanes 0..2 read the three neighbours at every step.
        if (TE8 >= 16 * bw)
        {
            const int wa = lane >> 3, wb = lane & 7;
            while (i > 0 && j > 0)
            {
                if (int64_t(bw) * max(i + j - 14, 0) < tb)
                    refill(i + j);
                const int i0 = i, j0 = j;
                const int wv = val(i0 - wa, j0 - wb);
                const int up = __builtin_amdgcn_ds_bpermute(4 * (lane + 8), wv);
                const int dg = __builtin_amdgcn_ds_bpermute(4 * (lane + 9), wv);
                const int lf = __builtin_amdgcn_ds_bpermute(4 * (lane + 1), wv);
                const bool mv_ins = lf + 1 == wv;
                const bool mv_del = !mv_ins && up + 1 == wv;
                const int r       = mv_ins ? int(ins) : (mv_del ? int(del) : (dg == wv ? int(kMatch) : int(kMismatch)));
                const bool term   = wa == 7 || wb == 7 || i0 - wa <= 0 || j0 - wb <= 0;
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
                {
                    const int at = pw.pos + __builtin_popcount(sums & ((1u << (wa + wb)) - 1u));
                    if (at < pw.cap)
                        pw.path[at] = int8_t(r);
                }
                pw.pos += steps;
                i = i0 - (o >> 3);
                j = j0 - (o & 7);
            }
            pw.overflow = pw.overflow || pw.pos > pw.cap;
        }
        else
        {
            // lane 0: above (i-1, j), lane 1: diagonal (i-1, j-1), lane 2: left (i, j-1)
            const int di = lane == 2 ? 0 : 1;
            const int dj = lane == 0 ? 0 : 1;
            while (i > 0 && j > 0)
            {
                if (int64_t(bw) * (i + j - 2) < tb)
                    refill(i + j);
                const int v     = val(i - di, j - dj);
                const int above = uni(__builtin_amdgcn_readlane(v, 0));
                const int dg    = uni(__builtin_amdgcn_readlane(v, 1));
                const int left  = uni(__builtin_amdgcn_readlane(v, 2));
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
        }
        pw.fill(del, i, lane);
        pw.fill(ins, j, lane);
        if (lane == 0)
            a.path_len[idx] = pw.overflow ? -1 : pw.pos;
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// Ukkonen for bands wider than one wave's kUkChunks * 64 rows (targets past
// ~8.2 kb at the 10 % rule): the reference's own shape, one workgroup of up
// to 1,024 threads per pair with row k on thread k % NT (ukkonen_compute_
// score_matrix loops k += blockDim.x, ukkonen_gpu.cu:145-185,213-257), here
// with at most kUkWideChunks rows per thread in registers.  Per anti-diagonal
// column l: the k-1 / k+1 neighbours of column l-1 come from the lane's
// neighbour by DPP, across 64-row groups from a double-buffered LDS edge
// array written in the previous column; one workgroup barrier per column.
// Cells, initial values, the int16 store and the backtrace tie order are the
// single-wave kernel's (ukkonen_kernel above).  The backtrace runs on wave 0
// over KT x LT tiles of the (k, l) matrix staged in LDS (the sequences'
// region, no longer needed then).
__global__ void __launch_bounds__(1024) ukkonen_wide_kernel(Args a)
{
    extern __shared__ __align__(16) uint8_t lds[];
    const int tid           = threadIdx.x;
    const int NT            = blockDim.x;
    const int lane          = tid & (kWave - 1);
    const int wave          = tid / kWave;
    const int nwv           = NT / kWave;
    GWAMD_LDS uint8_t* base = (GWAMD_LDS uint8_t*)(lds);
    GWAMD_LDS uint8_t* sA   = base + a.lds_target_off; // along i (the shorter sequence)
    GWAMD_LDS uint8_t* sB   = base + a.lds_seq2_off;   // along j
    // edge values of column l-1 per 64-row group g: [parity][0: row 64g, 1: row 64g+63][group]
    GWAMD_LDS int* edge     = (GWAMD_LDS int*)(base + a.lds_edge_off);
    constexpr int kG        = kUkWideChunks * 16;
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
        for (int k = tid; k < m - 1; k += NT)
            sA[k] = uint8_t(A[k]);
        for (int k = tid; k < n - 1; k += NT)
            sB[k] = uint8_t(B[k]);
        // column -1 (never a source of a computed cell, as in ukkonen_kernel)
        for (int e = tid; e < 4 * kG; e += NT)
            edge[e] = M;
        __syncthreads();
        const int bw        = (1 + n - m + 2 * p + 1) / 2;
        const int cols      = n + m;
        const int kmax_odd  = (n - m + 2 * p - 1) / 2 + 1;
        const int kmax_even = (n - m + 2 * p) / 2 + 1;
        const int nck       = uni((bw + NT - 1) / NT); // <= kUkWideChunks (host plan)
        if (tid == 0)
        {
            atomicAdd(a.stats + 1, 1ull);
            atomicMax(a.stats + 2, (unsigned long long)nck);
        }

        int V1[kUkWideChunks], V2[kUkWideChunks], V0[kUkWideChunks];
#pragma unroll
        for (int c = 0; c < kUkWideChunks; c++)
        {
            V1[c] = M;
            V2[c] = M;
        }
        for (int l = 0; l < cols; l++)
        {
            const bool even        = ((l - p) & 1) == 0;
            const int kmax         = even ? kmax_even : kmax_odd;
            GWAMD_LDS int* e_prev  = edge + ((l + 1) & 1) * 2 * kG; // column l-1
            GWAMD_LDS int* e_cur   = edge + (l & 1) * 2 * kG;       // column l
#pragma unroll
            for (int c = 0; c < kUkWideChunks; c++)
            {
                if (c < nck)
                {
                    const int k    = c * NT + tid;
                    const int g    = c * nwv + wave; // 64-row group of k
                    const int j    = k - (p + l) / 2 + l;
                    const int i    = l - j;
                    const int d    = even ? 2 * k : 2 * k + 1;
                    const int lmin = d >= p ? d - p : p - d;
                    const int lmax = d <= p ? 2 * (m - p + d) + lmin : 2 * min(m, n - d + p) + lmin;
                    const bool cmp = k < kmax && k < bw && l >= lmin + 1 && l < lmax;
                    int lo         = dpp_from_lower(V1[c]);
                    int hi         = dpp_from_upper(V1[c]);
                    if (lane == 0)
                        lo = g > 0 ? e_prev[kG + g - 1] : M; // row 64g - 1
                    if (lane == kWave - 1)
                        hi = g + 1 < kG ? e_prev[g + 1] : M; // row 64g + 64
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
                    if (lane == 0)
                        e_cur[g] = V0[c];
                    if (lane == kWave - 1)
                        e_cur[kG + g] = V0[c];
                }
            }
#pragma unroll
            for (int c = 0; c < kUkWideChunks; c++)
            {
                V2[c] = V1[c];
                V1[c] = V0[c];
            }
            __syncthreads();
        }
        // the matrix stores of every wave before wave 0 reads them back
        __threadfence();
        __syncthreads();
        if (wave == 0)
        {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            constexpr int KT = kUkTileRows, LT = kUkTileCols;
            int tk0 = INT_MIN / 2, tl0 = INT_MIN / 2;
            // rows [k - KT/2, k + KT/2) x columns [l - LT + 1, l], band edges as M
            auto refill = [&](int kc, int lc) {
                tk0 = kc - KT / 2;
                tl0 = lc - LT + 1;
                wave_sync();
                constexpr int kPer = KT * LT / kWave, kB = 8;
                for (int e0 = 0; e0 < kPer; e0 += kB)
                {
                    int16_t v[kB];
#pragma unroll
                    for (int u = 0; u < kB; u++)
                    {
                        const int e   = (e0 + u) * kWave + lane;
                        const int kk  = tk0 + e % KT;
                        const int ll  = tl0 + e / KT;
                        const bool ok = kk >= 0 && kk < bw && ll >= 0 && ll < cols;
                        v[u]          = S[ok ? size_t(kk) + size_t(bw) * ll : 0];
                        v[u]          = ok ? v[u] : int16_t(M);
                    }
#pragma unroll
                    for (int u = 0; u < kB; u++)
                        tile[(e0 + u) * kWave + lane] = v[u];
                }
                wave_sync();
            };
            auto val = [&](int i, int j) -> int {
                const int k = (j - i + p) / 2;
                const int l = j + i;
                if (k < 0 || k >= bw || l < 0 || l >= cols)
                    return M;
                if (k >= tk0 && k < tk0 + KT && l >= tl0 && l < tl0 + LT)
                    return int(tile[(l - tl0) * KT + (k - tk0)]);
                return int(S[size_t(k) + size_t(bw) * l]);
            };
            PathWriter pw{a.paths + size_t(idx) * a.max_path_length, a.max_path_length};
            int i = m - 1, j = n - 1;
            refill((j - i + p) / 2, i + j);
            int s = uni(val(i, j));
            // lane 0: above (i-1, j), lane 1: diagonal (i-1, j-1), lane 2: left (i, j-1)
            const int di = lane == 2 ? 0 : 1;
            const int dj = lane == 0 ? 0 : 1;
            while (i > 0 && j > 0)
            {
                i = uni(i);
                j = uni(j);
                {
                    // the three neighbours inside the tile, or refill around (k, l)
                    const int kc = (j - i + p) / 2, lc = i + j;
                    if (lc - 2 < tl0 || lc > tl0 + LT - 1 || kc - 1 < tk0 || kc + 1 >= tk0 + KT)
                        refill(kc, lc);
                }
                const int v     = val(i - di, j - dj);
                const int above = uni(__builtin_amdgcn_readlane(v, 0));
                const int dg    = uni(__builtin_amdgcn_readlane(v, 1));
                const int left  = uni(__builtin_amdgcn_readlane(v, 2));
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
        }
        // the tile aliases the sequences: the next pair's copy waits for wave 0
        __syncthreads();
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
    {
        const int nwv = a->band_waves;
        if (nwv != 1 && nwv != 4 && nwv != 8 && nwv != 16)
            return hipErrorInvalidValue;
        const void* k = nwv == 4    ? reinterpret_cast<const void*>(myers_banded_kernel<4>)
                        : nwv == 8  ? reinterpret_cast<const void*>(myers_banded_kernel<8>)
                        : nwv == 16 ? reinterpret_cast<const void*>(myers_banded_kernel<16>)
                                    : reinterpret_cast<const void*>(myers_banded_kernel<1>);
        if (a->lds_bytes > 65536)
        {
            const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, a->lds_bytes);
            if (e != hipSuccess)
                return e;
        }
        if (nwv == 4)
            hipLaunchKernelGGL(myers_banded_kernel<4>, dim3(grid), dim3(kWave * 4), size_t(a->lds_bytes), stream, *a);
        else if (nwv == 8)
            hipLaunchKernelGGL(myers_banded_kernel<8>, dim3(grid), dim3(kWave * 8), size_t(a->lds_bytes), stream, *a);
        else if (nwv == 16)
            hipLaunchKernelGGL(myers_banded_kernel<16>, dim3(grid), dim3(kWave * 16), size_t(a->lds_bytes), stream, *a);
        else
            hipLaunchKernelGGL(myers_banded_kernel<1>, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    }
    else if (a->uk_threads > 0)
    {
        if (a->uk_threads % kWave != 0 || a->uk_threads > 1024)
            return hipErrorInvalidValue;
        if (a->lds_bytes > 65536)
        {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ukkonen_wide_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, a->lds_bytes);
            if (e != hipSuccess)
                return e;
        }
        hipLaunchKernelGGL(ukkonen_wide_kernel, dim3(grid), dim3(a->uk_threads), size_t(a->lds_bytes), stream, *a);
    }
    else
    {
        if (a->lds_bytes > 65536)
        {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ukkonen_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, a->lds_bytes);
            if (e != hipSuccess)
                return e;
        }
        hipLaunchKernelGGL(ukkonen_kernel, dim3(grid), dim3(kWave), size_t(a->lds_bytes), stream, *a);
    }
    return hipGetLastError();
}

extern "C" hipError_t gwamd_internal_banded_occupancy(int algo, int lds_bytes, int band_waves, int* blocks_per_cu)
{
    using namespace gwamd::aln;
    if (algo == 2)
    {
        auto occ = [&](auto kern, int threads) -> hipError_t {
            if (lds_bytes > 65536)
            {
                const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
                if (e != hipSuccess)
                    return e;
            }
            return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, kern, threads, size_t(lds_bytes));
        };
        if (band_waves == 4)
            return occ(myers_banded_kernel<4>, kWave * 4);
        if (band_waves == 8)
            return occ(myers_banded_kernel<8>, kWave * 8);
        if (band_waves == 16)
            return occ(myers_banded_kernel<16>, kWave * 16);
        return occ(myers_banded_kernel<1>, kWave);
    }
    if (lds_bytes > 65536)
    {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ukkonen_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
        if (e != hipSuccess)
            return e;
    }
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, ukkonen_kernel, kWave, size_t(lds_bytes));
}

extern "C" hipError_t gwamd_internal_ukkonen_wide_occupancy(int threads, int lds_bytes, int* blocks_per_cu)
{
    using namespace gwamd::aln;
    if (lds_bytes > 65536)
    {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ukkonen_wide_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
        if (e != hipSuccess)
            return e;
    }
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, ukkonen_wide_kernel, threads,
                                                        size_t(lds_bytes));
}

// Anti-diagonal forward pass of the banded POA kernel (poa_band.hip).
//
// Same recurrence, band layout and traceback codes as band_forward (the
// reference's runNeedlemanWunschBanded, cudapoa_nw_banded.cuh:28-487), but a
// wave sweeps a block of 64 consecutive topological rows at once: lane i owns
// row r0 + i and at step t computes the cell of absolute column
// c = cs + t - i (cs = band start of the block's first row).  Every value a
// cell needs is then already final:
//   * the horizontal neighbour (r, c-1) is the lane's own previous emission,
//     so there is no in-row prefix scan;
//   * predecessor r-1 (lane i-1) emitted column c one step earlier: one DPP
//     wave_shr per step serves it (diagonal = the previous step's value);
//   * other predecessors are read from a kAdRing-row LDS ring that every lane
//     writes as it goes; a predecessor k >= 2 rows back wrote column c+1 k
//     steps before it is needed, so its LDS read is issued one step ahead;
//   * predecessors more than kWave rows before the block are read from the
//     HBM spill rows, which this pass writes for the rows with such a
//     successor (far rows, X.flags bit 1 from the row program) and for the
//     rows the traceback's out-of-band step may read (below).
// Per-row control (record decoding, predecessor lists) happens once per block
// and lane, not once per row for the whole wave.
//
// A wave issues at most one instruction every few cycles, so the window's
// blocks are pipelined over the workgroup's waves (one per SIMD): block b runs
// on wave b % nw and trails block b-1 by the steps that make every row of
// b-1 it reads final.  Lane i of block b reads block b-1's row j at column
// c+1 (prefetch) at its step c - cs_b + i; block b-1 wrote it at its step
// c + 1 - cs_{b-1} + j <= t + (cs_b - cs_{b-1}) + 64.  Block b therefore runs
// step t once block b-1 has completed t + (cs_b - cs_{b-1}) + 65 steps
// (progress words in LDS, published every kAdSync steps).  The same lag
// orders block b's ring writes (the slots of block b-2's rows) after block
// b-1's reads of those rows, so a 128-row ring is enough.
//
// Blocks whose rows all have band start > 0 and predecessors in the ring or
// at r-1 with a band shift <= 4 take the fast step: the diagonal and vertical
// maxima over predecessor slots are taken once (max_s F_s(c-1) is the previous
// step's max_s F_s(c)), and the first maximising slot gives the reference's
// tie order (first diagonal slot, else first vertical slot, else horizontal).
// Other blocks (column-0 rows, row 0, far or strongly shifted predecessors,
// whose values follow get_score()/get_scores() quirks: cut 4-cell groups and
// minv beyond idx bw) take the general step with per-slot values.
//
// Included by poa_band.hip inside namespace gwamd::poa, after band_forward
// (it uses BandAux, BandProf and the row-record helpers defined there).
#pragma once

// kAdRing, kAdSpillDist, kReadGuard: poa_common.hpp.  Reads whose graph has a
// node with more than kAdMaxSlots predecessors take band_forward instead.
constexpr int kAdMaxSlots   = 16;
constexpr int kAdSync       = 8; // steps between progress words (power of two)
constexpr int kAdProg       = 8; // progress word slots (block b: slot b % kAdProg)
constexpr uint32_t kAdDone  = 0xFFFFFu; // progress step field: block complete (HBM stores drained)

enum : int
{
    kAdNone  = 0, // slot >= predecessor count
    kAdDpp   = 1, // predecessor r-1 in the block: lane i-1 by DPP
    kAdLds   = 2, // predecessor in the LDS ring
    kAdSpill = 3, // predecessor in the HBM spill rows
    kAdRow0  = 4, // the virtual row 0 (node without predecessors)
};

// Workgroup-shared state of the pass (static LDS of the kernel).
struct AdShared
{
    int prog[kAdProg];        // (block & 0x7ff) << 20 | completed steps (kAdDone: complete)
    int best[kAdMaxWaves];    // per wave: greatest sink value in its blocks
    int end_row[kAdMaxWaves]; // per wave: first row with it
    int stalled;              // a progress wait ran out (set by ad_wait, read by wave 0 after the pass)
};

// Per-block context shared by the step loops.
template <typename ScoreT>
struct AdCtx
{
    int lane, r, r0, V, L, bw, gap, match, mismatch, minv, cs, T, bs, base, np;
    int blk, delta; // block index; steps block blk-1 must lead by (0: no wait)
    bool act;
    bool store;     // the lane's row goes to the spill rows
    bool any_store; // some row of the block does (block-uniform)
    uint32_t a, b, c2;
    GWAMD_LDS const uint8_t* read;
    GWAMD_LDS ScoreT* ring;
    GWAMD_LDS ScoreT* sink; // kWave words: target of ring writes outside a row
    GWAMD_GLB ScoreT* spill;
    GWAMD_GLB uint8_t* codes;
    int rowsz, codes_bytes, spill_bytes;
    GWAMD_LDS AdShared* sh;
};

// wrapping add: not-yet-valid lanes may hold anything
__device__ __forceinline__ int wadd(int a, int b)
{
    return int(uint32_t(a) + uint32_t(b));
}

__device__ __forceinline__ int ad_dpp_shr1(int v)
{
    return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false); // wave_shr:1, lane 0 keeps its own
}

__device__ __forceinline__ void ad_compiler_fence()
{
    asm volatile("" ::: "memory");
}

// Wait until block blk has completed `need` steps (kAdDone: completely).
__device__ __forceinline__ void ad_wait(GWAMD_LDS AdShared* sh, int blk, uint32_t need)
{
    GWAMD_LDS int* p     = &sh->prog[blk % kAdProg];
    const uint32_t want  = min(need, kAdDone);
    // bounded: a broken hand-over must not hang the device; if the wait runs
    // out the pass carries on with values that may not be final, so the flag
    // turns the window into a generic_error instead of a silently wrong result
    for (int spin = 0;; spin++)
    {
        const uint32_t v = uint32_t(uniform(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)));
        if ((v >> 20) == uint32_t(blk & 0x7ff) && (v & kAdDone) >= want)
            break;
        if (spin == (1 << 26))
        {
            __hip_atomic_store(&sh->stalled, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            break;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    ad_compiler_fence();
}

// LDS operations of one wave execute in order, so a consumer that sees the
// word also sees every ring value written before it.
__device__ __forceinline__ void ad_publish(GWAMD_LDS AdShared* sh, int blk, uint32_t steps, int lane)
{
    ad_compiler_fence();
    if (lane == 0)
        __hip_atomic_store(&sh->prog[blk % kAdProg], int((uint32_t(blk & 0x7ff) << 20) | min(steps, kAdDone)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    ad_compiler_fence();
}

// One block of rows; NS predecessor slots per lane, GEN: general step.
// Returns the lane's emission at column L (its row's sink candidate).  Rows
// with C.store set also go to the HBM spill rows (see band_forward_ad).
template <typename ScoreT, typename SizeT, int CPL, int NS, bool GEN>
__device__ __forceinline__ int ad_block(const AdCtx<ScoreT>& C, const WinGraphG<SizeT>& g, const BandAuxG& X)
{
    const int lane = C.lane, r = C.r, bw = C.bw, gap = C.gap, minv = C.minv;
    int mode[NS], dsh[NS], tcap[NS];
    bool valid[NS];
    GWAMD_LDS const ScoreT* sp[NS];
    GWAMD_GLB const ScoreT* gp[NS];
    const int nslot = max(C.np, 1);
#pragma unroll
    for (int s = 0; s < NS; s++)
    {
        int p = -1;
        if (C.act && s < nslot)
            p = band_pred2<SizeT>(g, X, r, C.a, C.b, C.c2, s); // np == 0: the virtual row 0
        const int bsp = p <= 0 ? 0 : ra_bs(X.reca[p]);
        int m         = kAdNone;
        if (p == 0)
            m = kAdRow0;
        else if (p > 0)
            m = (p == r - 1 && lane > 0) ? kAdDpp : (p >= C.r0 - kWave ? kAdLds : kAdSpill);
        const int off = C.cs - lane - bsp + CPL - 1; // ring position of column cs - lane
        valid[s]      = m != kAdNone;
        if (s > 0 && m == kAdNone)
        {
            // empty slot: a copy of slot 0 (never a larger value, and slot 0
            // wins the ties), so the fast step needs no masking
            mode[s] = mode[0], dsh[s] = dsh[0], sp[s] = sp[0], gp[s] = gp[0], tcap[s] = tcap[0];
            continue;
        }
        mode[s] = m;
        dsh[s]  = C.bs - bsp;
        sp[s]   = m == kAdLds ? C.ring + (p % kAdRing) * C.rowsz + off : C.ring;
        gp[s]   = m == kAdSpill ? C.spill + size_t(p) * C.rowsz + off : C.spill;
        tcap[s] = m == kAdSpill ? C.rowsz - 1 - off : C.T;
    }
    // block-uniform slot properties
    uint32_t any_dpp = 0, any_spill = 0;
#pragma unroll
    for (int s = 0; s < NS; s++)
    {
        any_dpp |= (__builtin_amdgcn_ballot_w64(mode[s] == kAdDpp) != 0 ? 1u : 0u) << s;
        any_spill |= (__builtin_amdgcn_ballot_w64(mode[s] == kAdSpill) != 0 ? 1u : 0u) << s;
    }
    any_dpp   = uint32_t(uniform(int(any_dpp)));
    any_spill = uint32_t(uniform(int(any_spill)));
    if (any_spill && C.blk >= 2)
    {
        // spill rows of blocks <= blk-2 (blocks <= blk-4 ran on this wave earlier)
        ad_wait(C.sh, C.blk - 2, kAdDone);
        if (C.blk >= 3)
            ad_wait(C.sh, C.blk - 3, kAdDone);
    }

    // idx at step 0; rows past V get an index that is never in a row
    const int k0 = C.act ? C.cs - lane - C.bs : -(1 << 28);
    GWAMD_LDS const uint8_t* rp = C.read + (C.cs - lane - 1);
    GWAMD_LDS ScoreT* wp        = C.ring + (r % kAdRing) * C.rowsz + (k0 + CPL - 1);
    GWAMD_LDS ScoreT* dw        = C.sink + lane;
    // HBM: codes (idx 1..bw) and the spill row (idx 0..bw); lanes out of
    // range store into row 0 of both, which no reader uses (rows start at 1)
    GWAMD_GLB uint8_t* const codes  = C.codes;
    GWAMD_GLB uint8_t* const spillb = (GWAMD_GLB uint8_t*)(C.spill);
    const int coff = C.act ? r * bw + (k0 - 1) : 0; // + t: code of idx t + k0
    // + t*size: byte offset of the spill value of idx t + k0
    const uint32_t soff = C.act ? uint32_t(sizeof(ScoreT)) * uint32_t(r * C.rowsz + k0 + CPL - 1) : 0u;
    const int base = C.base;
    const bool act = C.act;
    const bool store     = C.act && C.store;
    const bool any_store = C.any_store;
    const int T    = uniform(C.T);
    const int tL   = C.L - C.cs + lane; // step of column L
    // per-lane copies: keeps the step loop free of scalar reloads
    int vmatch, vmism;
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmatch) : "s"(__builtin_amdgcn_readfirstlane(C.match)));
    asm volatile("v_mov_b32 %0, %1" : "=v"(vmism) : "s"(__builtin_amdgcn_readfirstlane(C.mismatch)));
    GWAMD_LDS AdShared* sh = C.sh;
    const int blk          = uniform(C.blk);
    const int delta        = uniform(C.delta);

    // the first progress wait also covers the step-0 values read here
    if (delta)
        ad_wait(sh, blk - 1, uint32_t(kAdSync - 1 + delta));
    int lv[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
        lv[s] = int(sp[s][0]);
    uint32_t rbn = rp[0]; // read byte of the next step
    int cur      = minv; // emission of the previous step (column c-1)
    int sv       = minv; // emission at column L
    // fast step state: max_s F_s(c-1) and its first slot as a diagonal code
    int dmax = INT_MIN, dcode = 3;
    // general step state: F_s(c-1) raw (get_scores) and masked (get_score)
    int rprev[NS], gprev[NS];
#pragma unroll
    for (int s = 0; s < NS; s++)
        rprev[s] = gprev[s] = INT_MIN / 2;

    // groups of kAdSync steps, unrolled (steps past T compute nothing that is
    // stored: every index is then past the band)
    for (int t0 = 0; t0 < T; t0 += kAdSync)
    {
        if (t0)
        {
            if (delta)
                ad_wait(sh, blk - 1, uint32_t(t0 + kAdSync - 1 + delta));
            ad_publish(sh, blk, uint32_t(t0), lane);
        }
#pragma unroll
        for (int u = 0; u < kAdSync; u++)
        {
        const int t   = t0 + u;
        const int idx = t + k0;
        int cv[NS];
#pragma unroll
        for (int s = 0; s < NS; s++)
            cv[s] = lv[s];
        const uint32_t rb = rbn;
        // next step's LDS values (ring values written at least one step ago,
        // see header; the read byte) issued first, so their latency overlaps
        // this step's arithmetic instead of stalling the next step
#pragma unroll
        for (int s = 0; s < NS; s++)
            lv[s] = int(sp[s][t + 1]);
        rbn = rp[t + 1];
        ad_compiler_fence();
        const int dv  = ad_dpp_shr1(cur);
        const int sig = (int(rb) == base) ? vmatch : vmism;
        const int hl  = wadd(cur, gap);
        int H, code;
        if constexpr (!GEN)
        {
            int val[NS];
#pragma unroll
            for (int s = 0; s < NS; s++)
                val[s] = ((any_dpp >> s) & 1u) && mode[s] == kAdDpp ? dv : cv[s];
            int vmax = val[0];
#pragma unroll
            for (int s = 1; s < NS; s++)
                vmax = max(vmax, val[s]);
            int vcode = 1;
#pragma unroll
            for (int s = NS - 1; s >= 1; s--)
                vcode = val[s] == vmax ? ((s << 2) | 1) : vcode;
            vcode        = val[0] == vmax ? 1 : vcode;
            const int A  = wadd(dmax, sig);
            const int Bv = wadd(vmax, gap);
            H            = trunc_score<ScoreT>(max(max(A, Bv), hl));
            code         = A == H ? dcode : (Bv == H ? vcode : (hl == H ? 2 : 3));
            dmax         = vmax;
            dcode        = vcode - 1;
        }
        else
        {
            const int tt = idx - 1; // cell index within the band row
            int v        = INT_MIN;
            int c0       = INT_MIN;
            int graw[NS];
#pragma unroll
            for (int s = 0; s < NS; s++)
            {
                int R = cv[s];
                if ((any_dpp >> s) & 1u)
                    R = mode[s] == kAdDpp ? dv : R;
                if ((any_spill >> s) & 1u)
                {
                    const int gv = int(__builtin_nontemporal_load(&gp[s][min(t, tcap[s])]));
                    R            = mode[s] == kAdSpill ? gv : R;
                }
                const int idxp = idx + dsh[s];
                R              = mode[s] == kAdRow0 ? idxp * gap : R;
                const int G    = idxp > bw ? minv : R;
                const bool cut = ((tt & ~3) + dsh[s]) >= bw + 4;
                const int vl   = cut ? minv : trunc_score<ScoreT>(max(wadd(rprev[s], sig), wadd(R, gap)));
                v              = valid[s] ? max(v, vl) : v;
                c0             = valid[s] ? max(c0, R) : c0;
                graw[s]        = valid[s] ? G : INT_MIN / 2;
                rprev[s]       = R;
            }
            H       = trunc_score<ScoreT>(max(v, hl));
            int dsl = -1, vsl = -1;
#pragma unroll
            for (int s = NS - 1; s >= 0; s--)
            {
                dsl = (wadd(gprev[s], sig) == H) ? s : dsl;
                vsl = (wadd(graw[s], gap) == H) ? s : vsl;
            }
#pragma unroll
            for (int s = 0; s < NS; s++)
                gprev[s] = graw[s];
            code = dsl >= 0 ? (dsl << 2) : (vsl >= 0 ? ((vsl << 2) | 1) : (hl == H ? 2 : 3));
            if (idx == 0)
            {
                // column-0 value (:219-245) or the minv initialize_band writes
                const int h0 = C.bs == 0 ? (C.np == 0 ? gap : trunc_score<ScoreT>(wadd(c0, gap))) : minv;
                H            = h0;
                if (act && C.bs == 0)
                    X.col0[r] = h0;
            }
        }
        const bool cell = uint32_t(idx - 1) < uint32_t(bw); // idx 1 .. bw
        const bool row  = uint32_t(idx) <= uint32_t(bw);     // idx 0 .. bw
        int e;
        if constexpr (GEN)
            e = (cell || idx == 0) ? H : minv;
        else
            e = cell ? H : minv; // idx 0 is minv: every row of a fast block has band start > 0
        *(row ? wp + t : dw) = ScoreT(e);
        codes[cell ? uint32_t(coff + t) : uint32_t(lane)] = uint8_t(code);
        if (any_store)
            *(GWAMD_GLB ScoreT*)(spillb + (row && store ? soff + uint32_t(sizeof(ScoreT) * t)
                                                         : uint32_t(sizeof(ScoreT) * lane))) = ScoreT(e);
        sv  = t == tL ? e : sv;
        cur = e;
        }
    }
    return sv;
}

// Ring padding (idx bw+1 ..) and the progress words; run by one wave before
// the pass.
// Real-row bitmap of the pass (bit r: row r is real, see band_forward_ad),
// after the ring and the sink words.
template <typename ScoreT>
__device__ __forceinline__ GWAMD_LDS uint32_t* ad_real_bits(GWAMD_LDS ScoreT* ring, int rowsz)
{
    return (GWAMD_LDS uint32_t*)(ring + kAdRing * rowsz + kWave);
}

template <typename ScoreT, int CPL>
__device__ __forceinline__ void band_ad_init(GWAMD_LDS ScoreT* ring, int rowsz, int bw, int minv, int V,
                                             GWAMD_LDS AdShared* sh, int lane)
{
    for (int k = lane; k < kAdRing * rowsz; k += kWave)
        if (k % rowsz >= bw + CPL)
            ring[k] = ScoreT(minv);
    GWAMD_LDS uint32_t* rbits = ad_real_bits(ring, rowsz);
    for (int k = lane; k <= V / 32; k += kWave)
        rbits[k] = 0;
    if (lane < kAdProg)
        sh->prog[lane] = -1;
    if (lane == 0)
        sh->stalled = 0;
    wave_sync();
}

// Blocks wave, wave + nw, ... of the pass.  Each wave leaves its first
// strictly greatest sink candidate in sh->best / sh->end_row.
//
// Spill rows.  Far rows (a successor kAdSpillDist or more rows later, X.flags
// bit 1 from the row program) are stored for this pass's own far reads.  The
// traceback's out-of-band step (band_get_slow) compares min_score_value with a
// neighbour plus match, mismatch or gap, so it can only match values <= Tmax =
// max(minv - match, minv - mismatch, minv - gap); a row without such values
// may stay out of HBM (X.flags bit 0 clear: the step then knows none of its
// values matches).  A row is *real* when every in-band cell has a candidate
// that descends, cell by cell, from the boundary values (row 0: idx * gap,
// column 0) rather than from min_score_value:
//   * a row with band start 0 (its column-0 value is real and every cell has
//     the horizontal candidate), or with only the virtual row 0 as
//     predecessor and band start < bw, is real;
//   * so is a row with a real predecessor whose band covers the row's first
//     cell (shift = band start difference < bw: the vertical candidate of
//     index 1 reads the predecessor's in-band index shift + 1; later cells
//     have the horizontal one).
// Real values are >= min(gap, mismatch, 0) * (2V + L + bw + 16), and with no
// positive wrap of the score type (max(match, 0) * (V + L + 16) in range) that
// bound above Tmax means a real row holds no value <= Tmax.  When the bound
// fails every row is stored.  Realness is decided at block setup from the
// predecessors (bitmap in LDS; in-block predecessors are assumed real and the
// assumption checked: if a lane fails, a fixed point over the block decides)
// and published before the block's first progress word.
// The pass is out of line: its register allocation is its own, so the rest of
// the band kernel (the level sort's call, the serial phases) cannot push its
// step loop into SGPR spills (config C forward 77.6 -> 65.7 ms per window,
// round 6, gpurun_out/r6b).  GWAMD_BAND_AD_INLINE builds keep it inline.
#ifdef GWAMD_BAND_AD_INLINE
#define GWAMD_BAND_AD_ATTR __forceinline__
#else
#define GWAMD_BAND_AD_ATTR __noinline__
#endif
template <typename ScoreT, typename SizeT, int CPL>
__device__ GWAMD_BAND_AD_ATTR void band_forward_ad(WinGraph<SizeT> g0, BandAux X0, int V, GWAMD_LDS const uint8_t* read,
                                                int L, const Band& B, const Scores sc, GWAMD_LDS ScoreT* ring,
                                                ScoreT* spill0, int rowsz, int score_rows, int lane, int wave, int nw,
                                                GWAMD_LDS AdShared* sh, BandProf& bp)
{
    // global-typed views of the graph, aux arrays and spill rows: out of line,
    // the struct arguments arrive with flat pointers
    const WinGraphG<SizeT> g      = typed_graph(g0);
    const BandAuxG X              = typed_aux(X0);
    GWAMD_GLB ScoreT* const spill = (GWAMD_GLB ScoreT*)(spill0);
    const uint64_t f_t0 = BandProf::now();
    const int bw        = B.bw;
    const int minv      = int(band_min_value<ScoreT>(sc));

    AdCtx<ScoreT> C;
    C.lane        = lane;
    C.V           = V;
    C.L           = L;
    C.bw          = bw;
    C.gap         = sc.gap;
    C.match       = sc.match;
    C.mismatch    = sc.mismatch;
    C.minv        = minv;
    C.read        = read;
    C.ring        = ring;
    C.sink        = ring + kAdRing * rowsz;
    C.spill       = spill;
    C.codes       = X.codes;
    C.rowsz       = rowsz;
    C.codes_bytes = score_rows * bw;
    C.spill_bytes = score_rows * rowsz * int(sizeof(ScoreT));
    C.sh          = sh;
    GWAMD_LDS uint32_t* rbits = ad_real_bits(ring, rowsz);
    auto rbit = [&](int p) -> bool { return (rbits[p >> 5] >> (p & 31)) & 1u; };
    // the real-value bound (see above); fails: every row is stored
    bool store_all;
    {
        const int64_t tmax = max(max(minv - sc.match, minv - sc.mismatch), minv - sc.gap);
        const int64_t lo   = int64_t(min(min(sc.gap, sc.mismatch), 0)) * (2 * int64_t(V) + L + bw + 16);
        const int64_t hi   = int64_t(max(sc.match, 0)) * (int64_t(V) + L + 16);
        store_all          = !(lo > tmax && hi < (sizeof(ScoreT) == 2 ? int64_t(INT16_MAX) : int64_t(INT32_MAX)));
    }
    int best = INT_MIN, end_row = 0;
    for (int blk = wave; blk * kWave + 1 <= V; blk += nw)
    {
        const uint64_t s_t0 = BandProf::now();
        const int r0 = blk * kWave + 1;
        const int r  = r0 + lane;
        const bool a = r <= V;
        const int rr = a ? r : V;
        C.blk        = blk;
        C.r0         = r0;
        C.r          = r;
        C.act        = a;
        C.a          = X.reca[rr];
        C.b          = X.recb[rr];
        C.c2         = X.recc[rr];
        C.bs         = ra_bs(C.a);
        C.base       = ra_base(C.a);
        C.np         = a ? band_np2<SizeT>(g, rr, C.a, C.b) : 0;
        const bool far = a && (X.flags[rr] & 2) != 0;
        C.cs         = uniform(C.bs); // lane 0 is always a row
        const int last = min(kWave - 1, V - r0);
        const int bsl  = __builtin_amdgcn_readlane(C.bs, last);
        C.T            = bsl + bw - C.cs + last + 1;
        C.delta        = 0;
        if (blk > 0 && nw > 1)
        {
            // producer block blk-1 (a full block): band start of its first row
            const int cs_prev = ra_bs(uint32_t(uniform(int(X.reca[r0 - kWave]))));
            C.delta           = C.cs - cs_prev + kWave + 1;
        }
        // block-uniform dispatch: slot count and fast / general step; with
        // the same predecessor scan, the real-row test (earlier blocks' bits
        // are final once block blk-1 has published its first word)
        if (blk > 0 && nw > 1)
            ad_wait(sh, blk - 1, 0);
        const int ns  = uniform(wave_max(a ? max(C.np, 1) : 1));
        bool gen      = !a ? false : (C.bs == 0 || C.np == 0);
        const bool rb = !a || C.bs == 0 || (C.np == 0 && C.bs < bw);
        bool rl       = rb;
        if (a)
        {
            for (int s = 0; s < C.np; s++)
            {
                const int p   = band_pred2<SizeT>(g, X, r, C.a, C.b, C.c2, s);
                const int bsp = ra_bs(X.reca[p]);
                if (C.bs - bsp > 4 || (p < r0 - kWave))
                    gen = true;
                if (C.bs - bsp < bw && (p >= r0 || rbit(p)))
                    rl = true;
            }
        }
        gen = __builtin_amdgcn_ballot_w64(gen || (a && C.np > 8)) != 0;
        if (__builtin_amdgcn_ballot_w64(!rl) != 0)
        {
            // some row has no real predecessor outside the block and no base
            // case: decide the block exactly, bits of earlier rounds only
            rl = rb;
            for (int it = 0; it <= kWave; it++)
            {
                if (a && rl)
                    __hip_atomic_fetch_or(&rbits[r >> 5], 1u << (r & 31), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                wave_sync();
                bool nr = rl;
                if (a && !rl)
                    for (int s = 0; s < C.np; s++)
                    {
                        const int p = band_pred2<SizeT>(g, X, r, C.a, C.b, C.c2, s);
                        if (C.bs - ra_bs(X.reca[p]) < bw && rbit(p))
                            nr = true;
                    }
                if (__builtin_amdgcn_ballot_w64(nr && !rl) == 0)
                    break;
                rl = nr;
            }
        }
        if (a && rl)
            __hip_atomic_fetch_or(&rbits[r >> 5], 1u << (r & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ad_publish(sh, blk, 0, lane); // setup done: this block's bits are out
        C.store     = a && (far || !rl || store_all);
        C.any_store = __builtin_amdgcn_ballot_w64(C.store) != 0;
        const uint64_t l_t0 = BandProf::now();
        bp.add(kBpAdSetup, l_t0 - s_t0);
        bp.add(kBpAdBlocks, 1);
        bp.add(kBpAdSteps, uint64_t(C.T));
        int sv;
        if (!gen)
        {
            if (ns <= 1)
                sv = ad_block<ScoreT, SizeT, CPL, 1, false>(C, g, X);
            else if (ns == 2)
                sv = ad_block<ScoreT, SizeT, CPL, 2, false>(C, g, X);
            else if (ns == 3)
                sv = ad_block<ScoreT, SizeT, CPL, 3, false>(C, g, X);
            else if (ns == 4)
                sv = ad_block<ScoreT, SizeT, CPL, 4, false>(C, g, X);
            else if (ns <= 6)
                sv = ad_block<ScoreT, SizeT, CPL, 6, false>(C, g, X);
            else
                sv = ad_block<ScoreT, SizeT, CPL, 8, false>(C, g, X);
        }
        else
        {
            if (ns <= 2)
                sv = ad_block<ScoreT, SizeT, CPL, 2, true>(C, g, X);
            else if (ns <= 4)
                sv = ad_block<ScoreT, SizeT, CPL, 4, true>(C, g, X);
            else if (ns <= 8)
                sv = ad_block<ScoreT, SizeT, CPL, 8, true>(C, g, X);
            else
                sv = ad_block<ScoreT, SizeT, CPL, kAdMaxSlots, true>(C, g, X);
        }
        // every ring value of the block is out; once its HBM stores drained
        // the block is complete for spill-row readers too
        ad_publish(sh, blk, uint32_t(C.T), lane);
        vm_drain();
        ad_publish(sh, blk, kAdDone, lane);
        bp.add(kBpAdLoop, BandProf::now() - l_t0);
        // end cell candidates: sinks in topological order, first strictly greatest (:349-365)
        const bool sink = a && ra_sink(C.a);
        if (!(L >= C.bs && L <= C.bs + bw))
            sv = minv;
        sv          = sink ? sv : INT_MIN;
        const int m = uniform(wave_max(sv));
        if (m > best)
        {
            const uint64_t hit = __builtin_amdgcn_ballot_w64(sv == m && sink);
            best               = m;
            end_row            = r0 + int(__builtin_ctzll(hit));
        }
        if (a)
            X.flags[r] = C.store ? 1 : 0; // bit 0: the row is in the spill rows
        bp.add(kBpRows, uint64_t(last + 1));
        bp.add(kBpMulti, gen ? 1 : 0);
    }
    if (lane == 0)
    {
        sh->best[wave]    = best;
        sh->end_row[wave] = end_row;
    }
    bp.add(kBpFwdCyc, BandProf::now() - f_t0);
}

// First strictly greatest sink over the waves' candidates (rows in order).
__device__ __forceinline__ int band_ad_end_row(GWAMD_LDS const AdShared* sh, int nw)
{
    int best = INT_MIN, end_row = 0;
    for (int w = 0; w < nw; w++)
    {
        const int b = sh->best[w], e = sh->end_row[w];
        if (b > best || (b == best && b != INT_MIN && e < end_row))
            best = b, end_row = e;
    }
    return end_row;
}

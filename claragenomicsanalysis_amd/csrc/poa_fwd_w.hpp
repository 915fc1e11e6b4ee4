// Forward pass of the LDS-resident POA kernel with 32-bit scores.
//
// The reference switches a batch to int32 scores whenever its BatchSize could
// overflow int16 (use32bitScore, cudapoa_limits.hpp:28-37: max_sequence_size
// >= 1,490 at the default scores), e.g. racon windows of a few kb.  This pass
// computes the same recurrence as nw_forward_lds_pk / nw_forward_lds_v2
// (cudapoa_nw.cuh:222-327, traceback codes in the tie order of :361-443) on
// unpacked int32 E values, E_r[j] = H_r[j] - j * gap:
//
//  * each lane owns CPL consecutive columns, wave q the span of 64*CPL
//    columns from q*64*CPL; the waves are decoupled through 64-row channels
//    of tagged 64-bit words in LDS (row, carry), as in the 16-bit passes;
//  * only the last `ring_rows` rows live in an LDS ring (int32 rows are twice
//    as wide: 4 rows for multi-kb reads); rows read from farther back are
//    spilled to HBM by the row program's flags (bit 15 of the record);
//  * one traceback code per cell: 0 diagonal, 1 vertical, 2 horizontal, plus
//    the first maximising predecessor slot << 2, so traceback_codes and every
//    phase after it are shared with the 16-bit kernel.
// No value wraps: H is within int32 for every window the reference runs with
// 32-bit scores.  Ring, read and row program are addressed through LDS
// pointers and the code / spill / carry rows through global ones (no flat
// accesses, see poa_fwd2.hpp).
//
// Included by poa_kernels.hip inside namespace gwamd::poa, after the 16-bit
// passes (RowProg, row_preds, settle_vm1).
#pragma once

// (shared-region layout of this pass: kSh*W, poa_common.hpp)

template <int CPL>
__device__ __forceinline__ void load_row_w(const GWAMD_LDS int32_t* p, int (&Q)[CPL], int& prev)
{
    static_assert(CPL % 4 == 0, "whole 16-byte groups per lane");
#pragma unroll
    for (int q = 0; q < CPL / 4; q++)
    {
        const u32x4 v = *reinterpret_cast<const GWAMD_LDS u32x4*>(p + 1 + 4 * q);
        Q[4 * q] = int(v.x), Q[4 * q + 1] = int(v.y), Q[4 * q + 2] = int(v.z), Q[4 * q + 3] = int(v.w);
    }
    prev = p[0];
}

template <int CPL>
__device__ __forceinline__ void load_row_w_glb(const GWAMD_GLB int32_t* p, int (&Q)[CPL], int& prev)
{
#pragma unroll
    for (int q = 0; q < CPL / 4; q++)
    {
        const u32x4 v = *reinterpret_cast<const GWAMD_GLB u32x4*>(p + 1 + 4 * q);
        Q[4 * q] = int(v.x), Q[4 * q + 1] = int(v.y), Q[4 * q + 2] = int(v.z), Q[4 * q + 3] = int(v.w);
    }
    prev = p[0];
    // wait inside the rare branch (see settle_vm1)
#pragma unroll
    for (int i = 0; i < CPL; i++)
    {
        uint32_t t = uint32_t(Q[i]);
        settle_vm1(t);
        Q[i] = int(t);
    }
    uint32_t t = uint32_t(prev);
    settle_vm1(t);
    prev = int(t);
}

template <int CPL, int NW, typename SizeT>
__device__ int nw_forward_lds_w(WinGraph<SizeT> g, const RowProg& P, int V, const uint8_t* read_f, int L,
                                int32_t* ring_f, int ring_stride, int32_t* spill_f, int stride, uint8_t* codes_f,
                                int code_stride, const Scores sc, GWAMD_LDS uint8_t* shb, int32_t* carry_f, int tid)
{
    g = as_global(g);
    const GWAMD_LDS uint8_t* read = lds_of(read_f);
    GWAMD_LDS int32_t* ring       = lds_of(ring_f);
    GWAMD_GLB int32_t* spill      = glb_of(spill_f);
    GWAMD_GLB uint8_t* codes      = glb_of(codes_f);
    GWAMD_GLB int32_t* carry_hbm  = glb_of(carry_f);
    const GWAMD_LDS uint32_t* prec = lds_of(P.rec);
    constexpr int kSpan = kWave * CPL;
    const int lane      = tid & (kWave - 1);
    const int wave      = uniform(tid / kWave);
    V                   = uniform(V);
    L                   = uniform(L);
    const int gap       = sc.gap;
    const int s_eq      = sc.match - gap;
    const int s_ne      = sc.mismatch - gap;
    // wave-uniform (an SGPR): P arrives through a flat pointer, and a value
    // first used inside the row loop made the compiler wait for vmcnt(0) --
    // every outstanding code / spill store -- at the top of every row
    const int mask      = uniform(P.ring_mask);
    volatile GWAMD_LDS int* prog_v = (volatile GWAMD_LDS int*)(shb + kShProgW);
    GWAMD_LDS int32_t* bnd         = (GWAMD_LDS int32_t*)(shb + kShBndW) + wave * kMaxRingW;
    GWAMD_LDS uint64_t* chan       = (GWAMD_LDS uint64_t*)(shb + kShChanW);
    volatile GWAMD_LDS uint64_t* chan_in  = chan + (wave - 1) * kChanRows; // wave > 0
    volatile GWAMD_LDS uint64_t* chan_out = chan + wave * kChanRows;       // wave < NW-1
    // owner of the last column (L-1): span, lane, cell
    const int jl       = L > 0 ? L - 1 : 0;
    const int own_span = jl / kSpan;
    const int own_lane = (jl % kSpan) / CPL;
    const int own_c    = jl % CPL;
    const int nspan    = max(1, (L + kSpan - 1) / kSpan);
    const int nsweep   = (nspan + NW - 1) / NW;
    int best_row       = 0;
    int best_val       = INT_MIN;
    for (int sweep = 0; sweep < nsweep; sweep++)
    {
    if (sweep > 0)
    {
        // progress words and channels restart empty; the previous sweep's
        // carries are in HBM
        __syncthreads();
        for (int t = tid; t < (kShBytesW(NW) - kShProgW) / 4; t += kWave * NW)
            reinterpret_cast<GWAMD_LDS int*>(shb + kShProgW)[t] = 0;
        __syncthreads();
    }
    const int span      = sweep * NW + wave;
    const int cb        = span * kSpan;
    const bool first    = span == 0;                       // holds column 0
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
        // the lane's read bytes
        int rd[CPL];
#pragma unroll
        for (int q = 0; q < CPL / 4; q++)
        {
            const uint32_t w4 = *reinterpret_cast<const GWAMD_LDS uint32_t*>(read + ja + 4 * q);
#pragma unroll
            for (int k = 0; k < 4; k++)
                rd[4 * q + k] = int((w4 >> (8 * k)) & 0xffu);
        }
        int Eprev[CPL]; // final E of row r-1 (row 0: zeros)
#pragma unroll
        for (int i = 0; i < CPL; i++)
            Eprev[i] = 0;
        int cin_prev = 0;
        int hbm_c    = 0; // carries of 64 rows from the previous sweep, one per lane
        // software pipeline: records of rows r+1, r+2 and the predecessor
        // rows of r and r+1 are loaded ahead
        uint32_t rec_c = uniform(int(prec[1]));
        uint32_t rec_a = uniform(int(prec[min(2, V)]));
        uint32_t rec_b = uniform(int(prec[min(3, V)]));
        int np_c, np_a = 1;
        int pv_c = row_preds<SizeT>(P, g, 1, rec_c, lane, np_c);
        int pv_a = V >= 2 ? row_preds<SizeT>(P, g, 2, rec_a, lane, np_a) : 0;
        GWAMD_GLB uint8_t* crow = codes + code_stride;
        GWAMD_GLB int32_t* srow = spill + stride;
        for (int r = 1; r <= V; r++, crow += code_stride, srow += stride)
        {
            int np_b = 1, pv_b = 0;
            if (r + 2 <= V)
                pv_b = row_preds<SizeT>(P, g, r + 2, rec_b, lane, np_b);
            const uint32_t rec_bb = prec[min(r + 3, V)];

            const uint32_t rec = rec_c;
            const int np       = np_c;
            const int pv       = pv_c;
            const int base     = row_base<SizeT>(g, rec, r); // bit 7: the 16-bit pass's general-path flag
            const bool spill_r = (rec >> 15) & 1;
            GWAMD_LDS int32_t* row = ring + (r & mask) * ring_stride;
            const bool anyfar  = __builtin_amdgcn_ballot_w64(lane < np && pv != 0 && r - pv > mask) != 0;
            int sig[CPL];
#pragma unroll
            for (int i = 0; i < CPL; i++)
                sig[i] = rd[i] == base ? s_eq : s_ne;
            // E of predecessor row p for the lane's cells, and E_p[jb]
            auto load_pred = [&](int p, int (&Q)[CPL], int& qprev) {
                if (p == r - 1)
                {
#pragma unroll
                    for (int i = 0; i < CPL; i++)
                        Q[i] = Eprev[i];
                    qprev = __builtin_amdgcn_update_dpp(cin_prev, Eprev[CPL - 1], 0x138, 0xf, 0xf, false);
                }
                else if (p == 0)
                {
#pragma unroll
                    for (int i = 0; i < CPL; i++)
                        Q[i] = 0;
                    qprev = 0;
                }
                else if (anyfar && r - p > mask)
                    load_row_w_glb<CPL>(spill + size_t(p) * stride + ja + kColShift, Q, qprev);
                else
                {
                    load_row_w<CPL>(ring + (p & mask) * ring_stride + ja + kColShift, Q, qprev);
                    const int bv = bnd[p & mask];
                    if (lane == 0 && cb > 0)
                        qprev = bv;
                }
            };
            int dg[CPL], vt[CPL], kd[CPL], kv[CPL], E[CPL];
            int c0v, c0kv = 0;
            {
                int Pv[CPL], prev;
                load_pred(__builtin_amdgcn_readfirstlane(pv), Pv, prev);
                c0v = prev; // wave 0, lane 0: E_p[0]
#pragma unroll
                for (int i = 0; i < CPL; i++)
                {
                    dg[i] = (i == 0 ? prev : Pv[i - 1]) + sig[i];
                    vt[i] = Pv[i] + gap;
                }
            }
            if (np > 1)
            {
                // first maximising predecessor slot per cell, pre-scaled to the
                // code layout (diagonal 4*slot, vertical 4*slot + 1)
#pragma unroll
                for (int i = 0; i < CPL; i++)
                {
                    kd[i] = 0;
                    kv[i] = 1;
                }
                for (int k = 1; k < np; k++)
                {
                    int Q[CPL], qprev;
                    load_pred(__builtin_amdgcn_readlane(pv, k), Q, qprev);
                    c0kv = qprev > c0v ? k : c0kv; // column 0: first maximising slot
                    c0v  = max(c0v, qprev);
#pragma unroll
                    for (int i = 0; i < CPL; i++)
                    {
                        const int d = (i == 0 ? qprev : Q[i - 1]) + sig[i];
                        kd[i]       = d > dg[i] ? 4 * k : kd[i];
                        dg[i]       = max(dg[i], d);
                        const int v = Q[i] + gap;
                        kv[i]       = v > vt[i] ? 4 * k + 1 : kv[i];
                        vt[i]       = max(vt[i], v);
                    }
                }
            }
            // in-lane prefix maximum (the horizontal closure in the E domain)
#pragma unroll
            for (int i = 0; i < CPL; i++)
                E[i] = i == 0 ? max(dg[0], vt[0]) : max(max(dg[i], vt[i]), E[i - 1]);
            const int m    = active ? E[CPL - 1] : INT_MIN;
            const int incl = wave_incl_max_b(m);
            const int excl = __builtin_amdgcn_update_dpp(INT_MIN, incl, 0x138, 0xf, 0xf, false);
            const int wtot = __builtin_amdgcn_readlane(incl, kWave - 1);
            int cin;
            if (first)
            {
                cin           = __builtin_amdgcn_readfirstlane(c0v) + gap; // column 0
                const int c0k = __builtin_amdgcn_readfirstlane(c0kv);
                if (lane == 0)
                {
                    row[kColShift]  = cin;
                    crow[kColShift] = uint8_t(1 | (c0k << 2));
                    if (spill_r)
                        srow[kColShift] = cin;
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
                        uint32_t hc = x <= V ? uint32_t(carry_hbm[x]) : 0u;
                        settle_vm1(hc); // wait here, once per 64 rows, not at every row's readlane
                        hbm_c = int(hc);
                    }
                    cin = __builtin_amdgcn_readlane(hbm_c, (r - 1) & (kWave - 1));
                }
                else
                {
                    // carry of this row from the previous span
                    uint64_t w = chan_in[r & (kChanRows - 1)];
                    while (uint32_t(uniform(int(uint32_t(w)))) != uint32_t(r))
                    {
                        __builtin_amdgcn_s_sleep(1);
                        w = chan_in[r & (kChanRows - 1)];
                    }
                    cin = uniform(int(uint32_t(w >> 32)));
                    if ((r & 7) == 0 && lane == 0)
                        prog_v[wave] = r;
                }
                if (lane == 0)
                {
                    bnd[r & mask] = cin;
                    if (spill_r)
                        srow[cb + kColShift] = cin; // same value as the previous span's last cell
                }
            }
            if (feed)
            {
                // flow control: the consumer must have taken row r-kChanRows+32
                if ((r & 31) == 0 && r >= kChanRows)
                {
                    while (uniform(prog_v[wave + 1]) < r - 32)
                        __builtin_amdgcn_s_sleep(1);
                }
                if (lane == 0)
                    chan_out[r & (kChanRows - 1)] = uint64_t(uint32_t(r)) | (uint64_t(uint32_t(max(cin, wtot))) << 32);
            }
            if (to_hbm && lane == 0)
                carry_hbm[r] = max(cin, wtot);
            const int bv = max(excl, cin);
#pragma unroll
            for (int i = 0; i < CPL; i++)
                E[i] = max(E[i], bv);
            if (active)
            {
                // codes: 0 diagonal, 1 vertical, 2 horizontal (+ slot << 2)
                uint32_t code[CPL];
#pragma unroll
                for (int i = 0; i < CPL; i++)
                {
                    const bool dm = E[i] == dg[i], vm = E[i] == vt[i];
                    if (np > 1)
                        code[i] = uint32_t(dm ? kd[i] : (vm ? kv[i] : 2));
                    else
                        code[i] = dm ? 0u : (vm ? 1u : 2u);
                }
#pragma unroll
                for (int q = 0; q < CPL / 4; q++)
                {
                    const u32x4 ev = {uint32_t(E[4 * q]), uint32_t(E[4 * q + 1]), uint32_t(E[4 * q + 2]),
                                      uint32_t(E[4 * q + 3])};
                    *reinterpret_cast<GWAMD_LDS u32x4*>(row + jb + kColShift + 1 + 4 * q) = ev;
                    if (spill_r)
                        *reinterpret_cast<GWAMD_GLB u32x4*>(srow + jb + kColShift + 1 + 4 * q) = ev;
                }
#pragma unroll
                for (int q = 0; q < CPL / 8; q++)
                {
                    const uint32_t w0 = code[8 * q] | (code[8 * q + 1] << 8) | (code[8 * q + 2] << 16) |
                                        (code[8 * q + 3] << 24);
                    const uint32_t w1 = code[8 * q + 4] | (code[8 * q + 5] << 8) | (code[8 * q + 6] << 16) |
                                        (code[8 * q + 7] << 24);
                    __builtin_nontemporal_store(uint64_t(w0) | (uint64_t(w1) << 32),
                                                reinterpret_cast<GWAMD_GLB uint64_t*>(crow + jb + kColShift + 1 + 8 * q));
                }
                if constexpr (CPL % 8 != 0)
                {
                    const int q = CPL / 8;
                    const uint32_t w0 = code[8 * q] | (code[8 * q + 1] << 8) | (code[8 * q + 2] << 16) |
                                        (code[8 * q + 3] << 24);
                    __builtin_nontemporal_store(w0, reinterpret_cast<GWAMD_GLB uint32_t*>(crow + jb + kColShift + 1 +
                                                                                          8 * q));
                }
            }
            if ((rec & (1u << 14)) && owner)
            {
                // sink row: E at the last column (column 0 for an empty read)
                int endv = cin;
#pragma unroll
                for (int i = 0; i < CPL; i++)
                    endv = i == own_c ? E[i] : endv;
                const int v = L == 0 ? cin : __builtin_amdgcn_readlane(endv, own_lane);
                if (best_val < v)
                    best_val = v, best_row = r;
            }
#pragma unroll
            for (int i = 0; i < CPL; i++)
                Eprev[i] = E[i];
            cin_prev = cin;
            rec_c    = rec_a;
            np_c     = np_a;
            pv_c     = pv_a;
            rec_a    = rec_b;
            np_a     = np_b;
            pv_a     = pv_b;
            rec_b    = uniform(int(rec_bb));
        }
    }
    } // sweeps
    if (nsweep > 1 || NW > 1)
    {
        // publish the end row from the wave that owns the last column
        GWAMD_LDS int* endp = (GWAMD_LDS int*)(shb + kShEndW);
        if (wave == own_span % NW && lane == 0)
            *endp = best_row;
        __syncthreads();
        best_row = uniform(*endp);
    }
    return best_row;
}

// Forward pass of the LDS-resident POA kernel, round-4 row loop.
//
// Same recurrence, same outputs (E-domain ring rows, spill rows, one traceback
// code per cell with the reference's tie order, cudapoa_nw.cuh:222-327 and
// :361-443) as nw_forward_lds_pk; what changes is the instruction stream per
// graph row, which is what bounds config B (one wave issues at most one
// instruction every 4 cycles, and the round-3 loop spent ~390 issue slots per
// wave-row on 512 cells, 150 of them scalar):
//
//  * the row program marks every row the short paths cannot take (bit 7 of
//    its record, free because bases are ASCII): source nodes, predecessor
//    lists kept in HBM, predecessors farther back than the LDS ring, and
//    bases other than A/C/G/T.  Unmarked rows never test for any of these;
//  * a row with one predecessor takes a straight path: row r-1 from registers
//    (its last cell per lane by one DPP shift), any other from the ring
//    loaded into the same registers, so the two cases join without copies;
//  * the substitution scores come from a byte table per lane (score of the
//    lane's read column against A, C, T, G in one 32-bit word per column)
//    selected for the row's base with one v_perm per register pair, when
//    both scores fit a byte (otherwise the caller keeps nw_forward_lds_pk);
//  * the first span (column 0) and the carry-feeding wave are template
//    parameters of the row loop, so each wave runs a loop without the other
//    roles' branches.
//
// Included by poa_kernels.hip inside namespace gwamd::poa, after the round-3
// forward pass whose helpers (RowProg, load_row_pk, diag_src, pk_*) it uses.
#pragma once

// 0 <= score <= 255 for both substitution scores in the E domain
__device__ __forceinline__ bool fwd2_ok(const Scores sc)
{
    const int s_eq = sc.match - sc.gap, s_ne = sc.mismatch - sc.gap;
    return s_eq >= 0 && s_eq <= 255 && s_ne >= 0 && s_ne <= 255;
}

// inclusive max-scan over the wave (builtins, so the scheduler can place
// other work in the DPP hazard slots)
__device__ __forceinline__ int wave_incl_max_b(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x111, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x112, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x114, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x118, 0xf, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x142, 0xa, 0xf, false));
    v = max(v, __builtin_amdgcn_update_dpp(INT_MIN, v, 0x143, 0xc, 0xf, false));
    return v;
}

// The row loop addresses the ring, the read and the row program through LDS
// pointers (lds_of) and the code and spill rows through global ones, so no
// access is a flat one: a flat access counts against the LDS counter too, and
// every LDS wait would then wait for the HBM code stores (measured: forward
// 45.3 -> 36.8 ms per window at config B).
typedef u32x4 fwd_u32x4;
typedef u32x2 fwd_u32x2;

template <int NR>
__device__ __forceinline__ void load_row_glb(const GWAMD_GLB int16_t* p, uint32_t (&P)[NR], uint32_t& prev)
{
    static_assert(NR % 4 == 0 || NR == 2, "4 or a multiple of 8 cells per lane");
    if constexpr (NR % 4 == 0)
    {
#pragma unroll
        for (int q = 0; q < NR / 4; q++)
        {
            const fwd_u32x4 v = *reinterpret_cast<const GWAMD_GLB fwd_u32x4*>(p + 1 + 8 * q);
            P[4 * q] = v.x, P[4 * q + 1] = v.y, P[4 * q + 2] = v.z, P[4 * q + 3] = v.w;
        }
    }
    else
    {
        const fwd_u32x2 v = *reinterpret_cast<const GWAMD_GLB fwd_u32x2*>(p + 1);
        P[0] = v.x, P[1] = v.y;
    }
    prev = uint32_t(uint16_t(p[0]));
}

template <int NR>
__device__ __forceinline__ void load_row_lds(const GWAMD_LDS int16_t* p, uint32_t (&P)[NR], uint32_t& prev)
{
    static_assert(NR % 4 == 0 || NR == 2, "4 or a multiple of 8 cells per lane");
    if constexpr (NR % 4 == 0)
    {
#pragma unroll
        for (int q = 0; q < NR / 4; q++)
        {
            const fwd_u32x4 v = *reinterpret_cast<const GWAMD_LDS fwd_u32x4*>(p + 1 + 8 * q);
            P[4 * q] = v.x, P[4 * q + 1] = v.y, P[4 * q + 2] = v.z, P[4 * q + 3] = v.w;
        }
    }
    else
    {
        const fwd_u32x2 v = *reinterpret_cast<const GWAMD_LDS fwd_u32x2*>(p + 1);
        P[0] = v.x, P[1] = v.y;
    }
    prev = uint32_t(uint16_t(p[0]));
}

template <int CPL, int NW, bool FIRST, bool FEED, typename SizeT>
__device__ __forceinline__ void fwd2_rows(WinGraph<SizeT> g, const RowProg& P, int V, const uint8_t* read_f, int L,
                                          int16_t* ring_f, int ring_stride, int16_t* spill_f, int stride,
                                          uint8_t* codes_f, int code_stride, const Scores sc,
                                          GWAMD_LDS uint8_t* shb, int16_t* carry_f, int lane, int wave, int cb,
                                          bool to_hbm, bool from_hbm, bool owner, int xl_cap, int& best_row,
                                          int& best_val)
{
    g = as_global(g);
    GWAMD_LDS int16_t* ring          = lds_of(ring_f);
    const GWAMD_LDS uint8_t* read    = lds_of(read_f);
    const GWAMD_LDS uint32_t* prec   = lds_of(P.rec);
    const GWAMD_LDS uint16_t* pxl    = lds_of(P.xl);
    GWAMD_GLB int16_t* spill         = (GWAMD_GLB int16_t*)(spill_f);
    GWAMD_GLB uint8_t* codes         = (GWAMD_GLB uint8_t*)(codes_f);
    GWAMD_GLB int16_t* carry_hbm     = (GWAMD_GLB int16_t*)(carry_f);
    constexpr int NR    = CPL / 2;
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
    GWAMD_LDS int16_t* bnd               = (GWAMD_LDS int16_t*)(shb + kShBnd) + wave * (mask + 1);
    GWAMD_LDS uint32_t* chan             = (GWAMD_LDS uint32_t*)(shb + kShChan);
    volatile GWAMD_LDS uint32_t* chan_in  = chan + (wave - 1) * kChanRows; // wave > 0
    volatile GWAMD_LDS uint32_t* chan_out = chan + wave * kChanRows;       // wave < NW-1
    volatile GWAMD_LDS int* prog_v        = (GWAMD_LDS int*)(shb + kShProg);
    const int jb     = cb + lane * CPL;
    const bool active = jb < L;
    const int ja     = active ? jb : 0; // address used by inactive lanes
    // owner of the last column (L-1) within the span: lane, cell
    const int own_lane = ((L > 0 ? L - 1 : 0) % (kWave * CPL)) / CPL;
    const int own_c    = (L > 0 ? L - 1 : 0) % CPL;
    // a whole-wave list read at offset xl_cap still ends inside the shared
    // region that follows the lists (>= 64 entries), and real lists end
    // before xl_cap
    const int xl_last = xl_cap;

    // substitution byte table: byte b of T[c] = score of read column jb + c + 1
    // (read[jb + c]) against base code b = (base >> 1) & 3 (A 0, C 1, T 2, G 3)
    uint32_t T[CPL];
#pragma unroll
    for (int c = 0; c < CPL; c++)
    {
        const int ch = int(read[ja + c]);
        T[c] = uint32_t(ch == 'A' ? s_eq : s_ne) | (uint32_t(ch == 'C' ? s_eq : s_ne) << 8) |
               (uint32_t(ch == 'T' ? s_eq : s_ne) << 16) | (uint32_t(ch == 'G' ? s_eq : s_ne) << 24);
    }
    uint32_t Eprev[NR]; // final E of row r-1 (row 0: zeros); also the loaded predecessor row
#pragma unroll
    for (int i = 0; i < NR; i++)
        Eprev[i] = 0;
    int cin_prev = 0;
    int hbm_c    = 0;
    uint32_t rec_c = uint32_t(uniform(int(prec[1])));
    uint32_t rec_n = uint32_t(uniform(int(prec[min(2, V)])));
    // lanes k < np: predecessor rows of row r (rows with a list in LDS)
    auto xls_at = [&](int i) { return int(pxl[i]); };
    int pv_c = xls_at(min(int(rec_c >> 16), xl_last) + lane);
    GWAMD_GLB uint8_t* crow = codes + code_stride;
    GWAMD_GLB int16_t* srow = spill + stride;
    for (int r = 1; r <= V; r++, crow += code_stride, srow += stride)
    {
        const uint32_t rec = rec_c;
        // next rows: the record of row r+2, the predecessor list of row r+1
        const uint32_t rec_nn = prec[min(r + 2, V)];
        // (read for every row: rows without a list get garbage they never
        // use; the offset is clamped into the list region)
        const int pv_n = xls_at(min(int(rec_n >> 16), xl_last) + lane);
        const int np       = int((rec >> 8) & 63);
        const bool spill_r = (rec >> 15) & 1;
        GWAMD_LDS int16_t* row = ring + (r & mask) * ring_stride;
        uint32_t sig[NR];
        {
            const uint32_t bsel = 0x0c040c00u + ((rec >> 1) & 3u) * 0x00010001u;
#pragma unroll
            for (int i = 0; i < NR; i++)
                sig[i] = __builtin_amdgcn_perm(T[2 * i + 1], T[2 * i], bsel);
        }
        int cin = 0;
        // Rest of the row once dg, vt (and kd, kv) hold the maxima over the
        // predecessors: in-lane prefix, closure across lanes and spans,
        // codes and stores.  Instantiated once per path so each path is
        // straight-line code.
        auto finish = [&](auto multi_tag, const uint32_t(&dg)[NR], const uint32_t(&vt)[NR],
                          const uint32_t(&kd)[NR], const uint32_t(&kv)[NR], int c0v,
                          int c0kv) __attribute__((always_inline)) {
            constexpr bool kMulti = decltype(multi_tag)::value;
            uint32_t E[NR];
#pragma unroll
            for (int i = 0; i < NR; i++)
            {
                const uint32_t s = pk_max_lo_into_hi(pk_max(dg[i], vt[i]));
                E[i]             = i == 0 ? s : pk_max_hi_carry(s, E[i - 1]);
            }
            const int m    = active ? int(int16_t(E[NR - 1] >> 16)) : kNeg;
            const int incl = wave_incl_max_b(m);
            const int excl = __builtin_amdgcn_update_dpp(kNeg, incl, 0x138, 0xf, 0xf, false);
            const int wtot = __builtin_amdgcn_readlane(incl, kWave - 1);
            if (FIRST)
            {
                cin = c0v + gap; // column 0
                if (lane == 0)
                {
                    row[kColShift]  = int16_t(cin);
                    crow[kColShift] = uint8_t(1 | (c0kv << 2));
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
            if (FEED)
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
            const uint32_t b2v = pk_bcast(max(excl, cin));
#pragma unroll
            for (int i = 0; i < NR; i++)
                E[i] = pk_max(E[i], b2v);
            if (active)
            {
                // codes: 0 diagonal, 1 vertical, 2 horizontal (+ slot << 2)
                uint32_t code[NR];
#pragma unroll
                for (int i = 0; i < NR; i++)
                {
                    if constexpr (kMulti)
                    {
                        const uint32_t a   = pk_min_u(pk_sub(E[i], dg[i]), one2); // 0: diagonal match
                        const uint32_t bb  = pk_min_u(pk_sub(E[i], vt[i]), one2); // 0: vertical match
                        const uint32_t cvh = pk_mad(bb, pk_sub(two2, kv[i]), kv[i]); // vertical or horizontal
                        code[i]            = pk_mad(a, pk_sub(cvh, kd[i]), kd[i]);
                    }
                    else
                    {
                        // one predecessor (slot 0): a + min(a, E - vt)
                        const uint32_t a = pk_min_u(pk_sub(E[i], dg[i]), one2);
                        code[i]          = pk_add(a, pk_min_u(pk_sub(E[i], vt[i]), a));
                    }
                }
                if constexpr (NR % 4 == 0)
                {
#pragma unroll
                    for (int q = 0; q < NR / 4; q++)
                    {
                        const fwd_u32x4 ev = {E[4 * q], E[4 * q + 1], E[4 * q + 2], E[4 * q + 3]};
                        *reinterpret_cast<GWAMD_LDS fwd_u32x4*>(row + jb + kColShift + 1 + 8 * q) = ev;
                        if (spill_r)
                            *reinterpret_cast<GWAMD_GLB fwd_u32x4*>(srow + jb + kColShift + 1 + 8 * q) = ev;
                        const uint32_t w0 = __builtin_amdgcn_perm(code[4 * q + 1], code[4 * q], 0x06040200u);
                        const uint32_t w1 = __builtin_amdgcn_perm(code[4 * q + 3], code[4 * q + 2], 0x06040200u);
                        __builtin_nontemporal_store(uint64_t(w0) | (uint64_t(w1) << 32),
                                                    reinterpret_cast<GWAMD_GLB uint64_t*>(crow + jb + kColShift + 1 + 8 * q));
                    }
                }
                else
                {
                    const fwd_u32x2 ev = {E[0], E[1]};
                    *reinterpret_cast<GWAMD_LDS fwd_u32x2*>(row + jb + kColShift + 1) = ev;
                    if (spill_r)
                        *reinterpret_cast<GWAMD_GLB fwd_u32x2*>(srow + jb + kColShift + 1) = ev;
                    __builtin_nontemporal_store(__builtin_amdgcn_perm(code[1], code[0], 0x06040200u),
                                                reinterpret_cast<GWAMD_GLB uint32_t*>(crow + jb + kColShift + 1));
                }
            }
            if ((rec & (1u << 14)) && owner)
            {
                // sink row: E at the last column (column 0 for an empty read),
                // read back from the ring row just stored
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
        };
        if (!(rec & 0x80u) && np == 1)
        {
            // one predecessor, in registers (row r-1) or in the ring; the ring
            // row is loaded into Eprev, so both cases continue from there
            const int d = int(rec >> 16);
            uint32_t prev;
            if (d == 1)
                prev = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(uint16_t(cin_prev))),
                                                            int(Eprev[NR - 1] >> 16), 0x138, 0xf, 0xf, false));
            else
            {
                const int ps = (r - d) & mask;
                load_row_lds<NR>(ring + ps * ring_stride + ja + kColShift, Eprev, prev);
                if (!FIRST)
                {
                    const uint32_t bv = uint32_t(uint16_t(bnd[ps]));
                    prev              = lane == 0 ? bv : prev;
                }
            }
            const int c0v = FIRST ? int(int16_t(__builtin_amdgcn_readfirstlane(prev))) : 0;
            uint32_t dg[NR], vt[NR];
            diag_src<NR>(Eprev, prev, dg);
#pragma unroll
            for (int i = 0; i < NR; i++)
            {
                dg[i] = pk_add(dg[i], sig[i]);
                vt[i] = pk_add(Eprev[i], gap2);
            }
            finish(std::false_type{}, dg, vt, dg, vt, c0v, 0);
        }
        else
        {
            // Several predecessors (slot by slot with the first maximising
            // slot), and the rows the row program marked (sources, far or
            // escaped predecessors, other bases).  The two kinds get separate
            // predecessor loaders: a loader that tested the mark per slot was
            // miscompiled (ROCm 7.2: the flag reached the slot tests inverted).
            auto rows_general = [&](auto slow_tag, int pv, int n) __attribute__((always_inline)) {
                constexpr bool kSlow = decltype(slow_tag)::value;
                auto load_pred = [&](int p, uint32_t(&Q)[NR], uint32_t& qprev) __attribute__((always_inline)) {
                    if (p == r - 1)
                    {
#pragma unroll
                        for (int i = 0; i < NR; i++)
                            Q[i] = Eprev[i];
                        qprev = uint32_t(__builtin_amdgcn_update_dpp(int(uint32_t(uint16_t(cin_prev))),
                                                                     int(Eprev[NR - 1] >> 16), 0x138, 0xf, 0xf,
                                                                     false));
                        return;
                    }
                    if constexpr (kSlow)
                    {
                        if (p == 0)
                        {
#pragma unroll
                            for (int i = 0; i < NR; i++)
                                Q[i] = 0;
                            qprev = 0;
                            return;
                        }
                        if (r - p > mask)
                        {
                            load_row_glb<NR>(spill + size_t(p) * stride + ja + kColShift, Q, qprev);
                            settle_vm<NR>(Q, qprev);
                            return;
                        }
                    }
                    load_row_lds<NR>(ring + (p & mask) * ring_stride + ja + kColShift, Q, qprev);
                    if (!FIRST)
                    {
                        const uint32_t bv = uint32_t(uint16_t(bnd[p & mask]));
                        qprev             = lane == 0 ? bv : qprev;
                    }
                };
                uint32_t dg[NR], vt[NR];
                int c0v = 0, c0kv = 0;
                {
                    uint32_t Pv[NR], prev;
                    load_pred(__builtin_amdgcn_readfirstlane(pv), Pv, prev);
                    if (FIRST)
                        c0v = int(int16_t(__builtin_amdgcn_readfirstlane(prev)));
                    diag_src<NR>(Pv, prev, dg);
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        dg[i] = pk_add(dg[i], sig[i]);
                        vt[i] = pk_add(Pv[i], gap2);
                    }
                }
                if (n > 1)
                {
                    uint32_t kd[NR], kv[NR];
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        kd[i] = 0;
                        kv[i] = one2;
                    }
                    for (int k = 1; k < n; k++)
                    {
                        uint32_t Q[NR], qprev, dq[NR];
                        load_pred(__builtin_amdgcn_readlane(pv, k), Q, qprev);
                        if (FIRST)
                        {
                            // column 0: first maximising predecessor slot
                            const int pe = int(int16_t(__builtin_amdgcn_readfirstlane(qprev)));
                            c0kv         = pe > c0v ? k : c0kv;
                            c0v          = max(c0v, pe);
                        }
                        diag_src<NR>(Q, qprev, dq);
                        const uint32_t kk4 = pk_bcast(4 * k);
                        const uint32_t kk1 = pk_bcast(4 * k + 1);
#pragma unroll
                        for (int i = 0; i < NR; i++)
                        {
                            const uint32_t d  = pk_add(dq[i], sig[i]);
                            const uint32_t nd = pk_max(dg[i], d);
                            kd[i] = pk_mad(pk_min_u(pk_sub(nd, dg[i]), one2), pk_sub(kk4, kd[i]), kd[i]);
                            dg[i] = nd;
                            const uint32_t v  = pk_add(Q[i], gap2);
                            const uint32_t nv = pk_max(vt[i], v);
                            kv[i] = pk_mad(pk_min_u(pk_sub(nv, vt[i]), one2), pk_sub(kk1, kv[i]), kv[i]);
                            vt[i] = nv;
                        }
                    }
                    finish(std::true_type{}, dg, vt, kd, kv, c0v, c0kv);
                }
                else
                    finish(std::false_type{}, dg, vt, dg, vt, c0v, 0);
            };
            if (!(rec & 0x80u))
                rows_general(std::false_type{}, pv_c, np); // np >= 2, every predecessor in the ring
            else
            {
                // predecessor rows (sources: n = 1, row 0); lists through the
                // typed LDS pointer (P's own is flat: its loads count in
                // vmcnt, so a wait for them also waits for every code store)
                int n  = np;
                int pv = 0;
                if (np == int(kRecEscape))
                    pv = row_preds<SizeT>(P, g, r, rec, lane, n);
                else
                {
                    if (np >= 2)
                        pv = lane < np ? int(pxl[(rec >> 16) + lane]) : 0;
                    else if (np == 1)
                        pv = r - int(rec >> 16);
                    if (np == 0)
                        n = 1;
                }
                const uint32_t ub = uint32_t(row_base<SizeT>(g, rec, r));
                if (!((ub & 0xc0u) == 0x40u && ((0x10008aull >> (ub & 0x3fu)) & 1u)))
                {
                    const GWAMD_LDS uint32_t* rw = reinterpret_cast<const GWAMD_LDS uint32_t*>(read + ja);
#pragma unroll
                    for (int i = 0; i < NR; i++)
                    {
                        const uint32_t wv = rw[i / 2] >> ((i & 1) * 16);
                        const int ch0 = int(wv & 0xff), ch1 = int((wv >> 8) & 0xff);
                        sig[i]        = uint32_t(uint16_t(ch0 == int(ub) ? s_eq : s_ne)) |
                                 (uint32_t(uint16_t(ch1 == int(ub) ? s_eq : s_ne)) << 16);
                    }
                }
                rows_general(std::true_type{}, pv, uniform(n));
            }
        }
        cin_prev = cin;
        rec_c    = rec_n;
        rec_n    = uint32_t(uniform(int(rec_nn)));
        pv_c     = pv_n;
    }
}

// Drop-in for nw_forward_lds_pk (same arguments and result) when fwd2_ok(sc).
template <int CPL, int NW, typename SizeT>
__device__ int nw_forward_lds_v2(WinGraph<SizeT> g, const RowProg& P, int V, const uint8_t* read, int L,
                                 int16_t* ring, int ring_stride, int16_t* spill, int stride, uint8_t* codes,
                                 int code_stride, const Scores sc, GWAMD_LDS uint8_t* shb, int16_t* carry_hbm,
                                 int tid, int xl_cap)
{
    constexpr int kSpan = kWave * CPL;
    const int lane      = tid & (kWave - 1);
    const int wave      = uniform(tid / kWave);
    V                   = uniform(V);
    L                   = uniform(L);
    const int jl        = L > 0 ? L - 1 : 0;
    const int own_span  = jl / kSpan;
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
        if (!wact || V < 1)
            continue;
        if (first)
        {
            if (feed)
                fwd2_rows<CPL, NW, true, true>(g, P, V, read, L, ring, ring_stride, spill, stride, codes,
                                               code_stride, sc, shb, carry_hbm, lane, wave, cb, to_hbm, from_hbm,
                                               owner, xl_cap, best_row, best_val);
            else
                fwd2_rows<CPL, NW, true, false>(g, P, V, read, L, ring, ring_stride, spill, stride, codes,
                                                code_stride, sc, shb, carry_hbm, lane, wave, cb, to_hbm,
                                                from_hbm, owner, xl_cap, best_row, best_val);
        }
        else if (feed)
            fwd2_rows<CPL, NW, false, true>(g, P, V, read, L, ring, ring_stride, spill, stride, codes, code_stride,
                                            sc, shb, carry_hbm, lane, wave, cb, to_hbm, from_hbm, owner, xl_cap,
                                            best_row, best_val);
        else
            fwd2_rows<CPL, NW, false, false>(g, P, V, read, L, ring, ring_stride, spill, stride, codes,
                                             code_stride, sc, shb, carry_hbm, lane, wave, cb, to_hbm, from_hbm,
                                             owner, xl_cap, best_row, best_val);
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

// ============================================================================
// TEST INFRASTRUCTURE — NOT PRODUCT CODE.
//
// CPU restatement of the reference cudaaligner global aligners (GenomeWorks
// 0.5.0, /root/reference/cudaaligner/src).  It is the parity checker for the
// HIP aligner and the "port" CPU baseline in bench.py.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
//
// Parity pinning: the CIGAR known-answer vectors of the reference's own tests
// (Test_AlignerGlobal.cpp:95-141 for create_aligner / Hirschberg-Myers / Myers,
// pygenomeworks test_cudaaligner_bindings.py:28-31), the query-pattern words of
// Test_HirschbergMyers.cu:93-140, and the edit-distance property of
// Test_MyersAlgorithm.cpp:28-61 (Myers score == naive NW score) on
// cudaaligner_test_cases.cpp's fixed pairs; all in tests/golden/aligner_kat.json.
// The reference's CPU NW (needleman_wunsch_cpu.cpp) includes
// utils/mathutils.hpp, which needs <cuda_runtime_api.h>: it cannot be built
// here without stand-in headers, so there is no oracle/_ref build of it.
//
// Alphabet (myers_gpu.cu:145, hirschberg_myers_gpu.cu:241-244): a target
// character c selects the query pattern of "ACTG"[(c >> 1) & 3]; a query
// character sets pattern bits only where it equals that letter exactly.  The
// single-query-character base case compares raw characters
// (hirschberg_myers_gpu.cu:477-508).
// ============================================================================
#include <algorithm>
#include <climits>
#include <cstdint>
#include <cstring>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle_aligner
{

enum State : int8_t
{
    kMatch     = 0, // cudaaligner.hpp:46-52
    kMismatch  = 1,
    kInsertion = 2, // absent in query, present in target
    kDeletion  = 3  // present in query, absent in target
};

// Myers match rule: query char q against target char t.
static inline bool myers_eq(char q, char t)
{
    static const char letters[4] = {'A', 'C', 'T', 'G'};
    return q == letters[(int32_t(t) >> 1) & 3];
}

// Edit-distance matrix D[i][j] (query prefix i, target prefix j), row 0 = j,
// column 0 = i; the Myers bit-vector recurrences compute exactly these values
// (Test_MyersAlgorithm.cpp:44-61 vs needleman_wunsch_cpu.cpp:100-119).
struct EdMatrix
{
    int m, n;
    std::vector<int32_t> d;
    int32_t& at(int i, int j) { return d[size_t(i) * (n + 1) + j]; }
    int32_t at(int i, int j) const { return d[size_t(i) * (n + 1) + j]; }
};

static void ed_matrix(const char* q, int m, const char* t, int n, EdMatrix& M)
{
    M.m = m;
    M.n = n;
    M.d.assign(size_t(m + 1) * (n + 1), 0);
    for (int j = 0; j <= n; j++)
        M.at(0, j) = j;
    for (int i = 1; i <= m; i++)
    {
        M.at(i, 0) = i;
        for (int j = 1; j <= n; j++)
        {
            const int32_t a = M.at(i - 1, j) + 1;
            const int32_t b = M.at(i, j - 1) + 1;
            const int32_t c = M.at(i - 1, j - 1) + (myers_eq(q[i - 1], t[j - 1]) ? 0 : 1);
            M.at(i, j)      = std::min(a, std::min(b, c));
        }
    }
}

// Last row of the edit-distance matrix: out[j] = D(m, j), j = 0..n.
// rev: the query and the target are both read backwards (the reverse sweep of
// hirschberg_myers_compute_target_mid_warp, hirschberg_myers_gpu.cu:447-449).
static void ed_last_row(const char* q, int m, const char* t, int n, bool rev, std::vector<int32_t>& out)
{
    std::vector<int32_t> col(m + 1);
    for (int i = 0; i <= m; i++)
        col[i] = i;
    out.assign(n + 1, 0);
    out[0] = m;
    for (int j = 1; j <= n; j++)
    {
        const char tc = rev ? t[n - j] : t[j - 1];
        int32_t diag  = col[0];
        col[0]        = j;
        for (int i = 1; i <= m; i++)
        {
            const char qc   = rev ? q[m - i] : q[i - 1];
            const int32_t v = std::min(std::min(col[i] + 1, col[i - 1] + 1), diag + (myers_eq(qc, tc) ? 0 : 1));
            diag            = col[i];
            col[i]          = v;
        }
        out[j] = col[m];
    }
}

// Backtrace of myers_backtrace (myers_gpu.cu:181-245) / append_myers_backtrace
// (hirschberg_myers_gpu.cu:100-160): from (m, n), insertion (left) first, then
// deletion (above), else diagonal; emitted end -> start.
static int myers_backtrace(const EdMatrix& M, int8_t* path)
{
    int i = M.m, j = M.n, pos = 0;
    int32_t s = (i > 0) ? M.at(i, j) : 0;
    while (i > 0 && j > 0)
    {
        const int32_t above = M.at(i - 1, j);
        const int32_t diag  = M.at(i - 1, j - 1);
        const int32_t left  = M.at(i, j - 1);
        int8_t r;
        if (left + 1 == s)
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
            r = (diag == s) ? kMatch : kMismatch;
            s = diag;
            --i;
            --j;
        }
        path[pos++] = r;
    }
    while (i > 0)
    {
        path[pos++] = kDeletion;
        --i;
    }
    while (j > 0)
    {
        path[pos++] = kInsertion;
        --j;
    }
    return pos;
}

// Full Myers aligner (AlignerGlobalMyers, myers_gpu.cu:881-902): whole matrix,
// then the backtrace.  Returns the path length, path in emission order.
int full_myers(const char* q, int m, const char* t, int n, int8_t* path)
{
    EdMatrix M;
    ed_matrix(q, m, t, n, M);
    return myers_backtrace(M, path);
}

static inline uint32_t bitrev5(uint32_t x)
{
    uint32_t r = 0;
    for (int b = 0; b < 5; b++)
        r |= ((x >> b) & 1u) << (4 - b);
    return r;
}

// Target split point (hirschberg_myers_gpu.cu:411-475): t minimising
// fwd(t) + rev(T - t).  Lanes stride over t by 32 keeping the first strict
// minimum; the shfl_down tree (16, 8, 4, 2, 1) keeps the lower lane on ties, so
// among minimal t the lane with the smallest 5-bit-reversed index wins, then
// the smallest t in that lane.
static int target_mid(const char* q, int qb, int qm, int qe, const char* t, int tb, int te)
{
    const int T = te - tb;
    std::vector<int32_t> fwd, rev;
    ed_last_row(q + qb, qm - qb, t + tb, T, false, fwd);
    ed_last_row(q + qm, qe - qm, t + tb, T, true, rev);
    int best_t       = 0;
    int32_t best_sum = INT_MAX;
    uint32_t best_k  = UINT_MAX;
    for (int x = 0; x <= T; x++)
    {
        const int32_t s = fwd[x] + rev[T - x];
        const uint32_t k = bitrev5(uint32_t(x) & 31u);
        if (s < best_sum || (s == best_sum && (k < best_k || (k == best_k && x < best_t))))
        {
            best_sum = s;
            best_k   = k;
            best_t   = x;
        }
    }
    return tb + best_t;
}

struct Range
{
    int qb, qe, tb, te;
};

// Hirschberg + Myers (hirschberg_myers_gpu.cu:569-638, aligner_global_hirschberg_myers.cpp):
// explicit LIFO stack of 64 ranges; the second half is pushed last, i.e.
// processed first, so the path comes out end -> start.  Base cases:
// empty target / empty query / single query character / query shorter than 63
// whose (T+1)*ceil(m/32) fits the workspace matrix of ceil(max_q/4)*64 words
// (the reference sizes it with sizeof instead of bits,
// aligner_global_hirschberg_myers.cpp:51-54).  A full stack ends the alignment
// with path length 0 (:539-541, :634-637).
int hirschberg_myers(const char* q, int Q, const char* t, int T, int max_query_length, int8_t* path)
{
    constexpr int kStack     = 64; // hirschberg_myers_stackbuffer_size
    constexpr int kFullMyers = 63; // hirschberg_myers_switch_to_myers_size
    const int64_t max_elems  = int64_t((max_query_length + 3) / 4) * (kFullMyers + 1);
    std::vector<Range> stack;
    stack.push_back({0, Q, 0, T});
    bool success = true;
    int len      = 0;
    EdMatrix M;
    while (success && !stack.empty())
    {
        const Range e = stack.back();
        stack.pop_back();
        if (e.tb == e.te)
        {
            for (int k = 0; k < e.qe - e.qb; k++)
                path[len++] = kDeletion;
        }
        else if (e.qb == e.qe)
        {
            for (int k = 0; k < e.te - e.tb; k++)
                path[len++] = kInsertion;
        }
        else if (e.qb + 1 == e.qe)
        {
            // hirschberg_myers_single_char_warp: last matching target position
            const char c = q[e.qb];
            int x        = e.te - 1;
            while (x >= e.tb)
            {
                if (t[x] == c)
                {
                    path[len++] = kMatch;
                    --x;
                    break;
                }
                path[len++] = kInsertion;
                --x;
            }
            if (path[len - 1] != kMatch)
                path[len - 1] = kMismatch;
            while (x >= e.tb)
            {
                path[len++] = kInsertion;
                --x;
            }
        }
        else
        {
            const int m = e.qe - e.qb;
            if (m < kFullMyers)
            {
                const int nw = (m + 31) / 32;
                if (int64_t(e.te - e.tb + 1) * nw <= max_elems)
                {
                    ed_matrix(q + e.qb, m, t + e.tb, e.te - e.tb, M);
                    len += myers_backtrace(M, path + len);
                    continue;
                }
            }
            const int qm = e.qb + m / 2;
            const int tm = target_mid(q, e.qb, qm, e.qe, t, e.tb, e.te);
            if (int(stack.size()) < kStack)
                stack.push_back({e.qb, qm, e.tb, tm});
            else
                success = false;
            if (success)
            {
                if (int(stack.size()) < kStack)
                    stack.push_back({qm, e.qe, tm, e.te});
                else
                    success = false;
            }
        }
    }
    return success ? len : 0;
}

// Query pattern word (myers_generate_query_pattern[_reverse],
// hirschberg_myers_gpu.cu:180-235): bit i set where query[offset+i] (or the
// reversed query) equals x.
uint32_t query_pattern(const char* q, int Q, char x, int word, bool reverse)
{
    uint32_t r     = 0;
    const int off  = word * 32;
    const int maxi = std::min(Q - off, 32);
    for (int i = 0; i < maxi; i++)
    {
        const char c = reverse ? q[Q - 1 - (i + off)] : q[i + off];
        if (c == x)
            r |= 1u << i;
    }
    return r;
}

// ---------------------------------------------------------------------------
// Banded Myers (AlignerGlobalMyersBanded, myers_gpu.cu:377-780).
//
// Literal restatement of the reference's word-level arithmetic: the band is a
// column-major matrix of nwb 32-bit words per target column (pv, mv and the
// score of each word's tracked row), processed in chunks of 32 words (one CUDA
// warp; myers_advance_block over a chunk is one 1024-bit Myers step), with the
// reference's boundary assumptions (+1 entering the band's top row, +1 for the
// row that enters the diagonal band at the bottom) and its chunk hand-over
// (the diagonal phase passes the vertical delta of the chunk's last row to the
// next chunk, :597-611).  The backtrace reads the band exactly as
// myers_backtrace_banded does (:377-494), including its index arithmetic at
// the band edges (get_myers_score with C division/remainder, column-major
// flat indexing, and PTX shift semantics: a shift count outside [0, 31]
// yields 0).
namespace
{

constexpr int kWB = 32; // myers::word_size

struct BandMats
{
    int nwb = 0, cols = 0;
    std::vector<uint32_t> pv, mv;
    std::vector<int32_t> sc;
    size_t at(int w, int t) const { return size_t(w) + size_t(nwb) * size_t(t); }
};

// (~1u) << b with the reference GPU's shl semantics (shift >= 32 -> 0)
inline uint32_t shl_ptx(uint32_t x, int b) { return (b < 0 || b >= 32) ? 0u : (x << b); }

// query pattern words, [word][char_idx] with char_idx 0..3 = A C T G
// (myers_generate_query_pattern, myers_gpu.cu:127-138)
std::vector<uint32_t> band_patterns(const char* q, int Q)
{
    const int nw = (Q + kWB - 1) / kWB;
    std::vector<uint32_t> P(size_t(nw) * 4, 0u);
    static const char letters[4] = {'A', 'C', 'T', 'G'};
    for (int w = 0; w < nw; w++)
        for (int L = 0; L < 4; L++)
            P[size_t(w) * 4 + L] = query_pattern(q, Q, letters[L], w, false);
    return P;
}

// get_query_pattern (myers_gpu.cu:140-171)
inline uint32_t band_eq(const std::vector<uint32_t>& P, int nwq, int idx, int off, char x)
{
    const int ci = (int32_t(x) >> 1) & 3;
    const int io = off / kWB, sh = off % kWB;
    uint32_t r   = P[size_t(idx + io) * 4 + ci];
    if (sh != 0)
    {
        r >>= sh;
        if (idx + io + 1 < nwq)
            r |= P[size_t(idx + io + 1) * 4 + ci] << (kWB - sh);
    }
    return r;
}

// myers_advance_block over one chunk of cnt words (myers_gpu.cu:95-125):
// carry_in enters lane 0 only; out[l] = delta at hb[l].
void advance_chunk(uint32_t* pv, uint32_t* mv, const uint32_t* eq_in, const uint32_t* hb, int cnt, int carry_in,
                   int* out)
{
    uint32_t eq[kWB] = {}, xv[kWB] = {}, ph[kWB] = {}, mh[kWB] = {};
    for (int l = 0; l < cnt; l++)
    {
        eq[l] = eq_in[l];
        xv[l] = eq[l] | mv[l];
    }
    if (carry_in < 0)
        eq[0] |= 1u;
    uint64_t carry = 0;
    for (int l = 0; l < cnt; l++)
    {
        const uint64_t s  = uint64_t(eq[l] & pv[l]) + uint64_t(pv[l]) + carry;
        const uint32_t xh = (uint32_t(s) ^ pv[l]) | eq[l];
        carry             = s >> 32;
        ph[l]             = mv[l] | ~(xh | pv[l]);
        mh[l]             = pv[l] & xh;
        out[l]            = ((ph[l] & hb[l]) ? 1 : 0) - ((mh[l] & hb[l]) ? 1 : 0);
    }
    for (int l = cnt - 1; l >= 0; l--)
    {
        ph[l] = (ph[l] << 1) | (l > 0 ? ph[l - 1] >> 31 : 0u);
        mh[l] = (mh[l] << 1) | (l > 0 ? mh[l - 1] >> 31 : 0u);
    }
    if (carry_in < 0)
        mh[0] |= 1u;
    if (carry_in > 0)
        ph[0] |= 1u;
    for (int l = 0; l < cnt; l++)
    {
        pv[l] = mh[l] | ~(xv[l] | ph[l]);
        mv[l] = ph[l] & xv[l];
    }
}

// myers_compute_scores_horizontal_band_impl (myers_gpu.cu:496-538)
void band_horizontal(BandMats& M, const std::vector<uint32_t>& P, int nwq, const char* t, int tb, int te, int width,
                     int po)
{
    const int nw = M.nwb;
    for (int c = tb; c < te; c++)
    {
        int carry = 1; // worst case for the band's top row
        for (int w0 = 0; w0 < nw; w0 += kWB)
        {
            const int cnt = std::min(kWB, nw - w0);
            uint32_t pv[kWB], mv[kWB], eq[kWB], hb[kWB];
            int out[kWB];
            for (int l = 0; l < cnt; l++)
            {
                const int w = w0 + l;
                pv[l]       = M.pv[M.at(w, c - 1)];
                mv[l]       = M.mv[M.at(w, c - 1)];
                hb[l]       = 1u << (w == nw - 1 ? width - (nw - 1) * kWB - 1 : kWB - 1);
                eq[l]       = band_eq(P, nwq, w, po, t[c - 1]);
            }
            advance_chunk(pv, mv, eq, hb, cnt, carry, out);
            for (int l = 0; l < cnt; l++)
            {
                const int w          = w0 + l;
                M.sc[M.at(w, c)]     = M.sc[M.at(w, c - 1)] + out[l];
                M.pv[M.at(w, c)]     = pv[l];
                M.mv[M.at(w, c)]     = mv[l];
            }
            carry = cnt == kWB ? out[kWB - 1] : 0;
        }
    }
}

// myers_compute_scores_diagonal_band_impl (myers_gpu.cu:540-614)
void band_diagonal(BandMats& M, const std::vector<uint32_t>& P, int nwq, const char* t, int tb, int te, int bw)
{
    const int nw = M.nwb;
    for (int c = tb; c < te; c++)
    {
        int carry_down = 1;
        for (int w0 = 0; w0 < nw; w0 += kWB)
        {
            const int cnt = std::min(kWB, nw - w0);
            uint32_t opv[kWB], omv[kWB], pv[kWB], mv[kWB], eq[kWB], crb[kWB];
            int out[kWB];
            for (int l = 0; l < cnt; l++)
            {
                opv[l] = M.pv[M.at(w0 + l, c - 1)];
                omv[l] = M.mv[M.at(w0 + l, c - 1)];
            }
            for (int l = 0; l < cnt; l++)
            {
                const int w = w0 + l;
                pv[l]       = (opv[l] >> 1) | (l + 1 < cnt ? opv[l + 1] << (kWB - 1) : 0u);
                mv[l]       = (omv[l] >> 1) | (l + 1 < cnt ? omv[l + 1] << (kWB - 1) : 0u);
                if (l == kWB - 1 && w < nw - 1)
                {
                    pv[l] |= M.pv[M.at(w + 1, c - 1)] << (kWB - 1);
                    mv[l] |= M.mv[M.at(w + 1, c - 1)] << (kWB - 1);
                }
                crb[l]             = 1u << (w == nw - 1 ? bw - (nw - 1) * kWB - 2 : kWB - 2);
                const uint32_t cdb = crb[l] << 1;
                eq[l]              = band_eq(P, nwq, w, c - tb + 1, t[c - 1]);
                if (w == nw - 1)
                {
                    pv[l] |= cdb;
                    mv[l] &= ~cdb;
                }
            }
            advance_chunk(pv, mv, eq, crb, cnt, carry_down, out);
            int cd_last = 0;
            for (int l = 0; l < cnt; l++)
            {
                const int w        = w0 + l;
                const uint32_t cdb = crb[l] << 1;
                const int cd       = ((pv[l] & cdb) ? 1 : 0) - ((mv[l] & cdb) ? 1 : 0);
                M.sc[M.at(w, c)]   = M.sc[M.at(w, c - 1)] + out[l] + cd;
                M.pv[M.at(w, c)]   = pv[l];
                M.mv[M.at(w, c)]   = mv[l];
                cd_last            = cd;
            }
            carry_down = cnt == kWB ? cd_last : 0;
        }
    }
}

// get_myers_score (myers_gpu.cu:173-185) on the flat column-major band
inline int32_t band_gms(const BandMats& M, int i, int j, uint32_t lem)
{
    const int wi   = (i - 1) / kWB;
    const int bi   = (i - 1) % kWB;
    const long o   = long(wi) + long(M.nwb) * long(j);
    if (o < 0 || size_t(o) >= M.sc.size())
        return 0; // outside the band matrix (never reached on valid inputs)
    uint32_t mask = shl_ptx(~1u, bi);
    if (wi == M.nwb - 1)
        mask &= lem;
    return M.sc[o] - __builtin_popcount(mask & M.pv[o]) + __builtin_popcount(mask & M.mv[o]);
}

// myers_backtrace_banded (myers_gpu.cu:377-494)
int band_backtrace(const BandMats& M, int db, int de, int bw, int T, int8_t* path)
{
    int i = bw, j = T, pos = 0;
    const uint32_t lem = (bw % kWB) != 0 ? (1u << (bw % kWB)) - 1u : ~0u;
    // The reference starts from score(band_width / 32, T) (:393), one word past
    // the band when band_width % 32 == 0 (a read of uninitialised workspace);
    // both implementations here start from the band's last word, which is the
    // same word in every other case.
    int32_t s          = M.sc[M.at((bw - 1) / kWB, j)];
    auto step_hv = [&](int32_t left, int32_t above, int32_t diag, int di_left, int di_above, int di_diag, int dj_diag) {
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
            r = (diag == s) ? kMatch : kMismatch;
            s = diag;
            i += di_diag;
            j += dj_diag;
        }
        path[pos++] = r;
    };
    while (j >= de)
    {
        const int32_t above = i <= 1 ? j : band_gms(M, i - 1, j, lem);
        const int32_t diag  = i <= 1 ? j - 1 : band_gms(M, i - 1, j - 1, lem);
        const int32_t left  = band_gms(M, i, j - 1, lem);
        step_hv(left, above, diag, 0, -1, -1, -1);
    }
    while (j >= db)
    {
        const int32_t above = i <= 1 ? j : band_gms(M, i - 1, j, lem);
        const int32_t diag  = i <= 0 ? j - 1 : band_gms(M, i, j - 1, lem);
        const int32_t left  = band_gms(M, i + 1, j - 1, lem);
        step_hv(left, above, diag, +1, -1, 0, -1);
    }
    while (i > 0 && j > 0)
    {
        const int32_t above = i == 1 ? j : band_gms(M, i - 1, j, lem);
        const int32_t diag  = i == 1 ? j - 1 : band_gms(M, i - 1, j - 1, lem);
        const int32_t left  = band_gms(M, i, j - 1, lem);
        step_hv(left, above, diag, 0, -1, -1, -1);
    }
    while (i > 0)
    {
        path[pos++] = kDeletion;
        --i;
    }
    while (j > 0)
    {
        path[pos++] = kInsertion;
        --j;
    }
    return pos;
}

} // namespace

// Banded Myers aligner (myers_banded_kernel, myers_gpu.cu:706-780): Ukkonen
// band doubling from the estimate |T-Q| + min(T,Q)/20.  Empty sequences
// (the reference asserts non-empty) give the all-insertion / all-deletion path.
// Outputs the accepted band width and the number of tries when non-null.
int myers_banded(const char* q, int Q, const char* t, int T, int8_t* path, int* band_out, int* tries_out)
{
    if (Q == 0 || T == 0)
    {
        int pos = 0;
        for (int k = 0; k < Q; k++)
            path[pos++] = kDeletion;
        for (int k = 0; k < T; k++)
            path[pos++] = kInsertion;
        return pos;
    }
    const int nwq               = (Q + kWB - 1) / kWB;
    const std::vector<uint32_t> P = band_patterns(q, Q);
    const int dlen              = std::abs(T - Q);
    int est                     = std::max(1, dlen + std::min(T, Q) / 20);
    for (int tries = 1;; tries++)
    {
        int p  = std::min(std::min(T, Q), (est - dlen) / 2);
        int bw = std::min(1 + 2 * p + dlen, Q);
        if (bw % kWB == 1 && bw != Q)
        {
            p += 1;
            bw = std::min(1 + 2 * p + dlen, Q);
        }
        BandMats M;
        M.nwb  = (bw + kWB - 1) / kWB;
        M.cols = T + 1;
        M.pv.assign(size_t(M.nwb) * (T + 1), 0u);
        M.mv.assign(size_t(M.nwb) * (T + 1), 0u);
        M.sc.assign(size_t(M.nwb) * (T + 1), 0);
        for (int w = 0; w < M.nwb; w++)
        {
            M.pv[M.at(w, 0)] = ~0u;
            M.mv[M.at(w, 0)] = 0u;
            M.sc[M.at(w, 0)] = std::min((w + 1) * kWB, bw);
        }
        int db, de;
        if (bw >= Q)
        {
            db = de = T + 1;
            band_horizontal(M, P, nwq, t, 1, T + 1, Q, 0);
        }
        else
        {
            db = Q < T ? T - Q + p + 2 : p + 2;
            de = Q < T ? Q - p + 1 : Q - (Q - T) - p + 1;
            band_horizontal(M, P, nwq, t, 1, db, bw, 0);
            band_diagonal(M, P, nwq, t, db, de, bw);
            band_horizontal(M, P, nwq, t, de, T + 1, bw, Q - bw);
        }
        const int ed = M.sc[M.at(M.nwb - 1, T)];
        if (ed <= est || bw == Q)
        {
            if (band_out)
                *band_out = bw;
            if (tries_out)
                *tries_out = tries;
            return band_backtrace(M, db, de, bw, T, path);
        }
        est *= 2;
    }
}

// ---------------------------------------------------------------------------
// Ukkonen (AlignerGlobalUkkonen, ukkonen_gpu.cu:59-329): banded NW with unit
// costs over the diagonals [-p, n-m+p] of the (shorter x longer) matrix, in
// the reference's (k, l) coordinates k = (j - i + p) / 2, l = i + j, int16
// scores with 32766 for cells outside the band.  The matrix is initialised and
// filled exactly as ukkonen_init_score_matrix / ukkonen_compute_score_matrix_
// {even,odd} do, and the backtrace reads it through to_band_indices with C
// division (ukkonen_backtrace_kernel, :59-141).  Characters compare raw.
constexpr int kUkkonenP        = 100;   // aligner_global_ukkonen.cpp:29
constexpr int16_t kUkkonenMax  = 32766; // numeric_limits<int16_t>::max() - 1

int ukkonen(const char* q, int Q, const char* t, int T, int p, int8_t* path)
{
    int m = Q + 1, n = T + 1;
    const char* a = q; // along i (the shorter sequence after the swap)
    const char* b = t; // along j
    int8_t ins = kInsertion, del = kDeletion;
    if (m > n)
    {
        std::swap(n, m);
        std::swap(a, b);
        std::swap(ins, del);
    }
    const int bw   = (1 + n - m + 2 * p + 1) / 2;
    const int cols = n + m;
    std::vector<int16_t> S(size_t(bw) * cols);
    auto at = [&](int k, int l) -> int16_t& { return S[size_t(k) + size_t(bw) * size_t(l)]; };
    for (int k = 0; k < bw; k++)
        for (int l = 0; l < cols; l++)
        {
            const int j = k - (p + l) / 2 + l;
            const int i = l - j;
            at(k, l)    = i == 0 ? int16_t(j) : j == 0 ? int16_t(i) : kUkkonenMax;
        }
    const int kmax_odd  = (n - m + 2 * p - 1) / 2 + 1;
    const int kmax_even = (n - m + 2 * p) / 2 + 1;
    const int M         = kUkkonenMax;
    for (int l = 0; l < cols; l++)
    {
        const bool even = ((l - p) & 1) == 0;
        const int kmax  = even ? kmax_even : kmax_odd;
        for (int k = 0; k < kmax && k < bw; k++)
        {
            const int d    = even ? 2 * k : 2 * k + 1; // 2k(+1) - p + p
            const int lmin = std::abs(d - p);
            const int lmax = d <= p ? 2 * (m - p + d) + lmin : 2 * std::min(m, n - d + p) + lmin;
            if (!(lmin + 1 <= l && l < lmax))
                continue;
            const int j    = k - (p + l) / 2 + l;
            const int i    = l - j;
            const int diag = l - 2 < 0 ? M : at(k, l - 2) + (a[i - 1] == b[j - 1] ? 0 : 1);
            int left, above;
            if (even)
            {
                left  = (k - 1 < 0 || l - 1 < 0) ? M : at(k - 1, l - 1) + 1;
                above = l - 1 < 0 ? M : at(k, l - 1) + 1;
            }
            else
            {
                left  = l - 1 < 0 ? M : at(k, l - 1) + 1;
                above = (l - 1 < 0 || k + 1 >= bw) ? M : at(k + 1, l - 1) + 1;
            }
            at(k, l) = int16_t(std::min(diag, std::min(left, above)));
        }
    }
    auto val = [&](int i, int j) -> int {
        const int k = (j - i + p) / 2;
        const int l = j + i;
        return (k < 0 || k >= bw || l < 0 || l >= cols) ? M : int(at(k, l));
    };
    int i = m - 1, j = n - 1, pos = 0;
    int s = val(i, j);
    while (i > 0 && j > 0)
    {
        const int above = val(i - 1, j);
        const int diag  = val(i - 1, j - 1);
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
            r = (diag == s) ? kMatch : kMismatch;
            s = diag;
            --i;
            --j;
        }
        path[pos++] = r;
    }
    while (i > 0)
    {
        path[pos++] = del;
        --i;
    }
    while (j > 0)
    {
        path[pos++] = ins;
        --j;
    }
    return pos;
}

} // namespace oracle_aligner

extern "C" {

// algo: 0 = Hirschberg-Myers (create_aligner default), 1 = full Myers,
// 2 = banded Myers, 3 = Ukkonen (p = 100).
// Writes the path in emission order (end -> start, as the device kernels do;
// the host reverses it, aligner_global.cpp:185).  Returns the length, or -1 if
// path_cap is too small.
int oracle_align(int algo, const char* q, int qlen, const char* t, int tlen, int max_query_length, int8_t* path,
                 int path_cap)
{
    std::vector<int8_t> buf(size_t(qlen) + tlen + 8);
    int n = 0;
    switch (algo)
    {
    case 0: n = oracle_aligner::hirschberg_myers(q, qlen, t, tlen, max_query_length, buf.data()); break;
    case 1: n = oracle_aligner::full_myers(q, qlen, t, tlen, buf.data()); break;
    case 2: n = oracle_aligner::myers_banded(q, qlen, t, tlen, buf.data(), nullptr, nullptr); break;
    default: n = oracle_aligner::ukkonen(q, qlen, t, tlen, oracle_aligner::kUkkonenP, buf.data()); break;
    }
    if (n > path_cap)
        return -1;
    std::memcpy(path, buf.data(), size_t(n));
    return n;
}

// Batch (CPU baseline): pairs i at seqs + off[2i] (query) / off[2i+1] (target);
// path i at paths + i * path_stride.  OpenMP over pairs.  Returns threads used.
int oracle_align_batch(int algo, int n, const char* seqs, const int64_t* off, const int32_t* len, int max_query_length,
                       int8_t* paths, int32_t* path_len, int path_stride, int nthreads)
{
    int used = 1;
#ifdef _OPENMP
    if (nthreads > 0)
        omp_set_num_threads(nthreads);
#pragma omp parallel
    {
#pragma omp single
        used = omp_get_num_threads();
    }
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int i = 0; i < n; i++)
    {
        path_len[i] = oracle_align(algo, seqs + off[2 * i], len[2 * i], seqs + off[2 * i + 1], len[2 * i + 1],
                                   max_query_length, paths + size_t(i) * path_stride, path_stride);
    }
    return used;
}

int oracle_edit_distance(const char* q, int qlen, const char* t, int tlen)
{
    std::vector<int32_t> row;
    oracle_aligner::ed_last_row(q, qlen, t, tlen, false, row);
    return row[tlen];
}

// Banded Myers with the accepted band width and number of tries.
int oracle_myers_banded(const char* q, int qlen, const char* t, int tlen, int8_t* path, int* band, int* tries)
{
    return oracle_aligner::myers_banded(q, qlen, t, tlen, path, band, tries);
}

// Ukkonen with an explicit p (the aligner uses 100).
int oracle_ukkonen(const char* q, int qlen, const char* t, int tlen, int p, int8_t* path)
{
    return oracle_aligner::ukkonen(q, qlen, t, tlen, p, path);
}

uint32_t oracle_query_pattern(const char* q, int qlen, char x, int word, int reverse)
{
    return oracle_aligner::query_pattern(q, qlen, x, word, reverse != 0);
}

} // extern "C"

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

} // namespace oracle_aligner

extern "C" {

// algo: 0 = Hirschberg-Myers (create_aligner default), 1 = full Myers.
// Writes the path in emission order (end -> start, as the device kernels do;
// the host reverses it, aligner_global.cpp:185).  Returns the length, or -1 if
// path_cap is too small.
int oracle_align(int algo, const char* q, int qlen, const char* t, int tlen, int max_query_length, int8_t* path,
                 int path_cap)
{
    std::vector<int8_t> buf(size_t(qlen) + tlen + 8);
    int n = algo == 0 ? oracle_aligner::hirschberg_myers(q, qlen, t, tlen, max_query_length, buf.data())
                      : oracle_aligner::full_myers(q, qlen, t, tlen, buf.data());
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

uint32_t oracle_query_pattern(const char* q, int qlen, char x, int word, int reverse)
{
    return oracle_aligner::query_pattern(q, qlen, x, word, reverse != 0);
}

} // extern "C"

// ============================================================================
// TEST INFRASTRUCTURE — NOT PRODUCT CODE.
//
// CPU restatement of the reference cudapoa algorithm (GenomeWorks 0.5.0,
// /root/reference/cudapoa/src).  It is the parity checker for the HIP path and
// the "port" CPU baseline in bench.py.  Only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it.
//
// Parity pinning: checked against every known-answer vector the reference's own
// tests hold for this path (tests/golden/*.json, produced by
// tests/golden/make_golden.py from the reference test files):
//   Test_CudapoaTopSort.cu:37-58, Test_CudapoaNW.cu:76-180,
//   Test_CudapoaAddAlignment.cu:104-224, Test_CudapoaGenerateConsensus.cu:77-156,
//   Test_CudapoaBatch.cu:151-203, pygenomeworks test_cudapoa_bindings.py:95-146.
// SPOA itself is absent (empty submodule), so consensus-vs-SPOA is unpinned.
//
// Every function cites the reference file:line it restates.  Arithmetic is done
// in int32; for full alignment that equals the reference's int16/int32 ScoreT in
// every cell that feeds an output (cudapoa_limits.hpp:28-53 guarantees no
// overflow).  Banded alignment reads out-of-band cells through the reference's
// flat row layout (cudapoa_nw_banded.cuh:28-153), so it is emulated on a flat
// ScoreT array of the same shape, with ScoreT's own min value.
// ============================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace oracle
{

constexpr int kMaxEdges      = 50; // CUDAPOA_MAX_NODE_EDGES, cudapoa_structs.cuh:18
constexpr int kMaxAlignments = 50; // CUDAPOA_MAX_NODE_ALIGNMENTS, cudapoa_structs.cuh:21
constexpr int kCellsPerThread = 4; // CELLS_PER_THREAD, cudapoa_structs.cuh:25
constexpr int kBandPad        = 8; // CUDAPOA_BANDED_MATRIX_RIGHT_PADDING, :27

// StatusType values, cudapoa.hpp:26-38
enum Status : uint8_t
{
    kSuccess                 = 0,
    kExceededMaxPoas         = 1,
    kExceededMaxSeqSize      = 2,
    kExceededMaxSeqsPerPoa   = 3,
    kNodeCountExceeded       = 4,
    kEdgeCountExceeded       = 5,
    kSeqLenExceededNodes     = 6,
    kLoopCountExceeded       = 7,
    kOutputTypeUnavailable   = 8,
    kGenericError            = 9,
};

// Fixed-slot window graph, same slot semantics as GraphDetails
// (cudapoa_structs.cuh:108-167).  Node ids are int32 here.
struct Graph
{
    int max_nodes = 0;
    int max_seqs  = 0;
    int node_count = 0;
    std::vector<uint8_t> base;
    std::vector<int32_t> in_e, out_e, aln;
    std::vector<uint16_t> in_cnt, out_cnt, aln_cnt, in_w, cov;
    std::vector<int32_t> sorted, pos;
    // msa bookkeeping (cudapoa_add_alignment.cuh:237-264)
    bool msa = false;
    std::vector<uint16_t> ecov, ecov_cnt;
    std::vector<int32_t> seq_begin;

    void init(int maxn, int maxs, bool with_msa)
    {
        max_nodes = maxn;
        max_seqs  = maxs;
        msa       = with_msa;
        base.assign(maxn, 0);
        in_e.assign(size_t(maxn) * kMaxEdges, 0);
        out_e.assign(size_t(maxn) * kMaxEdges, 0);
        aln.assign(size_t(maxn) * kMaxAlignments, 0);
        in_cnt.assign(maxn, 0);
        out_cnt.assign(maxn, 0);
        aln_cnt.assign(maxn, 0);
        in_w.assign(size_t(maxn) * kMaxEdges, 0);
        cov.assign(maxn, 0);
        sorted.assign(maxn, 0);
        pos.assign(maxn, 0);
        if (msa)
        {
            ecov.assign(size_t(maxn) * kMaxEdges * maxs, 0);
            ecov_cnt.assign(size_t(maxn) * kMaxEdges, 0);
            seq_begin.assign(maxs, 0);
        }
    }
};

// --- backbone from read 0: cudapoa_kernels.cuh:171-209 -------------------------
static void build_backbone(Graph& g, const uint8_t* seq, const int8_t* w, int len)
{
    g.base[0]    = seq[0];
    g.sorted[0]  = 0;
    g.in_cnt[0]  = 0;
    g.aln_cnt[0] = 0;
    g.pos[0]     = 0;
    if (len >= 1)
        g.out_cnt[len - 1] = 0;
    g.in_w[0] = uint16_t(int(w[0]));
    g.cov[0]  = 1;
    if (g.msa)
        g.seq_begin[0] = 0;
    for (int n = 1; n < len; n++)
    {
        g.base[n]                     = seq[n];
        g.sorted[n]                   = n;
        g.out_e[(n - 1) * kMaxEdges]  = n;
        g.out_cnt[n - 1]              = 1;
        g.in_e[n * kMaxEdges]         = n - 1;
        g.in_w[n * kMaxEdges]         = uint16_t(int(w[n - 1]) + int(w[n]));
        g.in_cnt[n]                   = 1;
        g.aln_cnt[n]                  = 0;
        g.pos[n]                      = n;
        g.cov[n]                      = 1;
        if (g.msa)
        {
            g.ecov[size_t(n - 1) * kMaxEdges * g.max_seqs] = 0;
            g.ecov_cnt[(n - 1) * kMaxEdges]               = 1;
        }
    }
    g.node_count = len;
}

// Row in the score matrix of predecessor slot p of node id, or 0 for a source
// node (cudapoa_nw.cuh:233, :103).
static inline int pred_row(const Graph& g, int node, int p)
{
    return g.pos[g.in_e[node * kMaxEdges + p]] + 1;
}

// --- full-matrix NW on the DAG: cudapoa_nw.cuh:143-466 ---------------------------
// Returns alignment length (reversed arrays) or -1 when the traceback loop bound
// is hit (:454-457).
static int nw_full(const Graph& g, const uint8_t* read, int L, int gap, int mismatch, int match,
                   std::vector<int32_t>& H, std::vector<int32_t>& ag, std::vector<int32_t>& ar)
{
    const int V = g.node_count;
    const size_t W = size_t(L) + 1;
    H.assign(size_t(V + 1) * W, 0);
    // row 0 (:176-179)
    for (int j = 0; j <= L; j++)
        H[j] = j * gap;
    // column 0 (:187-210): max over predecessor column-0 values, plus gap
    for (int r = 0; r < V; r++)
    {
        int node = g.sorted[r];
        int np   = g.in_cnt[node];
        int v;
        if (np == 0)
            v = gap;
        else
        {
            v = std::numeric_limits<int>::min();
            for (int p = 0; p < np; p++)
                v = std::max(v, H[size_t(pred_row(g, node, p)) * W]);
            v += gap;
        }
        H[size_t(r + 1) * W] = v;
    }
    // interior (:222-327): diagonal/vertical over all predecessors, then the
    // horizontal closure left to right
    for (int r = 0; r < V; r++)
    {
        int node   = g.sorted[r];
        int np     = g.in_cnt[node];
        uint8_t b  = g.base[node];
        int32_t* row = &H[size_t(r + 1) * W];
        for (int j = 1; j <= L; j++)
        {
            int sigma = (b == read[j - 1]) ? match : mismatch;
            int best;
            if (np == 0)
            {
                best = std::max(H[j - 1] + sigma, H[j] + gap);
            }
            else
            {
                best = std::numeric_limits<int>::min();
                for (int p = 0; p < np; p++)
                {
                    const int32_t* pr = &H[size_t(pred_row(g, node, p)) * W];
                    best = std::max(best, std::max(pr[j - 1] + sigma, pr[j] + gap));
                }
            }
            row[j] = best;
        }
        for (int j = 1; j <= L; j++)
            row[j] = std::max(row[j], row[j - 1] + gap);
    }

    // end cell: first sink (topological order) with the strictly largest score in
    // the last column (:332-349)
    int i = 0, j = L;
    int best = std::numeric_limits<int>::min();
    for (int idx = 1; idx <= V; idx++)
    {
        if (g.out_cnt[g.sorted[idx - 1]] == 0)
        {
            int s = H[size_t(idx) * W + j];
            if (best < s)
            {
                best = s;
                i    = idx;
            }
        }
    }
    // traceback (:351-457): diagonal (predecessors in slot order), then vertical,
    // then horizontal; a miss keeps the stale previous move (as the reference).
    ag.clear();
    ar.clear();
    int prev_i = 0, prev_j = 0;
    int loop_count = 0;
    const int bound = L + V + 2;
    while (!(i == 0 && j == 0) && loop_count < bound)
    {
        loop_count++;
        int sij    = H[size_t(i) * W + j];
        bool found = false;
        if (i != 0 && j != 0)
        {
            int node  = g.sorted[i - 1];
            int cost  = (g.base[node] == read[j - 1]) ? match : mismatch;
            int np    = g.in_cnt[node];
            int pi    = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H[size_t(pi) * W + j - 1] + cost)
            {
                prev_i = pi;
                prev_j = j - 1;
                found  = true;
            }
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H[size_t(pi) * W + j - 1] + cost)
                {
                    prev_i = pi;
                    prev_j = j - 1;
                    found  = true;
                }
            }
        }
        if (!found && i != 0)
        {
            int node = g.sorted[i - 1];
            int np   = g.in_cnt[node];
            int pi   = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == H[size_t(pi) * W + j] + gap)
            {
                prev_i = pi;
                prev_j = j;
                found  = true;
            }
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == H[size_t(pi) * W + j] + gap)
                {
                    prev_i = pi;
                    prev_j = j;
                    found  = true;
                }
            }
        }
        // horizontal (:437-443); j == 0 never reaches here without a match above
        if (!found && j != 0 && sij == H[size_t(i) * W + j - 1] + gap)
        {
            prev_i = i;
            prev_j = j - 1;
            found  = true;
        }
        ag.push_back(i == prev_i ? -1 : g.sorted[i - 1]);
        ar.push_back(j == prev_j ? -1 : j - 1);
        i = prev_i;
        j = prev_j;
    }
    if (loop_count >= bound)
        return -1;
    return int(ag.size());
}

// --- banded NW on the DAG: cudapoa_nw_banded.cuh:28-487 --------------------------
// Emulates the reference's flat row layout (stride bw+8) bit for bit.
template <typename ScoreT>
struct Banded
{
    int bw;
    int stride;
    float gradient;
    int max_column;
    ScoreT* S; // row-major, rows x stride

    // get_band_start_for_row (:28-48); SizeT arithmetic is exact in int32
    int band_start(int row) const
    {
        int start = int(float(row) * gradient) - bw / 2;
        start     = std::max(start, 0);
        int end   = start + bw;
        if (end > max_column)
            start = max_column - bw + kCellsPerThread;
        start = std::max(start, 0);
        start = start - (start % kCellsPerThread);
        return start;
    }
    // get_score_ptr (:50-69)
    ScoreT* ptr(int row, int col) const
    {
        int bs  = band_start(row);
        int idx = (col == 0) ? 0 : col - bs;
        return &S[int64_t(idx) + int64_t(row) * stride];
    }
    // set_score (:71-87)
    void set(int row, int col, ScoreT v) const
    {
        int bs  = band_start(row);
        int idx = (col == 0) ? bs : col - bs;
        S[int64_t(idx) + int64_t(row) * stride] = v;
    }
    // get_score (:107-121)
    ScoreT get(int row, int col, ScoreT minv) const
    {
        int bs = band_start(row);
        int be = bs + bw;
        if ((col > be || col < bs) && col != 0)
            return minv;
        return *ptr(row, col);
    }
};

template <typename ScoreT>
static int nw_banded(const Graph& g, const uint8_t* read, int L, int bw, int gap, int mismatch, int match,
                     std::vector<ScoreT>& flat, std::vector<int32_t>& ag, std::vector<int32_t>& ar)
{
    const int V              = g.node_count;
    const ScoreT tmin        = std::numeric_limits<ScoreT>::min();
    // :197
    const ScoreT minv = ScoreT(2 * std::abs(std::min(std::min(gap, mismatch), -match) - 1) + int(tmin));
    Banded<ScoreT> B;
    B.bw         = bw;
    B.stride     = bw + kBandPad;
    B.gradient   = float(L + 1) / float(V + 1); // :206
    B.max_column = L + 1;
    // Rows 0..V are used; cells are never read before written except through
    // the layout quirks, whose stale values never reach an output.
    // set_score(row, 0) writes at the row's band start (:71-87), which for
    // late rows lies past the row, up to L + 1 cells past the last row: slack
    // for those writes (never read back)
    const size_t need = size_t(V + 2) * B.stride + size_t(L + 2 * B.stride);
    if (flat.size() < need)
        flat.resize(need, ScoreT(0));
    B.S = flat.data() + B.stride; // one guard row in front
    // horizontal boundary (:212-216)
    for (int j = 0; j < B.stride; j++)
        B.set(0, j, ScoreT(j * gap));
    // vertical boundary (:219-245)
    for (int r = 0; r < V; r++)
    {
        B.set(0, 0, ScoreT(0));
        int node = g.sorted[r];
        int i    = r + 1;
        int np   = g.in_cnt[node];
        if (np == 0)
            B.set(i, 0, ScoreT(gap));
        else
        {
            int pen = int(tmin);
            for (int p = 0; p < np; p++)
                pen = std::max(pen, int(B.get(pred_row(g, node, p), 0, minv)));
            B.set(i, 0, ScoreT(pen + gap));
        }
    }
    // DP rows (:249-344): the 32-lane warp walks the band 4 cells per lane
    const int lanes = 32;
    std::vector<int> s0(lanes), s1(lanes), s2(lanes), s3(lanes);
    for (int r = 0; r < V; r++)
    {
        int node = g.sorted[r];
        int row  = r + 1;
        int bs   = B.band_start(row);
        // initialize_band (:90-105)
        {
            int be   = bs + bw;
            int off  = (bs == 0) ? 1 : bs;
            B.set(row, off, minv);
            for (int j = be; j < be + kBandPad; j++)
                B.set(row, j, minv);
        }
        int carry = int(B.get(row, 0, minv));
        int np    = g.in_cnt[node];
        int p0    = (np == 0) ? 0 : pred_row(g, node, 0);
        uint8_t gb = g.base[node];
        for (int base_pos = bs; base_pos < bs + bw; base_pos += lanes * kCellsPerThread)
        {
            for (int l = 0; l < lanes; l++)
            {
                int rp = base_pos + l * kCellsPerThread;
                int prof[4];
                for (int c = 0; c < 4; c++)
                    prof[c] = (gb == read[rp + c]) ? match : mismatch;
                auto get4 = [&](int prow, int out[4]) {
                    // get_scores (:123-173)
                    int pbs = B.band_start(prow);
                    int pbe = pbs + bw + kCellsPerThread;
                    if ((rp + 1 > pbe || rp + 1 < pbs) && rp + 1 != 0)
                    {
                        for (int c = 0; c < 4; c++)
                            out[c] = int(minv);
                        return;
                    }
                    const ScoreT* q = B.ptr(prow, rp);
                    out[0]          = ScoreT(std::max(int(q[0]) + prof[0], int(q[1]) + gap));
                    out[1]          = ScoreT(std::max(int(q[1]) + prof[1], int(q[2]) + gap));
                    out[2]          = ScoreT(std::max(int(q[2]) + prof[2], int(q[3]) + gap));
                    out[3]          = ScoreT(std::max(int(q[3]) + prof[3], int(q[4]) + gap));
                };
                int sc[4];
                get4(p0, sc);
                for (int p = 1; p < np; p++)
                {
                    int t[4];
                    get4(pred_row(g, node, p), t);
                    for (int c = 0; c < 4; c++)
                        sc[c] = ScoreT(std::max(sc[c], t[c]));
                }
                s0[l] = sc[0];
                s1[l] = sc[1];
                s2[l] = sc[2];
                s3[l] = sc[3];
            }
            // horizontal closure (:292-331): the fix-point converges to the exact
            // left-to-right max-plus closure; values are stored as ScoreT.
            int left = carry;
            for (int l = 0; l < lanes; l++)
            {
                int a = std::max(int(s0[l]), left + gap);
                a     = int(ScoreT(a));
                int b = std::max(int(s1[l]), a + gap);
                b     = int(ScoreT(b));
                int c = std::max(int(s2[l]), b + gap);
                c     = int(ScoreT(c));
                int d = std::max(int(s3[l]), c + gap);
                d     = int(ScoreT(d));
                s0[l] = a;
                s1[l] = b;
                s2[l] = c;
                s3[l] = d;
                left  = d;
            }
            carry = s3[lanes - 1];
            for (int l = 0; l < lanes; l++)
            {
                int rp      = base_pos + l * kCellsPerThread;
                int64_t idx = int64_t(rp + 1 - bs) + int64_t(row) * B.stride;
                B.S[idx]     = ScoreT(s0[l]);
                B.S[idx + 1] = ScoreT(s1[l]);
                B.S[idx + 2] = ScoreT(s2[l]);
                B.S[idx + 3] = ScoreT(s3[l]);
            }
        }
    }
    // end cell (:349-365)
    int i = 0, j = L;
    int best = int(tmin);
    for (int idx = 1; idx <= V; idx++)
    {
        if (g.out_cnt[g.sorted[idx - 1]] == 0)
        {
            int s = int(B.get(idx, j, minv));
            if (best < s)
            {
                best = s;
                i    = idx;
            }
        }
    }
    // traceback (:367-477)
    ag.clear();
    ar.clear();
    int prev_i = 0, prev_j = 0;
    int loop_count = 0;
    const int bound = L + V + 2;
    while (!(i == 0 && j == 0) && loop_count < bound)
    {
        loop_count++;
        int sij    = int(B.get(i, j, minv));
        bool found = false;
        if (i != 0 && j != 0)
        {
            int node = g.sorted[i - 1];
            int cost = (g.base[node] == read[j - 1]) ? match : mismatch;
            int np   = g.in_cnt[node];
            int pi   = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == int(B.get(pi, j - 1, minv)) + cost)
            {
                prev_i = pi;
                prev_j = j - 1;
                found  = true;
            }
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == int(B.get(pi, j - 1, minv)) + cost)
                {
                    prev_i = pi;
                    prev_j = j - 1;
                    found  = true;
                }
            }
        }
        if (!found && i != 0)
        {
            int node = g.sorted[i - 1];
            int np   = g.in_cnt[node];
            int pi   = (np == 0) ? 0 : pred_row(g, node, 0);
            if (sij == int(B.get(pi, j, minv)) + gap)
            {
                prev_i = pi;
                prev_j = j;
                found  = true;
            }
            for (int p = 1; !found && p < np; p++)
            {
                pi = pred_row(g, node, p);
                if (sij == int(B.get(pi, j, minv)) + gap)
                {
                    prev_i = pi;
                    prev_j = j;
                    found  = true;
                }
            }
        }
        if (!found && sij == int(B.get(i, j - 1, minv)) + gap)
        {
            prev_i = i;
            prev_j = j - 1;
            found  = true;
        }
        ag.push_back(i == prev_i ? -1 : g.sorted[i - 1]);
        ar.push_back(j == prev_j ? -1 : j - 1);
        i = prev_i;
        j = prev_j;
    }
    if (loop_count >= bound)
        return -1;
    return int(ag.size());
}

// --- addAlignmentToGraph: cudapoa_add_alignment.cuh:59-279 -----------------------
static uint8_t add_alignment(Graph& g, const std::vector<int32_t>& ag, const std::vector<int32_t>& ar, int alen,
                             const uint8_t* read, const int8_t* w, int s)
{
    int head = -1, curr = -1;
    uint16_t prev_w = 0;
    int node_count  = g.node_count;
    for (int k = alen - 1; k >= 0; k--)
    {
        int rp = ar[k];
        if (rp == -1)
            continue;
        int8_t nw   = w[rp];
        uint8_t rb  = read[rp];
        int gid     = ag[k];
        auto new_node = [&](int id) {
            g.base[id]    = rb;
            g.out_cnt[id] = 0;
            g.in_cnt[id]  = 0;
            g.aln_cnt[id] = 0;
            g.cov[id]     = 0;
        };
        if (gid == -1)
        {
            curr = node_count++;
            if (node_count >= g.max_nodes)
            {
                g.node_count = node_count;
                return kNodeCountExceeded;
            }
            new_node(curr);
        }
        else if (g.base[gid] == rb)
        {
            curr = gid;
        }
        else
        {
            int na  = g.aln_cnt[gid];
            int hit = -1;
            for (int n = 0; n < na; n++)
            {
                int aid = g.aln[gid * kMaxAlignments + n];
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
                curr = node_count++;
                if (node_count >= g.max_nodes)
                {
                    g.node_count = node_count;
                    return kNodeCountExceeded;
                }
                new_node(curr);
                int cnt = 0;
                // ring update order (:182-198)
                for (int n = 0; n < na; n++)
                {
                    int aid                                      = g.aln[gid * kMaxAlignments + n];
                    int ac                                       = g.aln_cnt[aid];
                    g.aln[aid * kMaxAlignments + ac]             = curr;
                    g.aln_cnt[aid]                               = uint16_t(ac + 1);
                    g.aln[curr * kMaxAlignments + cnt]           = aid;
                    cnt++;
                }
                g.aln[gid * kMaxAlignments + na] = curr;
                g.aln_cnt[gid]                   = uint16_t(na + 1);
                g.aln[curr * kMaxAlignments + cnt] = gid;
                cnt++;
                g.aln_cnt[curr] = uint16_t(cnt);
            }
        }
        if (g.msa && rp == 0)
            g.seq_begin[s] = curr;
        if (head != -1)
        {
            bool exists = false;
            int ic      = g.in_cnt[curr];
            for (int e = 0; e < ic; e++)
            {
                if (g.in_e[curr * kMaxEdges + e] == head)
                {
                    exists = true;
                    g.in_w[curr * kMaxEdges + e] = uint16_t(g.in_w[curr * kMaxEdges + e] + (int(prev_w) + int(nw)));
                }
            }
            if (!exists)
            {
                g.in_e[curr * kMaxEdges + ic] = head;
                g.in_w[curr * kMaxEdges + ic] = uint16_t(int(prev_w) + int(nw));
                g.in_cnt[curr]                = uint16_t(ic + 1);
                int oc                        = g.out_cnt[head];
                g.out_e[head * kMaxEdges + oc] = curr;
                if (g.msa)
                {
                    g.ecov_cnt[head * kMaxEdges + oc]                          = 1;
                    g.ecov[size_t(head * kMaxEdges + oc) * g.max_seqs]        = uint16_t(s);
                }
                g.out_cnt[head] = uint16_t(oc + 1);
                if (oc + 1 >= kMaxEdges || ic + 1 >= kMaxEdges)
                {
                    g.node_count = node_count;
                    return kEdgeCountExceeded;
                }
            }
            else if (g.msa)
            {
                int oc = g.out_cnt[head];
                for (int e = 0; e < oc; e++)
                {
                    if (g.out_e[head * kMaxEdges + e] == curr)
                    {
                        int c = g.ecov_cnt[head * kMaxEdges + e];
                        g.ecov[size_t(head * kMaxEdges + e) * g.max_seqs + c] = uint16_t(s);
                        g.ecov_cnt[head * kMaxEdges + e]                       = uint16_t(c + 1);
                        break;
                    }
                }
            }
        }
        head = curr;
        g.cov[head]++;
        prev_w = uint16_t(int(nw));
    }
    g.node_count = node_count;
    return kSuccess;
}

// --- Kahn topological sort (default build): cudapoa_topsort.cuh:38-88 -----------
static void topsort_fast(Graph& g, std::vector<uint16_t>& local)
{
    const int n = g.node_count;
    local.resize(std::max(n, 1));
    int k = 0;
    for (int v = 0; v < n; v++)
    {
        local[v] = g.in_cnt[v];
        if (local[v] == 0)
        {
            g.pos[v]      = k;
            g.sorted[k++] = v;
        }
    }
    for (int q = 0; q < k; q++)
    {
        int v = g.sorted[q];
        for (int e = 0; e < g.out_cnt[v]; e++)
        {
            int o = g.out_e[v * kMaxEdges + e];
            local[o]--;
            if (local[o] == 0)
            {
                g.pos[o]      = k;
                g.sorted[k++] = o;
            }
        }
    }
}

// --- racon/SPOA DFS topological sort: cudapoa_topsort.cuh:94-189 -----------------
// The DFS stack holds at most 4 x max_nodes entries (the kernels' bound; the
// reference's nodes_to_visit has no bound check): beyond it the window fails
// with generic_error.
static bool topsort_racon(Graph& g)
{
    const int n = g.node_count;
    std::vector<uint8_t> mark(g.max_nodes, 0);
    std::vector<uint8_t> check(g.max_nodes, 1);
    const int cap = 4 * g.max_nodes;
    std::vector<int32_t> stack(cap, 0);
    int top = -1, k = 0;
    for (int v = 0; v < n; v++)
    {
        if (mark[v] != 0)
            continue;
        stack[++top] = v;
        while (top != -1)
        {
            int id     = stack[top];
            bool valid = true;
            if (mark[id] != 2)
            {
                for (int e = 0; e < g.in_cnt[id]; e++)
                {
                    int b = g.in_e[id * kMaxEdges + e];
                    if (mark[b] != 2)
                    {
                        if (top + 1 >= cap)
                            return false;
                        stack[++top] = b;
                        valid        = false;
                    }
                }
                if (check[id])
                {
                    for (int a = 0; a < g.aln_cnt[id]; a++)
                    {
                        int aid = g.aln[id * kMaxAlignments + a];
                        if (mark[aid] != 2)
                        {
                            if (top + 1 >= cap)
                                return false;
                            stack[++top] = aid;
                            check[aid]   = 0;
                            valid        = false;
                        }
                    }
                }
                if (valid)
                {
                    mark[id] = 2;
                    if (check[id])
                    {
                        g.sorted[k] = id;
                        g.pos[id]   = k;
                        k++;
                        for (int a = 0; a < g.aln_cnt[id]; a++)
                        {
                            int aid     = g.aln[id * kMaxAlignments + a];
                            g.sorted[k] = aid;
                            g.pos[aid]  = k;
                            k++;
                        }
                    }
                }
                else
                    mark[id] = 1;
            }
            if (valid)
                top--;
        }
    }
    return true;
}

// --- heaviest bundle: cudapoa_generate_consensus.cuh:28-276 ----------------------
static int branch_completion(const Graph& g, int max_pos, std::vector<int32_t>& score, std::vector<int32_t>& pred)
{
    const int n = g.node_count;
    int node    = g.sorted[max_pos];
    for (int oe = 0; oe < g.out_cnt[node]; oe++)
    {
        int o = g.out_e[node * kMaxEdges + oe];
        for (int ie = 0; ie < g.in_cnt[o]; ie++)
        {
            int id = g.in_e[o * kMaxEdges + ie];
            if (id != node)
                score[id] = -1;
        }
    }
    int max_score = 0, max_id = 0;
    for (int r = max_pos + 1; r < n; r++)
    {
        node       = g.sorted[r];
        pred[node] = -1;
        int sc     = -1;
        for (int e = 0; e < g.in_cnt[node]; e++)
        {
            int b = g.in_e[node * kMaxEdges + e];
            if (score[b] == -1)
                continue;
            int w = g.in_w[node * kMaxEdges + e];
            if (sc < w || (sc == w && score[pred[node]] <= score[b]))
            {
                sc         = w;
                pred[node] = b;
            }
        }
        if (pred[node] != -1)
            sc += score[pred[node]];
        if (max_score <= sc)
        {
            max_score = sc;
            max_id    = node;
        }
        score[node] = sc;
    }
    return max_id;
}

// Writes the consensus backwards with a '\0' terminator, exactly as the kernel
// does; returns a status code (0 = success).
static uint8_t consensus_raw(const Graph& g, uint8_t* cons, uint16_t* covg, int max_cons)
{
    const int n = g.node_count;
    std::vector<int32_t> score(std::max(n, 1), -1), pred(std::max(n, 1), -1);
    int max_id = 0, max_score = -1;
    for (int r = 0; r < n; r++)
    {
        int node = g.sorted[r];
        int sc   = score[node];
        for (int e = 0; e < g.in_cnt[node]; e++)
        {
            int w = g.in_w[node * kMaxEdges + e];
            int b = g.in_e[node * kMaxEdges + e];
            if (sc < w || (sc == w && score[pred[node]] <= score[b]))
            {
                sc         = w;
                pred[node] = b;
            }
        }
        if (pred[node] != -1)
            sc += score[pred[node]];
        if (max_score <= sc)
        {
            max_id    = node;
            max_score = sc;
        }
        score[node] = sc;
    }
    int loops = 0;
    if (g.out_cnt[max_id] != 0)
    {
        while (g.out_cnt[max_id] != 0 && loops < n)
        {
            max_id = branch_completion(g, g.pos[max_id], score, pred);
            loops++;
        }
    }
    if (loops >= n) // generate_consensus.cuh:222-228 (also fires for an empty graph)
        return kLoopCountExceeded;
    int cpos = 0, count = 0;
    auto node_cov = [&](int id) {
        uint16_t c = g.cov[id];
        for (int a = 0; a < g.aln_cnt[id]; a++)
            c = uint16_t(c + g.cov[g.aln[id * kMaxAlignments + a]]);
        return c;
    };
    while (pred[max_id] != -1)
    {
        cons[cpos] = g.base[max_id];
        covg[cpos] = node_cov(max_id);
        max_id     = pred[max_id];
        cpos       = std::min(cpos + 1, max_cons - 1);
        count++;
    }
    cons[cpos] = g.base[max_id];
    covg[cpos] = node_cov(max_id);
    if (count >= max_cons - 1)
        return kExceededMaxSeqSize;
    cons[cpos + 1] = 0;
    return kSuccess;
}

// --- MSA: cudapoa_generate_msa.cuh:27-118, kernel :121-224 -----------------------
static uint8_t generate_msa(Graph& g, int nseq, int max_cons, uint8_t* msa_out /* nseq x max_cons */)
{
    if (!topsort_racon(g))
        return kGenericError;
    const int n = g.node_count;
    std::vector<int32_t> mpos(g.max_nodes, 0);
    int msa_len = 0;
    for (int r = 0; r < n; r++)
    {
        int id   = g.sorted[r];
        mpos[id] = msa_len;
        int ac   = g.aln_cnt[id];
        for (int a = 0; a < ac; a++)
            mpos[g.sorted[++r]] = msa_len;
        msa_len++;
    }
    if (msa_len >= max_cons)
        return kExceededMaxSeqSize;
    for (int s = 0; s < nseq; s++)
    {
        uint8_t* row = msa_out + size_t(s) * max_cons;
        int node     = g.seq_begin[s];
        int filled   = 0;
        while (true)
        {
            int mp   = mpos[node];
            row[mp]  = g.base[node];
            for (int i = filled; i < mp; i++)
                row[i] = '-';
            filled   = mp + 1;
            bool end = true;
            for (int e = 0; e < g.out_cnt[node] && end; e++)
            {
                int to = g.out_e[node * kMaxEdges + e];
                int cc = g.ecov_cnt[node * kMaxEdges + e];
                for (int m = 0; m < cc; m++)
                {
                    if (g.ecov[size_t(node * kMaxEdges + e) * g.max_seqs + m] == s)
                    {
                        end  = false;
                        node = to;
                        break;
                    }
                }
            }
            if (end)
            {
                for (int i = filled; i < msa_len; i++)
                    row[i] = '-';
                break;
            }
        }
        row[msa_len] = 0;
    }
    return kSuccess;
}

struct WindowParams
{
    int gap, mismatch, match;
    int banded, band_width;
    int score_bits; // 16 or 32, only observable in banded mode
    int msa;
    int max_nodes, max_consensus, max_seqs;
    int spoa_accurate = 0; // per-read racon DFS sort (SPOA_ACCURATE builds)
};

struct WindowStats
{
    int64_t cells;       // sum over reads s>=1 of (|V_{s-1}|+1)*(|r_s|+1)
    int64_t band_cells;  // banded equivalent (|V|+1)*(bw+8)
    int32_t final_nodes;
};

// Window driver: cudapoa_kernels.cuh:171-358 followed by the consensus kernel
// (cudapoa_generate_consensus.cuh:279-347) or the MSA kernel (msa.cuh:121-224).
// Writes output in host form: consensus already reversed (cudapoa_batch.cuh:241).
static uint8_t run_window(const WindowParams& P, const uint8_t* seqs, const int32_t* lens, const int8_t* wts, int nseq,
                          uint8_t* cons, uint16_t* covg, int32_t* cons_len, uint8_t* msa_out, Graph& g, WindowStats* st)
{
    g.init(P.max_nodes, std::max(P.max_seqs, nseq), P.msa != 0);
    std::vector<int32_t> H, ag, ar;
    std::vector<int16_t> f16;
    std::vector<int32_t> f32;
    std::vector<uint16_t> local;
    if (st)
    {
        st->cells      = 0;
        st->band_cells = 0;
    }
    if (nseq <= 0) // not reachable with defined behaviour in the reference; empty result
        return kSuccess;
    if (lens[0] > P.max_nodes) // the host API rejects this earlier (max_seq <= max_nodes)
        return kSeqLenExceededNodes;
    const uint8_t* seq = seqs;
    const int8_t* w    = wts;
    build_backbone(g, seq, w, lens[0]);
    for (int s = 1; s < nseq; s++)
    {
        seq += lens[s - 1];
        w += lens[s - 1];
        int L = lens[s];
        if (g.node_count >= P.max_nodes)
            return kNodeCountExceeded;
        if (st)
        {
            st->cells += int64_t(g.node_count + 1) * (L + 1);
            st->band_cells += int64_t(g.node_count + 1) * (P.band_width + kBandPad);
        }
        int alen;
        if (P.banded)
        {
            if (P.score_bits == 16)
                alen = nw_banded<int16_t>(g, seq, L, P.band_width, P.gap, P.mismatch, P.match, f16, ag, ar);
            else
                alen = nw_banded<int32_t>(g, seq, L, P.band_width, P.gap, P.mismatch, P.match, f32, ag, ar);
        }
        else
            alen = nw_full(g, seq, L, P.gap, P.mismatch, P.match, H, ag, ar);
        if (alen == -1)
            return kLoopCountExceeded;
        uint8_t err = add_alignment(g, ag, ar, alen, seq, w, s);
        if (err != kSuccess)
            return err;
        if (P.spoa_accurate) // cudapoa_kernels.cuh:324-337 (SPOA_ACCURATE builds)
        {
            if (!topsort_racon(g))
                return kGenericError;
        }
        else
            topsort_fast(g, local);
    }
    if (st)
        st->final_nodes = g.node_count;
    if (P.msa)
        return generate_msa(g, nseq, P.max_consensus, msa_out);
    std::vector<uint8_t> raw(P.max_consensus + 1, 0);
    std::vector<uint16_t> rawc(P.max_consensus + 1, 0);
    uint8_t err = consensus_raw(g, raw.data(), rawc.data(), P.max_consensus);
    if (err != kSuccess)
        return err;
    int n = int(strnlen(reinterpret_cast<const char*>(raw.data()), P.max_consensus));
    for (int k = 0; k < n; k++)
    {
        cons[k] = raw[n - 1 - k];
        covg[k] = rawc[n - 1 - k];
    }
    *cons_len = n;
    return kSuccess;
}

} // namespace oracle

using namespace oracle;

// SPOA_ACCURATE for the calls below (the reference's build option, here a switch)
static int g_spoa_accurate = 0;

extern "C" {

void oracle_set_spoa_accurate(int32_t on) { g_spoa_accurate = on != 0; }

// One POA window.  Outputs: consensus (host order, length in *cons_len) and
// coverage, or MSA rows (nseq x max_consensus, NUL terminated), plus the final
// graph (node bases, incoming edges/weights in slot order) for get_graphs parity.
// Returns the window's StatusType.
int oracle_poa_window(const uint8_t* seqs, const int32_t* lens, const int8_t* wts, int32_t nseq,
                      int32_t gap, int32_t mismatch, int32_t match, int32_t banded, int32_t band_width,
                      int32_t score_bits, int32_t msa, int32_t max_nodes, int32_t max_consensus, int32_t max_seqs,
                      uint8_t* cons, uint16_t* covg, int32_t* cons_len, uint8_t* msa_out,
                      int64_t* cells, int32_t* final_nodes,
                      uint8_t* g_bases, int32_t* g_in_cnt, int32_t* g_in_e, int32_t* g_in_w)
{
    WindowParams P{gap, mismatch, match, banded, band_width, score_bits, msa, max_nodes, max_consensus, max_seqs,
                   g_spoa_accurate};
    Graph g;
    WindowStats st{0, 0, 0};
    *cons_len   = 0;
    uint8_t rc  = run_window(P, seqs, lens, wts, nseq, cons, covg, cons_len, msa_out, g, &st);
    if (cells)
        cells[0] = st.cells, cells[1] = st.band_cells;
    if (final_nodes)
        *final_nodes = g.node_count;
    if (g_bases)
    {
        for (int v = 0; v < g.node_count && v < max_nodes; v++)
        {
            g_bases[v]  = g.base[v];
            g_in_cnt[v] = g.in_cnt[v];
            for (int e = 0; e < g.in_cnt[v] && e < kMaxEdges; e++)
            {
                g_in_e[v * kMaxEdges + e] = g.in_e[v * kMaxEdges + e];
                g_in_w[v * kMaxEdges + e] = g.in_w[v * kMaxEdges + e];
            }
        }
    }
    return rc;
}

// Batch of windows, one window per OpenMP thread (CPU baseline).  Windows are
// described by (first sequence index, sequence count); outputs are strided by
// max_consensus.  Returns the number of threads used.
int oracle_poa_batch(const uint8_t* seqs, const int64_t* seq_offsets, const int32_t* lens, const int32_t* win_first,
                     const int32_t* win_nseq, int32_t nwin, int32_t gap, int32_t mismatch, int32_t match, int32_t banded,
                     int32_t band_width, int32_t score_bits, int32_t max_nodes, int32_t max_consensus, int32_t max_seqs,
                     int32_t nthreads, uint8_t* cons, uint16_t* covg, int32_t* cons_len, uint8_t* status, int64_t* cells,
                     int32_t msa, uint8_t* msa_out)
{
    // msa != 0: MSA output (generateMSAKernel) into msa_out, window wi at
    // wi * max_seqs * max_consensus (rows NUL terminated)
    WindowParams P{gap, mismatch, match, banded, band_width, score_bits, msa, max_nodes, max_consensus, max_seqs,
                   g_spoa_accurate};
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
    for (int wi = 0; wi < nwin; wi++)
    {
        Graph g;
        WindowStats st{0, 0, 0};
        int first  = win_first[wi];
        int n      = win_nseq[wi];
        std::vector<int8_t> wts(0);
        int64_t total = 0;
        for (int s = 0; s < n; s++)
            total += lens[first + s];
        wts.assign(size_t(total) + 1, 1);
        cons_len[wi] = 0;
        status[wi]   = run_window(P, seqs + seq_offsets[first], lens + first, wts.data(), n,
                                cons + size_t(wi) * max_consensus, covg + size_t(wi) * max_consensus, &cons_len[wi],
                                msa ? msa_out + size_t(wi) * max_seqs * max_consensus : nullptr, g, &st);
        if (cells)
            cells[wi] = st.cells;
    }
    return used;
}

// Final graph of one window with its aligned-node lists (tests of the racon
// sort on real window graphs): node count, in-edges (kMaxEdges slots) and
// aligned nodes (kMaxAlignments slots) in slot order.  Returns the status.
int oracle_poa_window_graph(const uint8_t* seqs, const int32_t* lens, const int8_t* wts, int32_t nseq, int32_t gap,
                            int32_t mismatch, int32_t match, int32_t banded, int32_t band_width, int32_t score_bits,
                            int32_t max_nodes, int32_t max_consensus, int32_t* final_nodes, uint16_t* in_cnt,
                            int32_t* in_e, uint16_t* aln_cnt, int32_t* aln)
{
    WindowParams P{gap, mismatch, match, banded, band_width, score_bits, 0, max_nodes, max_consensus, nseq,
                   g_spoa_accurate};
    Graph g;
    WindowStats st{0, 0, 0};
    int32_t clen = 0;
    std::vector<uint8_t> cons(size_t(max_consensus) + 1);
    std::vector<uint16_t> covg(size_t(max_consensus) + 1);
    uint8_t rc   = run_window(P, seqs, lens, wts, nseq, cons.data(), covg.data(), &clen, nullptr, g, &st);
    *final_nodes = g.node_count;
    for (int v = 0; v < g.node_count && v < max_nodes; v++)
    {
        in_cnt[v]  = g.in_cnt[v];
        aln_cnt[v] = g.aln_cnt[v];
        for (int e = 0; e < kMaxEdges; e++)
            in_e[v * kMaxEdges + e] = e < g.in_cnt[v] ? g.in_e[v * kMaxEdges + e] : 0;
        for (int a = 0; a < kMaxAlignments; a++)
            aln[v * kMaxAlignments + a] = a < g.aln_cnt[v] ? g.aln[v * kMaxAlignments + a] : 0;
    }
    return rc;
}

// topsort_racon (cudapoa_topsort.cuh:94-189) of a given graph; the MSA column
// of every node (getNodeIDToMSAPosDevice, cudapoa_generate_msa.cuh:27-45) and
// the column count.  Returns 1, or 0 when the DFS stack outgrows 4 x nodes.
int oracle_topsort_racon(int32_t node_count, const uint16_t* in_cnt, const int32_t* in_e, const uint16_t* aln_cnt,
                         const int32_t* aln, int32_t* sorted_out, int32_t* mpos_out, int32_t* ncols)
{
    Graph g;
    g.init(std::max(node_count, 1), 1, false);
    g.node_count = node_count;
    for (int v = 0; v < node_count; v++)
    {
        g.in_cnt[v]  = in_cnt[v];
        g.aln_cnt[v] = aln_cnt[v];
        for (int e = 0; e < in_cnt[v]; e++)
            g.in_e[v * kMaxEdges + e] = in_e[v * kMaxEdges + e];
        for (int a = 0; a < aln_cnt[v]; a++)
            g.aln[v * kMaxAlignments + a] = aln[v * kMaxAlignments + a];
    }
    if (!topsort_racon(g))
        return 0;
    int col = 0;
    for (int r = 0; r < node_count; r++)
    {
        const int id  = g.sorted[r];
        sorted_out[r] = id;
        mpos_out[id]  = col;
        for (int a = 0; a < g.aln_cnt[id]; a++)
        {
            ++r;
            sorted_out[r]          = g.sorted[r];
            mpos_out[g.sorted[r]] = col;
        }
        col++;
    }
    *ncols = col;
    return 1;
}

// ---- single-kernel known-answer hooks (reference test kernels) ----------------
// Graph inputs use the fixed-slot layout of the reference tests (50 slots).

// runTopSort, cudapoa_topsort.cuh:192-229 (Test_CudapoaTopSort.cu)
void oracle_topsort(int32_t node_count, const uint16_t* in_cnt, const int32_t* out_e, const uint16_t* out_cnt,
                    int32_t* sorted_out)
{
    Graph g;
    g.init(std::max(node_count, 1), 1, false);
    g.node_count = node_count;
    for (int v = 0; v < node_count; v++)
    {
        g.in_cnt[v]  = in_cnt[v];
        g.out_cnt[v] = out_cnt[v];
        for (int e = 0; e < out_cnt[v]; e++)
            g.out_e[v * kMaxEdges + e] = out_e[v * kMaxEdges + e];
    }
    std::vector<uint16_t> local;
    topsort_fast(g, local);
    for (int k = 0; k < node_count; k++)
        sorted_out[k] = g.sorted[k];
}

// runNW, cudapoa_nw.cuh:468-547 (Test_CudapoaNW.cu)
int oracle_nw(int32_t node_count, const uint8_t* bases, const int32_t* sorted, const int32_t* pos,
              const uint16_t* in_cnt, const int32_t* in_e, const uint16_t* out_cnt, const uint8_t* read, int32_t L,
              int32_t gap, int32_t mismatch, int32_t match, int32_t* ag_out, int32_t* ar_out)
{
    Graph g;
    g.init(std::max(node_count, 1), 1, false);
    g.node_count = node_count;
    for (int v = 0; v < node_count; v++)
    {
        g.base[v]    = bases[v];
        g.sorted[v]  = sorted[v];
        g.pos[v]     = pos[v];
        g.in_cnt[v]  = in_cnt[v];
        g.out_cnt[v] = out_cnt[v];
        for (int e = 0; e < in_cnt[v]; e++)
            g.in_e[v * kMaxEdges + e] = in_e[v * kMaxEdges + e];
    }
    std::vector<int32_t> H, ag, ar;
    int n = nw_full(g, read, L, gap, mismatch, match, H, ag, ar);
    for (int k = 0; k < n; k++)
        ag_out[k] = ag[k], ar_out[k] = ar[k];
    return n;
}

// addAlignmentKernel, cudapoa_add_alignment.cuh:281-369 (Test_CudapoaAddAlignment.cu)
// Graph arrays are updated in place; returns status, node count in *node_count.
int oracle_add_alignment(int32_t max_nodes, int32_t* node_count, uint8_t* bases, uint16_t* in_cnt, int32_t* in_e,
                         uint16_t* in_w, uint16_t* out_cnt, int32_t* out_e, uint16_t* aln_cnt, int32_t* aln,
                         uint16_t* cov, const int32_t* ag, const int32_t* ar, int32_t alen, const uint8_t* read,
                         const int8_t* w)
{
    Graph g;
    g.init(max_nodes, 1, false);
    g.node_count = *node_count;
    std::copy(bases, bases + max_nodes, g.base.begin());
    std::copy(in_cnt, in_cnt + max_nodes, g.in_cnt.begin());
    std::copy(out_cnt, out_cnt + max_nodes, g.out_cnt.begin());
    std::copy(aln_cnt, aln_cnt + max_nodes, g.aln_cnt.begin());
    std::copy(cov, cov + max_nodes, g.cov.begin());
    std::copy(in_e, in_e + size_t(max_nodes) * kMaxEdges, g.in_e.begin());
    std::copy(in_w, in_w + size_t(max_nodes) * kMaxEdges, g.in_w.begin());
    std::copy(out_e, out_e + size_t(max_nodes) * kMaxEdges, g.out_e.begin());
    std::copy(aln, aln + size_t(max_nodes) * kMaxAlignments, g.aln.begin());
    std::vector<int32_t> vag(ag, ag + alen), var(ar, ar + alen);
    uint8_t rc = add_alignment(g, vag, var, alen, read, w, 1);
    *node_count = g.node_count;
    std::copy(g.base.begin(), g.base.end(), bases);
    std::copy(g.in_cnt.begin(), g.in_cnt.end(), in_cnt);
    std::copy(g.out_cnt.begin(), g.out_cnt.end(), out_cnt);
    std::copy(g.aln_cnt.begin(), g.aln_cnt.end(), aln_cnt);
    std::copy(g.cov.begin(), g.cov.end(), cov);
    std::copy(g.in_e.begin(), g.in_e.end(), in_e);
    std::copy(g.in_w.begin(), g.in_w.end(), in_w);
    std::copy(g.out_e.begin(), g.out_e.end(), out_e);
    std::copy(g.aln.begin(), g.aln.end(), aln);
    return rc;
}

// generateConsensusTestKernel, cudapoa_generate_consensus.cuh:349-424
// (Test_CudapoaGenerateConsensus.cu).  Output is the raw kernel string (reversed).
int oracle_consensus_raw(int32_t node_count, const uint8_t* bases, const int32_t* sorted, const int32_t* pos,
                         const uint16_t* in_cnt, const int32_t* in_e, const uint16_t* in_w, const uint16_t* out_cnt,
                         const int32_t* out_e, const uint16_t* aln_cnt, const int32_t* aln, const uint16_t* cov,
                         int32_t max_cons, uint8_t* cons_out, uint16_t* cov_out)
{
    Graph g;
    g.init(std::max(node_count, 1), 1, false);
    g.node_count = node_count;
    for (int v = 0; v < node_count; v++)
    {
        g.base[v]    = bases[v];
        g.sorted[v]  = sorted[v];
        g.pos[v]     = pos[v];
        g.in_cnt[v]  = in_cnt[v];
        g.out_cnt[v] = out_cnt[v];
        g.aln_cnt[v] = aln_cnt[v];
        g.cov[v]     = cov[v];
        for (int e = 0; e < kMaxEdges; e++)
        {
            g.in_e[v * kMaxEdges + e]  = in_e[v * kMaxEdges + e];
            g.in_w[v * kMaxEdges + e]  = in_w[v * kMaxEdges + e];
            g.out_e[v * kMaxEdges + e] = out_e[v * kMaxEdges + e];
        }
        for (int a = 0; a < kMaxAlignments; a++)
            g.aln[v * kMaxAlignments + a] = aln[v * kMaxAlignments + a];
    }
    return consensus_raw(g, cons_out, cov_out, max_cons);
}

} // extern "C"

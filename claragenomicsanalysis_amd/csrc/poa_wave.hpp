// Wave-level building blocks shared by the POA kernels (poa_kernels.hip: the
// global-memory and LDS-resident full-alignment kernels; poa_band.hip: the
// banded kernel): phase timers, the consensus / MSA epilogue, DPP scans, the
// wave-parallel addAlignmentToGraph and the LDS Kahn topological sort.
#pragma once

#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "poa_device.hpp"

#define GWAMD_LDS __attribute__((address_space(3)))
#define GWAMD_GLB __attribute__((address_space(1)))

namespace gwamd
{
namespace poa
{

// LDS pointer from a flat pointer into the LDS image (its low 32 bits), with
// no null check (an addrspacecast adds one; the backend miscompiled that
// pattern in the forward pass).  Functions the compiler keeps out of line get
// their pointers as flat ones; typed pointers keep their LDS and HBM accesses
// off the flat path, where an access counts against both wait counters and
// every LDS wait also waits for outstanding HBM stores.
template <typename T>
__device__ __forceinline__ GWAMD_LDS T* lds_of(T* p)
{
    return (GWAMD_LDS T*)(uintptr_t)(uint32_t)(uintptr_t)(p);
}
template <typename T>
__device__ __forceinline__ GWAMD_GLB T* glb_of(T* p)
{
    return (GWAMD_GLB T*)(p);
}
// builtin vectors (HIP's uint4 is a class whose copy does not take a
// qualified address space)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Per-window phase timers (s_memrealtime, 100 MHz) kept in registers.
struct PhaseTimer
{
    uint64_t t0, mark;
    uint64_t v[kPhases - 1];
    __device__ PhaseTimer() : t0(now_ticks()), mark(t0)
    {
#pragma unroll
        for (int i = 0; i < kPhases - 1; i++)
            v[i] = 0;
    }
    template <int P>
    __device__ void lap()
    {
        const uint64_t t = now_ticks();
        v[P] += t - mark;
        mark = t;
    }
    __device__ void store(int64_t* out) const
    {
#pragma unroll
        for (int i = 0; i < kPhases - 1; i++)
            out[i] = int64_t(v[i]);
        out[kPhTotal] = int64_t(now_ticks() - t0);
    }
};

template <typename SizeT>
__device__ __forceinline__ bool topsort_racon_lds(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* scratch,
                                                  int scratch_bytes, int lane, SizeT* mpos = nullptr,
                                                  int* ncols = nullptr, int32_t* heads = nullptr);

// Consensus and/or MSA of one finished window (cudapoa_generate_consensus.cuh:
// 279-347, cudapoa_generate_msa.cuh:121-224).  scratch: free LDS of the
// workgroup for the MSA's racon sort (nullptr: the lane-0 sort in HBM).
template <typename SizeT, bool MSA>
__device__ __forceinline__ void finish_window(const Buffers& b, const Dims& d, int w, int lane, WinGraph<SizeT> g, int status,
                              int nseq, int node_count, int32_t* cscore, SizeT* cpred, uint16_t* ecov,
                              uint16_t* ecovc, SizeT* seq_begin, int& sh_len, int& sh_status,
                              GWAMD_LDS uint8_t* scratch = nullptr, int scratch_bytes = 0,
                              uint64_t* oprof = nullptr)
{
    g = as_global(g);
#ifdef GWAMD_OUTPUT_PROFILE
    uint64_t ot = now_ticks();
    auto olap = [&](int k) { const uint64_t t = now_ticks(); if (oprof) oprof[k] += t - ot; ot = t; };
#else
    auto olap = [&](int) {};
#endif
    uint8_t* cons_out = b.cons + size_t(w) * d.max_consensus;
    const int graph_status = status;
    if (!MSA || d.want_consensus)
    {
        uint16_t* cov_out = b.cov + size_t(w) * d.max_consensus;
        if (lane == 0)
        {
            int len = 0;
            int cst = graph_status;
            if (cst == kSuccess && nseq > 0)
            {
                int r = consensus_raw<SizeT>(g, node_count, cscore, cpred, cons_out, cov_out, d.max_consensus);
                if (r < 0)
                    cst = -r;
                else
                    len = r;
            }
            sh_len    = len;
            sh_status = cst;
        }
        wave_sync();
        const int len = sh_len;
        // reverse in place to host order (cudapoa_batch.cuh:241-246 does this on the host)
        for (int k = lane; k < len / 2; k += kWave)
        {
            uint8_t c0  = cons_out[k];
            uint8_t c1  = cons_out[len - 1 - k];
            uint16_t v0 = cov_out[k];
            uint16_t v1 = cov_out[len - 1 - k];
            cons_out[k] = c1, cons_out[len - 1 - k] = c0;
            cov_out[k] = v1, cov_out[len - 1 - k] = v0;
        }
        if (lane == 0)
        {
            b.cons_len[w] = len;
            b.status[w]   = uint8_t(sh_status);
            if (len < d.max_consensus)
                cons_out[len] = 0;
        }
        wave_sync();
    }
    if (MSA)
    {
        uint8_t* msa_out = b.msa + size_t(w) * d.max_seqs * d.max_consensus;
        // the racon sort and the node -> column map by the wave in LDS when the
        // graph fits; the racon stack region (cpred) holds node -> column
        int lds_cols        = 0;
        olap(0);
        const bool lds_done = graph_status == kSuccess && nseq > 0 &&
                              topsort_racon_lds<SizeT>(g, node_count, scratch, scratch_bytes, lane, cpred, &lds_cols,
                                                       (d.diag & 8) ? nullptr : cscore);
        olap(1);
        if (lane == 0)
        {
            int msa_len = 0;
            int mst     = graph_status;
            if (mst == kSuccess && nseq > 0 && lds_done)
            {
                msa_len = lds_cols;
                if (msa_len >= d.max_consensus)
                    mst = kExceededMaxSeqSize;
            }
            else if (mst == kSuccess && nseq > 0)
            {
                if (!topsort_racon<SizeT>(g, node_count, cscore, cpred, 4 * d.max_nodes))
                    mst = kGenericError;
                else
                {
                    // getNodeIDToMSAPosDevice (cudapoa_generate_msa.cuh:27-45); the racon stack
                    // region is free again and holds node -> column
                    SizeT* mpos = cpred;
                    for (int r = 0; r < node_count; r++)
                    {
                        const int id = int(g.sorted[r]);
                        mpos[id]     = SizeT(msa_len);
                        const int ac = int(g.aln_cnt[id]);
                        for (int a = 0; a < ac; a++)
                            mpos[int(g.sorted[++r])] = SizeT(msa_len);
                        msa_len++;
                    }
                    if (msa_len >= d.max_consensus)
                        mst = kExceededMaxSeqSize;
                }
            }
            sh_len    = msa_len;
            sh_status = mst;
        }
        wave_sync();
        const int msa_len = sh_len;
        const int mst     = sh_status;
        if (mst == kSuccess && nseq > 0)
        {
            const SizeT* mpos = cpred;
            // generateMSADevice (cudapoa_generate_msa.cuh:47-118).  Read s walks
            // from seq_begin[s] along the out-edge whose read list holds s; a
            // read's path is simple (its positions land on distinct nodes joined
            // by its own edges), so the walk visits exactly seq_begin[s] and the
            // ends of the edges listing s.  The rows are filled in parallel:
            // gaps everywhere, then the base of every visited node in its column.
            for (int t = lane; t < nseq * (msa_len + 1); t += kWave)
            {
                const int sr = t / (msa_len + 1), col = t - sr * (msa_len + 1);
                msa_out[size_t(sr) * d.max_consensus + col] = col == msa_len ? 0 : '-';
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            wave_sync();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            for (int v = lane; v < node_count; v += kWave)
            {
                const int oc = int(g.out_cnt[v]);
                if (oc == 0)
                    continue;
                const int mv     = int(mpos[v]);
                const uint8_t bv = g.base[v];
                for (int e = 0; e < oc; e++)
                {
                    const int to     = int(g.out_e[v * kMaxEdges + e]);
                    const int mt     = int(mpos[to]);
                    const uint8_t bt = g.base[to];
                    const int cc     = int(ecovc[v * kMaxEdges + e]);
                    for (int m = 0; m < cc; m++)
                    {
                        const int sr = int(ecov[size_t(v * kMaxEdges + e) * d.max_seqs + m]);
                        uint8_t* row = msa_out + size_t(sr) * d.max_consensus;
                        row[mv]      = bv;
                        row[mt]      = bt;
                    }
                }
            }
            for (int sr = lane; sr < nseq; sr += kWave)
            {
                const int node                                = int(seq_begin[sr]);
                msa_out[size_t(sr) * d.max_consensus + int(mpos[node])] = g.base[node];
            }
        }
        olap(2);
        if (lane == 0)
        {
            b.msa_len[w]    = msa_len;
            b.msa_status[w] = uint8_t(mst);
        }
    }
}


__device__ __forceinline__ int dpp_max(int v, int ctrl, int row_mask)
{
    // lanes without a source (or masked rows) keep kNeg, the max identity
    switch (ctrl)
    {
    case 0x111: return max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x111, 0xf, 0xf, false));
    case 0x112: return max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x112, 0xf, 0xf, false));
    case 0x114: return max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x114, 0xf, 0xf, false));
    case 0x118: return max(v, __builtin_amdgcn_update_dpp(kNeg, v, 0x118, 0xf, 0xf, false));
    default: return v;
    }
}

// Inclusive max-scan over the wave with DPP (row_shr 1/2/4/8, row_bcast 15/31).
// A lane with no source (outside the row, or a row masked off) keeps its own
// value as the DPP "old" operand, and max(v, v) = v: no identity constant has
// to be rematerialised for every step.
// One v_max_i32_dpp per step, written in place (dst = both sources): a lane
// whose DPP source is invalid is not written (bound_ctrl off).  The s_nop
// gives the 2 wait states a DPP read needs after the VALU write of its source.
__device__ __forceinline__ int wave_incl_max_dpp(int v)
{
    asm volatile("s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
                 "s_nop 1"
                 : "+v"(v));
    return v;
}

// Exclusive wave sum of small non-negative ints (row-program offsets): DPP
// inclusive scan (row_shr 1/2/4/8, row_bcast 15/31); the total is uniform.
__device__ __forceinline__ int wave_excl_sum(int v, int lane, int& total)
{
    int x = v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
    (void)lane;
    total = __builtin_amdgcn_readlane(x, kWave - 1);
    return x - v;
}

// ---------------------------------------------------------------------------
// Wave-parallel addAlignmentToGraph (cudapoa_add_alignment.cuh:59-279).
//
// The traceback visits every read position exactly once, in increasing
// order, so element rp of the sequential loop is read base rp and its head is
// element rp-1's node.  When every element's node is distinct and no two
// elements touch the same aligned-node group, the sequential loop's writes are
// independent and are done by one lane per element; the new node ids are a
// prefix sum, and the first error (node or edge limit) is found by a min
// over positions.  Otherwise nothing is written and -1 is returned so the
// caller runs the sequential restatement.
struct AddScratch
{
    GWAMD_LDS uint16_t* gid;   // [max_seq] aligned graph node per read position (0xffff = none)
    GWAMD_LDS uint16_t* curr;  // [max_seq] node the read base lands on
    GWAMD_LDS uint8_t* kind;   // [max_seq] 0 same base, 1 aligned hit, 2 new, 3 new + ring; bit 2: edge exists
    GWAMD_LDS uint16_t* owner; // [max_nodes + max_seq] element that claimed a node (last writer wins)
    GWAMD_LDS int* sh;         // [0] conflict
    // batched add only: slot of an existing edge head -> curr in curr's in-list
    // and (MSA) in head's out-list, found by the existence pass (0xff: none)
    GWAMD_LDS uint8_t* hit  = nullptr; // [max_seq]
    GWAMD_LDS uint8_t* ohit = nullptr; // [max_seq]
};

// writes 1 of the wave-parallel add: new nodes and aligned rings, one lane
// per new element.  The new elements' positions are first compacted into the
// owner array (free once the independence checks are done), so a 10 kb read
// with ~1,000 new nodes takes ~16 lane-parallel rounds instead of one per 64
// read positions; a ring's member loads are issued 4 at a time.
template <typename SizeT>
__device__ __forceinline__ void add_write_new_nodes(WinGraph<SizeT> g, const AddScratch& X, int L,
                                                    const uint8_t* read, int lane)
{
    GWAMD_LDS uint16_t* newpos = X.owner;
    int k = 0;
    for (int r0 = 0; r0 < L; r0 += kWave)
    {
        const int rp     = r0 + lane;
        const bool isnew = rp < L && (X.kind[rp] & 3) >= 2;
        int total        = 0;
        const int ex     = wave_excl_sum(isnew ? 1 : 0, lane, total);
        if (isnew)
            newpos[k + ex] = uint16_t(rp);
        k += total;
    }
    wave_sync();
    for (int i = lane; i < k; i += kWave)
    {
        const int rp    = int(newpos[i]);
        const int kind  = X.kind[rp] & 3;
        const int curr  = int(X.curr[rp]);
        g.base[curr]    = read[rp];
        g.out_cnt[curr] = 0;
        g.in_cnt[curr]  = 0;
        g.aln_cnt[curr] = 0;
        g.cov[curr]     = 0;
        if (kind == 3)
        {
            const int gid = int(X.gid[rp]);
            const int na  = int(g.aln_cnt[gid]);
            for (int n0 = 0; n0 < na; n0 += 4)
            {
                int aid[4], ac[4];
#pragma unroll
                for (int j = 0; j < 4; j++)
                    aid[j] = n0 + j < na ? int(g.aln[gid * kMaxAlignments + n0 + j]) : 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    ac[j] = n0 + j < na ? int(g.aln_cnt[aid[j]]) : 0;
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (n0 + j < na)
                    {
                        g.aln[aid[j] * kMaxAlignments + ac[j]] = SizeT(curr);
                        g.aln_cnt[aid[j]]                      = uint16_t(ac[j] + 1);
                        g.aln[curr * kMaxAlignments + n0 + j]  = SizeT(aid[j]);
                    }
            }
            g.aln[gid * kMaxAlignments + na]   = SizeT(curr);
            g.aln_cnt[gid]                     = uint16_t(na + 1);
            g.aln[curr * kMaxAlignments + na]  = SizeT(gid);
            g.aln_cnt[curr]                    = uint16_t(na + 1);
        }
    }
    wave_sync();
}

template <typename SizeT, bool MSA>
__device__ __forceinline__ int add_alignment_parallel(WinGraph<SizeT> g, int& node_count, const SizeT* ag, const SizeT* ar,
                                      int alen, int L, const uint8_t* read, const int8_t* w, int s, uint16_t* ecov,
                                      uint16_t* ecov_cnt, SizeT* seq_begin, int max_seqs, const AddScratch& X,
                                      int lane)
{
    g = as_global(g);
    const int nc0 = node_count;
    int err       = INT_MAX; // first error in read order: (pos << 8) | status
    if (lane == 0)
        X.sh[0] = 0;
    for (int k = lane; k < alen; k += kWave)
    {
        const int rp = int(ar[k]);
        if (rp >= 0 && rp < L)
            X.gid[rp] = uint16_t(int(ag[k]) < 0 ? 0xffff : int(ag[k]));
    }
    wave_sync();
    // kinds and existing targets
    for (int rp = lane; rp < L; rp += kWave)
    {
        const int gid    = int(X.gid[rp]);
        const uint8_t rb = read[rp];
        int kind = 2, curr = 0;
        if (gid != 0xffff)
        {
            if (g.base[gid] == rb)
                kind = 0, curr = gid;
            else
            {
                kind         = 3;
                const int na = int(g.aln_cnt[gid]);
                for (int n = 0; n < na; n++)
                {
                    const int aid = int(g.aln[gid * kMaxAlignments + n]);
                    if (g.base[aid] == rb)
                    {
                        kind = 1, curr = aid;
                        break;
                    }
                }
            }
        }
        X.kind[rp] = uint8_t(kind);
        X.curr[rp] = uint16_t(curr);
    }
    wave_sync();
    // new node ids: prefix sum over new-node elements in read order
    int nnew = 0;
    for (int r0 = 0; r0 < L; r0 += kWave)
    {
        const int rp     = r0 + lane;
        const bool isnew = rp < L && X.kind[rp] >= 2;
        int total        = 0;
        const int excl   = wave_excl_sum(isnew ? 1 : 0, lane, total);
        if (isnew)
        {
            const int id = nc0 + nnew + excl;
            X.curr[rp]   = uint16_t(id);
            if (id + 1 >= g.max_nodes)
                err = min(err, (rp << 8) | int(kNodeCountExceeded));
        }
        nnew += total;
    }
    wave_sync();
    // independence checks without atomics: every element claims its node (and,
    // for aligned hits / ring updates, its aligned group); after a barrier an
    // element that no longer owns a claimed node has a conflicting partner.
    for (int rp = lane; rp < L; rp += kWave)
        X.owner[int(X.curr[rp])] = uint16_t(rp);
    wave_sync();
    bool conflict = false;
    for (int rp = lane; rp < L; rp += kWave)
        conflict |= int(X.owner[int(X.curr[rp])]) != rp;
    wave_sync();
    for (int rp = lane; rp < L; rp += kWave)
    {
        const int kind = X.kind[rp];
        if (kind == 1 || kind == 3)
        {
            const int gid = int(X.gid[rp]);
            X.owner[gid]  = uint16_t(rp);
            const int na  = int(g.aln_cnt[gid]);
            for (int n = 0; n < na; n++)
                X.owner[int(g.aln[gid * kMaxAlignments + n])] = uint16_t(rp);
        }
    }
    wave_sync();
    for (int rp = lane; rp < L; rp += kWave)
    {
        const int kind = X.kind[rp];
        if (kind == 1 || kind == 3)
        {
            const int gid = int(X.gid[rp]);
            conflict |= int(X.owner[gid]) != rp;
            const int na = int(g.aln_cnt[gid]);
            for (int n = 0; n < na; n++)
                conflict |= int(X.owner[int(g.aln[gid * kMaxAlignments + n])]) != rp;
        }
    }
    if (conflict)
        X.sh[0] = 1;
    wave_sync();
    if (X.sh[0])
        return -1;
    // edge existence and edge-limit errors
    for (int rp = lane + 1; rp < L; rp += kWave)
    {
        const int head = int(X.curr[rp - 1]);
        const int curr = int(X.curr[rp]);
        const int kind = X.kind[rp];
        bool exists    = false;
        int ic         = 0;
        if (kind < 2)
        {
            ic = int(g.in_cnt[curr]);
            for (int e = 0; e < ic; e++)
                exists |= int(g.in_e[curr * kMaxEdges + e]) == head;
        }
        if (!exists)
        {
            // (bit 2 of a kind may already be set by this pass's previous iteration)
            const int oc = (X.kind[rp - 1] & 3) >= 2 ? 0 : int(g.out_cnt[head]);
            if (oc + 1 >= kMaxEdges || ic + 1 >= kMaxEdges)
                err = min(err, (rp << 8) | int(kEdgeCountExceeded));
        }
        else
            X.kind[rp] = uint8_t(kind | 4);
    }
    err = -wave_max(-err); // wave-wide minimum
    if (err != INT_MAX)
        return err & 0xff;
    wave_sync();
    add_write_new_nodes<SizeT>(g, X, L, read, lane);
    // writes 2: the edge head -> curr and the coverage of curr
    for (int rp = lane; rp < L; rp += kWave)
    {
        const int curr = int(X.curr[rp]);
        if (MSA && rp == 0)
            seq_begin[s] = SizeT(curr);
        if (rp > 0)
        {
            const int head = int(X.curr[rp - 1]);
            const int wsum = int(uint16_t(int(w[rp - 1]))) + int(w[rp]);
            if (X.kind[rp] & 4)
            {
                const int ic = int(g.in_cnt[curr]);
                for (int e = 0; e < ic; e++)
                    if (int(g.in_e[curr * kMaxEdges + e]) == head)
                        g.in_w[curr * kMaxEdges + e] = uint16_t(int(g.in_w[curr * kMaxEdges + e]) + wsum);
                if (MSA)
                {
                    const int oc = int(g.out_cnt[head]);
                    for (int e = 0; e < oc; e++)
                    {
                        if (int(g.out_e[head * kMaxEdges + e]) == curr)
                        {
                            const int c                                       = int(ecov_cnt[head * kMaxEdges + e]);
                            ecov[size_t(head * kMaxEdges + e) * max_seqs + c] = uint16_t(s);
                            ecov_cnt[head * kMaxEdges + e]                    = uint16_t(c + 1);
                            break;
                        }
                    }
                }
            }
            else
            {
                const int ic                   = int(g.in_cnt[curr]);
                g.in_e[curr * kMaxEdges + ic]  = SizeT(head);
                g.in_w[curr * kMaxEdges + ic]  = uint16_t(wsum);
                g.in_cnt[curr]                 = uint16_t(ic + 1);
                const int oc                   = int(g.out_cnt[head]);
                g.out_e[head * kMaxEdges + oc] = SizeT(curr);
                if (MSA)
                {
                    ecov_cnt[head * kMaxEdges + oc]                = 1;
                    ecov[size_t(head * kMaxEdges + oc) * max_seqs] = uint16_t(s);
                }
                g.out_cnt[head] = uint16_t(oc + 1);
            }
        }
        g.cov[curr]++;
    }
    node_count = nc0 + nnew;
    wave_sync();
    return kSuccess;
}

// The same add with kAU read positions per lane and pass and their graph
// loads issued together (one HBM round trip per dependent level instead of one
// per position): used by the banded kernel, whose windows are long (config C:
// 10 kb reads, 21 ms of adds per window before); the LDS full-alignment kernel
// keeps the one-position form (the batched one raises its register count and
// slows its forward pass).  nwv > 1: the nwv waves of the workgroup run it
// together (wave wv; every wave calls it with the same arguments): the
// order-free passes split the read positions among the waves and meet at
// workgroup barriers; the new-node numbering and the new nodes' writes stay
// on wave 0.  The return value and node_count are wave 0's.
template <typename SizeT, bool MSA, int kAU = 4>
__device__ __forceinline__ int add_alignment_parallel_batched(WinGraph<SizeT> g, int& node_count, const SizeT* ag, const SizeT* ar,
                                      int alen, int L, const uint8_t* read, const int8_t* w, int s, uint16_t* ecov,
                                      uint16_t* ecov_cnt, SizeT* seq_begin, int max_seqs, const AddScratch& X,
                                      int lane, uint64_t* prof = nullptr, int wv = 0, int nwv = 1)
{
    g = as_global(g);
    auto bar = [&]() {
        if (nwv > 1)
            __syncthreads();
        else
            wave_sync();
    };
    const int step1 = nwv * kWave, stepA = nwv * kAU * kWave;
#ifdef GWAMD_ADD_PROFILE
    uint64_t pt = now_ticks();
    auto lap = [&](int k) { const uint64_t t = now_ticks(); if (prof) prof[k] += t - pt; pt = t; };
#else
    auto lap = [&](int) {};
#endif
    const int nc0 = node_count;
    int err       = INT_MAX; // first error in read order: (pos << 8) | status
    if (lane == 0 && wv == 0)
        X.sh[0] = 0;
    for (int k0 = wv * 4 * kWave; k0 < alen; k0 += 4 * step1)
    {
        int rp[4], gv[4];
#pragma unroll
        for (int u = 0; u < 4; u++)
        {
            const int k = k0 + u * kWave + lane;
            rp[u]       = k < alen ? int(ar[k]) : -1;
            gv[u]       = k < alen ? int(ag[k]) : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (rp[u] >= 0 && rp[u] < L)
                X.gid[rp[u]] = uint16_t(gv[u] < 0 ? 0xffff : gv[u]);
    }
    bar();
    lap(0);
    // kinds and existing targets.  kAU positions per lane and pass, their
    // graph loads issued together (the graph is in HBM: one round trip per
    // dependent level instead of one per position)
    for (int r0 = wv * kAU * kWave; r0 < L; r0 += stepA)
    {
        int gid[kAU], kind[kAU], curr[kAU], na[kAU], gb[kAU];
        uint8_t rb[kAU];
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            gid[u]       = rp < L ? int(X.gid[rp]) : 0xffff;
            rb[u]        = rp < L ? read[rp] : uint8_t(0);
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const bool has = gid[u] != 0xffff;
            gb[u]          = has ? int(g.base[gid[u]]) : 0;
            na[u]          = has ? int(g.aln_cnt[gid[u]]) : 0;
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            kind[u] = gid[u] == 0xffff ? 2 : (gb[u] == int(rb[u]) ? 0 : 3);
            curr[u] = kind[u] == 0 ? gid[u] : 0;
        }
        // aligned-node lists of the mismatching positions, 4 entries at a
        // time: the first aligned node with the read's base (:130-150)
        for (int n0 = 0;; n0 += 4)
        {
            bool need = false;
#pragma unroll
            for (int u = 0; u < kAU; u++)
                need |= kind[u] == 3 && n0 < na[u];
            if (__builtin_amdgcn_ballot_w64(need) == 0)
                break;
            int aid[kAU][4], ab[kAU][4];
#pragma unroll
            for (int u = 0; u < kAU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    aid[u][j] = (kind[u] == 3 && n0 + j < na[u]) ? int(g.aln[gid[u] * kMaxAlignments + n0 + j]) : -1;
#pragma unroll
            for (int u = 0; u < kAU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    ab[u][j] = aid[u][j] >= 0 ? int(g.base[aid[u][j]]) : -1;
#pragma unroll
            for (int u = 0; u < kAU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (kind[u] == 3 && aid[u][j] >= 0 && ab[u][j] == int(rb[u]))
                        kind[u] = 1, curr[u] = aid[u][j];
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            if (rp < L)
            {
                X.kind[rp] = uint8_t(kind[u]);
                X.curr[rp] = uint16_t(curr[u]);
            }
        }
    }
    bar();
    lap(1);
    // new node ids: prefix sum over new-node elements in read order (wave 0)
    int nnew = 0;
    for (int r0 = 0; wv == 0 && r0 < L; r0 += kWave)
    {
        const int rp     = r0 + lane;
        const bool isnew = rp < L && X.kind[rp] >= 2;
        int total        = 0;
        const int excl   = wave_excl_sum(isnew ? 1 : 0, lane, total);
        if (isnew)
        {
            const int id = nc0 + nnew + excl;
            X.curr[rp]   = uint16_t(id);
            if (id + 1 >= g.max_nodes)
                err = min(err, (rp << 8) | int(kNodeCountExceeded));
        }
        nnew += total;
    }
    bar();
    lap(2);
    // independence checks without atomics: every element claims its node (and,
    // for aligned hits / ring updates, its aligned group); after a barrier an
    // element that no longer owns a claimed node has a conflicting partner.
    for (int rp = wv * kWave + lane; rp < L; rp += step1)
        X.owner[int(X.curr[rp])] = uint16_t(rp);
    bar();
    bool conflict = false;
    for (int rp = wv * kWave + lane; rp < L; rp += step1)
        conflict |= int(X.owner[int(X.curr[rp])]) != rp;
    bar();
    lap(3);
    // aligned groups of the mismatching positions: claim every member, then
    // check the claims (kAU positions per lane, loads batched as above)
    for (int pass = 0; pass < 2; pass++)
    {
        for (int r0 = wv * kAU * kWave; r0 < L; r0 += stepA)
        {
            int gid[kAU], na[kAU];
#pragma unroll
            for (int u = 0; u < kAU; u++)
            {
                const int rp   = r0 + u * kWave + lane;
                const int kind = rp < L ? int(X.kind[rp]) : 0;
                gid[u]         = (kind == 1 || kind == 3) ? int(X.gid[rp]) : -1;
            }
#pragma unroll
            for (int u = 0; u < kAU; u++)
                na[u] = gid[u] >= 0 ? int(g.aln_cnt[gid[u]]) : 0;
#pragma unroll
            for (int u = 0; u < kAU; u++)
            {
                const int rp = r0 + u * kWave + lane;
                if (gid[u] < 0)
                    continue;
                if (pass == 0)
                    X.owner[gid[u]] = uint16_t(rp);
                else
                    conflict |= int(X.owner[gid[u]]) != rp;
            }
            for (int n0 = 0;; n0 += 4)
            {
                bool need = false;
#pragma unroll
                for (int u = 0; u < kAU; u++)
                    need |= n0 < na[u];
                if (__builtin_amdgcn_ballot_w64(need) == 0)
                    break;
                int aid[kAU][4];
#pragma unroll
                for (int u = 0; u < kAU; u++)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        aid[u][j] = n0 + j < na[u] ? int(g.aln[gid[u] * kMaxAlignments + n0 + j]) : -1;
#pragma unroll
                for (int u = 0; u < kAU; u++)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                    {
                        if (aid[u][j] < 0)
                            continue;
                        const int rp = r0 + u * kWave + lane;
                        if (pass == 0)
                            X.owner[aid[u][j]] = uint16_t(rp);
                        else
                            conflict |= int(X.owner[aid[u][j]]) != rp;
                    }
            }
        }
        bar();
    }
    if (conflict)
        X.sh[0] = 1;
    bar();
    if (X.sh[0])
        return -1;
    lap(4);
    // edge existence and edge-limit errors (kAU positions per lane and pass)
    for (int r0 = 1 + wv * kAU * kWave; r0 < L; r0 += stepA)
    {
        int head[kAU], curr[kAU], kind[kAU], ic[kAU], oc[kAU], hitv[kAU], ohitv[kAU];
        bool exists[kAU];
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            const bool in = rp < L;
            head[u]       = in ? int(X.curr[rp - 1]) : 0;
            curr[u]       = in ? int(X.curr[rp]) : 0;
            kind[u]       = in ? int(X.kind[rp]) : 2;
            const int kp  = in ? int(X.kind[rp - 1]) & 3 : 2; // (bit 2 may be set by the previous pass)
            ic[u]         = kind[u] < 2 ? int(g.in_cnt[curr[u]]) : 0;
            oc[u]         = kp >= 2 ? 0 : int(g.out_cnt[head[u]]);
            exists[u]     = false;
            hitv[u]       = 0xff;
            ohitv[u]      = 0xff;
        }
        for (int e0 = 0;; e0 += 4)
        {
            bool need = false;
#pragma unroll
            for (int u = 0; u < kAU; u++)
                need |= !exists[u] && e0 < ic[u];
            if (__builtin_amdgcn_ballot_w64(need) == 0)
                break;
            int ie[kAU][4];
#pragma unroll
            for (int u = 0; u < kAU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    ie[u][j] = (!exists[u] && e0 + j < ic[u]) ? int(g.in_e[curr[u] * kMaxEdges + e0 + j]) : -1;
#pragma unroll
            for (int u = 0; u < kAU; u++)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (!exists[u] && ie[u][j] == head[u])
                        exists[u] = true, hitv[u] = e0 + j;
        }
        if (MSA)
        {
            // the same edge in head's out-list (its read list gets this read)
            for (int e0 = 0;; e0 += 4)
            {
                bool need = false;
#pragma unroll
                for (int u = 0; u < kAU; u++)
                    need |= exists[u] && ohitv[u] == 0xff && e0 < oc[u];
                if (__builtin_amdgcn_ballot_w64(need) == 0)
                    break;
                int oe[kAU][4];
#pragma unroll
                for (int u = 0; u < kAU; u++)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        oe[u][j] = (exists[u] && ohitv[u] == 0xff && e0 + j < oc[u])
                                       ? int(g.out_e[head[u] * kMaxEdges + e0 + j]) : -1;
#pragma unroll
                for (int u = 0; u < kAU; u++)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (ohitv[u] == 0xff && oe[u][j] >= 0 && oe[u][j] == curr[u])
                            ohitv[u] = e0 + j;
            }
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            if (rp >= L)
                continue;
            if (!exists[u])
            {
                if (oc[u] + 1 >= kMaxEdges || ic[u] + 1 >= kMaxEdges)
                    err = min(err, (rp << 8) | int(kEdgeCountExceeded));
            }
            else
                X.kind[rp] = uint8_t(kind[u] | 4);
            X.hit[rp]  = uint8_t(hitv[u]);
            X.ohit[rp] = uint8_t(ohitv[u]);
        }
    }
    err = -wave_max(-err); // wave-wide minimum
    if (nwv > 1)
    {
        // workgroup minimum through one word per wave
        if (lane == 0)
            X.sh[2 + wv] = err;
        __syncthreads();
        for (int q = 0; q < nwv; q++)
            err = min(err, int(X.sh[2 + q]));
    }
    if (err != INT_MAX)
        return err & 0xff;
    bar();
    lap(5);
    if (wv == 0)
        add_write_new_nodes<SizeT>(g, X, L, read, lane);
    bar();
    lap(6);
    // writes 2: the edge head -> curr and the coverage of curr.  Element rp
    // touches only curr's in-list and coverage and head's out-list (head =
    // element rp-1's curr), so the elements are independent; kAU per lane and
    // pass, with their loads issued together.
    for (int r0 = wv * kAU * kWave; r0 < L; r0 += stepA)
    {
        int curr[kAU], head[kAU], kind[kAU], wsum[kAU], ic[kAU], oc[kAU], cv[kAU], hit[kAU], ohit[kAU];
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            const bool in = rp < L;
            curr[u]       = in ? int(X.curr[rp]) : 0;
            head[u]       = (in && rp > 0) ? int(X.curr[rp - 1]) : 0;
            kind[u]       = (in && rp > 0) ? int(X.kind[rp]) : -1; // -1: no edge (rp 0 or out of range)
            wsum[u]       = (in && rp > 0) ? int(uint16_t(int(w[rp - 1]))) + int(w[rp]) : 0;
            // existing edges: their slots from the existence pass
            const int hs  = (in && rp > 0) ? int(X.hit[rp]) : 0xff;
            const int os  = (in && rp > 0) ? int(X.ohit[rp]) : 0xff;
            hit[u]        = hs == 0xff ? -1 : hs;
            ohit[u]       = os == 0xff ? -1 : os;
            if (MSA && in && rp == 0)
                seq_begin[s] = SizeT(curr[u]);
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp  = r0 + u * kWave + lane;
            const bool nw = kind[u] >= 0 && !(kind[u] & 4); // a new edge
            ic[u]         = nw ? int(g.in_cnt[curr[u]]) : 0;
            oc[u]         = nw ? int(g.out_cnt[head[u]]) : 0;
            cv[u]         = rp < L ? int(g.cov[curr[u]]) : 0;
        }
#pragma unroll
        for (int u = 0; u < kAU; u++)
        {
            const int rp = r0 + u * kWave + lane;
            if (rp >= L)
                continue;
            if (kind[u] >= 0)
            {
                const int cu = curr[u], hd = head[u];
                if (kind[u] & 4)
                {
                    if (hit[u] >= 0)
                        g.in_w[cu * kMaxEdges + hit[u]] = uint16_t(int(g.in_w[cu * kMaxEdges + hit[u]]) + wsum[u]);
                    if (MSA && ohit[u] >= 0)
                    {
                        const int c                                             = int(ecov_cnt[hd * kMaxEdges + ohit[u]]);
                        ecov[size_t(hd * kMaxEdges + ohit[u]) * max_seqs + c] = uint16_t(s);
                        ecov_cnt[hd * kMaxEdges + ohit[u]]                      = uint16_t(c + 1);
                    }
                }
                else
                {
                    g.in_e[cu * kMaxEdges + ic[u]] = SizeT(hd);
                    g.in_w[cu * kMaxEdges + ic[u]] = uint16_t(wsum[u]);
                    g.in_cnt[cu]                   = uint16_t(ic[u] + 1);
                    g.out_e[hd * kMaxEdges + oc[u]] = SizeT(cu);
                    if (MSA)
                    {
                        ecov_cnt[hd * kMaxEdges + oc[u]]                = 1;
                        ecov[size_t(hd * kMaxEdges + oc[u]) * max_seqs] = uint16_t(s);
                    }
                    g.out_cnt[hd] = uint16_t(oc[u] + 1);
                }
            }
            g.cov[curr[u]] = uint16_t(cv[u] + 1);
        }
    }
    node_count = nc0 + nnew;
    bar();
    lap(7);
    return kSuccess;
}

// racon/SPOA DFS sort (cudapoa_topsort.cuh:94-189) by one wave with the node
// marks and the DFS stack in LDS: the predecessor and aligned-node lists of
// the node on top of the stack are read one entry per lane, and the entries to
// visit are pushed in list order with a ballot (in-edges first, then aligned
// nodes, as the sequential loop does).  With mpos it also writes the MSA column
// of every node (getNodeIDToMSAPosDevice, cudapoa_generate_msa.cuh:27-45: one
// column per emitted node and its aligned nodes) and the column count to
// *ncols.  Returns false when the marks and a useful stack do not fit in the
// scratch, or when the stack outgrows it (after a partial sort): the caller
// then runs topsort_racon, which rewrites everything.
// CSR: when they fit next to the marks and a stack of at least kRaconCsrStack
// entries, the predecessor and aligned-node lists are first copied to LDS
// (per node one word: list offset | in-degree << 20 | aligned count << 26;
// entries u16, predecessors then aligned nodes), so a DFS step reads no HBM.
constexpr int kRaconCsrStack = 4096;

// The DFS of topsort_racon_lds over the LDS CSR copy, arranged so that a step
// waits on as few dependent LDS round trips as the order allows:
//  * a first visit reads the node's list (predecessors, then aligned nodes
//    while its check flag is set) one entry per lane, then the marks and list
//    words of all entries at once; the pushed entries are the entries whose
//    mark is not 2, in list order (cudapoa_topsort.cuh:134-158), and the new
//    top's mark and word come from the lane that read them;
//  * a node found again on top with mark 1 is emitted without re-reading its
//    lists: everything pushed above it has been popped, and entries are popped
//    only when done, so all its predecessors (and the aligned nodes it pushed)
//    are done, which is what the reference's second scan establishes;
//  * a pop reads the popped node's mark and word together with the stack
//    entry below it;
//  * the outer loop over node ids (cudapoa_topsort.cuh:117-126) scans the
//    marks 64 at a time;
//  * an emitted group (cudapoa_topsort.cuh:160-175) is recorded as its head
//    node in heads[] (HBM); the order and columns are expanded from the heads
//    after the DFS, in parallel.
// Returns false (partial output, nothing to trust) when the stack would
// outgrow cap entries.
template <typename SizeT>
__device__ __forceinline__ bool racon_dfs_csr(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* marks,
                                              GWAMD_LDS uint32_t* info, GWAMD_LDS uint16_t* lists,
                                              GWAMD_LDS uint16_t* stack, int cap, int lane, int32_t* heads_,
                                              SizeT* mpos, int* ncols)
{
    GWAMD_GLB int32_t* heads  = (GWAMD_GLB int32_t*)(heads_);
    const uint64_t lt         = (uint64_t(1) << lane) - 1;
    int kq                    = 0; // emitted groups
    int v0                    = 0;
    while (true)
    {
        // next node id whose mark is 0 (the outer loop of the reference)
        int id = -1, m = 0;
        uint32_t w = 0;
        for (; v0 < n; v0 += kWave)
        {
            // (reads at clamped addresses, then selects: no divergent branch
            // between the loads and their wait)
            const int v       = v0 + lane;
            const int vc      = v < n ? v : 0;
            const int mr      = int(marks[vc]);
            const uint32_t iw = info[vc];
            const int mk      = v < n ? mr : 2;
            const uint64_t bf = __builtin_amdgcn_ballot_w64((mk & 3) == 0);
            if (bf)
            {
                const int l = __builtin_ctzll(bf);
                id          = v0 + l;
                m           = __builtin_amdgcn_readlane(mk, l);
                w           = uint32_t(__builtin_amdgcn_readlane(int(iw), l));
                break;
            }
        }
        if (id < 0)
            break;
        v0        = id + 1;
        int top   = 0;
        int below = 0; // stack[top - 1] when top > 0
        if (lane == 0)
            stack[0] = uint16_t(id);
        while (true)
        {
            const int mm = m & 3; // 0: first visit; 1: emit; 2: pop only
            if (mm == 0)
            {
                const int ic  = int((w >> 20) & 63u);
                const int cnt = ic + ((m & 4) ? int(w >> 26) : 0);
                const int o   = int(w & 0xfffffu);
                const int e0 = lane, e1 = lane + kWave;
                const int l0r = int(lists[e0 < cnt ? o + e0 : 0]);
                const int n0  = e0 < cnt ? l0r : 0;
                const int k0r = int(marks[n0]);
                const uint32_t w0 = info[n0];
                const int k0      = e0 < cnt ? k0r : 2;
                int n1 = 0, k1 = 2;
                uint32_t w1 = 0;
                if (cnt > kWave) // (more than 64 list entries: rare)
                {
                    n1 = e1 < cnt ? int(lists[o + e1]) : 0;
                    k1 = e1 < cnt ? int(marks[n1]) : 2;
                    w1 = info[n1];
                }
                const bool p0     = (k0 & 3) != 2;
                const bool p1     = (k1 & 3) != 2;
                const uint64_t b0 = __builtin_amdgcn_ballot_w64(p0);
                const uint64_t b1 = __builtin_amdgcn_ballot_w64(p1);
                const int c0 = __popcll(b0), c1 = __popcll(b1);
                if (c0 + c1 != 0) // (else valid: emitted below)
                {
                    if (top + c0 + c1 >= cap)
                        return false;
                    if (p0)
                    {
                        stack[top + 1 + __popcll(b0 & lt)] = uint16_t(n0);
                        if (e0 >= ic) // aligned node: check_aligned_nodes = false
                            marks[n0] = uint8_t(k0 & 3);
                    }
                    if (p1)
                    {
                        stack[top + 1 + c0 + __popcll(b1 & lt)] = uint16_t(n1);
                        if (e1 >= ic)
                            marks[n1] = uint8_t(k1 & 3);
                    }
                    if (lane == 0)
                        marks[id] = uint8_t((m & 4) | 1);
                    // the last entry pushed is the new top, the one before it
                    // (or this node) lies below it
                    int nid, nm, ne;
                    uint32_t nw;
                    if (c1)
                    {
                        const int l = 63 - __builtin_clzll(b1);
                        nid = __builtin_amdgcn_readlane(n1, l), nm = __builtin_amdgcn_readlane(k1, l);
                        nw  = uint32_t(__builtin_amdgcn_readlane(int(w1), l));
                        ne  = kWave + l;
                        const uint64_t r1 = b1 & ~(uint64_t(1) << l);
                        below = r1 ? __builtin_amdgcn_readlane(n1, 63 - __builtin_clzll(r1))
                                   : (c0 ? __builtin_amdgcn_readlane(n0, 63 - __builtin_clzll(b0)) : id);
                    }
                    else
                    {
                        const int l = 63 - __builtin_clzll(b0);
                        nid = __builtin_amdgcn_readlane(n0, l), nm = __builtin_amdgcn_readlane(k0, l);
                        nw  = uint32_t(__builtin_amdgcn_readlane(int(w0), l));
                        ne  = l;
                        const uint64_t r0 = b0 & ~(uint64_t(1) << l);
                        below = r0 ? __builtin_amdgcn_readlane(n0, 63 - __builtin_clzll(r0)) : id;
                    }
                    top += c0 + c1;
                    id = nid, w = nw;
                    m  = ne >= ic ? (nm & 3) : nm;
                    continue;
                }
            }
            if (mm != 2)
            {
                // valid (cudapoa_topsort.cuh:160-176): mark 2; the group is
                // emitted when check_aligned_nodes is set
                if (lane == 0)
                {
                    marks[id] = uint8_t((m & 4) | 2);
                    if (m & 4)
                        heads[kq] = id;
                }
                kq += (m & 4) ? 1 : 0;
            }
            top--;
            if (top < 0)
                break;
            id = below;
            // the popped node's mark and word, and the entry below it
            const int mr      = int(marks[id]);
            const uint32_t wr = info[id];
            const int br      = top > 0 ? int(stack[top - 1]) : 0;
            m                 = __builtin_amdgcn_readfirstlane(mr);
            w                 = uint32_t(__builtin_amdgcn_readfirstlane(int(wr)));
            below             = __builtin_amdgcn_readfirstlane(br);
        }
    }
    // expansion: head i is column i; its group is the head then all its
    // aligned nodes (cudapoa_topsort.cuh:165-174, getNodeIDToMSAPosDevice)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wave_sync();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    GWAMD_GLB SizeT* sorted = (GWAMD_GLB SizeT*)(g.sorted);
    GWAMD_GLB SizeT* pos    = (GWAMD_GLB SizeT*)(g.pos);
    GWAMD_GLB SizeT* mp     = (GWAMD_GLB SizeT*)(mpos);
    int kbase               = 0;
    for (int c = 0; c < kq; c += kWave)
    {
        const int i       = c + lane;
        const bool act    = i < kq;
        const int h       = act ? int(heads[i]) : 0;
        const uint32_t hw = act ? info[h] : 0u;
        const int ic = int((hw >> 20) & 63u), ac = act ? int(hw >> 26) : 0, o = int(hw & 0xfffffu);
        int tot           = 0;
        const int k       = kbase + wave_excl_sum(act ? 1 + ac : 0, lane, tot);
        if (act)
        {
            sorted[k] = SizeT(h);
            pos[h]    = SizeT(k);
            if (mp)
                mp[h] = SizeT(i);
            for (int a = 0; a < ac; a++)
            {
                const int al     = int(lists[o + ic + a]);
                sorted[k + 1 + a] = SizeT(al);
                pos[al]           = SizeT(k + 1 + a);
                if (mp)
                    mp[al] = SizeT(i);
            }
        }
        kbase += tot;
    }
    if (ncols)
        *ncols = kq;
    return true;
}

template <typename SizeT, bool CSR>
__device__ __forceinline__ bool topsort_racon_lds_impl(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* scratch,
                                                       int scratch_bytes, int lane, SizeT* mpos, int* ncols,
                                                       int list_total, int32_t* heads)
{
    g = as_global(g);
    n                 = uniform(n);
    const int marks_b = (n + 15) & ~15;
    const int info_b  = CSR ? n * 4 : 0;
    const int list_b  = CSR ? ((list_total * 2 + 15) & ~15) : 0;
    const int used    = marks_b + info_b + list_b;
    const int cap     = scratch_bytes > used ? (scratch_bytes - used) / 2 : 0;
    if (scratch == nullptr || n <= 0 || n > 65535 || cap < 4 * kWave)
        return false;
    GWAMD_LDS uint8_t* marks  = scratch;
    GWAMD_LDS uint32_t* info  = (GWAMD_LDS uint32_t*)(scratch + marks_b);
    GWAMD_LDS uint16_t* lists = (GWAMD_LDS uint16_t*)(scratch + marks_b + info_b);
    GWAMD_LDS uint16_t* stack = (GWAMD_LDS uint16_t*)(scratch + used);
    for (int v = lane; v < n; v += kWave)
        marks[v] = 4; // mark 0, check_aligned_nodes = true
    if constexpr (CSR)
    {
        // two 64-node chunks per step, the counts and the first kPreE / kPreA
        // slots of every node loaded together (one HBM round trip per step;
        // longer lists read the rest one entry at a time)
        constexpr int kPreE = 8, kPreA = 4, kU = 2;
        int base = 0;
        for (int v0 = 0; v0 < n; v0 += kU * kWave)
        {
            int ic[kU], ac[kU], pe[kU][kPreE], pa[kU][kPreA];
#pragma unroll
            for (int u = 0; u < kU; u++)
            {
                const int v  = v0 + u * kWave + lane;
                const int vr = v < n ? v : 0;
                ic[u]        = v < n ? int(g.in_cnt[vr]) : 0;
                ac[u]        = v < n ? int(g.aln_cnt[vr]) : 0;
#pragma unroll
                for (int e = 0; e < kPreE; e++)
                    pe[u][e] = int(g.in_e[vr * kMaxEdges + e]);
#pragma unroll
                for (int e = 0; e < kPreA; e++)
                    pa[u][e] = int(g.aln[vr * kMaxAlignments + e]);
            }
#pragma unroll
            for (int u = 0; u < kU; u++)
            {
                const int v   = v0 + u * kWave + lane;
                int total     = 0;
                const int o   = base + wave_excl_sum(ic[u] + ac[u], lane, total);
                base         += total;
                if (v < n)
                {
                    info[v] = uint32_t(o) | (uint32_t(ic[u]) << 20) | (uint32_t(ac[u]) << 26);
#pragma unroll
                    for (int e = 0; e < kPreE; e++)
                        if (e < ic[u])
                            lists[o + e] = uint16_t(pe[u][e]);
                    for (int e = kPreE; e < ic[u]; e++)
                        lists[o + e] = uint16_t(int(g.in_e[v * kMaxEdges + e]));
#pragma unroll
                    for (int e = 0; e < kPreA; e++)
                        if (e < ac[u])
                            lists[o + ic[u] + e] = uint16_t(pa[u][e]);
                    for (int e = kPreA; e < ac[u]; e++)
                        lists[o + ic[u] + e] = uint16_t(int(g.aln[v * kMaxAlignments + e]));
                }
            }
        }
    }
    wave_sync();
    if constexpr (CSR)
    {
        if (heads)
            return racon_dfs_csr<SizeT>(g, n, marks, info, lists, stack, cap, lane, heads, mpos, ncols);
    }
    int k = 0, col = 0;
    for (int v0 = 0; v0 < n; v0++)
    {
        if ((uniform(int(marks[v0])) & 3) != 0)
            continue;
        int top = 0, id = v0;
        if (lane == 0)
            stack[0] = uint16_t(v0);
        while (top >= 0)
        {
            top         = uniform(top);
            id          = uniform(id);
            k           = uniform(k);
            col         = uniform(col);
            // the mark and (CSR) the list word of the node are read together
            const int mraw      = int(marks[id]);
            const uint32_t wraw = CSR ? info[id] : 0u;
            const int m = uniform(mraw);
            bool valid  = true;
            if ((m & 3) != 2)
            {
                int ic, ac, bl, al;
                if constexpr (CSR)
                {
                    const uint32_t w = uint32_t(uniform(int(wraw)));
                    const int o      = int(w & 0xfffffu);
                    ic               = int((w >> 20) & 63u);
                    ac               = (m & 4) ? int(w >> 26) : 0;
                    bl               = lane < ic ? int(lists[o + lane]) : 0;
                    al               = lane < ac ? int(lists[o + ic + lane]) : 0;
                }
                else
                {
                    // the lists are read in full (every slot of the node's
                    // rows is in bounds) in the same round trip as the counts
                    const int blr = lane < kMaxEdges ? int(g.in_e[id * kMaxEdges + lane]) : 0;
                    const int alr = lane < kMaxAlignments ? int(g.aln[id * kMaxAlignments + lane]) : 0;
                    ic            = uniform(int(g.in_cnt[id]));
                    ac            = (m & 4) ? uniform(int(g.aln_cnt[id])) : 0;
                    bl            = lane < ic ? blr : 0;
                    al            = lane < ac ? alr : 0;
                }
                const int mb      = lane < ic ? int(marks[bl]) : 2;
                const int ma      = lane < ac ? int(marks[al]) : 2;
                const bool nb     = lane < ic && (mb & 3) != 2;
                const bool na     = lane < ac && (ma & 3) != 2;
                const uint64_t bb = __builtin_amdgcn_ballot_w64(nb);
                const uint64_t ba = __builtin_amdgcn_ballot_w64(na);
                const int cb = __popcll(bb), ca = __popcll(ba);
                if (cb + ca > 0)
                {
                    if (top + cb + ca >= cap)
                        return false;
                    const uint64_t below = (uint64_t(1) << lane) - 1;
                    if (nb)
                        stack[top + 1 + __popcll(bb & below)] = uint16_t(bl);
                    if (na)
                    {
                        stack[top + 1 + cb + __popcll(ba & below)] = uint16_t(al);
                        marks[al] = uint8_t(ma & 3); // check_aligned_nodes = false
                    }
                    if (lane == 0)
                        marks[id] = uint8_t((m & 4) | 1);
                    valid = false;
                    // the last entry pushed is the new top
                    id = ca > 0 ? __builtin_amdgcn_readlane(al, 63 - __builtin_clzll(ba))
                                : __builtin_amdgcn_readlane(bl, 63 - __builtin_clzll(bb));
                    top += cb + ca;
                }
                else
                {
                    if (m & 4)
                    {
                        // emit the node, then all its aligned nodes
                        if (lane == 0)
                        {
                            g.sorted[k] = SizeT(id);
                            g.pos[id]   = SizeT(k);
                            if (mpos)
                                mpos[id] = SizeT(col);
                        }
                        if (lane < ac)
                        {
                            g.sorted[k + 1 + lane] = SizeT(al);
                            g.pos[al]              = SizeT(k + 1 + lane);
                            if (mpos)
                                mpos[al] = SizeT(col);
                        }
                        k += 1 + ac;
                        col++;
                    }
                    if (lane == 0)
                        marks[id] = uint8_t((m & 4) | 2);
                }
            }
            if (valid)
            {
                top--;
                if (top >= 0)
                    id = uniform(int(stack[top]));
            }
            wave_sync();
        }
    }
    if (ncols)
        *ncols = col;
    return true;
}

template <typename SizeT>
__device__ __forceinline__ bool topsort_racon_lds(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* scratch,
                                                  int scratch_bytes, int lane, SizeT* mpos, int* ncols,
                                                  int32_t* heads)
{
    g = as_global(g);
    n = uniform(n);
    if (scratch == nullptr || n <= 0 || n > 65535)
        return false;
    // list entries of the CSR copy
    int total = 0;
    for (int v0 = 0; v0 < n; v0 += kWave)
    {
        const int v = v0 + lane;
        int t       = 0;
        wave_excl_sum(v < n ? int(g.in_cnt[v]) + int(g.aln_cnt[v]) : 0, lane, t);
        total += t;
    }
    total = uniform(total);
    const int need = ((n + 15) & ~15) + n * 4 + ((total * 2 + 15) & ~15) + 2 * kRaconCsrStack;
    if (total < (1 << 20) && need <= scratch_bytes)
        return topsort_racon_lds_impl<SizeT, true>(g, n, scratch, scratch_bytes, lane, mpos, ncols, total, heads);
    return topsort_racon_lds_impl<SizeT, false>(g, n, scratch, scratch_bytes, lane, mpos, ncols, 0, nullptr);
}

// SPOA_ACCURATE per-read sort (cudapoa_kernels.cuh:324-337): the LDS racon
// sort when it fits in scratch, else the racon DFS on lane 0; returns the
// window status for every lane.
template <typename SizeT>
__device__ __forceinline__ int topsort_racon_wave(WinGraph<SizeT> g, int n, int32_t* marks, SizeT* stack, int cap,
                                                  int lane, GWAMD_LDS uint8_t* scratch = nullptr,
                                                  int scratch_bytes = 0)
{
    if (topsort_racon_lds<SizeT>(g, n, scratch, scratch_bytes, lane, nullptr, nullptr, marks))
        return int(kSuccess);
    int ok = 1;
    if (lane == 0)
        ok = topsort_racon<SizeT>(g, n, marks, stack, cap) ? 1 : 0;
    wave_sync();
    return __builtin_amdgcn_readfirstlane(ok) ? int(kSuccess) : int(kGenericError);
}

// ---------------------------------------------------------------------------
// Kahn topological sort (cudapoa_topsort.cuh:38-88) over an LDS copy of the
// out-edge lists.  One 32-bit word per node holds the remaining in-degree
// (bits 24-31), the out-degree (16-21) and either the single successor or the
// offset of the successor list (0-15).  The FIFO is run by the whole wave on
// uniform values (scalar control flow): every lane reads the same word (LDS
// broadcast) and writes the same value to the same address.  The next node
// comes from a register when it was released by the current step.  Returns
// false (nothing written) when the scratch is too small; node ids and list
// offsets must fit 16 bits.
template <typename SizeT>
__device__ __forceinline__ bool topsort_lds(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* scratch, int scratch_bytes,
                                            GWAMD_LDS int* sh, int lane, uint64_t* prof = nullptr,
                                            bool force_ring = false)
{
    g = as_global(g);
#ifdef GWAMD_TOPSORT_PROFILE
    const uint64_t tp0 = __builtin_amdgcn_s_memtime();
#endif
    // info[n]: a dummy word the branch-free pop of a sink decrements
    GWAMD_LDS uint32_t* info  = (GWAMD_LDS uint32_t*)(scratch);
    GWAMD_LDS uint16_t* queue = (GWAMD_LDS uint16_t*)(scratch + (n + 1) * 4);
    const int head_bytes      = ((n + 1) * 4 + (n + 1) * 2 + 15) & ~15;
    GWAMD_LDS uint16_t* edges = (GWAMD_LDS uint16_t*)(scratch + head_bytes);
    if (head_bytes > scratch_bytes || n > 65535 || n <= 0)
        return false;
    const int edge_cap = min((scratch_bytes - head_bytes) / 2, 65535);
    // staging from the HBM graph (the first kE successor slots of every node
    // are loaded with the counts; only nodes with more read the rest)
    constexpr int kTS = 4;
    constexpr int kE  = 8;
    int ebase         = 0;
    for (int v0 = 0; v0 < n; v0 += kTS * kWave)
    {
        int oc[kTS], ic[kTS], ev[kTS][kE];
#pragma unroll
        for (int u = 0; u < kTS; u++)
        {
            const int v = min(v0 + u * kWave + lane, n - 1);
            oc[u]       = int(g.out_cnt[v]);
            ic[u]       = int(g.in_cnt[v]);
#pragma unroll
            for (int e = 0; e < kE; e++)
                ev[u][e] = int(g.out_e[v * kMaxEdges + e]);
        }
#pragma unroll
        for (int u = 0; u < kTS; u++)
        {
            const int v      = v0 + u * kWave + lane;
            const bool real  = v < n;
            const int c      = real ? oc[u] : 0;
            const int listed = c >= 2 ? c : 0;
            int total        = 0;
            const int ex     = wave_excl_sum(listed, lane, total);
            if (ebase + total > edge_cap)
                return false;
            if (real)
            {
                const int o = ebase + ex;
                info[v]     = (uint32_t(ic[u]) << 24) | (uint32_t(c) << 16) |
                          uint32_t(uint16_t(c == 1 ? ev[u][0] : (c >= 2 ? o : 0)));
                if (c >= 2)
                {
#pragma unroll
                    for (int e = 0; e < kE; e++)
                        if (e < c)
                            edges[o + e] = uint16_t(ev[u][e]);
                    for (int e = kE; e < c; e++)
                        edges[o + e] = uint16_t(int(g.out_e[v * kMaxEdges + e]));
                }
            }
            ebase += total;
        }
    }
    wave_sync();
    // queued nodes' final info words next to the queue when they fit: a pop is
    // then one LDS read instead of two dependent ones
    const int qinfo_off          = (head_bytes + ebase * 2 + 15) & ~15;
    // (all n of them, or for graphs too large for that a ring of the last
    // kQRing pushes: a pop at q reads the ring while tail - q < kQRing, the
    // node word otherwise; the queue holds about the graph's width.
    // force_ring: Dims::diag bit 0, parity tests of the ring mode with a
    // 4-entry ring: ordinary windows queue 5-6 nodes at once, so they run
    // past it)
    constexpr int kQRing = 1024;
    const int qring      = force_ring ? 4 : kQRing;
    const int q_mode     = uniform((qinfo_off + (n + 1) * 4 <= scratch_bytes && !force_ring)
                                       ? 1
                                       : (qinfo_off + qring * 4 <= scratch_bytes ? 2 : 0));
    const bool use_q     = q_mode != 0;
    const uint32_t qmask = q_mode == 2 ? uint32_t(qring - 1) : 0xffffffffu;
    GWAMD_LDS uint32_t* qinfo    = (GWAMD_LDS uint32_t*)(scratch + qinfo_off);
    // sources in id order
    int k = 0;
    for (int v0 = 0; v0 < n; v0 += kWave)
    {
        const int v    = v0 + lane;
        const uint32_t vi = v < n ? info[v] : 1u << 24;
        const bool src = (vi >> 24) == 0;
        int total      = 0;
        const int ex   = wave_excl_sum(src ? 1 : 0, lane, total);
        if (src)
        {
            queue[k + ex] = uint16_t(v);
            if (use_q)
                qinfo[uint32_t(k + ex) & qmask] = vi;
        }
        k += total;
    }
    wave_sync();
#ifdef GWAMD_TOPSORT_PROFILE
    const uint64_t tp1 = __builtin_amdgcn_s_memtime();
#endif
    // FIFO (cudapoa_topsort.cuh:58-85), instantiated with and without the
    // queued info words so the loop carries no per-node mode test
    if (lane == 0)
        info[n] = 0xff000000u;
    wave_sync();
    auto fifo = [&](auto useq_tag) -> int {
        constexpr int kMode = decltype(useq_tag)::value; // 0 node words, 1 all queued words, 2 ring
        // (a VGPR value, made uniform where it is used, so the read stays in
        // flight next to the pop's own successor read).  Ring mode: every pop
        // stores at slot tail & (qring-1), released or not, so the entry at
        // qq is intact only while no position qq + qring has been written,
        // i.e. while tail - qq < qring.
        auto pop_info = [&](int qq, int tl) -> uint32_t {
            if (kMode == 1 || (kMode == 2 && tl - qq < qring))
                return qinfo[uint32_t(qq) & qmask];
            return info[int(queue[qq])];
        };
        // all queued words (kMode 1): entry q + 1 <= n is always in bounds, so
        // it is read without testing whether it is queued yet
        auto next_info = [&](int qq, int tl) -> uint32_t {
            if (kMode == 1)
                return qinfo[qq];
            return qq < tl ? pop_info(qq, tl) : 0u;
        };
        int tail       = uniform(k);
        int q          = 0;
        uint32_t vinfo = tail > 0 ? uint32_t(uniform(int(info[int(queue[0])]))) : 0u;
        while (q < tail)
        {
            // the loop state is wave-uniform; saying so keeps it in SGPRs with
            // scalar branches whatever the caller's control flow looks like
            tail      = uniform(tail);
            q         = uniform(q);
            vinfo     = uint32_t(uniform(int(vinfo)));
            const int deg = int((vinfo >> 16) & 63u);
            // The word of the next queue entry, when it is queued already, is
            // final (a queued node is never decremented again), so its read is
            // issued together with this pop's successor read.  Otherwise the
            // next node is the first one this pop releases.
            const bool have_next = q + 1 < tail;
            uint32_t nxt         = next_info(q + 1, tail);
            if (deg <= 1)
            {
                // no or one successor, without branches: a sink decrements the
                // dummy word info[n] and releases nothing; the queue / queued-
                // word stores at `tail` only count when the successor is
                // released (otherwise the slot is rewritten by the next push),
                // and writing a released node's word back is harmless (nothing
                // decrements it again, a pop reads only its degree and
                // successor bits)
                const int o       = deg == 1 ? int(vinfo & 0xffffu) : n;
                const uint32_t oi = uint32_t(uniform(int(info[o]))) - (1u << 24);
                const bool rel    = deg == 1 && (oi >> 24) == 0u;
                info[o]           = oi;
                queue[tail]       = uint16_t(o);
                if (kMode != 0)
                    qinfo[uint32_t(tail) & qmask] = oi;
                nxt = have_next ? nxt : oi;
                tail += rel ? 1 : 0;
            }
            else
            {
                // all successors at once, one per lane: children are distinct,
                // so the decrements are independent; ready ones are queued in
                // successor-slot order (cudapoa_topsort.cuh:72-83)
                // (lanes past the count repeat the last successor: they read
                // and store the same word as its lane, with the exec mask left
                // whole)
                const int off     = int(vinfo & 0xffffu);
                const bool act    = lane < deg;
                const int o       = int(edges[off + min(lane, deg - 1)]);
                const uint32_t oi = info[o] - (1u << 24);
                info[o]           = oi;
                const bool rdy       = act && (oi >> 24) == 0u;
                const uint64_t ready = __builtin_amdgcn_ballot_w64(rdy);
                if (ready)
                {
                    const int before = int(__builtin_amdgcn_mbcnt_hi(
                        uint32_t(ready >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(ready), 0u)));
                    if (rdy)
                    {
                        queue[tail + before] = uint16_t(o);
                        if (kMode != 0)
                            qinfo[uint32_t(tail + before) & qmask] = oi;
                    }
                    if (!have_next)
                        nxt = uint32_t(__builtin_amdgcn_readlane(int(oi), __builtin_ctzll(ready)));
                    tail += __popcll(ready);
                }
            }
            q++;
            vinfo = nxt;
        }
        return tail;
    };
    {
        const int tail = q_mode == 1 ? fifo(std::integral_constant<int, 1>{})
                                     : (q_mode == 2 ? fifo(std::integral_constant<int, 2>{})
                                                    : fifo(std::integral_constant<int, 0>{}));
        if (lane == 0)
            sh[0] = tail;
    }
    wave_sync();
#ifdef GWAMD_TOPSORT_PROFILE
    const uint64_t tp2 = __builtin_amdgcn_s_memtime();
#endif
    const int m = sh[0];
    for (int q = lane; q < m; q += kWave)
    {
        const int v = int(queue[q]);
        g.sorted[q] = SizeT(v);
        g.pos[v]    = SizeT(q);
    }
    wave_sync();
#ifdef GWAMD_TOPSORT_PROFILE
    if (prof)
    {
        const uint64_t tp3 = __builtin_amdgcn_s_memtime();
        prof[0] += tp1 - tp0;
        prof[1] += tp2 - tp1;
        prof[2] += tp3 - tp2;
        prof[3] += uint64_t(n);
    }
#endif
    return true;
}

// Kahn sort for graphs whose node words do not fit LDS (config C): only the
// remaining in-degrees (one byte per node) and the FIFO (u16) live in LDS,
// 3 bytes per node; the out-edge list of each popped node is read from HBM,
// all slots in one lane-parallel load issued with its count.  Same order as
// topsort_lds (successors released in slot order).  Returns false (nothing
// written) when it does not fit either.
template <typename SizeT>
__device__ __forceinline__ bool topsort_lds_big(WinGraph<SizeT> g, int n, GWAMD_LDS uint8_t* scratch,
                                                int scratch_bytes, int lane)
{
    g = as_global(g);
    n               = uniform(n);
    const int cnt_b = (n + 15) & ~15;
    if (scratch == nullptr || n <= 0 || n > 65535 || cnt_b + 2 * n > scratch_bytes)
        return false;
    GWAMD_LDS uint8_t* cnt    = scratch;
    GWAMD_LDS uint16_t* queue = (GWAMD_LDS uint16_t*)(scratch + cnt_b);
    // in-degrees and the sources in id order
    int k = 0;
    for (int v0 = 0; v0 < n; v0 += kWave)
    {
        const int v    = v0 + lane;
        const int ic   = v < n ? int(g.in_cnt[v]) : 1;
        if (v < n)
            cnt[v] = uint8_t(ic);
        const bool src = ic == 0;
        int total      = 0;
        const int ex   = wave_excl_sum(src ? 1 : 0, lane, total);
        if (src)
            queue[k + ex] = uint16_t(v);
        k += total;
    }
    wave_sync();
    int tail = uniform(k);
    for (int q = 0; q < tail; q++)
    {
        q                 = uniform(q);
        tail              = uniform(tail);
        const int v       = uniform(int(queue[q]));
        const int ov      = lane < kMaxEdges ? int(g.out_e[v * kMaxEdges + lane]) : 0;
        const int oc      = uniform(int(g.out_cnt[v]));
        const bool act    = lane < oc;
        const int c       = act ? int(cnt[ov]) - 1 : 1;
        if (act)
            cnt[ov] = uint8_t(c);
        const bool rdy       = act && c == 0;
        const uint64_t ready = __builtin_amdgcn_ballot_w64(rdy);
        if (rdy)
            queue[tail + __popcll(ready & ((uint64_t(1) << lane) - 1))] = uint16_t(ov);
        tail += __popcll(ready);
    }
    wave_sync();
    for (int q = lane; q < tail; q += kWave)
    {
        const int v = int(queue[q]);
        g.sorted[q] = SizeT(v);
        g.pos[v]    = SizeT(q);
    }
    wave_sync();
    return true;
}

// ---------------------------------------------------------------------------
// Kahn order by levels, on every wave of the workgroup (round 6).
//
// The reference's FIFO sort (cudapoa_topsort.cuh:56-85: sources in id order,
// then each popped node releases its successors in out-slot order) pops the
// nodes in increasing longest-path level from the sources (a node is released
// by its last-popped predecessor, which lies one level below it), and within
// a level in the order of (position of that releasing predecessor, the node's
// slot in its out-list); level 0 is in id order.  The releasing predecessor
// ("parent") is the highest-positioned predecessor of the level below.  So:
//   1. levels D(v) = 1 + max D(pred): every node points to one critical
//      predecessor c(v) (first guess: the one the previous read's sort found,
//      kept in `hint`, else the first in-edge), depths along c are found by
//      pointer jumping (one 32-bit LDS word per node, anc | depth << 16,
//      updated in place: any word a lane reads is a valid (ancestor, distance)
//      pair), and nodes with two or more predecessors check D(v) > D(p) for
//      every p (their in-lists cached in LDS); violators move c(v) to their
//      deepest predecessor and the jumping is redone (2-4 rounds of this per
//      read at configs B and C);
//   2. a counting sort by level (the counts and offsets live in the low halves
//      of the same words, indexed by level);
//   3. levels holding one node are placed directly; every run of consecutive
//      multi-node levels follows a one-node level (whose node is then every
//      member's parent) or starts at level 0, so each run is ordered by one
//      lane, level by level, from the previous level's positions.
// Same order as the FIFO by construction (tests/test_poa_topsort.py: the
// reference's topsort KATs, random DAGs, whole windows against the FIFO).
// LDS: 9 bytes per node + 128 (the in-list cache shares the level bucket's
// 2 bytes per node); returns false (nothing written, the caller runs the FIFO
// sort) when that does not fit, when n > 65535, when the cached in-lists
// exceed n entries, or when the checks have not converged after kLvIters (32)
// rounds.  Must be called by every thread of the workgroup (it holds
// barriers); n and n_hint must be workgroup-uniform.  hint[v] for v < n_hint:
// c(v) of the previous sort of this window (edges are never removed, so it is
// still a predecessor); the final c(v) is written back to hint[0..n).
constexpr int kLvIters  = 32;
constexpr int kLvRounds = 40;
constexpr int kLvU      = 4; // nodes per thread whose HBM loads are issued together
constexpr int kLvE      = 4; // edge slots loaded with a node's counts (more: a loop, rare)
constexpr int kLvC      = 8; // nodes per chunk of the in-order pass (their loads issued together)
#ifdef GWAMD_TS_INLINE // diagnostic builds: the sort inlined into its kernels
#define GWAMD_TS_ATTR __forceinline__
#else
#define GWAMD_TS_ATTR __noinline__
#endif
// kInst: one instantiation per calling kernel family (an out-of-line function
// is register-allocated for the most constrained of its callers; the LDS
// kernel's 4-wave diagnostic shapes would hold config B's 2-wave kernel to
// their 128 registers).
template <typename SizeT, int kInst = 0>
__device__ GWAMD_TS_ATTR bool topsort_levels(WinGraph<SizeT> g, int n, int n_prev, GWAMD_LDS uint8_t* scratch,
                                             int scratch_bytes, int tid, int nthr, SizeT* hint, int n_hint,
                                             uint64_t* prof = nullptr)
{
    // typed global pointers: the function is out of line, where the graph's
    // pointers would arrive flat, and a flat load counts against the LDS wait
    // counter too (every LDS wait would wait for the HBM loads in flight)
    GWAMD_GLB const uint16_t* g_in_cnt  = glb_of(g.in_cnt);
    GWAMD_GLB const uint16_t* g_out_cnt = glb_of(g.out_cnt);
    GWAMD_GLB const SizeT* g_in_e       = glb_of(g.in_e);
    GWAMD_GLB const SizeT* g_out_e      = glb_of(g.out_e);
    GWAMD_GLB SizeT* g_sorted           = glb_of(g.sorted);
    GWAMD_GLB SizeT* g_pos              = glb_of(g.pos);
    GWAMD_GLB SizeT* g_hint             = glb_of(hint);
    const int N8             = (n + 7) & ~7;
    const int nmw            = (n + 31) / 32; // anchor mask words
    const int acap           = max(64, N8 / 4); // anchor list entries (u16)
    const int need           = 128 + 9 * N8 + 4 * ((nmw + 3) & ~3) + 2 * acap;
    n_prev                   = min(max(n_prev, 0), n);
    if (n <= 0 || n > 65535 || need > scratch_bytes)
        return false;
#ifdef GWAMD_TOPSORT_PROFILE
    uint64_t tp = __builtin_amdgcn_s_memtime();
    auto lap    = [&](int k) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (prof && tid == 0)
            prof[k] += t - tp;
        tp = t;
    };
#else
    auto lap = [&](int) {};
#endif
    GWAMD_LDS int* ctl       = (GWAMD_LDS int*)(scratch);                     // [0..1] flags, [2] fail, [4..] wave sums
    GWAMD_LDS uint32_t* word = (GWAMD_LDS uint32_t*)(scratch + 128);          // anc | depth << 16; level counters
    GWAMD_LDS uint16_t* cc   = (GWAMD_LDS uint16_t*)(scratch + 128 + 4 * N8); // critical pred, then key, then pos
    GWAMD_LDS uint16_t* bkt  = cc + N8;                                       // in-list cache, then level buckets
    GWAMD_LDS uint8_t* meta  = (GWAMD_LDS uint8_t*)(bkt + N8);                // 0x80 multi-pred | 0x40 multi-parent | ic/slot
    GWAMD_LDS uint32_t* mask = (GWAMD_LDS uint32_t*)(meta + N8);              // anchor bits
    GWAMD_LDS uint16_t* alist = (GWAMD_LDS uint16_t*)(mask + ((nmw + 3) & ~3)); // anchors during the iterations
    const int wave           = tid / kWave;
    const int lane           = tid & (kWave - 1);
    const int nwaves         = nthr / kWave;
    // workgroup exclusive sum of one int per thread (wave sums through ctl[4..])
    auto wg_excl_sum = [&](int x, int& total) -> int {
        int wtot     = 0;
        const int ex = wave_excl_sum(x, lane, wtot);
        if (lane == 0)
            ctl[4 + wave] = wtot;
        __syncthreads();
        int before = 0;
        total      = 0;
        for (int k = 0; k < nwaves; k++)
        {
            const int t = ctl[4 + k];
            before += k < wave ? t : 0;
            total += t;
        }
        __syncthreads();
        return before + ex;
    };
    // 1a. in-degrees (coalesced); the thread's multi-predecessor in-lists are
    // cached in LDS in its node order, at an offset from a workgroup scan
    // (every per-node loop below issues the loads of kLvB nodes before their
    // stores: LDS stores and loads may alias, so one node at a time would
    // serialise a round trip per node)
    constexpr int kLvB = 8;
    int mine = 0;
    for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
    {
        int ic[kLvB];
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            ic[u] = int(g_in_cnt[min(v0 + u * nthr, n - 1)]);
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            if (v0 + u * nthr < n)
            {
                meta[v0 + u * nthr] = uint8_t((ic[u] >= 2 ? 0x80 : 0) | ic[u]);
                mine += ic[u] >= 2 ? ic[u] : 0;
            }
    }
    if (tid == 0)
    {
        ctl[0] = 0;
        ctl[1] = 0;
        ctl[2] = 0;
        ctl[3] = 0;
    }
    int ctotal          = 0;
    const int cbase     = wg_excl_sum(mine, ctotal);
    const bool cache_ok = ctotal <= N8; // uniform: else the checks read the in-lists from HBM
    // 1b. first guess of c(v) and the in-list cache: kLvU nodes per thread, the
    // counts (from LDS) and the first kLvE in-edge slots of each issued together
    {
        int cur = cbase;
        for (int v0 = tid; v0 < n; v0 += kLvU * nthr)
        {
            int ic[kLvU], hv[kLvU];
            SizeT ev[kLvU][kLvE];
#pragma unroll
            for (int u = 0; u < kLvU; u++)
            {
                const int v = min(v0 + u * nthr, n - 1);
                ic[u]       = meta[v] & 63;
                hv[u]       = v < n_hint ? int(g_hint[v]) : v;
#pragma unroll
                for (int e = 0; e < kLvE; e++)
                    ev[u][e] = e < ic[u] ? g_in_e[v * kMaxEdges + e] : SizeT(0);
            }
#pragma unroll
            for (int u = 0; u < kLvU; u++)
            {
                const int v = v0 + u * nthr;
                if (v >= n)
                    continue; // (not break: the loop must unroll, its arrays stay in registers)
                int c = v;
                if (ic[u] > 0)
                    c = hv[u] != v ? hv[u] : int(ev[u][0]);
                if (ic[u] >= 2 && cache_ok)
                {
#pragma unroll
                    for (int e = 0; e < kLvE; e++)
                        if (e < ic[u])
                            bkt[cur + e] = uint16_t(int(ev[u][e]));
                    for (int e = kLvE; e < ic[u]; e++)
                        bkt[cur + e] = uint16_t(int(g_in_e[v * kMaxEdges + e]));
                    cur += ic[u];
                }
                cc[v] = uint16_t(c);
            }
        }
    }
    __syncthreads();
    lap(0);
    int r   = 0; // flag generation: slot r & 1 holds r when some thread raised it
    bool ok = false;
    [[maybe_unused]] int rounds_total = 0; // profile counters (GWAMD_TOPSORT_PROFILE)
    [[maybe_unused]] int it_done      = 0;
    for (int it = 0; it < kLvIters; it++)
    {
        it_done = it + 1;
        // reset: every word (c(v), 1), sources (v, 0); anchor bits cleared
        for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
        {
            uint32_t c[kLvB];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
                c[u] = cc[min(v0 + u * nthr, n - 1)];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
            {
                const int v = v0 + u * nthr;
                if (v < n)
                    word[v] = c[u] | (c[u] != uint32_t(v) ? 1u << 16 : 0u);
            }
        }
        for (int k = tid; k < nmw; k += nthr)
            mask[k] = 0;
        __syncthreads();
        lap(1);
        // one pass per thread in topological order (a contiguous slice of the
        // previous read's order, then a slice of this read's new nodes in id
        // order, which follows the read): a node whose c is the node before it
        // takes that node's fresh word from a register, any other reads c's
        // word as it is (every word is a valid (ancestor, distance) pair), so
        // chains collapse in one pass; every ancestor a word ends on is marked
        // as an anchor
        {
            // the last four nodes this thread placed and their fresh words: in
            // level order a node's critical predecessor is usually one of them
            // (parallel branches interleave), so its word comes from a
            // register and the chain does not break into a new anchor
            uint32_t pv = 0xffffffffu, pw = 0, pv1 = 0xffffffffu, pw1 = 0, pv2 = 0xffffffffu, pw2 = 0,
                     pv3 = 0xffffffffu, pw3 = 0, last_mark = 0xffffffffu;
            auto seq_chunk = [&](const int(&vs)[kLvC], int cnt) {
                int cs[kLvC];
                uint32_t wc[kLvC];
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                    cs[u] = u < cnt ? int(cc[vs[u]]) : 0;
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                    wc[u] = word[cs[u]];
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                {
                    if (u >= cnt)
                        continue; // (not break: the loop must unroll, its arrays stay in registers)
                    const uint32_t v = uint32_t(vs[u]), c = uint32_t(cs[u]);
                    uint32_t w       = v; // a source keeps (v, 0)
                    if (c != v)
                    {
                        const uint32_t b = c == pv ? pw : (c == pv1 ? pw1 : (c == pv2 ? pw2 : (c == pv3 ? pw3 : wc[u])));
                        w                = (b & 0xffffu) | ((b & 0xffff0000u) + (1u << 16));
                        word[v]          = w;
                        const uint32_t a = w & 0xffffu;
                        if (a != last_mark)
                        {
                            __hip_atomic_fetch_or(&mask[a >> 5], 1u << (a & 31), __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
                            last_mark = a;
                        }
                    }
                    pv3 = pv2, pw3 = pw2;
                    pv2 = pv1, pw2 = pw1;
                    pv1 = pv, pw1 = pw;
                    pv = v, pw = w;
                }
            };
            const int ro = (n_prev + nthr - 1) / nthr;
            const int q0 = min(tid * ro, n_prev), q1 = min(q0 + ro, n_prev);
            SizeT nx[kLvC];
#pragma unroll
            for (int u = 0; u < kLvC; u++)
                nx[u] = q0 + u < q1 ? g_sorted[q0 + u] : SizeT(0);
            for (int q = q0; q < q1; q += kLvC)
            {
                int vs[kLvC];
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                    vs[u] = int(nx[u]);
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                    nx[u] = q + kLvC + u < q1 ? g_sorted[q + kLvC + u] : SizeT(0);
                seq_chunk(vs, min(kLvC, q1 - q));
            }
            pv = pv1 = pv2 = pv3 = 0xffffffffu;
            const int rn = (n - n_prev + nthr - 1) / nthr;
            const int i0 = n_prev + min(tid * rn, n - n_prev), i1 = min(i0 + rn, n);
            for (int i = i0; i < i1; i += kLvC)
            {
                int vs[kLvC];
#pragma unroll
                for (int u = 0; u < kLvC; u++)
                    vs[u] = i + u;
                seq_chunk(vs, min(kLvC, i1 - i));
            }
        }
        __syncthreads();
        lap(2);
        // the anchors as a list (batched rounds: every anchor's two reads in
        // flight together instead of one dependent pair after another), or
        // the mask walk when the list would not fit
        int na_mine = 0;
        for (int k = tid; k < nmw; k += nthr)
            na_mine += __popc(mask[k]);
        int na_total      = 0;
        const int na_base = wg_excl_sum(na_mine, na_total);
        const bool alist_ok = na_total <= acap; // uniform
        if (alist_ok)
        {
            int pos = na_base;
            for (int k = tid; k < nmw; k += nthr)
            {
                uint32_t bits = mask[k];
                while (bits)
                {
                    alist[pos++] = uint16_t(k * 32 + __builtin_ctz(bits));
                    bits &= bits - 1;
                }
            }
            __syncthreads();
        }
        // pointer jumping among the anchors only (an anchor's own word ends on
        // an anchor or a source)
        bool conv = false;
        for (int round = 0; round < kLvRounds; round++)
        {
            bool ch = false;
            if (alist_ok)
            {
                for (int i0 = tid; i0 < na_total; i0 += kLvB * nthr)
                {
                    int a[kLvB];
                    uint32_t wa[kLvB], wx[kLvB];
#pragma unroll
                    for (int u = 0; u < kLvB; u++)
                        a[u] = alist[min(i0 + u * nthr, na_total - 1)];
#pragma unroll
                    for (int u = 0; u < kLvB; u++)
                        wa[u] = word[a[u]];
#pragma unroll
                    for (int u = 0; u < kLvB; u++)
                        wx[u] = word[wa[u] & 0xffffu];
#pragma unroll
                    for (int u = 0; u < kLvB; u++)
                        if (i0 + u * nthr < na_total && (wx[u] & 0xffffu) != (wa[u] & 0xffffu))
                        {
                            word[a[u]] = (wx[u] & 0xffffu) | ((wa[u] & 0xffff0000u) + (wx[u] & 0xffff0000u));
                            ch         = true;
                        }
                }
            }
            else
                for (int k = tid; k < nmw; k += nthr)
                {
                    uint32_t bits = mask[k];
                    while (bits)
                    {
                        const int a = k * 32 + __builtin_ctz(bits);
                        bits &= bits - 1;
                        const uint32_t wa = word[a];
                        const uint32_t x  = wa & 0xffffu;
                        const uint32_t wx = word[x];
                        if ((wx & 0xffffu) != x)
                        {
                            word[a] = (wx & 0xffffu) | ((wa & 0xffff0000u) + (wx & 0xffff0000u));
                            ch      = true;
                        }
                    }
                }
            r++;
            rounds_total++;
            if (ch)
                ctl[r & 1] = r;
            __syncthreads();
            if (uniform(ctl[r & 1]) != r)
            {
                conv = true;
                break;
            }
        }
        lap(3);
#ifdef GWAMD_TOPSORT_PROFILE
        {
            int na = 0;
            for (int k = tid; k < nmw; k += nthr)
                na += __popc(mask[k]);
            __hip_atomic_fetch_add(&ctl[3], na, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#endif
        if (!conv)
            break;
        // every word one step through its (now final) anchor
        for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
        {
            uint32_t w[kLvB], wa[kLvB];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
                w[u] = word[min(v0 + u * nthr, n - 1)];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
                wa[u] = word[w[u] & 0xffffu];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
            {
                const int v = v0 + u * nthr;
                if (v < n && (wa[u] & 0xffffu) != (w[u] & 0xffffu))
                    word[v] = (wa[u] & 0xffffu) | ((w[u] & 0xffff0000u) + (wa[u] & 0xffff0000u));
            }
        }
        __syncthreads();
        lap(4);
        // check D(v) > D(p) on the nodes with several predecessors (cached
        // lists; kLvV nodes and their first kLvVE entries per batch)
        constexpr int kLvV  = 4;
        constexpr int kLvVE = 4;
        bool viol           = false;
        int cur             = cbase;
        for (int v0 = tid; v0 < n; v0 += kLvV * nthr)
        {
            int m[kLvV], D[kLvV], off[kLvV], vv[kLvV];
#pragma unroll
            for (int u = 0; u < kLvV; u++)
            {
                vv[u] = min(v0 + u * nthr, n - 1);
                m[u]  = v0 + u * nthr < n ? int(meta[vv[u]]) : 0;
                D[u]  = int(word[vv[u]] >> 16);
            }
#pragma unroll
            for (int u = 0; u < kLvV; u++)
            {
                off[u] = cur;
                cur += m[u] >= 0x80 ? (m[u] & 63) : 0;
            }
            int pe[kLvV][kLvVE], dp[kLvV][kLvVE];
#pragma unroll
            for (int u = 0; u < kLvV; u++)
#pragma unroll
                for (int e = 0; e < kLvVE; e++)
                {
                    const bool live = m[u] >= 0x80 && e < (m[u] & 63);
                    pe[u][e]        = !live ? vv[u]
                                            : (cache_ok ? int(bkt[off[u] + e]) : int(g_in_e[vv[u] * kMaxEdges + e]));
                }
#pragma unroll
            for (int u = 0; u < kLvV; u++)
#pragma unroll
                for (int e = 0; e < kLvVE; e++)
                    dp[u][e] = int(word[pe[u][e]] >> 16);
#pragma unroll
            for (int u = 0; u < kLvV; u++)
            {
                if (m[u] < 0x80)
                    continue;
                const int ic = m[u] & 63;
                int best = -1, bd = -1, ncand = 0;
#pragma unroll
                for (int e = 0; e < kLvVE; e++)
                {
                    if (e < ic)
                    {
                        if (dp[u][e] > bd)
                        {
                            bd   = dp[u][e];
                            best = pe[u][e];
                        }
                        ncand += dp[u][e] == D[u] - 1 ? 1 : 0;
                    }
                }
                for (int e = kLvVE; e < ic; e++)
                {
                    const int p = cache_ok ? int(bkt[off[u] + e]) : int(g_in_e[vv[u] * kMaxEdges + e]);
                    const int d = int(word[p] >> 16);
                    if (d > bd)
                    {
                        bd   = d;
                        best = p;
                    }
                    ncand += d == D[u] - 1 ? 1 : 0;
                }
                if (bd + 1 > D[u])
                {
                    cc[vv[u]] = uint16_t(best);
                    viol      = true;
                }
                else
                    meta[vv[u]] = uint8_t(0x80 | (ncand > 1 ? 0x40 : 0) | ic);
            }
        }
        r++;
        if (viol)
            ctl[r & 1] = r;
        __syncthreads();
        lap(4);
        if (uniform(ctl[r & 1]) != r)
        {
            ok = true;
            break;
        }
    }
    lap(4);
#ifdef GWAMD_TOPSORT_PROFILE
    if (prof && tid == 0)
    {
        prof[7] += uint64_t(rounds_total) * 1000000000ull; // (outputs time below 1e9)
        prof[8] += uint64_t(ctl[3]);                        // anchors over the iterations
        prof[9] += uint64_t(it_done);                       // iterations
    }
    (void)rounds_total;
#endif
    if (!ok)
        return false;
    // 2. counting sort by level: counts in the low halves (indexed by level),
    // exclusive offsets, then the running ends after placing the nodes
    for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
    {
        uint32_t w[kLvB];
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            w[u] = word[min(v0 + u * nthr, n - 1)];
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            if (v0 + u * nthr < n)
                word[v0 + u * nthr] = w[u] & 0xffff0000u;
    }
    __syncthreads();
    for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
    {
        uint32_t l[kLvB];
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            l[u] = word[min(v0 + u * nthr, n - 1)] >> 16;
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            if (v0 + u * nthr < n)
                __hip_atomic_fetch_add(&word[l[u]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    {
        const int per = (n + nthr - 1) / nthr;
        const int l0  = min(tid * per, n), l1 = min(l0 + per, n);
        int sum       = 0;
        for (int l = l0; l < l1; l++)
            sum += int(word[l] & 0xffffu);
        int total_unused = 0;
        int run          = wg_excl_sum(sum, total_unused);
        for (int b0 = l0; b0 < l1; b0 += kLvB)
        {
            uint32_t w[kLvB];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
                w[u] = word[min(b0 + u, l1 - 1)];
#pragma unroll
            for (int u = 0; u < kLvB; u++)
                if (b0 + u < l1)
                {
                    word[b0 + u] = (w[u] & 0xffff0000u) | uint32_t(run);
                    run += int(w[u] & 0xffffu);
                }
        }
    }
    __syncthreads();
    for (int v0 = tid; v0 < n; v0 += kLvB * nthr)
    {
        uint32_t l[kLvB], old[kLvB];
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            l[u] = word[min(v0 + u * nthr, n - 1)] >> 16;
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            old[u] = v0 + u * nthr < n ? __hip_atomic_fetch_add(&word[l[u]], 1u, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP)
                                       : 0u;
#pragma unroll
        for (int u = 0; u < kLvB; u++)
            if (v0 + u * nthr < n)
                bkt[old[u] & 0xffffu] = uint16_t(v0 + u * nthr);
    }
    __syncthreads();
    auto lv_end = [&](int l) -> int { return int(word[l] & 0xffffu); };
    auto lv_off = [&](int l) -> int { return l > 0 ? int(word[l - 1] & 0xffffu) : 0; };
    // 3a. c(v) back to the hint array; one-node levels take their position;
    // members of multi-node levels with one candidate parent (c(v), one level
    // below) find their slot in its out-list (kLvU nodes' count and first
    // kLvE out-slots issued together)
    for (int v0 = tid; v0 < n; v0 += kLvU * nthr)
    {
        int par[kLvU], oc[kLvU], lo[kLvU], le[kLvU], lvl[kLvU], mt[kLvU];
        SizeT ov[kLvU][kLvE];
        bool want[kLvU];
#pragma unroll
        for (int u = 0; u < kLvU; u++)
        {
            const int v = min(v0 + u * nthr, n - 1);
            lvl[u]      = int(word[v] >> 16);
            par[u]      = cc[v];
            mt[u]       = meta[v];
        }
#pragma unroll
        for (int u = 0; u < kLvU; u++)
        {
            lo[u]   = lv_off(lvl[u]);
            le[u]   = lv_end(lvl[u]);
            want[u] = v0 + u * nthr < n && lvl[u] > 0 && le[u] - lo[u] > 1 && (mt[u] & 0x40) == 0;
            oc[u]   = want[u] ? int(g_out_cnt[par[u]]) : 0;
#pragma unroll
            for (int e = 0; e < kLvE; e++)
                ov[u][e] = want[u] ? g_out_e[par[u] * kMaxEdges + e] : SizeT(0);
        }
#pragma unroll
        for (int u = 0; u < kLvU; u++)
        {
            const int v = v0 + u * nthr;
            if (v >= n)
                continue; // (not break: the loop must unroll, its arrays stay in registers)
            g_hint[v] = SizeT(par[u]);
            if (le[u] - lo[u] == 1)
                cc[v] = uint16_t(lo[u]);
            else if (want[u])
            {
                int slot = 0;
#pragma unroll
                for (int s = 0; s < kLvE; s++)
                    slot = (s < oc[u] && int(ov[u][s]) == v) ? s : slot;
                for (int s = kLvE; s < oc[u]; s++)
                    if (int(g_out_e[par[u] * kMaxEdges + s]) == v)
                        slot = s;
                meta[v] = uint8_t((mt[u] & 0xc0) | slot);
            }
        }
    }
    __syncthreads();
    lap(5);
    // 3b. runs of multi-node levels, one lane per run.  The key of a member
    // v of level ll: (rank of its parent in level ll-1, slot of v in the
    // parent's out-list), or v itself at level 0.
    auto key_of = [&](int v, int ll, int plo, int m, int c) -> int {
        if (ll == 0)
            return v;
        int par = c, slot = m & 63;
        if (m & 0x40)
        {
            // several predecessors one level below (about one member of a
            // multi-node level in sixty): the one placed last, from the
            // in-list and the parent's out-list in HBM
            const int ic = m & 63;
            par          = -1;
            int bp       = -1;
            for (int e = 0; e < ic; e++)
            {
                const int p = int(g_in_e[v * kMaxEdges + e]);
                if (int(word[p] >> 16) == ll - 1 && int(cc[p]) > bp)
                {
                    bp  = cc[p];
                    par = p;
                }
            }
            const int oc = int(g_out_cnt[par]);
            slot         = 0;
            for (int s = 0; s < oc; s++)
                if (int(g_out_e[par * kMaxEdges + s]) == v)
                    slot = s;
        }
        return ((int(cc[par]) - plo) << 6) | slot;
    };
    bool fail = false;
    // (code size matters as much as latency here: the scan below unrolls
    // only its loads, and the run loop exists once, so the section stays in
    // the instruction cache)
    constexpr int kLvS = 8; // levels whose bounds are loaded together by the scan
    constexpr int kLvM = 4; // members of a level kept in registers
    for (int l0 = tid; l0 < n; l0 += kLvS * nthr)
    {
        uint32_t starts = 0;
        {
            uint32_t wl[kLvS], wp[kLvS], wq[kLvS];
#pragma unroll
            for (int u = 0; u < kLvS; u++)
            {
                const int l = min(l0 + u * nthr, n - 1);
                wl[u]       = word[l];
                wp[u]       = l > 0 ? word[l - 1] : 0u;
                wq[u]       = l > 1 ? word[l - 2] : 0u;
            }
#pragma unroll
            for (int u = 0; u < kLvS; u++)
            {
                const int l  = l0 + u * nthr;
                const int lo = l > 0 ? int(wp[u] & 0xffffu) : 0;
                const int le = int(wl[u] & 0xffffu);
                const int pl = l > 1 ? int(wq[u] & 0xffffu) : 0;
                if (l < n && le - lo > 1 && (l == 0 || lo - pl <= 1))
                    starts |= 1u << u;
            }
        }
        while (starts)
        {
            const int l = l0 + __builtin_ctz(starts) * nthr;
            starts &= starts - 1;
            int lo  = lv_off(l), le = lv_end(l);
            int plo = l > 0 ? lv_off(l - 1) : 0;
            for (int ll = l;;)
            {
                const int m = le - lo;
                // members, their records and parents' positions in registers,
                // ranks by comparing the keys, when the level is small and no
                // member has several candidate parents
                int v[kLvM], mt[kLvM], c[kLvM];
                bool small = m <= kLvM && ll > 0;
                if (small)
                {
#pragma unroll
                    for (int k = 0; k < kLvM; k++)
                        v[k] = bkt[lo + min(k, m - 1)];
#pragma unroll
                    for (int k = 0; k < kLvM; k++)
                    {
                        mt[k] = meta[v[k]];
                        c[k]  = cc[v[k]];
                        small = small && (mt[k] & 0x40) == 0;
                    }
                }
                if (small)
                {
                    int key[kLvM];
#pragma unroll
                    for (int k = 0; k < kLvM; k++)
                        key[k] = ((int(cc[c[k]]) - plo) << 6) | (mt[k] & 63);
#pragma unroll
                    for (int k = 0; k < kLvM; k++)
                        fail = fail || (k < m && key[k] >= (1024 << 6));
#pragma unroll
                    for (int k = 0; k < kLvM; k++)
                    {
                        int rank = 0;
#pragma unroll
                        for (int j = 0; j < kLvM; j++)
                            rank += (j < m && key[j] < key[k]) ? 1 : 0;
                        if (k < m)
                            cc[v[k]] = uint16_t(lo + rank);
                    }
                }
                else
                {
                    // keys in place of c(v), ranks through LDS
                    for (int i = lo; i < le; i++)
                    {
                        const int vv  = bkt[i];
                        const int key = key_of(vv, ll, plo, meta[vv], cc[vv]);
                        fail          = fail || key >= (1024 << 6);
                        cc[vv]        = uint16_t(key);
                    }
                    fail = fail || m > 255;
                    for (int i = lo; i < le; i++)
                    {
                        const int vv = bkt[i];
                        const int k  = cc[vv];
                        int rank     = 0;
                        for (int j = lo; j < le; j++)
                            rank += int(cc[bkt[j]]) < k ? 1 : 0;
                        meta[vv] = uint8_t(rank);
                    }
                    for (int i = lo; i < le; i++)
                    {
                        const int vv = bkt[i];
                        cc[vv]       = uint16_t(lo + meta[vv]);
                    }
                }
                ll++;
                if (ll >= n)
                    break;
                plo = lo;
                lo  = le;
                le  = lv_end(ll);
                if (le - lo <= 1)
                    break;
            }
        }
    }
    if (fail)
        ctl[2] = 1;
    __syncthreads();
    lap(6);
    if (uniform(ctl[2]) != 0)
        return false;
    // 4. outputs
    for (int v = tid; v < n; v += nthr)
    {
        const int p = cc[v];
        if (p < n)
        {
            g_sorted[p] = SizeT(v);
            g_pos[v]    = SizeT(p);
        }
    }
    __syncthreads();
    lap(7);
    return true;
}

// ---------------------------------------------------------------------------
// Traceback move window: 128 cells around the walk whose moves are decoded
// lane-parallel, two per lane (cell t and t + 64).  Two shapes:
//  * rectangle (slope == 0): 16 rows x 8 columns, cell t = a * 8 + b at row
//    wi0 - a, column wj0 - b.  A path leaves it after ~8 diagonal steps;
//  * strip along the path (slope > 0, round 3): 16 columns, and in column b
//    the 8 rows around the line a = b * slope / 16 (cell t = b * 8 + o, row
//    wi0 - (b * slope / 16 + o - 3)); or 32 columns x 4 rows.  In topological order a
//    diagonal move usually skips rows of other branches (on config B the
//    path crosses ~1.5-2 rows per column), so the slope is the rows per
//    column of the previous window's path; a path that follows it stays in
//    the strip for up to 16 columns.
// Only the shape changes: moves, tie order and the general step are the
// same, so both shapes give the same path (parity tests run both).
constexpr int kTbSlopeMin = 4; // 0.25 rows per column

struct TbWin
{
    int wi0 = -1, wj0 = -1;
    int slope = 0; // 0: rectangle; else rows per column x 16
    int next  = 0; // slope of the next window (taken at refill(), so the
                   // decoded cells always match the geometry they were built for)
    int sh    = 3; // strip: log2 of the rows per column (3: 16 x 8, 2: 32 x 4)
    int smax  = 0; // strip: largest slope whose strip fits the code tile
    int ab    = 3; // strip rows above the line (room for horizontal moves)
    __device__ __forceinline__ int above() const { return ab; }
    __device__ __forceinline__ int cols() const { return 128 >> sh; }
    // rows above wi0 the window reaches (the tile must hold wi0 - span .. wi0)
    __device__ __forceinline__ int row_span() const
    {
        return slope ? (((cols() - 1) * slope) >> 4) + (1 << sh) - 1 - above() : 15;
    }
    __device__ __forceinline__ int col_span() const { return slope ? cols() - 1 : 7; }
    __device__ __forceinline__ int row(int t) const
    {
        return slope ? wi0 - ((((t >> sh) * slope) >> 4) + (t & ((1 << sh) - 1)) - above()) : wi0 - (t >> 3);
    }
    __device__ __forceinline__ int col(int t) const { return slope ? wj0 - (t >> sh) : wj0 - (t & 7); }
    // cell of (r, c), or -1 outside the window
    __device__ __forceinline__ int index(int r, int c) const
    {
        const int a = wi0 - r, b = wj0 - c;
        if (slope)
        {
            const int o = a - ((b * slope) >> 4) + above();
            return (uint32_t(b) < uint32_t(cols()) && uint32_t(o) < uint32_t(1 << sh)) ? (b << sh) + o : -1;
        }
        return (uint32_t(a) < 16u && uint32_t(b) < 8u) ? a * 8 + b : -1;
    }
    // next window's slope from the path the walk took through this one
    __device__ __forceinline__ void follow(int ci, int cj)
    {
        const int da = wi0 - ci, db = wj0 - cj;
        if (next && db >= 4)
            next = min(max((16 * da + db / 2) / db, kTbSlopeMin), smax);
    }
    // a new window with its corner at (i, j)
    __device__ __forceinline__ void refill(int i, int j)
    {
        slope = next;
        wi0   = i;
        wj0   = j;
    }
    // mode: the tb_rank bits (bit 1 strips, bit 2 32 x 4 strips, bits 3-5
    // rows above the line + 1, 0: default); strip windows start with the
    // slope of the whole path (rows x 16 / cols) and keep row_span() below
    // tile_rows
    __device__ __forceinline__ void init(int mode, int rows, int cols_, int tile_rows)
    {
        sh   = (mode & 4) ? 2 : 3;
        // default 3 above (16 x 8) measured best of 1-4 (profiles/r3ad_tbabove)
        ab   = ((mode >> 3) & 7) ? min(((mode >> 3) & 7) - 1, (1 << sh) - 1) : (sh == 3 ? 3 : 1);
        smax = (16 * (tile_rows - (1 << sh))) / (cols() - 1);
        next = !(mode & 2) ? 0
                           : (cols_ > 0 ? min(max((16 * rows + cols_ / 2) / cols_, kTbSlopeMin), smax) : kTbSlopeMin);
        slope = next;
    }
};

// Traceback move-window walk by pointer doubling over a TbWin window whose
// cells hold their moves packed (row << 16 | column) or kSlow when the
// general step must decide (wpk0: cell lane, wpk1: cell lane + 64).
// The scalar walk takes one cell per iteration (~350 cycles of dependent
// scalar code); here every lane finds the cell of one path step at once:
// J0 maps a cell to the next cell in the window (kX: the move leaves the
// window, a slow cell maps to itself), J^2, J^3, J^4, J^8, J^12 and J^16 are
// built in LDS (4 dependent rounds), and lane L follows step
// k = (L - cn) mod 64 by the base-4 digits of k (3 dependent reads), so one
// walk takes at most 32 steps (a longer path in the window continues in the
// next walk from the same window).  The
// steps taken are a prefix in k; each lane writes its own (eg, er) entry
// exactly as the scalar walk would have, with the flush at the 64-entry
// boundary in between.  Updates (ci, cj) to the cell after the last step, cn
// (entries) and cl (loop count, capped at bound).  kCmin: the smallest column
// that stays in the window (0 full mode, 1 banded).  Same results as the
// scalar walk by construction; parity is tested with both (GWAMD_TB_WALK).
template <int kCmin, typename Flush>
__device__ __forceinline__ void walk_window_ranked(uint32_t wpk0, uint32_t wpk1, const TbWin& G, int& ci, int& cj,
                                                   int& cn, int& cl, int bound, int lane, int& eg, int& er,
                                                   GWAMD_LDS uint8_t* scratch, Flush&& flush)
{
    constexpr uint32_t kSlow = 0xffffffffu;
    constexpr int kX         = 2 * kWave;
    constexpr int kS         = 144; // table stride (129 entries: index kX maps to itself)
    // tables: 0 J, 1 J^2, 2 J^3, 3 J^4, 4 J^8, 5 J^12, 6 J^16
    GWAMD_LDS uint8_t* J     = scratch;
    GWAMD_LDS uint32_t* W    = (GWAMD_LDS uint32_t*)(scratch + 7 * kS);
    auto next_cell = [&](int t, uint32_t nx) -> int {
        const int pi  = int(nx >> 16), pj = int(nx & 0xffffu);
        const int x   = G.index(pi, pj);
        const bool in = pi >= 1 && pj >= kCmin && x >= 0;
        return nx == kSlow ? t : (in ? x : kX);
    };
    auto put = [&](int tab, int va, int vb) {
        J[tab * kS + lane]         = uint8_t(va);
        J[tab * kS + lane + kWave] = uint8_t(vb);
    };
    const int ja = next_cell(lane, wpk0), jb = next_cell(lane + kWave, wpk1);
    wave_sync(); // the previous walk's readers are done with the tables
    put(0, ja, jb);
    W[lane]         = wpk0;
    W[lane + kWave] = wpk1;
    if (lane < 7)
        J[lane * kS + kX] = uint8_t(kX);
    wave_sync();
    const int a2 = int(J[ja]), b2 = int(J[jb]);
    put(1, a2, b2);
    wave_sync();
    const int a3 = int(J[a2]), b3 = int(J[b2]);
    const int a4 = int(J[kS + a2]), b4 = int(J[kS + b2]);
    put(2, a3, b3);
    put(3, a4, b4);
    wave_sync();
    const int a8 = int(J[3 * kS + a4]), b8 = int(J[3 * kS + b4]);
    put(4, a8, b8);
    wave_sync();
    const int a12 = int(J[3 * kS + a8]), b12 = int(J[3 * kS + b8]);
    const int a16 = int(J[4 * kS + a8]), b16 = int(J[4 * kS + b8]);
    put(5, a12, b12);
    put(6, a16, b16);
    wave_sync();
    // step k = d0 + 4 d1 + 16 d2: three dependent reads
    const int k  = (lane - cn) & (kWave - 1);
    const int d0 = k & 3, d1 = (k >> 2) & 3, d2 = (k >> 4) & 1;
    int c        = G.index(ci, cj);
    {
        const int c2 = int(J[max(d0 - 1, 0) * kS + c]);
        c            = d0 ? c2 : c;
    }
    {
        const int c2 = int(J[(d1 + 2) * kS + c]);
        c            = d1 ? c2 : c;
    }
    {
        const int c2 = int(J[6 * kS + c]);
        c            = d2 ? c2 : c;
    }
    const uint32_t nx = c < kX ? W[c] : kSlow;
    const bool taken  = k < 32 && nx != kSlow && cl + k < bound;
    const int steps   = __popcll(__builtin_amdgcn_ballot_w64(taken));
    if (steps == 0)
        return;
    const int r = G.row(c), col = G.col(c);
    const int pi = int(nx >> 16), pj = int(nx & 0xffffu);
    const int neg = r == pi ? -1 : r;
    const int ner = col == pj ? -1 : col - 1;
    const int e   = cn + k;
    const int B   = (cn | (kWave - 1)) + 1; // next 64-entry flush boundary
    if (taken && e < B)
        eg = neg, er = ner;
    if (cn + steps >= B)
    {
        flush(B);
        if (taken && e >= B)
            eg = neg, er = ner;
    }
    const int last = (cn + steps - 1) & (kWave - 1);
    ci             = __builtin_amdgcn_readlane(pi, last);
    cj             = __builtin_amdgcn_readlane(pj, last);
    cn += steps;
    cl += steps;
}

} // namespace poa
} // namespace gwamd

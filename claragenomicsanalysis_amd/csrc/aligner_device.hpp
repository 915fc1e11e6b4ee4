// Device helpers shared by the aligner kernels (aligner_kernels.hip,
// aligner_banded.hip): wave-uniform values, wave barrier, Myers letter index
// and the query pattern words in LDS.
#pragma once

#include <hip/hip_runtime.h>

#include "aligner_common.hpp"

#define GWAMD_LDS __attribute__((address_space(3)))
#define GWAMD_GLB __attribute__((address_space(1)))

namespace gwamd
{
namespace aln
{


__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uniu(uint32_t x) { return uint32_t(__builtin_amdgcn_readfirstlane(int(x))); }
__device__ __forceinline__ uint64_t uni64(uint64_t x)
{
    return uint64_t(uniu(uint32_t(x))) | (uint64_t(uniu(uint32_t(x >> 32))) << 32);
}
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// bit `lane` of a 64-bit wave mask
__device__ __forceinline__ uint32_t mask_bit(uint64_t m, uint32_t lo_or_hi_sel, int lane)
{
    const uint32_t half = lo_or_hi_sel ? uint32_t(m >> 32) : uint32_t(m);
    return __builtin_amdgcn_ubfe(half, uint32_t(lane & 31), 1u);
}

// Myers letter index of a target character: "ACTG"[(c >> 1) & 3]
// (hirschberg_myers_gpu.cu:241-244)
__device__ __forceinline__ int letter(int c) { return (c >> 1) & 3; }

// Query pattern words of the whole query: pat[k*8 + L] (L = A C T G forward,
// 4 + L reversed), bit i of word k set where query[32k+i] (resp.
// query[Q-1-(32k+i)]) equals the letter (myers_preprocess, :210-225).
// PatW: an LDS pointer, or a global one for queries whose patterns do not fit LDS.
template <typename PatW>
__device__ void build_patterns(PatW pat, const char* q, int Q, int lane)
{
    const int nw = (Q + kWordBits - 1) / kWordBits;
    const char letters[4] = {'A', 'C', 'T', 'G'};
    for (int k = lane; k < nw; k += kWave)
    {
        uint32_t f[4] = {0, 0, 0, 0}, r[4] = {0, 0, 0, 0};
        const int lim = min(Q - k * kWordBits, kWordBits);
        for (int i = 0; i < lim; i++)
        {
            const char cf = q[k * kWordBits + i];
            const char cr = q[Q - 1 - (k * kWordBits + i)];
#pragma unroll
            for (int L = 0; L < 4; L++)
            {
                f[L] |= (cf == letters[L] ? 1u : 0u) << i;
                r[L] |= (cr == letters[L] ? 1u : 0u) << i;
            }
        }
#pragma unroll
        for (int L = 0; L < 4; L++)
        {
            pat[k * 8 + L]     = f[L];
            pat[k * 8 + 4 + L] = r[L];
        }
    }
}

// Segment pattern word w for letter L: rows start at query offset `off` of the
// (forward or reversed) query (get_query_pattern, :246-268).
template <typename PatPtr>
__device__ __forceinline__ uint32_t seg_pattern(PatPtr pat, int pat_words, int off, int w, int L)
{
    const int k  = (off >> 5) + w;
    const int sh = off & 31;
    uint32_t r   = k < pat_words ? pat[k * 8 + L] : 0u;
    if (sh != 0)
    {
        r >>= sh;
        if (k + 1 < pat_words)
            r |= pat[(k + 1) * 8 + L] << (32 - sh);
    }
    return r;
}

// Target letter codes (letter(), 2 bits each, 16 per word) in LDS (or, for
// targets too long for it, in HBM).
template <typename TcW>
__device__ inline void pack_target(TcW tc, const char* t, int T, int lane)
{
    for (int k = lane; k * 16 < T; k += kWave)
    {
        uint32_t v    = 0;
        const int lim = min(T - k * 16, 16);
        for (int i = 0; i < lim; i++)
            v |= uint32_t(letter(t[k * 16 + i])) << (2 * i);
        tc[k] = v;
    }
}

template <typename TcPtr>
__device__ __forceinline__ int code_at(TcPtr tc, int idx)
{
    return int((tc[idx >> 4] >> (2 * (idx & 15))) & 3u);
}

} // namespace aln
} // namespace gwamd

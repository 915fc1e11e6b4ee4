// Dispatch of the banded POA kernel to the translation unit of the planned
// cells-per-lane value (poa_band_c<CPL>.hip, each built from poa_band.hip;
// CPL = band width / 64 for the reference's band widths 128 .. 1,024).
#include <hip/hip_runtime.h>

#include "poa_common.hpp"

#define GWAMD_BAND_DECL(N)                                                                                    \
    extern "C" hipError_t gwamd_internal_poa_band_launch_cpl##N(const gwamd::poa::Buffers*,                   \
                                                                const gwamd::poa::Dims*,                      \
                                                                const gwamd::poa::Scores*, int, int, int,     \
                                                                hipStream_t);                                 \
    extern "C" int gwamd_internal_poa_band_blocks_per_cu_cpl##N(const gwamd::poa::Dims*, int, int, int);
GWAMD_BAND_DECL(2)
GWAMD_BAND_DECL(4)
GWAMD_BAND_DECL(6)
GWAMD_BAND_DECL(8)
GWAMD_BAND_DECL(10)
GWAMD_BAND_DECL(12)
GWAMD_BAND_DECL(14)
GWAMD_BAND_DECL(16)
#undef GWAMD_BAND_DECL

// Launch of the banded kernel (called by gwamd_internal_poa_launch).
extern "C" hipError_t gwamd_internal_poa_band_launch(const gwamd::poa::Buffers* b, const gwamd::poa::Dims* d,
                                                     const gwamd::poa::Scores* sc, int score_bits, int size_bits,
                                                     int msa, hipStream_t stream)
{
    switch (d->lds_cpl)
    {
    case 2: return gwamd_internal_poa_band_launch_cpl2(b, d, sc, score_bits, size_bits, msa, stream);
    case 4: return gwamd_internal_poa_band_launch_cpl4(b, d, sc, score_bits, size_bits, msa, stream);
    case 6: return gwamd_internal_poa_band_launch_cpl6(b, d, sc, score_bits, size_bits, msa, stream);
    case 8: return gwamd_internal_poa_band_launch_cpl8(b, d, sc, score_bits, size_bits, msa, stream);
    case 10: return gwamd_internal_poa_band_launch_cpl10(b, d, sc, score_bits, size_bits, msa, stream);
    case 12: return gwamd_internal_poa_band_launch_cpl12(b, d, sc, score_bits, size_bits, msa, stream);
    case 14: return gwamd_internal_poa_band_launch_cpl14(b, d, sc, score_bits, size_bits, msa, stream);
    case 16: return gwamd_internal_poa_band_launch_cpl16(b, d, sc, score_bits, size_bits, msa, stream);
    default: return hipErrorInvalidConfiguration;
    }
}

// Resident workgroups per CU of the planned banded kernel (persistent grid).
extern "C" int gwamd_internal_poa_band_blocks_per_cu(const gwamd::poa::Dims* d, int score_bits, int size_bits, int msa)
{
    switch (d->lds_cpl)
    {
    case 2: return gwamd_internal_poa_band_blocks_per_cu_cpl2(d, score_bits, size_bits, msa);
    case 4: return gwamd_internal_poa_band_blocks_per_cu_cpl4(d, score_bits, size_bits, msa);
    case 6: return gwamd_internal_poa_band_blocks_per_cu_cpl6(d, score_bits, size_bits, msa);
    case 8: return gwamd_internal_poa_band_blocks_per_cu_cpl8(d, score_bits, size_bits, msa);
    case 10: return gwamd_internal_poa_band_blocks_per_cu_cpl10(d, score_bits, size_bits, msa);
    case 12: return gwamd_internal_poa_band_blocks_per_cu_cpl12(d, score_bits, size_bits, msa);
    case 14: return gwamd_internal_poa_band_blocks_per_cu_cpl14(d, score_bits, size_bits, msa);
    case 16: return gwamd_internal_poa_band_blocks_per_cu_cpl16(d, score_bits, size_bits, msa);
    default: return 0;
    }
}

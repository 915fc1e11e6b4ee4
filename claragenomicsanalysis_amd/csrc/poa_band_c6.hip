// Banded POA kernel, band widths with 6 cells per lane (bw 384): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 6
#include "poa_band.hip"

// Banded POA kernel, band widths with 12 cells per lane (bw 768): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 12
#include "poa_band.hip"

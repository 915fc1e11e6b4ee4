// Banded POA kernel, band widths with 10 cells per lane (bw 640): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 10
#include "poa_band.hip"

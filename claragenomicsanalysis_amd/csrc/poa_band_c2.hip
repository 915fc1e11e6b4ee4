// Banded POA kernel, band widths with 2 cells per lane (bw 128): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 2
#include "poa_band.hip"

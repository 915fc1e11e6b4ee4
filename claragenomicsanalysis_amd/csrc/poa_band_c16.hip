// Banded POA kernel, band widths with 16 cells per lane (bw 1024): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 16
#include "poa_band.hip"

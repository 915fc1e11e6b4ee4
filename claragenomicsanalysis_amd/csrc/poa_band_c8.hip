// Banded POA kernel, band widths with 8 cells per lane (bw 512): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 8
#include "poa_band.hip"

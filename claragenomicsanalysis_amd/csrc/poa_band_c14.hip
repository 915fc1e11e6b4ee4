// Banded POA kernel, band widths with 14 cells per lane (bw 896): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 14
#include "poa_band.hip"

// Banded POA kernel, band widths with 4 cells per lane (bw 256): see poa_band.hip.
#define GWAMD_BAND_TU_CPL 4
#include "poa_band.hip"

// Launchers whose MFMA kernels are still being brought up return -2 ("not implemented"); the Python
// side only calls them once ops/_backend reports the capability (see ops/attention.py, ops/nf4.py).
#include "common.h"

extern "C" int ftc_nf4_gemm(const void*, const uint8_t*, const uint8_t*, const float*, float, void*, int, int, int,
                            int, int, hipStream_t) {
  return -2;
}

// kfamd_info.hip — identity of the in-tree kernel library (used for the loud native-code check).
#include <hip/hip_runtime.h>
#include "kfamd_kernels.h"

#ifndef KFAMD_SRC_HASH
#define KFAMD_SRC_HASH "unknown"
#endif

extern "C" const char* kfamd_build_info(void) {
  return "kfamd-kernels gfx950 (MFMA bf16 GEMM 256x256 w4: 4 waves, LDS-DMA 5-slot ring; LayerNorm/RMSNorm wave-per-row) "
         "src " KFAMD_SRC_HASH ", built " __DATE__ " " __TIME__;
}

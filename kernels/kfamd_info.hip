// kfamd_info.hip — identity of the in-tree kernel library (used for the loud native-code check).
#include <hip/hip_runtime.h>
#include "kfamd_kernels.h"

extern "C" const char* kfamd_build_info(void) {
  return "kfamd-kernels gfx950 (MFMA bf16 GEMM 256x256x64 glds, LayerNorm/RMSNorm wave-per-row) "
         "built " __DATE__ " " __TIME__;
}

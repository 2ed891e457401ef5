// aa_common.hpp — constants and small device/host helpers shared by the decode kernels
// (aa_kernels.hip) and the teacher-forced training kernels (aa_train.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "adaptive_amd.h"
#include "aa_gemm.hpp"

namespace aa {

// Phase timestamps for tools/ktrace (an instrumented build only: -DAA_TS_ENABLE): thread 0 of each
// workgroup writes s_memrealtime (100 MHz) to aa_ts_buf[kernel][blockIdx.x][slot].  Empty in the
// product build.
#ifdef AA_TS_ENABLE
__device__ uint64_t* aa_ts_buf = nullptr;
__device__ __forceinline__ void aa_ts(int kid, int slot) {
  if (threadIdx.x == 0 && aa_ts_buf) {
    uint64_t* p = aa_ts_buf + ((size_t)kid * 2048 + blockIdx.x) * 16 + slot;
    p[0] = __builtin_amdgcn_s_memrealtime();
    p[8] = __builtin_amdgcn_s_memtime();  // shader clock: (memtime delta) / (realtime delta) = clock
  }
}
#define AA_TS(kid, slot) aa_ts(kid, slot)
// a value (e.g. a count) in slot 7 of the workgroup's record
#define AA_TSV(kid, v)                                                                      \
  do {                                                                                      \
    if (threadIdx.x == 0 && aa_ts_buf) aa_ts_buf[((size_t)(kid) * 2048 + blockIdx.x) * 16 + 7] = (v); \
  } while (0)
#else
#define AA_TS(kid, slot)
#define AA_TSV(kid, v)
#endif

constexpr int P = 49;          // attention width == 7x7 spatial locations (adaptive_attention.py:16-19)
constexpr int PP = 64;         // padded attention width (VWv row pitch, W_v rows)
constexpr int MAX_H = 1024;    // kernels keep h / s / u rows in LDS
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// accurate libm (expf / tanhf from the device library, no fast-math)
__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float reluf_(float x) { return x < 0.f ? 0.f : x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

}  // namespace aa

#define AA_TRY(expr)                           \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return (int)e_;      \
  } while (0)

static inline int aa_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? AA_OK : (int)e;
}
static inline bool aa_al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

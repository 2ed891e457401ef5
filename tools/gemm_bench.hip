// Standalone fp32-MFMA GEMM shape/variant micro-benchmark for gfx950 (not part of the product).
// C[M,N] = A[M,K] W[N,K]^T, fp32.  Times variants with hipEvents and checks them against variant 0.
//   hipcc -O3 --offload-arch=gfx950 -Iinclude -Iadaptive_amd/csrc tools/gemm_bench.hip -o build/gemm_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <math.h>
#include "aa_gemm.hpp"

using namespace aa;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// ---- V0: the product engine (LDS-staged A and W, 4 waves 2x2) --------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256) void g_engine(const float* A, const float* W, float* C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int MT = (M + BM - 1) / BM, NTn = N / BN;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;
  ARowMajor al{A, K, mt * BM, M};
  WRowMajor wl{W, K, nt * BN};
  floatx16 acc[BM / 64][BN / 64];
  gemm_mainloop<BM, BN>(al, wl, K / BK, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
#pragma unroll
  for (int tm = 0; tm < BM / 64; ++tm)
#pragma unroll
    for (int tn = 0; tn < BN / 64; ++tn) {
      const int col = nt * BN + wn * (BN / 2) + tn * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mt * BM + wm * (BM / 2) + tm * 32 + acc_row(r, lane);
        if (row < M) C[(int64_t)row * N + col] = acc[tm][tn][r];
      }
    }
}

// ---- V1: A block resident in LDS (BM rows x K), W streamed straight into VGPRs ---------------------
// Each wave owns whole 32-column tiles (ctiles); per ctile it walks K with a D-step register ring.
// Grid: MB row blocks x NG column groups; ctiles of a group are dealt to the 4 waves round-robin.
template <int BM, int D>
__global__ __launch_bounds__(256, 1) void g_ares(const float* A, const float* W, float* C, int M, int N, int K, int NG) {
  extern __shared__ __attribute__((aligned(16))) float As[];  // [BM][K + 4]
  const int LDA = K + 4;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, li = lane & 31, lh = lane >> 5;
  const int MB = (M + BM - 1) / BM;
  const int L = xcd_remap(blockIdx.x, MB * NG);
  const int g = L / MB, mb = L % MB;
  const int m0 = mb * BM;
  // stage A block
  for (int q = t; q < BM * K / 4; q += 256) {
    const int r = q / (K / 4), c = q % (K / 4);
    const int m = m0 + r < M ? m0 + r : M - 1;
    *reinterpret_cast<float4*>(As + r * LDA + 4 * c) = *reinterpret_cast<const float4*>(A + (int64_t)m * K + 4 * c);
  }
  __syncthreads();
  const int nct = N / 32;
  const int per = (nct + NG - 1) / NG;
  const int c0 = g * per, c1 = min(nct, c0 + per);
  const int nk = K / 32;
  for (int ct = c0 + wave; ct < c1; ct += 4) {
    const float* wrow = W + (int64_t)(ct * 32 + li) * K + 16 * lh;
    floatx16 acc[BM / 32];
#pragma unroll
    for (int tm = 0; tm < BM / 32; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][r] = 0.f;
    float4 wb[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int j = 0; j < 4; ++j) wb[d][j] = d < nk ? *reinterpret_cast<const float4*>(wrow + d * 32 + 4 * j) : make_float4(0, 0, 0, 0);
    for (int ks0 = 0; ks0 < nk; ks0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const int ks = ks0 + d;
        float4 w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = wb[d][j];
        const int kn = ks + D < nk ? ks + D : nk - 1;
#pragma unroll
        for (int j = 0; j < 4; ++j) wb[d][j] = *reinterpret_cast<const float4*>(wrow + kn * 32 + 4 * j);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float4 a[BM / 32];
#pragma unroll
          for (int tm = 0; tm < BM / 32; ++tm)
            a[tm] = *reinterpret_cast<const float4*>(As + (tm * 32 + li) * LDA + ks * 32 + 16 * lh + 4 * j);
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int tm = 0; tm < BM / 32; ++tm)
              acc[tm] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a[tm], e), f4c(w[j], e), acc[tm], 0, 0, 0);
        }
      }
    }
    const int col = ct * 32 + li;
#pragma unroll
    for (int tm = 0; tm < BM / 32; ++tm)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + tm * 32 + acc_row(r, lane);
        if (row < M) C[(int64_t)row * N + col] = acc[tm][r];
      }
  }
}

// ---- V2: compute-only ceiling: the engine's LDS-read + MFMA stream with no staging in the loop -------
template <int BM, int BN>
__global__ __launch_bounds__(256) void g_compute_only(const float* A, const float* W, float* C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  for (int i = threadIdx.x; i < Tile<BM, BN>::LDS_FLOATS; i += 256) lds[i] = A[i % 1024];
  __syncthreads();
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1, li = lane & 31, lh = lane >> 5;
  floatx16 acc[BM / 64][BN / 64];
  for (int tm = 0; tm < BM / 64; ++tm) for (int tn = 0; tn < BN / 64; ++tn) for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;
  const float* As = lds;
  const float* Ws = lds + BM * LDK;
  for (int ks = 0; ks < K / BK; ++ks) {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      float4 a[BM / 64], w[BN / 64];
#pragma unroll
      for (int tm = 0; tm < BM / 64; ++tm) a[tm] = *reinterpret_cast<const float4*>(As + (wm * (BM / 2) + tm * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
      for (int tn = 0; tn < BN / 64; ++tn) w[tn] = *reinterpret_cast<const float4*>(Ws + (wn * (BN / 2) + tn * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < BM / 64; ++tm)
#pragma unroll
          for (int tn = 0; tn < BN / 64; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a[tm], j), f4c(w[tn], j), acc[tm][tn], 0, 0, 0);
    }
  }
  float s = 0;
  for (int tm = 0; tm < BM / 64; ++tm) for (int tn = 0; tn < BN / 64; ++tn) for (int r = 0; r < 16; ++r) s += acc[tm][tn][r];
  C[blockIdx.x * 256 + threadIdx.x] = s;
}

// ---- V3: big-M weight streaming (16x16x4 f32 MFMA) ---------------------------------------------------
// WG = 4 waves; wave w owns rows [m0 + 16*RB*w, +16*RB) and all CB*16 columns of the WG's column
// group; W chunk [CB*16 cols][KC] staged in LDS (double-buffered, shared by the 4 waves); each wave
// streams its own A rows straight into VGPRs one chunk ahead.  Accumulators RB x CB of 16x16.
// K permutation per chunk: MFMA s (0..KC/4-1) takes k = (KC/4)*g + s from lane group g = lane>>4.
typedef float floatx4 __attribute__((ext_vector_type(4)));
template <int RB, int CB, int KC>
__global__ __launch_bounds__(256, 1) void g_bigm(const float* A, const float* W, float* C, int M, int N, int K) {
  constexpr int NC = CB * 16, KP = KC + 4, KG = KC / 4;  // KG = k per lane group per chunk
  constexpr int WF4 = NC * KC / 4 / 256;                 // W float4 per thread per chunk
  static_assert(NC * KC % 1024 == 0, "W chunk must split evenly over 256 threads");
  __shared__ __attribute__((aligned(16))) float Ws[2][NC * KP];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 15, lg = lane >> 4;
  const int MB = (M + 64 * RB - 1) / (64 * RB), NG = N / NC;
  const int L = xcd_remap(blockIdx.x, MB * NG);
  const int g = L / MB, mb = L % MB;  // row blocks of one column group share an XCD
  const int n0 = g * NC;
  const int rw0 = mb * 64 * RB + wave * 16 * RB;
  const float* arow[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int m = rw0 + rb * 16 + lr;
    arow[rb] = A + (int64_t)(m < M ? m : M - 1) * K + KG * lg;
  }
  floatx4 acc[RB][CB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc[rb][cb] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / KC;
  float4 ra[2][RB][KG / 4];
  float4 rw[WF4];
  auto aload = [&](int buf, int kc) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < KG / 4; ++q) ra[buf][rb][q] = *reinterpret_cast<const float4*>(arow[rb] + kc * KC + 4 * q);
  };
  auto wload = [&](int kc) {
#pragma unroll
    for (int i = 0; i < WF4; ++i) {
      const int q = t + 256 * i, c = q / (KC / 4), kq = q % (KC / 4);
      rw[i] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + c) * K + kc * KC + 4 * kq);
    }
  };
  auto wstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < WF4; ++i) {
      const int q = t + 256 * i, c = q / (KC / 4), kq = q % (KC / 4);
      *reinterpret_cast<float4*>(&Ws[buf][c * KP + 4 * kq]) = rw[i];
    }
  };
  aload(0, 0);
  wload(0);
  wstore(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) { aload(cur ^ 1, kc + 1); wload(kc + 1); }
    const float* ws = Ws[cur];
#pragma unroll
    for (int q = 0; q < KG / 4; ++q) {
      float4 w[CB];
#pragma unroll
      for (int cb = 0; cb < CB; ++cb) w[cb] = *reinterpret_cast<const float4*>(ws + (cb * 16 + lr) * KP + KG * lg + 4 * q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
          for (int cb = 0; cb < CB; ++cb)
            acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(ra[cur][rb][q], e), f4c(w[cb], e), acc[rb][cb], 0, 0, 0);
    }
    if (more) wstore(cur ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rw0 + rb * 16 + 4 * lg + r;
        if (row < M) C[(int64_t)row * N + n0 + cb * 16 + lr] = acc[rb][cb][r];
      }
}

static float frand(uint32_t& s) { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f; }

struct Shape { int M, N, K; const char* name; };

template <class F>
static float time_it(F launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1000.f / reps;
}

int main() {
  Shape shapes[] = {{512, 10240, 512, "vocab"}, {512, 2560, 1024, "lstm"}, {25088, 512, 2048, "enc_v"}};
  for (auto& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    std::vector<float> hA((size_t)M * K), hW((size_t)N * K);
    uint32_t s = 1;
    for (auto& x : hA) x = frand(s);
    for (auto& x : hW) x = frand(s);
    float *A, *W, *C0, *C1;
    CK(hipMalloc(&A, hA.size() * 4)); CK(hipMalloc(&W, hW.size() * 4));
    CK(hipMalloc(&C0, (size_t)M * N * 4)); CK(hipMalloc(&C1, (size_t)M * N * 4));
    CK(hipMemcpy(A, hA.data(), hA.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, hW.data(), hW.size() * 4, hipMemcpyHostToDevice));
    const double flop = 2.0 * M * N * K;
    std::vector<float> ref((size_t)M * N), got((size_t)M * N);
    auto check = [&](const char* tag, float us) {
      CK(hipMemcpy(got.data(), C1, got.size() * 4, hipMemcpyDeviceToHost));
      double md = 0;
      for (size_t i = 0; i < got.size(); ++i) md = fmax(md, fabs((double)got[i] - ref[i]));
      printf("%-6s %-28s %8.2f us  %6.1f TF/s  maxdiff %.3g\n", sh.name, tag, us, flop / us * 1e-6, md);
    };
    {
      auto l = [&] { hipLaunchKernelGGL((g_engine<64, 128>), dim3(((M + 63) / 64) * (N / 128)), dim3(256), 0, 0, A, W, C0, M, N, K); };
      float us = time_it(l, 20);
      CK(hipMemcpy(ref.data(), C0, ref.size() * 4, hipMemcpyDeviceToHost));
      printf("%-6s %-28s %8.2f us  %6.1f TF/s\n", sh.name, "engine 64x128 (ref)", us, flop / us * 1e-6);
    }
#define ENG(BM_, BN_)                                                                                   \
    if (N % BN_ == 0) {                                                                                 \
      auto l = [&] { hipLaunchKernelGGL((g_engine<BM_, BN_>), dim3(((M + BM_ - 1) / BM_) * (N / BN_)), dim3(256), 0, 0, A, W, C1, M, N, K); }; \
      check("engine " #BM_ "x" #BN_, time_it(l, 20));                                                  \
    }
    ENG(64, 64) ENG(128, 64) ENG(128, 128)
#define CO(BM_, BN_) { auto l = [&] { hipLaunchKernelGGL((g_compute_only<BM_, BN_>), dim3(((M + BM_ - 1) / BM_) * (N / BN_)), dim3(256), 0, 0, A, W, C1, M, N, K); }; \
      float us = time_it(l, 20); printf("%-6s %-28s %8.2f us  %6.1f TF/s (no staging)\n", sh.name, "compute-only " #BM_ "x" #BN_, us, flop / us * 1e-6); }
    CO(64, 64) CO(64, 128) CO(128, 128)
#define ARES(BM_, D_, NG_)                                                                              \
    if ((size_t)BM_ * (K + 4) * 4 <= 160 * 1024) {                                                     \
      const size_t lds = (size_t)BM_ * (K + 4) * 4;                                                    \
      CK(hipFuncSetAttribute((const void*)g_ares<BM_, D_>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
      const int MB = (M + BM_ - 1) / BM_;                                                              \
      const int NG = NG_ > 0 ? NG_ : (512 + MB - 1) / MB;                                               \
      auto l = [&] { hipLaunchKernelGGL((g_ares<BM_, D_>), dim3(MB * NG), dim3(256), lds, 0, A, W, C1, M, N, K, NG); }; \
      char tag[64]; snprintf(tag, 64, "ares BM%d D%d NG%d", BM_, D_, NG);                             \
      check(tag, time_it(l, 20));                                                                      \
    }
#define BIGM(RB_, CB_, KC_) if (N % (CB_ * 16) == 0) { \
      auto l = [&] { hipLaunchKernelGGL((g_bigm<RB_, CB_, KC_>), dim3(((M + 64 * RB_ - 1) / (64 * RB_)) * (N / (CB_ * 16))), dim3(256), 0, 0, A, W, C1, M, N, K); }; \
      check("bigm RB" #RB_ " CB" #CB_ " KC" #KC_, time_it(l, 20)); }
    BIGM(4, 5, 64) BIGM(2, 5, 64) BIGM(1, 5, 64) BIGM(4, 4, 64) BIGM(2, 8, 64) BIGM(4, 8, 32)
    if (K <= 1024) {
      ARES(32, 4, 16) ARES(64, 4, 32)
    }
    CK(hipFree(A)); CK(hipFree(W)); CK(hipFree(C0)); CK(hipFree(C1));
  }
  return 0;
}

// aa_gemm.hpp — fp32 MFMA tile engine for gfx950 (CDNA4).
//
// C[M, N] = A[M, K] · W[N, K]^T with exact-fp32 matrix cores (v_mfma_f32_32x32x2_f32: 32x32
// output block per wave-instruction, K = 2, a k-ordered fmaf chain — bit-for-bit an f32 FMA
// sequence).  The decode path must stay fp32 end to end: the smallest top-1/top-2 logit gap of
// the reference decode at B = 512 is ~8e-6 (tests/golden/manifest.json), so no bf16/xf32.
//
// Geometry: 256-thread workgroup = 4 waves in a 2 x 2 grid; a BM x BN tile, each wave owns
// (BM/2) x (BN/2) = (BM/64) x (BN/64) accumulator blocks of 32 x 32 (16 f32 regs per lane each).
// K is walked in BK = 32 steps through double-buffered LDS (row-major [row][k], +4-float pad:
// ds_read_b128 of 16 distinct rows is conflict-free because 36 = 4·9 and 9 is odd).
// Register prefetch of step k+1 is issued before the MFMAs of step k and written after them:
// one barrier per K-step.
//
// K permutation inside a step: MFMA s (s = 0..15) takes k = s from lanes 0-31 and k = 16 + s
// from lanes 32-63, so each lane reads its 16 A and 16 W values of the step as 4 x ds_read_b128.
// The accumulation order of every output element is fixed (independent of BM/BN, of the row's
// position and of the batch size): decode results are batch-invariant.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace aa {

constexpr int NT = 256;        // threads per workgroup
constexpr int BK = 32;         // K step
constexpr int LDK = BK + 4;    // LDS row pitch (floats)
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int BM, int BN>
struct Tile {
  static constexpr int TM = BM / 64;
  static constexpr int TN = BN / 64;
  static constexpr int AF4 = BM * BK / 4 / NT;   // A float4 per thread per K-step
  static constexpr int WF4 = BN * BK / 4 / NT;   // W float4 per thread per K-step
  static constexpr int STAGE = (BM + BN) * LDK;  // floats per LDS stage
  static constexpr int LDS_FLOATS = 2 * STAGE;
  static_assert(BM % 64 == 0 && BN % 64 == 0, "tile must be a multiple of 64");
  static_assert(AF4 >= 1 && WF4 >= 1, "tile too small for 256 threads");
};

__device__ __forceinline__ float f4c(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// Row of accumulator register r (0..15) of a 32x32 block, for this lane (C/D map of gfx950).
__device__ __forceinline__ int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Bijective XCD-aware remap: blocks that share an XCD (bid % 8 equal) get consecutive logical ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int x = bid & 7, slot = bid >> 3;
  const int base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + slot;
}

// Plain row-major A loader: row `r` of the tile = global row m0 + r.
struct ARowMajor {
  const float* A;
  int64_t lda;
  int m0, M;
  __device__ __forceinline__ void map(int q, int& r, int& kq) const { r = q >> 3; kq = q & 7; }
  // Rows >= M are clamped to row M-1 (a valid address) and NOT zeroed: an output row depends only
  // on its own A row, and rows >= M are never stored.  No branch and no select between the load and
  // its LDS store, so hipcc keeps every load of the K-step in flight under the MFMAs (an exec-masked
  // branch or a select per load makes it wait for each load right after issuing it).
  __device__ __forceinline__ float4 load(int /*i*/, int q, int k0) const {
    const int r = q >> 3, kq = q & 7;
    const int m = m0 + r;
    const int mc = m < M ? m : M - 1;
    return *reinterpret_cast<const float4*>(A + (int64_t)mc * lda + k0 + 4 * kq);
  }
};

// Row-major weights [N][K] (rows always valid: packed buffers are padded to the tile).
struct WRowMajor {
  const float* W;
  int64_t ldw;
  int n0;
  __device__ __forceinline__ float4 load(int q, int k0) const {
    const int r = q >> 3, kq = q & 7;
    return *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * ldw + k0 + 4 * kq);
  }
};

// Main loop: accumulates k-steps [0, nk) of the tile into acc.  `lds` holds Tile::LDS_FLOATS.
// `tid` is the thread's index inside its 256-thread group and `ks0` the first K-step, so a
// 512-thread workgroup can run two groups over the two halves of K (each with its own `lds`).
template <int BM, int BN, class AL, class WL>
__device__ __forceinline__ void gemm_mainloop(const AL& al, const WL& wl, int nk, float* lds,
                                              floatx16 (&acc)[BM / 64][BN / 64], int tid = -1, int ks0 = 0) {
  using T = Tile<BM, BN>;
  const int t = tid < 0 ? (int)threadIdx.x : tid, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
    for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tm][tn][r] = 0.f;

  float4 ra[T::AF4], rw[T::WF4];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) ra[i] = al.load(i, t + NT * i, (ks0 + ks) * BK);
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) rw[i] = wl.load(t + NT * i, (ks0 + ks) * BK);
  };
  auto lstore = [&](int buf) {
    float* As = lds + buf * T::STAGE;
    float* Ws = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) {
      int r, kq;
      al.map(t + NT * i, r, kq);
      *reinterpret_cast<float4*>(As + r * LDK + 4 * kq) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) {
      const int q = t + NT * i;
      *reinterpret_cast<float4*>(Ws + (q >> 3) * LDK + 4 * (q & 7)) = rw[i];
    }
  };

  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < nk;
    if (more) gload(ks + 1);
    const float* As = lds + buf * T::STAGE;
    const float* Ws = As + BM * LDK;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      float4 a[T::TM], w[T::TN];
#pragma unroll
      for (int tm = 0; tm < T::TM; ++tm)
        a[tm] = *reinterpret_cast<const float4*>(As + (wm * (BM / 2) + tm * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn)
        w[tn] = *reinterpret_cast<const float4*>(Ws + (wn * (BN / 2) + tn * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
          for (int tn = 0; tn < T::TN; ++tn)
            acc[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a[tm], j), f4c(w[tn], j), acc[tm][tn], 0, 0, 0);
    }
    if (more) lstore(buf ^ 1);
    __syncthreads();
  }
}

// Same pipeline, but K-step ks accumulates into partial p = ks / (nk / NP) (NP independent chains
// over contiguous K ranges, nk % NP == 0).  The caller combines the partials in a fixed tree; a
// VALU re-computation of one output (8 lanes x one chain each, then the same tree) is then
// bit-identical, which the vocab rescoring relies on.
template <int BM, int BN, int NP, class AL, class WL>
__device__ __forceinline__ void gemm_mainloop_np(const AL& al, const WL& wl, int nk, float* lds,
                                                 floatx16 (&acc)[NP][BM / 64][BN / 64]) {
  using T = Tile<BM, BN>;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < T::TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[p][tm][tn][r] = 0.f;

  float4 ra[T::AF4], rw[T::WF4];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) ra[i] = al.load(i, t + NT * i, ks * BK);
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) rw[i] = wl.load(t + NT * i, ks * BK);
  };
  auto lstore = [&](int buf) {
    float* As = lds + buf * T::STAGE;
    float* Ws = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) {
      int r, kq;
      al.map(t + NT * i, r, kq);
      *reinterpret_cast<float4*>(As + r * LDK + 4 * kq) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) {
      const int q = t + NT * i;
      *reinterpret_cast<float4*>(Ws + (q >> 3) * LDK + 4 * (q & 7)) = rw[i];
    }
  };
  const int per = nk / NP;
  gload(0);
  lstore(0);
  __syncthreads();
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    for (int k2 = 0; k2 < per; ++k2) {
      const int ks = p * per + k2;
      const int buf = ks & 1;
      const bool more = ks + 1 < nk;
      if (more) gload(ks + 1);
      const float* As = lds + buf * T::STAGE;
      const float* Ws = As + BM * LDK;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        float4 a[T::TM], w[T::TN];
#pragma unroll
        for (int tm = 0; tm < T::TM; ++tm)
          a[tm] = *reinterpret_cast<const float4*>(As + (wm * (BM / 2) + tm * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
        for (int tn = 0; tn < T::TN; ++tn)
          w[tn] = *reinterpret_cast<const float4*>(Ws + (wn * (BN / 2) + tn * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int tm = 0; tm < T::TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < T::TN; ++tn)
              acc[p][tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a[tm], j), f4c(w[tn], j), acc[p][tm][tn], 0, 0, 0);
      }
      if (more) lstore(buf ^ 1);
      __syncthreads();
    }
  }
}

// gemm_mainloop_np's arithmetic (NP chains over contiguous K ranges, each the same MFMA sequence)
// with the chains combined as they complete, in the fixed tree ((p0+p1)+(p2+p3))+((p4+p5)+(p6+p7))
// (NP = 8; a binary-counter reduction, so at most log2(NP) + 1 partial sets are live instead of NP):
// out is bit-identical to that tree over gemm_mainloop_np's partials, at a quarter of its
// accumulator registers for NP = 8 -- room for several 32 x 32 blocks per wave.
template <int BM, int BN, int NP, class AL, class WL>
__device__ __forceinline__ void gemm_mainloop_chain(const AL& al, const WL& wl, int nk, float* lds,
                                                    floatx16 (&out)[BM / 64][BN / 64]) {
  using T = Tile<BM, BN>;
  static_assert(NP == 8, "the combination tree below is written for 8 chains");
  constexpr int TM = T::TM, TN = T::TN;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  floatx16 cur[TM][TN], h0[TM][TN], h1[TM][TN], h2[TM][TN];
  float4 ra[T::AF4], rw[T::WF4];
  auto gload = [&](int ks) {
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) ra[i] = al.load(i, t + NT * i, ks * BK);
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) rw[i] = wl.load(t + NT * i, ks * BK);
  };
  auto lstore = [&](int buf) {
    float* As = lds + buf * T::STAGE;
    float* Ws = As + BM * LDK;
#pragma unroll
    for (int i = 0; i < T::AF4; ++i) {
      int r, kq;
      al.map(t + NT * i, r, kq);
      *reinterpret_cast<float4*>(As + r * LDK + 4 * kq) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < T::WF4; ++i) {
      const int q = t + NT * i;
      *reinterpret_cast<float4*>(Ws + (q >> 3) * LDK + 4 * (q & 7)) = rw[i];
    }
  };
  auto add = [](floatx16 (&d)[TM][TN], const floatx16 (&a)[TM][TN], const floatx16 (&b)[TM][TN]) {
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) d[tm][tn][r] = a[tm][tn][r] + b[tm][tn][r];
  };
  const int per = nk / NP;
  gload(0);
  lstore(0);
  __syncthreads();
#pragma unroll
  for (int p = 0; p < NP; ++p) {
#pragma unroll
    for (int tm = 0; tm < TM; ++tm)
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[tm][tn][r] = 0.f;
    for (int k2 = 0; k2 < per; ++k2) {
      const int ks = p * per + k2;
      const int buf = ks & 1;
      const bool more = ks + 1 < nk;
      if (more) gload(ks + 1);
      const float* As = lds + buf * T::STAGE;
      const float* Ws = As + BM * LDK;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        float4 a[TM], w[TN];
#pragma unroll
        for (int tm = 0; tm < TM; ++tm)
          a[tm] = *reinterpret_cast<const float4*>(As + (wm * (BM / 2) + tm * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          w[tn] = *reinterpret_cast<const float4*>(Ws + (wn * (BN / 2) + tn * 32 + li) * LDK + 16 * lh + 4 * s4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int tm = 0; tm < TM; ++tm)
#pragma unroll
            for (int tn = 0; tn < TN; ++tn)
              cur[tm][tn] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a[tm], j), f4c(w[tn], j), cur[tm][tn], 0, 0, 0);
      }
      if (more) lstore(buf ^ 1);
      __syncthreads();
    }
    // binary-counter combination: p0 -> h0; p1 -> h1 = h0 + p1; p2 -> h0; p3 -> h2 = h1 + (h0 + p3);
    // p4 -> h0; p5 -> h1 = h0 + p5; p6 -> h0; p7 -> out = h2 + (h1 + (h0 + p7))
    if (p == 0 || p == 2 || p == 4 || p == 6) {
#pragma unroll
      for (int tm = 0; tm < TM; ++tm)
#pragma unroll
        for (int tn = 0; tn < TN; ++tn) h0[tm][tn] = cur[tm][tn];
    } else if (p == 1 || p == 5) {
      add(h1, h0, cur);
    } else if (p == 3) {
      add(cur, h0, cur);
      add(h2, h1, cur);
    } else {  // p == 7
      add(cur, h0, cur);
      add(cur, h1, cur);
      add(out, h2, cur);
    }
  }
}

}  // namespace aa

// aa_kernels.hip — MI355X (gfx950) kernels and C-ABI for the adaptive-attention greedy decode
// ("Knowing When to Look"; reference: code_src/models/adaptive_attention.py,
// code_src/models/baseline_attention.py).  See DESIGN.md for the data layout and rooflines.
//
// Kernels (one launch each, all fp32):
//   encoder tail (once per batch)
//     k_avgpool    a_g = AvgPool2d(7)(A)                          baseline_attention.py:46-47
//     k_enc_v      V = relu(A^T W_a^T + b_a)   [B*49, H]           :50-51   MFMA 128x128 tiles
//     k_enc_heads  v_g | h0 | c0 = act(a_g [W_b;W_h0;W_c0]^T + b)  :53-60   MFMA 64x64
//     k_vwv        VWv = V W_v^T (step-invariant, hoisted)         adaptive_attention.py:34
//   decode step t (x T)
//     k_lstm       x_t = [embed[tok]; v_g] gathered in the A-loader; gates GEMM over [x_t; h]
//                  with the LSTM cell in the epilogue; sentinel pre-activation x_t W_x^T
//                  baseline_attention.py:151-172, adaptive_attention.py:79-80
//     k_atten      s_t, W_g h, W_s s, 49+1 tanh scores, softmax, context, beta mix, u = c_hat + h
//                  adaptive_attention.py:26-58, 83, 132 (input of mlp)
//     k_vocab      logits = u W_m^T + b_m with fused first-index argmax (64-bit key atomicMax)
//                  adaptive_attention.py:132, 201
//   k_finalize     ids [B,T] from the per-step argmax keys
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "adaptive_amd.h"
#include "aa_gemm.hpp"

namespace aa {

constexpr int P = 49;          // attention width == 7x7 spatial locations (adaptive_attention.py:16-19)
constexpr int PP = 64;         // padded attention width (VWv row pitch, W_v rows)
constexpr int MAX_H = 1024;    // k_atten keeps h and s of one row in LDS
constexpr uint64_t GOLDEN = 0x9E3779B97F4A7C15ull;

// ---------------------------------------------------------------------------------------------
// Packed weight layout (float offsets into aa_model.packed), 64-float aligned regions.
// ---------------------------------------------------------------------------------------------
struct Layout {
  int E, H, V, C;
  int NH, NHp;   // heads rows E + 2H, padded to 64
  int Vp;        // vocab rows padded to 128
  int KL, KX;    // LSTM K = 2E + H, sentinel K = 2E
  size_t enc_a_w, enc_a_b, heads_w, heads_b, wv, wg, ws, wh, embed, lstm_w, lstm_b, sent_w, mlp_w, mlp_b;
  size_t total_floats;
};

static inline size_t al64(size_t x) { return (x + 63) & ~size_t(63); }
static inline int rup(int x, int m) { return (x + m - 1) / m * m; }

static Layout make_layout(const aa_dims& d) {
  Layout L;
  L.E = d.embed; L.H = d.hidden; L.V = d.vocab; L.C = d.channels;
  L.NH = L.E + 2 * L.H; L.NHp = rup(L.NH, 64);
  L.Vp = rup(L.V, 128);
  L.KL = 2 * L.E + L.H; L.KX = 2 * L.E;
  size_t o = 0;
  auto take = [&](size_t n) { size_t r = o; o = al64(o + n); return r; };
  L.enc_a_w = take((size_t)L.H * L.C);
  L.enc_a_b = take(L.H);
  L.heads_w = take((size_t)L.NHp * L.C);
  L.heads_b = take(L.NHp);
  L.wv = take((size_t)PP * L.H);
  L.wg = take((size_t)P * L.H);
  L.ws = take((size_t)P * L.H);
  L.wh = take(PP);
  L.embed = take((size_t)L.V * L.E);
  L.lstm_w = take((size_t)4 * L.H * L.KL);
  L.lstm_b = take((size_t)4 * L.H);
  L.sent_w = take((size_t)L.H * L.KX);
  L.mlp_w = take((size_t)L.Vp * L.H);
  L.mlp_b = take(L.Vp);
  L.total_floats = o;
  return L;
}

struct MP {  // resolved device pointers of the packed weights
  const float *enc_a_w, *enc_a_b, *heads_w, *heads_b, *wv, *wg, *ws, *wh, *embed, *lstm_w, *lstm_b, *sent_w, *mlp_w, *mlp_b;
};

static MP resolve(const aa_model* m, const Layout& L) {
  const float* b = static_cast<const float*>(m->packed);
  MP p;
  p.enc_a_w = b + L.enc_a_w; p.enc_a_b = b + L.enc_a_b;
  p.heads_w = b + L.heads_w; p.heads_b = b + L.heads_b;
  p.wv = b + L.wv; p.wg = b + L.wg; p.ws = b + L.ws; p.wh = b + L.wh;
  p.embed = b + L.embed; p.lstm_w = b + L.lstm_w; p.lstm_b = b + L.lstm_b;
  p.sent_w = b + L.sent_w; p.mlp_w = b + L.mlp_w; p.mlp_b = b + L.mlp_b;
  return p;
}

// ---------------------------------------------------------------------------------------------
// small math helpers (accurate libm: expf/tanhf from the device library, no fast-math)
// ---------------------------------------------------------------------------------------------
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

// Argmax key: larger logit wins; on equal logits the smaller vocab index wins (torch max(2)[1]
// returns the first maximal index, adaptive_attention.py:201).
__device__ __forceinline__ uint64_t argmax_key(float x, int n) {
  uint32_t u = __float_as_uint(x);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((uint64_t)u << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)n);
}
__device__ __forceinline__ int64_t key_token(uint64_t k) { return (int64_t)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFu)); }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int o) {
  uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  lo = __shfl_xor(lo, o, 64);
  hi = __shfl_xor(hi, o, 64);
  return ((uint64_t)hi << 32) | lo;
}

// ---------------------------------------------------------------------------------------------
// E0: a_g[b, c] = (sum_p A[b, c, p]) / 49, sequential fp32 sum in p order (the order of ATen's
// cpu_avg_pool inner loop), one wave per 64 channels staged through LDS with 16-B loads.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_avgpool(const float* __restrict__ feats, int64_t nch, float* __restrict__ a_g) {
  __shared__ float buf[4][64 * P];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ch0 = ((int64_t)blockIdx.x * 4 + w) * 64;
  const int nhere = ch0 < nch ? (int)(nch - ch0 < 64 ? nch - ch0 : 64) : 0;
  const int nf4 = nhere * P / 4;  // nhere is a multiple of 32 -> whole float4s
  const float4* src = reinterpret_cast<const float4*>(feats + ch0 * P);
  float4* dst = reinterpret_cast<float4*>(buf[w]);
  for (int q = lane; q < nf4; q += 64) dst[q] = src[q];
  __syncthreads();
  if (lane < nhere) {
    const float* row = buf[w] + lane * P;
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += row[p];
    a_g[ch0 + lane] = s / 49.0f;
  }
}

// ---------------------------------------------------------------------------------------------
// E1: V = relu(A_rows W_a^T + b_a).  A row m = b*49 + p of the virtual [B*49, C] matrix is
// column p of image b's [C, 49] NCHW block: read straight from the feature map (no transpose
// pass), lanes over consecutive rows -> contiguous addresses.
// ---------------------------------------------------------------------------------------------
template <int BM>
struct ANCHW {
  const float* F;
  int C, m0, M;
  __device__ __forceinline__ void map(int q, int& r, int& kq) const { r = q % BM; kq = q / BM; }
  __device__ __forceinline__ float4 load(int /*i*/, int q, int k0) const {
    const int r = q % BM, kq = q / BM;
    const int m = m0 + r;
    if (m >= M) return make_float4(0.f, 0.f, 0.f, 0.f);
    const int b = m / P, p = m - b * P;
    const float* s = F + ((int64_t)b * C + k0 + 4 * kq) * P + p;
    return make_float4(s[0], s[P], s[2 * P], s[3 * P]);
  }
};

__global__ __launch_bounds__(256, 2) void k_enc_v(const float* __restrict__ feats, int B, int C, int H,
                                                  const float* __restrict__ W, const float* __restrict__ bias,
                                                  float* __restrict__ V) {
  constexpr int BM = 128, BN = 128;
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int M = B * P, MT = (M + BM - 1) / BM, NTn = H / BN;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int mt = L / NTn, nt = L % NTn;  // n fastest: the A tile is shared inside an XCD
  ANCHW<BM> al{feats, C, mt * BM, M};
  WRowMajor wl{W, C, nt * BN};
  floatx16 acc[2][2];
  gemm_mainloop<BM, BN>(al, wl, C / BK, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
#pragma unroll
  for (int tm = 0; tm < 2; ++tm)
#pragma unroll
    for (int tn = 0; tn < 2; ++tn) {
      const int col = nt * BN + wn * 64 + tn * 32 + (lane & 31);
      const float bv = bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = mt * BM + wm * 64 + tm * 32 + acc_row(r, lane);
        if (row < M) V[(int64_t)row * H + col] = reluf_(acc[tm][tn][r] + bv);
      }
    }
}

// ---------------------------------------------------------------------------------------------
// E2: heads.  [v_g | h0 | c0] = a_g · [W_b; W_h0; W_c0]^T + b, relu / tanh / tanh by column.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_enc_heads(const float* __restrict__ a_g, int B, int C, int E, int H, int NHp,
                                                   const float* __restrict__ W, const float* __restrict__ bias,
                                                   float* __restrict__ v_g, float* __restrict__ h0, float* __restrict__ c0) {
  constexpr int BM = 64, BN = 64;
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int MT = (B + BM - 1) / BM, NTn = NHp / BN;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;
  ARowMajor al{a_g, C, mt * BM, B};
  WRowMajor wl{W, C, nt * BN};
  floatx16 acc[1][1];
  gemm_mainloop<BM, BN>(al, wl, C / BK, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  const int col = nt * BN + wn * 32 + (lane & 31);
  if (col >= E + 2 * H) return;
  const float bv = bias[col];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = mt * BM + wm * 32 + acc_row(r, lane);
    if (row >= B) continue;
    const float x = acc[0][0][r] + bv;
    if (col < E) v_g[(int64_t)row * E + col] = reluf_(x);
    else if (col < E + H) h0[(int64_t)row * H + (col - E)] = tanhf(x);
    else c0[(int64_t)row * H + (col - E - H)] = tanhf(x);
  }
}

// ---------------------------------------------------------------------------------------------
// E3: VWv[m, j] = V[m, :] · W_v[j, :]  (j < 64, rows >= 49 of W_v are zero).  Step-invariant:
// the reference recomputes it every step (adaptive_attention.py:34); the values are identical.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_vwv(const float* __restrict__ V, int M, int H, const float* __restrict__ Wv,
                                             float* __restrict__ VWv) {
  constexpr int BM = 64, BN = 64;
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int mt = blockIdx.x;
  ARowMajor al{V, H, mt * BM, M};
  WRowMajor wl{Wv, H, 0};
  floatx16 acc[1][1];
  gemm_mainloop<BM, BN>(al, wl, H / BK, lds, acc);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wm = wave >> 1, wn = wave & 1;
  const int col = wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = mt * BM + wm * 32 + acc_row(r, lane);
    if (row < M) VWv[(int64_t)row * PP + col] = acc[0][0][r];
  }
}

// ---------------------------------------------------------------------------------------------
// D1: LSTM step + sentinel pre-activation.
//   A row b = x_t|h = [embed[tok_b] (E) ; v_g[b] (E) ; h_{t}[b] (H)], gathered by the A-loader
//   (K-steps never straddle a segment: E % 32 == 0).
//   N tiles 0 .. H/16-1: 64 packed columns = gates (i, f, g, o) x 16 hidden units, K = 2E + H;
//     epilogue: c' = s(f) c + s(i) tanh(g), h' = s(o) tanh(c') (torch LSTM cell, gate order i,f,g,o).
//   N tiles H/16 .. : 64 columns of x_t W_x^T (Sentinel.affine_x, K = 2E; the W_h h_{t-1} term
//     multiplies zeros while sampling, adaptive_attention.py:116-122, and is skipped).
// ---------------------------------------------------------------------------------------------
struct AGather {
  const float *embed, *vg, *h;
  int E, H, m0, M;
  int tok[2];
  __device__ __forceinline__ void map(int q, int& r, int& kq) const { r = q >> 3; kq = q & 7; }
  __device__ __forceinline__ float4 load(int i, int q, int k0) const {
    const int r = q >> 3, kq = q & 7;
    const int m = m0 + r;
    if (m >= M) return make_float4(0.f, 0.f, 0.f, 0.f);
    const float* s;
    if (k0 < E) s = embed + (int64_t)tok[i] * E + k0;
    else if (k0 < 2 * E) s = vg + (int64_t)m * E + (k0 - E);
    else s = h + (int64_t)m * H + (k0 - 2 * E);
    return *reinterpret_cast<const float4*>(s + 4 * kq);
  }
};

__global__ __launch_bounds__(256) void k_lstm(int B, int E, int H, int V, const uint64_t* __restrict__ keys_prev,
                                              const int64_t* __restrict__ tok_in, const float* __restrict__ embed,
                                              const float* __restrict__ vg, const float* __restrict__ h_in,
                                              const float* __restrict__ c_in, const float* __restrict__ lstm_w,
                                              const float* __restrict__ lstm_b, const float* __restrict__ sent_w,
                                              float* __restrict__ h_out, float* __restrict__ c_out, float* __restrict__ sx) {
  constexpr int BM = 64, BN = 64;
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int MT = (B + BM - 1) / BM, NL = H / 16, NS = H / 64, NTn = NL + NS;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;  // m fastest: a weight tile is shared inside an XCD
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  const int m0 = mt * BM;

  AGather al{embed, vg, h_in, E, H, m0, B, {0, 0}};
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + (t >> 3) + 32 * i;
    int64_t tk = 1;  // <start> (adaptive_attention.py:187-190)
    if (m < B) {
      if (keys_prev) tk = key_token(keys_prev[m]);
      else if (tok_in) tk = tok_in[m];
    }
    tk = tk < 0 ? 0 : (tk >= V ? V - 1 : tk);
    al.tok[i] = (int)tk;
  }

  floatx16 acc[1][1];
  if (nt < NL) {
    const int KL = 2 * E + H;
    WRowMajor wl{lstm_w, KL, nt * BN};
    gemm_mainloop<BM, BN>(al, wl, KL / BK, lds, acc);
    // exchange the 64x64 gate tile through LDS so one thread sees all four gates of a unit
    constexpr int CP = 68;
    float* Cs = lds;
#pragma unroll
    for (int r = 0; r < 16; ++r) Cs[(wm * 32 + acc_row(r, lane)) * CP + wn * 32 + (lane & 31)] = acc[0][0][r];
    __syncthreads();
    const int rr = t >> 2, u0 = (t & 3) * 4, m = m0 + rr;
    if (m < B) {
      const float* cr = Cs + rr * CP;
      const float* bb = lstm_b + nt * 64;
      const int j = nt * 16 + u0;
      const float4 cprev = *reinterpret_cast<const float4*>(c_in + (int64_t)m * H + j);
      float hn[4], cn[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float gi = cr[0 + u0 + q] + bb[0 + u0 + q];
        const float gf = cr[16 + u0 + q] + bb[16 + u0 + q];
        const float gg = cr[32 + u0 + q] + bb[32 + u0 + q];
        const float go = cr[48 + u0 + q] + bb[48 + u0 + q];
        const float i_ = sigmoidf_(gi), f_ = sigmoidf_(gf), g_ = tanhf(gg), o_ = sigmoidf_(go);
        const float c = f4c(cprev, q);
        cn[q] = f_ * c + i_ * g_;
        hn[q] = o_ * tanhf(cn[q]);
      }
      *reinterpret_cast<float4*>(c_out + (int64_t)m * H + j) = make_float4(cn[0], cn[1], cn[2], cn[3]);
      *reinterpret_cast<float4*>(h_out + (int64_t)m * H + j) = make_float4(hn[0], hn[1], hn[2], hn[3]);
    }
  } else {
    const int st = nt - NL, KX = 2 * E;
    WRowMajor wl{sent_w, KX, st * BN};
    gemm_mainloop<BM, BN>(al, wl, KX / BK, lds, acc);
    const int col = st * BN + wn * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = m0 + wm * 32 + acc_row(r, lane);
      if (row < B) sx[(int64_t)row * H + col] = acc[0][0][r];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// D2: adaptive attention for one row per workgroup (Atten.forward, adaptive_attention.py:26-58).
//   s     = sigmoid(x W_x^T) * tanh(c_t)                               (:79-83)
//   hg    = W_g h_t,  ss = W_s s_t                                     (:35, :45)
//   z_k   = w_h . tanh(VWv[k] + hg),  k < 49;  z_s = w_h . tanh(ss + hg)  (:38, :47)
//   alpha = softmax_49(z); beta = softmax_50([z; z_s])[49]              (:39, :51-55)
//   c_t   = sum_k alpha_k V[k];  u = beta s + (1 - beta) c_t + h_t       (:42, :56, :132)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_atten(int B, int H, const float* __restrict__ h_new, const float* __restrict__ c_new,
                                               const float* __restrict__ sx, const float* __restrict__ Vf,
                                               const float* __restrict__ VWv, const float* __restrict__ Wg,
                                               const float* __restrict__ Ws, const float* __restrict__ wh,
                                               float* __restrict__ alpha_out, int64_t alpha_ld,
                                               float* __restrict__ beta_out, int64_t beta_ld, float* __restrict__ u_out) {
  __shared__ __attribute__((aligned(16))) float sh_h[MAX_H];
  __shared__ __attribute__((aligned(16))) float sh_s[MAX_H];
  __shared__ float proj[2 * PP];
  __shared__ float zs[PP];
  __shared__ float sh_alpha[PP];
  __shared__ float sh_beta;
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float* hb = h_new + (int64_t)b * H;
  const float* cb = c_new + (int64_t)b * H;
  const float* xb = sx + (int64_t)b * H;
  for (int d = t; d < H; d += 256) {
    sh_h[d] = hb[d];
    sh_s[d] = sigmoidf_(xb[d]) * tanhf(cb[d]);
  }
  __syncthreads();
  // 98 dot products of length H: wave w takes j = w, w+4, ...; lanes cover H in float4s.
  for (int j = w; j < 2 * P; j += 4) {
    const float* wrow = j < P ? Wg + (int64_t)j * H : Ws + (int64_t)(j - P) * H;
    const float* vec = j < P ? sh_h : sh_s;
    float acc = 0.f;
    for (int d = lane * 4; d < H; d += 256) {
      const float4 a = *reinterpret_cast<const float4*>(wrow + d);
      const float4 v = *reinterpret_cast<const float4*>(vec + d);
      acc += a.x * v.x + a.y * v.y + a.z * v.z + a.w * v.w;
    }
    acc = wave_sum(acc);
    if (lane == 0) proj[j] = acc;
  }
  __syncthreads();
  // z_k (k < 49) and z_s (k == 49): lanes over j < 49
  const float* vwv = VWv + (int64_t)b * P * PP;
  const float whj = lane < P ? wh[lane] : 0.f;
  const float hgj = lane < P ? proj[lane] : 0.f;
  for (int k = w; k <= P; k += 4) {
    float term = 0.f;
    if (lane < P) {
      const float x = (k < P ? vwv[k * PP + lane] : proj[P + lane]) + hgj;
      term = whj * tanhf(x);
    }
    term = wave_sum(term);
    if (lane == 0) zs[k] = term;
  }
  __syncthreads();
  if (w == 0) {
    const float z = lane < P ? zs[lane] : -INFINITY;
    const float zsn = zs[P];
    const float m = wave_max(z);
    const float e = lane < P ? expf(z - m) : 0.f;
    const float S = wave_sum(e);
    const float a = e / S;
    if (lane < P) {
      sh_alpha[lane] = a;
      if (alpha_out) alpha_out[(int64_t)b * alpha_ld + lane] = a;
    }
    const float m2 = fmaxf(m, zsn);
    const float e2 = lane < P ? expf(z - m2) : 0.f;
    const float es = expf(zsn - m2);
    const float S2 = wave_sum(e2) + es;
    if (lane == 0) {
      const float beta = es / S2;
      sh_beta = beta;
      if (beta_out) beta_out[(int64_t)b * beta_ld] = beta;
    }
  }
  __syncthreads();
  const float beta = sh_beta;
  const float* vb = Vf + (int64_t)b * P * H;
  for (int d = t; d < H; d += 256) {
    float c = 0.f;
#pragma unroll 7
    for (int k = 0; k < P; ++k) c += sh_alpha[k] * vb[(int64_t)k * H + d];
    const float chat = beta * sh_s[d] + (1.f - beta) * c;
    u_out[(int64_t)b * H + d] = chat + sh_h[d];
  }
}

// ---------------------------------------------------------------------------------------------
// D3: logits = u W_m^T + b_m (AdaptiveBlock.mlp, adaptive_attention.py:132) with the argmax of
// sampler (:201) fused into the epilogue: per-row max over the tile's columns by 64-bit keys
// (lane shuffles, then LDS across the two column waves), one atomicMax per row per workgroup.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_vocab(int B, int H, int V, int Vp, const float* __restrict__ u,
                                               const float* __restrict__ W, const float* __restrict__ bias,
                                               float* __restrict__ scores, uint64_t* __restrict__ keys) {
  constexpr int BM = 64, BN = 128;
  __shared__ __attribute__((aligned(16))) float lds[Tile<BM, BN>::LDS_FLOATS];
  const int MT = (B + BM - 1) / BM, NTn = Vp / BN;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;
  ARowMajor al{u, H, mt * BM, B};
  WRowMajor wl{W, H, nt * BN};
  floatx16 acc[1][2];
  gemm_mainloop<BM, BN>(al, wl, H / BK, lds, acc);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  uint64_t best[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) best[r] = 0;
#pragma unroll
  for (int tn = 0; tn < 2; ++tn) {
    const int col = nt * BN + wn * 64 + tn * 32 + (lane & 31);
    const bool valid = col < V;
    const float bv = bias[col];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float x = acc[0][tn][r] + bv;
      const int row = mt * BM + wm * 32 + acc_row(r, lane);
      if (scores && valid && row < B) scores[(int64_t)row * V + col] = x;
      const uint64_t k = valid ? argmax_key(x, col) : 0ull;
      best[r] = k > best[r] ? k : best[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    uint64_t k = best[r];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) {
      const uint64_t x = shfl_xor_u64(k, o);
      k = x > k ? x : k;
    }
    best[r] = k;
  }
  uint64_t* red = reinterpret_cast<uint64_t*>(lds);  // [2 column waves][64 rows]
  if ((lane & 31) == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) red[wn * 64 + wm * 32 + acc_row(r, lane)] = best[r];
  }
  __syncthreads();
  if (t < 64) {
    const uint64_t a = red[t], c = red[64 + t];
    const int row = mt * BM + t;
    if (row < B) atomicMax(reinterpret_cast<unsigned long long*>(keys + row), (unsigned long long)(a > c ? a : c));
  }
}

__global__ void k_finalize(const uint64_t* __restrict__ keys, int B, int T, int64_t* __restrict__ ids) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * T) return;
  const int b = (int)(i / T), t = (int)(i % T);
  ids[i] = key_token(keys[(int64_t)t * B + b]);
}

// ---------------------------------------------------------------------------------------------
// packing / synthetic data
// ---------------------------------------------------------------------------------------------
// dst row r (r < dst_rows) = src row r for r < rows, zeros otherwise; cols contiguous.
__global__ void k_copy_rows(const float* __restrict__ src, int rows, int cols, float* __restrict__ dst, int dst_rows) {
  const int r = blockIdx.x;
  if (r >= dst_rows) return;
  for (int c = threadIdx.x; c < cols; c += blockDim.x)
    dst[(int64_t)r * cols + c] = (src && r < rows) ? src[(int64_t)r * cols + c] : 0.f;
}

// LSTM weights: packed row r = tile*64 + gate*16 + unit  <-  [W_ih | W_hh] row gate*H + tile*16 + unit
__global__ void k_pack_lstm(const float* __restrict__ w_ih, const float* __restrict__ w_hh, const float* __restrict__ b_ih,
                            const float* __restrict__ b_hh, int E, int H, float* __restrict__ w, float* __restrict__ bsum) {
  const int r = blockIdx.x;
  const int tile = r / 64, g = (r % 64) / 16, un = r % 16;
  const int src = g * H + tile * 16 + un;
  const int KX = 2 * E, KL = KX + H;
  for (int k = threadIdx.x; k < KX; k += blockDim.x) w[(int64_t)r * KL + k] = w_ih[(int64_t)src * KX + k];
  for (int k = threadIdx.x; k < H; k += blockDim.x) w[(int64_t)r * KL + KX + k] = w_hh[(int64_t)src * H + k];
  if (threadIdx.x == 0) bsum[r] = b_ih[src] + b_hh[src];
}

__device__ __forceinline__ uint64_t splitmix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_synth_uniform(float* __restrict__ dst, int64_t n, uint64_t key, int64_t start, double lo, double span, int plain) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t z = splitmix(key + (uint64_t)(start + i + 1) * GOLDEN);
    const double u = (double)(z >> 40) * (1.0 / 16777216.0);
    dst[i] = plain ? (float)u : (float)__dadd_rn(lo, __dmul_rn(span, u));
  }
}

}  // namespace aa

// =============================================================================================
// C-ABI
// =============================================================================================
using namespace aa;

#define AA_TRY(expr)                           \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return (int)e_;      \
  } while (0)

static int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? AA_OK : (int)e;
}

static bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// (exported functions get C linkage and default visibility from their declarations in adaptive_amd.h)

int aa_abi_version(void) { return AA_ABI_VERSION; }

const char* aa_error_string(int code) {
  switch (code) {
    case AA_OK: return "ok";
    case AA_ERR_NULL: return "a required pointer is NULL";
    case AA_ERR_DIMS: return "unsupported model dimensions (need embed%32==0, hidden%128==0, hidden<=1024, vocab>=1, channels%32==0, spatial==49)";
    case AA_ERR_SHAPE: return "bad batch size or step count";
    case AA_ERR_BUFFER: return "packed-weight or workspace buffer too small";
    case AA_ERR_ALIGN: return "a device pointer is not 16-byte aligned";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
  }
}

int aa_check_dims(const aa_dims* d) {
  if (!d) return AA_ERR_NULL;
  if (d->embed <= 0 || d->embed % 32 || d->hidden <= 0 || d->hidden % 128 || d->hidden > MAX_H || d->vocab < 1 ||
      d->channels <= 0 || d->channels % 32 || d->spatial != P)
    return AA_ERR_DIMS;
  return AA_OK;
}

size_t aa_packed_bytes(const aa_dims* d) {
  if (aa_check_dims(d) != AA_OK) return 0;
  return make_layout(*d).total_floats * sizeof(float);
}

static int check_model(const aa_model* m, Layout* L) {
  if (!m || !m->packed) return AA_ERR_NULL;
  int rc = aa_check_dims(&m->dims);
  if (rc) return rc;
  *L = make_layout(m->dims);
  if (m->packed_bytes < L->total_floats * sizeof(float)) return AA_ERR_BUFFER;
  if (((uintptr_t)m->packed & 255u) != 0) return AA_ERR_ALIGN;
  return AA_OK;
}

int aa_pack_weights(const aa_model* m, const aa_ref_weights* w, aa_stream_t stream) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  if (!w) return AA_ERR_NULL;
  const float* req[] = {w->enc_affine_a_w, w->enc_affine_a_b, w->enc_affine_b_w, w->enc_affine_b_b,
                        w->enc_affine_h0_w, w->enc_affine_h0_b, w->enc_affine_c0_w, w->enc_affine_c0_b,
                        w->embed_w, w->lstm_w_ih, w->lstm_w_hh, w->lstm_b_ih, w->lstm_b_hh,
                        w->sent_affine_x_w, w->att_affine_v_w, w->att_affine_g_w, w->att_affine_s_w,
                        w->att_affine_h_w, w->mlp_w, w->mlp_b};
  for (const float* p : req)
    if (!p) return AA_ERR_NULL;
  hipStream_t s = (hipStream_t)stream;
  float* base = static_cast<float*>(m->packed);
  const int E = L.E, H = L.H, V = L.V, C = L.C;
  AA_TRY(hipMemsetAsync(base, 0, L.total_floats * sizeof(float), s));
  auto cp = [&](const float* src, size_t off, size_t n) {
    return hipMemcpyAsync(base + off, src, n * sizeof(float), hipMemcpyDeviceToDevice, s);
  };
  AA_TRY(cp(w->enc_affine_a_w, L.enc_a_w, (size_t)H * C));
  AA_TRY(cp(w->enc_affine_a_b, L.enc_a_b, H));
  AA_TRY(cp(w->enc_affine_b_w, L.heads_w, (size_t)E * C));
  AA_TRY(cp(w->enc_affine_h0_w, L.heads_w + (size_t)E * C, (size_t)H * C));
  AA_TRY(cp(w->enc_affine_c0_w, L.heads_w + (size_t)(E + H) * C, (size_t)H * C));
  AA_TRY(cp(w->enc_affine_b_b, L.heads_b, E));
  AA_TRY(cp(w->enc_affine_h0_b, L.heads_b + E, H));
  AA_TRY(cp(w->enc_affine_c0_b, L.heads_b + E + H, H));
  AA_TRY(cp(w->att_affine_v_w, L.wv, (size_t)P * H));  // rows 49..63 stay zero
  AA_TRY(cp(w->att_affine_g_w, L.wg, (size_t)P * H));
  AA_TRY(cp(w->att_affine_s_w, L.ws, (size_t)P * H));
  AA_TRY(cp(w->att_affine_h_w, L.wh, P));
  AA_TRY(cp(w->embed_w, L.embed, (size_t)V * E));
  AA_TRY(cp(w->sent_affine_x_w, L.sent_w, (size_t)H * 2 * E));
  AA_TRY(cp(w->mlp_w, L.mlp_w, (size_t)V * H));        // rows V..Vp-1 stay zero
  AA_TRY(cp(w->mlp_b, L.mlp_b, V));
  hipLaunchKernelGGL(k_pack_lstm, dim3(4 * H), dim3(256), 0, s, w->lstm_w_ih, w->lstm_w_hh, w->lstm_b_ih,
                     w->lstm_b_hh, E, H, base + L.lstm_w, base + L.lstm_b);
  return launch_status();
}

static int encoder_launch(const Layout& L, const MP& p, const float* feats, int B, float* a_g, float* V, float* v_g,
                          float* h0, float* c0, float* VWv, hipStream_t s) {
  const int C = L.C, H = L.H, E = L.E;
  const int64_t nch = (int64_t)B * C;
  hipLaunchKernelGGL(k_avgpool, dim3((unsigned)((nch + 255) / 256)), dim3(256), 0, s, feats, nch, a_g);
  {
    const int M = B * P, MT = (M + 127) / 128, NTn = H / 128;
    hipLaunchKernelGGL(k_enc_v, dim3(MT * NTn), dim3(256), 0, s, feats, B, C, H, p.enc_a_w, p.enc_a_b, V);
  }
  {
    const int MT = (B + 63) / 64, NTn = L.NHp / 64;
    hipLaunchKernelGGL(k_enc_heads, dim3(MT * NTn), dim3(256), 0, s, a_g, B, C, E, H, L.NHp, p.heads_w, p.heads_b,
                       v_g, h0, c0);
  }
  if (VWv) {
    const int M = B * P;
    hipLaunchKernelGGL(k_vwv, dim3((M + 63) / 64), dim3(256), 0, s, V, M, H, p.wv, VWv);
  }
  return launch_status();
}

int aa_encoder_tail(const aa_model* m, const float* feats, int32_t B, float* a_g, float* V, float* v_g, float* h0,
                    float* c0, float* VWv, aa_stream_t stream) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  if (B < 0) return AA_ERR_SHAPE;
  if (B == 0) return AA_OK;
  if (!feats || !a_g || !V || !v_g || !h0 || !c0) return AA_ERR_NULL;
  if (!al16(feats) || !al16(a_g) || !al16(V) || !al16(VWv)) return AA_ERR_ALIGN;
  return encoder_launch(L, resolve(m, L), feats, B, a_g, V, v_g, h0, c0, VWv, (hipStream_t)stream);
}

// ---- workspace carving ----------------------------------------------------------------------
struct Carver {
  char* base;
  size_t off = 0;
  template <class T>
  T* take(size_t n) {
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off = (off + n * sizeof(T) + 255) & ~size_t(255);
    return p;
  }
};

struct StepWS {
  float *sx, *u, *vwv;
  uint64_t* keys;
};
static StepWS carve_step(char* base, const Layout& L, int B, size_t* bytes) {
  Carver c{base};
  StepWS w;
  w.sx = c.take<float>((size_t)B * L.H);
  w.u = c.take<float>((size_t)B * L.H);
  w.vwv = c.take<float>((size_t)B * P * PP);
  w.keys = c.take<uint64_t>((size_t)B);
  *bytes = c.off;
  return w;
}

struct DecodeWS {
  float *a_g, *V, *vwv, *vg, *h[2], *c[2], *sx, *u;
  uint64_t* keys;
};
static DecodeWS carve_decode(char* base, const Layout& L, int B, int T, size_t* bytes) {
  Carver c{base};
  DecodeWS w;
  w.a_g = c.take<float>((size_t)B * L.C);
  w.V = c.take<float>((size_t)B * P * L.H);
  w.vwv = c.take<float>((size_t)B * P * PP);
  w.vg = c.take<float>((size_t)B * L.E);
  for (int i = 0; i < 2; ++i) {
    w.h[i] = c.take<float>((size_t)B * L.H);
    w.c[i] = c.take<float>((size_t)B * L.H);
  }
  w.sx = c.take<float>((size_t)B * L.H);
  w.u = c.take<float>((size_t)B * L.H);
  w.keys = c.take<uint64_t>((size_t)T * B);
  *bytes = c.off;
  return w;
}

size_t aa_step_workspace_bytes(const aa_dims* d, int32_t B) {
  if (aa_check_dims(d) != AA_OK || B < 0) return 0;
  size_t n;
  carve_step(nullptr, make_layout(*d), B, &n);
  return n;
}

size_t aa_decode_workspace_bytes(const aa_dims* d, int32_t B, int32_t T) {
  if (aa_check_dims(d) != AA_OK || B < 0 || T < 0) return 0;
  size_t n;
  carve_decode(nullptr, make_layout(*d), B, T, &n);
  return n;
}

static void step_launch(const Layout& L, const MP& p, int B, const uint64_t* keys_prev, const int64_t* tok_in,
                        const float* V, const float* vwv, const float* vg, const float* h_in, const float* c_in,
                        float* h_out, float* c_out, float* sx, float* u, float* alpha, int64_t alpha_ld, float* beta,
                        int64_t beta_ld, float* scores, uint64_t* keys, const aa_trace* tr, int t, hipStream_t s) {
  const int E = L.E, H = L.H, Vv = L.V;
  const int MT = (B + 63) / 64;
  if (tr && tr->lstm_events) (void)hipEventRecord((hipEvent_t)tr->lstm_events[2 * t], s);
  hipLaunchKernelGGL(k_lstm, dim3(MT * (H / 16 + H / 64)), dim3(256), 0, s, B, E, H, Vv, keys_prev, tok_in, p.embed,
                     vg, h_in, c_in, p.lstm_w, p.lstm_b, p.sent_w, h_out, c_out, sx);
  if (tr && tr->lstm_events) (void)hipEventRecord((hipEvent_t)tr->lstm_events[2 * t + 1], s);
  if (tr && tr->atten_events) (void)hipEventRecord((hipEvent_t)tr->atten_events[2 * t], s);
  hipLaunchKernelGGL(k_atten, dim3(B), dim3(256), 0, s, B, H, h_out, c_out, sx, V, vwv, p.wg, p.ws, p.wh, alpha,
                     alpha_ld, beta, beta_ld, u);
  if (tr && tr->atten_events) (void)hipEventRecord((hipEvent_t)tr->atten_events[2 * t + 1], s);
  if (tr && tr->vocab_events) (void)hipEventRecord((hipEvent_t)tr->vocab_events[2 * t], s);
  hipLaunchKernelGGL(k_vocab, dim3(MT * (L.Vp / 128)), dim3(256), 0, s, B, H, Vv, L.Vp, u, p.mlp_w, p.mlp_b, scores,
                     keys);
  if (tr && tr->vocab_events) (void)hipEventRecord((hipEvent_t)tr->vocab_events[2 * t + 1], s);
}

int aa_decode_step(const aa_model* m, int32_t B, const int64_t* tokens_in, const float* V, const float* VWv,
                   const float* v_g, const float* h_in, const float* c_in, float* h_out, float* c_out, float* scores,
                   int64_t* tokens_out, float* alpha, float* beta, void* workspace, size_t workspace_bytes,
                   aa_stream_t stream) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  if (B < 0) return AA_ERR_SHAPE;
  if (B == 0) return AA_OK;
  if (!V || !v_g || !h_in || !c_in || !h_out || !c_out || !tokens_out || !workspace) return AA_ERR_NULL;
  if (!al16(V) || !al16(VWv) || !al16(v_g) || !al16(h_in) || !al16(c_in) || !al16(h_out) || !al16(c_out) ||
      !al16(workspace))
    return AA_ERR_ALIGN;
  size_t need;
  StepWS w = carve_step(static_cast<char*>(workspace), L, B, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  hipStream_t s = (hipStream_t)stream;
  const MP p = resolve(m, L);
  if (!VWv) {
    hipLaunchKernelGGL(k_vwv, dim3((B * P + 63) / 64), dim3(256), 0, s, V, B * P, L.H, p.wv, w.vwv);
    VWv = w.vwv;
  }
  AA_TRY(hipMemsetAsync(w.keys, 0, (size_t)B * sizeof(uint64_t), s));
  step_launch(L, p, B, nullptr, tokens_in, V, VWv, v_g, h_in, c_in, h_out, c_out, w.sx, w.u, alpha, P, beta, 1, scores,
              w.keys, nullptr, 0, s);
  hipLaunchKernelGGL(k_finalize, dim3((B + 255) / 256), dim3(256), 0, s, w.keys, B, 1, tokens_out);
  return launch_status();
}

int aa_greedy_decode(const aa_model* m, const float* feats, int32_t B, int32_t T, int64_t* ids, float* alpha,
                     float* beta, void* workspace, size_t workspace_bytes, const aa_trace* trace, aa_stream_t stream) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  if (B < 0 || T < 0) return AA_ERR_SHAPE;
  if (B == 0 || T == 0) return AA_OK;
  if (!feats || !ids || !workspace) return AA_ERR_NULL;
  if (!al16(feats) || !al16(workspace)) return AA_ERR_ALIGN;
  size_t need;
  DecodeWS w = carve_decode(static_cast<char*>(workspace), L, B, T, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  hipStream_t s = (hipStream_t)stream;
  const MP p = resolve(m, L);
  AA_TRY(hipMemsetAsync(w.keys, 0, (size_t)T * B * sizeof(uint64_t), s));
  if (trace && trace->encoder_events) (void)hipEventRecord((hipEvent_t)trace->encoder_events[0], s);
  rc = encoder_launch(L, p, feats, B, w.a_g, w.V, w.vg, w.h[0], w.c[0], w.vwv, s);
  if (rc) return rc;
  if (trace && trace->encoder_events) (void)hipEventRecord((hipEvent_t)trace->encoder_events[1], s);
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    step_launch(L, p, B, t ? w.keys + (size_t)(t - 1) * B : nullptr, nullptr, w.V, w.vwv, w.vg, w.h[cur], w.c[cur],
                w.h[nxt], w.c[nxt], w.sx, w.u, alpha ? alpha + (size_t)t * P : nullptr, (int64_t)T * P,
                beta ? beta + t : nullptr, T, nullptr, w.keys + (size_t)t * B, trace, t, s);
  }
  const int64_t n = (int64_t)B * T;
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w.keys, B, T, ids);
  return launch_status();
}

int aa_synth_uniform(float* dst, int64_t n, uint64_t key, int64_t start, double lo, double hi, aa_stream_t stream) {
  if (n < 0 || start < 0) return AA_ERR_SHAPE;
  if (n == 0) return AA_OK;
  if (!dst) return AA_ERR_NULL;
  const int plain = (lo == 0.0 && hi == 1.0) ? 1 : 0;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_synth_uniform, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0,
                     (hipStream_t)stream, dst, n, key, start, lo, hi - lo, plain);
  return launch_status();
}


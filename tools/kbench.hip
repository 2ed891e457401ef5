// Kernel-level timing harness (tools only, not part of the product): includes the product kernels,
// re-launches one of them `reps` times on a workspace populated by a real aa_greedy_decode, and
// returns the mean time per launch.  Variants under study live below as copies.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Iinclude \
//         tools/kbench.hip -o tools/_build/libkbench.so      (driven by tools/kbench.py)
#include "../adaptive_amd/csrc/aa_kernels.hip"
#include <stdlib.h>

using namespace aa;

namespace aa {
// VARIANTS BEGIN
template <int MODE>
__global__ __launch_bounds__(512) void kv_ls(int B, int V, const int64_t* __restrict__ tok, int tok_ld,
                                              const float* __restrict__ table,
                                              const float* __restrict__ xg, const bf16x8* __restrict__ hsp_in,
                                              const float* __restrict__ c_in, const int* __restrict__ par,
                                              const bf16x8* __restrict__ whh3,
                                              const float* __restrict__ wgs, float* __restrict__ h_out,
                                              bf16x8* __restrict__ hsp_out, float* __restrict__ c_out,
                                              float* __restrict__ s_out, float* __restrict__ part) {
  constexpr int H = 512; constexpr bool G = false;
  constexpr int BM = 64, CP = LS_CP, TS = 64 * LS_CP;
  constexpr int WSP = 100;  // 98 projection outputs padded to whole float4s
  __shared__ __attribute__((aligned(16))) float lds[8 * TS + 2 * 64 * 16 + 16 * WSP];
  constexpr int NTn = H / 16, KC = H / 16;
  const int MT = (B + BM - 1) / BM;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;  // m fastest: a weight tile is shared inside an XCD
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = mt * BM;
  float* Pt = lds;                 // [8][64][CP] partial tiles; slot 0 becomes the summed tile
  float* Hs = Pt + 8 * TS;         // [64][16] h' of the tile
  float* Ss = Hs + 64 * 16;        // [64][16] s of the tile
  float* Wsl = Ss + 64 * 16;       // [16][WSP] W_g / W_s rows (j < 49: W_g, else W_s) per unit

  // cell-epilogue mapping: thread -> row rr, units u0, u0 + 1 of the tile
  const int rr = t >> 3, u0 = (t & 7) * 2, m = m0 + rr;
  const int mc = m < B ? m : B - 1;  // rows >= B compute on row B-1 and store nothing
  const int j = nt * 16 + u0;
  // (token first, then the GEMM's first loads, then the token-dependent gathers: in-order vmcnt
  //  then waits for the token alone; the asm barriers keep the compiler from reordering the loads)
  int64_t tk = tok[(int64_t)mc * tok_ld];

  // ---- GEMM: this wave's K chunks, loads two chunks ahead ----
  constexpr int per = KC / 8;  // even for H in {256, 512, 768, 1024}
  const int kc0 = wave * per;
  const bf16x8* af0;
  const bf16x8* af1;
  int pc = mc;  // source row of c (and of h, through the fragments)
  if constexpr (G) {
    const int ra0 = m0 + (lane & 31), ra1 = ra0 + 32;
    const int p0 = par[ra0 < B ? ra0 : B - 1], p1 = par[ra1 < B ? ra1 : B - 1];
    const int hl = 32 * (lane >> 5);
    af0 = hsp_in + (size_t)(p0 >> 5) * KC * 3 * 64 + (p0 & 31) + hl;
    af1 = hsp_in + (size_t)(p1 >> 5) * KC * 3 * 64 + (p1 & 31) + hl;
    pc = par[mc];
  } else {
    af0 = hsp_in + (size_t)(m0 / 32) * KC * 3 * 64 + lane;
    af1 = af0 + (size_t)KC * 3 * 64;
  }
  const bf16x8* wf0 = whh3 + (size_t)(nt * 2) * KC * 3 * 64 + lane;
  const bf16x8* wf1 = wf0 + (size_t)KC * 3 * 64;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
  bf16x8 fa[2][2][3], fw[2][2][3];  // [slot][block][plane]
  auto load = [&](int slot, int kc) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const size_t o = ((size_t)kc * 3 + q) * 64;
      fa[slot][0][q] = af0[o];
      fa[slot][1][q] = af1[o];
      fw[slot][0][q] = wf0[o];
      fw[slot][1][q] = wf1[o];
    }
  };
  const int last = kc0 + per - 1;
  asm volatile("" ::: "memory");
  load(0, kc0);
  load(1, kc0 + 1 < last ? kc0 + 1 : last);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  // epilogue gathers behind the first GEMM loads: token -> table row, x_g, c, W_g/W_s slice
  float2 ta[4], xa[4], sa, sb, cprev;
  float4 wsv;
  {
    tk = tk < 0 ? 0 : (tk >= V ? V - 1 : tk);
    const int N5 = 5 * H;
    const float* trow = table + tk * N5;
    const float* xrow = xg + (int64_t)mc * N5;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      ta[g] = *reinterpret_cast<const float2*>(trow + nt * 64 + g * 16 + u0);
      xa[g] = *reinterpret_cast<const float2*>(xrow + nt * 64 + g * 16 + u0);
    }
    sa = *reinterpret_cast<const float2*>(trow + 4 * H + j);
    sb = *reinterpret_cast<const float2*>(xrow + 4 * H + j);
    cprev = *reinterpret_cast<const float2*>(c_in + (int64_t)pc * H + j);
    // W_g / W_s slice: wgs[tile] is [98][16] (j-major); thread t < 392 takes float4 t
    const float4* src = reinterpret_cast<const float4*>(wgs + (int64_t)nt * 2 * P * 16);
    wsv = src[t < 2 * P * 4 ? t : 2 * P * 4 - 1];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < per; i += 2) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) if (MODE != 1) x3_step(acc[a][c], fa[d][a], fw[d][c]); else acc[a][c][0] += fa[d][a][0][0] == fw[d][c][0][0] ? 1.f : 0.f;
      const int nk = kc0 + i + d + 2;
      load(d, nk < last ? nk : last);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // ---- partial tiles -> LDS, fixed-tree sum into slot 0 ----
  {
    float* dst = Pt + wave * TS;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(a * 32 + acc_row(r, lane)) * CP + c * 32 + (lane & 31)] = acc[a][c][r];
  }
  {  // transpose the W_g / W_s slice to [unit][j] (j = 98, 99 are zero)
    const int jj = t >> 2, uq = (t & 3) * 4;
    if (t < 2 * P * 4) {
      Wsl[(uq + 0) * WSP + jj] = wsv.x; Wsl[(uq + 1) * WSP + jj] = wsv.y;
      Wsl[(uq + 2) * WSP + jj] = wsv.z; Wsl[(uq + 3) * WSP + jj] = wsv.w;
    } else if (t < 2 * P * 4 + 32) {
      const int z = t - 2 * P * 4;  // 32 zeros: j = 98, 99 for 16 units
      Wsl[(z >> 1) * WSP + 2 * P + (z & 1)] = 0.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 512 threads x 2 float4 = the 64 x 64 tile
    const int q = t + 512 * i, r = q >> 4, c4 = (q & 15) * 4;
    const float* sp = Pt + r * CP + c4;
    float4 v[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) v[w] = *reinterpret_cast<const float4*>(sp + (MODE == 3 ? 0 : w) * TS);
    float4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float s01 = f4c(v[0], e) + f4c(v[1], e), s23 = f4c(v[2], e) + f4c(v[3], e);
      const float s45 = f4c(v[4], e) + f4c(v[5], e), s67 = f4c(v[6], e) + f4c(v[7], e);
      (&o.x)[e] = (s01 + s23) + (s45 + s67);
    }
    *reinterpret_cast<float4*>(Pt + r * CP + c4) = o;
  }
  __syncthreads();
  {
    const float* cr = Pt + rr * CP;
    float hn[2], cn[2], sn[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const float gi = cr[0 + u0 + q] + ((&ta[0].x)[q] + (&xa[0].x)[q]);
      const float gf = cr[16 + u0 + q] + ((&ta[1].x)[q] + (&xa[1].x)[q]);
      const float gg = cr[32 + u0 + q] + ((&ta[2].x)[q] + (&xa[2].x)[q]);
      const float go = cr[48 + u0 + q] + ((&ta[3].x)[q] + (&xa[3].x)[q]);
      const float i_ = sigmoidf_(gi), f_ = sigmoidf_(gf), g_ = tanhf(gg), o_ = sigmoidf_(go);
      cn[q] = f_ * (&cprev.x)[q] + i_ * g_;
      const float tc = tanhf(cn[q]);
      hn[q] = o_ * tc;
      sn[q] = sigmoidf_((&sa.x)[q] + (&sb.x)[q]) * tc;
    }
    *reinterpret_cast<float2*>(Hs + rr * 16 + u0) = make_float2(hn[0], hn[1]);
    *reinterpret_cast<float2*>(Ss + rr * 16 + u0) = make_float2(sn[0], sn[1]);
    if (m < B) {
      *reinterpret_cast<float2*>(c_out + (int64_t)m * H + j) = make_float2(cn[0], cn[1]);
      *reinterpret_cast<float2*>(h_out + (int64_t)m * H + j) = make_float2(hn[0], hn[1]);
      *reinterpret_cast<float2*>(s_out + (int64_t)m * H + j) = make_float2(sn[0], sn[1]);
      if (hsp_out) {
        // next step's A fragments: k = j.. in chunk nt, lane (m % 32) + 32 * (u0 / 8), elements u0 % 8..
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        bf16x2 p0, p1, p2;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          __bf16 x0, x1, x2;
          split3(hn[q], x0, x1, x2);
          p0[q] = x0; p1[q] = x1; p2[q] = x2;
        }
        bf16x8* o = hsp_out + ((size_t)((m >> 5) * KC + nt) * 3) * 64 + (m & 31) + 32 * (u0 >> 3);
        const int e = u0 & 7;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o) + e) = p0;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o + 64) + e) = p1;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o + 128) + e) = p2;
      }
    }
  }
  __syncthreads();
  // partial projections, four outputs j = 4 jq .. 4 jq + 3 of one row per task (float4 store):
  // part[row][tile][j] = sum_{u < 16} (j < 49 ? h'_u : s_u) W[j][u], fma chain in u order
  for (int task = t; task < (MODE == 2 ? 0 : BM * (WSP / 4)); task += 512) {
    const int r = task / (WSP / 4), jq = task % (WSP / 4);
    const int mr = m0 + r;
    if (mr < B) {
      float4 hv[4], sv[4];
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4) {
        hv[u4] = *reinterpret_cast<const float4*>(Hs + r * 16 + 4 * u4);
        sv[u4] = *reinterpret_cast<const float4*>(Ss + r * 16 + 4 * u4);
      }
      float acc4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float4 wv = *reinterpret_cast<const float4*>(Wsl + u * WSP + 4 * jq);
        const float hu = f4c(hv[u >> 2], u & 3), su = f4c(sv[u >> 2], u & 3);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc4[e] = __builtin_fmaf(4 * jq + e < P ? hu : su, f4c(wv, e), acc4[e]);
      }
      *reinterpret_cast<float4*>(part + ((int64_t)mr * NTn + nt) * PART + 4 * jq) =
          make_float4(acc4[0], acc4[1], acc4[2], acc4[3]);
    }
  }
}
template <int H, int MODE>
__global__ __launch_bounds__(512) void kv_at(int B, int kdiv, const float* __restrict__ h_new,
                                                const float* __restrict__ s_new, const float* __restrict__ part,
                                                const float* __restrict__ Vf, const float* __restrict__ VWv,
                                                const float* __restrict__ wh, float* __restrict__ alpha_out,
                                                int64_t alpha_ld, float* __restrict__ beta_out, int64_t beta_ld,
                                                float* __restrict__ u_out, uint16_t* __restrict__ ub_out,
                                                float* __restrict__ unorm, bf16x8* __restrict__ ub3_out) {
  constexpr int DPT = H / 512, NT16 = H / 16, NG = NT16 / 4;
  __shared__ float red[4][128];
  __shared__ float proj[PART];
  __shared__ float zs[PP];
  __shared__ float sh_alpha[PP];
  __shared__ float sh_beta;
  __shared__ float sh_norm[8];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int b = blockIdx.x;
  const int img = kdiv == 1 ? b : b / kdiv;
  // loads, oldest first in the order they are consumed; clamped addresses, no branches
  const int grp = t >> 7, jp = t & 127, jpc = jp < 2 * P ? jp : 2 * P - 1;
  float pv[NG];
  {
    const float* pp = part + ((int64_t)b * NT16 + grp) * PART + jpc;
#pragma unroll
    for (int i = 0; i < NG; ++i) pv[i] = pp[(int64_t)4 * i * PART];
  }
  const int k = t >> 3, q = t & 7;
  const int kc = k < P ? k : P - 1;
  const float* vw = VWv + ((int64_t)img * P + kc) * PP;
  float vwr[7], whr[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int j = q + 8 * i < P ? q + 8 * i : P - 1;
    vwr[i] = vw[j];
    whr[i] = q + 8 * i < P ? wh[j] : 0.f;
  }
  const float* vb = Vf + (int64_t)img * P * H;
  float hv[DPT], sv[DPT];
  if (MODE >= 2) {
#pragma unroll
    for (int i = 0; i < DPT; ++i) {
      hv[i] = h_new[(int64_t)b * H + t + 512 * i];
      sv[i] = s_new[(int64_t)b * H + t + 512 * i];
    }
    if (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float vv[DPT][P];
#pragma unroll
  for (int i = 0; i < DPT; ++i)
#pragma unroll
    for (int kk = 0; kk < P; ++kk) vv[i][kk] = MODE == 1 ? (float)(kk + t) * 1e-3f : vb[(int64_t)kk * H + t + 512 * i];
  if (MODE < 2) {
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    hv[i] = h_new[(int64_t)b * H + t + 512 * i];
    sv[i] = s_new[(int64_t)b * H + t + 512 * i];
  }
  }
  // 1) projections: tile partials in four fixed groups (tiles grp, grp + 4, ...), groups combined
  {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < NG; ++i) a += pv[i];
    red[grp][jp] = a;
  }
  __syncthreads();
  if (t < 2 * P) proj[t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  __syncthreads();
  // 2) scores: item k (0..49) by 8 lanes, j = q + 8i
  {
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const int j = q + 8 * i < P ? q + 8 * i : P - 1;
      const float x = (k < P ? vwr[i] : proj[P + j]) + proj[j];
      z = __builtin_fmaf(whr[i], tanhf(x), z);
    }
    z = z + __shfl_xor(z, 1, 64);
    z = z + __shfl_xor(z, 2, 64);
    z = z + __shfl_xor(z, 4, 64);
    if (q == 0 && k <= P) zs[k] = z;
  }
  __syncthreads();
  // 3) softmax (wave 0)
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
  // 4) context + u
  const float beta = sh_beta;
  float nsq = 0.f;
#pragma unroll
  for (int i = 0; i < DPT; ++i) {
    const int d = t + 512 * i;
    float c = 0.f;
#pragma unroll
    for (int kk = 0; kk < P; ++kk) c = __builtin_fmaf(sh_alpha[kk], vv[i][kk], c);
    const float chat = __builtin_fmaf(beta, sv[i], (1.f - beta) * c);
    const float u = chat + hv[i];
    nsq = __builtin_fmaf(u, u, nsq);
    u_out[(int64_t)b * H + d] = u;
    if (ub_out) ub_out[frag_off(b, d, H)] = f2bf(u);
    if (ub3_out) {
      __bf16 x0, x1, x2;
      split3(u, x0, x1, x2);
      __bf16* o = reinterpret_cast<__bf16*>(ub3_out + ((size_t)((b >> 5) * (H / 16) + (d >> 4)) * 3) * 64 +
                                            (b & 31) + 32 * ((d >> 3) & 1)) + (d & 7);
      o[0] = x0;
      o[64 * 8] = x1;
      o[128 * 8] = x2;
    }
  }
  if (unorm) {
    nsq = wave_sum(nsq);
    if (lane == 0) sh_norm[w] = nsq;
    __syncthreads();
    if (t == 0)
      unorm[b] = sqrtf(((sh_norm[0] + sh_norm[1]) + (sh_norm[2] + sh_norm[3])) +
                       ((sh_norm[4] + sh_norm[5]) + (sh_norm[6] + sh_norm[7]))) * 1.00001f;
  }
}

// MODE 0: V stream only (same loads as k_atten5), one float out per thread
__global__ __launch_bounds__(512) void kv_vstream(const float* __restrict__ Vf, float* __restrict__ out) {
  constexpr int H = 512;
  const int t = threadIdx.x, b = blockIdx.x;
  const float* vb = Vf + (int64_t)b * P * H;
  float vv[P];
#pragma unroll
  for (int kk = 0; kk < P; ++kk) vv[kk] = vb[(int64_t)kk * H + t];
  float c = 0.f;
#pragma unroll
  for (int kk = 0; kk < P; ++kk) c += vv[kk];
  out[(int64_t)b * H + t] = c;
}
template <int H, int MODE>
__device__ __forceinline__ void kv_tail(int B, int m0, int nt, const float (&gate)[4][2], float2 sa, float2 sb,
                                               float2 cprev, float4 wsv, float* Hs, float* h_out,
                                               bf16x8* __restrict__ hsp_out, float* __restrict__ c_out,
                                               float* __restrict__ s_out, float* __restrict__ part) {
  constexpr int HP = LS_HP, WSP = LS_WSP, NTn = H / 16, KC = H / 16;
  float* Ss = Hs + 16 * HP;   // [16][HP] s of the tile, transposed
  float* Wsl = Ss + 16 * HP;  // [16][WSP] W_g / W_s rows (j < 49: W_g, else W_s) per unit
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int rr = t >> 3, u0 = (t & 7) * 2, m = m0 + rr, j = nt * 16 + u0;
  {  // transpose the W_g / W_s slice to [unit][j] (j = 98, 99 are zero)
    const int jj = t >> 2, uq = (t & 3) * 4;
    if (t < 2 * P * 4) {
      Wsl[(uq + 0) * WSP + jj] = wsv.x; Wsl[(uq + 1) * WSP + jj] = wsv.y;
      Wsl[(uq + 2) * WSP + jj] = wsv.z; Wsl[(uq + 3) * WSP + jj] = wsv.w;
    } else if (t < 2 * P * 4 + 32) {
      const int z = t - 2 * P * 4;  // 32 zeros: j = 98, 99 for 16 units
      Wsl[(z >> 1) * WSP + 2 * P + (z & 1)] = 0.f;
    }
  }
  {
    float hn[2], cn[2], sn[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      if (MODE == 4) {
        const float i_ = gate[0][q] * 0.5f, f_ = gate[1][q] * 0.25f, g_ = gate[2][q], o_ = gate[3][q] * 0.5f;
        cn[q] = f_ * (&cprev.x)[q] + i_ * g_;
        const float tc = cn[q] * 0.9f;
        hn[q] = o_ * tc;
        sn[q] = ((&sa.x)[q] + (&sb.x)[q]) * tc;
      } else {
      const float i_ = sigmoidf_(gate[0][q]), f_ = sigmoidf_(gate[1][q]), g_ = tanhf(gate[2][q]),
                  o_ = sigmoidf_(gate[3][q]);
      cn[q] = f_ * (&cprev.x)[q] + i_ * g_;
      const float tc = tanhf(cn[q]);
      hn[q] = o_ * tc;
      sn[q] = sigmoidf_((&sa.x)[q] + (&sb.x)[q]) * tc;
      }
    }
    Hs[u0 * HP + rr] = hn[0];
    Hs[(u0 + 1) * HP + rr] = hn[1];
    Ss[u0 * HP + rr] = sn[0];
    Ss[(u0 + 1) * HP + rr] = sn[1];
    if (m < B) {
      *reinterpret_cast<float2*>(c_out + (int64_t)m * H + j) = make_float2(cn[0], cn[1]);
      *reinterpret_cast<float2*>(h_out + (int64_t)m * H + j) = make_float2(hn[0], hn[1]);
      *reinterpret_cast<float2*>(s_out + (int64_t)m * H + j) = make_float2(sn[0], sn[1]);
      if (hsp_out && MODE != 6) {
        // next step's A fragments: k = j.. in chunk nt, lane (m % 32) + 32 * (u0 / 8), elements u0 % 8..
        typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
        bf16x2 p0, p1, p2;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          __bf16 x0, x1, x2;
          split3(hn[q], x0, x1, x2);
          p0[q] = x0; p1[q] = x1; p2[q] = x2;
        }
        bf16x8* o = hsp_out + ((size_t)((m >> 5) * KC + nt) * 3) * 64 + (m & 31) + 32 * (u0 >> 3);
        const int e = u0 & 7;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o) + e) = p0;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o + 64) + e) = p1;
        *reinterpret_cast<bf16x2*>(reinterpret_cast<__bf16*>(o + 128) + e) = p2;
      }
    }
  }
  if (MODE == 5) return;
  __syncthreads();
  // Wave -> one 32x32 block: rows rb*32.., columns cb = 0, 1: W_g j = 0..63; cb = 2, 3: W_s j = 0..63.
  {
    const int rb = wave & 1, cb = wave >> 1, li = lane & 31, lh = lane >> 5;
    const float* X = cb < 2 ? Hs : Ss;
    const int jj = (cb & 1) * 32 + li, jg = (cb < 2 ? 0 : P) + jj, jgc = jg < WSP ? jg : WSP - 1;
    floatx16 pacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) pacc[r] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int u = i + 8 * lh;
      const float av = X[u * HP + rb * 32 + li];
      const float wv = jj < P ? Wsl[u * WSP + jgc] : 0.f;
      if (MODE != 7) pacc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, wv, pacc, 0, 0, 0);
      else pacc[i] += av * wv;
    }
    if (jj < P && MODE != 8) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mr = m0 + rb * 32 + acc_row(r, lane);
        if (mr < B) part[((int64_t)mr * NTn + nt) * PART + jg] = pacc[r];
      }
    }
  }
}

template <int H, int MODE, class F>
__device__ __forceinline__ void kv_lgp(const bf16x8* af0, const bf16x8* af1, const bf16x8* wf0,
                                                   const bf16x8* wf1, float* Pt, F&& between) {
  constexpr int KC = H / 16, CP = LS_CP, TS = 64 * LS_CP;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr int per = KC / 8;  // even for H in {256, 512, 768, 1024}
  const int kc0 = wave * per;
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
  bf16x8 fa[2][2][3], fw[2][2][3];  // [slot][block][plane]
  auto load = [&](int slot, int kc) {
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const size_t o = ((size_t)kc * 3 + q) * 64;
      fa[slot][0][q] = af0[o];
      fa[slot][1][q] = af1[o];
      fw[slot][0][q] = wf0[o];
      fw[slot][1][q] = wf1[o];
    }
  };
  const int last = kc0 + per - 1;
  asm volatile("" ::: "memory");
  load(0, kc0);
  load(1, kc0 + 1 < last ? kc0 + 1 : last);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  between();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < per; i += 2) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) { if (MODE != 1) x3_step(acc[a][c], fa[d][a], fw[d][c]); else acc[a][c][0] += (float)fa[d][a][0][0] * (float)fw[d][c][0][0]; }
      const int nk = kc0 + i + d + 2;
      load(d, nk < last ? nk : last);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float* dst = Pt + (wave & 3) * TS;
  const int li = lane & 31, lh = lane >> 5;
  if (wave >= 4) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
          *reinterpret_cast<float4*>(dst + (c * 32 + li) * CP + a * 32 + 8 * r4 + 4 * lh) =
              make_float4(acc[a][c][4 * r4], acc[a][c][4 * r4 + 1], acc[a][c][4 * r4 + 2], acc[a][c][4 * r4 + 3]);
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          float4* e = reinterpret_cast<float4*>(dst + (c * 32 + li) * CP + a * 32 + 8 * r4 + 4 * lh);
          const float4 v = *e;
          *e = make_float4(acc[a][c][4 * r4] + v.x, acc[a][c][4 * r4 + 1] + v.y, acc[a][c][4 * r4 + 2] + v.z,
                           acc[a][c][4 * r4 + 3] + v.w);
        }
  }
}

template <int H, int MODE, bool G = false>
__global__ __launch_bounds__(512) void kv_lstm(int B, int V, const int64_t* __restrict__ tok, int tok_ld,
                                              const float* __restrict__ table,
                                              const float* __restrict__ xg, const bf16x8* __restrict__ hsp_in,
                                              const float* __restrict__ c_in, const int* __restrict__ par,
                                              const bf16x8* __restrict__ whh3,
                                              const float* __restrict__ wgs, float* __restrict__ h_out,
                                              bf16x8* __restrict__ hsp_out, float* __restrict__ c_out,
                                              float* __restrict__ s_out, float* __restrict__ part) {
  constexpr int BM = 64, CP = LS_CP, TS = 64 * LS_CP;
  __shared__ __attribute__((aligned(16))) float lds[4 * TS + LS_TAIL_FLOATS];
  constexpr int NTn = H / 16, KC = H / 16;
  const int MT = (B + BM - 1) / BM;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;  // m fastest: a weight tile is shared inside an XCD
  const int t = threadIdx.x, lane = t & 63;
  const int m0 = mt * BM;
  float* Pt = lds;  // [4][64][CP] partial tiles
  const int rr = t >> 3, u0 = (t & 7) * 2, m = m0 + rr;
  const int mc = m < B ? m : B - 1;  // rows >= B compute on row B-1 and store nothing
  const int j = nt * 16 + u0;
  // (token first, then the GEMM's first loads, then the token-dependent gathers: in-order vmcnt
  //  then waits for the token alone; the asm barriers keep the compiler from reordering the loads)
  int64_t tk = tok[(int64_t)mc * tok_ld];
  const bf16x8* af0;
  const bf16x8* af1;
  int pc = mc;  // source row of c (and of h, through the fragments)
  if constexpr (G) {
    const int ra0 = m0 + (lane & 31), ra1 = ra0 + 32;
    const int p0 = par[ra0 < B ? ra0 : B - 1], p1 = par[ra1 < B ? ra1 : B - 1];
    const int hl = 32 * (lane >> 5);
    af0 = hsp_in + (size_t)(p0 >> 5) * KC * 3 * 64 + (p0 & 31) + hl;
    af1 = hsp_in + (size_t)(p1 >> 5) * KC * 3 * 64 + (p1 & 31) + hl;
    pc = par[mc];
  } else {
    af0 = hsp_in + (size_t)(m0 / 32) * KC * 3 * 64 + lane;
    af1 = af0 + (size_t)KC * 3 * 64;
  }
  const bf16x8* wf0 = whh3 + (size_t)(nt * 2) * KC * 3 * 64 + lane;
  const bf16x8* wf1 = wf0 + (size_t)KC * 3 * 64;
  // epilogue gathers behind the first GEMM loads: token -> table row, x_g, c, W_g/W_s slice
  float2 ta[4], xa[4], sa, sb, cprev;
  float4 wsv;
  kv_lgp<H, MODE>(af0, af1, wf0, wf1, Pt, [&] {
    tk = tk < 0 ? 0 : (tk >= V ? V - 1 : tk);
    const int N5 = 5 * H;
    const float* trow = table + tk * N5;
    const float* xrow = xg + (int64_t)mc * N5;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      ta[g] = *reinterpret_cast<const float2*>(trow + nt * 64 + g * 16 + u0);
      xa[g] = *reinterpret_cast<const float2*>(xrow + nt * 64 + g * 16 + u0);
    }
    sa = *reinterpret_cast<const float2*>(trow + 4 * H + j);
    sb = *reinterpret_cast<const float2*>(xrow + 4 * H + j);
    cprev = *reinterpret_cast<const float2*>(c_in + (int64_t)pc * H + j);
    // W_g / W_s slice: wgs[tile] is [98][16] (j-major); thread t < 392 takes float4 t
    const float4* src = reinterpret_cast<const float4*>(wgs + (int64_t)nt * 2 * P * 16);
    wsv = src[t < 2 * P * 4 ? t : 2 * P * 4 - 1];
  });
  if (MODE == 3) { if (t < 64) h_out[(int64_t)(m0 + (t & 63)) * H + nt * 16] = Pt[t] + ta[0].x + xa[0].x + sa.x + sb.x + cprev.x + wsv.x; return; }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {  // 512 threads x 2 float4 = the 64 x 64 tile
    const int q = t + 512 * i, cq = q >> 4, r4 = (q & 15) * 4;
    const float* sp = Pt + cq * CP + r4;
    float4 v[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) v[w] = *reinterpret_cast<const float4*>(sp + w * TS);
    float4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) (&o.x)[e] = (f4c(v[0], e) + f4c(v[1], e)) + (f4c(v[2], e) + f4c(v[3], e));
    *reinterpret_cast<float4*>(Pt + cq * CP + r4) = o;
  }
  __syncthreads();
  float gate[4][2];
  {
    const float* cr = Pt + rr;  // column j of the summed tile at cr[j * CP]
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int q = 0; q < 2; ++q) gate[g][q] = cr[(16 * g + u0 + q) * CP] + ((&ta[g].x)[q] + (&xa[g].x)[q]);
  }
  if (MODE == 2) { h_out[(int64_t)m * H + j] = gate[0][0] + gate[1][1] + gate[2][0] + gate[3][1] + sa.x + sb.y + cprev.x + wsv.x; return; }
  kv_tail<H, MODE>(B, m0, nt, gate, sa, sb, cprev, wsv, lds + 4 * TS, h_out, hsp_out, c_out, s_out, part);
}

template <int NCB, int MODE>
__global__ __launch_bounds__(512) void kv_enc4(const float* __restrict__ feats, int B, int C,
                                                const bf16x8* __restrict__ W4, const float* __restrict__ bias,
                                                float* __restrict__ V, float* __restrict__ a_g) {
  static_assert(NCB % 2 == 0, "columns are processed in pairs of 16-column blocks");
  constexpr int H = 128 * NCB, NPAIR = NCB / 2, PL = E4_RB * 16 * E4_LD;  // PL: one plane, bf16
  __shared__ __attribute__((aligned(16))) __bf16 As[2][3][PL];
  __shared__ __attribute__((aligned(16))) float Sg[2][2 * 32 * E4_SP];  // fp32 stage copy for a_g
  __shared__ __attribute__((aligned(16))) float Ag[2 * E4_MAXC];        // a_g of the two images
  __shared__ float Junk[MODE >= 3 ? 1024 : 1];
  const int M = B * P, KC = C / 32;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.x * E4_ROWS;
  // staging: thread t < 392 -> row r = t % 98, channels 8 kg .. 8 kg + 7 of each 32-channel stage;
  // threads 392..511 fill garbage rows 98..105 (never stored) from a valid address
  const int sr = t < 4 * E4_ROWS ? t % E4_ROWS : E4_ROWS + (t & 7);
  const int kg = t < 4 * E4_ROWS ? t / E4_ROWS : (t >> 3) & 3;
  int m = m0 + (t < 4 * E4_ROWS ? sr : 0);
  m = m < M ? m : M - 1;  // clamp, never zero (rows >= M are not stored)
  const int bi = m / P, pi = m - bi * P;
  const float* arow = feats + (int64_t)bi * C * P + pi + (int64_t)(8 * kg) * P;
  const int so = sr * E4_LD + 8 * kg;
  // fragment reads: lane l -> row 16 rb + (l & 15), k = 8 (l >> 4)
  const int fo = (lane & 15) * E4_LD + 8 * (lane >> 4);
  const bf16x8* wsrc = W4 + (size_t)(wave * NCB) * KC * 3 * 64 + lane;  // block nb = wave NCB + c
  float ra[8];
  bf16x8 wv[NCB][3];
  floatx4 acc[E4_RB][NCB];
#pragma unroll
  for (int rb = 0; rb < E4_RB; ++rb)
#pragma unroll
    for (int c = 0; c < NCB; ++c) acc[rb][c] = floatx4{0.f, 0.f, 0.f, 0.f};

  auto gload_a = [&](int s) {
    const float* src = arow + (int64_t)(32 * s) * P;
#pragma unroll
    for (int i = 0; i < 8; ++i) ra[i] = src[i * P];
  };
  auto gload_w = [&](int s, int c) {
#pragma unroll
    for (int q = 0; q < 3; ++q) wv[c][q] = wsrc[((size_t)c * KC * 3 + (size_t)s * 3 + q) * 64];
  };
  auto lstore_a = [&](int buf) {
    bf16x8 x[3];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __bf16 x0, x1, x2;
      split3(ra[i], x0, x1, x2);
      x[0][i] = x0; x[1][i] = x1; x[2][i] = x2;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x8*>(&As[buf][q][so]) = x[q];
    if (MODE >= 3) {  // branch-free: the garbage-row threads write a junk area
      const int img = sr >= P, pp = sr - img * P;
      float* g = t < 4 * E4_ROWS ? &Sg[buf][(img * 32 + 8 * kg) * E4_SP + pp] : &Junk[t & 127];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i * (t < 4 * E4_ROWS ? E4_SP : 128)] = ra[i];
    } else
    if (MODE != 1 && t < 4 * E4_ROWS) {  // sr = 49 image + p
      const int img = sr >= P, pp = sr - img * P;
      float* g = &Sg[buf][(img * 32 + 8 * kg) * E4_SP + pp];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i * E4_SP] = ra[i];
    }
  };

  const int ns = KC;
  gload_a(0);
#pragma unroll
  for (int c = 0; c < NCB; ++c) gload_w(0, c);
  lstore_a(0);
  gload_a(ns > 1 ? 1 : 0);
  __syncthreads();
  for (int s = 0; s < ns; ++s) {
    const int buf = s & 1, s1 = s + 1 < ns ? s + 1 : ns - 1, s2 = s + 2 < ns ? s + 2 : ns - 1;
    // A of stage s+1 (in ra) into the other buffer: its last readers (stage s-1) passed the barrier
    if (MODE < 3) {
    lstore_a(buf ^ 1);
    gload_a(s2);
    __builtin_amdgcn_sched_barrier(0);
    }
    const __bf16* Ab = &As[buf][0][fo];
    if constexpr (MODE == 5 || MODE == 6) {
      bf16x8 fb[2][3];
#pragma unroll
      for (int q = 0; q < 3; ++q) fb[0][q] = *reinterpret_cast<const bf16x8*>(Ab + q * PL);
#pragma unroll
      for (int g = 0; g < NPAIR * E4_RB; ++g) {
        const int cp = g / E4_RB, rb = g % E4_RB, cur = g & 1;
        if (g + 1 < NPAIR * E4_RB) {
          const int rn = (g + 1) % E4_RB;
#pragma unroll
          for (int q = 0; q < 3; ++q) fb[cur ^ 1][q] = *reinterpret_cast<const bf16x8*>(Ab + q * PL + rn * 16 * E4_LD);
        }
#pragma unroll
        for (int c = 2 * cp; c < 2 * cp + 2; ++c) {
          floatx4 x = acc[rb][c];
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][2], wv[c][0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][1], wv[c][1], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][0], wv[c][2], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][1], wv[c][0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][0], wv[c][1], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[cur][0], wv[c][0], x, 0, 0, 0);
          acc[rb][c] = x;
        }
        if (rb == E4_RB - 1) {
          gload_w(s1, 2 * cp);
          gload_w(s1, 2 * cp + 1);
        }
        if (MODE == 6 && g == 0) {
          lstore_a(buf ^ 1);
          gload_a(s2);
        }
      }
    } else
#pragma unroll
    for (int cp = 0; cp < NPAIR; ++cp) {
#pragma unroll
      for (int rb = 0; rb < E4_RB; ++rb) {
        bf16x8 fa[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) fa[q] = *reinterpret_cast<const bf16x8*>(Ab + q * PL + rb * 16 * E4_LD);
#pragma unroll
        for (int c = 2 * cp; c < 2 * cp + 2; ++c) {
          floatx4 x = acc[rb][c];
          if (MODE == 2) { x[0] += (float)fa[2][0] * (float)wv[c][0][1] + (float)fa[0][1] * (float)wv[c][2][3]; acc[rb][c] = x; continue; }
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], wv[c][0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], wv[c][1], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wv[c][2], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], wv[c][0], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wv[c][1], x, 0, 0, 0);
          x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wv[c][0], x, 0, 0, 0);
          acc[rb][c] = x;
        }
        if (MODE >= 3 && cp == 0 && rb == 0) {
          lstore_a(buf ^ 1);
          gload_a(s2);
        }
        if (MODE == 4 && cp == 0 && rb == 1) {
#pragma unroll
          for (int z = 0; z < 24; ++z) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 3 VALU
          }
        }
      }
      gload_w(s1, 2 * cp);
      gload_w(s1, 2 * cp + 1);
      // re-read the A fragments for the next pair instead of keeping all 21 live (VGPR budget)
      asm volatile("" ::: "memory");
    }
    if (MODE != 1 && wave == (s & 7)) {  // a_g of stage s's 32 channels: lane -> (image lane / 32, channel lane % 32)
      const float* g = &Sg[buf][lane * E4_SP];
      float sum = 0.f;
#pragma unroll 4
      for (int pp = 0; pp < 48; pp += 4) {  // 16-B reads (E4_SP * 4 B = 13 x 16 B), summed in p order
        const float4 v = *reinterpret_cast<const float4*>(g + pp);
        sum += v.x; sum += v.y; sum += v.z; sum += v.w;
      }
      sum += g[48];
      Ag[(lane >> 5) * C + 32 * s + (lane & 31)] = sum / 49.0f;
    }
    __syncthreads();
    __builtin_amdgcn_sched_barrier(0);
  }
  // a_g of the workgroup's images (the last workgroup of an odd batch holds one)
  for (int i = t; i < 2 * C; i += 512) {
    const int img = 2 * blockIdx.x + (i >= C);
    if (img < B) a_g[(int64_t)img * C + (i - (i >= C ? C : 0))] = Ag[i];
  }
  // epilogue: lane l holds column 16 nb + (l & 15), rows 16 rb + 4 (l >> 4) + i
#pragma unroll
  for (int c = 0; c < NCB; ++c) {
    const int col = (wave * NCB + c) * 16 + (lane & 15);
    const float bv = bias[col];
#pragma unroll
    for (int rb = 0; rb < E4_RB; ++rb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = rb * 16 + 4 * (lane >> 4) + i, row = m0 + r;
        if (r < E4_ROWS && row < M) V[(int64_t)row * H + col] = reluf_(acc[rb][c][i] + bv);
      }
  }
}

// VARIANTS END
}  // namespace aa

extern "C" int kb_time(const aa_model* m, const float* feats, void* ws, int B, int T, const char* which, int reps,
                       float* out_us) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  size_t need;
  DecodeWS w = carve_decode(static_cast<char*>(ws), L, B, T, &need);
  const MP p = resolve(m, L);
  hipStream_t s = nullptr;
  const int H = L.H, MT = (B + 63) / 64;
  const int t = 1;
  const uint64_t* kprev = w.keys;
  uint64_t* kt = w.keys + B;
  auto launch = [&]() -> bool {
    if (!strcmp(which, "lstm")) {
      hipLaunchKernelGGL(k_lstm<512>, dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "atten")) {
      hipLaunchKernelGGL(k_atten<2>, dim3(B), dim3(256), 0, s, B, H / 16, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "atten5")) {
      hipLaunchKernelGGL(k_atten5<512>, dim3(B), dim3(512), 0, s, B, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "vscreen")) {
      hipLaunchKernelGGL(k_vscreen<512>, dim3(((B + SC_BM - 1) / SC_BM) * (L.Vp / SC_BN)), dim3(256), 0, s, B, L.V,
                         L.Vp, reinterpret_cast<const bf16x8*>(w.ub), w.unorm,
                         reinterpret_cast<const bf16x8*>(p.mlp_wb), p.mlp_gs, p.mlp_b, w.summ);
    } else if (!strcmp(which, "vrescore")) {
      hipLaunchKernelGGL(k_vrescore<512>, dim3(B), dim3(RS_NT), 0, s, B, L.V, L.Vp, w.u, w.summ, p.mlp_w, p.mlp_b, kt,
                         (int64_t*)nullptr, T, t);
    } else if (!strcmp(which, "enc_v3")) {
      const int M = B * P;
      hipLaunchKernelGGL(k_enc_v3, dim3(((M + EV_BM - 1) / EV_BM) * (H / EV_BN)), dim3(256), 0, s, feats, B, L.C, H, p.enc_w3, p.enc_a_b, w.V);
    // VARIANT LAUNCH BEGIN
    } else if (!strcmp(which, "ls_m0")) {
      auto kern = kv_ls<0>;
      hipLaunchKernelGGL(kern, dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "ls_m1")) {
      auto kern = kv_ls<1>;
      hipLaunchKernelGGL(kern, dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "ls_m2")) {
      auto kern = kv_ls<2>;
      hipLaunchKernelGGL(kern, dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "ls_m3")) {
      auto kern = kv_ls<3>;
      hipLaunchKernelGGL(kern, dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "at_nov")) {
      hipLaunchKernelGGL((kv_at<512, 1>), dim3(B), dim3(512), 0, s, B, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "at_copy")) {
      hipLaunchKernelGGL((kv_at<512, 0>), dim3(B), dim3(512), 0, s, B, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "vstream")) {
      hipLaunchKernelGGL(kv_vstream, dim3(B), dim3(512), 0, s, w.V, w.s);
    } else if (!strcmp(which, "vscreen2")) {
      hipLaunchKernelGGL(k_vscreen2<512>, dim3(((B + SC2_BM - 1) / SC2_BM) * (L.Vp / SC2_BN)), dim3(256), 0, s, B,
                         L.V, L.Vp, reinterpret_cast<const bf16x8*>(w.ub), w.unorm,
                         reinterpret_cast<const bf16x8*>(p.mlp_wb), p.mlp_gs, p.mlp_b, w.summ);
    } else if (!strcmp(which, "enc_v4")) {
      hipLaunchKernelGGL(k_enc_v4<4>, dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "at_wait")) {
      hipLaunchKernelGGL((kv_at<512, 2>), dim3(B), dim3(512), 0, s, B, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "at_hsfirst")) {
      hipLaunchKernelGGL((kv_at<512, 3>), dim3(B), dim3(512), 0, s, B, 1, w.h[1], w.s, w.part, w.V, w.vwv, p.wh,
                         (float*)nullptr, (int64_t)0, (float*)nullptr, (int64_t)0, w.u, w.ub, w.unorm, (bf16x8*)nullptr);
    } else if (!strcmp(which, "lstm_m0")) {
      hipLaunchKernelGGL((kv_lstm<512, 0>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m1")) {
      hipLaunchKernelGGL((kv_lstm<512, 1>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m2")) {
      hipLaunchKernelGGL((kv_lstm<512, 2>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m3")) {
      hipLaunchKernelGGL((kv_lstm<512, 3>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m4")) {
      hipLaunchKernelGGL((kv_lstm<512, 4>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m5")) {
      hipLaunchKernelGGL((kv_lstm<512, 5>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m6")) {
      hipLaunchKernelGGL((kv_lstm<512, 6>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m7")) {
      hipLaunchKernelGGL((kv_lstm<512, 7>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "lstm_m8")) {
      hipLaunchKernelGGL((kv_lstm<512, 8>), dim3(MT * (H / 16)), dim3(512), 0, s, B, L.V, (const int64_t*)w.tok0, 1,
                         p.table, w.xg, w.hsp[0], w.c[0], (const int*)nullptr, p.whh3, p.wgs, w.h[1], w.hsp[1], w.c[1], w.s, w.part);
    } else if (!strcmp(which, "enc4_m0")) {
      hipLaunchKernelGGL((kv_enc4<4, 0>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m1")) {
      hipLaunchKernelGGL((kv_enc4<4, 1>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m2")) {
      hipLaunchKernelGGL((kv_enc4<4, 2>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m3")) {
      hipLaunchKernelGGL((kv_enc4<4, 3>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m4")) {
      hipLaunchKernelGGL((kv_enc4<4, 4>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m5")) {
      hipLaunchKernelGGL((kv_enc4<4, 5>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    } else if (!strcmp(which, "enc4_m6")) {
      hipLaunchKernelGGL((kv_enc4<4, 6>), dim3((B * P + E4_ROWS - 1) / E4_ROWS), dim3(512), 0, s, feats, B, L.C, p.enc_w4,
                         p.enc_a_b, w.V, w.a_g);
    // VARIANT LAUNCH END
    } else {
      return false;
    }
    return true;
  };
  (void)t;
  if (!launch()) return -100;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) launch();
  hipEventRecord(e1, s);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  *out_us = 1e3f * ms / reps;
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return (int)hipGetLastError();
}

// aa_train.hip — teacher-forced training step of Encoder2Decoder (forward + backward), compiled
// into the same translation unit as aa_kernels.hip (included at its end; it reuses k_avgpool and
// k_enc_v).  Reference: baseline_attention.py:206-230 (forward), 148-194 (Decoder), 36-62
// (AttentiveCNN tail); adaptive_attention.py:26-58 (Atten), 62-85 (Sentinel), 110-134
// (AdaptiveBlock); train.py:101,197-219 (packed targets, CrossEntropyLoss, backward).
//
// Layout: every per-step array is t-major ([T][B][...], row r = t * B + b), so the LSTM step t
// works on rows [tB, (t+1)B) and pack_padded_sequence's packed rows (t-major over b < batch
// size of t; lengths sorted descending) are a monotone subset of the rows.
//
// Arithmetic: fp32 throughout (with AA_TRAIN_BF16 the GEMMs take bf16 operands, fp32 accumulation).
// GEMMs run on the generic MFMA tile kernel k_tgemm below
// (operands in any of the layouts the backward pass needs, bounds-checked, fixed accumulation
// order); everything else is elementwise or one-workgroup-per-row / per-image kernels with fixed
// reduction orders, so a training step is deterministic run to run.  The cross-entropy loss is
// the caller's (train.py computes it on the packed scores): backward starts from dL/dscores.

namespace aa {

// ---------------------------------------------------------------------------------------------
// generic GEMM: C[M, N] (+)= act(sum_k A(m, k) W(n, k) + bias[n] + bias2[n])
//   A(m, k) = at ? A[k lda + m] : A[row(m) lda + k]        row(m) = arow ? arow[m] : m
//   W(n, k) = wm == 0 : W[n ldw + k]
//             wm == 1 : W[k ldw + n]
//             wm == 2 : NCHW feature map [B][C][49] read as the [B*49, C] row matrix transposed:
//                       W(n = c, k = b*49 + p) = W[b*ldw*49 + c*49 + p]   (ldw = C)
//   C row m -> crow ? crow[m] : m
// 64x64 tiles, 256 threads (2 x 2 waves of 32x32), K steps of TStep::KS through double-buffered LDS
// (fp32 MFMA: lanes 0-31 take k = s, lanes 32-63 k = KS/2 + s of each step).
// ---------------------------------------------------------------------------------------------
struct TG {
  int M, N, K;
  const float* A;
  int64_t lda;
  const int* arow;
  int at;
  const float* W;
  int64_t ldw;
  int wm;
  float* C;
  int64_t ldc;
  const int* crow;
  const float* bias;
  const float* bias2;
  int accumulate;
  int act;      // 0 none, 1 relu, 2 tanh
  int splits;   // split-K: > 1 -> raw partial tiles to part[split][M][N], reduced by k_tgemm_reduce
  int kper;     // K per split (multiple of the K step)
  float* part;
};

// K step of the training GEMM: 64 with bf16 operands (two 32-wide halves per thread, so a
// latency-bound GEMM -- the per-step recurrent ones, K = 128 per split -- pays half the global round
// trips), 32 with fp32 operands (a 64-deep fp32 tile pair would need 70 KB of LDS and halve the
// occupancy of the large GEMMs: measured slower).  Tiles [64 rows][pitch]: fp32 pitch KS + 4 floats,
// bf16 KS + 8 bf16 (conflict-free 16-B fragment reads either way).
template <bool BF>
struct TStep {
  static constexpr int KS = BF ? 64 : 32, HH = KS / 32, LDK = KS + 4, LDB = KS + 8;
  static constexpr int TILE_F = BF ? 64 * LDB / 2 : 64 * LDK;  // one operand tile, in floats
};

// value i of a split GEMM: its S partials summed in split order from 0 (+ 0, as the reduce adds absent
// biases), or src itself when it was not split.  Up to SK_MAX partials are loaded together before the
// ordered sum (a loop over a runtime count waits for each load in turn).
constexpr int SK_MAX = 16;
__device__ __forceinline__ float sk_sum(const float* __restrict__ src, int S, int64_t MN, int64_t i) {
  if (S == 1) return src[i];
  float x[SK_MAX];
#pragma unroll
  for (int sp = 0; sp < SK_MAX; ++sp) x[sp] = sp < S ? src[sp * MN + i] : 0.f;
  float v = 0.f;
#pragma unroll
  for (int sp = 0; sp < SK_MAX; ++sp)
    if (sp < S) v += x[sp];
  for (int sp = SK_MAX; sp < S; ++sp) v += src[sp * MN + i];
  return v + 0.f;
}

// BF: operands rounded to bf16 (RNE) as they are staged in LDS, products on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation (BASELINE config 5: bf16 compute, fp32 master
// weights); same tiles, loads and epilogue as the fp32 engine.
template <bool BF>
__global__ __launch_bounds__(256) void k_tgemm(TG g) {
  constexpr int TBK = TStep<BF>::KS, HH = TStep<BF>::HH, TLDK = TStep<BF>::LDK, TLDB = TStep<BF>::LDB;
  __shared__ __attribute__((aligned(16))) float lds[2][2][TStep<BF>::TILE_F];
  const int tilesN = (g.N + 63) / 64;
  const int split = blockIdx.x % g.splits, tile = blockIdx.x / g.splits;
  const int mt = tile / tilesN, nt = tile % tilesN;
  const int kbeg = split * g.kper, kend = g.splits > 1 ? (kbeg + g.kper < g.K ? kbeg + g.kper : g.K) : g.K;
  const int m0 = mt * 64, n0 = nt * 64;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wmv = wave >> 1, wnv = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  float ra[HH][8], rw[HH][8];  // [32-wide k half][8 consecutive elements]
  // operands are read 8 consecutive elements per thread along their contiguous dimension, as two
  // 16-B loads when the 8 are in bounds and aligned, else element by element with zero fill
  const bool a4 = ((g.lda & 3) == 0) && ((((uintptr_t)g.A) & 15) == 0);
  const bool w4 = ((g.ldw & 3) == 0) && ((((uintptr_t)g.W) & 15) == 0) && g.wm != 2;
  auto load8 = [&](float (&r)[8], const float* base) {
    const float4 x = *reinterpret_cast<const float4*>(base), y = *reinterpret_cast<const float4*>(base + 4);
    r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w; r[4] = y.x; r[5] = y.y; r[6] = y.z; r[7] = y.w;
  };
  auto gload = [&](int k0, float (&ra)[HH][8], float (&rw)[HH][8]) {
#pragma unroll
    for (int hh = 0; hh < HH; ++hh) {
      const int kh = k0 + 32 * hh;
      if (!g.at) {  // 4 threads per row, 8 consecutive k each
        const int r = t >> 2, kq = (t & 3) * 8, m = m0 + r;
        const int64_t base = (int64_t)(m < g.M ? (g.arow ? g.arow[m] : m) : 0) * g.lda;
        if (a4 && m < g.M && kh + kq + 8 <= kend) load8(ra[hh], g.A + base + kh + kq);
        else
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int k = kh + kq + i;
            ra[hh][i] = (m < g.M && k < kend) ? g.A[base + k] : 0.f;
          }
      } else {  // 8 threads per k, 8 consecutive m each
        const int k = kh + (t >> 3), mq = (t & 7) * 8;
        if (a4 && k < kend && m0 + mq + 8 <= g.M) load8(ra[hh], g.A + (int64_t)k * g.lda + m0 + mq);
        else
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = m0 + mq + i;
            ra[hh][i] = (m < g.M && k < kend) ? g.A[(int64_t)k * g.lda + m] : 0.f;
          }
      }
      if (g.wm == 1) {
        const int k = kh + (t >> 3), nq = (t & 7) * 8;
        if (w4 && k < kend && n0 + nq + 8 <= g.N) load8(rw[hh], g.W + (int64_t)k * g.ldw + n0 + nq);
        else
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int n = n0 + nq + i;
            rw[hh][i] = (n < g.N && k < kend) ? g.W[(int64_t)k * g.ldw + n] : 0.f;
          }
      } else {
        const int r = t >> 2, kq = (t & 3) * 8, n = n0 + r;
        if (w4 && n < g.N && kh + kq + 8 <= kend) load8(rw[hh], g.W + (int64_t)n * g.ldw + kh + kq);
        else
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int k = kh + kq + i;
            float v = 0.f;
            if (n < g.N && k < kend) {
              if (g.wm == 0) v = g.W[(int64_t)n * g.ldw + k];
              else v = g.W[((int64_t)(k / P) * g.ldw + n) * P + (k % P)];
            }
            rw[hh][i] = v;
          }
      }
    }
  };
  auto lstore = [&](int buf, float (&ra)[HH][8], float (&rw)[HH][8]) {
#pragma unroll
    for (int hh = 0; hh < HH; ++hh) {
      const int ko = 32 * hh;
      if constexpr (BF) {
        __bf16* As = reinterpret_cast<__bf16*>(lds[buf][0]);
        __bf16* Ws = reinterpret_cast<__bf16*>(lds[buf][1]);
        if (!g.at) {
          const int r = t >> 2, kq = (t & 3) * 8;
          bf16x8 v;
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = (__bf16)ra[hh][i];
          *reinterpret_cast<bf16x8*>(As + r * TLDB + ko + kq) = v;
        } else {
          const int k = t >> 3, mq = (t & 7) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) As[(mq + i) * TLDB + ko + k] = (__bf16)ra[hh][i];
        }
        if (g.wm == 1) {
          const int k = t >> 3, nq = (t & 7) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) Ws[(nq + i) * TLDB + ko + k] = (__bf16)rw[hh][i];
        } else {
          const int r = t >> 2, kq = (t & 3) * 8;
          bf16x8 v;
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = (__bf16)rw[hh][i];
          *reinterpret_cast<bf16x8*>(Ws + r * TLDB + ko + kq) = v;
        }
      } else {
        float* As = lds[buf][0];
        float* Ws = lds[buf][1];
        if (!g.at) {
          const int r = t >> 2, kq = (t & 3) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) As[r * TLDK + ko + kq + i] = ra[hh][i];
        } else {
          const int k = t >> 3, mq = (t & 7) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) As[(mq + i) * TLDK + ko + k] = ra[hh][i];
        }
        if (g.wm == 1) {
          const int k = t >> 3, nq = (t & 7) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) Ws[(nq + i) * TLDK + ko + k] = rw[hh][i];
        } else {
          const int r = t >> 2, kq = (t & 3) * 8;
#pragma unroll
          for (int i = 0; i < 8; ++i) Ws[r * TLDK + ko + kq + i] = rw[hh][i];
        }
      }
    }
  };
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  const int nk = (kend - kbeg + TBK - 1) / TBK;
  auto compute = [&](int buf) {
    if constexpr (BF) {
      const __bf16* As = reinterpret_cast<const __bf16*>(lds[buf][0]);
      const __bf16* Ws = reinterpret_cast<const __bf16*>(lds[buf][1]);
#pragma unroll
      for (int kb = 0; kb < TBK / 16; ++kb) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(As + (wmv * 32 + li) * TLDB + 16 * kb + 8 * lh);
        const bf16x8 w = *reinterpret_cast<const bf16x8*>(Ws + (wnv * 32 + li) * TLDB + 16 * kb + 8 * lh);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, w, acc, 0, 0, 0);
      }
    } else {
      const float* As = lds[buf][0];
      const float* Ws = lds[buf][1];
#pragma unroll
      for (int s8 = 0; s8 < TBK / 8; ++s8) {  // lane half lh: k = (TBK / 2) lh + 4 s8 + j
        const float4 a = *reinterpret_cast<const float4*>(As + (wmv * 32 + li) * TLDK + (TBK / 2) * lh + 4 * s8);
        const float4 w = *reinterpret_cast<const float4*>(Ws + (wnv * 32 + li) * TLDK + (TBK / 2) * lh + 4 * s8);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4c(a, j), f4c(w, j), acc, 0, 0, 0);
      }
    }
  };
  // (loading two K steps ahead from two register sets -- 145 VGPRs, three waves per SIMD instead of
  // four -- was bit-identical and 1-2 % slower over the training step: profiles/r06z6_train_tgemm_pf2_ab.txt)
  gload(kbeg, ra, rw);
  lstore(0, ra, rw);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    if (ks + 1 < nk) gload(kbeg + (ks + 1) * TBK, ra, rw);
    compute(ks & 1);
    if (ks + 1 < nk) lstore((ks & 1) ^ 1, ra, rw);
    __syncthreads();
  }
  const int col = n0 + wnv * 32 + li;
  if (g.splits > 1) {
    float* pt = g.part + (int64_t)split * g.M * g.N;
    if (col < g.N)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wmv * 32 + acc_row(r, lane);
        if (m < g.M) pt[(int64_t)m * g.N + col] = acc[r];
      }
    return;
  }
  if (col >= g.N) return;
  const float bv = (g.bias ? g.bias[col] : 0.f) + (g.bias2 ? g.bias2[col] : 0.f);
  // accumulate: the 16 old values are loaded together before any store (a load after a store to C
  // may alias it, so loads interleaved with the stores each waited a full round trip: 16 per thread)
  float* dst[16];
  float old[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wmv * 32 + acc_row(r, lane);
    const int mc = m < g.M ? m : g.M - 1;
    dst[r] = g.C + (int64_t)(g.crow ? g.crow[mc] : mc) * g.ldc + col;
  }
  if (g.accumulate) {
#pragma unroll
    for (int r = 0; r < 16; ++r) old[r] = m0 + wmv * 32 + acc_row(r, lane) < g.M ? *dst[r] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wmv * 32 + acc_row(r, lane);
    if (m >= g.M) continue;
    float v = acc[r] + bv;
    if (g.act == 1) v = reluf_(v);
    else if (g.act == 2) v = tanhf(v);
    *dst[r] = g.accumulate ? old[r] + v : v;
  }
}

// split-K epilogue: partials summed in split order, then bias / act / row map / accumulate
__global__ void k_tgemm_reduce(TG g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)g.M * g.N) return;
  const int m = (int)(i / g.N), n = (int)(i % g.N);
  float v = sk_sum(g.part, g.splits, (int64_t)g.M * g.N, i);
  v += (g.bias ? g.bias[n] : 0.f) + (g.bias2 ? g.bias2[n] : 0.f);
  if (g.act == 1) v = reluf_(v);
  else if (g.act == 2) v = tanhf(v);
  float* dst = g.C + (int64_t)(g.crow ? g.crow[m] : m) * g.ldc + n;
  *dst = g.accumulate ? *dst + v : v;
}

// k_tgemm_reduce four columns per thread (16-B partial loads and stores; every element's arithmetic
// and order exactly k_tgemm_reduce's): for N % 4 == 0 with 16-B aligned C rows, bias and partials
// (reduce_launch checks).  The element-wise form's 4-B loads ran the largest reduce (dW_m's, 5.2 M
// elements) at ~2 TB/s.
__global__ void k_tgemm_reduce4(TG g) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, i = 4 * q;
  if (i >= (int64_t)g.M * g.N) return;
  const int m = (int)(i / g.N), n = (int)(i % g.N);
  const int64_t MN = (int64_t)g.M * g.N;
  float4 x[SK_MAX];
#pragma unroll
  for (int sp = 0; sp < SK_MAX; ++sp)
    x[sp] = sp < g.splits ? *reinterpret_cast<const float4*>(g.part + sp * MN + i) : make_float4(0.f, 0.f, 0.f, 0.f);
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (g.splits == 1) {
    v[0] = x[0].x; v[1] = x[0].y; v[2] = x[0].z; v[3] = x[0].w;
  } else {
#pragma unroll
    for (int sp = 0; sp < SK_MAX; ++sp)
      if (sp < g.splits) {
        v[0] += x[sp].x; v[1] += x[sp].y; v[2] += x[sp].z; v[3] += x[sp].w;
      }
    for (int sp = SK_MAX; sp < g.splits; ++sp) {
      const float4 y = *reinterpret_cast<const float4*>(g.part + sp * MN + i);
      v[0] += y.x; v[1] += y.y; v[2] += y.z; v[3] += y.w;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = v[e] + 0.f;
  }
  float* dst = g.C + (int64_t)(g.crow ? g.crow[m] : m) * g.ldc + n;
  const float4 old = g.accumulate ? *reinterpret_cast<const float4*>(dst) : make_float4(0.f, 0.f, 0.f, 0.f);
  float r[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float t = v[e] + ((g.bias ? g.bias[n + e] : 0.f) + (g.bias2 ? g.bias2[n + e] : 0.f));
    if (g.act == 1) t = reluf_(t);
    else if (g.act == 2) t = tanhf(t);
    r[e] = g.accumulate ? (&old.x)[e] + t : t;
  }
  *reinterpret_cast<float4*>(dst) = make_float4(r[0], r[1], r[2], r[3]);
}

// the split-K reduce of `g`: four columns per thread when the shapes and pointers allow
static void reduce_launch(const TG& g, hipStream_t s) {
  const auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (g.N % 4 == 0 && g.ldc % 4 == 0 && a16(g.C) && a16(g.part))
    hipLaunchKernelGGL(k_tgemm_reduce4, dim3((unsigned)(((int64_t)g.M * g.N / 4 + 255) / 256)), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(k_tgemm_reduce, dim3((unsigned)(((int64_t)g.M * g.N + 255) / 256)), dim3(256), 0, s, g);
}

// ---------------------------------------------------------------------------------------------
// k_tgemm on 128 x 128 tiles for a bf16 step (AA_TRAIN_BF16): the same operand layouts (A
// row-major or transposed, W in layouts 0 / 1), RNE rounding while staging, bias / act / row maps /
// accumulate and split-K partials as k_tgemm; a workgroup computes a 128 x 128 tile (four waves of
// 64 x 64 = 2 x 2 v_mfma_f32_32x32x16_bf16 blocks, k_bgemm's MFMA arrangement), 64-deep K steps
// double-buffered in LDS.  Twice k_tgemm's FLOP per staged byte and four MFMAs per fragment pair read.
// LDS rows of 72 bf16 (144 B) with the 16-B chunk index XOR-swizzled by (row / 8) % 8: the
// transposed operands are staged as 2-byte stores down a column of rows 8 apart, which without the
// swizzle fall into two banks (8-way conflicts); with it into 16.  The 16-B fragment reads stay
// conflict-free (8 consecutive rows share the swizzle).
// ---------------------------------------------------------------------------------------------
constexpr int T8_T = 128, T8_KS = 64, T8_LD = T8_KS + 8;
__device__ __forceinline__ int t8_off(int r, int k) {  // bf16 index of (row r, k) in a swizzled tile
  return r * T8_LD + ((((k >> 3) ^ (r >> 3)) & 7) << 3) + (k & 7);
}
__global__ __launch_bounds__(256, 2) void k_tgemm128(TG g) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][T8_T * T8_LD];
  const int tilesN = (g.N + T8_T - 1) / T8_T;
  const int split = blockIdx.x % g.splits, tile = blockIdx.x / g.splits;
  const int mt = tile / tilesN, nt = tile % tilesN;
  const int kbeg = split * g.kper, kend = g.splits > 1 ? (kbeg + g.kper < g.K ? kbeg + g.kper : g.K) : g.K;
  const int m0 = mt * T8_T, n0 = nt * T8_T;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const bool a4 = ((g.lda & 3) == 0) && ((((uintptr_t)g.A) & 15) == 0);
  const bool w4 = ((g.ldw & 3) == 0) && ((((uintptr_t)g.W) & 15) == 0);
  float ra[4][8], rw[4][8];
  auto load8 = [&](float (&r)[8], const float* base) {
    const float4 x = *reinterpret_cast<const float4*>(base), y = *reinterpret_cast<const float4*>(base + 4);
    r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w; r[4] = y.x; r[5] = y.y; r[6] = y.z; r[7] = y.w;
  };
  // piece i of this thread: K-contiguous operands (A with at = 0, W with wm = 0) -> row q >> 3,
  // k 8 (q & 7) (8 lanes per 256-B row segment); transposed ones -> k q >> 4, rows 8 (q & 15) .. + 7
  // (16 lanes per 512-B segment of a k row); q = t + 256 i
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + 256 * i;
      if (!g.at) {
        const int r = q >> 3, kq = (q & 7) * 8, m = m0 + r, k = k0 + kq;
        const int64_t base = (int64_t)(m < g.M ? (g.arow ? g.arow[m] : m) : 0) * g.lda;
        if (a4 && m < g.M && k + 8 <= kend) load8(ra[i], g.A + base + k);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) ra[i][e] = (m < g.M && k + e < kend) ? g.A[base + k + e] : 0.f;
      } else {
        const int k = k0 + (q >> 4), mq = m0 + (q & 15) * 8;
        if (a4 && k < kend && mq + 8 <= g.M) load8(ra[i], g.A + (int64_t)k * g.lda + mq);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) ra[i][e] = (k < kend && mq + e < g.M) ? g.A[(int64_t)k * g.lda + mq + e] : 0.f;
      }
      if (g.wm == 0) {
        const int r = q >> 3, kq = (q & 7) * 8, n = n0 + r, k = k0 + kq;
        const int64_t base = (int64_t)(n < g.N ? n : 0) * g.ldw;
        if (w4 && n < g.N && k + 8 <= kend) load8(rw[i], g.W + base + k);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) rw[i][e] = (n < g.N && k + e < kend) ? g.W[base + k + e] : 0.f;
      } else {
        const int k = k0 + (q >> 4), nq = n0 + (q & 15) * 8;
        if (w4 && k < kend && nq + 8 <= g.N) load8(rw[i], g.W + (int64_t)k * g.ldw + nq);
        else
#pragma unroll
          for (int e = 0; e < 8; ++e) rw[i][e] = (k < kend && nq + e < g.N) ? g.W[(int64_t)k * g.ldw + nq + e] : 0.f;
      }
    }
  };
  auto lstore = [&](int buf) {
    __bf16* As = lds[buf][0];
    __bf16* Ws = lds[buf][1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int q = t + 256 * i;
      if (!g.at) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)ra[i][e];
        *reinterpret_cast<bf16x8*>(As + t8_off(q >> 3, (q & 7) * 8)) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) As[t8_off((q & 15) * 8 + e, q >> 4)] = (__bf16)ra[i][e];
      }
      if (g.wm == 0) {
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (__bf16)rw[i][e];
        *reinterpret_cast<bf16x8*>(Ws + t8_off(q >> 3, (q & 7) * 8)) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) Ws[t8_off((q & 15) * 8 + e, q >> 4)] = (__bf16)rw[i][e];
      }
    }
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
  const int nk = (kend - kbeg + T8_KS - 1) / T8_KS;
  gload(kbeg);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload(kbeg + (ks + 1) * T8_KS);
    const __bf16* As = lds[buf][0];
    const __bf16* Ws = lds[buf][1];
#pragma unroll
    for (int kb = 0; kb < T8_KS / 16; ++kb) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) a[x] = *reinterpret_cast<const bf16x8*>(As + t8_off(wm * 64 + x * 32 + li, 16 * kb + 8 * lh));
#pragma unroll
      for (int y = 0; y < 2; ++y) b[y] = *reinterpret_cast<const bf16x8*>(Ws + t8_off(wn * 64 + y * 32 + li, 16 * kb + 8 * lh));
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    if (ks + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int col = n0 + wn * 64 + y * 32 + li;
    if (col >= g.N) continue;
    const float bv = (g.bias ? g.bias[col] : 0.f) + (g.bias2 ? g.bias2[col] : 0.f);
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + x * 32 + acc_row(r, lane);
        if (m >= g.M) continue;
        if (g.splits > 1) {
          g.part[(int64_t)split * g.M * g.N + (int64_t)m * g.N + col] = acc[x][y][r];
        } else {
          float v = acc[x][y][r] + bv;
          if (g.act == 1) v = reluf_(v);
          else if (g.act == 2) v = tanhf(v);
          float* dst = g.C + (int64_t)(g.crow ? g.crow[m] : m) * g.ldc + col;
          *dst = g.accumulate ? *dst + v : v;
        }
      }
  }
}

// k_tgemm's split-K bound (floats of partials): its split counts, and so its fp32 sums, as before
// the scratch grew for k_bgemm
constexpr size_t TG_SPLIT_CAP = (size_t)4 << 20;

// launch context of a training call: stream + split-K scratch carved from its workspace
struct GemmCtx {
  hipStream_t s;
  float* split;
  size_t cap;  // floats
  bool bf16;   // AA_TRAIN_BF16: bf16 operands, fp32 accumulation
};

// C[M,N] (+)= A W^T style helper with the common cases spelled out at the call sites.  GEMMs with
// too few output tiles to fill the chip are split along K (deterministically reduced).
// `defer` (the recurrent LSTM GEMMs): a split-K GEMM leaves its partial tiles in gc.split and
// returns the split count, and the consumer (k_tr_cell_sk / k_tr_cell_bwd_sk) sums them in split order
// itself -- k_tgemm_reduce's arithmetic, one launch fewer per recurrent step; 1 = C written (no split,
// no bias / act / accumulate allowed with defer).
static int tgemm(const GemmCtx& gc, int M, int N, int K, const float* A, int64_t lda, int at, const float* W, int64_t ldw,
                 int wm, float* C, int64_t ldc, int accumulate = 0, const float* bias = nullptr,
                 const float* bias2 = nullptr, int act = 0, const int* arow = nullptr, const int* crow = nullptr,
                 bool defer = false) {
  if (M <= 0 || N <= 0) return 0;
  const hipStream_t s = gc.s;
  static const bool tlog = [] {  // AA_TG_LOG=1: one stderr line per GEMM (shape attribution of a trace)
    const char* e = getenv("AA_TG_LOG");
    return e && atoi(e) == 1;
  }();
  if (tlog) fprintf(stderr, "tgemm M %d N %d K %d at %d wm %d acc %d stream %p\n", M, N, K, at, wm, accumulate, (void*)s);
  // AA_TG128=1, bf16 weight gradients (both operands transposed, K >= 1024: dW_hh, dW_ih, dW_x, dW_h
  // over all T B rows): 128 x 128 tiles (k_tgemm128), split along K to ~512 workgroups (>= 256 deep
  // each) -- 30.7 / 31.0 us against 41.7 / 76.1 us for dW_hh / dW_ih on the 64 x 64 engine (split to
  // 1024 workgroups, four times the partials), but they run on the aux stream beside the LSTM
  // backward and the whole step did not gain (750 vs 752 steps/s); for the GEMMs reading one operand
  // along K the 64 x 64 engine measured faster (profiles/r06v_train_gemm_engines.txt)
  static const bool t128 = [] {  // AA_TG128=1: the deep weight gradients on k_tgemm128 (off: no gain in the step)
    const char* e = getenv("AA_TG128");
    return e && atoi(e) == 1;
  }();
  if (t128 && gc.bf16 && at == 1 && wm == 1 && M >= 128 && N >= 128 && (int64_t)M * N >= 128 * 256 && K >= 1024) {
    const int tiles8 = ((M + T8_T - 1) / T8_T) * ((N + T8_T - 1) / T8_T);
    int sp = 1;
    if (tiles8 < 256 && K >= 512 && gc.split) {
      sp = (512 + tiles8 - 1) / tiles8;
      if (sp > K / 256) sp = K / 256;
      const size_t capsp = gc.cap / ((size_t)M * N);
      if ((size_t)sp > capsp) sp = (int)capsp;
      if (sp < 2) sp = 1;
    }
    int kp = K;
    if (sp > 1) {
      kp = ((K + sp - 1) / sp + T8_KS - 1) / T8_KS * T8_KS;
      sp = (K + kp - 1) / kp;
    }
    TG g{M, N, K, A, lda, arow, at, W, ldw, wm, C, ldc, crow, bias, bias2, accumulate, act, sp, kp,
         sp > 1 ? gc.split : nullptr};
    hipLaunchKernelGGL(k_tgemm128, dim3(tiles8 * sp), dim3(256), 0, s, g);
    if (sp > 1 && !defer) reduce_launch(g, s);
    return sp;
  }
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  int splits = 1;
  // few tiles: split to ~256 workgroups (>= 128 deep each); long K over < 512 tiles (the vocab-sized
  // backward GEMMs, the weight gradients over all T*B rows): split to ~1024 (>= 512 deep each)
  const bool small = tiles < 128 && K >= 256, deep = tiles < 512 && K >= 1024;
  static const int deep_wg = [] {  // AA_TG_DEEP_WG: workgroups a deep split aims at (A/B probe)
    const char* e = getenv("AA_TG_DEEP_WG");
    return e ? atoi(e) : 1024;
  }();
  if ((small || deep) && gc.split) {
    splits = small ? (256 + tiles - 1) / tiles : (deep_wg + tiles - 1) / tiles;
    const int kmax = K / (small ? 128 : 512);
    if (splits > kmax) splits = kmax;
    const size_t capsp = (gc.cap < TG_SPLIT_CAP ? gc.cap : TG_SPLIT_CAP) / ((size_t)M * N);
    if ((size_t)splits > capsp) splits = (int)capsp;
    if (splits < 2) splits = 1;
  }
  int kper = K;
  if (splits > 1) {
    const int ks = gc.bf16 ? TStep<true>::KS : TStep<false>::KS;
    kper = ((K + splits - 1) / splits + ks - 1) / ks * ks;
    splits = (K + kper - 1) / kper;
  }
  // split-K partials reduced by k_tgemm_reduce unless the consumer sums them itself (defer).  (An
  // in-launch combine by each tile's last-arriving split -- device-scope ticket, write-through
  // partials -- was bit-identical and measured slower in round 4: 597-602 vs 683-698 steps/s.)
  TG g{M, N, K, A, lda, arow, at, W, ldw, wm, C, ldc, crow, bias, bias2, accumulate, act, splits, kper,
       splits > 1 ? gc.split : nullptr};
  if (gc.bf16)
    hipLaunchKernelGGL(k_tgemm<true>, dim3(tiles * splits), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(k_tgemm<false>, dim3(tiles * splits), dim3(256), 0, s, g);
  if (splits > 1 && !defer) reduce_launch(g, s);
  return splits;
}


// ---------------------------------------------------------------------------------------------
// The four large GEMMs of a bf16 step (vocab forward, dU = dS W_m, dW_m = dS^T U, dW_a = dV^T A) on
// pre-packed bf16 operands: k_tgemm converted fp32 operands while staging 64 x 64 tiles (16 FLOP
// per byte through the CU, 6-10 % of the bf16 peak on these shapes).  Here both operands are bf16,
// row-major and K-contiguous ("NT": C[m][n] = sum_k A[m][k] B[n][k]), K a multiple of 64 with
// zero padding, produced by the k_pk_* kernels below (RNE, the same rounding k_tgemm<true> applies
// while staging), and a workgroup computes a 128 x 128 tile (four waves of 64 x 64 = 2 x 2
// v_mfma_f32_32x32x16_bf16 blocks), 64-deep K steps double-buffered in LDS (144-B rows:
// conflict-free 16-B fragment reads and staging stores).  Split-K partials go through
// k_tgemm_reduce (fixed split order), so a step stays deterministic.
// ---------------------------------------------------------------------------------------------
constexpr int BG_T = 128, BG_KS = 64, BG_LD = BG_KS + 8;
struct BG {
  int M, N, K;
  const __bf16* A;
  int64_t lda;
  const __bf16* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  const int* crow;
  const float* bias;
  int accumulate, splits, kper;
  float* part;
  int act;  // 0 none, 1 relu (after the bias)
};
__global__ __launch_bounds__(256, 2) void k_bgemm(BG g) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][BG_T * BG_LD];
  const int tilesN = (g.N + BG_T - 1) / BG_T;
  const int split = blockIdx.x % g.splits, tile = blockIdx.x / g.splits;
  const int mt = tile / tilesN, nt = tile % tilesN;
  const int m0 = mt * BG_T, n0 = nt * BG_T;
  const int kbeg = split * g.kper, kend = kbeg + g.kper < g.K ? kbeg + g.kper : g.K;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  // staging: 128 rows x 64 k per operand and step = 1024 16-B pieces, four per thread: piece
  // q = t + 256 i -> row q >> 3, k 8 (q & 7) (8 lanes per 128-B row: coalesced loads, conflict-free
  // ds_write_b128); rows past M / N are clamped (never stored)
  const __bf16* pa[4];
  const __bf16* pb[4];
  int so[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = t + 256 * i, r = q >> 3, kq = (q & 7) * 8;
    const int m = m0 + r < g.M ? m0 + r : g.M - 1, n = n0 + r < g.N ? n0 + r : g.N - 1;
    pa[i] = g.A + (int64_t)m * g.lda + kq;
    pb[i] = g.B + (int64_t)n * g.ldb + kq;
    so[i] = r * BG_LD + kq;
  }
  bf16x8 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ra[i] = *reinterpret_cast<const bf16x8*>(pa[i] + k0);
      rb[i] = *reinterpret_cast<const bf16x8*>(pb[i] + k0);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      *reinterpret_cast<bf16x8*>(&lds[buf][0][so[i]]) = ra[i];
      *reinterpret_cast<bf16x8*>(&lds[buf][1][so[i]]) = rb[i];
    }
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
  const int nk = (kend - kbeg) / BG_KS;
  gload(kbeg);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) gload(kbeg + (ks + 1) * BG_KS);
    const __bf16* As = lds[buf][0];
    const __bf16* Bs = lds[buf][1];
#pragma unroll
    for (int kb = 0; kb < BG_KS / 16; ++kb) {
      bf16x8 a[2], b[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) a[x] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + x * 32 + li) * BG_LD + 16 * kb + 8 * lh);
#pragma unroll
      for (int y = 0; y < 2; ++y) b[y] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + y * 32 + li) * BG_LD + 16 * kb + 8 * lh);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[x], b[y], acc[x][y], 0, 0, 0);
    }
    if (ks + 1 < nk) lstore(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int y = 0; y < 2; ++y) {
    const int col = n0 + wn * 64 + y * 32 + li;
    if (col >= g.N) continue;
    const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + x * 32 + acc_row(r, lane);
        if (m >= g.M) continue;
        if (g.splits > 1) {
          g.part[(int64_t)split * g.M * g.N + (int64_t)m * g.N + col] = acc[x][y][r];
        } else {
          float v = acc[x][y][r] + bv;
          if (g.act == 1) v = reluf_(v);
          float* dst = g.C + (int64_t)(g.crow ? g.crow[m] : m) * g.ldc + col;
          *dst = g.accumulate ? *dst + v : v;
        }
      }
  }
}

// dst[r][k] = bf16(src[map ? map[r] : r][k]) for k < cols, 0 up to Kp (a multiple of 8): 8 per thread,
// as two 16-B loads when the source rows allow (vec: lds % 4 == 0, cols % 8 == 0, 16-B aligned base)
__global__ void k_pk_rows(const float* __restrict__ src, int64_t lds, const int* __restrict__ map, int rows, int cols,
                          __bf16* __restrict__ dst, int Kp, int vec) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = Kp / 8;
  if (i >= (int64_t)rows * per) return;
  const int r = (int)(i / per), k0 = (int)(i % per) * 8;
  const float* sr = src + (int64_t)(map ? map[r] : r) * lds;
  bf16x8 v;
  if (vec && k0 < cols) {
    const float4 x = *reinterpret_cast<const float4*>(sr + k0), y = *reinterpret_cast<const float4*>(sr + k0 + 4);
    v[0] = (__bf16)x.x; v[1] = (__bf16)x.y; v[2] = (__bf16)x.z; v[3] = (__bf16)x.w;
    v[4] = (__bf16)y.x; v[5] = (__bf16)y.y; v[6] = (__bf16)y.z; v[7] = (__bf16)y.w;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (__bf16)(k0 + j < cols ? sr[k0 + j] : 0.f);
  }
  *reinterpret_cast<bf16x8*>(dst + (int64_t)r * Kp + k0) = v;
}

// transpose: dst[c][r] = bf16(src[r lds + c]) for r < rows, 0 for rows <= r < Kp; dst has cols rows
// of Kp.  64 x 64 tiles through LDS (reads along c, writes along r, both coalesced).  S: float or
// __bf16 (a bf16 source is already rounded: the same values)
template <class S>
__global__ __launch_bounds__(256) void k_pk_trans(const S* __restrict__ src, int64_t lds, int rows, int cols,
                                                  __bf16* __restrict__ dst, int Kp) {
  __shared__ float tile[64][65];
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64, t = threadIdx.x;
  for (int i = t; i < 64 * 64; i += 256) {
    const int rr = i / 64, cc = i % 64, r = r0 + rr, c = c0 + cc;
    tile[rr][cc] = (r < rows && c < cols) ? (float)src[(int64_t)r * lds + c] : 0.f;
  }
  __syncthreads();
  for (int i = t; i < 64 * 64; i += 256) {
    const int cc = i / 64, rr = i % 64, c = c0 + cc, r = r0 + rr;
    if (c < cols && r < Kp) dst[(int64_t)c * Kp + r] = (__bf16)tile[rr][cc];
  }
}

// the NCHW feature map as the bf16 row matrix of the encoder GEMM V = relu(A W_a^T + b): dst[b 49 + p][c]
// = feats[b][c][p]; a workgroup per (image, 64 channels) reads its 64 x 49 contiguous floats and writes
// 49 rows of 128 B
__global__ __launch_bounds__(256) void k_pk_featrows(const float* __restrict__ feats, int C, __bf16* __restrict__ dst) {
  __shared__ float tile[64 * P];
  const int b = blockIdx.y, c0 = blockIdx.x * 64, t = threadIdx.x;
  const float* src = feats + ((int64_t)b * C + c0) * P;
  for (int i = t; i < 64 * P; i += 256) tile[i] = src[i];  // [c][p]
  __syncthreads();
  for (int i = t; i < P * 8; i += 256) {  // row p, 8-channel piece j
    const int p = i >> 3, j = i & 7;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)tile[(8 * j + e) * P + p];
    *reinterpret_cast<bf16x8*>(dst + ((int64_t)b * P + p) * C + c0 + 8 * j) = v;
  }
}

// One pass over the NCHW feature map for a bf16 step: a workgroup per (image, 64 channels) reads its
// 64 x 49 contiguous floats once and writes (1) the rows of the encoder GEMM's operand, as
// k_pk_featrows; (2) the K-contiguous operand of the backward's dW_a = dV^T A, cols[c][b 49 + p] (as
// k_pk_feats, zero past row B 49 up to Kp: the last image's workgroups); (3) a_g[b][c] = the 49 values
// summed in p order / 49 -- k_avgpool's arithmetic, bit-identical.  Replaces k_avgpool +
// k_pk_featrows + the backward's k_pk_feats (three reads of the map, one now).
__global__ __launch_bounds__(256) void k_pk_feats3(const float* __restrict__ feats, int B, int C,
                                                   __bf16* __restrict__ rows, __bf16* __restrict__ cols, int Kp,
                                                   float* __restrict__ a_g) {
  __shared__ float tile[64 * P];
  const int b = blockIdx.y, c0 = blockIdx.x * 64, t = threadIdx.x;
  const float* src = feats + ((int64_t)b * C + c0) * P;
  for (int i = t; i < 64 * P; i += 256) tile[i] = src[i];  // [c][p]
  __syncthreads();
  for (int i = t; i < P * 8; i += 256) {  // row p, 8-channel piece j
    const int p = i >> 3, j = i & 7;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)tile[(8 * j + e) * P + p];
    *reinterpret_cast<bf16x8*>(rows + ((int64_t)b * P + p) * C + c0 + 8 * j) = v;
  }
  for (int i = t; i < 64 * P; i += 256) {
    const int c = i / P, p = i - c * P;
    cols[(int64_t)(c0 + c) * Kp + b * P + p] = (__bf16)tile[i];
  }
  if (b == B - 1)
    for (int i = t; i < 64 * (Kp - B * P); i += 256) {
      const int c = i / (Kp - B * P), r = B * P + i % (Kp - B * P);
      cols[(int64_t)(c0 + c) * Kp + r] = (__bf16)0.f;
    }
  if (t < 64) {
    const float* g = tile + t * P;
    float sum = 0.f;
    for (int p = 0; p < P; ++p) sum += g[p];
    a_g[(int64_t)b * C + c0 + t] = sum / 49.0f;
  }
}

// the NCHW feature map as the K-contiguous operand of dW_a = dV^T A: dst[c][b 49 + p] = feats[b][c][p],
// zero for rows >= B 49 up to Kp; 8 consecutive rows per thread (one 16-B store)
__global__ void k_pk_feats(const float* __restrict__ feats, int B, int C, __bf16* __restrict__ dst, int Kp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int per = Kp / 8;
  if (i >= (int64_t)C * per) return;
  const int c = (int)(i / per), row0 = (int)(i % per) * 8;
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int row = row0 + j;
    float x = 0.f;
    if (row < B * P) {
      const int b = row / P, p = row - b * P;
      x = feats[((int64_t)b * C + c) * P + p];
    }
    v[j] = (__bf16)x;
  }
  *reinterpret_cast<bf16x8*>(dst + (int64_t)c * Kp + row0) = v;
}

// C[M,N] (+)= A B^T (+ bias) on k_bgemm; K a multiple of 64.  Fewer than 512 tiles: split K to
// ~1024 workgroups (bounded by the split scratch), partials reduced by k_tgemm_reduce in split order.
static void bgemm(const GemmCtx& gc, int M, int N, int K, const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb,
                  float* C, int64_t ldc, const float* bias = nullptr, const int* crow = nullptr, int accumulate = 0,
                  int act = 0) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  const int tiles = ((M + BG_T - 1) / BG_T) * ((N + BG_T - 1) / BG_T), ksteps = K / BG_KS;
  static const int wg_target = [] {  // AA_BG_WG: workgroups a split k_bgemm aims at (A/B probe)
    const char* e = getenv("AA_BG_WG");
    return e ? atoi(e) : 256;
  }();
  int splits = tiles >= 512 ? 1 : (wg_target + tiles - 1) / tiles;
  if (splits > ksteps) splits = ksteps;
  const size_t capsp = gc.split ? gc.cap / ((size_t)M * N) : 1;
  if ((size_t)splits > capsp) splits = (int)capsp;
  if (splits < 1) splits = 1;
  const int kper = (ksteps + splits - 1) / splits * BG_KS;
  splits = (K + kper - 1) / kper;
  const BG g{M, N, K, A, lda, B, ldb, C, ldc, crow, bias, accumulate, splits, kper, splits > 1 ? gc.split : nullptr, act};
  hipLaunchKernelGGL(k_bgemm, dim3(tiles * splits), dim3(256), 0, gc.s, g);
  if (splits > 1) {
    TG r{};
    r.M = M; r.N = N; r.K = K; r.C = C; r.ldc = ldc; r.crow = crow; r.bias = bias; r.accumulate = accumulate;
    r.splits = splits; r.kper = kper; r.part = gc.split; r.act = act;
    reduce_launch(r, gc.s);
  }
}
static inline int rup64(int x) { return (x + 63) / 64 * 64; }
static void pk_rows(hipStream_t st, const float* src, int64_t lds, const int* map, int rows, int cols, __bf16* dst, int Kp) {
  const int64_t n = (int64_t)rows * (Kp / 8);
  const int vec = lds % 4 == 0 && cols % 8 == 0 && ((uintptr_t)src & 15) == 0;
  hipLaunchKernelGGL(k_pk_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, src, lds, map, rows, cols, dst, Kp,
                     vec);
}
template <class S>
static void pk_trans(hipStream_t st, const S* src, int64_t lds, int rows, int cols, __bf16* dst, int Kp) {
  hipLaunchKernelGGL(k_pk_trans<S>, dim3((unsigned)(Kp / 64), (unsigned)((cols + 63) / 64)), dim3(256), 0, st, src, lds,
                     rows, cols, dst, Kp);
}

// column sums: out[n] (+)= sum_m X[m ldx + n], deterministic: rows split into CS_CH fixed chunks
// summed in order by k_colsum (one thread per (column, chunk)), the chunk sums added in chunk
// order by k_colsum_fin.
constexpr int CS_CH = 64;
__global__ void k_colsum(const float* __restrict__ X, int M, int N, int64_t ldx, float* __restrict__ part) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, ch = blockIdx.y;
  if (n >= N) return;
  const int per = (M + CS_CH - 1) / CS_CH, m0 = ch * per, m1 = m0 + per < M ? m0 + per : M;
  float s = 0.f;
  int m = m0;
  // eight loads in flight, then the eight adds in row order (the same sum, bit for bit, as one row
  // at a time; a chunk of 98 rows -- the dV bias gradient -- ran ~30 us one dependent load at a time)
  for (; m + 8 <= m1; m += 8) {
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = X[(int64_t)(m + j) * ldx + n];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += x[j];
  }
  for (; m < m1; ++m) s += X[(int64_t)m * ldx + n];
  part[(int64_t)ch * N + n] = s;
}
__global__ void k_colsum_fin(const float* __restrict__ part, int N, float* __restrict__ out) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int ch = 0; ch < CS_CH; ++ch) s += part[(int64_t)ch * N + n];
  out[n] = s;
}
// k_colsum + k_colsum_fin in one launch for short columns (M <= CS1_MAXM: the encoder-head bias
// gradients over the B rows): a workgroup per 64 columns, wave g sums chunks [16 g, 16 g + 16) of
// its lane's column (k_colsum's chunks, rows in order from 0), the 64 chunk sums go through LDS and
// lane c of wave 0 adds them in chunk order from 0 -- k_colsum_fin's arithmetic: the same bits, one
// launch instead of two, every load of a thread in flight at once.
constexpr int CS1_MAXM = 512;
__global__ __launch_bounds__(256) void k_colsum1(const float* __restrict__ X, int M, int N, int64_t ldx,
                                                 float* __restrict__ out) {
  __shared__ float cs[CS_CH][65];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6, n = blockIdx.x * 64 + c;
  const int per = (M + CS_CH - 1) / CS_CH;
  const int nc = n < N ? n : N - 1;
  for (int j = 0; j < CS_CH / 4; ++j) {
    const int ch = 16 * g + j, m0 = ch * per, m1 = m0 + per < M ? m0 + per : M;
    float x[CS1_MAXM / CS_CH];
#pragma unroll
    for (int i = 0; i < CS1_MAXM / CS_CH; ++i) x[i] = m0 + i < m1 ? X[(int64_t)(m0 + i) * ldx + nc] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CS1_MAXM / CS_CH; ++i)
      if (m0 + i < m1) s += x[i];
    cs[ch][c] = s;
  }
  __syncthreads();
  if (g == 0 && n < N) {
    float s = 0.f;
    for (int ch = 0; ch < CS_CH; ++ch) s += cs[ch][c];
    out[n] = s;
  }
}
static void colsum(hipStream_t st, const float* X, int M, int N, int64_t ldx, float* scratch, float* out) {
  if (M > 0 && M <= CS1_MAXM) {
    hipLaunchKernelGGL(k_colsum1, dim3((N + 63) / 64), dim3(256), 0, st, X, M, N, ldx, out);
    return;
  }
  hipLaunchKernelGGL(k_colsum, dim3((N + 255) / 256, CS_CH), dim3(256), 0, st, X, M, N, ldx, scratch);
  hipLaunchKernelGGL(k_colsum_fin, dim3((N + 255) / 256), dim3(256), 0, st, scratch, N, out);
}

// Two streams of one training call: `main` (the caller's) carries the chain the result depends on
// step by step (encoder head -> LSTM -> attention -> vocab; its backward in reverse), `aux` the
// work off that chain (the encoder's V GEMM beside the LSTM forward, the weight gradients beside
// the LSTM backward).  Each side has its own split-K scratch, arrival counters and column-sum
// scratch, and every buffer is written by one side only between two hand-overs, so the arithmetic
// and its order are those of the one-stream call: bit-identical results.  aux == main (or null):
// one stream, hand-overs are no-ops.  Events come from a per-thread pool, recorded again on the
// next call (a wait already queued is not affected by a later record).
struct Fork {
  hipStream_t main, aux;
  int used = 0;
  hipError_t err = hipSuccess;
  Fork(hipStream_t m, hipStream_t a) : main(m), aux(a && a != m ? a : m) {}
  bool split() const { return aux != main; }
  hipEvent_t next() {
    thread_local std::vector<hipEvent_t> pool;
    if (used == (int)pool.size()) {
      hipEvent_t e = nullptr;
      hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
      if (r != hipSuccess) {
        if (!err) err = r;
        return nullptr;
      }
      pool.push_back(e);
    }
    return pool[used++];
  }
  void hand(hipStream_t from, hipStream_t to) {  // `to` waits for everything queued on `from` so far
    if (!split() || err) return;
    hipEvent_t e = next();
    if (!e) return;
    hipError_t r = hipEventRecord(e, from);
    if (!r) r = hipStreamWaitEvent(to, e, 0);
    if (r && !err) err = r;
  }
  void to_aux() { hand(main, aux); }
  void to_main() { hand(aux, main); }
  hipEvent_t mark(hipStream_t from) {  // a point on `from` to wait for later (wait())
    if (!split() || err) return nullptr;
    hipEvent_t e = next();
    if (e) {
      hipError_t r = hipEventRecord(e, from);
      if (r && !err) err = r;
    }
    return e;
  }
  void wait(hipStream_t to, hipEvent_t e) {
    if (!e || err) return;
    hipError_t r = hipStreamWaitEvent(to, e, 0);
    if (r && !err) err = r;
  }
};

// ---------------------------------------------------------------------------------------------
// forward pieces
// ---------------------------------------------------------------------------------------------
// X[t B + b] = [embed[tok[b][t]]; v_g[b]]  (baseline_attention.py:151-154)
__global__ void k_tr_x(const int64_t* __restrict__ tok, int tld, const float* __restrict__ embed, int V, int E,
                       const float* __restrict__ vg, int B, int T, float* __restrict__ X) {
  const int r = blockIdx.x, t = r / B, b = r % B;
  int64_t tk = tok[(int64_t)b * tld + t];
  tk = tk < 0 ? 0 : (tk >= V ? V - 1 : tk);
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    X[(int64_t)r * 2 * E + e] = embed[tk * E + e];
    X[(int64_t)r * 2 * E + E + e] = vg[(int64_t)b * E + e];
  }
}

// LSTM cell of step t (torch gate order i, f, g, o): gates = G4 (h W_hh^T) + PRE (x W_ih^T + b), with
// the recurrent GEMM's split-K reduction folded in: G4 (b, n) = sk_sum(src, S, B 4H, .) (bit-identical
// to k_tgemm_reduce followed by a plain cell kernel; one launch per step fewer)
__global__ void k_tr_cell_sk(const float* __restrict__ src, int S, const float* __restrict__ PRE, int ldp,
                             const float* __restrict__ c_prev, int B, int H, float* __restrict__ h_out,
                             float* __restrict__ c_out, float* __restrict__ GA) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * H) return;
  const int b = (int)(i / H), j = (int)(i % H);
  const int64_t MN = (int64_t)B * 4 * H, g0 = (int64_t)b * 4 * H + j;
  const float* p = PRE + (int64_t)b * ldp;
  const float gi = sk_sum(src, S, MN, g0) + p[j], gf = sk_sum(src, S, MN, g0 + H) + p[H + j],
              gg = sk_sum(src, S, MN, g0 + 2 * H) + p[2 * H + j], go = sk_sum(src, S, MN, g0 + 3 * H) + p[3 * H + j];
  const float i_ = sigmoidf_(gi), f_ = sigmoidf_(gf), g_ = tanhf(gg), o_ = sigmoidf_(go);
  const float c = f_ * c_prev[i] + i_ * g_;
  c_out[i] = c;
  h_out[i] = o_ * tanhf(c);
  float* ga = GA + (int64_t)b * 4 * H;
  ga[j] = i_; ga[H + j] = f_; ga[2 * H + j] = g_; ga[3 * H + j] = o_;
}

// sentinel: SG = sigmoid(x W_x^T + h_{t-1} W_h^T) (pre-activation in SG), S = SG * tanh(c)
__global__ void k_tr_sent(float* __restrict__ SG, const float* __restrict__ Cs, float* __restrict__ S, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float sg = sigmoidf_(SG[i]);
  SG[i] = sg;
  S[i] = sg * tanhf(Cs[i]);
}

// copy columns [c0, c0 + n) of a row matrix
__global__ void k_copy_cols(const float* __restrict__ src, int64_t lds, int c0, float* __restrict__ dst, int64_t ldd,
                            int rows, int n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * n) return;
  const int r = (int)(i / n), c = (int)(i % n);
  dst[(int64_t)r * ldd + c] = src[(int64_t)r * lds + c0 + c];
}

// Atten.forward for one (t, b) row (adaptive_attention.py:34-56), projections precomputed:
// PG = W_g h_t, PS = W_s s_t (row pitch PP), VWv[b] = W_v V_b.  Writes alpha (pitch PP), beta,
// the context c_t and u = c_hat + h_t (the mlp input, :132).  256 threads.
__global__ __launch_bounds__(256) void k_tr_atten(int B, int H, const float* __restrict__ PG, const float* __restrict__ PS,
                                                  const float* __restrict__ VWv, const float* __restrict__ Vf,
                                                  const float* __restrict__ wh, const float* __restrict__ Hs,
                                                  const float* __restrict__ S, float* __restrict__ alpha,
                                                  float* __restrict__ beta, float* __restrict__ ctx,
                                                  float* __restrict__ U) {
  __shared__ float zs[PP], al[PP], sh_b;
  const int r = blockIdx.x, b = r % B, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float* pg = PG + (int64_t)r * PP;
  // scores z_k = w_h . tanh(VWv[b][k] + PG), k < 49; z_s = w_h . tanh(PS + PG): one wave per item
  for (int k = w; k <= P; k += 4) {
    float z = 0.f;
    if (lane < P) {
      const float x = (k < P ? VWv[((int64_t)b * P + k) * PP + lane] : PS[(int64_t)r * PP + lane]) + pg[lane];
      z = wh[lane] * tanhf(x);
    }
    z = wave_sum(z);
    if (lane == 0) zs[k] = z;
  }
  __syncthreads();
  if (w == 0) {  // softmax_49 (alpha), softmax_50 (beta = its last entry)
    const float z = lane < P ? zs[lane] : -INFINITY;
    const float m = wave_max(z);
    const float e = lane < P ? expf(z - m) : 0.f;
    const float a = e / wave_sum(e);
    if (lane < P) {
      al[lane] = a;
      alpha[(int64_t)r * PP + lane] = a;
    }
    const float zsn = zs[P];
    const float m2 = fmaxf(m, zsn);
    const float e2 = lane < P ? expf(z - m2) : 0.f;
    const float es = expf(zsn - m2);
    const float S2 = wave_sum(e2) + es;
    if (lane == 0) {
      sh_b = es / S2;
      beta[r] = es / S2;
    }
  }
  __syncthreads();
  const float be = sh_b;
  const float* vb = Vf + (int64_t)b * P * H;
  for (int d = t; d < H; d += 256) {
    float c = 0.f;
    for (int k = 0; k < P; ++k) c = __builtin_fmaf(al[k], vb[(int64_t)k * H + d], c);
    ctx[(int64_t)r * H + d] = c;
    const float chat = be * S[(int64_t)r * H + d] + (1.f - be) * c;
    U[(int64_t)r * H + d] = chat + Hs[(int64_t)r * H + d];
  }
}

// k_tr_atten's rows grouped by image, in three phases instead of a per-row chain: one workgroup of H
// threads per (image b, group of TS <= 32 consecutive steps).  V_b stays in registers (thread d holds
// column d: 49 floats), VWv_b and the group's PG / PS rows in LDS.
//   A: every (row, item) score of the group at once, one per thread: z = w_h . tanh(x) summed by the
//      same pairing tree as wave_sum's xor butterfly (a[i] += a[i + o], o = 32 .. 1, entries >= 49 zero),
//      so z is bit-identical to k_tr_atten's wave-cooperative sum, with no cross-lane dependence;
//   B: the two softmaxes, one wave per row, exactly as k_tr_atten;
//   C: the context of every row of the group, one fma chain over k per column, and u = c_hat + h.
// V_b and VWv_b are read once per group instead of once per row (2304 x 100 KB per training step at
// B = 128, T = 18), and the rows' scores run side by side rather than one wave-reduction at a time:
// bit-identical outputs to k_tr_atten.
constexpr int TRA_TS = 32;  // steps per group, at most
template <int H>
__global__ __launch_bounds__(H) void k_tr_atten_img(int B, int T, int TS, const float* __restrict__ PG,
                                                    const float* __restrict__ PS, const float* __restrict__ VWv,
                                                    const float* __restrict__ Vf, const float* __restrict__ wh,
                                                    const float* __restrict__ Hs, const float* __restrict__ S,
                                                    float* __restrict__ alpha, float* __restrict__ beta,
                                                    float* __restrict__ ctx, float* __restrict__ U) {
  constexpr int NW = H / 64;
  __shared__ float s_vwv[P * PP], s_wh[PP], s_pg[TRA_TS][PP], s_ps[TRA_TS][PP], s_z[TRA_TS][PP], s_al[TRA_TS][PP];
  __shared__ float s_be[TRA_TS];
  const int b = blockIdx.x, t0 = blockIdx.y * TS, t1 = t0 + TS < T ? t0 + TS : T, n = t1 - t0;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (n <= 0) return;
  float v[P];
  const float* vb = Vf + (int64_t)b * P * H;
#pragma unroll
  for (int k = 0; k < P; ++k) v[k] = vb[(int64_t)k * H + t];
  for (int e = t; e < P * PP; e += H) s_vwv[e] = VWv[(int64_t)b * P * PP + e];
  if (t < PP) s_wh[t] = t < P ? wh[t] : 0.f;
  for (int e = t; e < n * PP; e += H) {
    const int i = e / PP, j = e - i * PP;
    const int64_t r = (int64_t)(t0 + i) * B + b;
    s_pg[i][j] = PG[r * PP + j];
    s_ps[i][j] = PS[r * PP + j];
  }
  __syncthreads();
  // A: scores, one (row, item) per thread
  for (int q = t; q < n * (P + 1); q += H) {
    const int i = q / (P + 1), k = q - i * (P + 1);
    const float* xs = k < P ? &s_vwv[k * PP] : &s_ps[i][0];
    float a[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) a[j] = j < P ? s_wh[j] * tanhf(xs[j] + s_pg[i][j]) : 0.f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
      for (int j = 0; j < o; ++j) a[j] = a[j] + a[j + o];
    s_z[i][k] = a[0];
  }
  __syncthreads();
  // B: softmax_49 (alpha) and softmax_50 (beta = its last entry), one wave per row
  for (int i = w; i < n; i += NW) {
    const int64_t r = (int64_t)(t0 + i) * B + b;
    const float z = lane < P ? s_z[i][lane] : -INFINITY;
    const float m = wave_max(z);
    const float e = lane < P ? expf(z - m) : 0.f;
    const float al = e / wave_sum(e);
    if (lane < P) {
      s_al[i][lane] = al;
      alpha[r * PP + lane] = al;
    }
    const float zsn = s_z[i][P];
    const float m2 = fmaxf(m, zsn);
    const float e2 = lane < P ? expf(z - m2) : 0.f;
    const float es = expf(zsn - m2);
    const float S2 = wave_sum(e2) + es;
    if (lane == 0) {
      s_be[i] = es / S2;
      beta[r] = es / S2;
    }
  }
  __syncthreads();
  // C: context and u for every row of the group (column t)
  for (int i = 0; i < n; ++i) {
    const int64_t r = (int64_t)(t0 + i) * B + b;
    const float sv = S[r * H + t], hv = Hs[r * H + t];
    float c = 0.f;
#pragma unroll
    for (int k = 0; k < P; ++k) c = __builtin_fmaf(s_al[i][k], v[k], c);
    ctx[r * H + t] = c;
    const float be = s_be[i];
    const float chat = be * sv + (1.f - be) * c;
    U[r * H + t] = chat + hv;
  }
}

// packed row map: prow[p] = t B + b for the rows of pack_padded_sequence (lengths sorted desc)
__global__ void k_tr_prow(const int* __restrict__ len, int B, int T, int* __restrict__ prow) {
  // one thread per (t, b); batch size of t = #{b : len[b] > t}; offset = sum of earlier sizes
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T) return;
  const int t = i / B, b = i % B;
  if (len[b] <= t) return;
  int off = 0;
  for (int tt = 0; tt < t; ++tt) {
    int lo = 0, hi = B;  // first b with len[b] <= tt
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (len[mid] > tt) lo = mid + 1;
      else hi = mid;
    }
    off += lo;
  }
  prow[off + b] = t * B + b;
}

// ---------------------------------------------------------------------------------------------
// backward pieces
// ---------------------------------------------------------------------------------------------
// Atten backward in two passes.  Nothing in it is sequential over t (dU for every step is known
// once the vocab backward has run); only the per-image sums over t are, so:
// k_tr_atb_row: one workgroup per row r = t B + b (t < len[b]; rows past a caption's length carry
//   no loss gradient), 256 threads, HPT = H / 256 columns per thread.  In: dU (= dc_hat; u = c_hat +
//   h also gives dh = dU directly), alpha, beta, ctx (c_t), S, PG, PS, VWv, V, w_h.  Out per row:
//   dS = beta dU, dPG, dPS (pitch PP), and for the per-image pass dz (pitch PP) and the row's w_h
//   gradient term dwr[j] = sum_k dz_k tanh_kj + dz_s tanh_s,j.
//     beta = softmax_50([z; z_s])[49]:  dz_k += -dbeta beta (1 - beta) alpha_k, dz_s = dbeta beta (1 - beta)
//     alpha = softmax_49(z):           dz_k += alpha_k (dalpha_k - <alpha, dalpha>)
// k_tr_atb_img: one workgroup per image: dV[b] = sum_t alpha_t (x) dc_t, dVWv[b] = sum_t dcontent_v,t
//   (tanh recomputed from VWv and PG), dwh_part[b] = sum_t dwr_t, each summed over t in the step
//   groups of atb_groups, chained within a group and the group sums added in group order -- the
//   arithmetic of the one-pass kernel this replaced (a workgroup per (image, step group), 237 us at
//   B = 128, T = 18), so the gradients are bit-identical to it.
template <int HPT>
__global__ __launch_bounds__(256) void k_tr_atb_row(int B, const int* __restrict__ len, const float* __restrict__ dU,
                                                    const float* __restrict__ alpha, const float* __restrict__ beta,
                                                    const float* __restrict__ ctx, const float* __restrict__ S,
                                                    const float* __restrict__ PG, const float* __restrict__ PS,
                                                    const float* __restrict__ VWv, const float* __restrict__ Vf,
                                                    const float* __restrict__ wh, float* __restrict__ dS,
                                                    float* __restrict__ dPG, float* __restrict__ dPS,
                                                    float* __restrict__ dz_out, float* __restrict__ dwr,
                                                    float* __restrict__ dH) {
  constexpr int H = 256 * HPT;
  __shared__ float s_al[PP], s_da[PP], s_dz[PP], s_red[4], s_dzs;
  __shared__ float s_dc[H];
  __shared__ float s_cv[P * P], s_tz[P * P];
  const int r = blockIdx.x, b = r % B, tt = r / B;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // dh = dU (u = c_hat + h; the recurrent GEMMs add into dH later): written here for every row, zero
  // for the rows past a caption's length (their dU is zero: no loss gradient)
  if (tt >= len[b]) {  // uniform over the workgroup
#pragma unroll
    for (int i = 0; i < HPT; ++i) dH[(int64_t)r * H + t + 256 * i] = 0.f;
    return;
  }
  const float* vb = Vf + (int64_t)b * P * H;
  const float whj = t < P ? wh[t] : 0.f;
  const float be = beta[r];
  float part = 0.f;
#pragma unroll
  for (int i = 0; i < HPT; ++i) {
    const int d = t + 256 * i;
    const float du = dU[(int64_t)r * H + d];
    dH[(int64_t)r * H + d] = du;
    part += du * (S[(int64_t)r * H + d] - ctx[(int64_t)r * H + d]);
    dS[(int64_t)r * H + d] = be * du;
    s_dc[d] = (1.f - be) * du;
  }
  part = wave_sum(part);
  if (lane == 0) s_red[w] = part;
  if (t < PP) s_al[t] = t < P ? alpha[(int64_t)r * PP + t] : 0.f;
  __syncthreads();
  const float dbeta = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
  for (int k = w; k < P; k += 4) {  // dalpha_k = dc . V_k
    float a = 0.f;
    for (int d = lane; d < H; d += 64) a = __builtin_fmaf(s_dc[d], vb[(int64_t)k * H + d], a);
    a = wave_sum(a);
    if (lane == 0) s_da[k] = a;
  }
  __syncthreads();
  if (w == 0) {
    const float a = lane < P ? s_al[lane] : 0.f;
    const float da = lane < P ? s_da[lane] : 0.f;
    const float dot = wave_sum(a * da);
    const float dzb = dbeta * be * (1.f - be);
    const float dz = a * (da - dot) - dzb * a;
    if (lane < P) {
      s_dz[lane] = dz;
      dz_out[(int64_t)r * PP + lane] = dz;
    }
    if (lane == 0) s_dzs = dzb;
  }
  __syncthreads();
  // content_v[k][j] = VWv[b][k][j] + PG[j]: entries e = k * 49 + j spread over the threads
  const float* pgr = PG + (int64_t)r * PP;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int e = t + 256 * i;
    if (e < P * P) {
      const int k = e / P, j = e - k * P;
      const float th = tanhf(VWv[((int64_t)b * P + k) * PP + j] + pgr[j]);
      s_cv[e] = s_dz[k] * wh[j] * (1.f - th * th);
      s_tz[e] = s_dz[k] * th;
    }
  }
  __syncthreads();
  if (t < P) {  // column j: dPG[j] = sum_k dcv[k][j] + dcs[j]; dwr[j] = sum_k dz_k tanh + dz_s tanh_s
    const int j = t;
    float sdcv = 0.f, sdw = 0.f;
    for (int k = 0; k < P; ++k) {
      sdcv += s_cv[k * P + j];
      sdw += s_tz[k * P + j];
    }
    const float ths = tanhf(PS[(int64_t)r * PP + j] + pgr[j]);
    const float dcs = s_dzs * whj * (1.f - ths * ths);
    dPS[(int64_t)r * PP + j] = dcs;
    dPG[(int64_t)r * PP + j] = sdcv + dcs;
    dwr[(int64_t)r * PP + j] = sdw + s_dzs * ths;
  }
}

// grid (B, HPT + 1): y < HPT -> dV columns 256 y + t; y = HPT -> dVWv and dwh_part
template <int HPT>
__global__ __launch_bounds__(256) void k_tr_atb_img(int B, int TS, int G, const int* __restrict__ len,
                                                    const float* __restrict__ dU, const float* __restrict__ alpha,
                                                    const float* __restrict__ beta, const float* __restrict__ PG,
                                                    const float* __restrict__ VWv, const float* __restrict__ wh,
                                                    const float* __restrict__ dz_in, const float* __restrict__ dwr,
                                                    float* __restrict__ dV, float* __restrict__ dVWv,
                                                    float* __restrict__ dwh_part) {
  constexpr int H = 256 * HPT;
  __shared__ float s_al[PP], s_dz[PP], s_pg[PP];
  const int b = blockIdx.x, role = blockIdx.y, t = threadIdx.x, n = len[b];
  if (role < HPT) {  // dV[b][k][d] = sum_t alpha_t,k dc_t,d
    const int d = t + 256 * role;
    float tot[P], acc[P];
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int k = 0; k < P; ++k) acc[k] = 0.f;
      const int nt = min(n, (g + 1) * TS);
      for (int tt = g * TS; tt < nt; ++tt) {
        const int r = tt * B + b;
        __syncthreads();  // the previous step's alpha was read
        if (t < PP) s_al[t] = t < P ? alpha[(int64_t)r * PP + t] : 0.f;
        const float dc = (1.f - beta[r]) * dU[(int64_t)r * H + d];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < P; ++k) acc[k] = __builtin_fmaf(s_al[k], dc, acc[k]);
      }
      // group sums added in group order (as the group partials were summed: the first taken as is)
#pragma unroll
      for (int k = 0; k < P; ++k) tot[k] = g == 0 ? acc[k] : tot[k] + acc[k];
    }
#pragma unroll
    for (int k = 0; k < P; ++k) dV[((int64_t)b * P + k) * H + d] = tot[k];
    return;
  }
  float dvwv_tot[10], dvwv_acc[10], vwv[10], whv[10];
  float dwh_tot = 0.f, dwh_acc = 0.f;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int e = t + 256 * i, ec = e < P * P ? e : 0, k = ec / P, j = ec - k * P;
    vwv[i] = VWv[((int64_t)b * P + k) * PP + j];
    whv[i] = wh[j];
  }
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int i = 0; i < 10; ++i) dvwv_acc[i] = 0.f;
    dwh_acc = 0.f;
    const int nt = min(n, (g + 1) * TS);
    for (int tt = g * TS; tt < nt; ++tt) {
      const int r = tt * B + b;
      __syncthreads();
      if (t < PP) {
        s_dz[t] = t < P ? dz_in[(int64_t)r * PP + t] : 0.f;
        s_pg[t] = t < P ? PG[(int64_t)r * PP + t] : 0.f;
      }
      if (t < P) dwh_acc += dwr[(int64_t)r * PP + t];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 10; ++i) {
        const int e = t + 256 * i;
        if (e < P * P) {
          const int k = e / P, j = e - k * P;
          const float th = tanhf(vwv[i] + s_pg[j]);
          dvwv_acc[i] += s_dz[k] * whv[i] * (1.f - th * th);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 10; ++i) dvwv_tot[i] = g == 0 ? dvwv_acc[i] : dvwv_tot[i] + dvwv_acc[i];
    dwh_tot = g == 0 ? dwh_acc : dwh_tot + dwh_acc;
  }
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const int e = t + 256 * i;
    if (e < P * P) dVWv[((int64_t)b * P + e / P) * PP + e % P] = dvwv_tot[i];
  }
  if (t < P) dwh_part[(int64_t)b * PP + t] = dwh_tot;
}

// copy a [rows][cols] matrix into pitch `pitch` (zero padding)
// (and, for the bf16 step's k_bgemm, the same matrix rounded to bf16: dstb, same pitch)
__global__ void k_pad_rows(const float* __restrict__ src, int rows, int cols, int pitch, float* __restrict__ dst,
                           __bf16* __restrict__ dstb = nullptr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)rows * pitch) return;
  const int r = (int)(i / pitch), c = (int)(i % pitch);
  const float v = c < cols ? src[(int64_t)r * cols + c] : 0.f;
  if (dst) dst[i] = v;
  if (dstb) dstb[i] = (__bf16)v;
}

// bf16 steps: dscores [rows][cols] -> bf16 [rows][pitch] (zero columns past cols), with the column
// sums of the bias gradient db_m taken on the way: thread = column n, grid.y = the 64 row chunks of
// k_colsum, each chunk summed in row order into part[chunk][n] -- k_colsum's arithmetic on the same
// values (k_colsum_fin then adds the chunks in order), so db_m is bit-identical and dscores is read
// once instead of twice
__global__ void k_pad_rows_colsum(const float* __restrict__ src, int rows, int cols, int pitch,
                                  __bf16* __restrict__ dstb, float* __restrict__ part) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, ch = blockIdx.y;
  if (n >= pitch) return;
  const int per = (rows + CS_CH - 1) / CS_CH, m0 = ch * per, m1 = m0 + per < rows ? m0 + per : rows;
  float s = 0.f;
  for (int m = m0; m < m1; ++m) {
    const float v = n < cols ? src[(int64_t)m * cols + n] : 0.f;
    dstb[(int64_t)m * pitch + n] = (__bf16)v;
    s += v;
  }
  if (n < cols) part[(int64_t)ch * cols + n] = s;
}

// gather rows: dst[i] = src[rows[i]]
__global__ void k_gather_rows(const float* __restrict__ src, const int* __restrict__ rows, int n, int cols,
                              float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * cols) return;
  const int r = (int)(i / cols), c = (int)(i % cols);
  dst[i] = src[(int64_t)rows[r] * cols + c];
}

// sentinel backward: s = SG * tanh(c): dG = dS tanh(c) SG (1 - SG); dC += dS SG (1 - tanh(c)^2)
__global__ void k_tr_sent_bwd(const float* __restrict__ dS, const float* __restrict__ SG, const float* __restrict__ Cs,
                              float* __restrict__ dG, float* __restrict__ dC, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float sg = SG[i], tc = tanhf(Cs[i]), ds = dS[i];
  dG[i] = ds * tc * sg * (1.f - sg);
  dC[i] = ds * sg * (1.f - tc * tc);
}

// LSTM cell backward of step t (rows b < B): dh = dH[t] + dh_rec, dc = dC[t] + dc_rec; writes DG[t]
// (pre-activation gate grads) and dc_rec <- dc * f.  The later step's recurrent GEMM dh_rec =
// DG_{t+1} W_hh is folded in: dh_rec (b, j) = sk_sum(src, S, B H, .), S = 0 at the last step
// (dh_rec = 0) -- bit-identical to k_tgemm_reduce followed by a plain cell-backward kernel
__global__ void k_tr_cell_bwd_sk(const float* __restrict__ dH, const float* __restrict__ dC, const float* __restrict__ src,
                                 int S, float* __restrict__ dc_rec, const float* __restrict__ GA,
                                 const float* __restrict__ c_t, const float* __restrict__ c_prev, int B, int H,
                                 float* __restrict__ DG) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * H) return;
  const int b = (int)(i / H), j = (int)(i % H);
  const float* ga = GA + (int64_t)b * 4 * H;
  const float i_ = ga[j], f_ = ga[H + j], g_ = ga[2 * H + j], o_ = ga[3 * H + j];
  const float c = c_t[i], tc = tanhf(c);
  const float dh = dH[i] + (S > 0 ? sk_sum(src, S, (int64_t)B * H, i) : 0.f);
  float dc = dC[i] + dc_rec[i] + dh * o_ * (1.f - tc * tc);
  const float d_o = dh * tc;
  const float d_i = dc * g_, d_g = dc * i_, d_f = dc * c_prev[i];
  float* dg = DG + (int64_t)b * 4 * H;
  dg[j] = d_i * i_ * (1.f - i_);
  dg[H + j] = d_f * f_ * (1.f - f_);
  dg[2 * H + j] = d_g * (1.f - g_ * g_);
  dg[3 * H + j] = d_o * o_ * (1.f - o_);
  dc_rec[i] = dc * f_;
}

// ---------------------------------------------------------------------------------------------
// Fused recurrent LSTM steps (bf16 steps): ONE launch per timestep, forward and backward through
// time, in place of a split-K k_tgemm<true> of h_{t-1} W_hh^T (or DG_{t+1} W_hh) plus a cell kernel
// that sums its partials (k_tr_cell_sk / k_tr_cell_bwd_sk: two launches and a partial-slab round
// trip per step).  A workgroup owns 16 rows and 16 hidden units (all four gates of them, so the
// cell runs in its epilogue); the grid is ceil(B/16) x H/16 workgroups, unit group fastest, so the
// workgroups that read one W slice share an XCD.  The GEMM runs on v_mfma_f32_16x16x32_bf16 (bf16
// operands, RNE -- the rounding k_tgemm<true> applies while staging -- and fp32 accumulation) with K
// split over the 4 waves; every operand fragment is loaded straight into registers (16 B per lane,
// all of a wave's loads issued together: a step is a few dependent round trips, not a byte budget),
// and the 4 partial tiles are summed in LDS in a fixed order ((w0 + w1) + (w2 + w3)): deterministic.
// Operands come pre-packed: W_hh once per call as 16x16x32 B-fragments (k_pk_whh), h_t / DG_t as
// bf16 row copies written by the previous step's epilogue (the fp32 ones stay for the weight
// gradients).  The persistent alternative (W_hh resident in LDS across all T steps, a grid barrier
// per step) was priced and not built: DESIGN.md §9.
// ---------------------------------------------------------------------------------------------
typedef float floatx4 __attribute__((ext_vector_type(4)));

// W_hh [4H][H] fp32 -> bf16 16x16x32 B-fragments (lane l, element e).  mode 0 (forward, gates):
// whf[ug][g][kc][l][e] = W_hh[g H + 16 ug + (l & 15)][32 kc + 8 (l >> 4) + e]; mode 1 (backward,
// W_hh^T): whb[ug][kc][l][e] = W_hh[32 kc + 8 (l >> 4) + e][16 ug + (l & 15)], kc < 4H / 32.
__global__ void k_pk_whh(const float* __restrict__ w, int H, int mode, bf16x8* __restrict__ out) {
  const int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= (int64_t)4 * H * H / 8) return;
  const int l = (int)(f & 63);
  const int64_t q = f >> 6;
  bf16x8 v;
  if (mode == 0) {
    const int KC = H / 32, kc = (int)(q % KC), g = (int)((q / KC) % 4), ug = (int)(q / (4 * KC));
    const float* src = w + (int64_t)(g * H + 16 * ug + (l & 15)) * H + 32 * kc + 8 * (l >> 4);
    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
    v[0] = (__bf16)a.x; v[1] = (__bf16)a.y; v[2] = (__bf16)a.z; v[3] = (__bf16)a.w;
    v[4] = (__bf16)b.x; v[5] = (__bf16)b.y; v[6] = (__bf16)b.z; v[7] = (__bf16)b.w;
  } else {
    const int KC4 = 4 * H / 32, kc = (int)(q % KC4), ug = (int)(q / KC4);
    const float* src = w + (int64_t)(32 * kc + 8 * (l >> 4)) * H + 16 * ug + (l & 15);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (__bf16)src[(int64_t)e * H];
  }
  out[f] = v;
}

// Forward step t: gates = h_{t-1} W_hh^T + PRE[t] (x W_ih^T + b_ih + b_hh), then the cell exactly as
// k_tr_cell_sk (same expression order), writing h, c, the activated gates GA and h in bf16 (the
// next step's operand).  AF32: h_{t-1} is fp32 (t = 0: h0 from the encoder), else bf16.
template <int H, bool AF32>
__global__ __launch_bounds__(256) void k_tr_lstm_f(int B, const void* __restrict__ hprev, const float* __restrict__ PRE,
                                                   int ldp, const float* __restrict__ c_prev,
                                                   const bf16x8* __restrict__ whf, float* __restrict__ h_out,
                                                   float* __restrict__ c_out, float* __restrict__ GA,
                                                   __bf16* __restrict__ hb_out) {
  constexpr int NUG = H / 16, KC = H / 32, PER = KC / 4;
  __shared__ float red[4][4][16][17];  // [wave][gate][row][unit]
  const int ug = blockIdx.x % NUG, m0 = (blockIdx.x / NUG) * 16;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int kc0 = w * PER;
  const int arow = m0 + (lane & 15) < B ? m0 + (lane & 15) : B - 1;
  bf16x8 fw[4][PER], fa[PER];
  const bf16x8* ws = whf + (size_t)ug * 4 * KC * 64 + lane;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < PER; ++i) fw[g][i] = ws[((size_t)g * KC + kc0 + i) * 64];
  if constexpr (AF32) {
    const float* hp = static_cast<const float*>(hprev) + (int64_t)arow * H + 8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const float4 a = *reinterpret_cast<const float4*>(hp + 32 * (kc0 + i));
      const float4 b = *reinterpret_cast<const float4*>(hp + 32 * (kc0 + i) + 4);
      fa[i][0] = (__bf16)a.x; fa[i][1] = (__bf16)a.y; fa[i][2] = (__bf16)a.z; fa[i][3] = (__bf16)a.w;
      fa[i][4] = (__bf16)b.x; fa[i][5] = (__bf16)b.y; fa[i][6] = (__bf16)b.z; fa[i][7] = (__bf16)b.w;
    }
  } else {
    const __bf16* hp = static_cast<const __bf16*>(hprev) + (int64_t)arow * H + 8 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < PER; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(hp + 32 * (kc0 + i));
  }
  floatx4 acc[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) acc[g] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < PER; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fw[g][i], acc[g], 0, 0, 0);
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][g][4 * (lane >> 4) + i][lane & 15] = acc[g][i];
  __syncthreads();
  const int r = t >> 4, u = t & 15, m = m0 + r;
  if (m >= B) return;
  float G[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) G[g] = (red[0][g][r][u] + red[1][g][r][u]) + (red[2][g][r][u] + red[3][g][r][u]);
  const int j = 16 * ug + u;
  const float* p = PRE + (int64_t)m * ldp;
  const float gi = G[0] + p[j], gf = G[1] + p[H + j], gg = G[2] + p[2 * H + j], go = G[3] + p[3 * H + j];
  const float i_ = sigmoidf_(gi), f_ = sigmoidf_(gf), g_ = tanhf(gg), o_ = sigmoidf_(go);
  const int64_t i = (int64_t)m * H + j;
  const float c = f_ * c_prev[i] + i_ * g_;
  const float h = o_ * tanhf(c);
  c_out[i] = c;
  h_out[i] = h;
  hb_out[i] = (__bf16)h;
  float* ga = GA + (int64_t)m * 4 * H;
  ga[j] = i_; ga[H + j] = f_; ga[2 * H + j] = g_; ga[3 * H + j] = o_;
}

// Backward step t (reverse order): dh_rec = DG_{t+1} W_hh for the workgroup's 16 rows x 16 units (K =
// 4H over the 4 waves; LAST: t = T - 1, no later step, dh_rec = 0 and no GEMM), then the cell
// backward exactly as k_tr_cell_bwd_sk, writing DG_t (fp32, for the weight gradients, and bf16, the
// next backward step's operand) and dc_rec <- dc f.
template <int H, bool LAST>
__global__ __launch_bounds__(256) void k_tr_lstm_b(int B, const __bf16* __restrict__ dgb_next,
                                                   const bf16x8* __restrict__ whb, const float* __restrict__ dH,
                                                   const float* __restrict__ dC, float* __restrict__ dc_rec,
                                                   const float* __restrict__ GA, const float* __restrict__ c_t,
                                                   const float* __restrict__ c_prev, float* __restrict__ DG,
                                                   __bf16* __restrict__ dgb_out) {
  constexpr int NUG = H / 16, KC = 4 * H / 32, PER = KC / 4;
  __shared__ float red[4][16][17];  // [wave][row][unit]
  const int ug = blockIdx.x % NUG, m0 = (blockIdx.x / NUG) * 16;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if constexpr (!LAST) {
    const int kc0 = w * PER;
    const int arow = m0 + (lane & 15) < B ? m0 + (lane & 15) : B - 1;
    bf16x8 fw[PER], fa[PER];
    const bf16x8* ws = whb + ((size_t)ug * KC + kc0) * 64 + lane;
    const __bf16* ap = dgb_next + (int64_t)arow * 4 * H + 8 * (lane >> 4) + 32 * kc0;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      fw[i] = ws[(size_t)i * 64];
      fa[i] = *reinterpret_cast<const bf16x8*>(ap + 32 * i);
    }
    floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PER; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fw[i], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][4 * (lane >> 4) + i][lane & 15] = acc[i];
    __syncthreads();
  }
  const int r = t >> 4, u = t & 15, m = m0 + r;
  if (m >= B) return;
  const float dhr = LAST ? 0.f : (red[0][r][u] + red[1][r][u]) + (red[2][r][u] + red[3][r][u]);
  const int j = 16 * ug + u;
  const int64_t i = (int64_t)m * H + j;
  const float* ga = GA + (int64_t)m * 4 * H;
  const float i_ = ga[j], f_ = ga[H + j], g_ = ga[2 * H + j], o_ = ga[3 * H + j];
  const float c = c_t[i], tc = tanhf(c);
  const float dh = dH[i] + dhr;
  float dc = dC[i] + dc_rec[i] + dh * o_ * (1.f - tc * tc);
  const float d_o = dh * tc;
  const float d_i = dc * g_, d_g = dc * i_, d_f = dc * c_prev[i];
  const float v0 = d_i * i_ * (1.f - i_), v1 = d_f * f_ * (1.f - f_), v2 = d_g * (1.f - g_ * g_), v3 = d_o * o_ * (1.f - o_);
  float* dg = DG + (int64_t)m * 4 * H;
  dg[j] = v0; dg[H + j] = v1; dg[2 * H + j] = v2; dg[3 * H + j] = v3;
  __bf16* db = dgb_out + (int64_t)m * 4 * H;
  db[j] = (__bf16)v0; db[H + j] = (__bf16)v1; db[2 * H + j] = (__bf16)v2; db[3 * H + j] = (__bf16)v3;
  dc_rec[i] = dc * f_;
}

// embedding gradient dE[v] = sum over rows r (t-major) with tok(r) == v of dX[r][0:E], in r order:
// k_tok_rank: rank of r among the earlier rows with its token (and the token's count via the
// first occurrence); k_tok_place: position in a token-sorted list; k_tr_embed_bwd: one
// workgroup per row of that list that starts a token's run sums the run in order.
__device__ __forceinline__ int tok_of(const int64_t* tok, int tld, int B, int V, int r) {
  const int t = r / B, b = r % B;
  int64_t tk = tok[(int64_t)b * tld + t];
  return (int)(tk < 0 ? 0 : (tk >= V ? V - 1 : tk));
}
// one wave per row r: the 64 lanes stride over all R rows, counting (ballot + popcount) the rows
// with r's token before r, in total, and the rows with a smaller token (a thread per row looping
// over all R rows ran on R / 256 workgroups: 69 us at R = 2304)
__global__ __launch_bounds__(256) void k_tok_rank(const int64_t* __restrict__ tok, int tld, int B, int R, int V,
                                                  int* __restrict__ rank, int* __restrict__ count,
                                                  int* __restrict__ before_tok) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;  // wave-uniform
  const int v = tok_of(tok, tld, B, V, r);
  int before = 0, total = 0, smaller = 0;
  for (int i0 = 0; i0 < R; i0 += 64) {
    const int i = i0 + lane;
    const int u = i < R ? tok_of(tok, tld, B, V, i) : -1;
    const bool same = i < R && u == v;
    total += __popcll(__ballot(same));
    before += __popcll(__ballot(same && i < r));
    smaller += __popcll(__ballot(i < R && u < v));
  }
  if (lane == 0) {
    rank[r] = before;
    count[r] = total;
    before_tok[r] = smaller;
  }
}
// order[p]: rows sorted by (token, r)
__global__ void k_tok_place(int R, const int* __restrict__ rank, const int* __restrict__ before_tok,
                            int* __restrict__ order) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) order[before_tok[r] + rank[r]] = r;
}
__global__ void k_tr_embed_bwd(const int64_t* __restrict__ tok, int tld, int B, int R, int V,
                               const int* __restrict__ order, const int* __restrict__ rank,
                               const int* __restrict__ count, const float* __restrict__ dX, int E,
                               float* __restrict__ dE) {
  const int p = blockIdx.x;  // a position in the sorted list
  const int r0 = order[p];
  if (rank[r0] != 0) return;  // not the first row of its token's run
  const int v = tok_of(tok, tld, B, V, r0), n = count[r0];
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < n; ++i) s += dX[(int64_t)order[p + i] * 2 * E + e];
    dE[(int64_t)v * E + e] = s;
  }
}

// dv_g[b] = sum_t dX[t B + b][E:2E] (in t order), then relu'(v_g)
__global__ void k_tr_vg_bwd(const float* __restrict__ dX, const float* __restrict__ vg, int B, int T, int E,
                            float* __restrict__ dvg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * E) return;
  const int b = (int)(i / E), e = (int)(i % E);
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += dX[((int64_t)t * B + b) * 2 * E + E + e];
  dvg[i] = vg[i] > 0.f ? s : 0.f;
}

// dL/dA for the trunk (NCHW, baseline_attention.py:43-51): dfeats[b][c][p] = dA[b*49 + p][c] +
// dag[b][c] / 49 (AvgPool2d(7)'s gradient spreads d a_g evenly).  Tiles of 49 x 64 through LDS so
// both the read (along c) and the write (along p) are coalesced.
__global__ __launch_bounds__(256) void k_dfeats(const float* __restrict__ dA, const float* __restrict__ dag, int C,
                                                float* __restrict__ dfeats) {
  __shared__ float tile[P][65];
  const int b = blockIdx.y, c0 = blockIdx.x * 64, t = threadIdx.x;
  for (int i = t; i < P * 64; i += 256) {
    const int p = i / 64, c = i % 64;
    tile[p][c] = c0 + c < C ? dA[((int64_t)b * P + p) * C + c0 + c] : 0.f;
  }
  __syncthreads();
  for (int i = t; i < 64 * P; i += 256) {
    const int c = i / P, p = i % P;
    if (c0 + c < C) dfeats[((int64_t)b * C + c0 + c) * P + p] = tile[p][c] + dag[(int64_t)b * C + c0 + c] / 49.f;
  }
}

// elementwise helpers
__global__ void k_relu_mask(float* __restrict__ d, const float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !(y[i] > 0.f)) d[i] = 0.f;
}
__global__ void k_tanh_bwd(float* __restrict__ d, const float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] = d[i] * (1.f - y[i] * y[i]);
}
// [rows][PP] -> [P], each column summed in row order; the rows' values are loaded by all 256
// threads first (one thread looping over the rows waited for every load in turn: 30 us at 128 rows)
constexpr int RS_ROWS = 256;  // rows staged per LDS pass
__global__ __launch_bounds__(256) void k_rowsum_pp(const float* __restrict__ X, int rows, float* __restrict__ out) {
  __shared__ float xs[RS_ROWS * P];
  const int t = threadIdx.x;
  float s = 0.f;
  for (int r0 = 0; r0 < rows; r0 += RS_ROWS) {
    const int n = rows - r0 < RS_ROWS ? rows - r0 : RS_ROWS;
    __syncthreads();
    for (int i = t; i < n * P; i += 256) xs[i] = X[(int64_t)(r0 + i / P) * PP + i % P];
    __syncthreads();
    if (t < P)
      for (int r = 0; r < n; ++r) s += xs[r * P + t];
  }
  if (t < P) out[t] = s;
}

}  // namespace aa

// ---------------------------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------------------------
constexpr size_t TR_SPLIT_FLOATS = (size_t)16 << 20;  // 64 MB split-K scratch (k_bgemm's splits of dU / dW_a)

// Transposed copies of weights, several matrices per launch: dst_i[c][r] = src_i[r][c] (src row-major
// [rows][cols], dst [cols][ld], zero for rows <= r < ld), 64 x 64 tiles through LDS (reads along c, writes
// along r, both coalesced).  Exact copies: a GEMM reading the copy along K multiplies the same values in
// the same order as one reading the original down its columns.
constexpr int WT_MAX = 8;
constexpr int WT_LDP = (aa::P + 3) / 4 * 4;  // the [H][P] copies: rows padded to whole 16-B groups
struct WTArgs {
  int n;
  const float* src[WT_MAX];
  float* dst[WT_MAX];
  int rows[WT_MAX], cols[WT_MAX], ld[WT_MAX];
  int blk0[WT_MAX + 1];  // first tile of matrix i
};
__global__ __launch_bounds__(256) void k_wT(WTArgs a) {
  __shared__ float tile[64][65];
  int i = 0;
  while (i + 1 < a.n && (int)blockIdx.x >= a.blk0[i + 1]) ++i;
  const int tb = blockIdx.x - a.blk0[i], rows = a.rows[i], cols = a.cols[i], ld = a.ld[i];
  const int tr = (ld + 63) / 64;
  const int r0 = (tb % tr) * 64, c0 = (tb / tr) * 64, t = threadIdx.x;
  const float* __restrict__ src = a.src[i];
  float* __restrict__ dst = a.dst[i];
  for (int j = t; j < 64 * 64; j += 256) {
    const int rr = j / 64, cc = j % 64, r = r0 + rr, c = c0 + cc;
    tile[rr][cc] = (r < rows && c < cols) ? src[(int64_t)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int j = t; j < 64 * 64; j += 256) {
    const int cc = j / 64, rr = j % 64, c = c0 + cc, r = r0 + rr;
    if (c < cols && r < ld) dst[(int64_t)c * ld + r] = tile[rr][cc];
  }
}

struct TrainWS {
  float *a_g, *V, *vg, *h0, *c0, *VWv, *X, *PRE, *G4, *GA, *Hs, *Cs, *SG, *S, *PG, *PS, *alpha, *beta, *ctx, *U;
  int* prow;
  // backward scratch
  float *Up, *dU, *dS, *dPG, *dPS, *dV, *dVWv, *dwh, *dH, *dC, *dG, *DG, *dX, *dh_rec, *dc_rec, *dvg, *csum, *gsplit, *dsp;
  float *gsplit2, *csum2;  // the aux stream's split-K and column-sum scratch (Fork)
  float *dA, *dag;  // d(features) pieces: through V [B*49][C] and through a_g [B][C]
  float *dz, *dwr;  // per-row dz and w_h-gradient terms of k_tr_atb_row, summed per image by k_tr_atb_img
  // bf16 operands of the large GEMMs (AA_TRAIN_BF16, k_bgemm): U_p, W_m, dS (rows), W_m^T, dS^T, U_p^T,
  // dV^T, the feature map as [C][B 49]
  __bf16 *ub, *wmb, *dspb, *wmT, *dspT, *upT, *dvT, *ftT, *ftC;
  // fused recurrent steps (bf16): W_hh as forward / backward B-fragments, h_t and DG_t ping-pong bf16 copies
  bf16x8 *whf, *whb;
  __bf16 *hb[2], *dgb[2];
  int *trank, *tcount, *torder, *tsmall;
  // the weights the backward multiplies by untransposed (dx = dG W), stored transposed [in][out] by
  // the forward (k_wT, on aux): the backward's GEMMs then read both operands along K
  float *wgT, *wsT, *wvT, *wxT, *whT, *whhT, *wihT;
};

// step groups of the attention backward's per-image sums over t (k_tr_atb_img; they were the
// (image, group) workgroups of the one-pass kernel, sized to cover the chip at small B)
static void atb_groups(int B, int T, int* G, int* TS) {
  int g = B > 0 ? (512 + B - 1) / B : 1;
  g = g < T ? g : T;
  g = g > 1 ? g : 1;
  *TS = (T + g - 1) / g;
  *G = *TS > 0 ? (T + *TS - 1) / *TS : 1;
}

static TrainWS carve_train(char* base, const aa_dims& d, int B, int T, int Nmax, size_t* bytes) {
  Carver c{base};
  const size_t H = d.hidden, E = d.embed, Cc = d.channels, R = (size_t)T * B, P_ = aa::P, PP_ = aa::PP;
  TrainWS w;
  w.a_g = c.take<float>(B * Cc);
  w.V = c.take<float>(B * P_ * H);
  w.vg = c.take<float>(B * E);
  w.h0 = c.take<float>(B * H);
  w.c0 = c.take<float>(B * H);
  w.VWv = c.take<float>(B * P_ * PP_);
  w.X = c.take<float>(R * 2 * E);
  w.PRE = c.take<float>(R * 5 * H);
  w.G4 = c.take<float>(B * 4 * H);
  w.GA = c.take<float>(R * 4 * H);
  w.Hs = c.take<float>(R * H);
  w.Cs = c.take<float>(R * H);
  w.SG = c.take<float>(R * H);
  w.S = c.take<float>(R * H);
  w.PG = c.take<float>(R * PP_);
  w.PS = c.take<float>(R * PP_);
  w.alpha = c.take<float>(R * PP_);
  w.beta = c.take<float>(R);
  w.ctx = c.take<float>(R * H);
  w.U = c.take<float>(R * H);
  w.prow = c.take<int>(R);
  w.Up = c.take<float>((size_t)Nmax * H);
  w.dU = c.take<float>(R * H);
  w.dS = c.take<float>(R * H);
  w.dPG = c.take<float>(R * PP_);
  w.dPS = c.take<float>(R * PP_);
  w.dV = c.take<float>(B * P_ * H);
  w.dVWv = c.take<float>(B * P_ * PP_);
  w.dwh = c.take<float>(B * PP_);
  w.dH = c.take<float>(R * H);
  w.dC = c.take<float>(R * H);
  w.dG = c.take<float>(R * H);
  w.DG = c.take<float>(R * 4 * H);
  w.dX = c.take<float>(R * 2 * E);
  w.dh_rec = c.take<float>(B * H);
  w.dc_rec = c.take<float>(B * H);
  w.dvg = c.take<float>(B * E);
  w.dA = c.take<float>(B * P_ * Cc);
  w.dag = c.take<float>(B * Cc);
  w.csum = c.take<float>((size_t)CS_CH * (d.vocab > 4 * H ? d.vocab : 4 * H));
  w.trank = c.take<int>(R);
  w.gsplit = c.take<float>(TR_SPLIT_FLOATS);
  w.gsplit2 = c.take<float>(TR_SPLIT_FLOATS);
  w.csum2 = c.take<float>((size_t)CS_CH * (d.vocab > 4 * H ? d.vocab : 4 * H));
  w.dsp = c.take<float>(R * (size_t)((d.vocab + 63) / 64 * 64));
  w.tcount = c.take<int>(R);
  w.torder = c.take<int>(R);
  w.tsmall = c.take<int>(R);
  w.dz = c.take<float>(R * PP_);
  w.dwr = c.take<float>(R * PP_);
  {
    const size_t Kv = ((size_t)d.vocab + 63) / 64 * 64, Kr = (R + 63) / 64 * 64, Kb = ((size_t)B * P_ + 63) / 64 * 64;
    w.ub = c.take<__bf16>(R * H);
    w.wmb = c.take<__bf16>((size_t)d.vocab * H);
    w.dspb = c.take<__bf16>(R * Kv);
    // W_m^T [H][Kv] in the backward; the bf16 forward's encoder also packs W_a [H][C] here
    w.wmT = c.take<__bf16>(H * (Kv > Cc ? Kv : Cc));
    w.dspT = c.take<__bf16>((size_t)d.vocab * Kr);
    w.upT = c.take<__bf16>(H * Kr);
    w.dvT = c.take<__bf16>(H * Kb);
    w.ftT = c.take<__bf16>(Cc * Kb);
    w.ftC = c.take<__bf16>(Cc * Kb);  // [C][Kb]: the backward's dW_a operand, written by the forward's k_pk_feats3
    w.whf = c.take<bf16x8>(4 * H * H / 8);
    w.whb = c.take<bf16x8>(4 * H * H / 8);
    for (int i = 0; i < 2; ++i) {
      w.hb[i] = c.take<__bf16>((size_t)B * H);
      w.dgb[i] = c.take<__bf16>((size_t)B * 4 * H);
    }
  }
  w.wgT = c.take<float>(H * WT_LDP);
  w.wsT = c.take<float>(H * WT_LDP);
  w.wvT = c.take<float>(H * WT_LDP);
  w.wxT = c.take<float>(2 * E * H);
  w.whT = c.take<float>(H * H);
  w.whhT = c.take<float>(H * 4 * H);
  w.wihT = c.take<float>(2 * E * 4 * H);
  *bytes = c.off;
  return w;
}

static int train_check(const aa_dims* d, int B, int T) {
  if (!d) return AA_ERR_NULL;
  if (aa_check_dims(d) != AA_OK) return AA_ERR_DIMS;
  if (B < 0 || T < 0) return AA_ERR_SHAPE;
  if (2 * d->embed > 4096) return AA_ERR_DIMS;
  return AA_OK;
}

size_t aa_train_workspace_bytes(const aa_dims* d, int32_t B, int32_t T) {
  if (train_check(d, B, T) != AA_OK) return 0;
  size_t n;
  carve_train(nullptr, *d, B, T, B * T, &n);
  return n;
}

static inline unsigned nblk(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

// Decoder.forward over T teacher-forced steps (baseline_attention.py:148-194 with the adaptive
// block, adaptive_attention.py:110-134) from V, v_g, (h0, c0) already in the workspace: every
// activation of the T steps (Hs, Cs, S, alpha, beta, U = c_hat + h, ...) lands in ws, t-major.
// V and VWv = V W_v^T are the caller's: `join` (if set) makes the stream wait for them right before
// the attention, the first kernel that reads them.
static void decoder_core(const GemmCtx& gc, const aa_ref_weights* w, const TrainWS& s, const aa_dims& d, int B,
                         int T, const int64_t* tokens, int tok_ld, Fork* join = nullptr) {
  using namespace aa;
  const int H = d.hidden, E = d.embed, V = d.vocab, R = T * B;
  const hipStream_t st = gc.s;
  // x_t and the step-invariant input terms for all steps
  hipLaunchKernelGGL(k_tr_x, dim3(R), dim3(256), 0, st, tokens, tok_ld, w->embed_w, V, E, s.vg, B, T, s.X);
  tgemm(gc, R, 4 * H, 2 * E, s.X, 2 * E, 0, w->lstm_w_ih, 2 * E, 0, s.PRE, 5 * H, 0, w->lstm_b_ih, w->lstm_b_hh);
  tgemm(gc, R, H, 2 * E, s.X, 2 * E, 0, w->sent_affine_x_w, 2 * E, 0, s.PRE + 4 * H, 5 * H);
  // LSTM over T steps (baseline_attention.py:167-178)
  if (gc.bf16) {
    // one fused launch per step (k_tr_lstm_f), W_hh packed to bf16 fragments once
    hipLaunchKernelGGL(k_pk_whh, dim3(nblk((int64_t)4 * H * H / 8)), dim3(256), 0, st, w->lstm_w_hh, H, 0, s.whf);
    const unsigned grid = (unsigned)(((B + 15) / 16) * (H / 16));
    for (int t = 0; t < T; ++t) {
      const float* cp = t ? s.Cs + (size_t)(t - 1) * B * H : s.c0;
      const float* pre = s.PRE + (size_t)t * B * 5 * H;
      float *ho = s.Hs + (size_t)t * B * H, *co = s.Cs + (size_t)t * B * H, *ga = s.GA + (size_t)t * B * 4 * H;
#define AA_LF(H_)                                                                                                  \
  if (t == 0)                                                                                                      \
    hipLaunchKernelGGL((k_tr_lstm_f<H_, true>), dim3(grid), dim3(256), 0, st, B, (const void*)s.h0, pre, 5 * H, cp, \
                       s.whf, ho, co, ga, s.hb[0]);                                                              \
  else                                                                                                             \
    hipLaunchKernelGGL((k_tr_lstm_f<H_, false>), dim3(grid), dim3(256), 0, st, B, (const void*)s.hb[(t - 1) & 1],  \
                       pre, 5 * H, cp, s.whf, ho, co, ga, s.hb[t & 1])
      switch (H) {
        case 256: AA_LF(256); break;
        case 512: AA_LF(512); break;
        case 768: AA_LF(768); break;
        default: AA_LF(1024); break;
      }
#undef AA_LF
    }
  } else {
    for (int t = 0; t < T; ++t) {
      const float* hp = t ? s.Hs + (size_t)(t - 1) * B * H : s.h0;
      const float* cp = t ? s.Cs + (size_t)(t - 1) * B * H : s.c0;
      const int S = tgemm(gc, B, 4 * H, H, hp, H, 0, w->lstm_w_hh, H, 0, s.G4, 4 * H, 0, nullptr, nullptr, 0, nullptr,
                          nullptr, true);
      hipLaunchKernelGGL(k_tr_cell_sk, dim3(nblk((int64_t)B * H)), dim3(256), 0, st, S > 1 ? gc.split : s.G4, S,
                         s.PRE + (size_t)t * B * 5 * H, 5 * H, cp, B, H, s.Hs + (size_t)t * B * H,
                         s.Cs + (size_t)t * B * H, s.GA + (size_t)t * B * 4 * H);
    }
  }
  // sentinel (adaptive_attention.py:79-83, h_{t-1} = [0, h_0 .. h_{T-2}], :116-120)
  hipLaunchKernelGGL(k_copy_cols, dim3(nblk((int64_t)R * H)), dim3(256), 0, st, s.PRE, (int64_t)5 * H, 4 * H, s.SG,
                     (int64_t)H, R, H);
  tgemm(gc, R - B, H, H, s.Hs, H, 0, w->sent_affine_h_w, H, 0, s.SG + (size_t)B * H, H, 1);
  hipLaunchKernelGGL(k_tr_sent, dim3(nblk((int64_t)R * H)), dim3(256), 0, st, s.SG, s.Cs, s.S, (int64_t)R * H);
  // attention projections and the attention itself (adaptive_attention.py:26-58)
  tgemm(gc, R, P, H, s.Hs, H, 0, w->att_affine_g_w, H, 0, s.PG, PP);
  tgemm(gc, R, P, H, s.S, H, 0, w->att_affine_s_w, H, 0, s.PS, PP);
  if (join) join->to_main();
  static const bool tra_row = [] {  // AA_TRA_ROW=1: the per-row k_tr_atten (bitwise A/B of the two forms)
    const char* e = getenv("AA_TRA_ROW");
    return e && atoi(e) == 1;
  }();
  if (tra_row) {
    hipLaunchKernelGGL(k_tr_atten, dim3(R), dim3(256), 0, st, B, H, s.PG, s.PS, s.VWv, s.V, w->att_affine_h_w, s.Hs,
                       s.S, s.alpha, s.beta, s.ctx, s.U);
  } else {
    // rows grouped by image (V_b read once per group): groups of TS steps so that the grid covers
    // the chip (>= 256 workgroups when B is small)
    int G = B > 0 ? (256 + B - 1) / B : 1;
    G = G < T ? G : T;
    G = G > (T + TRA_TS - 1) / TRA_TS ? G : (T + TRA_TS - 1) / TRA_TS;  // at most TRA_TS steps per group
    const int TS = (T + G - 1) / G;
    G = (T + TS - 1) / TS;
#define AA_TRA(H_)                                                                                               \
  hipLaunchKernelGGL(k_tr_atten_img<H_>, dim3(B, G), dim3(H_), 0, st, B, T, TS, s.PG, s.PS, s.VWv, s.V,          \
                     w->att_affine_h_w, s.Hs, s.S, s.alpha, s.beta, s.ctx, s.U)
    switch (H) {
      case 256: AA_TRA(256); break;
      case 512: AA_TRA(512); break;
      case 768: AA_TRA(768); break;
      default: AA_TRA(1024); break;
    }
#undef AA_TRA
  }
}

int aa_train_forward(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B, int32_t T,
                     const int64_t* tokens, int32_t tok_ld, const int32_t* lengths, float* scores, int32_t N,
                     void* workspace, size_t workspace_bytes, int32_t flags, aa_stream_t stream) {
  return aa_train_forward_aux(w, dims, feats, B, T, tokens, tok_ld, lengths, scores, N, workspace, workspace_bytes,
                              flags, stream, nullptr);
}

int aa_train_forward_aux(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B, int32_t T,
                         const int64_t* tokens, int32_t tok_ld, const int32_t* lengths, float* scores, int32_t N,
                         void* workspace, size_t workspace_bytes, int32_t flags, aa_stream_t stream,
                         aa_stream_t aux) {
  using namespace aa;
  int rc = train_check(dims, B, T);
  if (rc) return rc;
  if (B == 0 || T == 0 || N == 0) return AA_OK;
  if (!w || !feats || !tokens || !lengths || !scores || !workspace || !w->sent_affine_h_w) return AA_ERR_NULL;
  if (N > B * T || tok_ld < T) return AA_ERR_SHAPE;
  size_t need;
  TrainWS s = carve_train(static_cast<char*>(workspace), *dims, B, T, B * T, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  const int H = dims->hidden, E = dims->embed, C = dims->channels, V = dims->vocab, R = T * B;
  hipStream_t st = (hipStream_t)stream;
  Fork f(st, (hipStream_t)aux);
  const bool bf = (flags & AA_TRAIN_BF16) != 0;
  const GemmCtx gc{st, s.gsplit, TR_SPLIT_FLOATS, bf};
  const GemmCtx ga{f.aux, s.gsplit2, TR_SPLIT_FLOATS, bf};
  // encoder tail (baseline_attention.py:46-60), reference weight layouts: a_g and the heads on the
  // main stream (the LSTM needs them), the spatial V = relu(A W_a^T + b) and VWv on aux beside the
  // LSTM (the attention is their first reader)
  if (gc.bf16 && H % 64 == 0 && C % 64 == 0) {
    // bf16 step: V on k_bgemm; one pass over the feature map packs both bf16 operand layouts (this
    // GEMM's rows, the backward's dW_a columns) and computes a_g
    hipLaunchKernelGGL(k_pk_feats3, dim3(C / 64, B), dim3(256), 0, st, feats, B, C, s.ftT, s.ftC, rup64(B * P), s.a_g);
    f.to_aux();
    pk_rows(ga.s, w->enc_affine_a_w, C, nullptr, H, C, s.wmT, C);
    bgemm(ga, B * P, H, C, s.ftT, C, s.wmT, C, s.V, H, w->enc_affine_a_b, nullptr, 0, 1);
  } else {
    hipLaunchKernelGGL(k_avgpool, dim3(nblk((int64_t)B * C)), dim3(256), 0, st, feats, (int64_t)B * C, s.a_g);
    f.to_aux();
    const int M = B * P, MT = (M + 63) / 64, NTn = H / 64;
    hipLaunchKernelGGL(k_enc_v, dim3(MT * NTn), dim3(256), 0, ga.s, feats, B, C, H, w->enc_affine_a_w,
                       w->enc_affine_a_b, s.V);
  }
  tgemm(ga, B * P, P, H, s.V, H, 0, w->att_affine_v_w, H, 0, s.VWv, PP);  // VWv = V W_v^T
  // the packed rows of the scores (pack_padded_sequence order), also off the chain
  hipLaunchKernelGGL(k_tr_prow, dim3(nblk(R)), dim3(256), 0, ga.s, lengths, B, T, s.prow);
  // the backward's transposed weights, off the chain too (the parameters do not change until the
  // optimizer step after the backward)
  {
    WTArgs a{};
    const struct { const float* src; float* dst; int rows, cols, ld; } m[] = {
        {w->att_affine_g_w, s.wgT, P, H, WT_LDP},   {w->att_affine_s_w, s.wsT, P, H, WT_LDP},
        {w->att_affine_v_w, s.wvT, P, H, WT_LDP},   {w->sent_affine_x_w, s.wxT, H, 2 * E, H},
        {w->sent_affine_h_w, s.whT, H, H, H},       {w->lstm_w_hh, s.whhT, 4 * H, H, 4 * H},
        {w->lstm_w_ih, s.wihT, 4 * H, 2 * E, 4 * H}};
    int tiles = 0;
    for (const auto& x : m) {
      a.src[a.n] = x.src; a.dst[a.n] = x.dst; a.rows[a.n] = x.rows; a.cols[a.n] = x.cols; a.ld[a.n] = x.ld;
      a.blk0[a.n++] = tiles;
      tiles += ((x.ld + 63) / 64) * ((x.cols + 63) / 64);
    }
    a.blk0[a.n] = tiles;
    hipLaunchKernelGGL(k_wT, dim3(tiles), dim3(256), 0, ga.s, a);
  }
  tgemm(gc, B, E, C, s.a_g, C, 0, w->enc_affine_b_w, C, 0, s.vg, E, 0, w->enc_affine_b_b, nullptr, 1);
  tgemm(gc, B, H, C, s.a_g, C, 0, w->enc_affine_h0_w, C, 0, s.h0, H, 0, w->enc_affine_h0_b, nullptr, 2);
  tgemm(gc, B, H, C, s.a_g, C, 0, w->enc_affine_c0_w, C, 0, s.c0, H, 0, w->enc_affine_c0_b, nullptr, 2);
  decoder_core(gc, w, s, *dims, B, T, tokens, tok_ld, &f);
  if (f.err) return (int)f.err;
  // packed scores = mlp(c_hat + h) on the packed rows (:132, baseline_attention.py:228)
  if (gc.bf16 && H % 64 == 0) {
    pk_rows(st, s.U, H, s.prow, N, H, s.ub, H);
    pk_rows(st, w->mlp_w, H, nullptr, V, H, s.wmb, H);
    bgemm(gc, N, V, H, s.ub, H, s.wmb, H, scores, V, w->mlp_b);
  } else {
    tgemm(gc, N, V, H, s.U, H, 0, w->mlp_w, H, 0, scores, V, 0, w->mlp_b, nullptr, 0, s.prow);
  }
  return aa_launch_status();
}

// batch-first row of t-major row r = t B + b: b T + t (Decoder.forward returns [B, T, ...])
__global__ void k_bt_rowmap(int B, int T, int* __restrict__ map) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < B * T) map[r] = (r % B) * T + r / B;
}

// alpha [R][PP], beta [R] (t-major) -> alpha_out [B][T][P], beta_out [B][T]
__global__ void k_bt_atten_out(int B, int T, const float* __restrict__ alpha, const float* __restrict__ beta,
                               float* __restrict__ alpha_out, float* __restrict__ beta_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (b, t, k) over k < P + 1
  if (i >= (int64_t)B * T * (aa::P + 1)) return;
  const int k = (int)(i % (aa::P + 1));
  const int bt = (int)(i / (aa::P + 1)), b = bt / T, t = bt % T;
  const int64_t r = (int64_t)t * B + b;
  if (k < aa::P) {
    if (alpha_out) alpha_out[(int64_t)bt * aa::P + k] = alpha[r * aa::PP + k];
  } else if (beta_out) {
    beta_out[bt] = beta[r];
  }
}

size_t aa_decoder_workspace_bytes(const aa_dims* d, int32_t B, int32_t T) {
  return aa_train_workspace_bytes(d, B, T);
}

int aa_decoder_forward(const aa_ref_weights* w, const aa_dims* dims, const float* V, const float* v_g,
                       const float* h0, const float* c0, int32_t B, int32_t T, const int64_t* tokens, int32_t tok_ld,
                       float* scores, float* alpha, float* beta, float* h_out, float* c_out, void* workspace,
                       size_t workspace_bytes, int32_t flags, aa_stream_t stream) {
  using namespace aa;
  int rc = train_check(dims, B, T);
  if (rc) return rc;
  if (B == 0 || T == 0) return AA_OK;
  if (!w || !V || !v_g || !h0 || !c0 || !tokens || !workspace || !w->sent_affine_h_w) return AA_ERR_NULL;
  if (tok_ld < T) return AA_ERR_SHAPE;
  size_t need;
  TrainWS s = carve_train(static_cast<char*>(workspace), *dims, B, T, B * T, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  const int H = dims->hidden, E = dims->embed, Vc = dims->vocab, R = T * B;
  hipStream_t st = (hipStream_t)stream;
  const GemmCtx gc{st, s.gsplit, TR_SPLIT_FLOATS, (flags & AA_TRAIN_BF16) != 0};
  hipError_t e = hipSuccess;
  if (!e) e = hipMemcpyAsync(s.V, V, sizeof(float) * (size_t)B * P * H, hipMemcpyDeviceToDevice, st);
  if (!e) e = hipMemcpyAsync(s.vg, v_g, sizeof(float) * (size_t)B * E, hipMemcpyDeviceToDevice, st);
  if (!e) e = hipMemcpyAsync(s.h0, h0, sizeof(float) * (size_t)B * H, hipMemcpyDeviceToDevice, st);
  if (!e) e = hipMemcpyAsync(s.c0, c0, sizeof(float) * (size_t)B * H, hipMemcpyDeviceToDevice, st);
  if (e) return (int)e;
  tgemm(gc, B * P, P, H, s.V, H, 0, w->att_affine_v_w, H, 0, s.VWv, PP);  // VWv = V W_v^T
  decoder_core(gc, w, s, *dims, B, T, tokens, tok_ld);
  if (scores) {  // mlp(c_hat + h) for every (b, t), batch-first (:132)
    hipLaunchKernelGGL(k_bt_rowmap, dim3(nblk(R)), dim3(256), 0, st, B, T, s.prow);
    tgemm(gc, R, Vc, H, s.U, H, 0, w->mlp_w, H, 0, scores, Vc, 0, w->mlp_b, nullptr, 0, nullptr, s.prow);
  }
  if (alpha || beta)
    hipLaunchKernelGGL(k_bt_atten_out, dim3(nblk((int64_t)R * (P + 1))), dim3(256), 0, st, B, T, s.alpha, s.beta,
                       alpha, beta);
  if (h_out) e = hipMemcpyAsync(h_out, s.Hs + (size_t)(T - 1) * B * H, sizeof(float) * (size_t)B * H,
                                hipMemcpyDeviceToDevice, st);
  if (!e && c_out) e = hipMemcpyAsync(c_out, s.Cs + (size_t)(T - 1) * B * H, sizeof(float) * (size_t)B * H,
                                      hipMemcpyDeviceToDevice, st);
  if (e) return (int)e;
  return aa_launch_status();
}

int aa_train_backward(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B, int32_t T,
                      const int64_t* tokens, int32_t tok_ld, const int32_t* lengths, const float* dscores, int32_t N,
                      const aa_ref_grads* grads, float* dfeats, void* workspace, size_t workspace_bytes,
                      int32_t flags, aa_stream_t stream) {
  return aa_train_backward_aux(w, dims, feats, B, T, tokens, tok_ld, lengths, dscores, N, grads, dfeats, workspace,
                               workspace_bytes, flags, stream, nullptr);
}

int aa_train_backward_aux(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B, int32_t T,
                          const int64_t* tokens, int32_t tok_ld, const int32_t* lengths, const float* dscores,
                          int32_t N, const aa_ref_grads* grads, float* dfeats, void* workspace, size_t workspace_bytes,
                          int32_t flags, aa_stream_t stream, aa_stream_t aux) {
  using namespace aa;
  int rc = train_check(dims, B, T);
  if (rc) return rc;
  if (B == 0 || T == 0 || N == 0) return AA_OK;
  if (!w || !feats || !tokens || !lengths || !dscores || !grads || !workspace) return AA_ERR_NULL;
  if (N > B * T || tok_ld < T) return AA_ERR_SHAPE;
  size_t need;
  TrainWS s = carve_train(static_cast<char*>(workspace), *dims, B, T, B * T, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  const int H = dims->hidden, E = dims->embed, C = dims->channels, V = dims->vocab, R = T * B, E2 = 2 * E;
  hipStream_t st = (hipStream_t)stream;
  Fork f(st, (hipStream_t)aux);
  const hipStream_t sa = f.aux;
  const bool bf = (flags & AA_TRAIN_BF16) != 0;
  const GemmCtx gc{st, s.gsplit, TR_SPLIT_FLOATS, bf};
  const GemmCtx ga{sa, s.gsplit2, TR_SPLIT_FLOATS, bf};
#define GRAD(f) (grads->f)
  const size_t RH = (size_t)R * H;
  // Streams (Fork): main = dscores -> dU -> attention backward -> sentinel -> LSTM through time ->
  // dx -> embedding / encoder-head gradients; aux = the weight gradients hanging off that chain
  // (dW_m, dW_g / dW_s / dW_v / the V-side encoder, dW_x / dW_h, dW_hh / dW_ih / b_ih) and the token
  // ranking of the embedding gradient.
  f.to_aux();
  // x_t = [embed(tok); v_g] (baseline_attention.py:151-154): the tokens' segmented-sum order
  AA_TRY(hipMemsetAsync(GRAD(embed_w), 0, sizeof(float) * (size_t)V * E, sa));
  hipLaunchKernelGGL(k_tok_rank, dim3((R + 3) / 4), dim3(256), 0, sa, tokens, tok_ld, B, R, V, s.trank, s.tcount,
                     s.tsmall);
  hipLaunchKernelGGL(k_tok_place, dim3(nblk(R)), dim3(256), 0, sa, R, s.trank, s.tsmall, s.torder);
  hipEvent_t tok_done = f.mark(sa);
  // mlp (adaptive_attention.py:132): dU[prow] = dS W_m; dW_m = dS^T U_p; db_m = colsum(dS)
  const int Vp = (V + 63) / 64 * 64;  // dscores re-pitched to whole 16-B rows for vector loads
  const bool bg = gc.bf16 && H % 64 == 0;  // the large GEMMs on k_bgemm
  // bf16 steps need dS only as bf16 (the GEMMs) and fp32 for db_m, which colsum reads from dscores
  // itself (same sums, same order): no fp32 re-pitched copy
  if (bg)  // dS to bf16 for the GEMMs, db_m's column partials on the way (finished below)
    hipLaunchKernelGGL(k_pad_rows_colsum, dim3((Vp + 255) / 256, CS_CH), dim3(256), 0, st, dscores, N, V, Vp, s.dspb,
                       s.csum);
  else
    hipLaunchKernelGGL(k_pad_rows, dim3(nblk((int64_t)N * Vp)), dim3(256), 0, st, dscores, N, V, Vp, s.dsp,
                       (__bf16*)nullptr);
  // dU, dS, dPG, dPS are carved back to back: one clear for the four (nothing below touches dS / dPG
  // / dPS before the attention backward accumulates into them)
  AA_TRY(hipMemsetAsync(s.dU, 0, (size_t)((char*)(s.dPS + (size_t)R * PP) - (char*)s.dU), st));
  hipLaunchKernelGGL(k_gather_rows, dim3(nblk((int64_t)N * H)), dim3(256), 0, st, s.U, s.prow, N, H, s.Up);
  f.to_aux();  // dW_m on aux
  if (bg) {
    const int Kv = Vp, Kn = rup64(N);                                     // dS as bf16 [N][Vp]: k_pad_rows
    pk_trans(sa, s.dspb, Vp, N, V, s.dspT, Kn);                            // dS^T [V][Kn]
    pk_trans(sa, s.Up, H, N, H, s.upT, Kn);                                // U_p^T [H][Kn]
    bgemm(ga, V, H, Kn, s.dspT, Kn, s.upT, Kn, GRAD(mlp_w), H);            // dW_m = dS^T U_p
    pk_trans(st, w->mlp_w, H, V, H, s.wmT, Kv);                            // W_m^T [H][Kv]
    bgemm(gc, N, H, Kv, s.dspb, Kv, s.wmT, Kv, s.dU, H, nullptr, s.prow);  // dU[prow] = dS W_m
  } else {
    tgemm(ga, V, H, N, s.dsp, Vp, 1, s.Up, H, 1, GRAD(mlp_w), H);
    tgemm(gc, N, H, V, s.dsp, Vp, 0, w->mlp_w, H, 1, s.dU, H, 0, nullptr, nullptr, 0, nullptr, s.prow);
  }
  if (bg) hipLaunchKernelGGL(k_colsum_fin, dim3((V + 255) / 256), dim3(256), 0, st, s.csum, V, GRAD(mlp_b));
  else colsum(st, s.dsp, N, V, (int64_t)Vp, s.csum, GRAD(mlp_b));
  // Atten backward (adaptive_attention.py:26-58)
  int G, TS;
  atb_groups(B, T, &G, &TS);
#define AA_ATB(HPT_)                                                                                          \
  hipLaunchKernelGGL(k_tr_atb_row<HPT_>, dim3(R), dim3(256), 0, st, B, lengths, s.dU, s.alpha, s.beta, s.ctx, s.S, \
                     s.PG, s.PS, s.VWv, s.V, w->att_affine_h_w, s.dS, s.dPG, s.dPS, s.dz, s.dwr, s.dH);          \
  hipLaunchKernelGGL(k_tr_atb_img<HPT_>, dim3(B, HPT_ + 1), dim3(256), 0, st, B, TS, G, lengths, s.dU, s.alpha, s.beta, s.PG, \
                     s.VWv, w->att_affine_h_w, s.dz, s.dwr, s.dV, s.dVWv, s.dwh)
  switch (H / 256) {
    case 1: AA_ATB(1); break;
    case 2: AA_ATB(2); break;
    case 3: AA_ATB(3); break;
    default: AA_ATB(4); break;
  }
#undef AA_ATB
  // dH = dU (u = c_hat + h) was written by k_tr_atb_row
  f.to_aux();  // the attention's weight gradients and the V side of the encoder on aux
  // (the weights the backward multiplies by untransposed are read from the forward's transposed
  // copies, s.w*T: both operands along K)
  tgemm(gc, R, H, P, s.dPG, PP, 0, s.wgT, WT_LDP, 0, s.dH, H, 1);                      // dh += dPG W_g
  tgemm(gc, R, H, P, s.dPS, PP, 0, s.wsT, WT_LDP, 0, s.dS, H, 1);                      // ds += dPS W_s
  tgemm(ga, P, H, R, s.dPG, PP, 1, s.Hs, H, 1, GRAD(att_affine_g_w), H);                 // dW_g = dPG^T h
  tgemm(ga, P, H, R, s.dPS, PP, 1, s.S, H, 1, GRAD(att_affine_s_w), H);                  // dW_s = dPS^T s
  tgemm(ga, B * P, H, P, s.dVWv, PP, 0, s.wvT, WT_LDP, 0, s.dV, H, 1);                 // dV += dVWv W_v
  tgemm(ga, P, H, B * P, s.dVWv, PP, 1, s.V, H, 1, GRAD(att_affine_v_w), H);             // dW_v = dVWv^T V
  hipLaunchKernelGGL(k_rowsum_pp, dim3(1), dim3(256), 0, sa, s.dwh, B, GRAD(att_affine_h_w));
  // encoder V = relu(A W_a^T + b) (baseline_attention.py:46-51)
  hipLaunchKernelGGL(k_relu_mask, dim3(nblk((int64_t)B * P * H)), dim3(256), 0, sa, s.dV, s.V, (int64_t)B * P * H);
  if (gc.bf16 && H % 64 == 0) {  // dW_a = dV^T A
    const int Kb = rup64(B * P);
    pk_trans(sa, s.dV, H, B * P, H, s.dvT, Kb);
    // the feature map's [C][Kb] bf16 operand was packed by the forward (k_pk_feats3, same workspace)
    bgemm(ga, H, C, Kb, s.dvT, Kb, s.ftC, Kb, GRAD(enc_affine_a_w), C);
  } else {
    tgemm(ga, H, C, B * P, s.dV, H, 1, feats, C, 2, GRAD(enc_affine_a_w), C);              // dW_a = dV^T A
  }
  colsum(sa, s.dV, B * P, H, (int64_t)H, s.csum2, GRAD(enc_affine_a_b));
  if (dfeats) tgemm(ga, B * P, C, H, s.dV, H, 0, w->enc_affine_a_w, C, 1, s.dA, C);      // dA = dV W_a
  // Sentinel backward (:79-83): h_{t-1} input = Hs[r - B] for r >= B, 0 for t = 0
  hipLaunchKernelGGL(k_tr_sent_bwd, dim3(nblk((int64_t)RH)), dim3(256), 0, st, s.dS, s.SG, s.Cs, s.dG, s.dC,
                     (int64_t)RH);
  f.to_aux();
  tgemm(ga, H, E2, R, s.dG, H, 1, s.X, E2, 1, GRAD(sent_affine_x_w), E2);               // dW_x = dG^T x
  tgemm(ga, H, H, R - B, s.dG + (size_t)B * H, H, 1, s.Hs, H, 1, GRAD(sent_affine_h_w), H);  // dW_h = dG^T h_{t-1}
  tgemm(gc, R, E2, H, s.dG, H, 0, s.wxT, H, 0, s.dX, E2);                               // dx = dG W_x
  tgemm(gc, R - B, H, H, s.dG + (size_t)B * H, H, 0, s.whT, H, 0, s.dH, H, 1);          // dh_{t-1} += dG W_h
  // LSTM backward through time (baseline_attention.py:167-178)
  AA_TRY(hipMemsetAsync(s.dh_rec, 0, (size_t)((char*)(s.dc_rec + (size_t)B * H) - (char*)s.dh_rec), st));  // adjacent
  if (gc.bf16) {
    // one fused launch per step (k_tr_lstm_b: dh_rec = DG_{t+1} W_hh, then the cell backward); the
    // gradient into h0 (dh_rec of step 0) is one GEMM after the loop
    hipLaunchKernelGGL(k_pk_whh, dim3(nblk((int64_t)4 * H * H / 8)), dim3(256), 0, st, w->lstm_w_hh, H, 1, s.whb);
    const unsigned grid = (unsigned)(((B + 15) / 16) * (H / 16));
    for (int t = T - 1; t >= 0; --t) {
      const size_t o = (size_t)t * B * H;
      const float* cp = t ? s.Cs + o - (size_t)B * H : s.c0;
      const float* ga4 = s.GA + (size_t)t * B * 4 * H;
      float* dg = s.DG + (size_t)t * B * 4 * H;
#define AA_LB(H_)                                                                                                   \
  if (t == T - 1)                                                                                                   \
    hipLaunchKernelGGL((k_tr_lstm_b<H_, true>), dim3(grid), dim3(256), 0, st, B, (const __bf16*)nullptr, s.whb,     \
                       s.dH + o, s.dC + o, s.dc_rec, ga4, s.Cs + o, cp, dg, s.dgb[t & 1]);                          \
  else                                                                                                              \
    hipLaunchKernelGGL((k_tr_lstm_b<H_, false>), dim3(grid), dim3(256), 0, st, B, (const __bf16*)s.dgb[(t + 1) & 1], \
                       s.whb, s.dH + o, s.dC + o, s.dc_rec, ga4, s.Cs + o, cp, dg, s.dgb[t & 1])
      switch (H) {
        case 256: AA_LB(256); break;
        case 512: AA_LB(512); break;
        case 768: AA_LB(768); break;
        default: AA_LB(1024); break;
      }
#undef AA_LB
    }
    f.to_aux();  // DG complete: the LSTM weight gradients on aux
    tgemm(gc, B, H, 4 * H, s.DG, 4 * H, 0, s.whhT, 4 * H, 0, s.dh_rec, H);
  } else {
    int S = 0;  // split count of the pending dh_rec GEMM (0: dh_rec = 0)
    for (int t = T - 1; t >= 0; --t) {
      const size_t o = (size_t)t * B * H;
      const float* cp = t ? s.Cs + o - (size_t)B * H : s.c0;
      hipLaunchKernelGGL(k_tr_cell_bwd_sk, dim3(nblk((int64_t)B * H)), dim3(256), 0, st, s.dH + o, s.dC + o,
                         S > 1 ? gc.split : s.dh_rec, S, s.dc_rec, s.GA + (size_t)t * B * 4 * H, s.Cs + o, cp, B, H,
                         s.DG + (size_t)t * B * 4 * H);
      // dh_{t-1}; the one of step 0 (into h0) is reduced into dh_rec itself
      S = tgemm(gc, B, H, 4 * H, s.DG + (size_t)t * B * 4 * H, 4 * H, 0, s.whhT, 4 * H, 0, s.dh_rec, H, 0, nullptr,
                nullptr, 0, nullptr, nullptr, t > 0);
    }
    f.to_aux();
  }
  tgemm(ga, 4 * H, H, B, s.DG, 4 * H, 1, s.h0, H, 1, GRAD(lstm_w_hh), H);                 // t = 0: h_{-1} = h0
  tgemm(ga, 4 * H, H, R - B, s.DG + (size_t)B * 4 * H, 4 * H, 1, s.Hs, H, 1, GRAD(lstm_w_hh), H, 1);
  tgemm(ga, 4 * H, E2, R, s.DG, 4 * H, 1, s.X, E2, 1, GRAD(lstm_w_ih), E2);
  colsum(sa, s.DG, R, 4 * H, (int64_t)4 * H, s.csum2, GRAD(lstm_b_ih));
  AA_TRY(hipMemcpyAsync(GRAD(lstm_b_hh), GRAD(lstm_b_ih), sizeof(float) * 4 * H, hipMemcpyDeviceToDevice, sa));
  tgemm(gc, R, E2, 4 * H, s.DG, 4 * H, 0, s.wihT, 4 * H, 0, s.dX, E2, 1);               // dx += dG W_ih
  // x_t = [embed(tok); v_g] (baseline_attention.py:151-154)
  f.wait(st, tok_done);
  hipLaunchKernelGGL(k_tr_embed_bwd, dim3(R), dim3(256), 0, st, tokens, tok_ld, B, R, V, s.torder, s.trank, s.tcount,
                     s.dX, E, GRAD(embed_w));
  hipLaunchKernelGGL(k_tr_vg_bwd, dim3(nblk((int64_t)B * E)), dim3(256), 0, st, s.dX, s.vg, B, T, E, s.dvg);
  // encoder heads (baseline_attention.py:52-60)
  tgemm(gc, E, C, B, s.dvg, E, 1, s.a_g, C, 1, GRAD(enc_affine_b_w), C);
  colsum(st, s.dvg, B, E, (int64_t)E, s.csum, GRAD(enc_affine_b_b));
  if (s.dc_rec == s.dh_rec + (size_t)B * H && s.c0 == s.h0 + (size_t)B * H) {  // carved back to back: one launch
    hipLaunchKernelGGL(k_tanh_bwd, dim3(nblk((int64_t)2 * B * H)), dim3(256), 0, st, s.dh_rec, s.h0, (int64_t)2 * B * H);
  } else {
    hipLaunchKernelGGL(k_tanh_bwd, dim3(nblk((int64_t)B * H)), dim3(256), 0, st, s.dh_rec, s.h0, (int64_t)B * H);
    hipLaunchKernelGGL(k_tanh_bwd, dim3(nblk((int64_t)B * H)), dim3(256), 0, st, s.dc_rec, s.c0, (int64_t)B * H);
  }
  tgemm(gc, H, C, B, s.dh_rec, H, 1, s.a_g, C, 1, GRAD(enc_affine_h0_w), C);
  colsum(st, s.dh_rec, B, H, (int64_t)H, s.csum, GRAD(enc_affine_h0_b));
  tgemm(gc, H, C, B, s.dc_rec, H, 1, s.a_g, C, 1, GRAD(enc_affine_c0_w), C);
  colsum(st, s.dc_rec, B, H, (int64_t)H, s.csum, GRAD(enc_affine_c0_b));
  if (dfeats) {  // gradient into the trunk's output A (CNN fine-tuning, train.py:89)
    tgemm(gc, B, C, E, s.dvg, E, 0, w->enc_affine_b_w, C, 1, s.dag, C);                // d a_g = dv_g W_b
    tgemm(gc, B, C, H, s.dh_rec, H, 0, w->enc_affine_h0_w, C, 1, s.dag, C, 1);         //   + dh0 W_h0
    tgemm(gc, B, C, H, s.dc_rec, H, 0, w->enc_affine_c0_w, C, 1, s.dag, C, 1);         //   + dc0 W_c0
  }
  f.to_main();  // everything on aux (dA above) is done before the call's work ends on main
  if (dfeats)
    hipLaunchKernelGGL(k_dfeats, dim3((C + 63) / 64, B), dim3(256), 0, st, s.dA, s.dag, C, dfeats);
  if (f.err) return (int)f.err;
#undef GRAD
  return aa_launch_status();
}

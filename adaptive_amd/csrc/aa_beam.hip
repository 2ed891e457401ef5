// aa_beam.hip — beam-search caption decode (BASELINE config 4: B = 512,
// beam 3).  The reference has no beam search (for_wzn:3 lists it as a TODO), so its semantics are
// defined here and restated on the CPU by oracle/adaptive_oracle.py BeamOracle:
//
//   rows r = b*K + k (the K hypotheses of image b are adjacent rows, sharing V / VWv of image b)
//   t = 0: every row holds <start> with the encoder's (h0, c0); only beam 0 is live, so the K
//          first hypotheses are the K best first tokens of one distribution
//   step t: logits of every row (the same AdaptiveBlock step as the greedy path), candidate score
//          cum[k] + logp[k][v] with logp = (x - max) - log(sum exp(x - max)) (torch log_softmax);
//          a finished beam (it emitted end_id) has exactly one candidate, end_id, at score cum[k]
//          (it is carried unchanged); the K best candidates of the image — score descending, ties
//          to the smaller flat index k*V + v — become the new beams
//   end:   beams come out sorted by score; ids / alpha / beta are those of beam 0, traced back
//          through the parent pointers.  All T steps run (as in the greedy sampler).
//
// Kernels: the greedy path's k_lstm (gathering h / c from each row's parent) and k_atten (kdiv =
// K rows per image), the exact fp32 vocab GEMM k_vocab writing the logits, then k_beam_select
// (one workgroup per image: row max / log-sum-exp / top-K in registers, K x K merge) and
// k_beam_final (backtrace).
namespace aa {

constexpr int BEAM_MAX = 8;      // AA_MAX_BEAM
constexpr int BEAM_VPT = 64;     // logits held per thread in k_beam_select: V <= 256 * 64

// dst[r][:] = src[r / K][:]  (n a multiple of 4)
__global__ void k_expand_rows(const float* __restrict__ src, int B, int K, int n, float* __restrict__ dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // float4 index
  const int n4 = n / 4;
  if (i >= (int64_t)B * K * n4) return;
  const int64_t r = i / n4, c = i % n4;
  reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[(r / K) * n4 + c];
}

__device__ __forceinline__ float block_max256(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ uint64_t block_max256_u64(uint64_t v, uint64_t* red) {
  v = wave_max_u64(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const uint64_t a = red[0] > red[1] ? red[0] : red[1], c = red[2] > red[3] ? red[2] : red[3];
  return a > c ? a : c;
}

// One workgroup per image: trace every final beam back (seqs [B][K][T], scores [B][K]); ids, alpha
// and beta follow beam 0.  path [B][T] scratch: the row whose step-t attention produced beam 0's
// token t.
__global__ __launch_bounds__(256) void k_beam_final(int K, int T, int R, const int* __restrict__ htok,
                                                    const int* __restrict__ hpar, const float* __restrict__ cum,
                                                    const float* __restrict__ ahist, const float* __restrict__ bhist,
                                                    int* __restrict__ path, int64_t* __restrict__ ids,
                                                    int64_t* __restrict__ seqs, float* __restrict__ scores,
                                                    float* __restrict__ alpha, float* __restrict__ beta) {
  const int b = blockIdx.x, tid = threadIdx.x;
  if (tid < K) {
    int j = tid;
    if (scores) scores[(int64_t)b * K + tid] = cum[b * K + tid];
    for (int t = T - 1; t >= 0; --t) {
      const int r = b * K + j;
      const int col = htok[(int64_t)t * R + r];
      const int pk = hpar[(int64_t)t * R + r];
      if (seqs) seqs[((int64_t)b * K + tid) * T + t] = col;
      if (tid == 0) {
        if (ids) ids[(int64_t)b * T + t] = col;
        path[(int64_t)b * T + t] = b * K + pk;
      }
      j = pk;
    }
  }
  if (!alpha && !beta) return;
  __syncthreads();
  for (int i = tid; i < T * P; i += 256) {
    const int t = i / P, q = i % P;
    const int r = path[(int64_t)b * T + t];
    if (alpha) alpha[((int64_t)b * T + t) * P + q] = ahist[((int64_t)t * R + r) * P + q];
    if (beta && q == 0) beta[(int64_t)b * T + t] = bhist[(int64_t)t * R + r];
  }
}

// ---------------------------------------------------------------------------------------------
// Default vocab stage (k_vbeam4 below): bf16x3 MFMA logits and per-granule log-sum-exp summaries.
// ---------------------------------------------------------------------------------------------
// transposing butterfly step for a plain reduction (OP 0: max, 1: sum) of 16 rows over 32 lanes
template <int M, int OP>
__device__ __forceinline__ void red_bfly(float (&v)[16], int li) {
  const bool hi = (li & M) != 0;
#pragma unroll
  for (int k = 0; k < M / 2; ++k) {
    const float sd = hi ? v[k] : v[k + M / 2];
    const float kp = hi ? v[k + M / 2] : v[k];
    const float rv = __uint_as_float(partner<M>(__float_as_uint(sd)));
    v[k] = OP == 0 ? fmaxf(kp, rv) : kp + rv;
  }
}

// Granule summary of one 32 x 32 block held in MFMA accumulator layout (lane li + 32 lh holds
// column li of rows acc_row(r, lane), r = 0..15): per row, (max, sum exp(x - max)) over the block's
// 32 columns (invalid columns: x = -inf, no term), by a transposing max-butterfly, a broadcast of the
// row max to the row's 32 lanes, one expf per element and a transposing add-butterfly -- a fixed
// pattern, so every kernel that calls this on the same values gets the same bits (the beam-search
// selection's log-sum-exp is built from these summaries).  Returns the summary in lanes with
// !(li & 1), for the row of the block acc_row-indexed by sum_row().
__device__ __forceinline__ float2 granule_summary(const float (&x)[16], bool valid, int li, int lh) {
  float m[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) m[r] = x[r];
  red_bfly<16, 0>(m, li);
  red_bfly<8, 0>(m, li);
  red_bfly<4, 0>(m, li);
  red_bfly<2, 0>(m, li);
  const float gmax = fmaxf(m[0], __uint_as_float(partner<1>(__float_as_uint(m[0]))));
  // lane pair (2 rr, 2 rr + 1) of half lh now holds the max of row rr of that half
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float g = __shfl(gmax, 2 * r + 32 * lh, 64);
    m[r] = valid ? expf(x[r] - g) : 0.f;
  }
  red_bfly<16, 1>(m, li);
  red_bfly<8, 1>(m, li);
  red_bfly<4, 1>(m, li);
  red_bfly<2, 1>(m, li);
  const float gs = m[0] + __uint_as_float(partner<1>(__float_as_uint(m[0])));
  return make_float2(gmax, gs);
}
// block row of the summary granule_summary leaves in lane li (valid in lanes with !(li & 1))
__device__ __forceinline__ int sum_row(int li, int lh) {
  const int rr = (li >> 1) & 15;
  return (rr & 3) + 8 * (rr >> 2) + 4 * lh;
}

// Granule summaries of logits already in memory (the exact path: k_vocab's fp32 logits, row pitch
// Vp): one wave per (32-row block, 32-column granule), the block loaded in accumulator layout and
// summarised by granule_summary -- bit-identical to the summaries a GEMM epilogue computes from the
// same logit values.
__global__ __launch_bounds__(256) void k_gsumm(int R, int V, int Vp, const float* __restrict__ logits,
                                               float2* __restrict__ gsum) {
  const int NG = Vp / 32, RB = (R + 31) / 32;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);  // global wave = (row block, granule)
  if (gw >= RB * NG) return;
  const int rb = gw / NG, g = gw % NG;
  const int lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int col = g * 32 + li;
  const bool valid = col < V;
  float x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int row = rb * 32 + acc_row(r, lane);
    row = row < R ? row : R - 1;
    x[r] = valid ? logits[(int64_t)row * Vp + col] : -INFINITY;
  }
  const float2 sm = granule_summary(x, valid, li, lh);
  const int row = rb * 32 + sum_row(li, lh);
  if (!(li & 1) && row < R) gsum[(int64_t)row * NG + g] = sm;
}

// k_vexact (the beam's default vocab stage): exact fp32 logits -- k_vocab's arithmetic (the same
// v_mfma_f32_32x32x2f32 sequence over NP_VOCAB chains and the same combination tree, via
// gemm_mainloop_chain: the 8 chains combined as they complete, so a wave holds 4 partial sets instead
// of k_vocab's 8), so the same bits -- with the granule summaries of k_gsumm fused into the epilogue
// (granule_summary on the same values: the same bits).
// k_vocab + k_gsumm stay as the cross-check path (AA_DECODE_EXACT_VOCAB).
// 64 x 64 tiles (3,840 workgroups at config 4, 200 VGPRs: two workgroups per CU) measured 0.187 ms per
// launch against 0.212 ms for 128 x 64 tiles (1,920 workgroups, 384 registers: one wave per SIMD, the
// LDS and barrier latencies exposed); beams bitwise unchanged (round 3, A/B on one box)
#ifndef AA_VX_BM
#define AA_VX_BM 64
#endif
constexpr int VX_BM = AA_VX_BM, VX_BN = 64;
// AA_VEXACT_OCC 3: three workgroups per CU (168 VGPRs, 5 spilled): 0.205 -> 0.183 ms per launch, beam
// 89.4K -> 96.7K captions/s on one box, bit-identical (round 3 A/B)
#ifndef AA_VEXACT_OCC
#define AA_VEXACT_OCC 3
#endif
__global__ __launch_bounds__(256, AA_VEXACT_OCC) void k_vexact(int R, int H, int V, int Vp, const float* __restrict__ u,
                                                   const float* __restrict__ W, const float* __restrict__ bias,
                                                   float* __restrict__ logits, float2* __restrict__ gsum) {
  __shared__ __attribute__((aligned(16))) float lds[Tile<VX_BM, VX_BN>::LDS_FLOATS];
  const int MT = (R + VX_BM - 1) / VX_BM, NTn = Vp / VX_BN, NG = Vp / 32;
  const int L = xcd_remap(blockIdx.x, MT * NTn);
  const int nt = L / MT, mt = L % MT;  // m fastest: a W tile is shared inside an XCD
  ARowMajor al{u, H, mt * VX_BM, R};
  WRowMajor wl{W, H, nt * VX_BN};
  floatx16 acc[VX_BM / 64][VX_BN / 64];
  gemm_mainloop_chain<VX_BM, VX_BN, NP_VOCAB>(al, wl, H / BK, lds, acc);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int tn = 0; tn < VX_BN / 64; ++tn) {
    const int c0 = nt * VX_BN + wn * (VX_BN / 2) + tn * 32, col = c0 + li;
    const bool valid = col < V;
    const float bv = bias[col];
#pragma unroll
    for (int tm = 0; tm < VX_BM / 64; ++tm) {
      const int rb = mt * VX_BM + wm * (VX_BM / 2) + tm * 32;
      float x[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[r] = acc[tm][tn][r] + bv;
        const int row = rb + acc_row(r, lane);
        if (row < R) logits[(int64_t)row * Vp + col] = x[r];
        x[r] = valid ? x[r] : -INFINITY;
      }
      const float2 sm = granule_summary(x, valid, li, lh);
      const int row = rb + sum_row(li, lh);
      if (!(li & 1) && row < R) gsum[(int64_t)row * NG + c0 / 32] = sm;
    }
  }
}

// k_vbeam4: logits (+ bias) and per (row, 32-column granule) (max, sum exp(x - max)), bf16x3 MFMA
// (fp32-accurate, as the encoder / LSTM GEMMs), from a 128x128 tile whose operand fragments
// are staged once per workgroup in LDS by global_load_lds (16 B per lane: one wave instruction
// moves one 1-KB fragment, so the LDS image is the fragment-order image itself) and shared by the
// four waves (each owns a 64x64 quadrant over the whole K: no partial-tile reduction).  Three
// stage buffers of one k16 chunk (A: 4 row blocks x 3 planes, W: 4 column blocks x 3 planes =
// 24 KB); chunk k + 2 is in flight while chunk k is multiplied (counted vmcnt, raw s_barrier).
constexpr int VB4_NBUF = 3;
template <int H>
__global__ __launch_bounds__(256, 2) void k_vbeam4(int R, int V, int Vp, const bf16x8* __restrict__ ua3,
                                                   const bf16x8* __restrict__ w3, const float* __restrict__ bias,
                                                   float* __restrict__ logits, float2* __restrict__ gsum) {
  constexpr int KC = H / 16;
  __shared__ __attribute__((aligned(16))) bf16x8 stg[VB4_NBUF][24 * 64];
  const int NG = Vp / 32, NTs = Vp / 128, MT = (R + 127) / 128;
  const int RB = (R + 63) / 64 * 2;  // row blocks present in ua3 (64-row padded)
  const int L = xcd_remap(blockIdx.x, MT * NTs);
  const int nt = L / MT, mt = L % MT;  // m fastest: a W tile is shared inside an XCD
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5, wr = wave >> 1, wc = wave & 1;
  const int m0 = mt * 128, n0 = nt * 128;
  // this wave's 6 fragments of every chunk: f = 6 wave + i; f < 12: A (row block f / 3, plane f % 3)
  const bf16x8* src[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int f = 6 * wave + i;
    if (f < 12) {
      int rb = m0 / 32 + f / 3;
      rb = rb < RB ? rb : RB - 1;
      src[i] = ua3 + ((size_t)rb * KC * 3 + f % 3) * 64 + lane;
    } else {
      const int cb = n0 / 32 + (f - 12) / 3;
      src[i] = w3 + ((size_t)cb * KC * 3 + (f - 12) % 3) * 64 + lane;
    }
  }
  auto issue = [&](int kc, int buf) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[i] + (size_t)kc * 3 * 64),
                                       (__attribute__((address_space(3))) void*)(&stg[buf][(6 * wave + i) * 64]),
                                       16, 0, 0);
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
  // fragments of chunk k are read from LDS while the MFMAs of chunk k - 1 run (two register sets);
  // chunk k + 2 is in flight meanwhile, so a buffer is refilled right after its last reader passed
  // the barrier
  bf16x8 fa[2][2][3], fw[2][2][3];  // [set][block][plane]
  auto lread = [&](int kc, int set) {
    const bf16x8* sb = stg[kc % VB4_NBUF];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        fa[set][a][q] = sb[((2 * wr + a) * 3 + q) * 64 + lane];
        fw[set][a][q] = sb[(12 + (2 * wc + a) * 3 + q) * 64 + lane];
      }
  };
  issue(0, 0);
  if (KC > 1) issue(1, 1);
  if (KC > 2) issue(2, 2);
  if (KC > 2)
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (KC > 1)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  lread(0, 0);
#pragma unroll 2
  for (int kc = 0; kc < KC; ++kc) {
    const int set = kc & 1;
    if (kc + 1 < KC) {
      if (kc + 2 < KC)
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // chunk kc + 1 landed everywhere; chunk kc's buffer is free
      if (kc + 3 < KC) issue(kc + 3, (kc + 3) % VB4_NBUF);
      lread(kc + 1, set ^ 1);
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) x3_step(acc[a][c], fa[set][a], fw[set][c]);
    // interleave: 2 MFMAs, then one of the 12 fragment reads of the next chunk
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // epilogue per 32x32 block: logits (+ bias) and the granule's (max, sum exp(x - max)): the row
  // max by a transposing max-butterfly, broadcast back to the row's 32 lanes, one expf per
  // element, and the sums by a transposing add-butterfly (fixed pattern: deterministic)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = n0 + wc * 64 + c * 32 + li;
    const bool valid = col < V;
    const float bv = bias[col];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      float x[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[r] = acc[a][c][r] + bv;
        const int row = m0 + wr * 64 + a * 32 + acc_row(r, lane);
        if (row < R) logits[(int64_t)row * Vp + col] = x[r];
        x[r] = valid ? x[r] : -INFINITY;
      }
      const float2 sm = granule_summary(x, valid, li, lh);
      const int row = m0 + wr * 64 + a * 32 + sum_row(li, lh);
      if (!(li & 1) && row < R) gsum[(int64_t)row * NG + (n0 + wc * 64 + c * 32) / 32] = sm;
    }
  }
}

// k_vbeam5: k_vbeam4's arithmetic and epilogue on 256 x 256 tiles: 16 waves (1024 threads, a 4 x 4
// grid of 64 x 64 quadrants over the whole K), one workgroup per CU (at R = 1536, Vp = 10240 the
// grid is 6 x 40 = 240 workgroups: one round, where k_vbeam4's 960 128 x 128 tiles take two rounds
// of two per CU).  A chunk (one k16 step: 8 A row blocks + 8 W column blocks, 3 planes each = 48
// fragments = 48 KB) is staged by global_load_lds, three fragments per wave; three stage buffers
// (144 KB), chunk k + 2 in flight while chunk k is multiplied, so the lead over the L2 / MALL
// latency is two chunks of 4 waves x 24 MFMAs per SIMD (k_vbeam4: two chunks of 2 x 24).  With
// four waves per SIMD (128 VGPRs each) a wave holds one fragment set: it reads chunk k from LDS
// right after the barrier and the other waves' MFMAs cover that latency.
constexpr int VB5_NBUF = 3, VB5_FR = 48;
template <int H>
__global__ __launch_bounds__(1024) void k_vbeam5(int R, int V, int Vp, const bf16x8* __restrict__ ua3,
                                                 const bf16x8* __restrict__ w3, const float* __restrict__ bias,
                                                 float* __restrict__ logits, float2* __restrict__ gsum) {
  constexpr int KC = H / 16;
  __shared__ __attribute__((aligned(16))) bf16x8 stg[VB5_NBUF][VB5_FR * 64];
  const int NG = Vp / 32, NTs = Vp / 256, MT = (R + 255) / 256;
  const int RB = (R + 63) / 64 * 2;  // row blocks present in ua3 (64-row padded)
  const int L = xcd_remap(blockIdx.x, MT * NTs);
  const int nt = L / MT, mt = L % MT;  // m fastest: a W tile is shared inside an XCD
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int li = lane & 31, lh = lane >> 5, wr = wave >> 2, wc = wave & 3;
  const int m0 = mt * 256, n0 = nt * 256;
  // this wave's 3 fragments of every chunk: f = 3 wave + i; f < 24: A (row block f / 3, plane f % 3)
  const bf16x8* src[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int f = 3 * wave + i;
    if (f < 24) {
      int rb = m0 / 32 + f / 3;
      rb = rb < RB ? rb : RB - 1;
      src[i] = ua3 + ((size_t)rb * KC * 3 + f % 3) * 64 + lane;
    } else {
      const int cb = n0 / 32 + (f - 24) / 3;
      src[i] = w3 + ((size_t)cb * KC * 3 + (f - 24) % 3) * 64 + lane;
    }
  }
  auto issue = [&](int kc, int buf) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src[i] + (size_t)kc * 3 * 64),
                                       (__attribute__((address_space(3))) void*)(&stg[buf][(3 * wave + i) * 64]),
                                       16, 0, 0);
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
  issue(0, 0);
  if (KC > 1) issue(1, 1);
  for (int kc = 0; kc < KC; ++kc) {
    // chunk kc landed (this wave's part: at most chunk kc + 1's three loads still in flight)
    if (kc + 1 < KC)
      asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // everywhere; and every wave has read chunk kc - 1's buffer
    if (kc + 2 < KC) issue(kc + 2, (kc + 2) % VB5_NBUF);
    const bf16x8* sb = stg[kc % VB5_NBUF];
    bf16x8 fa[2][3], fw[2][3];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        fa[a][q] = sb[((2 * wr + a) * 3 + q) * 64 + lane];
        fw[a][q] = sb[(24 + (2 * wc + a) * 3 + q) * 64 + lane];
      }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) x3_step(acc[a][c], fa[a], fw[c]);
  }
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = n0 + wc * 64 + c * 32 + li;
    const bool valid = col < V;
    const float bv = bias[col];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      float x[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        x[r] = acc[a][c][r] + bv;
        const int row = m0 + wr * 64 + a * 32 + acc_row(r, lane);
        if (row < R) logits[(int64_t)row * Vp + col] = x[r];
        x[r] = valid ? x[r] : -INFINITY;
      }
      const float2 sm = granule_summary(x, valid, li, lh);
      const int row = m0 + wr * 64 + a * 32 + sum_row(li, lh);
      if (!(li & 1) && row < R) gsum[(int64_t)row * NG + (n0 + wc * 64 + c * 32) / 32] = sm;
    }
  }
}

// Selection from the granule summaries: one wave per row (K waves per image).  Row log-sum-exp
// ls = log(sum_g s_g exp(m_g - M)) (lane-strided granules in order, then the wave tree); the row's
// top-K tokens lie in the granules whose max reaches the K-th largest granule max (ties kept), so
// only those granules' logits are read.  Wave 0 lane 0 then merges the image's K x K candidates.
__global__ __launch_bounds__(512) void k_beam_select3(int K, int V, int Vp, int R, int t, int end_id,
                                                      const float* __restrict__ logits,
                                                      const float2* __restrict__ gsum, float* __restrict__ cum,
                                                      int* __restrict__ fin, int64_t* __restrict__ tok,
                                                      int* __restrict__ par, int* __restrict__ htok,
                                                      int* __restrict__ hpar) {
  constexpr int GPL = 8;  // granule summaries held per lane: NG <= 512 (V <= 16384)
  __shared__ float s_mx[BEAM_MAX], s_ls[BEAM_MAX];
  __shared__ uint64_t s_top[BEAM_MAX][BEAM_MAX];
  __shared__ int s_cand[BEAM_MAX][64 * GPL];
  const int b = blockIdx.x, lane = threadIdx.x & 63, k = threadIdx.x >> 6;
  const int NG = Vp / 32;
  const int row = b * K + k;
  const bool live = !(t == 0 && k > 0) && fin[row] == 0;  // uniform over the wave
  if (live) {
    const float2* gs = gsum + (int64_t)row * NG;
    float gm[GPL], gv[GPL];
#pragma unroll
    for (int i = 0; i < GPL; ++i) {
      const int g = lane + 64 * i;
      const float2 x = g < NG ? gs[g] : make_float2(-INFINITY, 0.f);
      gm[i] = x.x;
      gv[i] = x.y;
    }
    float M = -INFINITY;
#pragma unroll
    for (int i = 0; i < GPL; ++i) M = fmaxf(M, gm[i]);
    M = wave_max(M);
    float S = 0.f;
#pragma unroll
    for (int i = 0; i < GPL; ++i)
      if (gm[i] != -INFINITY) S += gv[i] * expf(gm[i] - M);
    S = wave_sum(S);
    // K-th largest granule max (by value, then lower granule first)
    uint64_t prev = ~0ull, kth = 0;
    for (int j = 0; j < K; ++j) {
      uint64_t best = 0;
#pragma unroll
      for (int i = 0; i < GPL; ++i) {
        const int g = lane + 64 * i;
        const uint64_t key = (g < NG && gm[i] != -INFINITY) ? argmax_key(gm[i], g) : 0ull;
        if (key < prev && key > best) best = key;
      }
      best = wave_max_u64(best);
      prev = best;
      kth = best;
    }
    const float theta = key_value((uint32_t)(kth >> 32));
    // candidate granules (gm >= theta), compacted in granule order
    int n = 0;
#pragma unroll
    for (int i = 0; i < GPL; ++i) {
      const bool c = (lane + 64 * i) < NG && gm[i] != -INFINITY && gm[i] >= theta;
      const uint64_t bal = __ballot(c);
      if (c) s_cand[k][n + __popcll(bal & ((1ull << lane) - 1))] = lane + 64 * i;
      n += __popcll(bal);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const float* x = logits + (int64_t)row * Vp;
    prev = ~0ull;
    for (int j = 0; j < K; ++j) {
      uint64_t best = 0;
      for (int e = lane; e < n * 32; e += 64) {
        const int c = s_cand[k][e >> 5] * 32 + (e & 31);
        const uint64_t key = c < V ? argmax_key(x[c], c) : 0ull;
        if (key < prev && key > best) best = key;
      }
      best = wave_max_u64(best);
      if (lane == 0) s_top[k][j] = best;
      prev = best;
    }
    if (lane == 0) {
      s_mx[k] = M;
      s_ls[k] = logf(S);
    }
  }
  __syncthreads();
  // merge on wave 0: lane q K + j holds beam q's j-th candidate (a finished beam: only j = 0, the
  // token end_id at its unchanged score) as a key ordered by score, then by the smaller q V + v;
  // K rounds of a wave max pick the survivors, each written by the lane that holds it.  (Per-thread
  // candidate arrays indexed at run time lived in scratch memory: 12-20 us per launch.)
  if (threadIdx.x < 64) {
    const int q = lane / K, j = lane - q * K;
    uint64_t key = 0;
    int qfin = 0;
    if (q < K && !(t == 0 && q > 0)) {
      const float ocum = cum[b * K + q];
      qfin = fin[b * K + q];
      if (qfin) {
        if (j == 0) key = argmax_key(ocum + 0.0f, q * V + end_id);
      } else {
        const uint64_t tk = s_top[q][j];
        const float xv = key_value((uint32_t)(tk >> 32));
        key = argmax_key((ocum + ((xv - s_mx[q]) - s_ls[q])) + 0.0f, q * V + (int)key_token(tk));
      }
    }
    for (int jj = 0; jj < K; ++jj) {
      const uint64_t best = wave_max_u64(key);
      if (key == best && best != 0) {  // candidates are distinct (distinct q V + v)
        const int cf = (int)(0xFFFFFFFFu - (uint32_t)best);
        const int pk = cf / V, c = cf - pk * V, r = b * K + jj;
        cum[r] = key_value((uint32_t)(best >> 32));
        fin[r] = (qfin || c == end_id) ? 1 : 0;
        tok[r] = c;
        par[r] = b * K + pk;
        htok[(int64_t)t * R + r] = c;
        hpar[(int64_t)t * R + r] = pk;
        key = 0;
      }
    }
  }
}

struct BeamWS {
  float *a_g, *V, *vwv, *vg, *xg1, *xg, *h[2], *c[2], *s, *u, *part, *logits, *cum, *ahist, *bhist;
  float2* gsum;
  bf16x8 *hsp[2], *u3;
  int64_t *tok0, *tok;
  int *par, *fin, *htok, *hpar, *path;
};
static BeamWS carve_beam(char* base, const Layout& L, int B, int T, int K, size_t* bytes) {
  Carver c{base};
  BeamWS w;
  const size_t R = (size_t)B * K;
  w.a_g = c.take<float>((size_t)B * L.C);
  w.V = c.take<float>((size_t)B * P * L.H);
  w.vwv = c.take<float>((size_t)B * P * PP);
  w.vg = c.take<float>((size_t)B * L.E);
  w.xg1 = c.take<float>((size_t)B * L.N5);
  w.xg = c.take<float>(R * L.N5);
  for (int i = 0; i < 2; ++i) {
    w.h[i] = c.take<float>(R * L.H);
    w.c[i] = c.take<float>(R * L.H);
    w.hsp[i] = c.take<bf16x8>(hsp_frags(L, (int)R));
  }
  w.s = c.take<float>(R * L.H);
  w.u = c.take<float>(R * L.H);
  w.part = c.take<float>(R * (L.H / 16) * PART);
  w.u3 = c.take<bf16x8>(hsp_frags(L, (int)R));
  w.logits = c.take<float>(R * L.Vp);
  w.gsum = c.take<float2>(R * (L.Vp / 32));
  w.cum = c.take<float>(R);
  w.ahist = c.take<float>((size_t)T * R * P);
  w.bhist = c.take<float>((size_t)T * R);
  w.tok0 = c.take<int64_t>(R);
  w.tok = c.take<int64_t>(R);
  w.par = c.take<int>(R);
  w.fin = c.take<int>(R);
  w.htok = c.take<int>((size_t)T * R);
  w.hpar = c.take<int>((size_t)T * R);
  w.path = c.take<int>((size_t)B * T);
  *bytes = c.off;
  return w;
}

static int beam_check(const aa_dims* d, int B, int T, int K) {
  if (!d) return AA_ERR_NULL;
  if (aa_check_dims(d) != AA_OK) return AA_ERR_DIMS;
  if (d->vocab > 256 * BEAM_VPT) return AA_ERR_DIMS;
  if (B < 0 || T < 0 || K < 1 || K > BEAM_MAX || K > d->vocab) return AA_ERR_SHAPE;
  if ((int64_t)B * K > (int64_t)1 << 24) return AA_ERR_SHAPE;
  return AA_OK;
}

}  // namespace aa

using namespace aa;

size_t aa_beam_workspace_bytes(const aa_dims* d, int32_t B, int32_t T, int32_t K) {
  if (beam_check(d, B, T, K) != AA_OK) return 0;
  size_t n;
  carve_beam(nullptr, make_layout(*d), B, T, K, &n);
  return n;
}

int aa_beam_decode(const aa_model* m, const float* feats, int32_t B, int32_t T, int32_t K, int32_t end_id,
                   int64_t* ids, int64_t* seqs, float* scores, float* alpha, float* beta, void* workspace,
                   size_t workspace_bytes, int32_t flags, aa_stream_t stream, aa_event_t* vocab_events) {
  Layout L;
  int rc = check_model(m, &L);
  if (rc) return rc;
  rc = beam_check(&m->dims, B, T, K);
  if (rc) return rc;
  if (end_id >= L.V) return AA_ERR_SHAPE;
  if (B == 0 || T == 0) return AA_OK;
  if (!feats || !workspace) return AA_ERR_NULL;
  if (!al16(feats) || !al16(workspace)) return AA_ERR_ALIGN;
  size_t need;
  BeamWS w = carve_beam(static_cast<char*>(workspace), L, B, T, K, &need);
  if (workspace_bytes < need) return AA_ERR_BUFFER;
  hipStream_t s = (hipStream_t)stream;
  const MP p = resolve(m, L);
  const int H = L.H, R = B * K;
  const bool exact = (flags & AA_BEAM_FAST) == 0;  // default: exact fp32 logits
  // encoder tail for the B images; h0 / c0 / x_g expanded to the R = B*K rows
  rc = encoder_launch(L, p, feats, B, w.a_g, w.V, w.vg, w.h[1], w.c[1], w.vwv, w.xg1, nullptr, 0, s);
  if (rc) return rc;
  auto expand = [&](const float* src, int n, float* dst) {
    hipLaunchKernelGGL(k_expand_rows, dim3((unsigned)(((int64_t)R * (n / 4) + 255) / 256)), dim3(256), 0, s, src, B, K,
                       n, dst);
  };
  expand(w.h[1], H, w.h[0]);
  expand(w.c[1], H, w.c[0]);
  expand(w.xg1, L.N5, w.xg);
  hipLaunchKernelGGL(k_split_rows, dim3((unsigned)(((int64_t)R * (H / 8) + 255) / 256)), dim3(256), 0, s, w.h[0], R, H,
                     w.hsp[0]);
  hipLaunchKernelGGL(k_fill_tok, dim3((R + 255) / 256), dim3(256), 0, s, w.tok0, R, (int64_t)1);  // <start>
  AA_TRY(hipMemsetAsync(w.cum, 0, sizeof(float) * R, s));
  AA_TRY(hipMemsetAsync(w.fin, 0, sizeof(int) * R, s));
  const int MT = (R + 63) / 64;
  for (int t = 0; t < T; ++t) {
    const int cur = t & 1, nxt = cur ^ 1;
    lstm_atten_launch(L, p, R, t ? w.tok : w.tok0, 1, w.V, w.vwv, w.xg, w.hsp[cur], w.c[cur], w.h[nxt], w.hsp[nxt],
                      w.c[nxt], w.s, w.part, w.u, nullptr, nullptr, w.ahist + (size_t)t * R * P, P,
                      w.bhist + (size_t)t * R, 1, nullptr, t, s, t ? w.par : nullptr, K, exact ? nullptr : w.u3);
    if (exact) {
      if (flags & AA_DECODE_EXACT_VOCAB) rec(vocab_events, 2 * t, s);
      // exact fp32 logits (k_vocab's fma chains, pitch Vp) and their granule summaries: one fused
      // launch (k_vexact), or -- AA_DECODE_EXACT_VOCAB, the cross-check -- k_vocab then k_gsumm
      if (flags & AA_DECODE_EXACT_VOCAB) {
        hipLaunchKernelGGL(k_vocab, dim3(MT * (L.Vp / 64)), dim3(256), 0, s, R, H, L.V, L.Vp, L.Vp, w.u, p.mlp_w,
                           p.mlp_b, w.logits, (uint64_t*)nullptr);
        hipLaunchKernelGGL(k_gsumm, dim3((unsigned)((((R + 31) / 32) * (L.Vp / 32) + 3) / 4)), dim3(256), 0, s, R,
                           L.V, L.Vp, w.logits, w.gsum);
      } else {
        AA_TLAUNCH(vocab_events, 2 * t, k_vexact, dim3(((R + VX_BM - 1) / VX_BM) * (L.Vp / VX_BN)), dim3(256), 0, s,
                   R, H, L.V, L.Vp, (const float*)w.u, p.mlp_w, p.mlp_b, w.logits, w.gsum);
      }
      if (flags & AA_DECODE_EXACT_VOCAB) rec(vocab_events, 2 * t + 1, s);
      hipLaunchKernelGGL(k_beam_select3, dim3(B), dim3(64 * K), 0, s, K, L.V, L.Vp, R, t, end_id < 0 ? -1 : end_id,
                         w.logits, w.gsum, w.cum, w.fin, w.tok, w.par, w.htok, w.hpar);
    } else {
#define AA_VB3(H_)                                                                                            \
  if (wide)                                                                                                   \
    AA_TLAUNCH(vocab_events, 2 * t, k_vbeam5<H_>, dim3(((R + 255) / 256) * (L.Vp / 256)), dim3(1024), 0, s, R, L.V, \
               L.Vp, (const bf16x8*)w.u3, p.mlp_w3, p.mlp_b, w.logits, w.gsum);                                 \
  else                                                                                                        \
    AA_TLAUNCH(vocab_events, 2 * t, k_vbeam4<H_>, dim3(((R + 127) / 128) * (L.Vp / 128)), dim3(256), 0, s, R, L.V, \
               L.Vp, (const bf16x8*)w.u3, p.mlp_w3, p.mlp_b, w.logits, w.gsum)
      // 256 x 256 tiles when the padded vocabulary is whole 256-column tiles (V = 10,123: 40 of them)
      const bool wide = L.Vp % 256 == 0;  // else 128 x 128 tiles (k_vbeam4)
      switch (H) {
        case 256: AA_VB3(256); break;
        case 512: AA_VB3(512); break;
        case 768: AA_VB3(768); break;
        default: AA_VB3(1024); break;
      }
#undef AA_VB3
      hipLaunchKernelGGL(k_beam_select3, dim3(B), dim3(64 * K), 0, s, K, L.V, L.Vp, R, t, end_id < 0 ? -1 : end_id,
                         w.logits, w.gsum, w.cum, w.fin, w.tok, w.par, w.htok, w.hpar);
    }
  }
  hipLaunchKernelGGL(k_beam_final, dim3(B), dim3(256), 0, s, K, T, R, w.htok, w.hpar, w.cum, w.ahist, w.bhist, w.path,
                     ids, seqs, scores, alpha, beta);
  return launch_status();
}

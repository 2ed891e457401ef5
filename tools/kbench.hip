// Kernel-level timing harness (tools only, not part of the product): includes the product kernels,
// re-launches one of them `reps` times on a workspace populated by a real aa_greedy_decode, and
// returns the mean time per launch.  Variants under study live below as copies.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fPIC -shared -Iinclude \
//         tools/kbench.hip -o tools/_build/libkbench.so      (driven by tools/kbench.py)
#include "../adaptive_amd/csrc/aa_kernels.hip"
#include <stdlib.h>

using namespace aa;

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
      hipLaunchKernelGGL(k_vrescore, dim3(B), dim3(256), 0, s, B, L.H, L.V, L.Vp, w.u, w.summ, p.mlp_w, p.mlp_b, kt,
                         (int64_t*)nullptr, T, t);
    } else if (!strcmp(which, "enc_v3")) {
      const int M = B * P;
      hipLaunchKernelGGL(k_enc_v3, dim3(((M + EV_BM - 1) / EV_BM) * (H / EV_BN)), dim3(256), 0, s, feats, B, L.C, H, p.enc_w3, p.enc_a_b, w.V);
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

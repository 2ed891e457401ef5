/*
 * adaptive_amd.h — C-ABI of the MI355X-native adaptive-attention ("Knowing When to Look")
 * greedy-decode path.  Plain C: device pointers, sizes, opaque stream/event handles.
 *
 * The reference has no FFI: its boundary is the Python module API of
 *   code_src/models/adaptive_attention.py:159-216  (Encoder2Decoder, .sampler)
 *   code_src/models/baseline_attention.py:36-62    (AttentiveCNN.forward, the encoder tail)
 *   code_src/models/baseline_attention.py:148-194  (Decoder.forward, one step when T == 1)
 * Each entry point below names the reference interface it replaces.  The Python host layer
 * (adaptive_amd/adaptive_attention.py) binds them with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - All tensors are fp32 (ids int64), contiguous, row-major, caller-owned DEVICE memory.
 *  - No call allocates memory or synchronises the stream; scratch comes from a caller-provided
 *    workspace whose size is returned by the *_workspace_bytes queries.  Every launch goes to
 *    the given stream, so a caller may capture a call into a hipGraph.
 *  - Return value: 0 = success; negative = argument/shape error (see AA_ERR_*); positive = the
 *    hipError_t of a failed HIP call.  Nothing throws across the ABI.
 *  - Stateless and re-entrant: no hidden globals.
 *  - Load the library only after the process's HIP runtime is loaded (e.g. after `import torch`)
 *    so that one libamdhip64.so.7 serves both.
 */
#ifndef ADAPTIVE_AMD_H
#define ADAPTIVE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AA_ABI_VERSION 16
#define AA_API __attribute__((visibility("default")))

/* error codes (negative); positive codes are hipError_t values */
#define AA_OK 0
#define AA_ERR_NULL (-1)      /* a required pointer is NULL */
#define AA_ERR_DIMS (-2)      /* unsupported model dimensions */
#define AA_ERR_SHAPE (-3)     /* bad batch size / step count */
#define AA_ERR_BUFFER (-4)    /* packed-weight or workspace buffer too small */
#define AA_ERR_ALIGN (-5)     /* a pointer is not 16-byte aligned */

typedef void* aa_stream_t; /* hipStream_t (NULL = legacy default stream) */
typedef void* aa_event_t;  /* hipEvent_t */

/* Model dimensions: cf.adaptive_word_embed_size, cf.adaptive_lstm_hidden_size, cf.vocab_length
 * (code_src/config/cfg_wzn.py:115-116, code_src/train.py:40), ResNet channels and 7x7 locations.
 * Supported: embed % 32 == 0, hidden % 256 == 0 and <= 1024, vocab >= 1, channels % 32 == 0,
 * spatial == 49. */
typedef struct aa_dims {
  int32_t embed;    /* E = 256 */
  int32_t hidden;   /* H = 512 */
  int32_t vocab;    /* V = 10123 */
  int32_t channels; /* C = 2048 */
  int32_t spatial;  /* P = 49 */
} aa_dims;

/* Parameters in the reference state-dict layout (device pointers, fp32, contiguous).
 * Names follow Encoder2Decoder.state_dict() keys. */
typedef struct aa_ref_weights {
  const float* enc_affine_a_w;  /* encoder.affine_a.weight  [H, C] */
  const float* enc_affine_a_b;  /* encoder.affine_a.bias    [H]    */
  const float* enc_affine_b_w;  /* encoder.affine_b.weight  [E, C] */
  const float* enc_affine_b_b;  /* encoder.affine_b.bias    [E]    */
  const float* enc_affine_h0_w; /* encoder.affine_h0.weight [H, C] */
  const float* enc_affine_h0_b; /* encoder.affine_h0.bias   [H]    */
  const float* enc_affine_c0_w; /* encoder.affine_c0.weight [H, C] */
  const float* enc_affine_c0_b; /* encoder.affine_c0.bias   [H]    */
  const float* embed_w;         /* decoder.embed.weight     [V, E] */
  const float* lstm_w_ih;       /* decoder.LSTM.weight_ih_l0 [4H, 2E] (gates i,f,g,o) */
  const float* lstm_w_hh;       /* decoder.LSTM.weight_hh_l0 [4H, H]  */
  const float* lstm_b_ih;       /* decoder.LSTM.bias_ih_l0   [4H]     */
  const float* lstm_b_hh;       /* decoder.LSTM.bias_hh_l0   [4H]     */
  const float* sent_affine_x_w; /* decoder.adaptive.sentinel.affine_x.weight [H, 2E] */
  const float* sent_affine_h_w; /* decoder.adaptive.sentinel.affine_h.weight [H, H]
                                   (multiplies h_{t-1} = 0 while sampling; may be NULL) */
  const float* att_affine_v_w;  /* decoder.adaptive.atten.affine_v.weight [P, H] */
  const float* att_affine_g_w;  /* decoder.adaptive.atten.affine_g.weight [P, H] */
  const float* att_affine_s_w;  /* decoder.adaptive.atten.affine_s.weight [P, H] */
  const float* att_affine_h_w;  /* decoder.adaptive.atten.affine_h.weight [1, P] */
  const float* mlp_w;           /* decoder.adaptive.mlp.weight [V, H] */
  const float* mlp_b;           /* decoder.adaptive.mlp.bias   [V]    */
} aa_ref_weights;

/* Gradient outputs of aa_train_backward, same fields and shapes as aa_ref_weights. */
typedef struct aa_ref_grads {
  float* enc_affine_a_w;
  float* enc_affine_a_b;
  float* enc_affine_b_w;
  float* enc_affine_b_b;
  float* enc_affine_h0_w;
  float* enc_affine_h0_b;
  float* enc_affine_c0_w;
  float* enc_affine_c0_b;
  float* embed_w;
  float* lstm_w_ih;
  float* lstm_w_hh;
  float* lstm_b_ih;
  float* lstm_b_hh;
  float* sent_affine_x_w;
  float* sent_affine_h_w;
  float* att_affine_v_w;
  float* att_affine_g_w;
  float* att_affine_s_w;
  float* att_affine_h_w;
  float* mlp_w;
  float* mlp_b;
} aa_ref_grads;

/* A model = dims + a caller-owned device buffer holding the packed (kernel-layout) weights. */
typedef struct aa_model {
  aa_dims dims;
  void* packed;        /* device buffer, >= aa_packed_bytes(&dims) bytes, 256-B aligned */
  size_t packed_bytes;
} aa_model;

/* Optional per-kernel timing (hipEvent_t handles created by the caller), one array per kernel so
 * the figures line up with rocprofv3's per-kernel statistics.  For each non-NULL array, the pair
 * ([2i], [2i+1]) of the i-th launch of that kernel is handed to the launch itself
 * (hipExtLaunchKernel start / stop events): it carries the dispatch's own begin / end timestamps,
 * and no event packet sits between the traced launches:
 *   encoder_events: 2*AA_TRACE_ENCODER_KERNELS events, launches in the order
 *                   k_avgpool (not launched by k_enc_v4, which fuses it: pair 0 stays unrecorded),
 *                   k_enc_v, k_enc_heads, VWv GEMM, x_g GEMM;
 *   lstm/atten/screen/rescore_events: 2*T events, launch i = step i.  screen = k_vscreen2 /
 *                   k_vscreen (k_vocab under AA_DECODE_EXACT_VOCAB), rescore = k_vrescore (unused
 *                   under AA_DECODE_EXACT_VOCAB; by default only pair T-1 is recorded: the rescoring
 *                   of steps 0..T-2 runs inside the next step's LSTM launch); lstm = k_lstm (steps
 *                   >= 1 by default include the previous step's rescoring);
 *   gemm_events:    unused (kept for layout stability; may be NULL). */
#define AA_TRACE_ENCODER_KERNELS 5
typedef struct aa_trace {
  aa_event_t* encoder_events;
  aa_event_t* lstm_events;
  aa_event_t* atten_events;
  aa_event_t* screen_events;
  aa_event_t* rescore_events;
  aa_event_t* gemm_events;
} aa_trace;

AA_API int aa_abi_version(void);
AA_API const char* aa_error_string(int code);
AA_API int aa_check_dims(const aa_dims* dims);

/* Bytes of the packed weight buffer for these dims. */
AA_API size_t aa_packed_bytes(const aa_dims* dims);

/* Pack reference-layout weights into m->packed (device-side reorder; async on `stream`).
 * Replaces: the parameter set built by Encoder2Decoder.__init__ / load_state_dict
 * (adaptive_attention.py:159-165, model_factory.py:16). */
AA_API int aa_pack_weights(const aa_model* m, const aa_ref_weights* w, aa_stream_t stream);

/* Encoder tail: a_g = AvgPool2d(7)(A); V = relu(A^T W_a^T + b_a); v_g = relu(a_g W_b^T + b_b);
 * h0/c0 = tanh(a_g W^T + b); plus the step-invariant VWv = V W_v^T used by every decode step.
 * Replaces AttentiveCNN.forward after resnet_conv (baseline_attention.py:46-62).
 * feats: [B, C, 7, 7] NCHW post-trunk features.  Outputs: a_g [B,C], V [B,P,H], v_g [B,E],
 * h0 [B,H], c0 [B,H], VWv [B,P,64] (columns >= P are zero; may be NULL).  flags: 0 or
 * AA_DECODE_FP32_ENCODER. */
AA_API int aa_encoder_tail(const aa_model* m, const float* feats, int32_t B, float* a_g, float* V,
                           float* v_g, float* h0, float* c0, float* VWv, int32_t flags,
                           aa_stream_t stream);

/* Workspace for aa_decode_step at batch B. */
AA_API size_t aa_step_workspace_bytes(const aa_dims* dims, int32_t B);

/* One greedy decode step = Decoder.forward with T == 1 (baseline_attention.py:148-194) through
 * AdaptiveBlock (adaptive_attention.py:110-134) and the argmax of Encoder2Decoder.sampler (:201).
 * tokens_in [B] int64 (NULL = <start> = 1); VWv from aa_encoder_tail (may be NULL: recomputed);
 * h_in/c_in [B,H] -> h_out/c_out [B,H]; scores [B,V] (NULL = not written); tokens_out [B] int64
 * (first index on ties); alpha [B,P]; beta [B].  h_out/c_out must not alias h_in/c_in. */
AA_API int aa_decode_step(const aa_model* m, int32_t B, const int64_t* tokens_in, const float* V,
                          const float* VWv, const float* v_g, const float* h_in, const float* c_in,
                          float* h_out, float* c_out, float* scores, int64_t* tokens_out,
                          float* alpha, float* beta, void* workspace, size_t workspace_bytes,
                          aa_stream_t stream);

/* Workspace for aa_greedy_decode at batch B and T steps. */
AA_API size_t aa_decode_workspace_bytes(const aa_dims* dims, int32_t B, int32_t T);

/* Decode flags */
#define AA_DECODE_EXACT_VOCAB 1 /* compute every fp32 logit (fp32 MFMA GEMM + fused argmax) instead of
                                   the bf16 screen + exact fp32 rescoring; both give the same ids */
#define AA_DECODE_FP32_ENCODER 2 /* V = relu(A W_a^T + b) on fp32 MFMA (v_mfma_f32_32x32x2f32) instead of
                                    the default fp32-accurate 3-way-split bf16 MFMA (k_enc_v4) */
#define AA_DECODE_ONE_STREAM 512 /* decode plans: capture the whole decode on one stream (no side-stream
                                     branch for the encoder's a_g work); for several plans in flight */
#define AA_DECODE_SPLIT_RESCORE 1024 /* rescore each step in its own launch (k_vrescore) instead of inside
                                        the next step's LSTM launch; the same ids (cross-check path) */
#define AA_DECODE_RS_SELF 2048 /* test hook: the LSTM workgroups do not wait for the rescoring workgroups
                                  of their launch but rescore every row not yet published themselves
                                  (the fallback that keeps the fused launch deadlock-free); same ids */
#define AA_DECODE_SCREEN4 4096 /* the vocab screen on four waves per 128 x 160 tile (k_vscreen2) instead
                                  of eight (k_vscreen8); the same summaries bit for bit (cross-check) */

/* Whole greedy decode = Encoder2Decoder.sampler(images, max_len=T) (adaptive_attention.py:168-216,
 * with the baseline's states transpose, baseline_attention.py:251-252).  feats [B,C,7,7];
 * ids [B,T] int64; alpha [B,T,P] and beta [B,T] may be NULL.  All T steps run (no early stop),
 * the first input token is <start> = 1.  trace may be NULL.
 * Vocab argmax (adaptive_attention.py:201): by default every logit is first bounded with a bf16
 * MFMA screen whose error is bounded rigorously (Cauchy-Schwarz on the rounding-error vectors of u
 * and w_n plus the fp32 accumulation terms, per 32-column granule);
 * only columns whose upper bound reaches the best lower bound are rescored in exact fp32 (the same
 * fma order as the fp32 GEMM), so the ids equal those of AA_DECODE_EXACT_VOCAB bit for bit. */
AA_API int aa_greedy_decode(const aa_model* m, const float* feats, int32_t B, int32_t T,
                            int64_t* ids, float* alpha, float* beta, void* workspace,
                            size_t workspace_bytes, const aa_trace* trace, int32_t flags,
                            aa_stream_t stream);

/* aa_greedy_decode with a second stream `aux_stream` for the encoder's a_g branch (heads, x_g GEMM)
 * beside the V branch's VWv GEMM.  Fork/join through events: the call is complete (and
 * graph-capturable) on `stream`.  aux_stream NULL or equal to `stream`: aa_greedy_decode.  The
 * results equal aa_greedy_decode's bit for bit. */
AA_API int aa_greedy_decode_aux(const aa_model* m, const float* feats, int32_t B, int32_t T,
                                int64_t* ids, float* alpha, float* beta, void* workspace,
                                size_t workspace_bytes, const aa_trace* trace, int32_t flags,
                                aa_stream_t stream, aa_stream_t aux_stream);

/* Decode plan: the complete greedy decode for fixed (B, T, flags) and fixed buffers, captured once
 * into a hipGraph (one graph launch replaces the ~4T+6 kernel launches).  Launch it as often as
 * needed on any stream; the buffers it was created with -- feats included -- are read/written at
 * every launch, so the caller owns them for the plan's lifetime (adaptive_amd.DecodePlan owns its
 * own input buffer and copies each batch into it).  Results equal aa_greedy_decode's bit for bit.
 * The plan captures aa_greedy_decode_aux's two-stream encoder unless flags &
 * AA_DECODE_ONE_STREAM.  It holds no device memory of its own besides the instantiated graph;
 * destroy it only after its last launch has completed. */
typedef struct aa_decode_plan aa_decode_plan;
AA_API int aa_decode_plan_create(const aa_model* m, const float* feats, int32_t B, int32_t T,
                                 int64_t* ids, float* alpha, float* beta, void* workspace,
                                 size_t workspace_bytes, int32_t flags, aa_decode_plan** plan);
AA_API int aa_decode_plan_launch(const aa_decode_plan* plan, aa_stream_t stream);
AA_API int aa_decode_plan_destroy(aa_decode_plan* plan);

/* ---- teacher-forced training step ----------------------------------------
 * Encoder2Decoder.forward(images, captions, lengths) (baseline_attention.py:206-230) and its
 * backward, fp32, deterministic.  feats [B,C,7,7]; tokens: captions [B][tok_ld] int64 (column t is
 * the input token of step t, <start> first); lengths: DEVICE int32 [B], sorted descending (as
 * pack_padded_sequence requires), T = lengths[0] steps, N = sum(lengths) packed rows.
 * aa_train_forward writes the packed scores [N][V] (pack_padded_sequence(scores, lengths).data:
 * rows t-major over the batch entries still running at step t) and keeps the activations in the
 * workspace; aa_train_backward takes dL/dscores [N][V] with the same arguments and workspace and
 * writes the gradient of every parameter (assigned, not accumulated), and, if dfeats is not NULL,
 * dL/dfeats [B,C,7,7] (the gradient into the ResNet trunk's output, for CNN fine-tuning).  The reference's loss
 * (train.py: CrossEntropyLoss on the packed scores) stays with the caller.  Token ids are not
 * validated on the device: the caller must keep them in [0, V) (the Python layer raises IndexError
 * as nn.Embedding does); an out-of-range id is clamped into [0, V) by the gather (no out-of-bounds
 * read) and then feeds the wrong embedding row. */
AA_API size_t aa_train_workspace_bytes(const aa_dims* dims, int32_t B, int32_t T);
#define AA_TRAIN_BF16 128 /* aa_train_forward / aa_train_backward flags: every GEMM on bf16 MFMA
                               (operands rounded to bf16, fp32 accumulation; BASELINE config 5's
                               "bf16 compute / fp32 master"); elementwise work and the encoder V GEMM
                               stay fp32.  0 = fp32 GEMMs (fp32 MFMA).  Pass the same flags to both. */
AA_API int aa_train_forward(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B,
                            int32_t T, const int64_t* tokens, int32_t tok_ld, const int32_t* lengths,
                            float* scores, int32_t N, void* workspace, size_t workspace_bytes,
                            int32_t flags, aa_stream_t stream);
AA_API int aa_train_backward(const aa_ref_weights* w, const aa_dims* dims, const float* feats,
                             int32_t B, int32_t T, const int64_t* tokens, int32_t tok_ld,
                             const int32_t* lengths, const float* dscores, int32_t N,
                             const aa_ref_grads* grads, float* dfeats, void* workspace,
                             size_t workspace_bytes, int32_t flags, aa_stream_t stream);
/* The same two calls with a second stream `aux` (another stream of the same device, or NULL = one
 * stream): the work off the step's dependency chain -- the encoder's spatial V GEMM beside the LSTM
 * forward, the weight gradients beside the LSTM backward -- runs on aux, handed over by events.
 * Results are bit-identical to the one-stream calls (same kernels, same arithmetic order); both
 * calls end with `stream` waiting for everything they queued on aux, so the caller orders only
 * against `stream`.  aux must not be used by anything else during a call. */
AA_API int aa_train_forward_aux(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B,
                                int32_t T, const int64_t* tokens, int32_t tok_ld, const int32_t* lengths,
                                float* scores, int32_t N, void* workspace, size_t workspace_bytes, int32_t flags,
                                aa_stream_t stream, aa_stream_t aux);
AA_API int aa_train_backward_aux(const aa_ref_weights* w, const aa_dims* dims, const float* feats, int32_t B,
                                 int32_t T, const int64_t* tokens, int32_t tok_ld, const int32_t* lengths,
                                 const float* dscores, int32_t N, const aa_ref_grads* grads, float* dfeats,
                                 void* workspace, size_t workspace_bytes, int32_t flags, aa_stream_t stream,
                                 aa_stream_t aux);

/* ---- Decoder.forward over T > 1 teacher-forced steps -------------------------------------------
 * decoder(V, v_g, captions, states) (baseline_attention.py:148-194 with the adaptive block,
 * adaptive_attention.py:110-134; called with whole captions from Encoder2Decoder.forward, :225):
 * V [B,P,H], v_g [B,E], h0 / c0 [B,H] (the states, any of the [1,B,H] / [B,1,H] views of one
 * contiguous buffer), tokens [B][tok_ld] int64 (column t feeds step t).  Every row runs all T steps
 * (no packing); the sentinel's h_{t-1} is 0 at t = 0 (init_hidden, :116-120).  Outputs (each may be
 * NULL): scores [B,T,V], alpha [B,T,P], beta [B,T], h_out / c_out [B,H] = the states after step
 * T-1.  Forward only (the training path with gradients is aa_train_forward/backward); flags:
 * AA_TRAIN_BF16 or 0 as for aa_train_forward.  Workspace: aa_decoder_workspace_bytes.  Token ids:
 * the caller keeps them in [0, V), as for aa_train_forward (out-of-range ids are clamped, not
 * reported). */
AA_API size_t aa_decoder_workspace_bytes(const aa_dims* dims, int32_t B, int32_t T);
AA_API int aa_decoder_forward(const aa_ref_weights* w, const aa_dims* dims, const float* V, const float* v_g,
                              const float* h0, const float* c0, int32_t B, int32_t T, const int64_t* tokens,
                              int32_t tok_ld, float* scores, float* alpha, float* beta, float* h_out,
                              float* c_out, void* workspace, size_t workspace_bytes, int32_t flags,
                              aa_stream_t stream);

/* ---- beam-search decode (BASELINE config 4) ------------------------------
 * Not in the reference (its for_wzn:3 lists beam search as a TODO): semantics defined here and in
 * oracle/adaptive_oracle.py BeamOracle.  K (1..AA_MAX_BEAM) hypotheses per image over the same
 * decoder step as aa_greedy_decode; at step 0 only beam 0 is live; a candidate's score is the
 * parent's cumulative score + log_softmax(logits) of the token; a beam that emitted end_id is
 * finished and carried unchanged (its only continuation is end_id at no cost; end_id < 0: none);
 * the K best candidates per image (score desc, ties to the smaller parent*V + token) survive.
 * All T steps run.  Outputs (each may be NULL): ids [B,T] int64, alpha [B,T,P], beta [B,T] of the
 * best final beam; seqs [B,K,T] int64 and scores [B,K] of all K final beams, best first.
 * Logits (default): exact fp32 -- the fma chains of aa_vocab_logits' fp32 MFMA GEMM, so the same
 * bits -- with per-32-column (max, sum exp(x - max)) summaries in a fixed butterfly order fused into
 * the GEMM epilogue (one launch per step); the selection builds each row's log-sum-exp from them.
 * flags & AA_DECODE_EXACT_VOCAB: the same values by two launches (the plain fp32 GEMM, then the
 * summaries) -- the cross-check path, bitwise equal to the default.  flags & AA_BEAM_FAST: the logits by bf16x3
 * MFMA (fp32-accurate but rounded differently) with the summaries fused into the GEMM epilogue --
 * about 2.3x faster, and the beams equal the exact ones except where two candidates are within the
 * logits' rounding difference of each other (measured: >= 98% of images at config 4).
 * Requires vocab <= 16384.  Replaces, for beam decoding, the greedy sampler's role in coco_eval
 * (code_src/tools/utils.py:171).  vocab_events (may be NULL): 2T hipEvent handles recorded on the
 * stream around each step's vocab stage (logits + summaries), for per-launch timing. */
#define AA_MAX_BEAM 8
#define AA_BEAM_FAST 256 /* aa_beam_decode: bf16x3 logits with fused summaries instead of exact fp32 */
AA_API size_t aa_beam_workspace_bytes(const aa_dims* dims, int32_t B, int32_t T, int32_t K);
AA_API int aa_beam_decode(const aa_model* m, const float* feats, int32_t B, int32_t T, int32_t K,
                          int32_t end_id, int64_t* ids, int64_t* seqs, float* scores, float* alpha,
                          float* beta, void* workspace, size_t workspace_bytes, int32_t flags,
                          aa_stream_t stream, aa_event_t* vocab_events);

/* Full fp32 vocab logits scores[B,V] = u W_m^T + b_m (AdaptiveBlock.mlp, adaptive_attention.py:132)
 * for given u = c_hat + h rows [B,H] (fp32 MFMA GEMM). */
AA_API int aa_vocab_logits(const aa_model* m, int32_t B, const float* u, float* scores,
                           aa_stream_t stream);

/* Exact fp32 vocab logits of selected columns: out[b][i] = u[b] . W_m[cols[b][i]] + b_m[cols[b][i]]
 * (AdaptiveBlock.mlp, adaptive_attention.py:132), computed in the fma order of the fp32 GEMM path,
 * i.e. bit-identical to the corresponding aa_decode_step scores.  u [B,H]; cols [B,n] int32
 * (entries outside [0, vocab) give 0); out [B,n].  Used to rescore candidate tokens. */
AA_API int aa_vocab_logits_at(const aa_model* m, int32_t B, const float* u, const int32_t* cols,
                              int32_t n, float* out, aa_stream_t stream);

/* ---- the rest of train.py's closure: CrossEntropyLoss and Adam ------------
 * aa_cross_entropy_forward: nn.CrossEntropyLoss()(logits, targets) (train.py:63,208; reduction
 * 'mean', ignore_index as torch's, default -100): logits [N][ldx] fp32 (V used columns), targets [N]
 * int64; writes loss[0] = mean over counted rows of (logsumexp(x_i) - x_i[t_i]) and count[0] = the
 * number of counted rows (as float), and keeps the per-row log-sum-exp in the workspace
 * (aa_cross_entropy_workspace_bytes(N)) for the backward.  A target outside [0, V) that is not
 * ignore_index makes the loss NaN (torch raises a device-side assert).  Deterministic (fixed-order
 * reductions).  aa_cross_entropy_backward: dlogits = (softmax(x_i) - onehot(t_i)) * dloss[0] /
 * count[0] (0 for ignored rows), dloss a DEVICE scalar (the incoming gradient of the loss), with the
 * forward's workspace (workspace_bytes >= aa_cross_entropy_workspace_bytes(N), else AA_ERR_BUFFER);
 * dlogits may alias logits (in place) only if lddx == ldx (else AA_ERR_SHAPE). */
AA_API size_t aa_cross_entropy_workspace_bytes(int32_t N);
AA_API int aa_cross_entropy_forward(const float* logits, int32_t N, int32_t V, int64_t ldx,
                                    const int64_t* targets, int64_t ignore_index, float* loss,
                                    float* count, void* workspace, size_t workspace_bytes,
                                    aa_stream_t stream);
AA_API int aa_cross_entropy_backward(const float* logits, int32_t N, int32_t V, int64_t ldx,
                                     const int64_t* targets, int64_t ignore_index, const float* dloss,
                                     const float* count, const void* workspace, size_t workspace_bytes,
                                     float* dlogits, int64_t lddx, aa_stream_t stream);

/* aa_adam_step: one torch.optim.Adam step (model_factory.py:71: Adam(params, lr, betas, weight_decay); amsgrad=False,
 * maximize=False, L2 weight_decay added to the gradient) over n fp32 tensors, every tensor in one
 * launch per AA_ADAM_MAX_TENSORS.  step = the step count AFTER this step's increment (1 on the first
 * step).  Element-wise in torch's foreach op order (optim/adam.py _multi_tensor_adam):
 * m = lerp(m, g, 1-b1); v = v*b2 + (1-b2)*g*g; p += (-lr/(1-b1^step)) * m / (sqrt(v)/sqrt(1-b2^step) + eps).
 * Tensors with numel 0 are skipped; the four pointers of a tensor must not overlap each other. */
#define AA_ADAM_MAX_TENSORS 24
typedef struct aa_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
} aa_adam_tensor;
AA_API int aa_adam_step(const aa_adam_tensor* tensors, int32_t n, double step, double lr, double beta1,
                        double beta2, double eps, double weight_decay, aa_stream_t stream);

/* aa_clip_grad_norm: torch.nn.utils.clip_grad_norm_(params, max_norm) with the 2-norm (train.py:213-214
 * clips the LSTM's gradients to 5): total = sqrt(sum_i ||g_i||^2) over the tensors' norms, coef =
 * max_norm / (total + 1e-6), every gradient multiplied in place by min(coef, 1) (NaN kept); the total
 * norm is written to total_norm (a device float).  Fixed reduction order: deterministic.  Up to
 * AA_CLIP_MAX_TENSORS tensors; workspace from aa_clip_grad_norm_workspace_bytes (0 = invalid input). */
#define AA_CLIP_MAX_TENSORS 24
typedef struct aa_grad_tensor {
  float* grad;
  int64_t numel;
} aa_grad_tensor;
AA_API size_t aa_clip_grad_norm_workspace_bytes(const aa_grad_tensor* tensors, int32_t n);
AA_API int aa_clip_grad_norm(const aa_grad_tensor* tensors, int32_t n, float max_norm, float* total_norm,
                             void* workspace, size_t workspace_bytes, aa_stream_t stream);

/* Measurement helper (bench.py's roofline block; not on the decode path): one streaming read of
 * nbytes (multiple of 16, 16-B aligned) from src by `blocks` workgroups, each writing its partial sum
 * to out[block].  Timed over a buffer resident in the 256 MiB Infinity Cache it gives the MALL-served
 * read ceiling that the attention's per-step re-read of V is priced against. */
AA_API int aa_read_probe(const void* src, size_t nbytes, float* out, int32_t blocks, aa_stream_t stream);

/* Counter-based synthetic data (same bits as adaptive_amd/synth.py):
 * dst[i] = fp32(lo + (hi - lo) * u(key, start + i)), u = (splitmix64(key + (start+i+1)*GOLDEN) >> 40) / 2^24.
 * For lo = 0, hi = 1 the value is u exactly. */
AA_API int aa_synth_uniform(float* dst, int64_t n, uint64_t key, int64_t start, double lo,
                            double hi, aa_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ADAPTIVE_AMD_H */

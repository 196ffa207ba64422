/* endossl C-ABI: the MI355X (gfx950) kernels behind the FixMatch / CoMatch SSL training step.
 *
 * libendossl_hip.so exports exactly these functions.  Conventions:
 *  - every pointer is a caller-owned DEVICE pointer; no function allocates or synchronises;
 *  - every call takes the HIP stream it is enqueued on (last argument) and returns an int
 *    status: 0 = OK, -1 = bad shape, -2 = bad argument (null / inconsistent), -3 = HIP error;
 *  - no C++ exception crosses this boundary; functions are stateless and re-entrant;
 *  - bf16 tensors are passed as void* (raw 16-bit bfloat16 storage), fp32 as float*;
 *  - token-major activations are row-major [tokens, features]; buffers read by the GEMMs are
 *    padded to a multiple of 256 rows whose pad rows are zero (DESIGN.md "HBM layout").
 *
 * The reference has no FFI (pure Python / PyTorch); each entry point cites the
 * reference computation it replaces.  The Python host side (endossl/_lib.py) binds them with
 * ctypes exactly as INTEGRATION.md shows.
 */
#ifndef ENDOSSL_H
#define ENDOSSL_H
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- identity ---------------------------------------------------------------------------- */
int es_abi_version(void);

/* ---- GEMMs (code/models/conformer.py:13-23,35-50 nn.Linear; timm PatchEmbed Conv2d) ------- */
/* C[M,N] = A[M,K] . B[N,K]^T with a fused epilogue:
 *   epi 0: C bf16 = acc (+bias)                      (qkv, dgrad to a bf16 operand)
 *   epi 1: C bf16 = acc+bias, C2 bf16 = GELU(acc+bias) (Mlp.fc1 + act, conformer.py:19-20)
 *   epi 2: C f32 = acc (+bias) + aux f32              (Attention.proj / Mlp.fc2 + residual, :70-71)
 *   epi 3: C bf16 = acc * GELU'(aux bf16)             (fc2 dgrad through the activation)
 *   epi 4: C f32 = acc (+bias)                        (dgrad into LayerNorm backward)
 *   epi 5: C f32 at token row img*(np+1)+1+p = acc + bias + aux[1+p]   (patch embed + pos_embed)
 *   epi 6: C bf16 = GELU(acc+bias) only                (fc1 + act in inference forwards)
 *   epi 7: C bf16 = GELU'(acc+bias), C2 bf16 = GELU(acc+bias)   (train fc1: keeps the derivative, not the
 *          pre-activation, so the backward needs no erf; activation bits identical to epi 1)
 *   epi 8: C bf16 = acc * aux bf16                     (fc2 dgrad times the stored GELU')
 * N % 128 == 0, K % 64 == 0; A readable for round_up(M,256) rows. */
int es_gemm_nt(int epi, const void* A, int lda, const void* B, int ldb, const float* bias, void* C, int ldc,
               void* C2, const void* aux, int ldaux, int M, int N, int K, int np, hipStream_t stream);
/* x = A B^T + bias + aux, h = LayerNorm(x; gamma, beta, eps) with per-row mean / rstd, in one launch, for
 * N == K == 384 (ViT-S's attention projection followed by norm2): the bits of es_gemm_nt(epi 2) followed by
 * es_layernorm_fwd.  x fp32 [M, ldc], aux fp32 [M, ldaux] (16-B aligned rows), h bf16 [M, ldh]; bias nullable.
 * Replaces code/models/conformer.py:65-66 (x + attn(...), then norm2).  ES_BAD_SHAPE for other N / K;
 * ES_BAD_ARG for a null or misaligned operand (A, B, aux, gamma, beta, bias 16-B; C 8-B; h 4-B). */
int es_gemm_nt_resid_ln(const void* A, int lda, const void* B, int ldb, const float* bias, float* C, int ldc,
                        const float* aux, int ldaux, const float* gamma, const float* beta, void* h, int ldh,
                        float* mean, float* rstd, int M, int N, int K, float eps, hipStream_t stream);
/* tuning knob: NT kernel family (-1 = per-shape default; 0, 1, 2, 5, 6, 10, 11 = fixed tilings, see gemm.hip;
 * 12 = the weight-stationary K = 384 kernel where it applies -- epi 0 / 1 / 4 / 6 / 7, K == 384, N a multiple
 * of 384 up to 3072 -- and the per-shape rules elsewhere; opt-in, bit-identical to the tilings);
 * returns the old one, or -2 (state unchanged) for a family that does not exist */
int es_set_gemm_variant(int variant);
/* 1 (default): the 64 x 128 NT tile rules (N <= 384 outputs of small token shards, M < 32768, and the residual
 * proj forward); 0: without them.  Returns the old value. */
int es_set_gemm_small_tile(int v);
/* weight gradient: out[N1,N2] (+)= sum_m A1[m,N1]^T A2[m,N2], token axis split `splits` ways into
 * fp32 slabs (workspace = es_gemm_tn_workspace floats) and reduced; bias_out (nullable) (+)=
 * sum_m A1[m,:] computed from the same tiles.  splits <= 0: sized by the library for the kernel it
 * picks (es_gemm_tn_workspace(N1, N2, 0) bounds the workspace).  N1,N2 % 128 == 0, or N1 % 384 == 0
 * and N2 % 192 == 0; rows in [M, round_up(M,64)) of A1 must be zero. */
/* tuning knob for es_gemm_tn: -1 = default (384x192 tile for M >= 65536 where it tiles, else
 * 128x128), 0 = the 128x128 tile (32-token steps, two stages), 7 = the 384x192 tile (64-token steps,
 * two stages); a pin >= 0 also overrides the variant es_gemm_tn_ex callers pass.  Returns the previous
 * value, or -2 (state unchanged) for any other value */
int es_set_tn_variant(int variant);
size_t es_gemm_tn_workspace(int N1, int N2, int splits);
int es_gemm_tn(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
               float* workspace, float* out, int accumulate, float* bias_out, hipStream_t stream);
/* es_gemm_tn with an explicit kernel choice (0 or 7, the es_set_tn_variant numbering; -1 = the
 * library's per-shape choice; anything else -2): the engine passes the 384x192 tile for its
 * CU-share-sized launches this way instead of toggling the global knob around each call */
int es_gemm_tn_ex(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
                  float* workspace, float* out, int accumulate, float* bias_out, int variant, hipStream_t stream);
int es_splitk_reduce(const float* P, float* out, int S, int n, int accumulate, hipStream_t stream);
/* Grouped weight gradients: many independent es_gemm_tn problems in ONE launch, each 128x128 tile
 * over its problem's whole token axis (no split-K slabs, no reduction launches) -- the small-shard
 * backward (strong scaling: M = 12,608 tokens per rank at N = 8), where split-K slabs and per-GEMM
 * reductions cost more than the products.  N1, N2 % 128 == 0; rows [M, round_up(M, 32)) of dy zero;
 * out / bias_out overwritten.  es_gemm_tn_grouped_prepare fills mchunk / tile0 of a HOST table and
 * returns the total tile count; the caller copies the table to the device and launches. */
typedef struct {
  const void* dy;     /* A1 [M, N1] bf16, row stride ld1 */
  const void* x;      /* A2 [M, N2] bf16, row stride ld2 */
  float* out;         /* [N1, N2] fp32 */
  float* bias_out;    /* [N1] fp32 column sums of dy, nullable */
  int M, N1, N2, ld1, ld2;
  int mchunk, tile0, pad;  /* filled by es_gemm_tn_grouped_prepare */
} es_tn_problem;
size_t es_tn_problem_size(void);
int es_gemm_tn_grouped_prepare(void* host_table, int count);
int es_gemm_tn_grouped(const void* device_table, int count, int total_tiles, hipStream_t stream);
/* A Linear layer's weight gradients as ONE split-K launch on the 384x192 tile (the long-token-axis
 * backward: fc1 + fc2 + qkv + proj of a ViT block in one grid), then ONE reduce launch over every
 * problem's fp32 slabs and bias partials.  Input: `count` es_tn_problem entries (dy, x, out, bias_out,
 * M, N1, N2, ld1, ld2; mchunk / tile0 / pad ignored), N1 % 384 == 0, N2 % 192 == 0, rows
 * [M, round_up(M, 64)) of dy zero; out / bias_out overwritten.  Every problem gets
 * max(1, target_wgs / its-and-the-others' 384x192 tiles) splits (at most one per 64 tokens), so the
 * slabs are S x the layer's outputs with S a few, not 16-32 per GEMM (one split: written in place).
 * count <= 8.  _prepare writes the table (es_gemm_tn_big_grouped_table_bytes(count) bytes of HOST memory;
 * es_gemm_tn_big_grouped passes it by value in the kernel arguments) and dims[3] = {workgroups, reduce
 * blocks, reduce entries}; workspace >= es_gemm_tn_big_grouped_workspace floats.  Replaces the per-Linear es_gemm_tn launches of code/models/conformer.py:13-23,35-50's
 * backward (autograd's addmm weight gradients). */
size_t es_gemm_tn_big_grouped_table_bytes(int count);
size_t es_gemm_tn_big_grouped_workspace(const void* problems, int count, int target_wgs);
int es_gemm_tn_big_grouped_prepare(const void* problems, int count, int target_wgs, float* workspace,
                                   size_t workspace_floats, void* table, int* dims);
int es_gemm_tn_big_grouped(const void* table, int count, const int* dims, hipStream_t stream);
/* the same launch with timing: `start` is stamped at the grouped kernel's own start, `stop` at the end of its
   reduce launch (hipExtLaunchKernelGGL events: the kernels' execution, as a rocprofv3 kernel trace sees it, not
   the stream position of a hipEventRecord).  Events from es_event_create. */
int es_gemm_tn_big_grouped_timed(const void* table, int count, const int* dims, void* start, void* stop,
                                 hipStream_t stream);
/* timing events for the *_timed launches (hipEvent_t handles): create, elapsed ms (waits for `stop`), destroy */
int es_event_create(void** ev);
int es_event_elapsed(void* start, void* stop, float* ms);
int es_event_destroy(void* ev);
/* bias gradient: out[n] (+)= sum_m Y[m][n]  (workspace >= blocks*N floats) */
int es_colsum(const void* Y, int ld, int M, int N, float* workspace, int blocks, float* out, int accumulate,
              hipStream_t stream);
/* out[n] (+)= sum_g P[g][n]  (per-workgroup partials -> parameter gradient) */
int es_reduce_partials(const float* P, float* out, int G, int N, int accumulate, hipStream_t stream);

/* tuning knob: forward attention kernel -- 7 (default) = seven waves per workgroup at 13 key tiles (193 <= T <= 208: ViT/16 at 224^2),
   else as 2; 2 = four waves, register budget of two workgroups per CU; 3 = four waves, three per CU;
   returns previous */
int es_set_attn_variant(int occ);
/* attention backward loops: 4 (default) = the single-pass kernel for 13-tile heads (192 < T <= 208), else
   as 3; 3 = two query / key tiles per wave item (dq2 / dkv2), 2 = pipelined dQ + dkv2, 1 = software-pipelined,
   0 = plain (all bit-identical); returns the previous value, or -2 (state unchanged) for any other value */
int es_set_attn_bwd_variant(int v);
/* tuning knob: the single-pass attention backward's workgroups (-1, the default: max(CUs, heads / 4);
   0: one persistent workgroup per CU); returns the previous value */
int es_set_attn_bwd_grid(int workgroups);
/* 1 (default): the backward variant above also for T > 256 (the 37-tile kernels); 0: plain loops there. */
int es_set_attn_bwd_long(int v);
/* ---- attention (code/models/conformer.py:40-50), head dim 64, tokens T <= 592 (384^2 / 16) ------ */
int es_attn_fwd(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                hipStream_t stream);
/* delta: fp32 workspace [nimg*H*T] (rowsum(dO*O), produced by the dQ pass for the dK/dV pass; the single-pass
   kernel that 13-tile heads (192 < T <= 208) use by default keeps it on chip and leaves the workspace untouched) */
int es_attn_bwd(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, float* delta, const void* dout,
                int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream);
/* CLS-query attention for a block whose non-CLS outputs are unused (the last block: only the CLS
 * token reaches timm's head, VisionTransformer.forward_features x[:, 0]).  o / dout are compact
 * [nimg, ld] CLS rows, lse [nimg*H]; the backward writes dqkv for every token (q part zero off the
 * CLS rows), as es_attn_bwd would for a dout that is zero off the CLS rows. */
int es_attn_cls_fwd(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                    hipStream_t stream);
int es_attn_cls_bwd(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, const void* dout, int lddo,
                    void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream);

/* ---- LayerNorm(eps) (code/models/conformer.py:58,60,65) -------------------------------------- */
/* tuning knob: 0 = the one-shot forward (a workgroup per 8 rows), > 0 = the grid-stride forward on this many
   workgroups (bit-identical); returns the previous value */
int es_set_ln_fwd_grid(int workgroups);
int es_layernorm_fwd(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, float* mean,
                     float* rstd, int M, int D, float eps, hipStream_t stream);
int es_layernorm_bwd(const float* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                     const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                     float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                     hipStream_t stream);
// es_layernorm_bwd with dy = d(LN output) in bf16 (what the ViT engine's dgrad GEMMs write: the
// GEMM operands downstream are bf16 already; half the bytes of the fp32 form on both sides)
int es_layernorm_bwd_b16(const void* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                         float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                         hipStream_t stream);
// Both backwards with dgamma == dbeta == NULL leave their per-workgroup partials in `workspace`
// (es_layernorm_bwd_grid(blocks, M) rows of D floats for dgamma, then as many for dbeta);
// es_ln_param_grads_multi then reduces up to 32 such workspaces in ONE launch (the ViT engine defers its
// LayerNorms' parameter gradients off the data-gradient chain).  Table entries (host memory, passed by value):
// {const float* workspace; float* dgamma; float* dbeta; int grid; int D; int accumulate; int pad}, all with the
// same (grid >= 64 && D <= 2048) class.  Same sums, bit for bit, as the undeferred backward.
int es_layernorm_bwd_grid(int blocks, int M);
int es_ln_param_grads_entry_size(void);
int es_ln_param_grads_multi(const void* table, int n, hipStream_t stream);

/* ---- standalone GELU (nn.GELU, exact erf) ---------------------------------------------------- */
int es_gelu_fwd(const void* x, void* y, long n, hipStream_t stream);
int es_gelu_bwd(const void* x, const void* dy, void* dx, long n, hipStream_t stream);

/* ---- ViT ends: patches, CLS/pos rows, embedding backward, final LN + head on CLS ------------- */
int es_patch_im2col(const float* img, void* patches, int n, int S, int P, hipStream_t stream);

// es_patch_im2col from uint8 pixels [n, 3, S, S]: ToTensor (x / 255) then Normalize ((x - mean[c]) /
// std[c]) in fp32, IEEE divisions (code/dataset.py:21-22,49-51 -- torchvision's transforms on the
// host), then the same bf16 patch permutation.  img 8-byte aligned.
int es_patch_im2col_u8(const void* img, float mean0, float mean1, float mean2, float std0, float std1, float std2,
                       void* patches, int n, int S, int P, hipStream_t stream);
int es_cls_init(float* x, int ldx, const float* cls, const float* pos, int n, int T, int D, hipStream_t stream);
int es_embed_bwd(const float* dx, int lddx, void* dpatch, int ldp, float* dpos, float* dcls, int n, int T, int D,
                 int accumulate, hipStream_t stream);
int es_cls_head_fwd(const float* x, int ldx, int T, const float* gamma, const float* beta, const float* W,
                    const float* b, float* logits, int ldl, float* xhat, float* rstd, int n, int D, int C, float eps,
                    hipStream_t stream);
int es_cls_head_bwd(const float* dl, int lddl, const float* W, const float* gamma, const float* beta,
                    const float* xhat, const float* rstd, float* dyn, float* dx, int lddx, int T, float* dW, float* db,
                    float* dgamma, float* dbeta, int n, int D, int C, hipStream_t stream);
/* the same with dW / db / dgamma / dbeta written (accumulate = 0) instead of added to (1): the first writer of
 * those gradient entries in a step, so the flat gradient buffer needs no zero fill before the backward */
int es_cls_head_bwd_ex(const float* dl, int lddl, const float* W, const float* gamma, const float* beta,
                       const float* xhat, const float* rstd, float* dyn, float* dx, int lddx, int T, float* dW,
                       float* db, float* dgamma, float* dbeta, int n, int D, int C, int accumulate, hipStream_t stream);

/* CoMatch features: fts [n, D] = LN(x_cls) (ModelwEmb's `fts` over the ViT trunk,
 * code/models/custom_model.py:207-209) and its backward into the CLS rows of dx; dgamma / dbeta
 * accumulated (+=). */
int es_cls_ln_fwd(const float* x, int ldx, int T, const float* gamma, const float* beta, float* fts, int ldf,
                  float* xhat, float* rstd, int n, int D, float eps, hipStream_t stream);
int es_cls_ln_bwd(const float* dfts, int lddf, const float* gamma, const float* xhat, const float* rstd, float* dx,
                  int lddx, int T, float* dgamma, float* dbeta, int n, int D, hipStream_t stream);

/* ---- CoMatch heads (fp32; code/models/custom_model.py:107-145,201-205) ------------------------- */
/* Y = act(X W^T + b) (* keep * keep_scale, the replayed Dropout keep-mask, uint8 [n, N]);
 * act 0 = none, 1 = ReLU, 2 = LeakyReLU(slope) */
int es_dense_fwd(const float* X, int ldx, const float* W, const float* b, float* Y, int ldy, int n, int K, int N,
                 int act, float slope, const void* keep, float keep_scale, hipStream_t stream);
size_t es_dense_bwd_workspace(int n, int N);
/* backward of es_dense_fwd given its output Yact: dW, db overwritten; dX (+)= when dX != NULL */
int es_dense_bwd(const float* dY, int lddy, const float* Yact, int ldya, int act, float slope, const void* keep,
                 float keep_scale, const float* X, int ldx, const float* W, float* dX, int lddx, int accumulate_dx,
                 float* dW, float* db, int n, int K, int N, float* workspace, hipStream_t stream);
/* BatchNorm1d (nn.BatchNorm1d semantics): train = batch statistics + running-buffer update
 * (momentum, unbiased variance, num_batches_tracked int64 += 1), eval = running statistics */
int es_bn1d_fwd(const float* U, int ldu, const float* gamma, const float* beta, float* running_mean, float* running_var,
                void* num_batches_tracked, float momentum, float eps, int train, float* Y, int ldy, float* xhat,
                float* rstd, int n, int F, hipStream_t stream);
int es_bn1d_bwd(const float* dY, int lddy, const float* xhat, const float* rstd, const float* gamma, float* dU,
                int lddu, float* dgamma, float* dbeta, int n, int F, hipStream_t stream);
/* SyncBatchNorm1d pieces for the data-parallel CoMatch head (statistics over the global batch of N
 * rows, the caller all-reducing the per-feature sums between launches; code/models/custom_model.py:
 * 110-116 BatchNorm1d as one process computes it on the concatenated batch):
 *   es_bn1d_sums: out[f] = sum_i U[i][f] (S1 NULL) or sum_i (U[i][f] - S1[f]/N)^2;
 *   es_bn1d_fwd_global: y / xhat / rstd from the global S1, S2, running-buffer update (unbiased var);
 *   es_bn1d_bwd_sums: out[f] = sum dY, out[F+f] = sum dY xhat over this rank's rows;
 *   es_bn1d_bwd_global: dU from the all-reduced sums, dgamma / dbeta = this rank's sums. */
int es_bn1d_sums(const float* U, int ldu, int n, int F, const float* S1, float N, float* out, hipStream_t stream);
int es_bn1d_fwd_global(const float* U, int ldu, const float* gamma, const float* beta, const float* S1,
                       const float* S2, float N, float* running_mean, float* running_var, void* num_batches_tracked,
                       float momentum, float eps, float* Y, int ldy, float* xhat, float* rstd, int n, int F,
                       hipStream_t stream);
int es_bn1d_bwd_sums(const float* dY, int lddy, const float* xhat, int n, int F, float* out, hipStream_t stream);
int es_bn1d_bwd_global(const float* dY, int lddy, const float* xhat, const float* rstd, const float* gamma,
                       const float* sums_global, const float* sums_local, float N, float* dU, int lddu,
                       float* dgamma, float* dbeta, int n, int F, hipStream_t stream);
/* Dropout(p) keep-mask (uint8 0/1), counter-based hash of (seed, offset + i) */
int es_dropout_keep(void* keep, long n, float p, unsigned long long seed, unsigned long long offset,
                    hipStream_t stream);
/* Normalize(2) (code/models/custom_model.py:136-145) */
int es_l2norm_fwd(const float* V, int ldv, float* Z, int ldz, float* norm, int n, int L, hipStream_t stream);
int es_l2norm_bwd(const float* dZ, int lddz, const float* Z, int ldz, const float* norm, float* dV, int lddv, int n,
                  int L, hipStream_t stream);

/* ---- CoMatch step (code/comatch.py:162-220) ---------------------------------------------------- */
size_t es_comatch_pseudo_workspace(int nu, int C, int Q);
/* softmax(weak) -> distribution alignment (batch mean appended at hist[hist_pos] of a hist_cap
 * ring, mean of the hist_len newest) -> memory smoothing against the Q-row bank -> argmax / mask.
 * C <= 32, L <= 64. */
int es_comatch_pseudo(const float* logits_w, int ldl, int nu, int C, float* hist, int hist_cap, int hist_len,
                      int hist_pos, const float* z_w, int ldz, int L, const float* bank_feats, const float* bank_probs,
                      int Q, float temperature, float alpha, float thres, float* probs, float* probs_orig, int* pl,
                      float* mask, float* workspace, hipStream_t stream);
/* as es_comatch_pseudo; hist_given = 1: hist[hist_pos] already holds the step's batch mean (the
 * data-parallel path writes the all-ranks mean there: es_softmax_colmean + all-reduce) */
int es_comatch_pseudo_ex(const float* logits_w, int ldl, int nu, int C, float* hist, int hist_cap, int hist_len,
                         int hist_pos, int hist_given, const float* z_w, int ldz, int L, const float* bank_feats,
                         const float* bank_probs, int Q, float temperature, float alpha, float thres, float* probs,
                         float* probs_orig, int* pl, float* mask, float* workspace, hipStream_t stream);
/* out[c] = mean over rows of softmax(logits)[c], C <= 32 (the DA batch mean) */
int es_softmax_colmean(const float* logits, int ldl, int n, int C, float* out, hipStream_t stream);
/* ring write of [z_w; z_x] and [probs_orig; onehot(y)] at bank row ptr (code/comatch.py:187-196) */
int es_comatch_bank_write(const float* z_w, int ldzw, int nu, const float* z_x, int ldzx, int bt, int L,
                          const float* probs_orig, const void* y_int64, int C, float* bank_feats, float* bank_probs,
                          int ptr, int Q, hipStream_t stream);
size_t es_comatch_contrastive_workspace(int nu);
/* loss_out[0] = L_c = mean_i L_i; dz0 / dz1 = grad_scale * d(sum_i L_i)/dz -- pass lambda_c / nu for the
 * gradient of lambda_c * L_c (code/comatch.py:199-213) */
int es_comatch_contrastive_fwd_bwd(const float* z0, int ldz0, const float* z1, int ldz1, const float* probs, int nu,
                                   int L, int C, float temperature, float contrast_th, float grad_scale,
                                   float* loss_out, float* dz0, int lddz0, float* dz1, int lddz1, float* workspace,
                                   hipStream_t stream);
/* the data-parallel form: nr local anchor rows (global rows row_off..) against the nc global columns
 * (all-gathered z1 / probs); loss_out[0] = local row-loss sum / loss_div; dz1_all [nc, L] is this
 * rank's share of d/dz1 for every column (sum it over ranks, keep the own rows) */
size_t es_comatch_contrastive_ex_workspace(int nr, int nc);
int es_comatch_contrastive_fwd_bwd_ex(const float* z0, int ldz0, const float* z1_all, int ldz1,
                                      const float* probs_rows, const float* probs_all, int nr, int nc, int row_off,
                                      int L, int C, float temperature, float contrast_th, float grad_scale,
                                      float loss_div, float* loss_out, float* dz0, int lddz0, float* dz1_all,
                                      int lddz1, float* workspace, hipStream_t stream);
/* loss_out[0] = L_u = mean_i L_i; dls = grad_scale * d(sum_i L_i)/dlogits -- pass lambda_u / nu
 * (code/comatch.py:215-220); workspace nu floats */
int es_comatch_focal_fwd_bwd(const float* ls, int ldl, const float* probs, const float* mask, int nu, int C,
                             float gamma, float grad_scale, float* loss_out, float* dls, int lddl, float* workspace,
                             hipStream_t stream);

/* ---- FixMatch losses, forward + gradient fused ------------------------------------------------ */
/* code/loss.py:126-164 consistency_loss(name='ce', use_hard_labels=True); out[0]=loss, out[1]=mask mean */
int es_fm_consistency_fwd_bwd(const float* logits_w, int ldw, const float* logits_s, int lds, int n, int C,
                              float tau, float grad_scale, int* pseudo_label, uint8_t* mask, float* row_loss,
                              float* dlogits_s, int lddls, float* out, hipStream_t stream);
/* code/loss.py:103-114,308-364 ce_loss(type_loss='poly') = PolyLoss(epsilon=2); out[0]=loss */
int es_poly_ce_fwd_bwd(const float* logits, int ldl, const int64_t* targets, const float* weights, int n, int C,
                       float epsilon, float grad_scale, float* dlogits, int lddl, float* out, hipStream_t stream);

/* ---- Conformer CNN branch (SemiFormer backbone, code/models/conformer.py:75-445) ---------------
 * fp32 NHWC maps with element strides; Conv2d groups = 1, weights in the reference layout
 * [Cout][Cin][kh][kw].  Replaces the reference's aten conv2d / batch_norm / max_pool2d /
 * avg_pool2d / upsample_nearest2d calls in ConvBlock, FCUDown, FCUUp and the stem. */
/* 1 (default): the 3 -> 64 channel 7x7 / stride-2 / pad-3 stem (Conformer.conv1, resnet18.conv1) on NHWC fp32
 * images runs on its own forward (bit-identical to the generic kernel) and weight-gradient kernels inside
 * es_conv2d_fwd / es_conv2d_bwd_weight; 0: the generic kernels.  Returns the previous value. */
int es_set_stem_kernels(int v);
int es_conv2d_fwd(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                  const float* w, const float* bias, int Cout, int kh, int kw, int stride, int pad, float* y, long syn,
                  long syh, long syw, int accumulate, hipStream_t stream);
int es_conv2d_bwd_data(const float* dy, long syn, long syh, long syw, const float* w, int N, int H, int W, int Cin,
                       int Cout, int kh, int kw, int stride, int pad, float* dx, long sxn, long sxh, long sxw, long sxc,
                       int accumulate, hipStream_t stream);
// workgroup tiles (Cout x Cin kh kw) one pixel split of es_conv2d_bwd_weight launches: callers size
// `splits` so that tiles x splits fills the chip
int es_conv2d_dw_tiles(int Cout, int Cin, int kh, int kw);
size_t es_conv2d_bwd_weight_workspace(int Cout, int Cin, int kh, int kw, int splits);
int es_conv2d_bwd_weight(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                         const float* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride, int pad,
                         int splits, float* workspace, float* dw, int accumulate, hipStream_t stream);
/* bf16-operand forms of the three convs above (csrc/conv_bf16.hip): the same fp32 maps and
 * geometry arguments, operands rounded to bf16 as they are staged, fp32 accumulation on
 * v_mfma_f32_16x16x32_bf16.  Taken for eligible convs (Cin, Cout multiples of 32) when
 * the maps have channel stride 1 with 16-byte aligned pixel rows.  Weights go through
 * es_conv2d_pack_bf16 first: wp [Cout][kh kw][Cin] (forward), wt [Cin][kh kw][Cout] (data grad),
 * Cout Cin kh kw bf16 each, either pointer may be null. */
int es_conv2d_bf16_eligible(int Cin, int Cout, int kh, int kw);
/* tuning knob: the workgroup count the bf16 weight gradient's automatic pixel split aims at (default 512;
   each split writes an fp32 slab of the gradient that a reduce kernel sums); returns the previous value */
int es_set_conv_dw_target(int v);
/* tuning knob: the bf16-map data-gradient convs and the forwards that do not widen the channels on the LDS-DMA
 * ring kernel with 3 or 4 stages (default 3), or 0 = the register-staged gather (bit-identical); returns the
 * previous value, or -2 (unchanged) otherwise */
int es_set_conv_ring(int stages);
/* tuning knob: 1 (default) = the register-staged bf16 conv kernels (weight gradient; forward / data gradient off the
 * ring) with branch-free (range-checked buffer) loads and pixel walk where they apply, 0 = the branchy loads
 * (bit-identical); returns the previous value, or -2 otherwise */
int es_set_conv_dw_buf(int v);
/* tuning knob: a bf16 conv forward / data gradient whose 128-channel tiling would launch fewer than `wgs`
 * workgroups (default 128; 0 = never) runs on the 64-channel tile: twice the workgroups on small maps, the same
 * per-element reduction order (bit-identical); returns the previous value, or -2 (unchanged) for wgs < 0 */
int es_set_conv_small(int wgs);
int es_conv2d_pack_bf16(const float* w, int Cout, int Cin, int kh, int kw, void* wp, void* wt, hipStream_t stream);
/* es_conv2d_pack_bf16 for n weights in ONE launch (a model's conv weights after each optimizer step):
 * table = n device-resident entries of es_conv_pack_entry_size() bytes
 * {const float* w; void* wp; void* wt; int Cout; int Cin; int kh_x_kw; int pad}, max_elems = the largest
 * Cout * Cin * kh * kw (sizes the grid).  Same images, bit for bit. */
int es_conv_pack_entry_size(void);
int es_conv2d_pack_bf16_multi(const void* table, int n, long max_elems, hipStream_t stream);
int es_conv2d_fwd_bf16(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                       const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad, float* y,
                       long syn, long syh, long syw, int accumulate, hipStream_t stream);
int es_conv2d_bwd_data_bf16(const float* dy, long syn, long syh, long syw, const void* wt, int N, int H, int W,
                            int Cin, int Cout, int kh, int kw, int stride, int pad, float* dx, long sxn, long sxh,
                            long sxw, long sxc, int accumulate, hipStream_t stream);
/* es_conv2d_fwd_bf16 (overwrite) that also writes y's BatchNorm statistics per 128-pixel block:
 * partials[b][0][c] = block sum, partials[b][1][c] = block-centred sum of squares
 * (es_conv2d_bnstats_size floats) -- es_bn2d_fwd_partials needs no statistics pass over y. */
size_t es_conv2d_bnstats_size(int M, int Cout);
int es_conv2d_fwd_bf16_bnstats(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                               const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                               float* y, long syn, long syh, long syw, float* partials, hipStream_t stream);
/* workspace floats for M = N Ho Wo output pixels; splits <= 0 sizes the pixel split automatically */
size_t es_conv2d_bwd_weight_bf16_workspace(int M, int Cout, int Cin, int kh, int kw, int splits);
int es_conv2d_bwd_weight_bf16(const float* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                              const float* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride,
                              int pad, int splits, float* workspace, float* dw, int accumulate, hipStream_t stream);
size_t es_chan_workspace(int rows, int C);
/* out[c] (+)= sum_r v[(r / HW) * sn + (r % HW) * sp + c]  (bias gradients) */
int es_chan_sum(const float* v, int rows, int C, long sn, long sp, int HW, float* workspace, float* out,
                int accumulate, hipStream_t stream);
/* BatchNorm2d (train: batch stats, running update, num_batches_tracked += 1; eval: running stats),
 * y = bn(x) (+ res) then ReLU if relu.  workspace: es_chan_workspace(rows, C) floats. */
int es_bn2d_fwd(const float* x, int rows, int C, const float* gamma, const float* beta, float* running_mean,
                float* running_var, void* num_batches_tracked, float momentum, float eps, int train, const float* res,
                int relu, float* y, float* mean, float* rstd, float* workspace, hipStream_t stream);
int es_bn2d_bwd(const float* x, const float* y, const float* dy, int rows, int C, int relu, const float* gamma,
                const float* mean, const float* rstd, int train, const float* running_var, float eps, float* dx,
                float* gout, float* dgamma, float* dbeta, int accumulate, float* workspace, hipStream_t stream);
/* Train-mode BatchNorm2d with the batch statistics from es_conv2d_fwd_bf16_bnstats' partials of x
 * (128-row blocks, combined as Chan et al. in two levels of 64 blocks; the first level overwrites
 * partials in place): running stats, num_batches_tracked, mean / rstd and y = bn(x) (+ res) (relu)
 * as es_bn2d_fwd. */
int es_bn2d_fwd_partials(const float* x, int rows, int C, float* partials, const float* gamma,
                         const float* beta, float* running_mean, float* running_var, void* num_batches_tracked,
                         float momentum, float eps, const float* res, int relu, float* y, float* mean, float* rstd,
                         hipStream_t stream);
/* SyncBatchNorm2d: the Conformer's BatchNorm2d over the global batch at N > 1 (SURVEY.md §8(e):
 * exact parity with the single-process step needs the statistics of every rank's rows).  Flow per
 *  BatchNorm: es_bn2d_sums [mode 0] -> all-reduce -> es_bn2d_sums [mode 1: centred on the global mean]
 * -> all-reduce -> es_bn2d_fwd_global; backward: es_bn2d_bwd_sums -> all-reduce of a copy ->
 * es_bn2d_bwd_global [dx from the global sums, dgamma / dbeta from the local ones].  rows_g = the
 * rows of every rank together; workspace = es_chan_workspace(rows, C) floats. */
int es_bn2d_sums(const float* x, int rows, int C, int mode, const float* sum_g, int rows_g, float* out,
                 float* workspace, hipStream_t stream);
int es_bn2d_fwd_global(const float* x, int rows, int C, const float* gamma, const float* beta, float* running_mean,
                       float* running_var, void* num_batches_tracked, float momentum, float eps, const float* sum_g,
                       const float* sq_g, int rows_g, const float* res, int relu, float* y, float* mean, float* rstd,
                       hipStream_t stream);
int es_bn2d_bwd_sums(const float* x, const float* y, const float* dy, int rows, int C, int relu, const float* mean,
                     const float* rstd, float* out, float* workspace, hipStream_t stream);
int es_bn2d_bwd_global(const float* x, const float* y, const float* dy, int rows, int C, int relu, const float* gamma,
                       const float* mean, const float* rstd, const float* sums_local, const float* sums_g, int rows_g,
                       float* dx, float* gout, float* dgamma, float* dbeta, int accumulate, hipStream_t stream);
int es_maxpool2d_fwd(const float* x, int N, int H, int W, int C, int k, int s, int p, float* y, void* arg,
                     hipStream_t stream);
int es_maxpool2d_bwd(const float* dy, const void* arg, int N, int H, int W, int C, int k, int s, int p, float* dx,
                     hipStream_t stream);
int es_avgpool2d_fwd(const float* x, int N, int H, int W, int C, int k, float* y, hipStream_t stream);
int es_avgpool2d_bwd(const float* dy, int N, int H, int W, int C, int k, float* dx, int accumulate,
                     hipStream_t stream);
int es_upsample_add_fwd(const float* base, const float* src, int N, int H, int W, int C, int s, float* out,
                        hipStream_t stream);
int es_upsample_bwd(const float* dout, int N, int H, int W, int C, int s, float* dsrc, hipStream_t stream);

/* ---- bf16 activation / gradient maps (the Conformer CNN branch when every conv of the branch takes the
 * bf16 kernels: conformer.NativeConformer.map_bf16).  Same arguments as the fp32 entry points above plus
 * `flags`: conv fwd / data grad, pools: bit 0 = the input map is bf16, bit 1 = the output map is bf16;
 * conv weight grad: bit 0 = x bf16, bit 1 = dy bf16; BatchNorm / chan_sum / upsampling: bit 0 = every map
 * argument bf16.  Arithmetic in fp32, each output rounded once (an accumulating store adds in fp32).
 * These replace the same reference ops as their fp32 forms (code/models/conformer.py:75-200 ConvBlock /
 * FCUDown / FCUUp, torch autocast's bf16 conv outputs). */
int es_conv2d_fwd_bf16_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                          const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad, void* y,
                          long syn, long syh, long syw, int accumulate, float* bn_partials, int flags,
                          hipStream_t stream);
int es_conv2d_bwd_data_bf16_ex(const void* dy, long syn, long syh, long syw, const void* wt, int N, int H, int W,
                               int Cin, int Cout, int kh, int kw, int stride, int pad, void* dx, long sxn, long sxh,
                               long sxw, long sxc, int accumulate, int flags, hipStream_t stream);
int es_conv2d_bwd_weight_bf16_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                                 const void* dy, long syn, long syh, long syw, int Cout, int kh, int kw, int stride,
                                 int pad, int splits, float* workspace, float* dw, int accumulate, int flags,
                                 hipStream_t stream);
/* The same forward / weight-gradient convs when x is the INPUT of a train-mode BatchNorm2d + ReLU whose output
 * feeds this conv alone (ConvBlock bn1 -> conv2, bn2 -> conv3, code/models/conformer.py:118-134): the gathers
 * apply relu((x - mean) rstd gamma + beta), rounded to x's map type exactly as es_bn2d_fwd*_ex stores it,
 * so the normalised map is never written (es_bn2d_fwd_partials_ex with y = NULL gives mean / rstd; the
 * backward is es_bn2d_bwd_recompute_ex).  Per-channel arrays 16-byte aligned. */
int es_conv2d_fwd_bf16_bnin_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw, long sxc,
                               const void* wp, const float* bias, int Cout, int kh, int kw, int stride, int pad,
                               void* y, long syn, long syh, long syw, int accumulate, float* bn_partials, int flags,
                               const float* in_mean, const float* in_rstd, const float* in_gamma,
                               const float* in_beta, hipStream_t stream);
int es_conv2d_bwd_weight_bf16_bnin_ex(const void* x, int N, int H, int W, int Cin, long sxn, long sxh, long sxw,
                                      long sxc, const void* dy, long syn, long syh, long syw, int Cout, int kh, int kw,
                                      int stride, int pad, int splits, float* workspace, float* dw, int accumulate,
                                      int flags, const float* in_mean, const float* in_rstd, const float* in_gamma,
                                      const float* in_beta, hipStream_t stream);
int es_chan_sum_ex(const void* v, int rows, int C, long sn, long sp, int HW, float* workspace, float* out,
                   int accumulate, int flags, hipStream_t stream);
/* tuning knob: 1 (default) = the channel-stationary BatchNorm apply kernels (forward apply and the backward's dx
 * pass), 0 = the per-iteration forms (bit-identical); returns the previous value, or -2 (unchanged) otherwise */
int es_set_bn_cs(int v);
/* test knob: 1 = the BatchNorm channel sums over 8-channel groups (a different fp32 summation order of the same
 * sums), 0 (default) = 4-channel groups; returns the previous value, or -2 (unchanged) otherwise */
int es_set_bn_sum8(int v);
int es_bn2d_fwd_ex(const void* x, int rows, int C, const float* gamma, const float* beta, float* running_mean,
                   float* running_var, void* num_batches_tracked, float momentum, float eps, int train, const void* res,
                   int relu, void* y, float* mean, float* rstd, float* workspace, int flags, hipStream_t stream);
int es_bn2d_bwd_ex(const void* x, const void* y, const void* dy, int rows, int C, int relu, const float* gamma,
                   const float* mean, const float* rstd, int train, const float* running_var, float eps, void* dx,
                   void* gout, float* dgamma, float* dbeta, int accumulate, float* workspace, int flags,
                   hipStream_t stream);
/* es_bn2d_bwd_ex for a train-mode ReLU BatchNorm without residual whose output y was not kept: the ReLU mask
   is rebuilt from x with the forward's affine map and rounding, so the backward reads x and dy only */
int es_bn2d_bwd_recompute_ex(const void* x, const void* dy, int rows, int C, const float* gamma, const float* beta,
                             const float* mean, const float* rstd, void* dx, float* dgamma, float* dbeta, int accumulate,
                             float* workspace, int flags, hipStream_t stream);
/* es_bn2d_fwd_partials(_ex) with y = NULL (and no residual): statistics, running buffers, mean / rstd only */
int es_bn2d_fwd_partials_ex(const void* x, int rows, int C, float* partials, const float* gamma, const float* beta,
                            float* running_mean, float* running_var, void* num_batches_tracked, float momentum,
                            float eps, const void* res, int relu, void* y, float* mean, float* rstd, int flags,
                            hipStream_t stream);
int es_bn2d_sums_ex(const void* x, int rows, int C, int mode, const float* sum_g, int rows_g, float* out,
                    float* workspace, int flags, hipStream_t stream);
int es_bn2d_fwd_global_ex(const void* x, int rows, int C, const float* gamma, const float* beta, float* running_mean,
                          float* running_var, void* num_batches_tracked, float momentum, float eps, const float* sum_g,
                          const float* sq_g, int rows_g, const void* res, int relu, void* y, float* mean, float* rstd,
                          int flags, hipStream_t stream);
int es_bn2d_bwd_sums_ex(const void* x, const void* y, const void* dy, int rows, int C, int relu, const float* mean,
                        const float* rstd, float* out, float* workspace, int flags, hipStream_t stream);
int es_bn2d_bwd_global_ex(const void* x, const void* y, const void* dy, int rows, int C, int relu, const float* gamma,
                          const float* mean, const float* rstd, const float* sums_local, const float* sums_g, int rows_g,
                          void* dx, void* gout, float* dgamma, float* dbeta, int accumulate, int flags,
                          hipStream_t stream);
int es_maxpool2d_fwd_ex(const float* x, int N, int H, int W, int C, int k, int s, int p, void* y, void* arg, int flags,
                        hipStream_t stream);
int es_maxpool2d_bwd_ex(const void* dy, const void* arg, int N, int H, int W, int C, int k, int s, int p, float* dx,
                        int flags, hipStream_t stream);
int es_avgpool2d_fwd_ex(const void* x, int N, int H, int W, int C, int k, void* y, int flags, hipStream_t stream);
int es_avgpool2d_bwd_ex(const void* dy, int N, int H, int W, int C, int k, void* dx, int accumulate, int flags,
                        hipStream_t stream);
int es_upsample_add_fwd_ex(const void* base, const void* src, int N, int H, int W, int C, int s, void* out, int flags,
                           hipStream_t stream);
int es_upsample_bwd_ex(const void* dout, int N, int H, int W, int C, int s, void* dsrc, int flags, hipStream_t stream);
/* FCUDown LayerNorm + GELU + cat(cls) fused with ConvTransBlock's x_st + x_t */
int es_fcu_down_tokens_fwd(const float* pooled, const float* xt, const float* ln_w, const float* ln_b, float* out,
                           float* mean, float* rstd, int N, int np, int D, float eps, hipStream_t stream);
size_t es_fcu_down_workspace(int N, int np, int D);
int es_fcu_down_tokens_bwd(const float* dout, const float* pooled, const float* ln_w, const float* ln_b,
                           const float* mean, const float* rstd, float* dxt, float* dpooled, float* dln_w,
                           float* dln_b, int accumulate, int N, int np, int D, float* workspace, hipStream_t stream);
/* es_fcu_down_tokens_bwd with dxt (+)= when dxt_accumulate (the second consumer of a gradient sink) */
int es_fcu_down_tokens_bwd_ex(const float* dout, const float* pooled, const float* ln_w, const float* ln_b,
                              const float* mean, const float* rstd, float* dxt, float* dpooled, float* dln_w,
                              float* dln_b, int accumulate, int N, int np, int D, float* workspace, int dxt_accumulate,
                              hipStream_t stream);
int es_tokens_cls_set(float* xt, int N, int T, int D, const float* cls, hipStream_t stream);
/* F.cross_entropy(weight=w, reduction='mean') (code/loss.py:118): out[0] = sum w_y l / sum w_y;
 * dlogits = grad_scale * d(out[0]) / d logits */
int es_ce_weighted_fwd_bwd(const float* logits, int ldl, const int64_t* targets, const float* weights, int n, int C,
                           float grad_scale, float* dlogits, int lddl, float* out, hipStream_t stream);
/* out[0] = sum_i w[y_i] over this rank's rows (weights nullable -> n) */
int es_ce_weight_sum(const int64_t* targets, const float* weights, int n, int C, float* out, hipStream_t stream);
/* the data-parallel weighted mean (code/loss.py:118 over the GLOBAL batch): *wsum_global = the weight sum over every
 * rank's rows; out[0] = sum_{own rows} w_y l / W_global; dlogits = grad_scale * d(out[0]) / d logits */
int es_ce_weighted_fwd_bwd_global(const float* logits, int ldl, const int64_t* targets, const float* weights,
                                  const float* wsum_global, int n, int C, float grad_scale, float* dlogits, int lddl,
                                  float* out, hipStream_t stream);

/* ---- optimizer / EMA (code/optimizer.py:50-51, code/ema.py:51-62) ----------------------------- */
int es_adam_ema_step(float* p, const float* g, float* m, float* v, float* ema, long n, float beta1, float beta2,
                     float eps, float neg_step, float bc2_sqrt, float decay, float one_minus_decay,
                     float grad_scale, hipStream_t stream);
int es_ema_entry_size(void);
int es_ema_update_multi(const void* entries, const void* chunks, int nchunks, float decay, float one_minus_decay,
                        hipStream_t stream);
int es_pack_entry_size(void);
int es_pack_weights(const float* flat, const void* entries, int nmat, hipStream_t stream);
int es_cast_f32_bf16(const float* x, void* y, long n, hipStream_t stream);

// y += x over n fp32 values (n % 4 == 0, 16-byte aligned).  Sums the second lane's flat gradient into the
// first (two-lane backward, endossl/vit.py Engine.backward); no reference counterpart (autograd accumulates).
int es_add_f32(float* y, const float* x, long n, hipStream_t stream);

/* ---- fp32 parity mode (csrc/parity.hip) --------------------------------------------------------
 * The same arguments as the bf16 entry points above, with fp32 storage wherever those read or write
 * bf16 (GEMM operands and epilogue outputs, qkv / attention output, LN output, patches, the packed
 * weight images).  endossl/vit.py's Engine(precision="fp32") runs its one forward / backward sequence
 * over these, so the 12-layer step is pinned to the fp32 oracle at 1e-3.  Same reference ops as the
 * bf16 forms (code/models/conformer.py:13-72, timm PatchEmbed); GEMMs on fp32 MFMA, no shape
 * restrictions beyond head dim 64 and T <= 1024 for attention, D % 64 == 0 for LayerNorm. */
int es_gemm_nt_f32(int epi, const void* A, int lda, const void* B, int ldb, const float* bias, void* C, int ldc,
                   void* C2, const void* aux, int ldaux, int M, int N, int K, int np, hipStream_t stream);
size_t es_gemm_tn_f32_workspace(int N1, int N2, int splits);
int es_gemm_tn_f32(const void* A1, int ld1, const void* A2, int ld2, int M, int N1, int N2, int splits,
                   float* workspace, float* out, int accumulate, float* bias_out, hipStream_t stream);
int es_attn_fwd_f32(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                    hipStream_t stream);
int es_attn_bwd_f32(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, float* delta,
                    const void* dout, int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale,
                    hipStream_t stream);
int es_attn_cls_fwd_f32(const void* qkv, int ldqkv, void* o, int ldo, float* lse, int nimg, int T, int H, float scale,
                        hipStream_t stream);
int es_attn_cls_bwd_f32(const void* qkv, int ldqkv, const void* o, int ldo, const float* lse, const void* dout,
                        int lddo, void* dqkv, int lddqkv, int nimg, int T, int H, float scale, hipStream_t stream);
int es_layernorm_fwd_f32(const float* x, int ldx, const float* gamma, const float* beta, void* y, int ldy, float* mean,
                         float* rstd, int M, int D, float eps, hipStream_t stream);
int es_layernorm_bwd_f32(const float* dy, int lddy, const float* x, int ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, int ldres, float* dx, int lddx, void* dxb, int lddxb,
                         float* dgamma, float* dbeta, float* workspace, int blocks, int M, int D, int accumulate,
                         hipStream_t stream);
int es_patch_im2col_f32(const float* img, void* patches, int n, int S, int P, hipStream_t stream);
int es_patch_im2col_u8_f32(const void* img, float mean0, float mean1, float mean2, float std0, float std1, float std2,
                           void* patches, int n, int S, int P, hipStream_t stream);
int es_embed_bwd_f32(const float* dx, int lddx, void* dpatch, int ldp, float* dpos, float* dcls, int n, int T, int D,
                     int accumulate, hipStream_t stream);
int es_pack_weights_f32(const float* flat, const void* entries, int nmat, hipStream_t stream);
/* y = x, n fp32 values (the parity form of es_cast_f32_bf16) */
int es_copy_f32(const float* x, void* y, long n, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* ENDOSSL_H */

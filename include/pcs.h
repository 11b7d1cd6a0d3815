/*
 * pcs.h — C ABI of the MI355X (gfx950) HIP library behind pcs_amd.PointNetSegmentation.
 *
 * The reference (seokjuchung/point-cloud-cnn-segmentation, point_cloud_segmentation.py,
 * cited P:<line>) has no native code: its hot path is PyTorch ATen ops called from
 * PointNetSegmentation.forward (P:98-133), CrossEntropyLoss (P:216,251), autograd
 * (P:254) and Adam (P:217,255).  Each entry point below replaces a group of those ATen
 * calls; the comment on each cites the reference lines whose semantics it implements.
 *
 * Contract (all entry points):
 *  - plain device pointers and sizes; no torch types.  The CALLER owns every buffer
 *    (torch caching allocator); the library never allocates, frees or retains pointers.
 *  - all work is enqueued on the given stream; no device synchronisation inside; no
 *    global mutable state (safe from several host threads / processes).
 *  - return 0 on success, a negative code on error (-hipError_t, or PCS_EINVAL);
 *    pcs_last_error() returns a thread-local message.  No exceptions cross the ABI.
 *  - activations are points-major [M, C] row-major (M = B*N rows, one per point,
 *    scene-major), stored as fp32 (PCS_F32: parity path, exact-f32 MFMA) or bf16
 *    (PCS_BF16: bench path, bf16 MFMA with fp32 accumulation and fp32 BN statistics).
 *    Weights arrive as fp32 in the state-dict layout (Cout, Cin, 1) == [Cout, Cin].
 */
#ifndef PCS_H
#define PCS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t *pcs_stream_t; /* == hipStream_t */

enum { PCS_F32 = 0, PCS_BF16 = 1, PCS_FP8 = 2 /* OCP e4m3fn, 1 byte (wide-layer operands only) */ };
enum { PCS_OK = 0, PCS_EINVAL = -1000 };
/* pcs_gemm_args.flags */
enum {
  PCS_FLAG_GENERIC = 1, /* force the generic 128x{64,128} kernel (cross-checks)            */
  PCS_FLAG_NO_GLDS = 2, /* never pick the LDS-DMA 256x256 kernel (A/B timing, cross-checks) */
  PCS_FLAG_AW_FP8 = 4,  /* A (and Yp) and W are fp8 e4m3 (dtype still names C, stats in fp32):
                           W rows carry E8M0 scales in w_scale, A is unscaled; the LDS-DMA
                           kernel runs v_mfma_scale_f32_16x16x128_f8f6f4 (K % 256 == 0; RAW
                           prologue; FWD statistics / pool or DGRAD)                         */
  PCS_FLAG_C_FP8 = 8,   /* EPI_BNRELU of the bf16 256-wide kernel stores C as fp8 e4m3      */
  PCS_FLAG_POOL_SIGNED_W = 16, /* FWD max-pool on the LDS-DMA kernel: the caller has multiplied
                           W's rows (pcs_sign_rows) and bias by sign(es), so the pool keeps the
                           plain column max of acc (no multiply); es still names the sign.
                           Needs pool and es, no statistics (they would be of the signed y)  */
  /* 64: unused since ABI 2 (was the 8-wave seg_conv2/3 backward, an A/B-only kernel)        */
};

/* prologue applied to an operand element A[m,k] as it is staged into LDS */
enum {
  PCS_PRO_RAW = 0,      /* a = A                                                        */
  PCS_PRO_BNRELU = 1,   /* a = max(A*s[k] + t[k], 0) [* keep(m,k) * keep_scale]  P:106-127 */
  PCS_PRO_BWD = 2,      /* a = alpha[k]*dZ[m,k] + beta[k] + gamma[k]*Y[m,k]   BN backward */
  PCS_PRO_BWD_POOL = 3, /* a = beta[k] + gamma[k]*Y[m,k] + (m==am[b,k] ? sp[b,k] : 0)
                           BN backward of bn_global fed by the max-pool (P:113-114)      */
  PCS_PRO_CAT = 4       /* a = [A | relu(A2*s + t)] concatenated along k: columns k < K1 raw
                           from A [M, K1], columns K1.. from A2 [M, K-K1] through BN+ReLU
                           (s = pa, t = pb over A2's channels); W [Ncols, K1] for the first
                           part, W2 [Ncols, K-K1] for the second (generic kernel only).
                           conv5's folded input gradient dz5 Ws + a4 H4 in one pass        */
};

/* epilogue of the points-major GEMM */
enum {
  PCS_EPI_FWD = 0,   /* y = acc + bias; store y (C may be NULL: statistics only); per-chunk
                        BN statistics (mean, M2); optional per-chunk max/min + arg for the
                        global max-pool                                                    */
  PCS_EPI_DGRAD = 1, /* v = acc (+bias) (+addend) (+sparse rows) (*keep*keep_scale);
                        dz = (Yp*s+t > 0) ? v : 0 (es/et NULL: Yp > 0); store dz; per-chunk
                        S1 = sum dz, S2 = sum dz*(Yp-mean)*rstd (0 when erstd is NULL)      */
  PCS_EPI_RAW = 2,   /* store acc                                                          */
  PCS_EPI_BNRELU = 3 /* y = acc + bias; store relu(y*es + et): the BN+ReLU of this layer
                        applied on the way out, from a finished statistics pass (P:106-110);
                        with stats (bf16 256-wide kernel only): per-chunk column sums of the
                        stored output as (sum, 0) pairs                                     */
};

/*
 * Points-major GEMM  C[m, n] = sum_k pro(A)[m, k] * W[n, k]  (+ epilogue).
 * Used for every 1x1 Conv1d forward (P:106-128) and every input-gradient (dgrad) of the
 * backward (P:254).  Rows are processed in scene-aligned chunks (a chunk never straddles
 * two clouds), so BN statistics, per-scene sums and the max-pool come out per scene.
 */
typedef struct {
  int64_t num_scenes;   /* B */
  int64_t scene_rows;   /* N: padded points per scene; M = B*N */
  int32_t K;            /* reduction length (input channels) */
  int32_t Ncols;        /* output channels */
  int32_t dtype;        /* PCS_F32 | PCS_BF16 */
  int32_t prologue;     /* PCS_PRO_* */
  int32_t epilogue;     /* PCS_EPI_* */
  int32_t chunks_per_scene; /* 0 = auto; pcs_gemm_geometry() reports the value used */
  const void *A;        /* [M,K] dtype: Y_{l-1} (fwd) | dZ_l (PRO_BWD) | Y_l (PRO_BWD_POOL) */
  const void *A2;       /* [M,K] dtype: Y_l (PRO_BWD) */
  const float *pa;      /* [K] s (BNRELU) | alpha (BWD) */
  const float *pb;      /* [K] t (BNRELU) | beta (BWD, BWD_POOL) */
  const float *pc;      /* [K] gamma (BWD, BWD_POOL) */
  const uint8_t *a_mask;/* [M, K/8] dropout keep bits (BNRELU) or NULL */
  float a_keep_scale;   /* 1/(1-p) */
  const int32_t *pool_idx; /* [B,K] argmax row (global index) (BWD_POOL) */
  const float *pool_coef;  /* [B,K] alpha*dz at the argmax row (BWD_POOL) */
  const void *W;        /* [Ncols, K] dtype */
  void *C;              /* [M, Ncols] dtype output */
  const float *bias;    /* [Ncols] (FWD) or NULL */
  const float *scene_bias; /* [B, Ncols] per-scene bias (FWD; seg_conv1 global half) */
  const void *addend;   /* [M, Ncols] dtype added before the mask (DGRAD) or NULL */
  const uint8_t *c_mask;/* [M, Ncols/8] keep bits of the dropout after BN_{l-1} (DGRAD) */
  float c_keep_scale;
  const void *Yp;       /* [M, Ncols] dtype: Y_{l-1} (DGRAD) */
  const float *es, *et; /* [Ncols] BN_{l-1} scale/shift (DGRAD ReLU mask); BNRELU: this layer's;
                           FWD with pool: optional, only sign(es) is used (the pool may then keep
                           just the max (es >= 0) or the min (es < 0) that pcs_pool_finalize reads) */
  const float *emean, *erstd; /* [Ncols] BN_{l-1} batch mean / rstd (DGRAD S2) */
  float *stats;         /* [B*chunks_per_scene, Ncols, 2] partials (FWD, DGRAD) or NULL */
  float *pool;          /* [B*chunks_per_scene, Ncols, 4] (maxv, argmax, minv, argmin) or NULL */
  int32_t flags;        /* PCS_FLAG_* */
  /* EPI_DGRAD with PRO_RAW: sparse rows of a folded max-pool gradient (global_feat, P:114):
   *   v[m, n] += sum_{c < pool_c : pool_idx[b, c] == m} pool_coef[b, c] * pool_w[c*pool_ldw + n]
   * with pool_idx / pool_coef [B, pool_c] (global row index, coefficient); NULL = none. */
  const float *pool_w;
  int64_t pool_ldw;
  int32_t pool_c;
  const uint8_t *w_scale; /* [Ncols] E8M0 scale of each W row (PCS_FLAG_AW_FP8) */
  const void *W2;       /* [Ncols, K - K1] dtype: the second W block (PCS_PRO_CAT) */
  int32_t K1;           /* PCS_PRO_CAT: width of A (a multiple of the 32/16-element k-step) */
  /* bf16 EPI_FWD / PRO_BNRELU with K = Ncols = 64 and no dropout bits (conv3 on the streaming
   * kernel): per chunk [K*K + K] fp32 = x^T x and the column sums of the prologue's output
   * x = relu(A*s + t) as rounded to bf16 -- conv3's input a2, whose Gram gives bn_seg1's
   * statistics (pcs_bn_stats_gram_sbias).  [B*chunks_per_scene][K*K + K]; NULL = none. */
  float *gram;
} pcs_gemm_args;

/* Fills chunks_per_scene (if 0) and returns rows per chunk (>0) or a negative error.  The
 * kernel (and so the row tile: 256 for the bf16 wide-layer kernel, 128 otherwise) is chosen
 * from dtype, K, Ncols and flags, so call it with the same values as pcs_gemm. */
int64_t pcs_gemm_geometry(pcs_gemm_args *args);
/* Launch the GEMM. */
int pcs_gemm(const pcs_gemm_args *args, pcs_stream_t stream);
/* conv1 (Cin = K = input_dim, 1..8; the reference's points carry 4, P:70, P:106) forward:
 * A = points f32 [M,K] (RAW), W f32 [64,K]; epilogue PCS_EPI_FWD semantics (C in dtype,
 * stats).  Same geometry rules. */
int pcs_conv1_fwd(const pcs_gemm_args *args, pcs_stream_t stream);

/*
 * Weight gradient  dW[n, k] = sum_m dy[m, n] * x[m, k]   (autograd of P:106-128, P:254)
 * dy = pro_dy(dZ, Y) (PCS_PRO_BWD or PCS_PRO_BWD_POOL), x = pro_x(X) (PCS_PRO_BNRELU or
 * PCS_PRO_RAW).  The reduction over M is split into scene-aligned slices whose fp32
 * partials are summed in a fixed order (deterministic).
 */
typedef struct {
  int64_t num_scenes, scene_rows;
  int32_t Cout, Cin;    /* dW is [Cout, Cin] */
  int32_t dtype;
  int32_t splits_per_scene; /* 0 = auto */
  int32_t dy_mode;      /* PCS_PRO_BWD | PCS_PRO_BWD_POOL */
  const void *dZ;       /* [M, Cout] */
  const void *Y;        /* [M, Cout] */
  const float *alpha, *beta, *gamma; /* [Cout] */
  const int32_t *pool_idx; const float *pool_coef; /* [B, Cout] (BWD_POOL) */
  int32_t x_mode;       /* PCS_PRO_BNRELU | PCS_PRO_RAW */
  const void *X;        /* [M, Cin] dtype (f32 for conv1) */
  const float *s, *t;   /* [Cin] */
  const uint8_t *x_mask; float x_keep_scale;
  float *partial;       /* workspace: pcs_wgrad_workspace() bytes */
  float *dW;            /* [Cout, Cin] f32 output, row stride ldw */
  int64_t ldw;          /* 0 = Cin */
  int32_t flags;        /* PCS_FLAG_GENERIC: never use the 256x256 wide-layer kernel */
  float *dy_colsum;     /* [Cout] f32 or NULL: sum_m dy[m, n] (RAW dy, conv5's R pass only:
                           bn5's S1 = the column sums of dz5 as stored, one ones-fragment MFMA
                           per dz5 fragment beside R's; the workspace grows by one Cout row per
                           slice).  Other kernels refuse it. */
} pcs_wgrad_args;

int64_t pcs_wgrad_workspace(pcs_wgrad_args *args); /* bytes; fills splits_per_scene */
int pcs_wgrad(const pcs_wgrad_args *args, pcs_stream_t stream);
int pcs_conv1_wgrad(const pcs_wgrad_args *args, pcs_stream_t stream); /* X = points f32 [M, Cin], Cin 1..8;
                                                                          partial: B*splits*64*Cin f32 */

/*
 * Fused input + weight gradient of seg_conv1's local half (bf16; Cout 512, Cin 64):
 * dy = alpha*dZ + beta + gamma*Y (dy_mode PCS_PRO_BWD), x = relu(X*s + t) (x_mode
 * PCS_PRO_BNRELU, no x_mask);  dX[M, 64] = dy . Wt^T (Wt = W^T, [64, 512] bf16, no epilogue)
 * and dW += dy^T x as pcs_wgrad (fp32 partials summed in a fixed order into dW, row stride
 * ldw).  Replaces the pcs_gemm(PRO_BWD, EPI_RAW) + pcs_wgrad pair, reading dy's inputs once.
 */
int64_t pcs_dgrad_wgrad_workspace(pcs_wgrad_args *args); /* bytes; fills splits_per_scene */
int pcs_dgrad_wgrad(const pcs_wgrad_args *args, const void *Wt, void *dX, pcs_stream_t stream);

/*
 * The same two gradients in folded form, without reading bn_seg1's stored output Y'
 * (dy_mode PCS_PRO_RAW: dZ is bn_seg1's output gradient dz; x_mode PCS_PRO_BNRELU as above).
 * With dy = alpha dz + beta + gamma Y' and Y' = x W^T + scene_bias[b] (the stored seg_conv1
 * output, W = its local half as the forward GEMM saw it, fp32 [512, ldw]):
 *   dX[m]  = dz[m] WaT^T + x[m] H + cvec[b],  cvec[b] = W^T (beta + gamma * scene_bias[b])
 *   dW     = diag(alpha) dz^T x + beta (x) S + diag(gamma) (W G + sum_b scene_bias[b] (x) S_b)
 * with WaT = (diag(alpha) W)^T [64, 512] and H = W^T diag(gamma) W [64, 64] in bf16 (pcs_bn_fold),
 * G = x^T x, S_b = per-scene column sums of x (collected by the same pass).  dW (fp32, columns
 * 0..63 of rows with stride ldw, as W) is written, not accumulated.  Workspace:
 * pcs_dgrad_wgrad_folded_workspace() bytes (partials, their sums and cvec).  One pass reads
 * dz [M, 512] and X [M, 64] and writes dX: 1.2 KB per point instead of 2.3 KB.
 */
int64_t pcs_dgrad_wgrad_folded_workspace(pcs_wgrad_args *args); /* bytes; fills splits_per_scene */
int pcs_dgrad_wgrad_folded(const pcs_wgrad_args *args, const void *WaT, const void *H, const float *W,
                           const float *scene_bias, void *dX, pcs_stream_t stream);

/*
 * Fused input + weight gradient of a layer whose input gradient ends in the previous
 * layer's ReLU / dropout / BN-statistics epilogue (bf16; (Cout, Cin) = (K, Ncols) in
 * {64x64, 128x64}: conv2, conv3, conv4).  Takes the pcs_gemm arguments
 * of the PRO_BWD / EPI_DGRAD call (A = dZ, A2 = Y, pa/pb/pc, W = W^T [Cin, Cout], C, Yp,
 * es, et, emean, erstd, stats, c_mask | addend) and also writes dW = dy^T relu(es*Yp + et)
 * (* c_mask * c_keep_scale) into dW (row stride ldw, 0 = Cin) through the fp32 workspace.
 * chunks_per_scene (and so the stats rows) must come from the _workspace call.
 */
int64_t pcs_dgrad_wgrad_bn_workspace(pcs_gemm_args *args); /* bytes; fills chunks_per_scene */
int pcs_dgrad_wgrad_bn(const pcs_gemm_args *args, float *workspace, float *dW, int64_t ldw,
                       pcs_stream_t stream);

/*
 * Streaming column statistics of a stored activation Y [M, C] (C/8 (bf16) or C/4 (fp32)
 * must divide 256): per-chunk (mean, M2) BN partials and optional max-pool partials, in
 * pcs_gemm's epilogue formats.  One HBM pass; used for the 1024-wide global_feat output.
 */
int64_t pcs_colstats_geometry(int64_t num_scenes, int64_t scene_rows, int32_t C,
                              int32_t *chunks_per_scene);
int pcs_colstats(const void *Y, int64_t num_scenes, int64_t scene_rows, int32_t C, int32_t dtype,
                 int32_t chunks_per_scene, int64_t rows_per_chunk, float *stats, float *pool,
                 pcs_stream_t stream);

/*
 * The EPI_DGRAD epilogue as a streaming pass, in place on a raw dgrad output D [M, C]
 * (written by pcs_gemm with PCS_EPI_RAW): D = (Yp*s+t > 0) ? (D + addend)*keep : 0 and
 * per-chunk (S1, S2) partials; chunking as pcs_colstats_geometry.
 */
int pcs_bnrelu_bwd(void *D, const void *Yp, const void *addend, const uint8_t *mask, float keep_scale,
                   const float *s, const float *t, const float *mean, const float *rstd,
                   int64_t num_scenes, int64_t scene_rows, int32_t C, int32_t dtype,
                   int32_t chunks_per_scene, int64_t rows_per_chunk, float *stats, pcs_stream_t stream);

/*
 * BatchNorm1d train-mode statistics (P:86-94 semantics used at P:106-127): merge the
 * per-chunk (mean, M2) partials (Chan, fp64) into the batch mean / biased variance over
 * all B*N rows (pads included), derive the fused affine y*scale+shift, and update the
 * running buffers (momentum, unbiased variance) when update_running != 0.
 * The stored pre-BN activations may omit a per-channel constant (the conv bias, which BN
 * cancels): mean_offset[C] (NULL = 0) is added back for running_mean only.
 * scene_sum[B, C] receives the per-scene sum of the stored y (may be NULL).
 */
int pcs_bn_fwd_finalize(const float *stats, int64_t num_scenes, int64_t scene_rows,
                        int32_t C, int32_t chunks_per_scene, int64_t rows_per_chunk,
                        const float *gamma, const float *beta, const float *mean_offset,
                        float *running_mean, float *running_var, float momentum, float eps,
                        int32_t update_running, float *mean, float *rstd, float *scale,
                        float *shift, float *scene_sum, pcs_stream_t stream);
/* eval-mode BatchNorm: scale/shift from the running buffers (P:432 eval path), for stored
 * activations that omit mean_offset (NULL = 0) */
int pcs_bn_eval_coefs(const float *gamma, const float *beta, const float *running_mean,
                      const float *running_var, const float *mean_offset, float eps, int32_t C,
                      float *scale, float *shift, pcs_stream_t stream);
/*
 * BatchNorm1d backward from per-chunk (S1 = sum dz, S2 = sum dz*xhat) partials:
 * dy = alpha*dz + beta_c + gamma_c*y, dgamma = S2, dbeta = S1, and the conv-bias
 * gradient sum_m dy.  scene_s1[B,C] (sum dz per scene) may be NULL.
 */
int pcs_bn_bwd_finalize(const float *stats, int64_t num_scenes, int64_t scene_rows, int32_t C,
                        int32_t chunks_per_scene, const float *mean, const float *rstd,
                        const float *gamma, const float *scene_sum, float *alpha,
                        float *beta_c, float *gamma_c, float *dgamma, float *dbeta,
                        float *dbias, float *scene_s1, pcs_stream_t stream);

/*
 * Global max-pool (P:114) from per-chunk max/min partials of the global_feat conv output:
 * g[b,c] = max_n relu(y*s+t) taken at argmax (s>0) / argmin (s<0) of y; am = that row.
 */
int pcs_pool_finalize(const float *pool, int64_t num_scenes, int64_t scene_rows, int32_t C,
                      int32_t chunks_per_scene, const float *s, const float *t, float *g,
                      int32_t *am, float *ysel, pcs_stream_t stream);

/* v[b, n] = bias[n] + sum_k W[n, col_off + k] * g[b, k]   (seg_conv1 global half, P:117-123).
 * offset == NULL: out = v.  Otherwise out[b,n] = v[b,n] - mean_b v[b,n] (centred: the stored
 * seg_conv1 activations keep full precision) and offset[n] = mean_b v[b,n]. */
int pcs_scene_gemv(const float *g, int64_t num_scenes, int32_t Kg, const float *W, int64_t ldw,
                   int32_t col_off, const float *bias, int32_t Nout, float *out, float *offset,
                   pcs_stream_t stream);

/*
 * Backward through repeat+cat (P:117-120), the max-pool (P:114) and bn_global (P:113):
 * from bn_seg1's backward coefficients builds csum[b,n] = sum_{rows of b} dy_seg1[:, n],
 * dW_seg1[:, 64:] = sum_b csum_b (x) g_b, dg = W_seg1[:, 64:]^T csum_b, dz_g = dg*(g>0),
 * then bn_global's (alpha, beta, gamma, dgamma, dbeta, dbias) and the sparse coefficient
 * sp[b,c] = alpha_c*dz_g[b,c] consumed by PCS_PRO_BWD_POOL.
 */
typedef struct {
  int64_t num_scenes, scene_rows;
  int32_t Cs;           /* 512: seg_conv1 outputs */
  int32_t Cg;           /* 1024: global channels */
  int32_t col_off;      /* 64: first global column of W_seg1 */
  const float *s1_alpha, *s1_beta, *s1_gamma;  /* [Cs] bn_seg1 backward coefficients */
  const float *s1_scene_s1;   /* [B, Cs] sum dz per scene */
  const float *s1_scene_sum;  /* [B, Cs] sum y per scene (forward) */
  const float *W_s1;    /* [Cs, ldw] f32 */
  int64_t ldw;
  const float *g;       /* [B, Cg] pooled features */
  const float *ysel;    /* [B, Cg] global conv output at the argmax row */
  const float *g_mean, *g_rstd, *g_gamma; /* [Cg] bn_global */
  const float *g_scene_sum; /* [B, Cg] sum y_global per scene */
  float *dW_s1_global;  /* [Cs, ldw] f32: columns col_off.. written */
  float *csum;          /* [B, Cs] workspace */
  float *alpha, *beta_c, *gamma_c; /* [Cg] out */
  float *dgamma, *dbeta, *dbias;    /* [Cg] out */
  float *sp;            /* [B, Cg] out */
} pcs_pool_bwd_args;
int pcs_pool_bwd(const pcs_pool_bwd_args *args, pcs_stream_t stream);

/*
 * Segmentation head: seg_conv4 (P:128, no BN) on relu(bn_seg3(y)) and, by mode,
 *  PCS_HEAD_FWD: logits only;
 *  PCS_HEAD_CE : logits, weighted CE with ignore_index=-1 (P:216, P:251) and its gradient,
 *                then the seg_conv4 backward: dz_s3 = relu'(z)*(dlogits W), S1/S2 partials,
 *                dW_s4 / db_s4 partials;
 *  PCS_HEAD_BWD: the same backward from caller-supplied dlogits (autograd drop-in path).
 */
enum { PCS_HEAD_FWD = 0, PCS_HEAD_CE = 1, PCS_HEAD_BWD = 2 };
typedef struct {
  int64_t num_scenes, scene_rows;
  int32_t Cin;          /* 128 */
  int32_t num_classes;  /* 1 <= C <= 256 (C > 64: the wide head, 16-row tiles) */
  int32_t dtype, mode;
  int32_t chunks_per_scene; /* 0 = auto */
  const void *Y;        /* [M, Cin] y_seg3 */
  const float *s, *t;   /* bn_seg3 scale/shift */
  const float *W, *bias;/* seg_conv4 f32 [C, Cin], [C] */
  float *logits;        /* [M, C] f32 out or NULL */
  const int64_t *labels;/* [M] (CE) */
  const float *class_weight; /* [C] (CE) */
  const float *wsum;    /* device scalar D: CE gradient is divided by D (the global
                           sum of class weights over valid points, P:216); NULL = 1 */
  const float *dlogits; /* (BWD) */
  int64_t dl_stride_row, dl_stride_col; /* element strides of dlogits viewed as [M, C] */
  void *dZ;             /* [M, Cin] dz_seg3 (CE, BWD) */
  const float *mean, *rstd; /* bn_seg3 batch stats (S2) */
  float *stats;         /* [chunks, Cin, 2] */
  float *wpartial;      /* [chunks, C*Cin + C]: dW_s4 (row-major) then db_s4 partials */
  float *loss_partial;  /* [chunks]: sum w*nll (CE) */
} pcs_head_args;
int64_t pcs_head_geometry(pcs_head_args *args); /* fills chunks_per_scene; rows per chunk */
int pcs_head(const pcs_head_args *args, pcs_stream_t stream);

/* sum of class_weight[label] over labels != -1 (the CE denominator, P:216) -> out[0] (f32),
 * count of valid labels -> out[1], 1/out[0] -> out[2].  Exact: integer class counts (counts_ws[C], int64
 * workspace) times the weights, summed in fp64.  1 <= C <= 256. */
int pcs_ce_weight_sum(const int64_t *labels, int64_t M, const float *class_weight,
                      int32_t C, int64_t *counts_ws, float *out, pcs_stream_t stream);

/* Dropout(p) keep bits (P:96, P:124, P:126): Philox4x32-7 keyed by seed, counter (call index,
 * offset), one call per 16 elements; 16-bit uniforms u, keep = u >= round(p * 65536) (p within
 * 2^-17 of 1 keeps nothing); 8 bits per byte along the channel dimension; bits[M, C/8]. */
int pcs_dropout_bits(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                     uint8_t *bits, pcs_stream_t stream);
/* The same bits from at most max_workgroups 256-thread workgroups (<= 0: as many as the words
 * need), striding over the words: a draw that shares the GPU with a register-heavy kernel
 * (the training step draws beside the Gram of a5) occupies few wave slots for longer. */
int pcs_dropout_bits_bounded(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                             uint8_t *bits, int32_t max_workgroups, pcs_stream_t stream);
/* Opt-in for parity runs: the same keep rule with every element's 16-bit uniform from its own
 * two Philox bytes (i.i.d. Bernoulli, as nn.Dropout; pcs_dropout_bits lets elements 2k and
 * 2k + 1 share a byte pair: joint keep 0.490463 against 0.49 at p = 0.3), one call per 8
 * elements (twice pcs_dropout_bits's calls).  A different stream of bits from the same seed. */
int pcs_dropout_bits_independent(uint64_t seed, uint64_t offset, int64_t M, int32_t C, float p,
                                 uint8_t *bits, pcs_stream_t stream);

/*
 * Gram of the BN+ReLU activations a = relu(Y * s + t) (Y [M, C] scene-major rows), or of Y
 * itself when s = t = NULL (the stored a5 of global_feat; bf16, C % 256 == 0, no transform
 * pass in the kernel): G = a^T a (fp32 [C, C], symmetric, filled) and
 * colsum[k] = sum_m a[m, k].  Used by pcs_gram_wgrad in place of the M x C x C weight-
 * gradient GEMM of global_feat (autograd of P:113 at P:254).  pcs_gram_workspace returns
 * the fp32 workspace bytes and the row splits per scene to pass to pcs_gram.
 */
int64_t pcs_gram_workspace(int64_t num_scenes, int64_t scene_rows, int32_t C, int32_t dtype,
                           int32_t *splits_per_scene);
int pcs_gram(const void *Y, const float *s, const float *t, int64_t num_scenes, int64_t scene_rows,
             int32_t C, int32_t dtype, int32_t splits_per_scene, float *workspace, float *G,
             float *colsum, pcs_stream_t stream);

/*
 * out[r, :] = W[r, :] with its sign flipped where sign_of[r] < 0 (exact: the sign bit), rows x
 * cols contiguous, dtype F32, BF16 or FP8 (e4m3 bytes; an E8M0 row scale is unchanged).  The
 * forward global_feat weight for PCS_FLAG_POOL_SIGNED_W (sign_of = bn_global's gamma, P:113).
 */
int pcs_sign_rows(const void *W, int32_t dtype, int64_t rows, int64_t cols, const float *sign_of, void *out,
                  pcs_stream_t stream);

/*
 * fp8 e4m3 (OCP) rows with one E8M0 scale per row, for the fp8 wide layer (MX-scaled MFMA
 * operands whose 32-element blocks share the row's scale):
 *   scale[r] = 127 + ceil(log2(max_k |W[r, k]| / 448)) (clamped to [1, 254]; 127 for a zero row)
 *   Wq[r, k] = e4m3(W[r, k] * 2^(127 - scale[r]))   (round to nearest even, saturating)
 * deq (optional, [rows, cols] fp32): the values the MFMA sees, Wq[r, k] * 2^(scale[r] - 127).
 */
int pcs_quant_fp8_rows(const float *W, int64_t rows, int64_t cols, int64_t ldw, uint8_t *Wq, uint8_t *scale,
                       float *deq, pcs_stream_t stream);

/*
 * The max-pool rows' term of global_feat's folded input gradient (autograd of P:114 at P:254),
 * applied after a PCS_EPI_DGRAD pcs_gemm that ran without pool_w (the LDS-DMA kernel):
 *   dz[m, n] += (Yp[m, n] > 0) * sum_{c : pool_idx[b, c] == m} pool_coef[b, c] pool_w[c, n]
 * for every distinct argmax row m (global row index) of scene b; the same term is added to
 * S1 (stats[.].x) of the scene's chunk partials (spread over its first min(16,
 * chunks_per_scene) chunks; their sum is what the BN backward reads).  pool_idx / pool_coef:
 * [B, pool_c].
 */
int pcs_pool_rows_add(void *dz, int32_t dz_dtype, const void *Yp, int32_t yp_dtype, int64_t num_scenes,
                      int64_t scene_rows, int32_t Ncols, const int32_t *pool_idx, const float *pool_coef,
                      const float *pool_w, int64_t pool_ldw, int32_t pool_c, float *stats, int32_t chunks_per_scene,
                      pcs_stream_t stream);

/*
 * Gram G = A^T A [C, C] of a stored activation A [M, C] (C % 256 == 0; dtype PCS_BF16, or
 * PCS_FP8 for the e4m3 a5 of the fp8 path) on the LDS-DMA pipeline (csrc/gram_glds.hip):
 * upper 256-tiles x row splits in one wave of workgroups (a split's tiles share its rows
 * through one XCD's L2), fp32 partial tiles summed in a fixed order, lower tiles mirrored.
 * Products are exact in fp32 for both dtypes.  No column sums (they come from conv5's BN+ReLU
 * epilogue).  pcs_gram_raw_workspace returns the fp32 workspace bytes (one tile per workgroup).
 */
int64_t pcs_gram_raw_workspace(int64_t M, int32_t C);
int pcs_gram_raw(const void *A, int64_t M, int32_t C, int32_t dtype, float *workspace, int64_t workspace_bytes,
                 float *G, pcs_stream_t stream);

/*
 * Weight gradient of a BN-fed layer from the Gram of its input a (G, S from pcs_gram):
 *   dW[c, k] = alpha[c] R[c, k] + beta[c] S[k] + gamma[c] sum_j W[c, j] G[j, k]
 *              + sum_b sp[b, c] a[am[b, c], k]
 * i.e. dy^T a for dy = alpha*dz + beta + gamma*y (+ max-pool rows) and y = a W^T, without
 * reading y.  global_feat (P:113): R = NULL, dy from the max-pool (sp/am: pcs_pool_bwd /
 * pcs_pool_finalize; Y/s/t: stored conv5 output and bn5 scale/shift, a recomputed at the
 * argmax rows).  conv5 (P:110): R = dz^T a (pcs_wgrad with dy_mode RAW), sp = NULL.
 * W: fp32 [Cout, Cin] with row stride ldw_in; dW row stride ldw (multiple of 4).  dtype names
 * Y's storage (PCS_F32, PCS_BF16, or PCS_FP8 for the fp8 path's e4m3 a5).
 */
int pcs_gram_wgrad(const float *G, const float *S, const float *W, int64_t ldw_in,
                   const float *beta, const float *gamma, const float *sp, const int32_t *am,
                   const void *Y, const float *s, const float *t, int64_t num_scenes,
                   int32_t Cout, int32_t Cin, int32_t dtype, const float *R, const float *alpha,
                   float *dW, int64_t ldw, pcs_stream_t stream);

/*
 * Folded operands of the input gradient of a BN-fed layer y = a W^T (W fp32 [Cout, Cin],
 * row stride ldw) with BN-backward coefficients (alpha, beta, gamma) over Cout:
 *   dA = dz (diag(alpha) W) + a H + 1 c^T,  WsT = (diag(alpha) W)^T [Cin, Cout] (dtype),
 *   c = W^T beta [Cin] (fp32),  H = W^T diag(gamma) W [Cin, Cin] (dtype).
 * Two pcs_gemm launches then give dA without reading y (conv5 backward, P:110 at P:254).
 * WsT (and alpha) may be NULL: global_feat's dz is the sparse max-pool gradient, whose rows
 * pcs_gemm adds in its EPI_DGRAD epilogue (pool_w).  c (and beta) may be NULL when the caller
 * forms the constant row itself (pcs_dgrad_wgrad_folded's per-scene cvec).
 */
int pcs_bn_fold(const float *W, int32_t Cout, int32_t Cin, int64_t ldw, const float *alpha,
                const float *beta, const float *gamma, int32_t dtype, void *WsT, float *c, void *H,
                pcs_stream_t stream);

/*
 * BatchNorm statistics of y = a W^T (W [C, Cin] in dtype, row stride ldw) from the Gram of a
 * (G = a^T a [Cin, Cin] fp32, S = column sums [Cin], count rows): mean = W S / count and
 * M2[c] = w_c (G - S S^T / count) w_c^T, assembled in fp64.  Written as per-scene partials
 * stats[b, c] = (mean[c], M2[c] / num_scenes) for pcs_bn_fwd_finalize with
 * chunks_per_scene = 1 and rows_per_chunk = scene_rows (merging B identical partials gives
 * the totals).  The bf16 path's bn5 statistics (P:110): the Gram of a4 is needed by conv5's
 * weight gradient anyway, and this replaces a statistics-only pass of the 1024-wide GEMM.
 * Conditioning: the relative error is the Gram's times sum|w||w|G / var (~1e2 here), so the
 * fp32 parity path keeps the direct statistics.
 */
int pcs_bn_stats_from_gram(const float *G, const float *S, int64_t count, const void *W, int32_t dtype,
                           int64_t ldw, int32_t C, int32_t Cin, int64_t num_scenes, float *stats,
                           pcs_stream_t stream);

/*
 * As pcs_bn_stats_from_gram from per-scene column sums Sb [num_scenes, Cin] (each scene
 * scene_rows rows): exact per-scene means (pcs_bn_fwd_finalize's scene sums), per-scene M2
 * partials whose merge is the total M2.  bn_global's statistics on the bf16 / fp8 path
 * (P:113): the Gram of the stored a5 (global_feat's weight gradient needs it anyway) and the
 * per-chunk column sums of conv5's BN+ReLU epilogue replace the LDS-DMA forward's statistics
 * epilogue.  Requires C == Cin (G is read k-major, as its own transpose), both multiples of
 * 64, 1 <= num_scenes <= 64; the workspace (fp64 per-tile partials of w G w^T) is
 * pcs_bn_stats_from_gram_scenes_workspace(C, Cin) bytes.  Two launches: an fp64 64x64-tiled
 * G W^T contracted with W in its epilogue, then a per-channel fixed-order finalize.
 */
int64_t pcs_bn_stats_from_gram_scenes_workspace(int32_t C, int32_t Cin);
int pcs_bn_stats_from_gram_scenes(const float *G, const float *Sb, int64_t scene_rows, const void *W, int32_t dtype,
                                  int64_t ldw, int32_t C, int32_t Cin, int64_t num_scenes, void *workspace,
                                  int64_t workspace_bytes, float *stats, pcs_stream_t stream);

/*
 * S2 of a BN-fed layer's backward from R = dz^T a (pcs_wgrad with dy_mode RAW) instead of the
 * stored output: y = a W^T (bias-free, W [C, Cin] in dtype, row stride ldw), so
 *   S2[c] = sum_m dz[m,c] (y[m,c] - mean[c]) rstd[c] = rstd[c] (sum_k W[c,k] R[c,k] - mean[c] S1[c]).
 * Rewrites the S2 slots of the per-chunk (S1, S2) partials [num_chunks, C, 2]: chunk 0 holds
 * the total, the others 0 (pcs_bn_bwd_finalize sums them).  conv5 (P:110) when its output
 * is kept only as relu(bn5(y)) for global_feat.
 */
int pcs_bn_s2_from_r(float *stats, int64_t num_chunks, int32_t C, const float *R, const void *W,
                     int32_t dtype, int64_t ldw, int32_t Cin, const float *mean, const float *rstd,
                     pcs_stream_t stream);

/*
 * Confusion matrix of argmax predictions (P:261-266 accuracy, P:314-346 F1 / mIoU inputs):
 * cm[y, argmax_c logits[m, c]] += 1 for every point m with 0 <= labels[m] < C (labels -1 =
 * padding are skipped).  logits: fp32 rows of stride ld; cm: int64 [C, C], accumulated
 * (zero it once per epoch).  1 <= C <= 256 (LDS histogram up to 64 classes, global atomics above).
 */
int pcs_confusion(const float *logits, int64_t ld, const int64_t *labels, int64_t M, int32_t C,
                  int64_t *cm, pcs_stream_t stream);

/* out[m] = argmax_c logits[m, c] (first maximum; int64), the inference path of P:448-452 */
int pcs_argmax(const float *logits, int64_t ld, int64_t M, int32_t C, int64_t *out, pcs_stream_t stream);

/* out[i] = scale * sum_s partial[s*len + i]  (fixed order) */
int pcs_reduce_partials(const float *partial, int64_t nslabs, int64_t len, float scale,
                        float *out, int64_t out_stride_rows, int64_t row_len,
                        pcs_stream_t stream);

/* grouped form, one launch: out[g*len + i] = scale * sum_s partial[(g*nslabs + s)*len + i] for
 * g < ngroups (e.g. per-scene sums of scene-aligned chunk partials), fixed order */
int pcs_reduce_partials_grouped(const float *partial, int64_t ngroups, int64_t nslabs, int64_t len,
                                float scale, float *out, pcs_stream_t stream);

/* fp32 [rows, cols] (row stride ldw) -> dtype copies W ([rows, cols] contiguous) and W^T
 * ([cols, rows]); either output may be NULL */
int pcs_cast_weight(const float *W, int64_t rows, int64_t cols, int64_t ldw, int32_t dtype,
                    void *Wc, void *WcT, pcs_stream_t stream);

/*
 * torch.optim.Adam step with L2 (coupled) weight decay, amsgrad=False (P:217, P:255) on
 * flat fp32 buffers.  g_eff = g * (*grad_scale if non-NULL) + wd * p; with a grad_scale
 * the scaled gradient g * (*grad_scale) is written back into grad (the data-parallel step
 * normalises the all-reduced gradient by the global CE weight sum this way).
 */
int pcs_adam(float *param, float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
             const float *grad_scale, float lr, float beta1, float beta2, float eps,
             float weight_decay, int64_t step, pcs_stream_t stream);

/*
 * Device-side collate (replaces collate_fn's host padding, P:44-63).
 * CSR input: scene b owns rows offsets[b] .. offsets[b+1] (int64 [num_scenes+1], device) of
 * points (fp32 [T, 4], 16-byte aligned) and labels (int32 or int64 [T], label_bytes 4 / 8).
 * Outputs [num_scenes, scene_rows] (each may be NULL): points_out fp32 [.., 4] with (0,0,0,0)
 * pads, labels_out int64 with -1 pads, mask_out bool (uint8) 1 on real points.  The caller
 * guarantees every scene length <= scene_rows (the batch max, like collate_fn).
 */
int pcs_pad_scatter(const float *points, const void *labels, int32_t label_bytes,
                    const int64_t *offsets, int64_t num_scenes, int64_t scene_rows,
                    float *points_out, int64_t *labels_out, uint8_t *mask_out, pcs_stream_t stream);

/*
 * out = W rounded to the compute dtype and widened back to fp32 (bf16: round-to-nearest-even,
 * as pcs_cast_weight).  The bf16 path passes these to pcs_gram_wgrad: its dense terms
 * beta S^T + diag(gamma) W G cancel to O(pool rows / M) of their size, so W must be the W the
 * forward GEMM used, or the 2^-9 weight rounding dominates the gradient at large M.
 */
int pcs_round_weight(const float *W, int64_t n, int32_t dtype, float *out, pcs_stream_t stream);

/*
 * seg_conv1's local half and seg_conv2 in one streaming pass (the bf16 training forward,
 * P:117-125; csrc/fwd_s12.hip), replacing pcs_gemm's seg_conv1 pass plus its seg_conv2 pass:
 *   a2 = relu(y2 * s2 + t2);  Y1 = a2 W1^T + sbias[b]  (stored bf16 [M, 512], as pcs_gemm's
 *   FWD with scene_bias would store it);  x = relu(Y1 * s1 + t1) * keep * keep_scale, from the
 *   stored (rounded) Y1;  Y2 = x W2^T  (stored bf16 [M, 256]) with per-chunk (mean, M2) of the
 *   stored values in stats [B * chunks_per_scene, 256, 2] (pcs_bn_fwd_finalize's partials).
 * W1 is bf16 [512, 64] (seg_conv1's local half, pcs_cast_weight), W2 bf16 [256, 512]; s1 / t1
 * are bn_seg1's coefficients from batch statistics known before Y1 exists
 * (pcs_bn_stats_gram_sbias).  keep1 [M, 64] keep bits (bit i of byte j = channel 8j + i) or
 * NULL (no dropout).  pcs_fwd_seg12_geometry fills chunks_per_scene (0 = auto) and returns the
 * rows per chunk.
 */
typedef struct {
  int64_t num_scenes;
  int64_t scene_rows;
  int32_t chunks_per_scene;
  const void *y2;       /* [M, 64] bf16: conv2's stored pre-BN output */
  const float *s2, *t2; /* [64] bn2 scale / shift */
  const void *W1;       /* [512, 64] bf16 */
  const float *sbias;   /* [B, 512] per-scene bias of the stored Y1 (pcs_scene_gemv, centred) */
  void *Y1;             /* [M, 512] bf16 out */
  const float *s1, *t1; /* [512] bn_seg1 scale / shift */
  const uint8_t *keep1; /* [M, 64] dropout keep bits after bn_seg1 (P:124) or NULL */
  float keep_scale;     /* 1 / (1 - p) */
  const void *W2;       /* [256, 512] bf16 */
  void *Y2;             /* [M, 256] bf16 out */
  float *stats;         /* [B * chunks_per_scene, 256, 2] or NULL */
} pcs_seg12_args;
int64_t pcs_fwd_seg12_geometry(pcs_seg12_args *args);
int pcs_fwd_seg12(const pcs_seg12_args *args, pcs_stream_t stream);

/*
 * BatchNorm statistics of y = a W^T + sbias[b] (W [C, Cin] fp32, row stride ldw; Cin <= 64)
 * from the Gram of a (G = a^T a over all rows, fp32 [Cin, Cin]) and per-scene column sums Sb
 * [num_scenes, Cin] (scene_rows rows each): per-scene partials stats[b, c] = (mean_b,
 * M2w / num_scenes) with mean_b = Sb_b w / N + sbias[b, c] and M2w = w (G - sum_b Sb_b Sb_b^T /
 * N) w^T (fp64), for pcs_bn_fwd_finalize with chunks_per_scene = 1, rows_per_chunk = scene_rows
 * (its Chan merge adds the between-scene term).  bn_seg1's statistics for pcs_fwd_seg12
 * (P:123): seg_conv1's output is never read back for them.  sbias may be NULL.
 */
int pcs_bn_stats_gram_sbias(const float *G, const float *Sb, int64_t num_scenes, int64_t scene_rows,
                            const float *W, int64_t ldw, int32_t Cin, int32_t C, const float *sbias,
                            float *stats, pcs_stream_t stream);

/*
 * Bridge of the bf16 / fp8 EVAL forward's fp32 trunk (BatchNorm eval, P:106-110 with
 * model.eval(), P:313): a = relu(Y*s[k] + t[k]) of an fp32 pre-BN output Y [M, K] (row
 * stride K), stored as bf16 for a bf16 GEMM.  split = 0: out [M, K] = bf16(a).  split = 1:
 * out [M, 2K] = [hi | lo] with hi = bf16(a), lo = bf16(a - hi), so that a GEMM over 2K
 * against [W | W] sees a to 16 significant bits (conv5's input a4 in eval: the trained
 * network amplifies a4's bf16 rounding into logit-margin error).
 * K % 8 == 0.
 */
int pcs_bnrelu_bf16(const float *Y, int64_t M, int32_t K, const float *s, const float *t, int32_t split,
                    void *out, pcs_stream_t stream);

/*
 * Point -> voxel path (north-star voxel vocabulary; build-defined, the
 * reference has no voxelisation: parity is against oracle/voxel_oracle.py, not the reference).
 * Voxel id of a point: ix = clamp(floor((x - lo_x) / (hi_x - lo_x) * G), 0, G-1) (fp32, in this
 * order), likewise iy, iz; id = (ix * G + iy) * G + iz.  points: fp32 [T, 4] (x, y, z, e).
 */
int pcs_voxel_ids(const float *points, int64_t T, int32_t grid, float lo_x, float lo_y, float lo_z,
                  float hi_x, float hi_y, float hi_z, int64_t *ids, pcs_stream_t stream);
/*
 * Occupied-voxel scatter of a CSR batch (offsets [num_scenes+1], device): one voxel per
 * distinct (scene, voxel id), ordered scene-major then by id.  vox_points[v] = (mean x, mean y,
 * mean z, sum e) of its points (fp32 sums in point order), vox_labels[v] = most frequent label
 * (ties: smaller; labels < 0 ignored; -1 when none; labels may be NULL), vox_counts[v] = points,
 * vox_offsets [num_scenes+1] = voxel CSR, *num_voxels = V (device scalar), voxel_of_point[p] =
 * p's voxel (the gather back to points).  Output capacities: T voxels.  Deterministic: stable
 * radix sort of 64-bit keys + flag scan; integer outputs are bit-exact with the oracle.
 */
int64_t pcs_voxelize_workspace(int64_t T);   /* bytes */
int pcs_voxelize(const float *points, const int64_t *labels, const int64_t *offsets, int64_t num_scenes,
                 int64_t T, int32_t grid, float lo_x, float lo_y, float lo_z, float hi_x, float hi_y,
                 float hi_z, int32_t num_classes, void *workspace, int64_t workspace_bytes,
                 int64_t *voxel_of_point, float *vox_points, int64_t *vox_labels, int64_t *vox_counts,
                 int64_t *vox_offsets, int64_t *num_voxels, pcs_stream_t stream);
/* out[p] = row of p's voxel in a padded [num_scenes, scene_rows] voxel batch
 * (b * scene_rows + voxel_of_point[p] - vox_offsets[b]) */
int pcs_voxel_padded_index(const int64_t *voxel_of_point, int64_t T, const int64_t *vox_offsets,
                           int64_t num_scenes, int64_t scene_rows, int64_t *out, pcs_stream_t stream);
/* dst[r, :] = src[idx[r], 0:C] (row stride ld_src): per-voxel outputs back to their points */
int pcs_gather_rows(const float *src, int64_t ld_src, const int64_t *idx, int64_t n, int32_t C,
                    float *dst, pcs_stream_t stream);

/*
 * Dense 3-D convolution on channels-last voxel grids (the north star's 3x3x3 Conv3d
 * U-Net with LDS-staged stencils and transposed convolutions; build-defined, the reference has no
 * voxel grid: parity is against torch conv3d / conv_transpose3d in fp64, not the reference).
 * X [B, Di, Hi, Wi, Cin] bf16, W [Cout, k, k, k, Cin] bf16 (torch Conv3d weight permuted
 * (0, 2, 3, 4, 1); ConvTranspose3d weight permuted (1, 2, 3, 4, 0)), bias [Cout] f32 or NULL,
 * Y [B, Do, Ho, Wo, Cout] in ydtype (PCS_F32 | PCS_BF16), fp32 accumulation:
 *   transposed = 0:  Y[o] = b + sum_t W_t X[o s - p + t]                  Do = (Di + 2p - k) / s + 1
 *   transposed = 1:  Y[o] = b + sum_t W_t X[(o + p - t) / s] (exact only)  Do = (Di - 1) s - 2p + k + op
 * (op = torch's output_padding, 0 <= op < s, taken from the Do / Ho / Wo given).
 * k in 1..3, s in {1, 2}, 0 <= p < k.  pcs_conv3d: Cin % 32 == 0, Cout % 32 == 0 (64-channel
 * tiles, 32-channel tiles where a count is an odd multiple of 32; the Python layer zero-pads other
 * channel counts to multiples of 32).  The input gradient of either form is
 * the other form applied to dY with pcs_conv3d_weight_t(W) and the grids swapped (a strided
 * convolution's skipped trailing input planes come back as the transposed form's op).  pcs_conv3d_wgrad: dW [Cout, k, k, k, Cin] f32 = sum_o dY[o] (x) X[in(o, t)]
 * over the forward's index map, db [Cout] f32 = sum_o dY[o] (may be NULL); Cin, Cout % 32 == 0;
 * fp32 partials summed in a fixed order (deterministic).
 */
typedef struct {
  int64_t B;
  int32_t Di, Hi, Wi;   /* input grid */
  int32_t Do, Ho, Wo;   /* output grid */
  int32_t Cin, Cout;
  int32_t k, s, p;      /* cubic kernel, stride, padding */
  int32_t transposed;
} pcs_conv3d_geom;
int pcs_conv3d(const pcs_conv3d_geom *g, const void *X, const void *W, const float *bias, void *Y,
               int32_t ydtype, pcs_stream_t stream);
int64_t pcs_conv3d_wgrad_workspace(const pcs_conv3d_geom *g);   /* bytes */
int pcs_conv3d_wgrad(const pcs_conv3d_geom *g, const void *X, const void *dY, void *workspace,
                     int64_t workspace_bytes, float *dW, float *db, pcs_stream_t stream);
/* W [Cout][taps][Cin] -> Wt [Cin][taps][Cout] (bf16) */
int pcs_conv3d_weight_t(const void *W, int32_t Cout, int32_t taps, int32_t Cin, void *Wt, pcs_stream_t stream);

/*
 * Occupied-voxel (sparse) path: the north star's "hash-indexed gather" (BASELINE configs[2],
 * SURVEY §8 f4; build-defined, the reference has no voxel grid: parity is against the numpy
 * restatement oracle/sparse_oracle.py and against torch's dense conv3d on the occupied sites).
 *   key = scene * G^3 + (ix * G + iy) * G + iz (the voxel key of pcs_voxelize: keys are in voxel
 *         order, ascending).
 * pcs_voxel_keys: keys[voxel_of_point[p]] = key of point p (the box / grid of pcs_voxelize).
 * pcs_voxel_hash_*: open-addressing table, capacity a power of two >= 2 n
 *   (pcs_voxel_hash_capacity); table_keys u64 [cap], table_vals i32 [cap] (row of the key);
 *   find: out[i] = row of queries[i] or -1.
 *   Keys must be unique and below 2^64 - 1 (the EMPTY sentinel): a duplicate key keeps
 *   whichever row its insert wins, so pcs_amd.sparse.sparse_from_keys checks uniqueness.
 * pcs_sparse_neighbors: nbr [n][27] i32, nbr[v][t] = row of the voxel at (ix + a - 1, iy + b - 1,
 *   iz + c - 1), t = (a * 3 + b) * 3 + c, same scene, or -1 (the tap order of a torch Conv3d
 *   weight [Cout, Cin, 3, 3, 3] on a dense [B, C, G(x), G(y), G(z)] grid).
 * pcs_sparse_conv: submanifold convolution Y[m] = b + sum_t W[tw(t)] X[nbr[m][t]] over the M rows
 *   (X rows addressed by nbr), tw(t) = flip ? taps - 1 - t : t; X bf16 [*, Cin], W bf16
 *   [Cout][taps][Cin], Y [M, Cout] in ydtype; Cin % 32 == 0, Cout % 64 == 0.  The input gradient
 *   is the same call on dY with pcs_conv3d_weight_t(W) and flip = 1 (flip needs taps == 27, the
 *   centred neighbour map, or taps == 1).  A 64-row tile runs only the
 *   taps one of its rows has a neighbour at.
 * pcs_sparse_conv_wgrad: dW [Cout][taps][Cin] f32 = sum_m dY[m] (x) X[nbr[m][t]], db [Cout] (may be
 *   NULL); Cin, Cout % 64 == 0; fixed-order partial sums (deterministic).
 *
 * Per-tap pair lists (the same convolutions as gather-GEMM-reduce, for low occupancy where most
 * (row, tap) entries of nbr are -1): built once per neighbour map and shared by every layer.
 * pcs_sparse_pairs_count: tap_counts [taps] i64 (device) = valid entries per tap; workspace of
 *   pcs_sparse_pairs_workspace bytes, kept for the build.  The caller copies tap_counts to the host
 *   and forms tap_off [taps + 1] (exclusive prefix, P = tap_off[taps] pairs).
 * pcs_sparse_pairs_build: pair_in / pair_out [P] i32: tap t's pairs at [tap_off[t], tap_off[t + 1]),
 *   out rows ascending, pair_in = nbr[pair_out][t]; pair_pos [M][taps] i32 = the pair index of
 *   (m, t) or -1.
 * pcs_sparse_conv_pairs: pcs_sparse_conv's Y (same flip rule) from Z [P][Cout] f32 (workspace):
 *   Z[p] = W[tw(t)] X[pair_in[p]], then Y[m] = b + sum over t in order of Z[pair_pos[m][t]];
 *   tap_off is a HOST array.  Cin % 32 == 0, Cout % 64 == 0.
 * pcs_sparse_conv_wgrad_pairs: pcs_sparse_conv_wgrad's dW / db over the pairs only (dW_t = sum over
 *   tap t's pairs of dY[pair_out] (x) X[pair_in]); tap_off a host array; Cin, Cout % 64 == 0;
 *   fixed-order partial sums (deterministic).
 */
int pcs_voxel_keys(const float *points, const int64_t *offsets, int64_t num_scenes, int64_t T, int32_t grid,
                   float lo_x, float lo_y, float lo_z, float hi_x, float hi_y, float hi_z,
                   const int64_t *voxel_of_point, uint64_t *keys, pcs_stream_t stream);
int64_t pcs_voxel_hash_capacity(int64_t n);
int pcs_voxel_hash_build(const uint64_t *keys, int64_t n, uint64_t *table_keys, int32_t *table_vals,
                         int64_t capacity, pcs_stream_t stream);
int pcs_voxel_hash_find(const uint64_t *table_keys, const int32_t *table_vals, int64_t capacity,
                        const uint64_t *queries, int64_t nq, int32_t *out, pcs_stream_t stream);
int pcs_sparse_neighbors(const uint64_t *table_keys, const int32_t *table_vals, int64_t capacity,
                         const uint64_t *keys, int64_t n, int32_t grid, int32_t *nbr, pcs_stream_t stream);
int pcs_sparse_conv(const int32_t *nbr, int64_t M, int32_t taps, const void *X, int32_t Cin, const void *W,
                    int32_t Cout, const float *bias, void *Y, int32_t ydtype, int32_t flip, pcs_stream_t stream);
int64_t pcs_sparse_conv_wgrad_workspace(int64_t M, int32_t taps, int32_t Cin, int32_t Cout);   /* bytes */
int pcs_sparse_conv_wgrad(const int32_t *nbr, int64_t M, int32_t taps, const void *X, int32_t Cin, const void *dY,
                          int32_t Cout, void *workspace, int64_t workspace_bytes, float *dW, float *db,
                          pcs_stream_t stream);
int64_t pcs_sparse_pairs_workspace(int64_t M, int32_t taps);   /* bytes */
int pcs_sparse_pairs_count(const int32_t *nbr, int64_t M, int32_t taps, void *workspace, int64_t *tap_counts,
                           pcs_stream_t stream);
int pcs_sparse_pairs_build(const int32_t *nbr, int64_t M, int32_t taps, const void *workspace,
                           const int64_t *tap_counts, int32_t *pair_in, int32_t *pair_out, int32_t *pair_pos,
                           pcs_stream_t stream);
int pcs_sparse_conv_pairs(const int32_t *pair_in, const int32_t *pair_pos, const int64_t *tap_off, int32_t taps,
                          int64_t M, const void *X, int32_t Cin, const void *W, int32_t Cout, const float *bias,
                          float *Z, void *Y, int32_t ydtype, int32_t flip, pcs_stream_t stream);
int64_t pcs_sparse_conv_wgrad_pairs_workspace(const int64_t *tap_off, int32_t taps, int64_t M, int32_t Cin,
                                              int32_t Cout);   /* bytes */
int pcs_sparse_conv_wgrad_pairs(const int32_t *pair_in, const int32_t *pair_out, const int64_t *tap_off,
                                int32_t taps, int64_t M, const void *X, int32_t Cin, const void *dY, int32_t Cout,
                                void *workspace, int64_t workspace_bytes, float *dW, float *db, pcs_stream_t stream);

/* Build-time identification and error string.  pcs_abi_version() returns PCS_ABI_VERSION,
 * bumped with every change to an argument struct's layout or an entry point's signature
 * (2: pcs_gemm_args gained `gram`, the w4 entry points were removed); a binding checks it
 * before its first call. */
#define PCS_ABI_VERSION 2
int pcs_abi_version(void);
const char *pcs_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PCS_H */

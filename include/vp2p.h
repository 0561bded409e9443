/*
 * vp2p.h — C ABI of libvp2p_hip.so, the MI355X (gfx950) kernels of Video-P2P's controlled-attention
 * path.  Plain pointers, sizes and strides only; no torch types.  Every entry point:
 *   - takes caller-allocated DEVICE pointers and a hipStream_t (passed as void*, 0 = null stream),
 *   - never allocates, frees or synchronises (safe inside hipGraph capture),
 *   - returns VP2P_OK (0) or a negative VP2P_E_* status for an unsupported shape/dtype/argument,
 *     checked on the host BEFORE anything is launched.
 * Strides are in ELEMENTS; the channel dimension of every activation is contiguous (stride 1) and a
 * head's channels are [head*head_dim, (head+1)*head_dim).
 *
 * Which reference interface each entry point replaces (paths relative to emilycai99/Video-P2P):
 *   vp2p_frame_attn_fwd       FrameAttention core: tuneavideo/models/attention.py:282-322
 *                              (first-frame K/V gather :296-302 + xformers/_attention :314-322)
 *   vp2p_cross_attn_p2p_fwd   hooked attn2 forward after the projections: ptp_utils.py:206-220,
 *                              with the controller call :218 -> run_videop2p.py:212-224, 255-259,
 *                              304-317, 333-363 fused into the softmax epilogue, and the
 *                              AttentionStore sum that LocalBlend reads (:261-268, :145-146)
 *   vp2p_temporal_attn_p2p_fwd hooked attn_temp forward (attention.py:262-268 -> ptp_utils.py:206-220)
 *                              with replace_self_attention (run_videop2p.py:293-298, 306, 315)
 *   vp2p_cross_kv_prep        layout pass for vp2p_cross_attn_p2p_fwd's 77-token K/V (no reference
 *                              counterpart: the reference repeats the context per frame,
 *                              attention.py:95)
 *   vp2p_step_fused           CFG + DDIM step + LocalBlend: pipeline_tuneavideo.py:409-424 ->
 *                              dependent_ddim.py:268-309 (eta = 0) -> run_videop2p.py:142-155;
 *                              also NullInversion.next_step/prev_step (run_videop2p.py:445-463)
 *   vp2p_group_norm_* / vp2p_layer_norm_* / vp2p_geglu_*  (K7-K9, their backward K7b-K9b)
 *                              resnet.py:142,158, attention.py:110,200-216, FeedForward GEGLU
 *   vp2p_conv2d_fwd           (K10) InflatedConv3d / resnet convs, resnet.py:11-19, 111-205
 */
#ifndef VP2P_H
#define VP2P_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VP2P_ABI_VERSION 16

enum vp2p_status {
  VP2P_OK = 0,
  VP2P_E_ARG = -1,        /* null pointer / negative size / inconsistent sizes */
  VP2P_E_DTYPE = -2,      /* dtype not supported by this entry point */
  VP2P_E_HEAD_DIM = -3,   /* head_dim without a compiled kernel instance */
  VP2P_E_SHAPE = -4,      /* size above a kernel limit (frames > 128 temporal, tokens_kv > 128 cross) */
  VP2P_E_LAUNCH = -5      /* hipLaunchKernelGGL reported an error */
};

enum vp2p_dtype { VP2P_F32 = 0, VP2P_BF16 = 1 };

enum vp2p_edit_mode { VP2P_EDIT_NONE = 0, VP2P_EDIT_REPLACE = 1, VP2P_EDIT_REFINE = 2 };

/* ---- K1: FrameAttention (first-frame K/V), flash-style, MFMA -------------------------------- */
typedef struct vp2p_frame_attn_args {
  const void* q;            /* (batch, frames, tokens_q, heads*head_dim) strided */
  const void* k;            /* frame-0 keys   (batch, tokens_kv, heads*head_dim) strided */
  const void* v;            /* frame-0 values (batch, tokens_kv, heads*head_dim) strided */
  void* o;                  /* (batch, frames, tokens_q, heads*head_dim) strided */
  int64_t q_sb, q_sf, q_sn;
  int64_t k_sb, k_sn;
  int64_t v_sb, v_sn;
  int64_t o_sb, o_sf, o_sn;
  int32_t batch, frames, tokens_q, tokens_kv, heads, head_dim;
  float scale;              /* softmax scale (head_dim ** -0.5 in the reference) */
  int32_t dtype;            /* vp2p_dtype of q/k/v/o */
  float* lse;               /* optional (batch, heads, frames*tokens_q) fp32: log2 of each query row's
                             * sum_k exp2(score*scale*log2(e)), for the backward; NULL = off */
  int32_t q_prescaled;      /* 1: q already holds q * scale * log2(e) (the caller folded the softmax
                             * scale into its projection, e.g. as the GEMM's alpha: one rounding);
                             * `scale` is then ignored and lse is in the same units.  Selects the
                             * folded-max kernel at head_dim 40 (bf16). */
} vp2p_frame_attn_args;

int vp2p_frame_attn_fwd(const vp2p_frame_attn_args* args, void* stream);

/* ---- K1b: backward of the shared-K/V attention above (dQ, dK, dV) --------------------------------
 * Gradient of out = softmax(scale * Q K^T) V where every frame of batch element b attends to the
 * same keys/values K_b, V_b: FrameAttention (attention.py:282-322) and -- with tokens_kv = 77 --
 * the plain (uncontrolled) hooked cross-attention (ptp_utils.py:206-220 under the DummyController
 * of :225-234) that the null-text optimisation differentiates (run_videop2p.py:580-612,
 * loss.backward() at :601).  P is recomputed from the forward's lse; dK/dV sum over all
 * frames*tokens_q queries of b.  q, o, dout, dq share the query strides; k, v, dk, dv the key strides. */
typedef struct vp2p_frame_attn_bwd_args {
  const void* q; const void* k; const void* v; const void* o; const void* dout;
  const float* lse;         /* written by vp2p_frame_attn_fwd */
  void* dq; void* dk; void* dv;
  void* workspace;          /* vp2p_frame_attn_bwd_workspace_bytes() bytes, 16-byte aligned */
  int64_t q_sb, q_sf, q_sn; /* (batch, frames, tokens_q) element strides of q, o, dout, dq */
  int64_t kv_sb, kv_sn;     /* (batch, tokens_kv) element strides of k, v, dk, dv */
  int32_t batch, frames, tokens_q, tokens_kv, heads, head_dim;
  float scale;
  int32_t dtype;
} vp2p_frame_attn_bwd_args;

int64_t vp2p_frame_attn_bwd_workspace_bytes(const vp2p_frame_attn_bwd_args* args);
int vp2p_frame_attn_bwd(const vp2p_frame_attn_bwd_args* args, void* stream);

/* ---- K2: hooked cross-attention (<= 128 context tokens) + fused P2P edit --------------------- */
typedef struct vp2p_cross_attn_args {
  const void* q;            /* (batch, frames, tokens_q, heads*head_dim) strided */
  const void* kv_ws;        /* workspace written by vp2p_cross_kv_prep for this context */
  void* o;                  /* (batch, frames, tokens_q, heads*head_dim) strided */
  int64_t q_sb, q_sf, q_sn;
  int64_t o_sb, o_sf, o_sn;
  int32_t batch, frames, tokens_q, tokens_kv, heads, head_dim;
  float scale;
  int32_t dtype;
  /* P2P.  batch = 2 * prompts: rows [0, prompts) are the unconditional half, rows
   * [prompts, 2*prompts) the conditional half whose first prompt is the edit source. */
  int32_t prompts;
  int32_t edit_mode;        /* vp2p_edit_mode; applied to conditional rows of prompts 1.. */
  int32_t reweight;         /* multiply by equalizer inside the edit (AttentionReweight) */
  const float* alpha_words; /* (prompts-1, 77) cross_replace_alpha[cur_step] */
  const int32_t* map_ptr;   /* REPLACE: CSC column pointers (prompts-1, tokens_kv+1) */
  const int32_t* map_idx;   /* REPLACE: source word of each nonzero; REFINE: (prompts-1, tokens_kv) gather index */
  const float* map_val;     /* REPLACE: value of each nonzero */
  const float* refine_alpha;/* REFINE: (prompts-1, tokens_kv) */
  const float* equalizer;   /* (tokens_kv) */
  /* AttentionStore sum consumed by LocalBlend: lb_acc[s][p][frame][token] += sum over heads and words
   * of lb_word_alpha[s][p][w] * post-edit prob (conditional rows only).  NULL = off.  Set s = 0 holds
   * the blend words (alpha_layers), set 1 -- when lb_sets = 2 -- LocalBlend's substruct_words
   * (substruct_layers, run_videop2p.py:149-151, 166-174). */
  float* lb_acc;            /* (lb_sets, prompts, frames, tokens_q) fp32 */
  const float* lb_word_alpha; /* (lb_sets, prompts, tokens_kv) */
  /* Optional post-edit probabilities in the reference's attn layout
   * ((batch*frames*heads), tokens_q, tokens_kv) fp32.  NULL = off. */
  float* probs_out;
  /* Scratch for the per-head LocalBlend partials, (lb_sets, prompts, heads, frames*tokens_q) fp32;
   * required when lb_acc is set (the head sum is finished in a fixed order by a second pass). */
  float* lb_ws;
  int32_t lb_sets;          /* word-weight sets accumulated: 1 (0 is read as 1) or 2 */
  /* 1: the batch holds ONLY the conditional half (batch = prompts) -- a rank of a CFG-split edit
   * (the unconditional rank runs with prompts = 0, i.e. plain attention); 0: batch = 2*prompts. */
  int32_t cond_only;
} vp2p_cross_attn_args;

/* Bytes of the K/V workspace for one context of the given shape (<0: unsupported). */
int64_t vp2p_cross_kv_workspace_bytes(int32_t batch, int32_t tokens_kv, int32_t heads,
                                      int32_t head_dim, int32_t dtype);

/* Pads / transposes the projected context K, V ((batch, tokens_kv, heads*head_dim) strided) into
 * the MFMA fragment layout vp2p_cross_attn_p2p_fwd reads (one pass over B*77*C elements). */
int vp2p_cross_kv_prep(const void* k, const void* v, int64_t k_sb, int64_t k_sn, int64_t v_sb,
                       int64_t v_sn, int32_t batch, int32_t tokens_kv, int32_t heads,
                       int32_t head_dim, int32_t dtype, void* kv_ws, void* stream);

int vp2p_cross_attn_p2p_fwd(const vp2p_cross_attn_args* args, void* stream);

/* ---- K3: hooked temporal attention (frames <= 128) + self-attention replace ------------------- */
typedef struct vp2p_temporal_attn_args {
  const void* q; const void* k; const void* v; void* o;   /* (batch, frames, tokens, C) strided */
  int64_t q_sb, q_sf, q_sn;
  int64_t k_sb, k_sf, k_sn;
  int64_t v_sb, v_sf, v_sn;
  int64_t o_sb, o_sf, o_sn;
  int32_t batch, frames, tokens, heads, head_dim;
  float scale;
  int32_t dtype;
  int32_t prompts;          /* batch = 2*prompts when self_replace is set */
  int32_t self_replace;     /* conditional rows of prompts 1.. use the source prompt's probs */
  float* probs_out;         /* ((batch*tokens*heads), frames, frames) fp32 in '(b d)' order, or NULL */
  int32_t cond_only;        /* as vp2p_cross_attn_args.cond_only (batch = prompts, all conditional) */
} vp2p_temporal_attn_args;

int vp2p_temporal_attn_p2p_fwd(const vp2p_temporal_attn_args* args, void* stream);

/* ---- K3b: backward of the plain hooked temporal attention (no self-replace) --------------------
 * attn_temp under the DummyController (attention.py:262-268 -> ptp_utils.py:206-220, 225-234),
 * differentiated by the null-text optimisation (run_videop2p.py:601).  All tensors are
 * (batch, frames, tokens, C) strided views; dq/dk/dv may be views of one (.., 3C) buffer. */
typedef struct vp2p_temporal_attn_bwd_args {
  const void* q; const void* k; const void* v; const void* dout;
  void* dq; void* dk; void* dv;
  int64_t q_sb, q_sf, q_sn;
  int64_t k_sb, k_sf, k_sn;
  int64_t v_sb, v_sf, v_sn;
  int64_t do_sb, do_sf, do_sn;
  int64_t dq_sb, dq_sf, dq_sn;
  int64_t dk_sb, dk_sf, dk_sn;
  int64_t dv_sb, dv_sf, dv_sn;
  int32_t batch, frames, tokens, heads, head_dim;   /* frames <= 32, head_dim % 8 == 0 */
  float scale;
  int32_t dtype;
} vp2p_temporal_attn_bwd_args;

int vp2p_temporal_attn_bwd(const vp2p_temporal_attn_bwd_args* args, void* stream);

/* ---- K5+K6: classifier-free guidance + DDIM update + LocalBlend, one launch --------------------
 *   e_p   = cfg ? u_p + g*(t_p - u_p) : n_p        (fast: e_0 = t_0)
 *   x'_p  = c4 * ((x_p - c1*e_p) / c2) + c3*e_p    (each op rounded separately, as torch does)
 *   blend : x''_p = x'_0 + m_p*(x'_p - x'_0), m_p = (mask_0 | mask_p) & ~(sub_0 | sub_p),
 *           mask_p = up(pool3x3(lb_acc_p / lb_count)) / max(...) > th
 *           sub_p  = up(lb_sub_p / lb_count) / max(...) > sub_th   (no pool; only when lb_sub)    */
typedef struct vp2p_step_args {
  const void* noise;        /* (cfg ? 2*prompts : prompts, channels, frames, height, width) contiguous */
  int32_t noise_dtype;
  const float* latents;     /* (prompts, channels, frames, height, width) contiguous fp32 */
  float* out;               /* same shape; may alias latents */
  int32_t prompts, channels, frames, height, width;
  int32_t cfg, fast;
  float guidance;
  float c1, c2, c3, c4;
  const float* lb_acc;      /* (prompts, frames, lb_h*lb_w) or NULL = no blend */
  int32_t lb_h, lb_w;
  float lb_count;           /* number of maps summed per step (layers*heads): the reference's mean */
  float lb_th;
  const float* lb_sub;      /* (prompts, frames, lb_h*lb_w) substruct_words sum, or NULL (run_videop2p.py:149-151) */
  float lb_sub_th;          /* th[1] */
  /* Optional (prompts, frames, height, width) uint8: the blend mask m_p this launch applied (0/1; the
   * reference's `mask` after `mask[:1] + mask` and the substruct product, run_videop2p.py:137-153).
   * Written only when lb_acc is set.  NULL = off (a debug / parity output). */
  uint8_t* mask_out;
} vp2p_step_args;

int vp2p_step_fused(const vp2p_step_args* args, void* stream);

/* ---- K6b: null-text inner loss + gradient ---------------------------------------------------------
 * NullInversion.null_optimization (run_videop2p.py:594-599): e = u + g*(c - u),
 * rec = prev_step(e) = c4*((x - c1*e)/c2) + c3*e, loss = mean((rec - x_prev)^2); writes loss[0] and
 * grad_uncond = dloss/du (what loss.backward() feeds the UNet).  partials: workspace of
 * vp2p_nulltext_loss_partials() floats. */
typedef struct vp2p_nulltext_loss_args {
  const void* noise_uncond; const void* noise_cond;   /* (n) contiguous, noise_dtype */
  int32_t noise_dtype;
  const float* latents; const float* latents_prev;    /* (n) fp32 */
  void* grad_uncond;                                  /* (n) noise_dtype */
  float* partials;
  float* loss;
  int64_t n;
  float guidance, c1, c2, c3, c4;
} vp2p_nulltext_loss_args;

int vp2p_nulltext_loss(const vp2p_nulltext_loss_args* args, void* stream);
int32_t vp2p_nulltext_loss_partials(void);

/* ================================================================================================
 * Non-attention UNet path.  Activations are channels-last and contiguous:
 * element (row, c) of a (rows, channels) matrix, row = (sample, h, w) flattened.
 * ============================================================================================== */

/* ---- K7: 5-D GroupNorm (+ per-sample channel add, + SiLU) ---------------------------------------
 * Replaces nn.GroupNorm on the (b, c, f, h, w) tensor (statistics over c/G x f x h x w):
 * tuneavideo/models/resnet.py:142,158 (+ the h + temb add at :149-156 and nonlinearity :143,159),
 * unet.py:206 (conv_norm_out + SiLU) and Transformer3DModel.norm (attention.py:110, frames = 1).
 * Two kernels: _stats writes per-chunk (count, mean, M2) partials; _apply merges partials (Chan)
 * and normalises.  A frame-sharded caller gathers the partials of every rank between the two. */
typedef struct vp2p_group_norm_args {
  const void* x;            /* (batch*frames*rows, channels), dtype */
  const void* add;          /* optional (batch*frames, channels), dtype: added to x before the norm */
  void* y;                  /* like x; may alias x */
  const void* weight;       /* (channels) dtype, or NULL (affine off) */
  const void* bias;         /* (channels) dtype, or NULL */
  float* partials;          /* (batch, parts, groups, 3) fp32, parts = vp2p_group_norm_parts() */
  int32_t batch;            /* statistics groups: samples = batch * frames */
  int32_t frames;           /* samples sharing one set of statistics */
  int32_t rows;             /* h*w rows per sample */
  int32_t channels, groups; /* channels % 8 == 0 and <= 4096, channels % groups == 0, groups <= 64 */
  float eps;
  int32_t silu;             /* apply x * sigmoid(x) after the affine */
  int32_t dtype;
  /* two-source input (the up blocks' torch.cat([hidden, skip], dim=1), unet_blocks.py: the cat is
   * never written): x holds channels [0, channels - channels2) with that row stride, x2 the last
   * channels2 (row stride channels2); both % 8 == 0.  NULL / 0: x holds all channels.  Forward only. */
  const void* x2;
  int32_t channels2;
} vp2p_group_norm_args;

int32_t vp2p_group_norm_parts(const vp2p_group_norm_args* args);   /* <0: unsupported shape */
int vp2p_group_norm_stats(const vp2p_group_norm_args* args, void* stream);
/* nsets partial arrays laid out back to back, each (batch, parts, groups, 3) */
int vp2p_group_norm_apply(const vp2p_group_norm_args* args, const float* partials, int32_t nsets,
                          void* stream);
int vp2p_group_norm_fwd(const vp2p_group_norm_args* args, void* stream);   /* stats + finalize + apply */
/* Merge the nsets partial arrays once into per-(batch, group) {mean, rstd} fp32 (batch, groups, 2)
 * (resnet.py:142,158: nn.GroupNorm's statistics over c/G x f x h x w), so that the apply blocks read
 * two floats per group instead of each merging every partial. */
int vp2p_group_norm_finalize(const vp2p_group_norm_args* args, const float* partials, int32_t nsets,
                             float* stats, void* stream);
/* The apply of vp2p_group_norm_apply on finalized statistics. */
int vp2p_group_norm_apply_stats(const vp2p_group_norm_args* args, const float* stats, void* stream);
/* Frame-sharded callers: merge this rank's partial array into one (count, mean, M2) triple per
 * (batch, group), fp32 (batch, groups, 3) -- what the ranks exchange (B*G*12 bytes instead of the
 * B*parts*G*12 of the raw partials) -- and, after the gather, finalize nsets such triple arrays laid
 * out back to back into {mean, rstd} (batch, groups, 2) for vp2p_group_norm_apply_stats. */
int vp2p_group_norm_merge(const vp2p_group_norm_args* args, const float* partials, float* triples, void* stream);
/* The same two merges over a partial array of `parts` entries per (batch, group) produced elsewhere
 * (vp2p_conv_args.gn_partials: the producing convolution's epilogue) instead of by _stats:
 * _finalize_parts -> {mean, rstd} (batch, groups, 2) for vp2p_group_norm_apply_stats, _merge_parts ->
 * the (batch, groups, 3) triples of a frame-sharded exchange. */
int vp2p_group_norm_finalize_parts(const vp2p_group_norm_args* args, const float* partials, int32_t parts,
                                   float* stats, void* stream);
/* The apply of vp2p_group_norm_apply on such partials, merged inside every apply block (one launch:
 * cheaper than _finalize_parts + _apply_stats at small part counts). */
int vp2p_group_norm_apply_parts(const vp2p_group_norm_args* args, const float* partials, int32_t parts,
                                void* stream);
int vp2p_group_norm_merge_parts(const vp2p_group_norm_args* args, const float* partials, int32_t parts,
                                float* triples, void* stream);
int vp2p_group_norm_finalize_merged(const vp2p_group_norm_args* args, const float* triples, int32_t nsets,
                                    float* stats, void* stream);

/* ---- K8: LayerNorm over the channel axis --------------------------------------------------------
 * nn.LayerNorm of BasicTransformerBlock.norm1/norm2/norm3/norm_temp (attention.py:200-216). */
typedef struct vp2p_layer_norm_args {
  const void* x; void* y;   /* (rows, channels), dtype; y may alias x */
  const void* weight; const void* bias;   /* (channels) dtype or NULL */
  int64_t rows;
  int32_t channels;         /* channels % 8 == 0, <= 2048 */
  float eps;
  int32_t dtype;
} vp2p_layer_norm_args;

int vp2p_layer_norm_fwd(const vp2p_layer_norm_args* args, void* stream);
/* The transformer block's residual add fused in front of the next LayerNorm (attention.py:247-268):
 * sum = round(x + residual) (dtype), y = LayerNorm(sum).  sum may alias x or residual. */
int vp2p_add_layer_norm_fwd(const vp2p_layer_norm_args* args, const void* residual, void* sum, void* stream);

/* ---- K9: GEGLU gate ------------------------------------------------------------------------------
 * diffusers 0.11.1 GEGLU.forward after its projection: y = a * gelu(g), (a, g) = proj(x).chunk(2)
 * (FeedForward of attention.py:190, 259).  x: (rows, 2*inner), y: (rows, inner); exact erf GELU,
 * rounded like torch's eager ops (gelu result to dtype, then the product). */
int vp2p_geglu_fwd(const void* x, void* y, int64_t rows, int32_t inner, int32_t dtype, void* stream);

/* ---- K7b-K9b: input gradients of K7-K9 (weights frozen: run_videop2p.py:580-612 optimises only
 * the unconditional embedding).  GroupNorm: _reduce writes (batch, parts, groups, 2) fp32 partial
 * sums (sum g, sum g*xhat) from the forward partials; _apply merges bsets such arrays (a
 * frame-sharded caller gathers them between the two) and writes dx.  `add` / `silu` as in the
 * forward (d(add) is not produced). */
int vp2p_group_norm_bwd_reduce(const vp2p_group_norm_args* args, const float* partials, int32_t nsets,
                               const void* dy, float* bwd_partials, void* stream);
int vp2p_group_norm_bwd_apply(const vp2p_group_norm_args* args, const float* partials, int32_t nsets,
                              const void* dy, const float* bwd_partials, int32_t bsets, void* dx,
                              void* stream);
int vp2p_layer_norm_bwd(const vp2p_layer_norm_args* args, const void* dy, void* dx, void* stream);
/* x: the forward input (rows, 2*inner); dy: (rows, inner); dx: (rows, 2*inner) */
int vp2p_geglu_bwd(const void* x, const void* dy, void* dx, int64_t rows, int32_t inner, int32_t dtype,
                   void* stream);

/* ---- K10: implicit-GEMM convolution, channels-last bf16 -----------------------------------------
 * nn.Conv2d of InflatedConv3d (tuneavideo/models/resnet.py:11-19: conv1/conv2/conv_shortcut of
 * ResnetBlock3D :111-205, Downsample3D/Upsample3D convs) with the bias and, optionally, the resnet's
 * shortcut add 'input_tensor + hidden_states' (:196-205) fused:  y = conv(x, w) + bias (+ residual).
 * x: (batch, in_h, in_w, cin) contiguous; w: (cout, kernel, kernel, cin) contiguous (the memory of a
 * channels_last conv weight); bias: (cout) or NULL; residual, y: (batch, out_h, out_w, cout).
 * Supported: bf16, kernel 1 or 3, pad = (kernel-1)/2, stride 1 or 2, cin % 64 == 0, cout % 160 == 0;
 * vp2p_conv2d_supported() reports it without launching (1 = yes). */
enum vp2p_conv_epilogue {
  VP2P_CONV_EPI_NONE = 0,
  /* diffusers GEGLU after its projection (FeedForward, attention.py:190,259): kernel 1, no residual;
   * w/bias rows interleaved per 16 rows as [8 value rows, the 8 matching gate rows] (ABI 13; was per
   * 160); y is (batch*in_h*in_w, cout/2) = value * gelu(gate), rounded like K9. */
  VP2P_CONV_EPI_GEGLU = 1
};

typedef struct vp2p_conv_args {
  const void* x; const void* w; const void* bias; const void* residual; void* y;
  int32_t batch, in_h, in_w, cin;
  int32_t cout, out_h, out_w;
  int32_t kernel, stride, pad;
  int32_t dtype;
  int32_t epilogue;         /* vp2p_conv_epilogue */
  float* workspace;         /* fp32 split-K slices, vp2p_conv2d_workspace_bytes() bytes, or NULL (one pass) */
  int32_t ksplit;           /* set by the library; callers leave 0 */
  int32_t upsample;         /* 1: x is (batch, in_h/2, in_w/2, cin), nearest-upsampled x2 on the fly
                               (Upsample3D's F.interpolate, resnet.py:79-99); stride 1 only */
  /* two-source input of a 1x1 conv (the up blocks' resnet conv_shortcut on torch.cat([hidden, skip])):
   * x holds input channels [0, cin - cin2) (row stride cin - cin2), x2 the last cin2 (row stride
   * cin2); both % 64 == 0.  NULL / 0: x holds all cin channels. */
  const void* x2;
  int32_t cin2;
  /* output scale of the one-pass / split-K epilogue without a residual: y = alpha * (x * w + bias),
   * one rounding (the FrameAttention to_q projection pre-scaled by scale * log2 e for K1's folded
   * max, torch.addmm(bias, x, w^T, beta=alpha, alpha=alpha) of the reference-precision path);
   * 0 = 1 (zero-initialised callers). */
  float alpha;
  /* (since ABI 15) a per-image add after the bias -- the resnet's h + temb (resnet.py:149-156):
   * y = round(round(x * w + bias) + img_add[p / (out_h * out_w), c]), img_add (batch, cout) dtype, the
   * two roundings of the reference; NULL = none.  Plain one-pass epilogue without a residual. */
  const void* img_add;
  /* (since ABI 15) GroupNorm statistics of the stored output (the next norm2, resnet.py:158), written
   * by the epilogue: (count, mean, M2) fp32 per (statistics sample s, M tile t, group g) at
   * gn_partials[((s * parts + t) * gn_groups + g) * 3], s = p / gn_rows, parts =
   * vp2p_conv2d_gn_parts(); NULL = none.  gn_rows: output pixels per sample (frames * out_h * out_w). */
  float* gn_partials;
  int32_t gn_groups;
  int32_t gn_rows;
} vp2p_conv_args;

int vp2p_conv2d_supported(const vp2p_conv_args* args);
/* M tiles per GroupNorm statistics sample of the tile this launch would use (the partial count per
 * (sample, group) that gn_partials receives), or <= 0 when the shape cannot produce them in the
 * epilogue (split-K, a GEGLU / scaled epilogue, gn_rows not a multiple of the tile, groups not whole
 * within a tile).  With a residual the statistics are those of residual + conv (the stored values). */
int32_t vp2p_conv2d_gn_parts(const vp2p_conv_args* args);
/* Workspace the shape wants for split-K (small-M shapes: fewer tiles than CUs); 0 = none. */
int64_t vp2p_conv2d_workspace_bytes(const vp2p_conv_args* args);
/* (since ABI 16) The launch plan vp2p_conv2d_fwd takes for this shape (given a workspace where it wants
 * one): *tile = 0 128x160, 1 256x160, 2 256x320, 3 64x160, 4 192x320, or 5 the K = 320 stream (K10s);
 * *ksplit = K slices (1 = one pass).  Host logic only; VP2P_OK or VP2P_E_SHAPE (unsupported). */
int vp2p_conv2d_plan(const vp2p_conv_args* args, int32_t* tile, int32_t* ksplit);
int vp2p_conv2d_fwd(const vp2p_conv_args* args, void* stream);

/* ---- introspection ---------------------------------------------------------------------------- */
int vp2p_abi_version(void);
/* Head dims with compiled kernel instances, written to out[0..n); returns the count. */
int vp2p_supported_head_dims(int32_t* out, int32_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* VP2P_H */

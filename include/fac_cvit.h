/*
 * fac_cvit.h - C ABI of the MI355X (gfx950) CViT per-crop face-forgery path.
 *
 * Drop-in boundary for the reference's hot path.  The reference has no FFI:
 * its boundary is the Python class `CViT` (CViT-main/model/cvit.py:80-179)
 * that `cvit_prediction.py:20,24,62-70` imports, loads a state_dict into and
 * calls under torch.no_grad().  Each entry point below replaces one piece of
 * that contract; the Python mirror (fac_fake_amd/cvit.py) binds them with
 * ctypes and keeps the reference's class name, constructor, state_dict keys
 * and forward() semantics.  See INTEGRATION.md for the bindings.
 *
 * Conventions: plain pointers and sizes only.  Pointers named d_* are device
 * pointers owned by the caller; `stream` is a hipStream_t (NULL = default
 * stream).  Every call returns 0 (FAC_OK) or a negative fac_status and never
 * throws; fac_last_error() describes the last failure on a context.  All work
 * is stream-ordered with no host synchronisation, so a forward call can be
 * captured into a hipGraph once fac_reserve() has sized the workspace.
 */
#ifndef FAC_CVIT_H
#define FAC_CVIT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct fac_ctx fac_ctx;

typedef enum {
  FAC_OK = 0,
  FAC_ERR_ARG = -1,        /* null pointer / bad enum / bad size */
  FAC_ERR_SHAPE = -2,      /* tensor shape does not match the CViT config */
  FAC_ERR_MISSING = -3,    /* a required state_dict key was not supplied */
  FAC_ERR_HIP = -4,        /* HIP runtime error (message in fac_last_error) */
  FAC_ERR_NOT_LOADED = -5, /* forward before fac_load_weights */
  FAC_ERR_OOM = -6         /* device allocation failed */
} fac_status;

/* Operand type of the MFMA path (accumulation and epilogues are fp32). */
typedef enum { FAC_DTYPE_BF16 = 0, FAC_DTYPE_F16 = 1 } fac_dtype;

/* One host fp32 tensor of a CViT state_dict (cvit_train.py:210 layout).
 * `name` is the state_dict key, e.g. "features.0.weight". */
typedef struct {
  const char* name;
  const float* data;
  int ndim;
  int64_t shape[4];
} fac_tensor_desc;

/* Replaces `CViT(image_size=224, patch_size=7, num_classes=2, channels=512,
 * dim=1024, depth=6, heads=8, mlp_dim=2048).to(device)`
 * (cvit.py:81-82, cvit_prediction.py:62-64).  Only that configuration is
 * supported. */
int fac_create(int device, int dtype, fac_ctx** out);

/* Replaces `model.load_state_dict(sd)` (cvit_prediction.py:67-69).  Takes the
 * 193-key state_dict as host fp32 tensors (num_batches_tracked keys may be
 * omitted), folds eval-mode BatchNorm into the convs, repacks to NHWC/K-major
 * 16-bit and uploads.  Synchronous. */
int fac_load_weights(fac_ctx* ctx, const fac_tensor_desc* descs, int n);

/* Size the device workspace for batches of up to max_batch crops (allocates;
 * call before graph capture).  forward() grows it on demand otherwise. */
int fac_reserve(fac_ctx* ctx, int max_batch);

/* Bytes of device workspace a batch of B crops needs. */
int fac_workspace_bytes(fac_ctx* ctx, int B, size_t* out);

/* Replaces `model(x)` (cvit.py:167-179 via cvit_prediction.py:229):
 * d_in = normalised fp32 NCHW [B,3,224,224]; d_pos_index = int32 [B] batch
 * slot of each crop in [0,32) (pos_embedding row, cvit.py:154,175);
 * d_logits = fp32 [B,2]; d_probs = fp32 [B,2] per-logit sigmoid (pred_sig,
 * cvit_prediction.py:258-259) or NULL. */
int fac_forward_nchw_f32(fac_ctx* ctx, const float* d_in, int B, const int32_t* d_pos_index, float* d_logits,
                         float* d_probs, void* stream);

/* Same, from raw uint8 NHWC face crops [B,224,224,3] (RGB, the crop format of
 * cvit_prediction.py:106-121,202): the /255 + ImageNet normalisation of
 * cvit_prediction.py:41-45,212-215 is fused into conv1.
 * Both forwards: with B <= the "graph_max_b" option (default 32, which covers
 * the reference's one-video call of <= 29 crops, cvit_prediction.py:224-229)
 * on a stream that is not being captured, the forward replays a hipGraph
 * captured once per (B, input kind, d_probs != NULL): d_in and d_pos_index are
 * copied into context-owned buffers, the graph runs, the outputs are copied
 * out -- one graph launch instead of ~60 kernel launches, bit-identical
 * outputs.  Graphs are dropped on fac_load_weights, fac_set_option and
 * workspace growth.  Calls on one context from different streams are ordered
 * on the device (each waits for the context's previous forward). */
int fac_forward_nhwc_u8(fac_ctx* ctx, const uint8_t* d_in, int B, const int32_t* d_pos_index, float* d_logits,
                        float* d_probs, void* stream);

/* Everything after the conv stem (cvit.py:170-179): d_feat = 16-bit NHWC
 * stem features [B,7,7,512] (the (p1 p2 c) flatten of cvit.py:170) ->
 * patch embedding, cls/pos, transformer, head.  d_hidden (fp32 [B,2048],
 * or NULL) receives ReLU(mlp_head.0(cls)); d_logits/d_probs (or NULL) the
 * final layer.  With fac_set_option(ctx, "tail_only", 1) before
 * fac_load_weights only the embedding/transformer/head keys are needed:
 * ResVitKan (CViT-main/ResVitKan/ResVitKan.py:316-329) shares this tail
 * behind its ResNet-50 stem, with kan_head.0 as mlp_head.0 and the KAN
 * (fac_ops.h) on d_hidden. */
int fac_forward_features(fac_ctx* ctx, const void* d_feat, int B, const int32_t* d_pos_index, float* d_hidden,
                         float* d_logits, float* d_probs, void* stream);

/* Software-pipelined forward for streams of batches (a video-scoring
 * server; bench.py's default mode).  Enqueues batch k's conv stack on
 * `stream` (into one of two context-owned stem buffers) and its patch
 * embedding + encoder + head (+ video score into d_score if non-NULL) on a
 * context-owned stream that waits only for that conv stack, so batch k's
 * latency-bound encoder overlaps batch k+1's conv stack.  Same arithmetic as
 * fac_forward_nhwc_u8 (bit-identical logits).  d_in may be reused once
 * `stream` has passed this call; d_pos / d_logits / d_probs / d_score must
 * stay valid, and are complete, only after fac_pipeline_join.
 * fac_pipeline_join: makes `stream` wait for every enqueued batch except the
 * `keep` most recent ones (keep = 0: all; keep = 1: all but the last). */
int fac_forward_nhwc_u8_pipelined(fac_ctx* ctx, const uint8_t* d_in, int B, const int32_t* d_pos_index,
                                  float* d_logits, float* d_probs, float* d_score, void* stream);
int fac_pipeline_join(fac_ctx* ctx, int keep, void* stream);

/* Test/measurement entry points ------------------------------------------
 * fac_debug_features_u8: run conv1..conv{layer+1} (layer 0..16) on uint8
 * crops and copy that block's NHWC 16-bit output (after ReLU, and after the
 * MaxPool where one follows) to d_out.  For per-layer parity tests; layers
 * 0 and 1 always use the unfused conv1/conv2 kernels.
 * fac_profile_forward_u8: one forward with a hipEvent between stages;
 * synchronises and writes FAC_PROFILE_STAGES durations (ms): conv1..conv17,
 * patch embedding, transformer (6 layers), head.  With the fused 224 block
 * its whole time is stage conv1 and conv2/conv3 read 0.
 * fac_debug_conv: run stem conv `layer` (1..16 = conv2..conv17) alone on a
 * given NHWC 16-bit input.  fac_debug_tail: patch embedding + transformer +
 * head from a given NHWC 16-bit stem output [B,7,7,512].
 * fac_debug_gemm: one encoder GEMM out[M][N] = A[M][K] . W[N][K]^T (16-bit
 * row-major operands, fp32 accumulation) with epilogue `epi` (0 fp32 + bias,
 * 1 fp32 relu, 2 16-bit gelu, 3 fp32 residual +=, 4 split-K fp32 partial
 * slabs [splits][M][N], 5 16-bit + bias), tile `variant` (-1 default, 0..6):
 * the nn.Linear calls of cvit.py:28,39,50,164 in isolation. */
#define FAC_PROFILE_STAGES 20
int fac_debug_features_u8(fac_ctx* ctx, const uint8_t* d_in, int B, int layer, uint16_t* d_out, void* stream);
int fac_debug_conv(fac_ctx* ctx, int layer, const uint16_t* d_in, int B, uint16_t* d_out, void* stream);
int fac_debug_tail(fac_ctx* ctx, const uint16_t* d_stem, int B, const int32_t* d_pos_index, float* d_logits,
                   void* stream);
int fac_debug_gemm(fac_ctx* ctx, int epi, const uint16_t* d_a, const uint16_t* d_w, const float* d_bias, void* d_out,
                   int M, int N, int K, int splits, int variant, void* stream);
int fac_profile_forward_u8(fac_ctx* ctx, const uint8_t* d_in, int B, const int32_t* d_pos_index, float* d_logits,
                           float* stage_ms, int n_stages, void* stream);

/* Mean duration of the fused-stem launches recorded since option
 * "stem_events" was set (hipEvent pairs on the launching stream), and their
 * count; resets the record.  The bench's roofline for the stem kernel is
 * taken over its timed region with this. */
int fac_stem_event_ms(fac_ctx* ctx, float* avg_ms, int* n_launches);

/* pos_index outside [0,32): the device clamps it (the kernel cannot return
 * an error) and raises a host-visible flag; the context's NEXT forward call
 * (fac_forward_*, fac_forward_features, pipelined) then returns FAC_ERR_ARG
 * before enqueueing anything and clears the flag; fac_last_error names the
 * offending forward by its encoder-launch number on the context (one per
 * batch; a graph replay reports the number of its capture).  fac_check_device_errors
 * reads (and clears) the flag after synchronising the device: 0, or the call
 * number (>= 1) of a forward since the last check that saw such an index.  Not for use inside graph
 * capture (a captured forward's flag is seen by the first eager call after
 * the replay completes). */
int fac_check_device_errors(fac_ctx* ctx, int* flags);

/* Video-level score over n logit pairs (pred_sig + pre_process_prediction,
 * cvit_prediction.py:240,258-281): d_score = fp32 scalar. */
int fac_video_score(const float* d_logits, int n, float* d_score, void* stream);

/* The same score for nv videos whose crops were scored in one batch:
 * video v owns logit rows [d_seg[v], d_seg[v+1]) (int32 [nv+1], device,
 * non-decreasing); d_scores = fp32 [nv].  Each score is bit-identical to
 * fac_video_score on that video's rows alone (same sigmoid, same fp32 sums in
 * crop order).  Replaces predict_on_video's one-video-at-a-time loop
 * (cvit_prediction.py:73-83) with batched forwards. */
int fac_video_score_seg(const float* d_logits, const int* d_seg, int nv, float* d_scores, void* stream);

/* Face crops of config 3 (cvit_prediction.py:111-116): for each box
 * (frame, left, top, right, bottom) in d_boxes (int32 [n_boxes][5]), take
 * frame[top:bottom, left:right] of the BGR uint8 frames [n_frames][H][W][3],
 * area-resize it to 224x224 (cv2.INTER_AREA's area weights, evaluated in
 * exact integer arithmetic, round half up) and swap BGR -> RGB (the
 * cvtColor of :115) into d_crops [n_boxes][224][224][3]: the input of
 * fac_forward_nhwc_u8.  Boxes are clipped to the frame; empty boxes give 0. */
int fac_crop_resize_u8(const uint8_t* d_frames, int n_frames, int H, int W, const int32_t* d_boxes, int n_boxes,
                       uint8_t* d_crops, void* stream);

/* Tuning knob: run the conv stem in sub-batches of `crops` crops (0 = whole
 * batch), so intermediate activations stay resident in the Infinity Cache. */
int fac_set_stem_chunk(fac_ctx* ctx, int crops);

/* Named knobs: "stem_chunk" (as above), "fuse_stem224" (1 = conv1..conv3 +
 * pool as one fused kernel, the default; 0 = one kernel per conv),
 * "gemm_patch" / "gemm_qkv" / "gemm_out" / "gemm_ff1" / "gemm_ff2" /
 * "gemm_head" (GEMM tile variant 0..6 per call site; -1, the default, picks
 * by shape: 64x32 at <= 64 rows, 64x128 above 1024 rows, in the pipelined
 * forward's encoder and for the patch GEMM, else 32x128), "proj_splits" (split-K
 * of to_out and FF2: 1, 2 or 4), "tail_only" (before fac_load_weights: no
 * conv stem, fac_forward_features only), "tail_priority", "stem_events" (1 =
 * time every fused-stem launch, fac_stem_event_ms), "stem_nwg" (persistent
 * fused-stem workgroups; 0 = one per CU, the default), "ffn_ln_eps_exp" (n:
 * the FeedForward PreNorm LayerNorm uses eps = 10^-n; default 5, the RepBn8
 * variant's LinearNorm is 6, cvit_GGCA_ADD_DEConv_RepBn8.py:48),
 * "graph_max_b" (forwards of B <= n crops replay a captured hipGraph, see
 * fac_forward_nhwc_u8; default 32, 0 = always eager), "conv_small" (1 = the
 * 28x28 / 14x14 convs run on half-width output-channel blocks when the
 * default grid would leave CUs idle, i.e. few crops; the default; 0 = never;
 * bit-identical outputs), "conv_small14" (1 = with conv_small, the 14x14 convs
 * on 32-channel blocks while that grid fits one workgroup per CU, i.e. <= 16
 * crops; the default; 0 = the 64-channel blocks only; bit-identical).
 * Process-wide knobs of the fac_ops.h layer kernels (A/B measurements; any
 * context sets them; every fac_set_option call makes every context recapture
 * its small-batch graphs before their next replay): "conv_ring9" (0..7, bit mask of
 * the conv kernels that take a 9-slice weight ring when the grid is at most 2
 * workgroups per CU, i.e. few crops: bits 0 and 1 the two 9-slice variants
 * of the 14x14 BN-64 tile (bit 1 wins), bit 2 the 28x28 conv3x3_db register
 * ring; default 6; 0 = never; bit-identical outputs), "gemm_small" (the GEMM tile
 * variant 0..6 of calls with <= 64 rows, i.e. forwards of <= 32 crops; default
 * 5, a 64x32 tile; -1 = the wide tiles; every variant gives bit-identical
 * results), "nd_pt_wide" (n >= 0: convnd_pt
 * also takes uniform-tap convs whose cout is not a multiple of 128, and
 * fac_conv_nd_split's column segments, from n 256-row tiles on; default 32,
 * 0 = convnd_igemm), "nd_occ3" (convnd_igemm's 3-per-CU 2-slot 128x64 tile
 * for cout <= 64 up to n K steps; default 4, 0 = K <= 128 only), "pool_roll" (MaxPool3d(3,1,1) on 7-wide maps by
 * maxpool3_roll: 1 = every frame in one thread, the default; k >= 2 = k frames
 * per thread; 0 = maxpool3_s1), "pool3_zg" (output frames per thread of
 * maxpool3_s1, 0 = all, the default), "pool_win" (1 = the (1,3,3) / (3,3,3) /
 * (2,2,2) max pools by the compile-time-window kernel, the default; 0 =
 * pool_nd); every setting gives bit-identical max pools.  Round 6:
 * "pool_lds14" (1 = MaxPool3d(3,1,1) on 14x14 maps by maxpool3_lds14, the
 * default; 0 = maxpool3_s1), "pool3_g" (frames per maxpool3_pw unit on 7x7
 * maps when the pool is fused into the branch-3 1x1 conv: 0 = the default 2,
 * 1, 2 or 4), "pw_res" (1 = ResNet-50's K 128 / 256 conv3 + identity, layer1's
 * conv3 + downsample and S3D's merged K 192 / 256 heads on pw_res, layer2's
 * conv3 + strided downsample on pw_dual2, the default; 2 = pw_res only; 0 =
 * convnd_pt / conv_pw), "tk_wreg" (1 = S3D's cin-128 / 192 (3,1,1) temporal
 * convs with the weights in VGPRs, the default; 0 = in LDS; bit-identical). */
int fac_set_option(fac_ctx* ctx, const char* key, int value);

const char* fac_last_error(fac_ctx* ctx);
void fac_destroy(fac_ctx* ctx);

/* Library version / build string (for logs). */
const char* fac_version(void);

#ifdef __cplusplus
}
#endif

#endif /* FAC_CVIT_H */

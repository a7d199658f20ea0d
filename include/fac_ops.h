/* fac_ops.h — C ABI of the layer-level gfx950 kernels behind the §8f model
 * families: ResVitKan (config 5) and S3D (config 4).
 *
 * The CViT path has one fused entry point per forward (fac_cvit.h); the
 * ResNet-50 stem of ResVitKan and the Inception-3D blocks of S3D are
 * sequences of ordinary layers, orchestrated by their Python mirrors
 * (fac_fake_amd/resvitkan.py, fac_fake_amd/s3d.py) and captured into one
 * hipGraph per forward.  Every entry point is stream-ordered, takes device
 * pointers and plain sizes, returns 0 or a negative fac_status
 * (fac_cvit.h) and never throws.
 *
 * Activations are 16-bit (bf16 or fp16, `dtype` as in fac_cvit.h)
 * channels-last N·D·H·W·C tensors, C a multiple of 8 (inputs with 3
 * channels are packed to 8 by fac_pack_input).  2-D layers are D = 1.
 */
#ifndef FAC_OPS_H
#define FAC_OPS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Epilogue flags of fac_conv_nd. */
#define FAC_CONV_RELU 1      /* v = max(acc + bias, 0) */
#define FAC_CONV_RESID 2     /* v = v + residual[m][r_off + c] (16-bit) */
#define FAC_CONV_RELU2 4     /* v = max(v, 0) after the residual */
#define FAC_CONV_OUT_F32 8   /* fp32 output instead of 16-bit */
#define FAC_CONV_MAXPOOL3S2 16 /* then MaxPool2d(3, 2, 1) over H, W: out is
                                [n][od][oh/2][ow/2][ldo]; only with
                                FAC_CONV_RELU alone, on the space-to-depth
                                first conv below (ResNet-50's conv1 + bn1 +
                                relu + maxpool, ResVitKan.py:187/205);
                                FAC_ERR_ARG otherwise */
#define FAC_CONV_PREPOOL3S2 64 /* MaxPool3d((1,3,3), (1,2,2), (0,1,1)) over the
                                INPUT first, then the conv: a 1x1x1 conv,
                                cin = cout = 64, input width 56 (rows of
                                28 pooled positions); desc->d/h/w are the
                                unpooled input's, od/oh/ow the pooled
                                output's; flags FAC_CONV_RELU at most besides
                                this one; FAC_ERR_ARG otherwise.  S3D's
                                base.1 + base.2 (model.py:19-20) without
                                the pooled map in memory */
#define FAC_CONV_MAXPOOL3S1 32 /* MaxPool3d(3, 1, 1) over the INPUT first
                                (-inf padding), then the conv: a 1x1x1 conv
                                (stride 1, no padding) over an S x S map,
                                S in {14, 7, 3}, cout % 32 == 0, ldo and
                                c_off % 8 == 0, flags FAC_CONV_RELU at most
                                besides this one; FAC_ERR_ARG otherwise.
                                S3D's Inception branch3 (MaxPool3d +
                                BasicConv3d(cin, cout, 1), model.py:84-342)
                                without the pooled map in memory */

/* One N-d convolution (Conv2d / Conv3d, any kernel, stride, zero padding,
 * dilation 1, groups 1) with folded BatchNorm, as an implicit GEMM on MFMA:
 * rows = output positions (n, z, y, x), columns = output channels,
 * k = (tap, input channel).
 *
 * Replaces nn.Conv2d + nn.BatchNorm2d(eval) (+ nn.ReLU, + the residual add
 * of a ResNet Bottleneck) — CViT-main/ResVitKan/ResVitKan.py:124-152,
 * :187-200, :232-240 — and nn.Conv3d + BatchNorm3d(eval) + ReLU of S3D's
 * BasicConv3d / SepConv3d — sx_exp_deepfakedetect-master/S3D/model.py:50-82.
 *
 * weight: 16-bit [cout_pad][k_pad], row o = output channel, k index =
 *   ((tz*kh + ty)*kw + tx)*cin + c, zero beyond taps*cin; cout_pad a
 *   multiple of 128, k_pad a multiple of 64 (fac_conv_weight_layout).
 * bias: fp32 [cout_pad] (BN shift folded in), or NULL for none (every
 *   routed kernel honours NULL).
 * out: row m = ((n*Do + z)*Ho + y)*Wo + x, element [m*ldo + c_off + c];
 *   c_off lets Inception branches write straight into their concat slot.
 * residual (FAC_CONV_RESID): 16-bit [m*ldr + r_off + c].
 * Shapes with a dedicated kernel are routed to it inside this call (same
 * contract): the 4x4/1 16->64 conv over space-to-depth cells (conv_s2d4:
 * ResNet-50's / S3D's first conv) and temporal (kd,1,1) convs with 8 output
 * frames, cin % 64 == 0, cout % 64 == 0 (conv_tk), and
 * stride-1 1x1 convs with cin 64, 128 or 256, cout % 64 == 0, no fp32
 * output (conv_pw: ResNet-50's K <= 256 bottleneck 1x1s), of which the
 * residual ones with cin 128 (cout % 256 == 0) or 256 (cout % 128 == 0) take
 * pw_res (ResNet-50 layer2 / layer3 conv3 + identity; fac_set_option
 * "pw_res" 0 routes them to the generic kernel for A/B), and 1x1 residual
 * convs with cin 512, cout % 256 == 0 (layer4's conv3 + identity) take
 * pw_res2 (weights in VGPRs; "pw_res" 2 or 0 routes them to convnd_pt). */
typedef struct fac_conv_desc {
  int dtype;
  const void* in;
  int n, d, h, w, cin;          /* input dims; cin % 8 == 0 */
  const void* weight;
  const float* bias;
  int cout, k_pad;              /* k_pad: weight row length (elements) */
  int kd, kh, kw;               /* kernel */
  int sd, sh, sw;               /* stride */
  int pd, ph, pw;               /* zero padding */
  int od, oh, ow;               /* output dims (floor mode) */
  void* out;
  int ldo, c_off;
  const void* residual;
  int ldr, r_off;
  int flags;
} fac_conv_desc;

int fac_conv_nd(const fac_conv_desc* desc, void* stream);

/* fac_conv_nd whose output columns go to three tensors: [0, split1) to
 * desc->out (ldo, c_off), [split1, split2) to out1 (row stride ldo1, from
 * column 0), [split2, cout) to out2 (ldo2).  For convs that share an input,
 * e.g. the three 1x1x1 heads of an S3D Inception block (model.py:84-342:
 * branch0, branch1.0, branch2.0) as one GEMM over concatenated weights:
 * every output column is computed exactly as by its own launch.  Splits are
 * multiples of 8; no residual, no fp32 output. */
int fac_conv_nd_split(const fac_conv_desc* desc, void* out1, int ldo1, int split1, void* out2, int ldo2, int split2,
                      void* stream);

/* relu(conv(desc) + bias, if desc->flags has FAC_CONV_RELU) + conv(ds) +
 * ds bias, then ReLU if desc->flags has FAC_CONV_RELU2: a ResNet bottleneck's
 * conv3 + bn3 (+ReLU, ResVitKan.py:146-152) with its downsample branch
 * (conv + bn, ResVitKan.py:150) added in the same launch, so the downsample
 * output never goes through memory.  Both convs: cin % 64 == 0, the same
 * output positions [n, od, oh, ow] and cout (% 128 == 0); ds->out is ignored
 * and ds->flags must be 0; no FAC_CONV_RESID / FAC_CONV_OUT_F32 on desc.
 * Replaces fac_conv_nd(ds) + fac_conv_nd(desc with residual = its output).
 * Layer1's 64 -> 256 pair with a stride-1 1x1 downsample runs on pw_res
 * DUAL (both weight blocks resident in LDS), layer2's 128 -> 512 and
 * layer3's 256 -> 1024 conv3 with the stride-2 256 -> 512 / 512 -> 1024
 * downsample (cout % 256 == 0) on pw_dual2 (both weight blocks in VGPRs;
 * fac_set_option "pw_res" 2
 * routes it to convnd_pt for A/B, 0 routes both), the others on convnd_pt
 * DUAL. */
int fac_conv_nd_dual(const fac_conv_desc* desc, const fac_conv_desc* ds, void* stream);

/* A ResNet-50 layer1 / layer2 bottleneck's conv3 and the next block's conv1
 * in one launch (ResVitKan.py:146-152; torchvision resnet50): c3 = the 1x1
 * 64 -> 256 (layer1) or 128 -> 512 (layer2) conv3 + bn3 with flags exactly
 * FAC_CONV_RELU | FAC_CONV_RESID | FAC_CONV_RELU2 (out = relu(relu(conv + b)
 * + residual), the block output, ldo = cout); c1 = the next block's 1x1
 * 256 -> 64 / 128 (layer1) or 512 -> 128 (layer2) conv1 + bn1 with
 * flags exactly FAC_CONV_RELU over the same positions: its input is c3's
 * output (c1->in is ignored), written to c1->out (ldo = cout).  Every
 * output is what fac_conv_nd(c3) then fac_conv_nd(c1) would produce up to
 * fp32 summation order; the 256-channel map is written once and not read
 * back.  FAC_ERR_ARG / FAC_ERR_SHAPE for anything else. */
int fac_bottleneck_pw2(const fac_conv_desc* c3, const fac_conv_desc* c1, void* stream);

/* S3D Mixed_3b's branch2 SepConv3d(16, 32, 3) (model.py:84-110) in one
 * launch: sdsc = the (1,3,3) conv 16 -> 32 (+ BN folded, FAC_CONV_RELU at
 * most) over desc->in = [n][8][14][14][16], tdsc = the (3,1,1) conv 32 -> 32
 * over its output (tdsc->in is ignored: the 32-channel map stays in LDS),
 * written to tdsc->out [m*ldo + c_off + c] (the block output's channel
 * slot).  Every output is what fac_conv_nd(sdsc) then fac_conv_nd(tdsc)
 * would produce up to fp32 summation order.  FAC_ERR_SHAPE for any other
 * shape. */
int fac_sep_tiny(const fac_conv_desc* sdsc, const fac_conv_desc* tdsc, void* stream);

/* S3D Mixed_3c's branch2 SepConv3d(32, 96, 3) (model.py:84-110) in one
 * launch: sdsc = the (1,3,3) conv 32 -> 96 over [n][8][14][14][32] with its
 * output channels zero-padded to 128 (cout 128: rows 96..127 zero weights
 * and bias, which this kernel skips), tdsc = the (3,1,1) conv over those 128
 * channels (cin 128) -> 96, written to tdsc->out [m*ldo + c_off + c]; the
 * middle map stays in LDS.  Every output is what fac_conv_nd(sdsc) then
 * fac_conv_nd(tdsc) would produce up to fp32 summation order.
 * FAC_ERR_SHAPE for any other shape. */
int fac_sep_mid(const fac_conv_desc* sdsc, const fac_conv_desc* tdsc, void* stream);

/* Weight packing geometry for fac_conv_nd: *cout_pad = cout rounded up to
 * 128, *k_pad = taps*cin rounded up to 64. */
int fac_conv_weight_layout(int cout, int cin, int kd, int kh, int kw, int* cout_pad, int* k_pad);

/* Max or average pooling, channels-last 16-bit (MaxPool2d/3d: padding is
 * -inf, i.e. ignored; AvgPool: count_include_pad=True, the PyTorch default).
 * mode 0 = max, 1 = avg.  out element [m*ldo + c_off + c].
 * Replaces nn.MaxPool2d(3, 2, 1) (ResVitKan.py:205), S3D's nn.MaxPool3d
 * layers and F.avg_pool3d (S3D/model.py:31-45). */
typedef struct fac_pool_desc {
  int dtype;
  const void* in;
  int n, d, h, w, c;
  int kd, kh, kw, sd, sh, sw, pd, ph, pw;
  int od, oh, ow;
  int mode;
  void* out;
  int ldo, c_off;
} fac_pool_desc;

int fac_pool_nd(const fac_pool_desc* desc, void* stream);

/* Input staging: 3-channel images -> 16-bit channels-last with c_pad
 * channels (zeros beyond 3): out[n][s][c] = (x / div - mean[c]) / std[c]
 * in fp32.  src_kind 0: uint8 [n][s][3] (face crops: div = 255 gives the
 * reference's x/255. then Normalize, cvit_prediction.py:214-215);
 * src_kind 1: fp32 planar [n][3][s] (an already normalised NCHW tensor, or
 * S3D's raw 0..255 NCTHW clip: div 1, mean 0, std 1).  s = spatial
 * positions per image; mean3/std3 may be NULL (0 / 1). */
int fac_pack_input(int dtype, const void* src, int src_kind, int n, int s, float div, const float* mean3,
                   const float* std3, void* out, int c_pad, void* stream);

/* Space-to-depth staging for a stride-2 first conv (ResNet-50's 7x7/2,
 * ResVitKan.py:187): [n][h/2 + pad_before + pad_after]^2 cells of 16
 * channels, cell (Y, X) channel ((dy*2 + dx)*4 + c) = normalised pixel
 * (2(Y - pad_before) + dy, 2(X - pad_before) + dx), channel c < 3 (zero
 * outside the image and for c = 3).  A 7x7/2 conv with padding 3 is then a
 * 4x4/1 conv without padding over this image (pad_before 2, pad_after 1),
 * with weights w'[o][ty][tx][(dy*2+dx)*4 + c] = w[o][c][2ty+dy-1][2tx+dx-1]:
 * K = 256 instead of 49 taps x 8 padded channels.  src_kind as in
 * fac_pack_input; with frames > 1 the fp32 source is a clip batch
 * [n][3][frames][h][w] (S3D's (1,7,7)/(1,2,2) first conv, model.py:18) and
 * the output [n][frames][cells][cells][16]. */
int fac_pack_input_s2d(int dtype, const void* src, int src_kind, int n, int frames, int h, int w, int pad_before,
                       int pad_after, float div, const float* mean3, const float* std3, void* out, void* stream);

/* fac_conv_nd over fac_pack_input_s2d(src_kind 1, div 1, no mean / std)'s
 * cells of the fp32 clip batch `clip` [n][3][frames][h][w], with the packing
 * folded into the conv's halo staging (S3D's base.0 spatial conv,
 * model.py:18): `desc` describes that conv exactly as fac_conv_nd would get
 * it (cells [n][frames][h/2+pad_before+pad_after]^2[16], the 4x4/1 cout-64
 * s2d kernel, flags 0 or FAC_CONV_RELU); desc->in is not read.  The output
 * is bit-identical to fac_pack_input_s2d + fac_conv_nd. */
int fac_conv_s2d4_clip(const fac_conv_desc* desc, const float* clip, int h, int w, int pad_before, void* stream);

/* fac_conv_s2d4_clip over a uint8 clip batch [n][3][frames][h][w] (decoded
 * video frames, S3D-test.py:94-96's 0..255 values before the float cast): the
 * same output as fac_conv_s2d4_clip on that clip cast to fp32, a quarter of
 * the input bytes.  Round-4 addition, no reference counterpart. */
int fac_conv_s2d4_clip_u8(const fac_conv_desc* desc, const uint8_t* clip, int h, int w, int pad_before,
                          void* stream);

/* S3D's base.0 (SepConv3d(3, 64, k 7, s 2, p 3), model.py:18,63-82) in one
 * launch from a uint8 clip batch [n][3][16][h][w] with h / 2 = w / 2 = 56
 * (the 112 x 112 clips of S3D-test.py): `sdesc` is the spatial half as
 * fac_conv_s2d4_clip_u8 takes it (the space-to-depth 4x4 conv, cout 64),
 * `tdesc` the temporal (7,1,1)/(2,1,1) conv (64 -> 64, 16 -> 8 frames, its
 * `in` unused) whose `out` receives [n][8][56][56][64].  The 16-frame
 * half-resolution map between the two never goes through HBM; the output is
 * bit-identical to fac_conv_s2d4_clip_u8 followed by fac_conv_nd(tdesc). */
int fac_s3d_base0_u8(const fac_conv_desc* sdesc, const fac_conv_desc* tdesc, const uint8_t* clip, int h, int w,
                     int pad_before, void* stream);

/* KANLinear forward (CViT-main/ResVitKan/kan.py:189-206), fp32:
 *   y = silu(x) · base_weightᵀ + b_splines(x) · (spline_weight ⊙ spline_scaler)ᵀ
 * with order-3 B-spline bases over the per-feature knot vector `grid`
 * [in][n_knots] (kan.py:90-132, the Cox–de Boor recursion in the
 * reference's operation order).  `wcat` is the fused weight, k-major
 * [in][1 + nb][out] (index 0 = base_weight[o][i], 1.. = the scaled spline
 * weights spline_weight[o][i][k] * spline_scaler[o][i], nb = n_knots - 4).
 * x [rows][in] fp32 -> y [rows][out] fp32.  `partial` is a scratch buffer of
 * fac_kan_scratch_bytes() bytes. */
int fac_kan_linear(const float* x, int rows, int in_f, int out_f, const float* grid, int n_knots, const float* wcat,
                   float* y, void* partial, void* stream);
size_t fac_kan_scratch_bytes(int rows, int in_f, int out_f);

/* GGCA(c, h, w, reduction 16, groups) of the CViT RepBn8 variant fused with
 * its x = x * GGCA(x) — CViT-main/model/cvit_GGCA_ADD_DEConv_RepBn8.py:144-207,
 * :436-437 — on 16-bit channels-last features x [n][h][w][c]:
 *   att_h[y][c] = sigmoid(z(mean_x x) + z(max_x x)), att_w likewise over y,
 *   z = shared_conv: 1x1 (c/groups -> c/groups/16) + BatchNorm(eval, eps
 *   1e-5) + ReLU + 1x1 back, applied per channel group;
 *   out = x * ((x * att_h) * att_w), fp32 arithmetic, 16-bit out.
 * w1 [cr][cg], b1 [cr], bn4 [4][cr] = running_mean, running_var, weight,
 * bias; w2 [cg][cr], b2 [cg] (fp32; cg = c/groups, cr = cg/16).
 * h, w <= 16, cg a multiple of 16, h*w*cg <= 16384. */
int fac_ggca(int dtype, const void* x, int n, int h, int w, int c, int groups, const float* w1, const float* b1,
             const float* bn4, const float* w2, const float* b2, void* out, void* stream);

/* The CViT conv-stack kernels as layers (fac_cvit.h runs them inside its
 * fused forward; the CViT variants of the reference stack them differently —
 * the RepBn8 variant, SURVEY §8f-4, whose DEConv blocks fold into plain 3x3
 * convs, fac_fake_amd/repbn8.py).  Activations 16-bit NHWC.
 *
 * fac_conv3x3: Conv2d(3x3, stride 1, padding 1) + folded BN (+ ReLU if relu)
 * (+ MaxPool2d(2,2) if pool) — cvit.py:86-148 — on the halo-staged implicit
 * GEMM of conv.hip: in [n][h][h][cin] -> out [n][h'][h'][cout] (h' = h/2 with
 * pool); h in {112, 56, 28, 14} (224: cout 32, the unfused kernel), cin a
 * multiple of 32, cout a multiple of one of the resolution's blocks (64 at
 * 112; 128 or 64 at 56; 256, 192 or 128 at 28; 128 at 14 — the largest that
 * divides cout is used).  wpk: fac_conv3x3_pack of the folded fp32 weight
 * [cout][cin][3][3]; bias fp32 [cout]; zero256: 256 zero bytes of device
 * memory (the source of zero-padding loads).
 * fac_conv3x3_packed_elems: 16-bit elements of the packed weight (0: shape
 * not supported).  Packing runs on the host (host pointers). */
size_t fac_conv3x3_packed_elems(int h, int cin, int cout);
int fac_conv3x3_pack(int dtype, int h, int cin, int cout, const float* w, uint16_t* out);
int fac_conv3x3(int dtype, const void* in, const void* wpk, const float* bias, void* out, int n, int h, int cin,
                int cout, int pool, int relu, const void* zero256, void* stream);

/* The fused 224x224 block (stem224.hip): input normalisation, conv 3->32,
 * conv 32->32, conv 32->32 (each + folded BN + ReLU), MaxPool2d(2,2) ->
 * [n][112][112][32].  u8: uint8 NHWC crops [n][224][224][3] (x/255 and
 * Normalize fused); else normalised fp32 NCHW [n][3][224][224].  w1p:
 * fac_stem224_pack_conv1 of the folded [32][3][3][3] conv-1 weight (host ->
 * host, 32 x 64 16-bit); w2, w3: fac_conv3x3_pack with h = 224. */
int fac_stem224_pack_conv1(int dtype, const float* w, uint16_t* out);
int fac_stem224(int dtype, int u8, const void* in, const void* w1p, const float* b1, const void* w2, const float* b2,
                const void* w3, const float* b3, void* out, int n, void* stream);

/* Row-wise sigmoid of logits (the per-logit pred_sig of the heads). */
int fac_sigmoid(const float* x, float* y, int n, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* FAC_OPS_H */

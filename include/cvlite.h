/*
 * cvlite — C ABI of the MI355X (gfx950) detector-training hot path.
 *
 * Drop-in boundary for the numeric work that WD-Leong/CV-Lite-Object-Detection does in
 * TF2-eager ops and numpy loops (the reference has no FFI of its own).  Each entry
 * point below names the reference function it replaces.  The Python host layer
 * (cv-lite-object-detection_amd/cvlite) binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (all functions):
 *  - every pointer is a DEVICE pointer unless the parameter says "host";
 *  - the caller allocates every buffer, including workspaces (query *_workspace_size first);
 *    the library allocates nothing and keeps no pointer past return;
 *  - all work is enqueued on `stream` (a hipStream_t); nothing synchronises;
 *  - return value: CVL_OK, CVL_EINVAL (bad argument; nothing enqueued) or CVL_EHIP + hipError_t;
 *  - stateless and re-entrant; safe to capture into a hipGraph.
 *  - tensors are row-major; activations NHWC; "bf16" = raw uint16 bfloat16 bits.
 */
#ifndef CVLITE_H_
#define CVLITE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* cvl_stream_t; /* hipStream_t */

enum { CVL_OK = 0, CVL_EINVAL = 1, CVL_EHIP = 1000 };

int cvl_version(void);

/* ------------------------------------------------------------------------------------------
 * FCOS target assignment.  Replaces FCOS/fcos.py:136-378 `format_data` (per image, numpy loops)
 * with one batched launch.  boxes[b, i] = (yc, xc, h, w, class) normalised to img_dim[b] (the
 * unpadded size, fp32, as data_preprocess.resize_and_pad_image returns it); only the first
 * nbox[b] rows of image b are used.  Output targets[b, p, 0:5+C] float32, p running level-major
 * over the 5 maps of size (pad_h/stride_l) x (pad_w/stride_l) (row-major inside a level); this is
 * the reference's list of 5 float64 maps rounded to fp32 (bit-exact).  num_targets[b, l] int32.
 * strides[5], size_bounds[4] are host arrays (reference defaults {8,16,32,64,128}, {32,64,128,256}).
 * ---------------------------------------------------------------------------------------- */
int cvl_fcos_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                    int pad_h, int pad_w, int num_classes, const int32_t* strides /*host[5]*/,
                    const float* size_bounds /*host[4]*/, float* targets, int32_t* num_targets,
                    cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Fused FCOS loss forward + backward.  Replaces FCOS/fcos.py:380-496 (`focal_loss`,
 * `smooth_l1_loss`, `iou_loss`, `model_loss`; alpha 0.25, gamma 2, plain sums) and the matching
 * GradientTape backward.  Per cell p of image b:
 *   reg_pred[(b*P+p)*ld_reg + 0..4] = (t, b, l, r, centerness-logit)
 *   cls_pred[(b*P+p)*ld_cls + 0..C-1] = class logits
 *   targets[(b*P+p)*(5+C) + ...] as produced by cvl_fcos_assign.
 * losses[b*3 + {0,1,2}] = (cls, reg, cen) float32 sums for image b (model_loss's tuple).
 * If d_reg / d_cls are non-null, writes grad_scale * d(cls+reg+cen)/d(pred) with the same
 * strides (padding channels zeroed); *_dtype 0 = float32, 1 = bf16.
 * reg_type bits 0-1: 0 = "l1" (smooth-L1), 1 = "iou"; flags for the centre variants: +4 focal
 * centerness (fcos_center.py:386-389 cen_type="focal", fcos_center_v1.py:305-307), +8 smooth-L1 on
 * sigmoid(reg[:4]) (fcos_center_v1.py:115, l1 only), +16 the centerness logit / gradient is column
 * round_up(C, 8) of the class rows (cen_output_l lives on the cls tower).
 * `workspace` >= cvl_fcos_loss_workspace_size(B, P) bytes, passed as `workspace_bytes`
 * (CVL_EINVAL when smaller: the size grew in round 5 to 64-cell tiles, so a buffer sized by an
 * older formula is rejected instead of overrun).
 * ---------------------------------------------------------------------------------------- */
size_t cvl_fcos_loss_workspace_size(int B, int P);
int cvl_fcos_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                  const float* targets, int B, int P, int num_classes, int reg_type,
                  float grad_scale, float* losses, void* d_reg, int ld_dreg, int dreg_dtype,
                  void* d_cls, int ld_dcls, int dcls_dtype, void* workspace, size_t workspace_bytes,
                  cvl_stream_t stream);
/* cvl_fcos_loss with the loss keywords of FCOS/fcos.py:380 smooth_l1_loss(delta) and :443-444
 * focal_loss(alpha, gamma) (RetinaNet/retinanet_module.py:367-401 has the same two), and one more
 * reg_type flag: +32 the regression mask is the float value targets[5] itself instead of
 * (max class target >= 1) -- the drop-in smooth_l1_loss / iou_loss(mask=<float map>) (C = 1).
 * cvl_fcos_loss(...) == cvl_fcos_loss_ex(..., 0.25f, 2.0f, 1.0f, ...).  gamma >= 0, delta > 0. */
int cvl_fcos_loss_ex(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                     const float* targets, int B, int P, int num_classes, int reg_type,
                     float grad_scale, float alpha, float gamma, float delta, float* losses, void* d_reg,
                     int ld_dreg, int dreg_dtype, void* d_cls, int ld_dcls, int dcls_dtype, void* workspace,
                     size_t workspace_bytes, cvl_stream_t stream);

/* FCOS/fcos.py:112-134 prediction_to_corners: pred [S0][S1][ld>=4] (t, b, l, r) fp32 ->
 * out [S0][S1][4] float64 = stride * (y_lo, x_lo, y_hi, x_hi) around cell centres (fp32 math). */
int cvl_fcos_decode(const float* pred, int ld, int S0, int S1, double stride, double* out,
                    cvl_stream_t stream);
/* FCOS/fcos_center_v1.py:124-147 prediction_to_corners(xy_pred, box_sc, stride): pred [S0][S1][ld>=4]
 * (y_off, x_off, h, w) fp32 -> out [S0][S1][4] float64 corners of the box centred at
 * ((cell + off) * stride) with size (h, w) * box_sc (fp32 arithmetic, stored as float64). */
int cvl_fcos_v1_decode(const float* pred, int ld, int S0, int S1, float box_sc, float stride, double* out,
                       cvl_stream_t stream);


/* FCOS/fcos_center.py:149-317 format_data (the variant of train_fcos_center_voc.py): level by
 * max(h, w) px against b_dim [4] (HOST, reference default {32,64,128,256}); per level, boxes in
 * ascending area paint the 3x3 cells around int(centre * img_dim / stride + 0.5) (only the centre
 * cell when center_only): centerness = max(1 / 0.5 / 0.25), ltrb = last box's offsets about the
 * cell centre (unclamped), class bits OR-ed.  Layout as cvl_fcos_assign: targets [B][P][5+C]
 * level-major over (pad_h/stride) x (pad_w/stride) maps, num_targets [B][5]; strides [5] HOST. */
int cvl_fcos_center_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                           int pad_h, int pad_w, int num_classes, const int32_t* strides, const float* b_dim,
                           int center_only, float* targets, int32_t* num_targets, cvl_stream_t stream);
/* FCOS/fcos_center_v1.py:149-281 format_data (train_fcos_center_v1_voc.py): same level selection and
 * ascending-area order as cvl_fcos_center_assign; each box writes ONLY its centroid cell
 * (int(centre * img_dim / stride)): (y_off, x_off, h / box_sc, w / box_sc) of the last box there,
 * centre score 1, class bits OR-ed; box_sc = b_dim[l] (l < 4) or max(img_dim) (l = 4). */
int cvl_fcos_center_v1_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                              int pad_h, int pad_w, int num_classes, const int32_t* strides, const float* b_dim,
                              float* targets, int32_t* num_targets, cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Segmented implicit-GEMM convolution (bf16 MFMA, fp32 accumulate).  Replaces every Conv2D of
 * the reference graphs (Keras ResNet50 backbone; FCOS/fcos.py:49-101 FPN, towers and heads;
 * RetinaNet/retinanet_module.py:74-148) forward (mode FWD) and backward-input (mode DGRAD).
 * A "segment" is one feature map of B images: rows of image b live at source/destination rows
 * base + b*img_stride + (y*W + x), each row holding `Cin` (source) / `ld_dst` (dest) channels.
 * Several segments in one call share the forward geometry (kernel/stride/pad) but may each have
 * their own packed weights and bias: the five FPN levels through a shared tower, or the five
 * per-level heads, are one launch.
 * Weights: FWD  -> packed [Npad][KH*KW*Cin]   (cvl_pack_conv_weights w_fwd)
 *          DGRAD-> packed [Npad=Cin_pad][KH*KW*Cout_pad] (w_dgrad); then `Cin` = Cout_pad.
 * TF "same" padding: pad_t/pad_l = floor(total/2) (asymmetric for stride 2).
 * bn_stats (nullable) receives per-(image, out channel) (sum, sumsq) as BN accumulators (below;
 * zero it first), which requires H*W % 4 == 0.
 *
 * BN accumulators (cvl_bn_acc): the statistics many workgroups add into one (image, channel) --
 * (sum, sumsq) of a conv output, (sum g, sum g*xhat) of a BN backward.  Two modes, chosen for the
 * whole library by cvl_bn_set_exact() before any buffer is made (cvl_bn_acc_slots() = S reports it):
 *  - default (S = 1): one float64 per statistic, fp64 atomic adds of fp32 partials (the order of
 *    the adds can change the last bits of a sum);
 *  - exact (S = 8, cvl_bn_set_exact(1)): each fp32 partial is added as an integer into one of 7
 *    uint64 bins chosen by its exponent (bin k holds multiples of 2^(22k - 123); partials below
 *    2^-100 are dropped, slot 7 counts non-finite ones), so the result is bit-identical whatever
 *    order the atomics land in.  The value of a statistic is
 *    sum_k (double)(int64)slot[k] * 2^(22k - 123) over k = 0..6 in that order (NaN if slot[7] != 0).
 *    The consumers (cvl_bn_finalize[_apply], cvl_bn_backward_*_sums) first DECODE THE BUFFER IN
 *    PLACE -- slot 0 of each statistic becomes its float64 value and slot 7 the marker ~0 -- so each
 *    statistic is decoded once; a decoded buffer stays valid input for every reader.
 * Layout: uint64 [B][C][2][S] (zero it before the producer); cvl_bn_acc_decode writes the values of
 * n statistics as float64 [n] in either mode.
 * ---------------------------------------------------------------------------------------- */
#define CVL_BN_ACC_SLOTS 8          /* S of the exact mode */
int cvl_bn_set_exact(int on);
int cvl_bn_acc_slots(void);
int cvl_bn_acc_decode(const uint64_t* acc, double* out, int64_t n, cvl_stream_t stream);
#define CVL_CONV_MAX_SEG 10
enum { CVL_CONV_FWD = 0, CVL_CONV_DGRAD = 1 };

typedef struct {
  int Hr, Wr;          /* spatial size of the GEMM rows: FWD output map / DGRAD input map */
  int Hs, Ws;          /* spatial size of the gathered source: FWD input map / DGRAD dY map */
  int64_t src_base, src_img;  /* source row of image 0 and rows per image */
  int64_t dst_base, dst_img;  /* destination row of image 0 and rows per image */
  const void* w;       /* packed bf16 weights for this segment */
  const float* bias;   /* per output channel, or NULL */
} cvl_conv_seg;

typedef struct {
  int mode;            /* CVL_CONV_FWD / CVL_CONV_DGRAD */
  int B;               /* images per segment */
  int Cin;             /* channels of each gathered source row (multiple of 32) */
  int KH, KW, stride, pad_t, pad_l;   /* FORWARD conv geometry */
  int Npad;            /* GEMM columns = packed weight rows (multiple of 32) */
  int n_store;         /* columns written (<= Npad) */
  int ld_dst, dst_coff;/* destination row pitch and channel offset (elements) */
  int dst_f32;         /* 1: fp32 destination, 0: bf16 */
  int relu_out;        /* ReLU on the result */
  int relu_in;         /* ReLU on the gathered source values */
  float beta;          /* dst = result + beta * dst */
  int nseg;
  cvl_conv_seg seg[CVL_CONV_MAX_SEG];
  int prec;            /* CVL_PREC_BF16 (0): bf16 source / weights / destination (dst_f32 aside),
                          bf16 MFMA.  CVL_PREC_F32 (1): the fp32 parity mode -- fp32 source, fp32
                          packed weights (cvl_pack_item.f32_out), fp32 destination, fp32 FMA,
                          deterministic; bn_stats then needs nseg == 1 (cvl_conv_wgrad* take the
                          same field for x / dy). */
} cvl_conv_desc;
enum { CVL_PREC_BF16 = 0, CVL_PREC_F32 = 1 };

/* workspace (optional, >= cvl_conv_igemm_workspace_size(d) bytes) enables split-K for grids too
 * small to fill the GPU (fp32 partial slabs + a finishing pass); NULL = no split. */
size_t cvl_conv_igemm_workspace_size(const cvl_conv_desc* d);
int cvl_conv_igemm(const cvl_conv_desc* d, const void* src, void* dst, uint64_t* bn_stats,
                   void* workspace, size_t workspace_bytes, cvl_stream_t stream);
/* A data gradient through a ReLU (the TF gradient of the FCOS towers' final ReLU behind the heads,
 * FCOS/fcos.py:16-27, 76-101): dst = conv data gradient of src (mode CVL_CONV_DGRAD, prec bf16, beta 0,
 * no relu_out) masked by y > 0, y [rows][ld_dst] laid out as dst.  The tower kernel applies the mask
 * in its register epilogue; otherwise the plain launch is followed by cvl_relu_backward (then dst
 * must be dense: ld_dst == n_store, dst_coff 0).  Bit-identical to cvl_conv_igemm + cvl_relu_backward. */
int cvl_conv_igemm_relu_mask(const cvl_conv_desc* d, const void* src, void* dst, const void* y, void* workspace,
                             size_t workspace_bytes, cvl_stream_t stream);

/* Test / profiling hook: the kernel variant the last cvl_conv_igemm / cvl_conv_wgrad* call on THIS
 * host thread launched.  CVL_CK_* codes; cvl_conv_kernel_name(code) is a static string.  Codes 6
 * (X256) and 12 (X32H) belong to retired kernels and are no longer returned. */
enum { CVL_CK_NONE = 0, CVL_CK_BASE = 1, CVL_CK_BASE_SPLITK = 2, CVL_CK_L64 = 3, CVL_CK_L128 = 4,
       CVL_CK_L256 = 5, CVL_CK_X256 = 6, CVL_CK_X32 = 7,
       CVL_CK_WG_S = 8, CVL_CK_WG_L128 = 9, CVL_CK_WG_L256 = 10, CVL_CK_WG_X = 11, CVL_CK_X32H = 12, CVL_CK_WG_SN = 13,
       CVL_CK_H64 = 14, CVL_CK_WG_H = 15, CVL_CK_P = 16 };
int cvl_conv_igemm_last_kernel(void);
const char* cvl_conv_kernel_name(int code);

/* Measurement hook (no reference counterpart: bench.py's in-step roofline timing).  cvl_probe_arm
 * hands slot (uint64 x4 device buffer, zero it first) to the NEXT cvl_conv_igemm call: when that
 * call runs the tower kernel (cvl_conv_igemm_last_kernel() == CVL_CK_X32) the kernel times itself
 * (workgroup 0's start to the last workgroup's end): slot[1] += elapsed ticks, slot[2] += 1 (slot[0]
 * / slot[3]: start stamp / workgroup counter); any other kernel leaves the slot untouched.  The slot
 * travels in the launch arguments, so graph capture keeps it.  cvl_probe_clock_hz = ticks per
 * second of the GPU wall clock. */
int cvl_probe_arm(uint64_t* slot);
double cvl_probe_clock_hz(void);

/* Weight gradient (replaces Conv2DBackpropFilter + the per-image gradient accumulation of
 * FCOS/train_fcos.py:173-176): dw[KH][KW][Cin][n_store] (HWIO fp32) = beta*dw + sum over all
 * rows of all segments of im2col(x) * dy.  `d` is the FORWARD descriptor (its ld_dst/dst_coff
 * address dy; all segments must share one weight pointer).  workspace >= *_workspace_size(d). */
size_t cvl_conv_wgrad_workspace_size(const cvl_conv_desc* d);
int cvl_conv_wgrad(const cvl_conv_desc* d, const void* x, const void* dy, float* dw, float beta,
                   void* workspace, size_t workspace_bytes, cvl_stream_t stream);

/* Grouped weight gradient: the segments of `d` split into `ngroups` consecutive equal groups (each
 * sharing one weight pointer), group g summed into dw[g] (a HOST array of device pointers).  The
 * FCOS cls and reg tower layers (FCOS/fcos.py:16-27, 76-101: same geometry, own weights) are one
 * call with 10 segments and 2 groups.  workspace >= cvl_conv_wgrad_grouped_workspace_size(d, ngroups). */
/* Deferred split reductions of the weight gradients.  cvl_wgrad_defer(1): the split-M weight
 * gradients (cvl_conv_wgrad / _grouped) leave their fp32 slabs pending instead of reducing them into
 * dW at once; cvl_wgrad_flush reduces everything pending in ONE batched launch (deterministic, the
 * same arithmetic as the immediate form).  The caller keeps every pending call's workspace alive and
 * dW unread until the flush; cvl_wgrad_defer(0) flushes and turns deferral off.  A reduction or
 * unsplit write into a dW that is already pending flushes first. */
int cvl_wgrad_defer(int on, cvl_stream_t stream);
int cvl_wgrad_flush(cvl_stream_t stream);
size_t cvl_conv_wgrad_grouped_workspace_size(const cvl_conv_desc* d, int ngroups);
int cvl_conv_wgrad_grouped(const cvl_conv_desc* d, int ngroups, const void* x, const void* dy, float* const* dw,
                           float beta, void* workspace, size_t workspace_bytes, cvl_stream_t stream);

/* Batched weight gradients (round 6): the weight gradients of n independent convolutions, d / x /
 * dy / dw HOST arrays of n entries (dw pairwise distinct), each as cvl_conv_wgrad(d[i], x[i], dy[i],
 * dw[i], beta) would form it -- the per-image gradient accumulation of FCOS/train_fcos.py:173-176 for
 * every 1x1 and 3x3 conv of a ResNet stage at once.  The 1x1 bf16 single-segment problems (pad 0,
 * stride 1 or 2, dense rows) share ONE launch per <= 16 and tile width, the 3x3 stride-1 problems the
 * halo weight-gradient kernel takes ONE launch per <= 12 (each problem its own tile grid, a common
 * rows-per-workgroup chunk chosen for the whole launch), with their split reductions deferred as by
 * cvl_wgrad_defer; any other problem runs as its own cvl_conv_wgrad.  Sums are fixed-order
 * (deterministic); the chunking differs from the one-conv calls, so results agree with them to fp32
 * rounding, not bit for bit.  workspace >= cvl_conv_wgrad_batch_workspace_size(d, n). */
size_t cvl_conv_wgrad_batch_workspace_size(const cvl_conv_desc* const* d, int n);
int cvl_conv_wgrad_batch(const cvl_conv_desc* const* d, int n, const void* const* x, const void* const* dy,
                         float* const* dw, float beta, void* workspace, size_t workspace_bytes, cvl_stream_t stream);

/* fp32 HWIO [KH][KW][Cin][Cout] master weights -> bf16 forward pack [Npad][KH*KW*Cin_k]
 * (zero rows >= Cout and channels >= Cin) and/or dgrad pack [Cin_pad][KH*KW*Cout_pad]. */
int cvl_pack_conv_weights(const float* w_hwio, int KH, int KW, int Cin, int Cout, int Cin_k, int Npad,
                          void* w_fwd, int Cin_pad, int Cout_pad, void* w_dgrad, cvl_stream_t stream);

/* Batched form of cvl_pack_conv_weights: every conv of a network in ONE launch (run after each
 * optimizer step).  items: DEVICE array of cvl_pack_item; tiles: DEVICE int32 [ntiles][4] =
 * (item, tap, ci0, co0), one per 64x64 (Cin x Cout) block of each tap, covering ci < max(Cin_k,
 * Cin_pad) and co < max(Npad, Cout_pad) (multiples of 64 from 0).  Cin_k, Cin_pad, Cout_pad % 8 == 0. */
typedef struct {
  const float* w;      /* HWIO fp32 master [KH*KW][Cin][Cout] */
  void* w_fwd;         /* bf16 [Npad][KHW*Cin_k] or NULL */
  void* w_dgrad;       /* bf16 [Cin_pad][KHW*Cout_pad] or NULL */
  int KHW, Cin, Cout, Cin_k, Npad, Cin_pad, Cout_pad;
  int f32_out;         /* 1: w_fwd / w_dgrad are fp32 (the CVL_PREC_F32 parity mode; any Cin_k) */
} cvl_pack_item;
int cvl_pack_conv_weights_multi(const cvl_pack_item* items, const int32_t* tiles, int ntiles,
                                cvl_stream_t stream);

/* ResNet stem straight from the image (Keras ResNet50 conv1: ZeroPadding2D(3) + Conv2D(64, 7,
 * strides=2) + bias, behind FCOS/fcos.py:30-46 and RetinaNet/retinanet_module.py:39-72; no im2col
 * matrix in HBM).  img fp32 NHWC [B][H][W][3]; Ho = (H-1)/2+1, Wo = (W-1)/2+1.  K order k = ky*24 +
 * kx*3 + c (each kernel row's 21 taps x channels padded to 24): w_packed = cvl_pack_conv_weights of
 * the HWIO [7][7][3][64] kernel viewed as KH=7, KW=1, Cin=21, Cin_k=24, Npad=64 ([64][168] bf16).
 * Forward: z [B][Ho][Wo][64] bf16 = bf16(conv(bf16(img)) + bias), bn_stats (nullable) = the BN
 * accumulators of z.  Weight gradient: dw [192][64] fp32 = beta*dw + sum over pixels, rows in the
 * same padded K order (HWIO row ky*21+kx*3+c = dw row ky*24+kx*3+c; pad rows 0); deterministic. */
int cvl_stem_conv7x7s2(const float* img, int B, int H, int W, const void* w_packed, const float* bias, void* z,
                       uint64_t* bn_stats, cvl_stream_t stream);
size_t cvl_stem_wgrad_workspace_size(int B, int H, int W);
int cvl_stem_wgrad(const float* img, int B, int H, int W, const void* dz, float* dw, float beta, void* workspace,
                   size_t workspace_bytes, cvl_stream_t stream);

/* fp32 NHWC image -> bf16 im2col rows [B*Ho*Wo][Kp] (ResNet50 conv1 after ZeroPadding2D(3)). */
int cvl_im2col(const float* x, int B, int H, int W, int C, int KH, int KW, int stride, int pad_t,
               int pad_l, int Ho, int Wo, int Kp, void* out, cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * BatchNormalization in training mode with per-image statistics (the reference forwards one
 * image at a time, train_fcos.py:137-153; Keras eps 1.001e-5, momentum 0.99, running variance
 * unbiased as TF's fused kernel).  stats: BN accumulators [B][C][2][S] from cvl_conv_igemm(bn_stats)
 * or cvl_bn_stats; mean_rstd [B][C][2].
 * ---------------------------------------------------------------------------------------- */
int cvl_bn_finalize(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var, int B,
                    int C, int HW, float eps, float momentum, cvl_stream_t stream);
int cvl_bn_apply(const void* z, const float* mean_rstd, const float* gamma, const float* beta,
                 const void* residual, void* y, int B, int HW, int C, int relu, cvl_stream_t stream);
/* cvl_bn_finalize + cvl_bn_apply in ONE launch (bit-identical results): every block derives the
 * (mean, rstd) of its image from stats; mean_rstd is still written for the backward and the running
 * statistics advanced (run_mean/run_var NULL together: inference-style, no EMA). */
int cvl_bn_finalize_apply(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                          const void* z, const float* gamma, const float* beta, const void* residual, void* y,
                          int B, int HW, int C, int relu, float eps, float momentum, cvl_stream_t stream);
/* cvl_bn_finalize_apply whose residual is ANOTHER BN's output that was never stored: the projection
 * shortcut of a Keras ResNet block1, y = act(BN_3(z) + BN_0(res_z)).  Both finalizes run in the one
 * launch (res_mean_rstd written, res running statistics advanced with res_eps / res_momentum), and the
 * residual term is bf16(BN_0(res_z)) rounded as the stored shortcut output was: bit-identical to
 * cvl_bn_finalize_apply(res) + cvl_bn_finalize_apply(z, residual) without writing or re-reading it.
 * Replaces the shortcut's apply of resnet.py block1 (Keras applications, behind FCOS/fcos.py:30-35). */
int cvl_bn_finalize_apply_bnres(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                                const void* z, const float* gamma, const float* beta, uint64_t* res_stats,
                                float* res_mean_rstd, float* res_run_mean, float* res_run_var,
                                const void* res_z, const float* res_gamma, const float* res_beta,
                                float res_eps, float res_momentum, void* y, int B, int HW, int C, int relu,
                                float eps, float momentum, cvl_stream_t stream);
/* dy: grad of y; y_relu: y when the unit ends in ReLU (mask), else NULL; writes dz (bf16),
 * optionally g_out = masked dy (the residual branch's gradient), dgamma/dbeta (= + beta_acc*old)
 * and, if conv_dbias != NULL, the gradient of the preceding conv's bias, which is exactly 0
 * behind training-mode BN (the per-image mean subtraction cancels any constant shift of z).  workspace >= cvl_bn_backward_workspace_size(B, HW, C) bytes; reductions are
 * deterministic (per-block partials summed in a fixed order, no atomics). */
size_t cvl_bn_backward_workspace_size(int B, int HW, int C);
int cvl_bn_backward(const void* dy, const void* y_relu, const void* z, const float* mean_rstd,
                    const float* gamma, void* workspace, size_t workspace_bytes, void* dz, void* g_out,
                    float* dgamma, float* dbeta, float beta_acc, float* conv_dbias, int B, int HW, int C,
                    cvl_stream_t stream);
/* cvl_bn_backward for a unit that ends in ReLU WITHOUT a residual add (the conv1/conv2 units of a
 * Keras ResNet bottleneck, the stem): the ReLU mask is recomputed from z as
 * fma(gamma, (z - mean) * rstd, beta) > 0 -- the forward's own arithmetic (cvl_bn_apply) -- so y
 * is not read (two passes read 2 tensors instead of 3).  beta = the BN's beta parameter. */
int cvl_bn_backward_relu(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                         const float* beta, void* workspace, size_t workspace_bytes, void* dz, float* dgamma,
                         float* dbeta, float beta_acc, float* conv_dbias, int B, int HW, int C,
                         cvl_stream_t stream);
/* Fused BN-backward first pass.  cvl_conv_igemm_dgrad_bnsum runs a DGRAD conv (beta 0) whose
 * result is dy of a BN -> ReLU (act_hi = INFINITY) / ReLU6 (act_hi = 6) unit without a residual
 * (the bottleneck's conv1 / conv2 units: their dy has one producer) and, when the 256-row
 * LDS-DMA kernel takes the launch with one image per tile, adds per (image, channel)
 * (sum g, sum g*xhat), g = dy * mask(bn(z)), into sums (BN accumulators [B][C][2][S], zero them first) and sets
 * *fused (HOST) = 1; otherwise it runs the plain data gradient and sets *fused = 0.  z / mean_rstd
 * / gamma / beta are the unit's pre-BN conv output (same layout as dst), (mean, rstd) [B][C][2]
 * and BN parameters.  cvl_bn_backward_relu_sums is cvl_bn_backward_relu's second pass from those
 * sums (the first pass and its reduction are skipped). */
int cvl_conv_igemm_dgrad_bnsum(const cvl_conv_desc* d, const void* src, void* dst, const void* z,
                               const float* mean_rstd, const float* gamma, const float* beta, float act_hi,
                               uint64_t* sums, int32_t* fused, void* workspace, size_t workspace_bytes,
                               cvl_stream_t stream);
int cvl_bn_backward_relu_sums(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                              const float* beta, uint64_t* sums, void* dz, float* dgamma, float* dbeta,
                              float beta_acc, float* conv_dbias, float act_hi, int B, int HW, int C,
                              cvl_stream_t stream);
/* The residual-unit form (a bottleneck's BN3: BN -> + shortcut -> ReLU, the block output y).  The
 * block-input gradient of the NEXT block is completed by its first 1x1 data gradient accumulating
 * into dst (d->beta != 0); cvl_conv_igemm_dgrad_bnsum_res runs that launch and, on the persistent
 * 1x1 kernel, adds (sum g, sum g*xhat), g = final dst * (y > 0), into sums (zeroed) and sets
 * *fused = 1 (else the plain data gradient, *fused = 0).  cvl_bn_backward_res_sums is then that BN
 * backward's second pass from the sums: dz, g_out (= g, the shortcut's gradient) and dgamma/dbeta
 * (replaces cvl_bn_backward with y_relu given). */
int cvl_conv_igemm_dgrad_bnsum_res(const cvl_conv_desc* d, const void* src, void* dst, const void* y, const void* z,
                                   const float* mean_rstd, const float* gamma, const float* beta, uint64_t* sums,
                                   int32_t* fused, void* workspace, size_t workspace_bytes, cvl_stream_t stream);
int cvl_bn_backward_res_sums(const void* dy, const void* y, const void* z, const float* mean_rstd, const float* gamma,
                             uint64_t* sums, void* dz, void* g_out, float* dgamma, float* dbeta, float beta_acc,
                             float* conv_dbias, int B, int HW, int C, cvl_stream_t stream);
/* A projection block's residual unit (Keras ResNet50 block1: conv3 BN -> + shortcut BN -> ReLU, the
 * TF gradient through both BNs behind FCOS/fcos.py:30-35): cvl_bn_backward_res_sums that also forms
 * the shortcut BN backward's first pass on the same masked gradient (the shortcut's dy is g_out) from
 * the shortcut's pre-BN z_sc and (mean, rstd) -- per-block partials in `workspace`, then a fixed-order
 * column sum into sc_sums [B][C][2] (float64 values, slot mode 1); cvl_bn_backward_sums then runs the
 * shortcut's second pass.  The separate first pass over g_out and z_sc is gone. */
size_t cvl_bn_backward_res_sums_sc_workspace_size(int B, int HW, int C);
int cvl_bn_backward_res_sums_sc(const void* dy, const void* y, const void* z, const float* mean_rstd,
                                const float* gamma, uint64_t* sums, void* dz, void* g_out, float* dgamma,
                                float* dbeta, float beta_acc, float* conv_dbias, const void* z_sc,
                                const float* mean_rstd_sc, void* workspace, size_t workspace_bytes,
                                uint64_t* sc_sums, int B, int HW, int C, cvl_stream_t stream);
/* The same when the residual unit's first pass is not fused upstream: cvl_bn_backward (mask y > 0,
 * g_out) whose second pass also forms the shortcut BN's first pass into sc_sums. */
size_t cvl_bn_backward_sc_workspace_size(int B, int HW, int C);
int cvl_bn_backward_sc(const void* dy, const void* y, const void* z, const float* mean_rstd, const float* gamma,
                       void* workspace, size_t workspace_bytes, void* dz, void* g_out, float* dgamma, float* dbeta,
                       float beta_acc, float* conv_dbias, const void* z_sc, const float* mean_rstd_sc,
                       uint64_t* sc_sums, int B, int HW, int C, cvl_stream_t stream);
/* Second pass only of a BN without ReLU from first-pass sums [B][C][2] (slot mode 1). */
int cvl_bn_backward_sums(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                         const uint64_t* sums, void* dz, float* dgamma, float* dbeta, float beta_acc,
                         float* conv_dbias, int B, int HW, int C, cvl_stream_t stream);

/* BN -> ReLU6 unit without a residual (MobileNetV2: Keras ReLU(6.)): as cvl_bn_backward_relu with
 * the TF Relu6Grad mask 0 < bn(z) < 6 rebuilt from z in fp32 (the forward's exact pre-clamp value);
 * cvl_bn_apply / cvl_bn_finalize_apply take relu = 2 for ReLU6. */
int cvl_bn_backward_relu6(const void* dy, const void* z, const float* mean_rstd, const float* gamma,
                          const float* beta, void* workspace, size_t workspace_bytes, void* dz, float* dgamma,
                          float* dbeta, float beta_acc, float* conv_dbias, int B, int HW, int C, cvl_stream_t stream);

/* ResNet50 pool1: ZeroPadding2D(1) + MaxPooling2D(3, 2); argmax [B][Ho][Wo][C] uint8 (0..8). */
/* Stem BN -> ReLU -> ZeroPadding2D(1) -> MaxPool 3x3/2 fused (Keras ResNet50 conv1_bn .. pool1_pool):
 * from the pre-BN z [B,H,W,C] bf16 and (mean, rstd) [B][C][2]; writes the pooled y and argmax as
 * cvl_maxpool3x3s2 would from the stored BN output (bit-identical), without that full-size output. */
int cvl_bn_relu_maxpool3x3s2(const void* z, const float* mean_rstd, const float* gamma, const float* beta, void* y,
                             uint8_t* argmax, int B, int H, int W, int C, cvl_stream_t stream);
int cvl_maxpool3x3s2(const void* x, void* y, uint8_t* argmax, int B, int H, int W, int C,
                     cvl_stream_t stream);
int cvl_maxpool3x3s2_backward(const void* dy, const uint8_t* argmax, void* dx, int B, int H, int W,
                              int C, cvl_stream_t stream);
/* The stem's backward front (pool1_pool -> conv1_relu -> conv1_bn backward, the TF gradient of
 * Keras ResNet50's first block behind FCOS/fcos.py:30): max-pool backward of dp [B,Ho,Wo,64] through
 * argmax into dy [B,H,W,64] (bit-identical to cvl_maxpool3x3s2_backward) with the BN -> ReLU
 * backward's first pass (mask rebuilt from z) fused into that kernel, then the second pass as
 * cvl_bn_backward_relu (dz, dgamma, dbeta, conv_dbias = 0).  C = 64 (ResNet conv1) only. */
size_t cvl_maxpool3x3s2_backward_bn_relu_workspace_size(int B, int H, int W, int C);
int cvl_maxpool3x3s2_backward_bn_relu(const void* dp, const uint8_t* argmax, const void* z, const float* mean_rstd,
                                      const float* gamma, const float* beta, void* workspace,
                                      size_t workspace_bytes, void* dy, void* dz, float* dgamma, float* dbeta,
                                      float beta_acc, float* conv_dbias, int B, int H, int W, int C,
                                      cvl_stream_t stream);
/* FPN top-down (fcos.py:57-60): out[B,H,W,C] = a + nearest_up2(b[B,H/2,W/2,C]); backward:
 * db = sum of dout over each 2x2 block (+ beta*db). */
int cvl_upsample2x_add(const void* a, const void* b, void* out, int B, int H, int W, int C,
                       cvl_stream_t stream);
int cvl_upsample2x_backward(const void* dout, void* db, int B, int H, int W, int C, float beta,
                            cvl_stream_t stream);
int cvl_relu_backward(const void* dy, const void* y, void* dx, long n, float beta, cvl_stream_t stream);
int cvl_add(const void* a, const void* b, void* out, long n, cvl_stream_t stream);
/* bias gradient over a segment's rows: db[c] = beta*db + sum dy[row][coff + c] (rows base +
 * b*img_stride + q, q < HW); deterministic (per-block partials summed in a fixed order).  Needs
 * ld, coff % 8 == 0 and coff + round_up(ncol, 8) <= ld; workspace >= *_workspace_size bytes. */
size_t cvl_bias_grad_workspace_size(int ncol, int HW, int B);
int cvl_bias_grad(const void* dy, int ld, int coff, int ncol, int64_t base, int64_t img_stride, int HW,
                  int B, void* workspace, size_t workspace_bytes, float* db, float beta, cvl_stream_t stream);
/* Batched form of cvl_bias_grad: up to CVL_BIAS_MAX_ITEMS bias gradients (e.g. the per-level
 * heads `logits_output_l` / `reg_output_l` of FCOS/fcos.py:85-101, the FPN convs of fcos.py:49-74)
 * in ONE partial-sum launch + ONE fixed-order finish launch.  items: HOST array (passed by value to
 * the kernels, so the call is graph-capturable); same per-item contract as cvl_bias_grad with
 * ncol <= 2048; workspace >= cvl_bias_grad_multi_workspace_size(items, n) bytes. */
#define CVL_BIAS_MAX_ITEMS 16
typedef struct {
  const void* dy;      /* bf16 rows [*][ld] */
  float* db;           /* fp32 [ncol] */
  int64_t base, img_stride;
  int ld, coff, ncol, HW, B;
  float beta;
} cvl_bias_item;
size_t cvl_bias_grad_multi_workspace_size(const cvl_bias_item* items, int n);
int cvl_bias_grad_multi(const cvl_bias_item* items, int n, void* workspace, size_t workspace_bytes,
                        cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * fp32 parity mode (SURVEY.md §8b "Parity modes", CVL_PRECISION=fp32): the same training graph
 * with fp32 activations and activation gradients, for whole-graph parity with the reference's
 * fp32 Keras graph (FCOS/fcos.py:6-110, RetinaNet/retinanet_module.py:8-159).  Convolutions take
 * cvl_conv_desc.prec = CVL_PREC_F32; the memory-bound ops below are the fp32 forms of the
 * entry points of the same names (same arguments, float tensors; every reduction fixed-order).
 * cvl_bn_backward_f32 covers cvl_bn_backward (y_relu = the ReLU output, bn_beta NULL) and
 * cvl_bn_backward_relu (y_relu NULL, bn_beta = the BN's beta: mask rebuilt from z), act_hi =
 * INFINITY (ReLU) or 6 (ReLU6); workspace >= cvl_bn_backward_f32_workspace_size(B, C).
 * cvl_bias_grad_multi_f32 takes cvl_bias_item rows of fp32 dy (no workspace).
 * ---------------------------------------------------------------------------------------- */
int cvl_bn_apply_f32(const float* z, const float* mean_rstd, const float* gamma, const float* beta,
                     const float* residual, float* y, int B, int HW, int C, int relu, cvl_stream_t stream);
int cvl_bn_finalize_apply_f32(uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var,
                              const float* z, const float* gamma, const float* beta, const float* residual,
                              float* y, int B, int HW, int C, int relu, float eps, float momentum,
                              cvl_stream_t stream);
size_t cvl_bn_backward_f32_workspace_size(int B, int C);
int cvl_bn_backward_f32(const float* dy, const float* y_relu, const float* z, const float* mean_rstd,
                        const float* gamma, const float* bn_beta, void* workspace, size_t workspace_bytes,
                        float* dz, float* g_out, float* dgamma, float* dbeta, float beta_acc,
                        float* conv_dbias, float act_hi, int B, int HW, int C, cvl_stream_t stream);
int cvl_maxpool3x3s2_f32(const float* x, float* y, uint8_t* argmax, int B, int H, int W, int C,
                         cvl_stream_t stream);
int cvl_maxpool3x3s2_backward_f32(const float* dy, const uint8_t* argmax, float* dx, int B, int H, int W,
                                  int C, cvl_stream_t stream);
int cvl_upsample2x_add_f32(const float* a, const float* b, float* out, int B, int H, int W, int C,
                           cvl_stream_t stream);
int cvl_upsample2x_backward_f32(const float* dout, float* db, int B, int H, int W, int C, float beta,
                                cvl_stream_t stream);
int cvl_relu_backward_f32(const float* dy, const float* y, float* dx, long n, float beta, cvl_stream_t stream);
int cvl_add_f32(const float* a, const float* b, float* out, long n, cvl_stream_t stream);
int cvl_bias_grad_multi_f32(const cvl_bias_item* items, int n, cvl_stream_t stream);
/* cvl_retina_loss with fp32 gradient outputs (the parity mode's RetinaNet heads). */
int cvl_retina_loss_f32(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, const float* targets,
                        int B, const int32_t* level_cells, int n_anchors, int num_classes, const float* img_weight,
                        float grad_scale, float* losses, float* d_reg, int ld_dreg, float* d_cls, int ld_dcls,
                        void* workspace, cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * Optimizer (train_fcos.py:179-185): g <- (g * inv_bs) clipped by global norm `clip`
 * (tf.clip_by_global_norm), then Keras SGD momentum v = m*v - lr*g; w += v.  Flat fp32 buffers;
 * lr read from device memory (graph-capturable); sumsq_ws: CVL_SUMSQ_WS float64 (total + the
 * per-block partials of the deterministic norm reduction); w / g / v 16-byte aligned.
 * cvl_lr_schedule: lr = max(init*rate^floor(step/decay_step), min_lr); step += 1 (device ints).
 * cvl_lr_schedule_capped: the same with the exponent capped at max_decays (>= 0): the centre
 * variants' step schedule (FCOS/train_fcos_center_voc.py:150-157: init_lr below step 8000, init/10
 * from then on -- its init/100 branch is unreachable) is rate 0.1, decay_step 8000, max_decays 1.
 * ---------------------------------------------------------------------------------------- */
#define CVL_SUMSQ_WS 1025
int cvl_sgd_clip_update(float* w, const float* g, float* v, int64_t n, const float* lr_dev,
                        float momentum, float inv_bs, float clip, double* sumsq_ws, cvl_stream_t stream);
int cvl_lr_schedule(int32_t* step, float* lr, double init_lr, double min_lr, double decay_rate,
                    int decay_step, cvl_stream_t stream);
int cvl_lr_schedule_capped(int32_t* step, float* lr, double init_lr, double min_lr, double decay_rate,
                           int decay_step, int max_decays, cvl_stream_t stream);

/* l2_params_reg of train_fcos.py:118-120 = sum over tensors v of sqrt(sum(tf.nn.l2_loss(v)))
 * = sum_v sqrt(0.5 * sum(v^2)), over the tensors at device offsets[i] / sizes[i] of the flat
 * parameter buffer; terms: n_tensors floats of workspace; *out (device float).  The reference
 * computes it outside the GradientTape, so it enters the reported loss, not the gradient. */
int cvl_l2_params_reg(const float* flat, const int64_t* offsets, const int64_t* sizes, int n_tensors,
                      float* terms, float* out, cvl_stream_t stream);

/* RetinaNet candidate selection (train_retinanet_coco.py:190-209: images without matches are
 * skipped, the first batch_size usable candidates are trained on): idx[k] = the first k indices
 * i < n (in order) with counts[i] > 0, weight[k] = 1 for a filled slot and 0 for an empty one.
 * cvl_gather_rows: dst row i = src row idx[i], rows of row_bytes (multiple of 16). */
int cvl_select_first_nonzero(const int32_t* counts, int n, int k, int32_t* idx, float* weight,
                             cvl_stream_t stream);
int cvl_gather_rows(const void* src, int64_t row_bytes, const int32_t* idx, int n, void* dst, cvl_stream_t stream);

/* ------------------------------------------------------------------------------------------
 * RetinaNet target assignment.  Replaces RetinaNet/retinanet_module.py:205-365
 * (`RetinaNet.__init__` anchor dims are passed in; `get_anchors` + `format_data` + utils.compute_iou
 * run per output cell): anchor_dims [5][n_anchors][2] fp32 (h, w); square pad (pad x pad);
 * output targets [B][sum_l n_anchors*S_l^2][4+C] ordered (level, anchor, u, v), the reference's
 * nested [5][9] maps of [S,S,4+C] (float64 there) rounded to fp32, bit-exact; match iff fp32
 * IoU > iou_thresh; num_targets[b] = number of (box, anchor) matches. */
int cvl_retina_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                      int pad, int num_classes, const float* anchor_dims, int n_anchors,
                      const int32_t* strides /*host[5]*/, float iou_thresh, float* targets,
                      int32_t* num_targets, cvl_stream_t stream);

/* CenterNet (hourglass) centroid targets: CenterNet/tf_centernet_hourglass.py:379-456.
 * Output [B][pad_w/stride][pad_h/stride][4+C] (the reference's h_max/w_max swap kept). */
int cvl_centernet_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                         int pad_h, int pad_w, int num_classes, int stride, float* targets,
                         cvl_stream_t stream);

/* CenterNet centre "splat": CenterNet/tf_centernet.py:152-342 (inverse-power kernel, spread 8,
 * sigma sub-box).  Output [B][pad_h/stride][pad_w/stride][5+C]. */
int cvl_centernet_splat(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                        int pad_h, int pad_w, int num_classes, int stride, float sigma, float* targets,
                        cvl_stream_t stream);
/* CenterNet/tf_centernet.py:6-19 center_dist_1d (grid_y NULL) / center_dist_2d: out[i] =
 * g[i] / max(g), g = 1 / (grid_x - mu_x)^spread [* 1 / (grid_y - mu_y)^spread], float64, n points. */
int cvl_center_dist(const double* grid_x, const double* grid_y, int n, double mu_x, double mu_y, double spread,
                    double* out, cvl_stream_t stream);

/* Focal (alpha .25, gamma 2) on C class logits + smooth-L1 on 4 box channels masked by
 * max(class target) > 0: CenterNet model_loss (tf_centernet_hourglass.py:492-505) and one
 * (level, anchor) term of RetinaNet.train_loss (retinanet_module.py:403-426).  targets
 * [B][P][4+C]; losses [B][2] = (cls, reg); d_reg / d_cls (fp32, same strides) nullable. */
size_t cvl_det_loss_workspace_size(int B, int P);
int cvl_det_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, const float* targets,
                 int B, int P, int num_classes, float grad_scale_cls, float grad_scale_reg, float* losses,
                 float* d_reg, float* d_cls, void* workspace, cvl_stream_t stream);

/* RetinaNet.train_loss fwd + bwd over all (level, anchor) terms (retinanet_module.py:367-426) in
 * one launch.  reg_pred / cls_pred: the grouped head outputs [B][P][ld] fp32 (P = sum of
 * level_cells, level-major cells; anchor a's boxes at channels 4a..4a+3, its classes at
 * aC..aC+C-1); targets: cvl_retina_assign's [B][n_anchors*P][4+C] in (level, anchor, cell) order.
 * losses [B][2] = (cls, reg) sums; d_reg / d_cls (nullable): bf16 grad_scale * dloss/dpred at the
 * prediction positions (other channels untouched).  img_weight [B] (nullable) multiplies image b's
 * loss and gradient (0 = an image the reference loop skipped for having no matches). */
size_t cvl_retina_loss_workspace_size(int B, int P, int n_anchors);
int cvl_retina_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, const float* targets,
                    int B, const int32_t* level_cells /*host[5]*/, int n_anchors, int num_classes,
                    const float* img_weight, float grad_scale, float* losses, void* d_reg, int ld_dreg,
                    void* d_cls, int ld_dcls, void* workspace, cvl_stream_t stream);

/* Greedy per-class NMS (CenterNet/tf_centernet_hourglass.py:44-85, method 'nms'): boxes [n][6] =
 * (x1, y1, x2, y2, score, cls) float64; classes [ncls] processed in the given order; keep
 * [ncls][n] indices in selection order (first maximum among survivors), nkeep [ncls]. */
size_t cvl_nms_workspace_size(int n, int ncls);
int cvl_nms(const double* boxes, int n, const double* classes, int ncls, double iou_threshold,
            int32_t* keep, int32_t* nkeep, void* workspace, cvl_stream_t stream);
/* Soft-NMS (tf_centernet_hourglass.py:44-85, method 'soft-nms'; Bodla et al. 2017, Gaussian
 * decay): per class, emit the first maximum of the running scores, then scale every survivor's
 * score by exp(-(iou^2 / sigma)) (float64) and drop scores that are no longer > 0.  Same layout as
 * cvl_nms plus keep_score [ncls][n] = the emitted (decayed) score of each kept row. */
size_t cvl_soft_nms_workspace_size(int n, int ncls);
int cvl_soft_nms(const double* boxes, int n, const double* classes, int ncls, double sigma, int32_t* keep,
                 double* keep_score, int32_t* nkeep, void* workspace, cvl_stream_t stream);

/* ==========================================================================================
 * CenterNet hourglass training path (CenterNet/tf_centernet_hourglass.py:87-353 build_model,
 * :492-564 model_loss / train_step).
 * ========================================================================================== */

/* BatchNormalization over sub-batches: train_step (:527-545) runs one Keras training-mode forward
 * per sub-batch of `group` images, so statistics span the sub-batch (groups [g*G, min(g*G+G, B)),
 * the last may be short); running stats are updated once per group, in order.
 * cvl_bn_stats: stats[b][c] = (sum, sum of squares) over H*W of a bf16 NHWC tensor (BN
 *   accumulators [B][C][2][S], deterministic), the input of cvl_bn_finalize[_grouped].
 * cvl_bn_backward_grouped: as cvl_bn_backward (no ReLU output / conv bias terms) with group
 *   statistics; dz = BN-backward + dz_beta * dz (accumulate into an existing gradient). */
size_t cvl_bn_stats_workspace_size(int B, int HW, int C);
int cvl_bn_stats(const void* x, int B, int HW, int C, uint64_t* stats, void* workspace, size_t workspace_bytes,
                 cvl_stream_t stream);
int cvl_bn_finalize_grouped(const uint64_t* stats, float* mean_rstd, float* run_mean, float* run_var, int B, int C,
                            int HW, int group, float eps, float momentum, cvl_stream_t stream);
size_t cvl_bn_backward_grouped_workspace_size(int B, int HW, int C);
int cvl_bn_backward_grouped(const void* dy, const void* y_relu, const void* z, const float* mean_rstd,
                            const float* gamma, void* workspace, size_t workspace_bytes, void* dz, float dz_beta,
                            float* dgamma, float* dbeta, int B, int HW, int C, int group, cvl_stream_t stream);

/* downsample_block (:158-161): MaxPooling2D(2, 2, "same") -> [B][ceil(H/2)][ceil(W/2)][C];
 * argmax [B][Ho][Wo][C] uint8 (0..3, first maximum in window order). */
int cvl_maxpool2x2(const void* x, void* y, uint8_t* argmax, int B, int H, int W, int C, cvl_stream_t stream);
int cvl_maxpool2x2_backward(const void* dy, const uint8_t* argmax, void* dx, int B, int H, int W, int C,
                            cvl_stream_t stream);

/* Decoder merge (:276-284): out[B][2h][2w][C] = other + UpSampling2D(bilinear)(prev[B][h][w][C]),
 * TF resize_bilinear with half-pixel centres.  Backward: dprev = adjoint(dout) (+ beta * dprev). */
int cvl_upsample_bilinear2x_add(const void* prev, const void* other, void* out, int B, int h, int w, int C,
                                cvl_stream_t stream);
int cvl_upsample_bilinear2x_backward(const void* dout, void* dprev, int B, int h, int w, int C, float beta,
                                     cvl_stream_t stream);

/* Depthwise convolution (Keras DepthwiseConv2D, depth_multiplier 1, no bias; the MobileNetV2
 * backbone of FCOS/fcos.py:36-41 and its siblings): x [B][H][W][C] bf16, w [k][k][C] fp32 (Keras
 * depthwise_kernel [k][k][C][1]), y [B][Ho][Wo][C] bf16, explicit top/left padding (TF "same" or
 * ZeroPadding2D(correct_pad) + "valid"), C % 8 == 0.  dgrad: dx = beta*dx + conv^T(dy).  wgrad
 * (k = 3): dw = beta*dw + sum over all output pixels, deterministic; workspace >= *_size. */
int cvl_depthwise_fwd(const void* x, const float* w, void* y, int B, int H, int W, int C, int k, int stride,
                      int pad_t, int pad_l, int Ho, int Wo, cvl_stream_t stream);
int cvl_depthwise_dgrad(const void* dy, const float* w, void* dx, int B, int H, int W, int C, int k, int stride,
                        int pad_t, int pad_l, int Ho, int Wo, float beta, cvl_stream_t stream);
size_t cvl_depthwise_wgrad_workspace_size(int B, int Ho, int Wo, int C, int k);
int cvl_depthwise_wgrad(const void* x, const void* dy, float* dw, float beta, int B, int H, int W, int C, int k,
                        int stride, int pad_t, int pad_l, int Ho, int Wo, void* workspace, size_t workspace_bytes,
                        cvl_stream_t stream);

/* CenterNet v2 (CenterNet/tf_hourglass_net.py:115-449, n_filters 12 in train_hourglass_voc.py:298-331)
 * --------------------------------------------------------------------------------------------
 * out = UpSampling2D(bilinear)(a + b) (:252-305; b nullable): taps of a + b in fp32, one pass. */
int cvl_upsample_bilinear2x_sum(const void* a, const void* b, void* out, int B, int h, int w, int C,
                                cvl_stream_t stream);
/* The "pass through" reshape-concat (:307-344): map k [B][hw][c_ld] bf16 (c real channels, pads
 * zero) is tf.reshape'd to [B][S2][c*hw/S2] (row-major reinterpretation, Q36) and the maps are
 * concatenated on channels into dst [B][S2][ld_dst] (columns past the sum zeroed).  c % 4 == 0,
 * (c*hw/S2) % 4 == 0.  Backward: dsrc = beta*dsrc + the inverse gather of d_dst (pads of dsrc
 * written zero when beta == 0).  items: HOST array. */
#define CVL_RC_MAX_ITEMS 16
typedef struct {
  const void* src;     /* forward source map */
  void* dsrc;          /* backward destination (gradient of the map) */
  int c, c_ld, hw;     /* real channels, channel pitch, pixels per image */
  float beta;          /* backward accumulate factor */
} cvl_rc_item;
int cvl_reshape_concat(const cvl_rc_item* items, int n_items, int B, int S2, void* dst, int ld_dst,
                       cvl_stream_t stream);
int cvl_reshape_concat_backward(const cvl_rc_item* items, int n_items, int B, int S2, const void* d_dst,
                                int ld_dst, cvl_stream_t stream);
/* b_focal on every scale's class channels (:380-385): b_eff[c] = bias[c] + ((c % period) >= c0 ?
 * *scalar : 0); unfold: g_bias = g_eff, *g_scalar = sum over those channels (fixed order). */
int cvl_bias_scalar_fold_periodic(const float* bias, const float* scalar, float* b_eff, int n, int period, int c0,
                                  cvl_stream_t stream);
int cvl_bias_scalar_unfold_periodic(const float* g_eff, float* g_bias, float* g_scalar, int n, int period, int c0,
                                    cvl_stream_t stream);
/* Targets of train_hourglass_voc.py train() :96-160 for one batch: boxes [B][n_max][5] = the
 * dataset's corner rows + label (utils.convert_to_xywh :16-27 applied inside), one (raw_dims,
 * img_dims) per batch (pad_dims = (img - raw) / 2); targets [B][S][S][4][5+C] fp32, S = img/8:
 * ascending w*h*100, last writer per (cell, scale) sets (y_off, x_off, h_reg, w_reg, 1), class
 * bits OR'd.  Bit-exact to the reference's float32 arithmetic. */
int cvl_hourglass_v2_assign(const float* boxes, const int32_t* nbox, int B, int n_max, int raw_dims, int img_dims,
                            int num_classes, float* targets, cvl_stream_t stream);
/* model_loss (:398-413) fwd + bwd off the head conv: pred [B*P][ld_pred] fp32 (channel sc*(5+C)+j,
 * b_focal folded), targets [B*P][4][5+C]; loss_type bit 0: sigmoid cross-entropy (else focal) on
 * channels 4..4+C; L1 on sigmoid(pred[0..3]) masked by t[4] (bit 1: pred[0..3] are already the
 * model's sigmoid outputs, as model_loss receives them).  losses [B][2] = (cls, reg); d_pred bf16
 * [B*P][ld_d] = d(cls_scale*cls + reg_scale*reg)/d(pred).  workspace >= *_workspace_size(B, P). */
/* CenterNet ResNet stride-8 multi-scale (CenterNet/tf_centernet_resnet_s8.py) targets, format_data
 * (:243-330) batched: boxes [B][n_max][5] normalised (y, x, h, w, cls) fp32, img_dim [B][2] the
 * resized size, (pad_h, pad_w) the padded size, box_scales HOST [n_scales] (<= 8), stride 8 in the
 * reference.  targets [B][pad_w/stride][pad_h/stride][n_scales][4+C] fp32; float64 arithmetic
 * (the reference's gt_labels are float64), bit-exact. */
int cvl_centernet_s8_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                            int pad_h, int pad_w, int num_classes, const float* box_scales, int n_scales, int stride,
                            float* targets, cvl_stream_t stream);
/* model_loss (:368-385) fwd + bwd off the two head convs: reg_pred [B*P][ld_reg] (n_scales x 4 raw
 * box logits per cell, sigmoid applied here), cls_pred [B*P][ld_cls] (n_scales x C logits),
 * targets [B*P][n_scales][4+C]; focal + smooth-L1 of sigmoid(box) masked by max(class) > 0.
 * losses [B][2] = (cls, reg); d_reg / d_cls bf16 (pitches ld_dreg / ld_dcls, pads zeroed). */
size_t cvl_centernet_s8_loss_workspace_size(int B, int P, int n_scales);
int cvl_centernet_s8_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, const float* targets,
                          int B, int P, int n_scales, int num_classes, float cls_scale, float reg_scale, float* losses,
                          void* d_reg, int ld_dreg, void* d_cls, int ld_dcls, void* workspace, cvl_stream_t stream);
size_t cvl_hourglass_v2_loss_workspace_size(int B, int P);
int cvl_hourglass_v2_loss(const float* pred, int ld_pred, const float* targets, int B, int P, int num_classes,
                          int loss_type, float cls_scale, float reg_scale, float* losses, void* d_pred, int ld_d,
                          void* workspace, cvl_stream_t stream);

/* SeparableConv2D (:110-123, :178-181; depth_multiplier 1) runs as ONE dense conv on the MFMA
 * conv kernels with the folded kernel W[t][ci][co] = D[t][ci] * P[ci][co] (t = kh*kw taps; D =
 * Keras depthwise_kernel [kh][kw][Cin][1], P = pointwise_kernel [1][1][Cin][Cout]).
 * cvl_sep_fold_multi writes weff (fp32 HWIO) for every item; cvl_sep_unfold_multi turns the dense
 * kernel gradient gweff into gdw / gpw (weff / gweff [t][cin_ld][cout_ld] when the pitches are set,
 * pads untouched).  rows: DEVICE int32 [nrows][2] = (item, ci), one row per
 * input channel of every item.  items: DEVICE array. */
typedef struct {
  const float* dw;
  const float* pw;
  float* weff;
  const float* gweff;
  float* gdw;
  float* gpw;
  int taps, cin, cout;
  int cin_ld, cout_ld;  /* weff / gweff channel pitches (0 = cin / cout): padded dense kernels */
  int pad_;
} cvl_sep_item;
int cvl_sep_fold_multi(const cvl_sep_item* items, const int32_t* rows, int nrows, cvl_stream_t stream);
int cvl_sep_unfold_multi(const cvl_sep_item* items, const int32_t* rows, int nrows, cvl_stream_t stream);

/* BiasLayer b_focal (tf_bias_layer.py:4-14; :347) folded into the output conv bias:
 * b_eff[c] = bias[c] + (c >= c0 ? *scalar : 0); unfold: g_bias = g_eff, *g_scalar = sum_{c>=c0} g_eff. */
int cvl_bias_scalar_fold(const float* bias, const float* scalar, float* b_eff, int n, int c0, cvl_stream_t stream);
int cvl_bias_scalar_unfold(const float* g_eff, float* g_bias, float* g_scalar, int n, int c0, cvl_stream_t stream);

/* model_loss (:492-505) fwd + bwd off the output conv: pred [B*P][ld_pred] fp32 (reg 0..3, class
 * logits 4..4+C), targets [B*P][4+C] (cvl_centernet_assign); losses [B][2] = (cls, reg) sums;
 * d_pred bf16 [B*P][ld_d] = d(cls_scale*cls + reg_scale*reg)/d(pred), channels >= 4+C zeroed.
 * workspace >= cvl_det_loss_workspace_size(B, P). */
int cvl_centernet_loss(const float* pred, int ld_pred, const float* targets, int B, int P, int num_classes,
                       float cls_scale, float reg_scale, float* losses, void* d_pred, int ld_d, void* workspace,
                       cvl_stream_t stream);

/* obj_detect_results decode (tf_centernet_hourglass.py:576-650, before `nms`): pred [H][W][ld] fp32
 * (one image of the model output: ltrb 0..3, class logits 4..4+C) -> rows [n][6] float64 =
 * (x_low, y_low, w, h, int(100 * max prob), argmax class) for every cell whose max sigmoid
 * probability >= thresh, in np.nonzero (row-major) order; *count = n (<= H*W).  stride = the
 * reference's `downsample`; w_ratio = img_width / img_rows, h_ratio = img_height / img_cols with
 * img_width/img_height the source image's shape[0]/shape[1] (as the reference names them). */
int cvl_centernet_decode(const float* pred, int ld, int H, int W, int num_classes, double stride, float thresh,
                         double w_ratio, double h_ratio, double img_width, double img_height, double* rows,
                         int32_t* count, cvl_stream_t stream);

/* The variant CenterNets' obj_detect_results decodes (one image, before any plotting): pred
 * [H][W][ld] fp32 with scale s's channels at s*ch_per_scale (4 box channels, the class logits at
 * cls0 .. cls0+num_classes-1); rows [n][6] float64 for every (scale, cell) whose max sigmoid class
 * probability >= thresh, scale-major and np.nonzero order within a scale; *count = n (<= n_scales*H*W).
 * box_mode 1 = CenterNet/tf_centernet_resnet_s8.py:446-547 (prediction_to_corners :210-241 with
 *   box_scales[s] and `stride` = downsample, then (x_low, y_low, w, h, int(100 p), argmax class):
 *   the input of `nms` :44-85, iou 0.213);
 * box_mode 2 = CenterNet/tf_hourglass_net.py:517-578 (stride 8, box_scales[s] = the per-scale box
 *   scale of :518-524): (x_lower, y_lower, box_width, box_height, int(100 p), class index) of the
 *   drawn rectangles (x = the row axis, as the reference names it; cls0 = 5 skips channel 4 when the
 *   model has more than one class channel).
 * w_ratio = img_width / img_rows, h_ratio = img_height / img_cols (the source image's shape[0] /
 * shape[1], as the reference names them).  n_scales <= 16. */
int cvl_centernet_scale_decode(const float* pred, int ld, int H, int W, int n_scales, int ch_per_scale, int cls0,
                               int num_classes, int box_mode, const double* box_scales /*host[n_scales]*/,
                               float stride, float thresh, double w_ratio, double h_ratio, double img_width,
                               double img_height, double* rows, int32_t* count, cvl_stream_t stream);

/* CenterNet 3x3 max-pool peak decode (the north_star's peak decode; the reference's own decode is
 * cvl_centernet_decode above): pred [B][H][W][ld] fp32 (ltrb 0..3, class logits 4..4+C).  A
 * (cell, class) is a peak when sigmoid(logit) equals the 3x3 max-pool of its class map (-inf
 * padding, ties kept) and >= thresh; per image the K highest (probability desc, flat index
 * cell*C+class asc) peaks -> dets [B][K][6] float64 = (y_lo, x_lo, y_hi, x_hi, prob, class), the
 * corners as prediction_to_corners (tf_centernet_hourglass.py:355-377) x stride in fp32;
 * count [B] = rows written (<= K).  Sigmoid in float64 rounded to fp32.  Deterministic.
 * workspace >= cvl_centernet_peak_decode_workspace_size(B, H, W, C). */
size_t cvl_centernet_peak_decode_workspace_size(int B, int H, int W, int num_classes);
int cvl_centernet_peak_decode(const float* pred, int ld, int B, int H, int W, int num_classes, float stride,
                              float thresh, int K, double* dets, int32_t* count, void* workspace,
                              size_t workspace_bytes, cvl_stream_t stream);

/* train_step update (:555-563) with tf.keras.optimizers.Adam (train_hourglass_voc.py:330):
 * g <- clip_by_global_norm(g * inv_bs, clip); t = *iterations + 1;
 * m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2); w -= lr sqrt(1 - b2^t) / (1 - b1^t) * m / (sqrt(v) + eps);
 * then *iterations += 1.  lr read from device memory; sumsq_ws: one float64. */
int cvl_adam_clip_update(float* w, const float* g, float* m, float* v, int64_t n, const float* lr_dev,
                         int32_t* iterations, float beta1, float beta2, float eps, float inv_bs, float clip,
                         double* sumsq_ws, cvl_stream_t stream);

/* ==========================================================================================
 * RetinaNet inference decode (RetinaNet/retinanet_module.py:428-529).
 * ========================================================================================== */

/* prediction_to_corners (:428-451) of one (level, anchor) map: xy [H][W][ld] fp32 (t_y, t_x, t_h,
 * t_w at 0..3) -> out [H][W][4] = (y1, x1, y2, x2) fp32, centre = (col|row) * stride - t * anchor
 * (no +0.5, Q21), size = t * anchor; the reference's fp32 operation order. */
int cvl_retina_corners(const float* xy, int ld, int H, int W, float anchor_h, float anchor_w, int stride,
                       float* out, cvl_stream_t stream);

/* image_detections (:483-520) up to cpu_nms, for B images of the fused head outputs
 * (reg [B][P][ld_reg]: anchor a at 4a..4a+3; cls [B][P][ld_cls]: anchor a at aC..aC+C-1; rows
 * level-major, P = sum h*w).  level_hw [5][2] and strides [5] are HOST arrays; anchor_dims
 * [5][A][2] fp32 (h, w) on the device.  dets [B][A*P][6] fp32 = (y1, x1, y2, x2, max sigmoid
 * prob, first-argmax class) for the rows with prob >= cls_thresh, in the reference's
 * concatenation order (level, anchor, row-major cell); count [B] (device). */
size_t cvl_retina_decode_workspace_size(int B, const int32_t* level_hw, int n_anchors);
int cvl_retina_decode(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, int B,
                      const int32_t* level_hw, const int32_t* strides, const float* anchor_dims, int n_anchors,
                      int num_classes, float cls_thresh, float* dets, int32_t* count, void* workspace,
                      size_t workspace_bytes, cvl_stream_t stream);

/* cpu_nms (:453-481) per image over the first min(count[b], n_cap) rows of dets + b*rows_per_img*6
 * (count on the device: chains after cvl_retina_decode with no host sync): greedy, class-agnostic,
 * highest score first (lowest row among equal scores), survivors kept iff
 * inter / (a_i + a_j - inter + 1e-8) <= iou_thresh in fp32.  keep [B][n_cap] = selected rows in
 * selection order, nkeep [B]. */
size_t cvl_retina_nms_workspace_size(int B, int n_cap);
int cvl_retina_nms(const float* dets, int rows_per_img, const int32_t* count, int B, int n_cap, float iou_thresh,
                   int32_t* keep, int32_t* nkeep, void* workspace, cvl_stream_t stream);

/* FCOS/infer_fcos.py:27-62 image_detections for B images of the FCOS head outputs (reg [B][P][ld_reg]
 * = t, b, l, r, centerness; cls [B][P][ld_cls]; rows level-major, P = sum h*w <= 16384; level_hw
 * [5][2] and strides [5] HOST arrays): boxes = fcos.prediction_to_corners rounded to fp32, scores =
 * sigmoid(cls) (center != 0: sigmoid(centerness) * sigmoid(cls)), then
 * tf.image.combined_non_max_suppression(max_output_size_per_class = max_per_class, max_total_size =
 * max_total, clip_boxes=False): out_boxes [B][max_total][4] (y1, x1, y2, x2), out_scores /
 * out_classes [B][max_total] (zero padded), valid [B].  TF's op is restated (parity unpinned at
 * the reference level; equal-score order: lower box index, then lower class). */
size_t cvl_fcos_detect_workspace_size(int B, int P, int num_classes, int max_per_class);
int cvl_fcos_detect(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, int B,
                    const int32_t* level_hw, const int32_t* strides, int num_classes, int center, float iou_thresh,
                    float score_thresh, int max_per_class, int max_total, float* out_boxes, float* out_scores,
                    float* out_classes, int32_t* valid, void* workspace, size_t workspace_bytes,
                    cvl_stream_t stream);

/* ==========================================================================================
 * Input pipeline (FCOS/data_preprocess.py:24-133): resize_and_pad_image + random_flip_horizontal.
 * ========================================================================================== */

/* One decoded image src [H][W][C] (uint8 when src_u8, else fp32; C <= 4) -> out [pad_h][pad_w][C]
 * fp32 = (flip == 1 ? flip_left_right(src) : src) resized to out_h x out_w by TF2's bilinear
 * tf.image.resize (half-pixel centres, antialias off; restated), flip == 2: the resized image's
 * left-right flip (preprocess_data pad_flag=False: resize, then flip), then / 127.5 - 1, zero padded
 * bottom/right (tf.image.pad_to_bounding_box).  out may point into a batch slot. */
int cvl_resize_pad_normalize(const void* src, int src_u8, int H, int W, int C, int flip, int out_h, int out_w,
                             int pad_h, int pad_w, float* out, cvl_stream_t stream);

/* CenterNet/train_hourglass_voc.py:24-67 image_augment over a batch, the draws made by the caller
 * (cvlite.train_hourglass_v2.draw_augment): ops[b] / params[b] DEVICE int32 / fp32 per image,
 * 0 none, 1 brightness (x + params[b]), 2 contrast ((x - mean_c) * params[b] + mean_c, mean over
 * the N x N pixels of channel c), 3 flip left-right, 4 transpose (90 degrees), 5 transpose + flip
 * up-down (270 degrees); other codes copy.  img [B][N][N][3] fp32 (square padded images); tgt
 * [B][S][S][4][T] fp32 target maps (T = 5 + C), moved with the image (3: channel 1 := 1 - v;
 * 4 / 5: channels 0 := 1 and 2 := 3 of the transposed cell, the reference's aliased swap; 5: then
 * channel 0 := 1 - v) -- tgt_src = tgt_dst = NULL skips them.  src and dst must not overlap.
 * workspace: cvl_image_augment_workspace_size(B, N) bytes.  Two launches, deterministic. */
size_t cvl_image_augment_workspace_size(int B, int N);
int cvl_image_augment(const float* img_src, float* img_dst, const float* tgt_src, float* tgt_dst,
                      const int32_t* ops, const float* params, int B, int N, int S, int T, void* workspace,
                      size_t workspace_bytes, cvl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CVLITE_H_ */

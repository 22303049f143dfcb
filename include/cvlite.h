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
 * reg_type 0 = "l1" (smooth-L1), 1 = "iou".  `workspace` >= cvl_fcos_loss_workspace_size(B, P).
 * ---------------------------------------------------------------------------------------- */
size_t cvl_fcos_loss_workspace_size(int B, int P);
int cvl_fcos_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                  const float* targets, int B, int P, int num_classes, int reg_type,
                  float grad_scale, float* losses, void* d_reg, int ld_dreg, int dreg_dtype,
                  void* d_cls, int ld_dcls, int dcls_dtype, void* workspace, cvl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CVLITE_H_ */

"""ctypes binding of the cvlite C ABI (include/cvlite.h) -> libcvlite_hip.so (built in-tree).

torch is imported first on purpose: it loads its bundled HIP runtime (soname libamdhip64.so.7),
and the library then binds to that same runtime instance, so torch's hipStream_t handles and
device pointers are valid inside it.  There is no CPU fallback: every op fails loudly when the
library or the GPU is missing.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CVL_LIB: another build of the library (same-box A/B of two builds, tools/build_base.sh; the
# measurement build, tools/build_measure.sh)
LIB_PATH = os.environ.get("CVL_LIB") or os.path.join(_HERE, "libcvlite_hip.so")


def dispatch(key, default=0):
    """The CVL_DISPATCH test hooks (cvl_common.h; INTEGRATION.md "Environment"): "key" (= 1) or
    "key=value", comma-separated -- the Python side's fusion switches read here, the C library's
    kernel-family and planner hooks in cvl_dispatch_int.  Unset: the production path."""
    for tok in os.environ.get("CVL_DISPATCH", "").split(","):
        k, _, v = tok.strip().partition("=")
        if k == key:
            return int(v) if v else 1
    return default

c_int, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
P = c_void_p

# name -> (restype, argtypes); must match include/cvlite.h exactly
SIGNATURES = {
    "cvl_version": (c_int, []),
    "cvl_fcos_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "cvl_fcos_loss_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_fcos_loss": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_float, P,
                              P, c_int, c_int, P, c_int, c_int, P, c_size_t, P]),
    "cvl_fcos_loss_ex": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_float, c_float, c_float,
                                 c_float, P, P, c_int, c_int, P, c_int, c_int, P, c_size_t, P]),
    "cvl_fcos_decode": (c_int, [P, c_int, c_int, c_int, ctypes.c_double, P, P]),
    "cvl_fcos_v1_decode": (c_int, [P, c_int, c_int, c_int, c_float, c_float, P, P]),
    "cvl_conv_igemm_workspace_size": (c_size_t, [P]),
    "cvl_conv_igemm": (c_int, [P, P, P, P, P, c_size_t, P]),
    "cvl_conv_igemm_relu_mask": (c_int, [P, P, P, P, P, c_size_t, P]),
    "cvl_conv_igemm_last_kernel": (c_int, []),
    "cvl_conv_kernel_name": (ctypes.c_char_p, [c_int]),
    "cvl_centernet_peak_decode_workspace_size": (ctypes.c_size_t, [c_int, c_int, c_int, c_int]),
    "cvl_centernet_peak_decode": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_float, c_float, c_int, P, P, P,
                                          ctypes.c_size_t, P]),
    "cvl_conv_igemm_dgrad_bnsum": (c_int, [P, P, P, P, P, P, P, c_float, P, P, P, ctypes.c_size_t, P]),
    "cvl_bn_backward_relu_sums": (c_int, [P, P, P, P, P, P, P, P, P, c_float, P, c_float, c_int, c_int, c_int, P]),
    "cvl_conv_igemm_dgrad_bnsum_res": (c_int, [P, P, P, P, P, P, P, P, P, P, P, ctypes.c_size_t, P]),
    "cvl_bn_backward_res_sums": (c_int, [P, P, P, P, P, P, P, P, P, P, c_float, P, c_int, c_int, c_int, P]),
    "cvl_bn_backward_res_sums_sc_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bn_backward_res_sums_sc": (c_int, [P, P, P, P, P, P, P, P, P, P, c_float, P, P, P, P, c_size_t, P, c_int,
                                            c_int, c_int, P]),
    "cvl_bn_backward_sums": (c_int, [P, P, P, P, P, P, P, P, c_float, P, c_int, c_int, c_int, P]),
    "cvl_bn_backward_sc_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bn_backward_sc": (c_int, [P, P, P, P, P, P, c_size_t, P, P, P, P, c_float, P, P, P, P, c_int, c_int, c_int, P]),
    "cvl_probe_arm": (c_int, [P]),
    "cvl_probe_clock_hz": (ctypes.c_double, []),
    "cvl_conv_wgrad_workspace_size": (c_size_t, [P]),
    "cvl_conv_wgrad": (c_int, [P, P, P, P, c_float, P, c_size_t, P]),
    "cvl_conv_wgrad_grouped_workspace_size": (c_size_t, [P, c_int]),
    "cvl_conv_wgrad_grouped": (c_int, [P, c_int, P, P, P, c_float, P, c_size_t, P]),
    "cvl_conv_wgrad_batch_workspace_size": (c_size_t, [P, c_int]),
    "cvl_conv_wgrad_batch": (c_int, [P, c_int, P, P, P, c_float, P, c_size_t, P]),
    "cvl_pack_conv_weights": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, P]),
    "cvl_pack_conv_weights_multi": (c_int, [P, P, c_int, P]),
    "cvl_im2col": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                           c_int, c_int, P, P]),
    "cvl_bn_finalize": (c_int, [P, P, P, P, c_int, c_int, c_int, c_float, c_float, P]),
    "cvl_bn_acc_decode": (c_int, [P, P, ctypes.c_int64, P]),
    "cvl_bn_set_exact": (c_int, [c_int]),
    "cvl_bn_acc_slots": (c_int, []),
    "cvl_stem_conv7x7s2": (c_int, [P, c_int, c_int, c_int, P, P, P, P, P]),
    "cvl_stem_wgrad_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_stem_wgrad": (c_int, [P, c_int, c_int, c_int, P, P, c_float, P, c_size_t, P]),
    "cvl_bn_apply": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_bn_finalize_apply": (c_int, [P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_float, P]),
    "cvl_bn_finalize_apply_bnres": (c_int, [P, P, P, P, P, P, P, P, P, P, P, P, P, P, c_float, c_float, P, c_int,
                                            c_int, c_int, c_int, c_float, c_float, P]),
    "cvl_bn_backward_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bn_backward": (c_int, [P, P, P, P, P, P, c_size_t, P, P, P, P, c_float, P, c_int, c_int, c_int, P]),
    "cvl_bn_backward_relu": (c_int, [P, P, P, P, P, P, c_size_t, P, P, P, c_float, P, c_int, c_int, c_int, P]),
    "cvl_maxpool3x3s2": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_bn_relu_maxpool3x3s2": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_maxpool3x3s2_backward": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_maxpool3x3s2_backward_bn_relu_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cvl_maxpool3x3s2_backward_bn_relu": (c_int, [P, P, P, P, P, P, P, c_size_t, P, P, P, P, c_float, P, c_int, c_int,
                                                  c_int, c_int, P]),
    "cvl_upsample2x_add": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_upsample2x_backward": (c_int, [P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "cvl_relu_backward": (c_int, [P, P, P, ctypes.c_long, c_float, P]),
    "cvl_add": (c_int, [P, P, P, ctypes.c_long, P]),
    "cvl_bias_grad_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bias_grad_multi_workspace_size": (c_size_t, [P, c_int]),
    "cvl_bias_grad_multi": (c_int, [P, c_int, P, c_size_t, P]),
    "cvl_bias_grad": (c_int, [P, c_int, c_int, c_int, ctypes.c_int64, ctypes.c_int64, c_int, c_int, P, c_size_t,
                              P, c_float, P]),
    "cvl_wgrad_defer": (c_int, [c_int, P]),
    "cvl_wgrad_flush": (c_int, [P]),
    "cvl_sgd_clip_update": (c_int, [P, P, P, ctypes.c_int64, P, c_float, c_float, c_float, P, P]),
    "cvl_lr_schedule": (c_int, [P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int, P]),
    "cvl_lr_schedule_capped": (c_int, [P, P, ctypes.c_double, ctypes.c_double, ctypes.c_double, c_int, c_int, P]),
    "cvl_l2_params_reg": (c_int, [P, P, P, c_int, P, P, P]),
    "cvl_select_first_nonzero": (c_int, [P, c_int, c_int, P, P, P]),
    "cvl_gather_rows": (c_int, [P, ctypes.c_int64, P, c_int, P, P]),
    "cvl_retina_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, c_float, P, P, P]),
    "cvl_centernet_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "cvl_center_dist": (c_int, [P, P, c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double, P, P]),
    "cvl_centernet_splat": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_float, P, P]),
    "cvl_det_loss_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_det_loss": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_float, c_float, P, P, P, P, P]),
    "cvl_retina_loss_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_retina_loss": (c_int, [P, c_int, P, c_int, P, c_int, P, c_int, c_int, P, c_float, P, P, c_int, P, c_int,
                                P, P]),
    "cvl_bn_stats_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bn_stats": (c_int, [P, c_int, c_int, c_int, P, P, c_size_t, P]),
    "cvl_bn_finalize_grouped": (c_int, [P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_float, P]),
    "cvl_bn_backward_grouped_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_bn_backward_grouped": (c_int, [P, P, P, P, P, P, c_size_t, P, c_float, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_maxpool2x2": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_maxpool2x2_backward": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_upsample_bilinear2x_add": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_upsample_bilinear2x_backward": (c_int, [P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "cvl_upsample_bilinear2x_sum": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_bn_backward_relu6": (c_int, [P, P, P, P, P, P, c_size_t, P, P, P, c_float, P, c_int, c_int, c_int, P]),
    "cvl_depthwise_fwd": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P]),
    "cvl_depthwise_dgrad": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_float, P]),
    "cvl_depthwise_wgrad_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    "cvl_depthwise_wgrad": (c_int, [P, P, P, c_float, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                    c_int, P, c_size_t, P]),
    "cvl_reshape_concat": (c_int, [P, c_int, c_int, c_int, P, c_int, P]),
    "cvl_reshape_concat_backward": (c_int, [P, c_int, c_int, c_int, P, c_int, P]),
    "cvl_bias_scalar_fold_periodic": (c_int, [P, P, P, c_int, c_int, c_int, P]),
    "cvl_bias_scalar_unfold_periodic": (c_int, [P, P, P, c_int, c_int, c_int, P]),
    "cvl_hourglass_v2_assign": (c_int, [P, P, c_int, c_int, c_int, c_int, c_int, P, P]),
    "cvl_centernet_s8_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, P]),
    "cvl_centernet_s8_loss_workspace_size": (c_size_t, [c_int, c_int, c_int]),
    "cvl_centernet_s8_loss": (c_int, [P, c_int, P, c_int, P, c_int, c_int, c_int, c_int, c_float, c_float, P, P, c_int,
                                      P, c_int, P, P]),
    "cvl_hourglass_v2_loss_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_hourglass_v2_loss": (c_int, [P, c_int, P, c_int, c_int, c_int, c_int, c_float, c_float, P, P, c_int, P, P]),
    "cvl_sep_fold_multi": (c_int, [P, P, c_int, P]),
    "cvl_sep_unfold_multi": (c_int, [P, P, c_int, P]),
    "cvl_bias_scalar_fold": (c_int, [P, P, P, c_int, c_int, P]),
    "cvl_bias_scalar_unfold": (c_int, [P, P, P, c_int, c_int, P]),
    "cvl_centernet_loss": (c_int, [P, c_int, P, c_int, c_int, c_int, c_float, c_float, P, P, c_int, P, P]),
    "cvl_adam_clip_update": (c_int, [P, P, P, P, ctypes.c_int64, P, P, c_float, c_float, c_float, c_float, c_float,
                                     P, P]),
    "cvl_centernet_decode": (c_int, [P, c_int, c_int, c_int, c_int, ctypes.c_double, c_float, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, ctypes.c_double, P, P, P]),
    "cvl_centernet_scale_decode": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, c_float,
                                           c_float, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, P, P, P]),
    "cvl_nms_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_nms": (c_int, [P, c_int, P, c_int, ctypes.c_double, P, P, P, P]),
    "cvl_soft_nms_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_soft_nms": (c_int, [P, c_int, P, c_int, ctypes.c_double, P, P, P, P, P]),
    "cvl_retina_corners": (c_int, [P, c_int, c_int, c_int, c_float, c_float, c_int, P, P]),
    "cvl_retina_decode_workspace_size": (c_size_t, [c_int, P, c_int]),
    "cvl_retina_decode": (c_int, [P, c_int, P, c_int, c_int, P, P, P, c_int, c_int, c_float, P, P, P, c_size_t,
                                  P]),
    "cvl_retina_nms_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_retina_nms": (c_int, [P, c_int, P, c_int, c_int, c_float, P, P, P, P]),
    "cvl_fcos_center_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, P, P]),
    "cvl_fcos_center_v1_assign": (c_int, [P, P, P, c_int, c_int, c_int, c_int, c_int, P, P, P, P, P]),
    "cvl_resize_pad_normalize": (c_int, [P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    "cvl_image_augment_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_image_augment": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P, c_size_t, P]),
    "cvl_fcos_detect_workspace_size": (c_size_t, [c_int, c_int, c_int, c_int]),
    "cvl_fcos_detect": (c_int, [P, c_int, P, c_int, c_int, P, P, c_int, c_int, c_float, c_float, c_int, c_int, P, P,
                                P, P, P, c_size_t, P]),
    # fp32 parity mode (include/cvlite.h "fp32 parity mode")
    "cvl_bn_apply_f32": (c_int, [P, P, P, P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_bn_finalize_apply_f32": (c_int, [P, P, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, c_float, c_float,
                                          P]),
    "cvl_bn_backward_f32_workspace_size": (c_size_t, [c_int, c_int]),
    "cvl_bn_backward_f32": (c_int, [P, P, P, P, P, P, P, c_size_t, P, P, P, P, c_float, P, c_float, c_int, c_int,
                                    c_int, P]),
    "cvl_maxpool3x3s2_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_maxpool3x3s2_backward_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_upsample2x_add_f32": (c_int, [P, P, P, c_int, c_int, c_int, c_int, P]),
    "cvl_upsample2x_backward_f32": (c_int, [P, P, c_int, c_int, c_int, c_int, c_float, P]),
    "cvl_relu_backward_f32": (c_int, [P, P, P, ctypes.c_long, c_float, P]),
    "cvl_add_f32": (c_int, [P, P, P, ctypes.c_long, P]),
    "cvl_bias_grad_multi_f32": (c_int, [P, c_int, P]),
    "cvl_retina_loss_f32": (c_int, [P, c_int, P, c_int, P, c_int, P, c_int, c_int, P, c_float, P, P, c_int, P, c_int,
                                    P, P]),
}


class CvlError(RuntimeError):
    pass


_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CvlError("cvlite native library not built (%s): run __graft_entry__.build() or "
                           "make -C cv-lite-object-detection_amd/csrc" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        if os.environ.get("CVL_BN_EXACT", "0") == "1":      # the exact BN accumulator mode (bn_acc.h)
            lib.cvl_bn_set_exact(1)
    return _lib


def call(name, *args):
    """Calls a C entry point; raises on an error status."""
    st = getattr(load(), name)(*args)
    if st != 0:
        if st >= 1000:
            raise CvlError("%s failed: hipError %d" % (name, st - 1000))
        raise CvlError("%s: invalid argument (status %d)" % (name, st))
    return True


def ptr(t):
    return None if t is None else c_void_p(t.data_ptr())


def stream():
    return c_void_p(torch.cuda.current_stream().cuda_stream)


def require_cuda(*tensors):
    if not torch.cuda.is_available():
        raise CvlError("cvlite ops need an MI355X GPU (no CPU fallback)")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise CvlError("cvlite ops take device tensors")
        if t is not None and not t.is_contiguous():
            raise CvlError("cvlite ops take contiguous tensors")

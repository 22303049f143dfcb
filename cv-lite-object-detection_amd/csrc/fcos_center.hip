// FCOS-center target assignment on gfx950 — restates FCOS/fcos_center.py:149-317 (`format_data`,
// and, with the v1 switch, FCOS/fcos_center_v1.py:149-281's centroid-cell variant;
// the variant trained by train_fcos_center_voc.py with center_only=True): per level, the boxes of
// that size class (max(h, w) px against b_dim) are painted in ascending-area order onto the 3x3
// cells around int(centre * img_dim / stride + 0.5) (centre cell only when center_only); a cell's
// centerness is the max of 1.0 / 0.5 / 0.25 (centre / edge / corner neighbour), its ltrb box
// offsets (unclamped, stride units about the cell centre) come from the LAST box painted there,
// class bits are OR-ed.
//
// Every output cell is owned by one thread that walks its level's boxes in that order.  Box
// parameters are computed once per workgroup into LDS with the reference's fp32 operation
// sequence (numpy >= 2 scalar promotion; -ffp-contract=off), so the maps are bit-exact.
// Work: HBM-write bound, (5+C)*4 bytes per cell.
#include "cvl_common.h"

namespace {

constexpr int kBoxes = 256;
constexpr int kT = 256;
constexpr int kWords = 8;

struct CenterAssignArgs {
  const float* boxes;
  const int32_t* nbox;
  const float* img_dim;
  float* targets;
  int32_t* num_targets;
  int n_max, C, P, tiles, center_only;
  int v1;            // fcos_center_v1.py:149-281: centroid cell only, (off, size / box_sc) regression
  int stride[5], hmax[5], wmax[5], off[6];
  float bdim[4];
};

__global__ void __launch_bounds__(kT) fcos_center_assign_kernel(CenterAssignArgs a) {
  const int b = blockIdx.y;
  __shared__ float s_area[kBoxes];
  __shared__ int s_lev[kBoxes], s_ord[kBoxes], s_cls[kBoxes], s_yc[kBoxes], s_xc[kBoxes];
  __shared__ float s_c0[kBoxes], s_c1[kBoxes], s_c2[kBoxes], s_c3[kBoxes];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const float dh = a.img_dim[2 * b], dw = a.img_dim[2 * b + 1];
  for (int i = threadIdx.x; i < n; i += kT) {
    const float* g = a.boxes + ((size_t)b * a.n_max + i) * 5;
    const float gh = g[2] * dh, gw = g[3] * dw;                       // :165-166
    const float m = gw > gh ? gw : gh;
    int lev;
    if (m < a.bdim[0]) lev = 0;                                       // :180-191
    else if (m >= a.bdim[3]) lev = 4;
    else { lev = 1; while (lev < 3 && !(m < a.bdim[lev])) ++lev; }
    s_lev[i] = lev;
    s_area[i] = (g[2] * dh) * (g[3] * dw);                            // :210-212
    s_cls[i] = (int)g[4];
    const float st = (float)a.stride[lev];
    if (a.v1) {
      // fcos_center_v1.py:238-258 (fp32, numpy >= 2 promotion): raw centre, int(raw / stride),
      // offset (raw - cell*stride) / stride, size / box_sc
      const float ry = g[0] * dh, rx = g[1] * dw;
      const int yc = (int)(ry / st), xc = (int)(rx / st);
      s_yc[i] = yc;
      s_xc[i] = xc;
      const float sc = lev == 4 ? (dh > dw ? dh : dw) : a.bdim[lev];
      s_c0[i] = (ry - (float)(yc * a.stride[lev])) / st;
      s_c1[i] = (rx - (float)(xc * a.stride[lev])) / st;
      s_c2[i] = (g[2] * dh) / sc;
      s_c3[i] = (g[3] * dw) / sc;
    } else {
      const float hr = dh / st, wr = dw / st;                         // :174-175
      s_yc[i] = (int)(g[0] * hr + 0.5f);                              // :226-227
      s_xc[i] = (int)(g[1] * wr + 0.5f);
      s_c0[i] = ((g[0] - 0.5f * g[2]) * dh) / st;                     // :219-223, /stride at :254-258
      s_c1[i] = ((g[1] - 0.5f * g[3]) * dw) / st;
      s_c2[i] = ((g[0] + 0.5f * g[2]) * dh) / st;
      s_c3[i] = ((g[1] + 0.5f * g[3]) * dw) / st;
    }
  }
  __syncthreads();
  // rank of each box inside its level by (area, input index): the stable ascending order
  for (int i = threadIdx.x; i < n; i += kT) {
    int r = 0;
    for (int j = 0; j < n; ++j)
      r += (s_lev[j] == s_lev[i] && (s_area[j] < s_area[i] || (s_area[j] == s_area[i] && j < i))) ? 1 : 0;
    s_ord[i] = r;
  }
  __shared__ int s_pre[6], s_list[kBoxes];
  if (threadIdx.x == 0) {
    int cnt[5] = {0, 0, 0, 0, 0};
    for (int j = 0; j < n; ++j) ++cnt[s_lev[j]];
    s_pre[0] = 0;
    for (int l2 = 0; l2 < 5; ++l2) s_pre[l2 + 1] = s_pre[l2] + cnt[l2];
    if (blockIdx.x == 0)
      for (int l2 = 0; l2 < 5; ++l2) a.num_targets[b * 5 + l2] = cnt[l2];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += kT) s_list[s_pre[s_lev[i]] + s_ord[i]] = i;
  __syncthreads();
  const int p = blockIdx.x * kT + threadIdx.x;
  if (p >= a.P) return;
  int l = 0;
  while (l < 4 && p >= a.off[l + 1]) ++l;
  const int cell = p - a.off[l];
  const int y = cell / a.wmax[l], x = cell - (cell / a.wmax[l]) * a.wmax[l];
  float o0 = 0.f, o1 = 0.f, o2 = 0.f, o3 = 0.f, cen = 0.f;
  uint32_t bits[kWords] = {0, 0, 0, 0, 0, 0, 0, 0};
  int last = -1;
  for (int k = s_pre[l]; k < s_pre[l + 1]; ++k) {     // boxes of level l, ascending area
    const int i = s_list[k];
    const int yo = s_yc[i] - y, xo = s_xc[i] - x;                    // y_off / x_off (:250-251)
    const int lim = (a.center_only || a.v1) ? 0 : 1;
    if (yo < -lim || yo > lim || xo < -lim || xo > lim) continue;
    float sc;
    if (yo == 0 && xo == 0) sc = 1.0f;
    else if ((yo == 1 || yo == -1) && (xo == 1 || xo == -1)) sc = 0.25f;
    else sc = 0.5f;
    if (sc >= cen) cen = sc;                                          // :260-262
    last = i;
    const int c = s_cls[i];
    if (c >= 0 && c < a.C) bits[c >> 5] |= 1u << (c & 31);
  }
  if (last >= 0 && a.v1) {                                            // v1 :260-268 (last writer)
    o0 = s_c0[last];
    o1 = s_c1[last];
    o2 = s_c2[last];
    o3 = s_c3[last];
  } else if (last >= 0) {                                             // :264-269 (last writer)
    const float fy = (float)y, fx = (float)x;
    o0 = (fy + 0.5f) - s_c0[last];
    o1 = (s_c2[last] - fy) - 0.5f;
    o2 = (fx + 0.5f) - s_c1[last];
    o3 = (s_c3[last] - fx) - 0.5f;
  }
  float* t = a.targets + ((size_t)b * a.P + p) * (5 + a.C);
  t[0] = o0; t[1] = o1; t[2] = o2; t[3] = o3; t[4] = cen;
  for (int c = 0; c < a.C; ++c) t[5 + c] = (bits[c >> 5] >> (c & 31)) & 1u ? 1.0f : 0.0f;
}

}  // namespace

static int center_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max, int pad_h,
                         int pad_w, int num_classes, const int32_t* strides, const float* b_dim, int center_only,
                         int v1, float* targets, int32_t* num_targets, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && img_dim && strides && b_dim && targets && num_targets);
  CVL_CHECK_ARG(B > 0 && n_max > 0 && n_max <= kBoxes && num_classes > 0 && num_classes <= 32 * kWords);
  CVL_CHECK_ARG(pad_h > 0 && pad_w > 0);
  CenterAssignArgs a;
  a.boxes = boxes; a.nbox = nbox; a.img_dim = img_dim; a.targets = targets; a.num_targets = num_targets;
  a.n_max = n_max; a.C = num_classes; a.center_only = center_only ? 1 : 0; a.v1 = v1;
  a.off[0] = 0;
  for (int l = 0; l < 5; ++l) {
    CVL_CHECK_ARG(strides[l] > 0);
    a.stride[l] = strides[l];
    a.hmax[l] = pad_h / strides[l];                                   // int(img_pad / stride)
    a.wmax[l] = pad_w / strides[l];
    CVL_CHECK_ARG(a.hmax[l] > 0 && a.wmax[l] > 0);
    a.off[l + 1] = a.off[l] + a.hmax[l] * a.wmax[l];
  }
  for (int k = 0; k < 4; ++k) a.bdim[k] = b_dim[k];
  a.P = a.off[5];
  a.tiles = (a.P + kT - 1) / kT;
  hipLaunchKernelGGL(fcos_center_assign_kernel, dim3(a.tiles, B), dim3(kT), 0, (hipStream_t)stream, a);
  return cvl_launch_status();
}

extern "C" int cvl_fcos_center_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B,
                                      int n_max, int pad_h, int pad_w, int num_classes, const int32_t* strides,
                                      const float* b_dim, int center_only, float* targets, int32_t* num_targets,
                                      cvl_stream_t stream) {
  return center_assign(boxes, nbox, img_dim, B, n_max, pad_h, pad_w, num_classes, strides, b_dim, center_only, 0,
                       targets, num_targets, stream);
}

extern "C" int cvl_fcos_center_v1_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B,
                                         int n_max, int pad_h, int pad_w, int num_classes, const int32_t* strides,
                                         const float* b_dim, float* targets, int32_t* num_targets,
                                         cvl_stream_t stream) {
  return center_assign(boxes, nbox, img_dim, B, n_max, pad_h, pad_w, num_classes, strides, b_dim, 1, 1, targets,
                       num_targets, stream);
}

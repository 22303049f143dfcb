// RetinaNet inference decode on MI355X (RetinaNet/retinanet_module.py:428-529):
//   cvl_retina_corners   prediction_to_corners (:428-451) for one (level, anchor) map
//   cvl_retina_decode    image_detections (:483-520) up to the NMS call: corners of every
//                        (level, anchor, cell), sigmoid class probabilities, per-row max / first
//                        argmax, `score >= cls_thresh`, rows compacted in the reference's order
//   cvl_retina_nms       cpu_nms (:453-481): greedy, class-agnostic, score-descending
//   cvl_fcos_detect      FCOS/infer_fcos.py:27-62 image_detections: corners, sigmoid scores and
//                        tf.image.combined_non_max_suppression (restated; TF is absent here)
//
// Arithmetic follows the reference's fp32 operation sequence (this file is built with
// -ffp-contract=off): anchor dims are fp32 (tf.math.sqrt of a python float, :207-209), the grid is
// a fp32 tf.range, so every corner is fl(fl(g * stride) - fl(t * a)) -+ fl(fl(t' * a') / 2) in
// fp32.  The sigmoid is evaluated in float64 and rounded to fp32 (TF's own fp32 kernel is an
// implementation detail outside this image: ulp-level parity unpinned, as for CenterNet).
//
// Layout: the model's fused head outputs, row (level offset + cell) of [B][P][ld] with anchor a
// at box channels 4a..4a+3 (t_y, t_x, t_h, t_w) and class channels aC..aC+C-1.  Output rows are
// numbered in the reference's concatenation order: level-major, anchor, then cell (row-major).
#include "cvl_common.h"

namespace {

constexpr int DT = 256;            // decode workgroup
constexpr int MT = 1024;           // NMS workgroup (one per image)

struct DecodeArgs {
  const float* reg;
  const float* cls;
  const float* adims;              // [5][A][2] (h, w) fp32
  float* rows;                     // workspace [B][R][6]
  int32_t* tile_cnt;               // workspace [B][tiles]
  uint8_t* flag;                   // workspace [B][R]
  float* dets;                     // [B][R][6]
  int32_t* count;                  // [B]
  int ld_reg, ld_cls, A, C, P, R, tiles;
  int h[5], w[5], stride[5], off[6], roff[6];
  float thresh;
};

__device__ __forceinline__ void corners(float ty, float tx, float th, float tw, int y, int x, int stride,
                                        float ah, float aw, float* o) {
  const float fs = (float)stride;
  const float xc = (float)x * fs - tx * aw;             // pred_x_cen (:441)
  const float yc = (float)y * fs - ty * ah;             // pred_y_cen (:442)
  const float bw = tw * aw, bh = th * ah;               // (:443-444)
  const float hh = bh / 2.0f, hw = bw / 2.0f;
  o[0] = yc - hh;                                       // (:446-449)
  o[2] = yc + hh;
  o[1] = xc - hw;
  o[3] = xc + hw;
}

__global__ void __launch_bounds__(DT) corners_kernel(const float* xy, int ld, int H, int W, float ah, float aw,
                                                     int stride, float* out) {
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= H * W) return;
  const float* p = xy + (size_t)i * ld;
  const int y = i / W, x = i - (i / W) * W;
  float o[4];
  corners(p[0], p[1], p[2], p[3], y, x, stride, ah, aw, o);
  float4 v;
  v.x = o[0]; v.y = o[1]; v.z = o[2]; v.w = o[3];
  reinterpret_cast<float4*>(out)[i] = v;
}

// Pass 1: every output row of image blockIdx.y -> its 6 values + keep flag; per-tile counts.
__global__ void __launch_bounds__(DT) retina_decode_rows(DecodeArgs a) {
  const int b = blockIdx.y;
  const int r = blockIdx.x * DT + threadIdx.x;
  bool keep = false;
  if (r < a.R) {
    int l = 0;
    while (l < 4 && r >= a.roff[l + 1]) ++l;
    const int hw = a.h[l] * a.w[l];
    const int rl = r - a.roff[l];
    const int an = rl / hw, cell = rl - an * hw;
    const int y = cell / a.w[l], x = cell - (cell / a.w[l]) * a.w[l];
    const size_t prow = (size_t)b * a.P + a.off[l] + cell;
    const float* rp = a.reg + prow * a.ld_reg + 4 * an;
    const float* cp = a.cls + prow * a.ld_cls + (size_t)an * a.C;
    const float* ad = a.adims + ((size_t)l * a.A + an) * 2;
    float o[6];
    corners(rp[0], rp[1], rp[2], rp[3], y, x, a.stride[l], ad[0], ad[1], o);
    float pmax = 0.f;
    int lab = 0;
    for (int c = 0; c < a.C; ++c) {
      const float pr = (float)(1.0 / (1.0 + exp(-(double)cp[c])));
      if (c == 0 || pr > pmax) { pmax = pr; lab = c; }      // tf.math.argmax: first maximum
    }
    o[4] = pmax;
    o[5] = (float)lab;
    keep = pmax >= a.thresh;
    float* dst = a.rows + ((size_t)b * a.R + r) * 6;
    for (int k = 0; k < 6; ++k) dst[k] = o[k];
    a.flag[(size_t)b * a.R + r] = keep ? 1 : 0;
  }
  __shared__ int wc[DT / 64];
  const unsigned long long m = __ballot(keep);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int k = 0; k < DT / 64; ++k) s += wc[k];
    a.tile_cnt[(size_t)b * a.tiles + blockIdx.x] = s;
  }
}

// Pass 2: ordered compaction (tile prefix from the per-tile counts + in-tile ballot prefix).
__global__ void __launch_bounds__(DT) retina_decode_compact(DecodeArgs a) {
  const int b = blockIdx.y;
  const int* cnt = a.tile_cnt + (size_t)b * a.tiles;
  __shared__ int part[DT];
  __shared__ int wc[DT / 64];
  int s = 0, tot = 0;
  for (int t = threadIdx.x; t < a.tiles; t += DT) {
    const int c = cnt[t];
    tot += c;
    if (t < (int)blockIdx.x) s += c;
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = DT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
    __syncthreads();
  }
  const int base = part[0];
  __syncthreads();
  if (blockIdx.x == 0) {
    part[threadIdx.x] = tot;
    __syncthreads();
    for (int o = DT / 2; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) a.count[b] = part[0];
  }
  const int r = blockIdx.x * DT + threadIdx.x;
  const bool keep = r < a.R && a.flag[(size_t)b * a.R + r];
  const unsigned long long m = __ballot(keep);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) wc[wv] = __popcll(m);
  __syncthreads();
  if (keep) {
    int off = base + __popcll(m & ((1ull << lane) - 1ull));
    for (int k = 0; k < wv; ++k) off += wc[k];
    const float* src = a.rows + ((size_t)b * a.R + r) * 6;
    float* dst = a.dets + ((size_t)b * a.R + off) * 6;
    for (int k = 0; k < 6; ++k) dst[k] = src[k];
  }
}

// cpu_nms over image blockIdx.x's first count[b] rows: repeatedly select the highest score among
// the survivors (lowest row among equal scores: the reference's np.argsort(-scores) is an
// unstable quicksort, so its tie order is unspecified -- Q1-style, ties are avoided in the
// goldens), then keep only survivors with ovr <= thr, ovr = inter / (((a_i + a_j) - inter) + 1e-8)
// in fp32 (:466-478; NaN overlaps are dropped, as `ovr <= thr` is false for them).
__global__ void __launch_bounds__(MT) retina_nms_kernel(const float* dets, int rows_per_img, const int32_t* count,
                                                        int n_cap, float thr, int32_t* keep, int32_t* nkeep,
                                                        uint8_t* alive_ws) {
  const int b = blockIdx.x;
  int n = count[b];
  n = n < n_cap ? n : n_cap;
  const float* D = dets + (size_t)b * rows_per_img * 6;
  uint8_t* alive = alive_ws + (size_t)b * n_cap;
  int32_t* kp = keep + (size_t)b * n_cap;
  for (int i = threadIdx.x; i < n; i += MT) alive[i] = 1;
  __shared__ float bs[MT / 64];
  __shared__ int bi[MT / 64];
  __shared__ int sel;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int cnt = 0;
  __syncthreads();
  for (;;) {
    float s = -INFINITY;
    int si = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += MT) {
      if (!alive[i]) continue;
      const float sc = D[(size_t)i * 6 + 4];
      if (sc > s) { s = sc; si = i; }                   // i ascends: first maximum per thread
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float s2 = __shfl_xor(s, o);
      const int i2 = __shfl_xor(si, o);
      if (s2 > s || (s2 == s && i2 < si)) { s = s2; si = i2; }
    }
    if (lane == 0) { bs[wv] = s; bi[wv] = si; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float s0 = bs[0];
      int i0 = bi[0];
      for (int k = 1; k < MT / 64; ++k)
        if (bs[k] > s0 || (bs[k] == s0 && bi[k] < i0)) { s0 = bs[k]; i0 = bi[k]; }
      sel = (i0 == 0x7fffffff) ? -1 : i0;
      if (sel >= 0) { kp[cnt] = sel; alive[sel] = 0; }
    }
    __syncthreads();
    const int q = sel;
    if (q < 0) break;
    ++cnt;
    const float* Q = D + (size_t)q * 6;
    const float qx1 = Q[0], qy1 = Q[1], qx2 = Q[2], qy2 = Q[3];
    const float qa = (qx2 - qx1) * (qy2 - qy1);
    for (int i = threadIdx.x; i < n; i += MT) {
      if (!alive[i]) continue;
      const float* Rr = D + (size_t)i * 6;
      const float ra = (Rr[2] - Rr[0]) * (Rr[3] - Rr[1]);
      const float xx1 = fmaxf(qx1, Rr[0]), yy1 = fmaxf(qy1, Rr[1]);
      const float xx2 = fminf(qx2, Rr[2]), yy2 = fminf(qy2, Rr[3]);
      const float w = fmaxf(0.0f, xx2 - xx1), h = fmaxf(0.0f, yy2 - yy1);
      const float inter = w * h;
      const float ovr = inter / (((qa + ra) - inter) + 1e-8f);
      if (!(ovr <= thr)) alive[i] = 0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) nkeep[b] = cnt;
}

// ------------------------------------------------------------------------------------------------
// FCOS inference (FCOS/infer_fcos.py:27-62): boxes = fcos.prediction_to_corners (fp32 grid + 0.5
// -+ t, times the python-int stride in float64, stored back into the fp32 output array),
// scores = sigmoid(cls) (or sigmoid(centerness) * sigmoid(cls) with center=True), then
// tf.image.combined_non_max_suppression (q = 1 shared boxes, clip_boxes=False): per class,
// candidates with score > score_threshold, greedy by score, a candidate is selected iff no
// already-selected box of its class has IoU > iou_threshold (TF's IOUGreaterThanThreshold: corners
// normalised with min/max, a non-positive area never suppresses), at most max_per_class per class;
// then every class's selections merged by descending score, the first max_total kept, rest zero.
// TF's priority queue and std::sort leave equal-score order unspecified: here lower box index
// (per class) and then lower class / earlier selection (merge) win.
// ------------------------------------------------------------------------------------------------
constexpr int FT = 1024;
constexpr int kMaxCells = 16384;           // P held in LDS by the per-class NMS (scores + flags)

struct FcosDetArgs {
  const float* reg;                        // [B][P][ld_reg] (t, b, l, r, centerness)
  const float* cls;                        // [B][P][ld_cls]
  float* boxes;                            // workspace [B][P][4]
  float* sel_score;                        // workspace [B][C][mpc]
  int32_t* sel_idx;                        // workspace [B][C][mpc]
  int32_t* sel_n;                          // workspace [B][C]
  float* out_boxes;                        // [B][max_total][4]
  float* out_scores;                       // [B][max_total]
  float* out_classes;                      // [B][max_total]
  int32_t* valid;                          // [B]
  int ld_reg, ld_cls, C, P, center, mpc, max_total;
  int h[5], w[5], stride[5], off[6];
  float iou, thr;
};

__global__ void __launch_bounds__(DT) fcos_boxes_kernel(FcosDetArgs a) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * DT + threadIdx.x;
  if (i >= a.P) return;
  int l = 0;
  while (l < 4 && i >= a.off[l + 1]) ++l;
  const int cell = i - a.off[l];
  const int y = cell / a.w[l], x = cell - (cell / a.w[l]) * a.w[l];
  const float* q = a.reg + ((size_t)b * a.P + i) * a.ld_reg;
  const float gy = (float)y + 0.5f, gx = (float)x + 0.5f;
  const double st = (double)a.stride[l];
  float4 v;
  v.x = (float)(st * (double)(gy - q[0]));
  v.y = (float)(st * (double)(gx - q[2]));
  v.z = (float)(st * (double)(gy + q[1]));
  v.w = (float)(st * (double)(gx + q[3]));
  reinterpret_cast<float4*>(a.boxes)[(size_t)b * a.P + i] = v;
}

__device__ __forceinline__ float sigm(float x) { return (float)(1.0 / (1.0 + exp(-(double)x))); }

__device__ __forceinline__ bool iou_gt(float4 bi, float4 bj, float thr) {
  const float ymin_i = fminf(bi.x, bi.z), xmin_i = fminf(bi.y, bi.w);
  const float ymax_i = fmaxf(bi.x, bi.z), xmax_i = fmaxf(bi.y, bi.w);
  const float ymin_j = fminf(bj.x, bj.z), xmin_j = fminf(bj.y, bj.w);
  const float ymax_j = fmaxf(bj.x, bj.z), xmax_j = fmaxf(bj.y, bj.w);
  const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
  const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
  if (area_i <= 0.f || area_j <= 0.f) return false;
  const float iy = fmaxf(fminf(ymax_i, ymax_j) - fmaxf(ymin_i, ymin_j), 0.0f);
  const float ix = fmaxf(fminf(xmax_i, xmax_j) - fmaxf(xmin_i, xmin_j), 0.0f);
  const float inter = iy * ix;
  return inter / (area_i + area_j - inter) > thr;
}

// One workgroup per (class, image): scores of the class staged in LDS (-inf = not a candidate).
__global__ void __launch_bounds__(FT) fcos_class_nms_kernel(FcosDetArgs a) {
  const int c = blockIdx.x, b = blockIdx.y;
  __shared__ float sc[kMaxCells];
  __shared__ float bs[FT / 64];
  __shared__ int bi[FT / 64];
  __shared__ int sel;
  const float4* B4 = reinterpret_cast<const float4*>(a.boxes) + (size_t)b * a.P;
  for (int i = threadIdx.x; i < a.P; i += FT) {
    const size_t row = (size_t)b * a.P + i;
    float s = sigm(a.cls[row * a.ld_cls + c]);
    if (a.center) s = sigm(a.reg[row * a.ld_reg + 4]) * s;
    sc[i] = s > a.thr ? s : -INFINITY;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t so = ((size_t)b * a.C + c) * a.mpc;
  int n = 0;
  __syncthreads();
  while (n < a.mpc) {
    float s = -INFINITY;
    int si = 0x7fffffff;
    for (int i = threadIdx.x; i < a.P; i += FT)
      if (sc[i] > s) { s = sc[i]; si = i; }
    for (int o = 32; o > 0; o >>= 1) {
      const float s2 = __shfl_xor(s, o);
      const int i2 = __shfl_xor(si, o);
      if (s2 > s || (s2 == s && i2 < si)) { s = s2; si = i2; }
    }
    if (lane == 0) { bs[wv] = s; bi[wv] = si; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float s0 = bs[0];
      int i0 = bi[0];
      for (int k = 1; k < FT / 64; ++k)
        if (bs[k] > s0 || (bs[k] == s0 && bi[k] < i0)) { s0 = bs[k]; i0 = bi[k]; }
      sel = (s0 == -INFINITY) ? -1 : i0;
      if (sel >= 0) {
        a.sel_score[so + n] = s0;
        a.sel_idx[so + n] = i0;
        sc[i0] = -INFINITY;
      }
    }
    __syncthreads();
    const int q = sel;
    if (q < 0) break;
    ++n;
    const float4 bq = B4[q];
    for (int i = threadIdx.x; i < a.P; i += FT)
      if (sc[i] != -INFINITY && iou_gt(B4[i], bq, a.iou)) sc[i] = -INFINITY;
    __syncthreads();
  }
  if (threadIdx.x == 0) a.sel_n[(size_t)b * a.C + c] = n;
}

// Merge per image: each selection's rank under (score desc, class asc, selection order asc);
// ranks < max_total are written to their slot, the remaining slots are zero.
__global__ void __launch_bounds__(FT) fcos_merge_kernel(FcosDetArgs a) {
  const int b = blockIdx.x;
  const int N = a.C * a.mpc;
  const float* S = a.sel_score + (size_t)b * N;
  const int32_t* ns = a.sel_n + (size_t)b * a.C;
  __shared__ int tot_s;
  if (threadIdx.x == 0) {
    int t = 0;
    for (int c = 0; c < a.C; ++c) t += ns[c];
    tot_s = t;
  }
  for (int k = threadIdx.x; k < a.max_total; k += FT) {
    float* ob = a.out_boxes + ((size_t)b * a.max_total + k) * 4;
    ob[0] = ob[1] = ob[2] = ob[3] = 0.f;
    a.out_scores[(size_t)b * a.max_total + k] = 0.f;
    a.out_classes[(size_t)b * a.max_total + k] = 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < N; e += FT) {
    const int c = e / a.mpc, k = e - c * a.mpc;
    if (k >= ns[c]) continue;
    const float s = S[e];
    int rank = 0;
    for (int c2 = 0; c2 < a.C && rank < a.max_total; ++c2) {
      const int n2 = ns[c2];
      const float* S2 = S + (size_t)c2 * a.mpc;
      for (int k2 = 0; k2 < n2; ++k2) {
        const float t = S2[k2];
        rank += (t > s || (t == s && (c2 < c || (c2 == c && k2 < k)))) ? 1 : 0;
      }
    }
    if (rank < a.max_total) {
      const float4 bx = reinterpret_cast<const float4*>(a.boxes)[(size_t)b * a.P + a.sel_idx[(size_t)b * N + e]];
      float* ob = a.out_boxes + ((size_t)b * a.max_total + rank) * 4;
      ob[0] = bx.x; ob[1] = bx.y; ob[2] = bx.z; ob[3] = bx.w;
      a.out_scores[(size_t)b * a.max_total + rank] = s;
      a.out_classes[(size_t)b * a.max_total + rank] = (float)c;
    }
  }
  if (threadIdx.x == 0) a.valid[b] = tot_s < a.max_total ? tot_s : a.max_total;
}

bool fill_levels(DecodeArgs& a, const int32_t* level_hw, const int32_t* strides, int A) {
  a.off[0] = 0;
  a.roff[0] = 0;
  for (int l = 0; l < 5; ++l) {
    if (level_hw[2 * l] <= 0 || level_hw[2 * l + 1] <= 0) return false;
    if (strides && strides[l] <= 0) return false;
    a.h[l] = level_hw[2 * l];
    a.w[l] = level_hw[2 * l + 1];
    a.stride[l] = strides ? strides[l] : 0;
    const long hw = (long)a.h[l] * a.w[l];
    a.off[l + 1] = a.off[l] + (int)hw;
    if ((long)a.roff[l] + hw * A > 0x7fffffffL / 8) return false;
    a.roff[l + 1] = a.roff[l] + (int)(hw * A);
  }
  a.P = a.off[5];
  a.R = a.roff[5];
  a.tiles = (a.R + DT - 1) / DT;
  return true;
}

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

#define S_ ((hipStream_t)stream)

extern "C" int cvl_retina_corners(const float* xy, int ld, int H, int W, float anchor_h, float anchor_w, int stride,
                                  float* out, cvl_stream_t stream) {
  CVL_CHECK_ARG(xy && out && H > 0 && W > 0 && ld >= 4 && stride > 0);
  hipLaunchKernelGGL(corners_kernel, dim3((H * W + DT - 1) / DT), dim3(DT), 0, S_, xy, ld, H, W, anchor_h,
                     anchor_w, stride, out);
  return cvl_launch_status();
}

extern "C" size_t cvl_retina_decode_workspace_size(int B, const int32_t* level_hw, int n_anchors) {
  DecodeArgs a;
  if (B <= 0 || n_anchors <= 0 || !level_hw || !fill_levels(a, level_hw, nullptr, n_anchors)) return 0;
  return align256((size_t)B * a.R * 6 * sizeof(float)) + align256((size_t)B * a.tiles * sizeof(int32_t)) +
         align256((size_t)B * a.R);
}

extern "C" int cvl_retina_decode(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, int B,
                                 const int32_t* level_hw, const int32_t* strides, const float* anchor_dims,
                                 int n_anchors, int num_classes, float cls_thresh, float* dets, int32_t* count,
                                 void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(reg_pred && cls_pred && level_hw && strides && anchor_dims && dets && count && workspace);
  CVL_CHECK_ARG(B > 0 && n_anchors > 0 && num_classes > 0);
  CVL_CHECK_ARG(ld_reg >= 4 * n_anchors && ld_cls >= n_anchors * num_classes);
  DecodeArgs a;
  CVL_CHECK_ARG(fill_levels(a, level_hw, strides, n_anchors));
  CVL_CHECK_ARG(workspace_bytes >= cvl_retina_decode_workspace_size(B, level_hw, n_anchors));
  a.reg = reg_pred; a.cls = cls_pred; a.adims = anchor_dims; a.dets = dets; a.count = count;
  a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.A = n_anchors; a.C = num_classes; a.thresh = cls_thresh;
  char* ws = (char*)workspace;
  a.rows = (float*)ws;
  ws += align256((size_t)B * a.R * 6 * sizeof(float));
  a.tile_cnt = (int32_t*)ws;
  ws += align256((size_t)B * a.tiles * sizeof(int32_t));
  a.flag = (uint8_t*)ws;
  hipLaunchKernelGGL(retina_decode_rows, dim3(a.tiles, B), dim3(DT), 0, S_, a);
  hipLaunchKernelGGL(retina_decode_compact, dim3(a.tiles, B), dim3(DT), 0, S_, a);
  return cvl_launch_status();
}

extern "C" size_t cvl_retina_nms_workspace_size(int B, int n_cap) {
  return B > 0 && n_cap > 0 ? align256((size_t)B * n_cap) : 0;
}

extern "C" int cvl_retina_nms(const float* dets, int rows_per_img, const int32_t* count, int B, int n_cap,
                              float iou_thresh, int32_t* keep, int32_t* nkeep, void* workspace, cvl_stream_t stream) {
  CVL_CHECK_ARG(dets && count && keep && nkeep && workspace && B > 0 && n_cap > 0 && rows_per_img >= n_cap);
  hipLaunchKernelGGL(retina_nms_kernel, dim3(B), dim3(MT), 0, S_, dets, rows_per_img, count, n_cap, iou_thresh,
                     keep, nkeep, (uint8_t*)workspace);
  return cvl_launch_status();
}

extern "C" size_t cvl_fcos_detect_workspace_size(int B, int P, int num_classes, int max_per_class) {
  if (B <= 0 || P <= 0 || num_classes <= 0 || max_per_class <= 0) return 0;
  const size_t sel = (size_t)B * num_classes * max_per_class;
  return align256((size_t)B * P * 4 * sizeof(float)) + align256(sel * sizeof(float)) +
         align256(sel * sizeof(int32_t)) + align256((size_t)B * num_classes * sizeof(int32_t));
}

extern "C" int cvl_fcos_detect(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls, int B,
                               const int32_t* level_hw, const int32_t* strides, int num_classes, int center,
                               float iou_thresh, float score_thresh, int max_per_class, int max_total,
                               float* out_boxes, float* out_scores, float* out_classes, int32_t* valid,
                               void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(reg_pred && cls_pred && level_hw && strides && out_boxes && out_scores && out_classes && valid &&
                workspace);
  CVL_CHECK_ARG(B > 0 && num_classes > 0 && ld_reg >= 5 && ld_cls >= num_classes && max_per_class > 0 &&
                max_total > 0);
  FcosDetArgs a;
  a.off[0] = 0;
  for (int l = 0; l < 5; ++l) {
    CVL_CHECK_ARG(level_hw[2 * l] > 0 && level_hw[2 * l + 1] > 0 && strides[l] > 0);
    a.h[l] = level_hw[2 * l];
    a.w[l] = level_hw[2 * l + 1];
    a.stride[l] = strides[l];
    a.off[l + 1] = a.off[l] + a.h[l] * a.w[l];
  }
  a.P = a.off[5];
  CVL_CHECK_ARG(a.P <= kMaxCells);
  a.mpc = max_per_class < a.P ? max_per_class : a.P;      // TF: min(max_output_size_per_class, boxes)
  CVL_CHECK_ARG(workspace_bytes >= cvl_fcos_detect_workspace_size(B, a.P, num_classes, a.mpc));
  a.reg = reg_pred; a.cls = cls_pred; a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.C = num_classes;
  a.center = center; a.max_total = max_total; a.iou = iou_thresh; a.thr = score_thresh;
  a.out_boxes = out_boxes; a.out_scores = out_scores; a.out_classes = out_classes; a.valid = valid;
  const size_t sel = (size_t)B * num_classes * a.mpc;
  char* ws = (char*)workspace;
  a.boxes = (float*)ws;
  ws += align256((size_t)B * a.P * 4 * sizeof(float));
  a.sel_score = (float*)ws;
  ws += align256(sel * sizeof(float));
  a.sel_idx = (int32_t*)ws;
  ws += align256(sel * sizeof(int32_t));
  a.sel_n = (int32_t*)ws;
  hipLaunchKernelGGL(fcos_boxes_kernel, dim3((a.P + DT - 1) / DT, B), dim3(DT), 0, S_, a);
  hipLaunchKernelGGL(fcos_class_nms_kernel, dim3(num_classes, B), dim3(FT), 0, S_, a);
  hipLaunchKernelGGL(fcos_merge_kernel, dim3(B), dim3(FT), 0, S_, a);
  return cvl_launch_status();
}

// ---------------------------------------------------------------------------------------------
// CenterNet 3x3 max-pool peak decode (BASELINE north_star's "3x3 max-pool peak decode"; the
// reference itself thresholds every cell's max class probability and runs NMS,
// tf_centernet_hourglass.py:566-656 = cvl_centernet_decode).  Standard CenterNet form on the same
// model output [B][H][W][ld] (ltrb 0..3, class logits 4..4+C): a (cell, class) is a peak when its
// sigmoid probability equals the 3x3 max-pool of that class map (-inf padding: ties keep every
// equal cell), and it is kept when the probability >= thresh.  The K highest (probability, then
// lower flat index cell*C + class) peaks of each image become rows (y_lo, x_lo, y_hi, x_hi, prob,
// class) with the corners of prediction_to_corners (:355-377) in fp32 times `stride`.
// Pass 1 (one thread per (cell, class)) appends 64-bit keys (ordered probability bits << 32 |
// ~flat index) to a per-image list; pass 2 (one workgroup per image) takes the K largest keys in
// K rounds of a block max below the previous key -- keys are unique, so the result is independent
// of the append order (deterministic).  No parity anchor exists in the reference: pinned to the
// numpy restatement (oracle/centernet_peak_ref.py), parity unpinned at the reference level.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int PK = 1024;

__device__ __forceinline__ float cn_sigmoid(float v) { return (float)(1.0 / (1.0 + exp(-(double)v))); }

__global__ void __launch_bounds__(DT) peak_candidates_kernel(const float* __restrict__ pred, int ld, int H, int W,
                                                             int C, float thresh, unsigned long long* keys,
                                                             int32_t* n_keys) {
  const long per = (long)H * W * C;
  const long i = (long)blockIdx.x * DT + threadIdx.x;
  const int b = blockIdx.y;
  if (i >= per) return;
  const int c = (int)(i % C);
  const int cell = (int)(i / C);
  const int y = cell / W, x = cell % W;
  const float* img = pred + (long)b * H * W * ld;
  const float p = cn_sigmoid(img[(long)cell * ld + 4 + c]);
  if (!(p >= thresh)) return;
  for (int dy = -1; dy <= 1; ++dy)
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = y + dy, xx = x + dx;
      if ((dy == 0 && dx == 0) || yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
      if (cn_sigmoid(img[((long)yy * W + xx) * ld + 4 + c]) > p) return;
    }
  const int slot = atomicAdd(n_keys + b, 1);
  // probabilities are in [0, 1]: their fp32 bit patterns order as unsigned integers
  keys[(long)b * per + slot] = ((unsigned long long)__float_as_uint(p) << 32) | (unsigned)(~(unsigned)i);
}

__global__ void __launch_bounds__(PK) peak_select_kernel(const float* __restrict__ pred, int ld, int H, int W, int C,
                                                         float stride, int K, const unsigned long long* keys,
                                                         const int32_t* n_keys, double* dets, int32_t* count) {
  const int b = blockIdx.x;
  const long per = (long)H * W * C;
  const int n = n_keys[b];
  const unsigned long long* kb = keys + (long)b * per;
  __shared__ unsigned long long red[PK / 64];
  __shared__ unsigned long long sel;
  unsigned long long prev = ~0ull;
  const int kk = n < K ? n : K;
  for (int r = 0; r < kk; ++r) {
    unsigned long long m = 0;
    for (int j = threadIdx.x; j < n; j += PK) {
      const unsigned long long v = kb[j];
      if (v < prev && v > m) m = v;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned long long v = __shfl_xor(m, o);
      m = v > m ? v : m;
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = red[0];
      for (int w = 1; w < PK / 64; ++w) t = red[w] > t ? red[w] : t;
      sel = t;
      const unsigned idx = ~(unsigned)(t & 0xffffffffull);
      const int c = (int)(idx % (unsigned)C), cell = (int)(idx / (unsigned)C);
      const int y = cell / W, x = cell % W;
      const float* q = pred + ((long)b * H * W + cell) * ld;
      const float gy = (float)y + 0.5f, gx = (float)x + 0.5f;
      double* o = dets + ((long)b * K + r) * 6;
      o[0] = (double)(stride * (gy - q[0]));
      o[1] = (double)(stride * (gx - q[2]));
      o[2] = (double)(stride * (gy + q[1]));
      o[3] = (double)(stride * (gx + q[3]));
      o[4] = (double)__uint_as_float((unsigned)(t >> 32));
      o[5] = (double)c;
    }
    __syncthreads();
    prev = sel;
    __syncthreads();
  }
  if (threadIdx.x == 0) count[b] = kk;
}

}  // namespace

extern "C" size_t cvl_centernet_peak_decode_workspace_size(int B, int H, int W, int num_classes) {
  return (size_t)B * H * W * num_classes * sizeof(unsigned long long) + (size_t)B * sizeof(int32_t) + 256;
}

extern "C" int cvl_centernet_peak_decode(const float* pred, int ld, int B, int H, int W, int num_classes,
                                         float stride, float thresh, int K, double* dets, int32_t* count,
                                         void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && dets && count && workspace && B > 0 && H > 0 && W > 0 && num_classes > 0 && K > 0);
  CVL_CHECK_ARG(ld >= 4 + num_classes);
  CVL_CHECK_ARG(workspace_bytes >= cvl_centernet_peak_decode_workspace_size(B, H, W, num_classes));
  CVL_CHECK_ARG((long)H * W * num_classes < 0x7fffffffL);
  hipStream_t s = (hipStream_t)stream;
  unsigned long long* keys = reinterpret_cast<unsigned long long*>(workspace);
  int32_t* nk = reinterpret_cast<int32_t*>(keys + (size_t)B * H * W * num_classes);
  if (hipMemsetAsync(nk, 0, sizeof(int32_t) * B, s) != hipSuccess) return cvl_launch_status();
  const long per = (long)H * W * num_classes;
  hipLaunchKernelGGL(peak_candidates_kernel, dim3((unsigned)((per + DT - 1) / DT), B), dim3(DT), 0, s, pred, ld, H,
                     W, num_classes, thresh, keys, nk);
  int st = cvl_launch_status();
  if (st) return st;
  hipLaunchKernelGGL(peak_select_kernel, dim3(B), dim3(PK), 0, s, pred, ld, H, W, num_classes, stride, K, keys, nk,
                     dets, count);
  return cvl_launch_status();
}

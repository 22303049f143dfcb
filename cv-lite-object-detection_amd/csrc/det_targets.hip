// RetinaNet anchor matching, CenterNet centroid targets and centre splat, the shared
// focal + masked smooth-L1 loss, and greedy per-class NMS on gfx950.
//
//   cvl_retina_assign    RetinaNet/retinanet_module.py:205-365 + RetinaNet/utils.py:42-83
//   cvl_centernet_assign CenterNet/tf_centernet_hourglass.py:379-456
//   cvl_centernet_splat  CenterNet/tf_centernet.py:6-19, 152-342
//   cvl_det_loss         tf_centernet_hourglass.py:458-505 / retinanet_module.py:367-426
//   cvl_nms              tf_centernet_hourglass.py:22-85 (method 'nms')
//   cvl_hourglass_v2_*   CenterNet/train_hourglass_voc.py:96-160, tf_hourglass_net.py:398-447
//   cvl_centernet_s8_*   CenterNet/tf_centernet_resnet_s8.py:243-385
// Index/target kernels follow the reference's fp32 operation sequences exactly (this file is
// compiled with -ffp-contract=off) and keep float64 where the reference computes in float64.
#include "cvl_common.h"

namespace {

constexpr int NT = 256;
constexpr int RT = 128;                   // retina_assign block (LDS stage of 128 rows x (4+C))
constexpr int kMaxBox = 256;
constexpr int kWords = 8;                  // class bitmask words (C <= 256)

__device__ __forceinline__ float relu0(float v) { return v > 0.f ? v : 0.f; }

// ------------------------------------------------------------------------------------------------
// RetinaNet: output [B][sum_l A*S_l^2][4+C] ordered (level, anchor, u, v); cell (u, v) of level l
// is the anchor centred at (u*s, v*s) with dims (h_a, w_a) (the reference builds its grid as
// (col, row) and writes it back transposed, Q21: self-consistent for square maps).
// ------------------------------------------------------------------------------------------------
struct RetinaArgs {
  const float* boxes;
  const int32_t* nbox;
  const float* img_dim;
  const float* adims;      // [5][A][2] fp32 (h, w)
  float* out;
  int32_t* ntgt;
  int n_max, C, A, P, pad;
  float thresh;
  int S[5], stride[5], off[6];
};

__global__ void __launch_bounds__(RT) retina_assign_kernel(RetinaArgs a) {
  const int b = blockIdx.y;
  const int p0 = blockIdx.x * RT;
  const int tid = threadIdx.x;
  const int row = 4 + a.C;
  __shared__ float gy[kMaxBox], gx[kMaxBox], gh[kMaxBox], gw[kMaxBox], ga[kMaxBox], lo0[kMaxBox],
      lo1[kMaxBox], hi0[kMaxBox], hi1[kMaxBox];
  __shared__ int gc[kMaxBox];
  __shared__ int cnt;
  extern __shared__ __attribute__((aligned(16))) float stage[];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const float H = a.img_dim[2 * b], W = a.img_dim[2 * b + 1];
  if (tid == 0) cnt = 0;
  for (int i = tid; i < n; i += RT) {
    const float* r = a.boxes + ((size_t)b * a.n_max + i) * 5;
    // gt_boxes[:, :4] * [H, W, H, W]  (retinanet_module.py:274-278, fp32)
    const float y = r[0] * H, x = r[1] * W, h = r[2] * H, w = r[3] * W;
    gy[i] = y; gx[i] = x; gh[i] = h; gw[i] = w;
    ga[i] = h * w;                                       // boxes1_area (utils.py:73)
    lo0[i] = y - h / 2.0f; lo1[i] = x - w / 2.0f;       // convert to corners (utils.py:62-67)
    hi0[i] = y + h / 2.0f; hi1[i] = x + w / 2.0f;
    gc[i] = (int)r[4];
  }
  __syncthreads();
  const int p = p0 + tid;
  int matches = 0;
  if (p < a.P) {
    int l = 0;
    while (l < 4 && p >= a.off[l + 1]) ++l;
    const int S = a.S[l], s = a.stride[l];
    const int q = p - a.off[l];
    const int an = q / (S * S);
    const int cell = q - an * S * S;
    const int u = cell / S, v = cell - (cell / S) * S;
    const float ah = a.adims[(l * a.A + an) * 2], aw = a.adims[(l * a.A + an) * 2 + 1];
    const float c0 = (float)(u * s), c1 = (float)(v * s);
    const float alo0 = c0 - ah / 2.0f, alo1 = c1 - aw / 2.0f;
    const float ahi0 = c0 + ah / 2.0f, ahi1 = c1 + aw / 2.0f;
    const float aa = ah * aw;
    uint32_t bits[kWords];
#pragma unroll
    for (int k = 0; k < kWords; ++k) bits[k] = 0u;
    int last = -1;
    for (int i = 0; i < n; ++i) {
      const float i0 = relu0(fminf(hi0[i], ahi0) - fmaxf(lo0[i], alo0));
      const float i1 = relu0(fminf(hi1[i], ahi1) - fmaxf(lo1[i], alo1));
      const float inter = i0 * i1;
      float uni = (ga[i] + aa) - inter;
      uni = uni > 1e-8f ? uni : 1e-8f;
      float iou = inter / uni;
      iou = iou < 0.f ? 0.f : (iou > 1.f ? 1.f : iou);
      if (iou > a.thresh) {                               // strict > (retinanet_module.py:301)
        ++matches;
        last = i;
        const int c = gc[i];
        if (c >= 0 && c < a.C) bits[c >> 5] |= 1u << (c & 31);
      }
    }
    float* st = stage + (size_t)tid * row;
    if (last >= 0) {                                      // linear box targets in float64 (Q24)
      st[0] = (float)(((double)u * s - (double)gy[last]) / (double)ah);
      st[1] = (float)(((double)v * s - (double)gx[last]) / (double)aw);
      st[2] = (float)((double)gh[last] / (double)ah);
      st[3] = (float)((double)gw[last] / (double)aw);
    } else {
      st[0] = st[1] = st[2] = st[3] = 0.f;
    }
    for (int c = 0; c < a.C; ++c) st[4 + c] = ((bits[c >> 5] >> (c & 31)) & 1u) ? 1.0f : 0.0f;
  }
  if (matches) atomicAdd(&cnt, matches);
  __syncthreads();
  if (tid == 0 && cnt) atomicAdd(&a.ntgt[b], cnt);
  const int ncell = min(RT, a.P - p0);
  float* out = a.out + ((size_t)b * a.P + p0) * row;
  for (int e = tid; e < ncell * row; e += RT) out[e] = stage[e];
}

// ------------------------------------------------------------------------------------------------
// CenterNet hourglass centroid targets: one-hot at the centroid cell, ascending-area order
// (tf_centernet_hourglass.py:403-453).  Output [B][hm][wm][4+C].
// ------------------------------------------------------------------------------------------------
struct CenterArgs {
  const float* boxes;
  const int32_t* nbox;
  const float* img_dim;
  float* out;
  int n_max, C, hm, wm, stride;
  float pad_h, pad_w;
};

__device__ void sort_by_area(const float* boxes, int n, float H, float W, int* order, float* area) {
  // stable ascending rank (np.argsort on distinct areas)
  for (int i = threadIdx.x; i < n; i += blockDim.x) area[i] = (boxes[i * 5 + 2] * H) * (boxes[i * 5 + 3] * W);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    int r = 0;
    for (int j = 0; j < n; ++j) r += (area[j] < area[i]) || (area[j] == area[i] && j < i);
    order[r] = i;
  }
  __syncthreads();
}

__global__ void __launch_bounds__(NT) centernet_assign_kernel(CenterArgs a) {
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  __shared__ int order[kMaxBox];
  __shared__ float area[kMaxBox];
  __shared__ int cy[kMaxBox], cx[kMaxBox], cc[kMaxBox];
  __shared__ float off4[kMaxBox][4];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const float H = a.img_dim[2 * b], W = a.img_dim[2 * b + 1];
  const float* bx = a.boxes + (size_t)b * a.n_max * 5;
  sort_by_area(bx, n, H, W, order, area);
  const float sf = (float)a.stride;
  // pad_y = int((img_pad[1] - img_dim[1]) / 2.0), pad_x from index 0 (:397-398, fp32)
  const float py = (float)(int)((a.pad_w - W) / 2.0f), px = (float)(int)((a.pad_h - H) / 2.0f);
  for (int k = tid; k < n; k += NT) {
    const float* r = bx + order[k] * 5;
    const float c0 = (r[0] - 0.5f * r[2]) * H, c1 = (r[1] - 0.5f * r[3]) * W;   // :431-435
    const float c2 = (r[0] + 0.5f * r[2]) * H, c3 = (r[1] + 0.5f * r[3]) * W;
    const float ycf = (c0 + c2) / 2.0f, xcf = (c1 + c3) / 2.0f;                  // :437-438
    const int yc = (int)((py + ycf) / sf), xc = (int)((px + xcf) / sf);          // :439-440
    cy[k] = yc; cx[k] = xc; cc[k] = (int)r[4];
    off4[k][0] = (float)((double)yc + 0.5) - (py + c0) / sf;                     // :444-448
    off4[k][1] = ((py + c2) / sf - (float)yc) - 0.5f;
    off4[k][2] = (float)((double)xc + 0.5) - (px + c1) / sf;
    off4[k][3] = ((px + c3) / sf - (float)xc) - 0.5f;
  }
  __syncthreads();
  const int row = 4 + a.C;
  const int cells = a.hm * a.wm;
  for (int cell = blockIdx.x * NT + tid; cell < cells; cell += gridDim.x * NT) {
    const int y = cell / a.wm, x = cell - (cell / a.wm) * a.wm;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    uint32_t bits[kWords];
#pragma unroll
    for (int k = 0; k < kWords; ++k) bits[k] = 0u;
    for (int k = 0; k < n; ++k) {
      if (cy[k] == y && cx[k] == x) {
        v[0] = off4[k][0]; v[1] = off4[k][1]; v[2] = off4[k][2]; v[3] = off4[k][3];
        if (cc[k] >= 0 && cc[k] < a.C) bits[cc[k] >> 5] |= 1u << (cc[k] & 31);
      }
    }
    float* o = a.out + ((size_t)b * cells + cell) * row;
    o[0] = v[0]; o[1] = v[1]; o[2] = v[2]; o[3] = v[3];
    for (int c = 0; c < a.C; ++c) o[4 + c] = ((bits[c >> 5] >> (c & 31)) & 1u) ? 1.0f : 0.0f;
  }
}

// ------------------------------------------------------------------------------------------------
// CenterNet centre splat (tf_centernet.py:152-342): FCOS-style ltrb over the sigma sub-box, an
// inverse-power (spread 8) centre kernel normalised by its maximum in ch4, class bits.
// Output [B][Hs][Ws][5+C].  Last covering box (ascending area) wins ch0..4.
// ------------------------------------------------------------------------------------------------
struct SplatArgs {
  const float* boxes;
  const int32_t* nbox;
  const float* img_dim;
  float* out;
  int n_max, C, Hs, Ws, stride;
  float sigma, spread;
};

struct SplatBox {
  int ylo, yup, xlo, xup, ycen, xcen, ny, nx, br, cls;
  float t0, t1, t2, t3;
  double zy, zx;   // per-axis maxima of the inverse-power kernel over the region
};

__device__ __forceinline__ double ipow_kernel(double g, double mu, double spread) {
  return 1.0 / pow(g - mu, spread);
}

__global__ void __launch_bounds__(NT) centernet_splat_kernel(SplatArgs a) {
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  __shared__ int order[kMaxBox];
  __shared__ float area[kMaxBox];
  __shared__ SplatBox bs[kMaxBox];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const float H = a.img_dim[2 * b], W = a.img_dim[2 * b + 1];
  const float* bx = a.boxes + (size_t)b * a.n_max * 5;
  sort_by_area(bx, n, H, W, order, area);
  const float sf = (float)a.stride;
  const float hr = H / sf, wr = W / sf;
  const int ylim = (int)(H / sf), xlim = (int)(W / sf);
  for (int k = tid; k < n; k += NT) {
    const float* r = bx + order[k] * 5;
    SplatBox q;
    const float c0 = (r[0] - 0.5f * r[2]) * H, c1 = (r[1] - 0.5f * r[3]) * W;
    const float c2 = (r[0] + 0.5f * r[2]) * H, c3 = (r[1] + 0.5f * r[3]) * W;
    q.t0 = c0 / sf; q.t1 = c1 / sf; q.t2 = c2 / sf; q.t3 = c3 / sf;
    q.ycen = (int)(r[0] * hr);                                                   // :208-209
    q.xcen = (int)(r[1] * wr);
    int ylo = 1 + (int)((r[0] - a.sigma * r[2] / 2.0f) * hr);                   // :211-218
    int xlo = 1 + (int)((r[1] - a.sigma * r[3] / 2.0f) * wr);
    int yup = 1 + (int)((r[0] + a.sigma * r[2] / 2.0f) * hr);
    int xup = 1 + (int)((r[1] + a.sigma * r[3] / 2.0f) * wr);
    ylo = ylo > 0 ? ylo : 0;
    xlo = xlo > 0 ? xlo : 0;
    yup = yup < ylim ? yup : ylim;                                               // upper clamp: img_dim (Q32)
    xup = xup < xlim ? xup : xlim;
    q.ylo = ylo; q.yup = yup; q.xlo = xlo; q.xup = xup;
    q.br = ((yup - ylo) > 0 ? 1 : 0) | ((xup - xlo) > 0 ? 2 : 0);
    q.ny = (int)(0.5 * (double)(ylo + yup));
    q.nx = (int)(0.5 * (double)(xlo + xup));
    q.cls = (int)r[4];
    // maxima over the region of 1/|g - mu|^spread (the normaliser, separable: tf_centernet.py:17)
    double zy = 0.0, zx = 0.0;
    if (q.br & 1)
      for (int z = ylo; z < yup; ++z) { const double g = ipow_kernel(z + 0.5, q.ny, a.spread); zy = g > zy ? g : zy; }
    if (q.br & 2)
      for (int z = xlo; z < xup; ++z) { const double g = ipow_kernel(z + 0.5, q.nx, a.spread); zx = g > zx ? g : zx; }
    q.zy = zy; q.zx = zx;
    bs[k] = q;
  }
  __syncthreads();
  const int row = 5 + a.C;
  const int cells = a.Hs * a.Ws;
  for (int cell = blockIdx.x * NT + tid; cell < cells; cell += gridDim.x * NT) {
    const int y = cell / a.Ws, x = cell - (cell / a.Ws) * a.Ws;
    uint32_t bits[kWords];
#pragma unroll
    for (int k = 0; k < kWords; ++k) bits[k] = 0u;
    int last = -1;
    for (int k = 0; k < n; ++k) {
      const SplatBox& q = bs[k];
      bool cov;
      switch (q.br) {
        case 3: cov = y >= q.ylo && y < q.yup && x >= q.xlo && x < q.xup; break;
        case 1: cov = y >= q.ylo && y < q.yup && x == q.xcen; break;
        case 2: cov = y == q.ycen && x >= q.xlo && x < q.xup; break;
        default: cov = y == q.ycen && x == q.xcen; break;
      }
      if (cov) {
        last = k;
        if (q.cls >= 0 && q.cls < a.C) bits[q.cls >> 5] |= 1u << (q.cls & 31);
      }
    }
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    if (last >= 0) {
      const SplatBox& q = bs[last];
      const float gy = (float)y + 0.5f, gx = (float)x + 0.5f;
      if (q.br & 1) { v[0] = relu0(gy - q.t0); v[1] = relu0(q.t2 - gy); }
      else { v[0] = relu0((float)((double)q.ycen + 0.5) - q.t0); v[1] = relu0((q.t2 - (float)q.ycen) - 0.5f); }
      if (q.br & 2) { v[2] = relu0(gx - q.t1); v[3] = relu0(q.t3 - gx); }
      else { v[2] = relu0((float)((double)q.xcen + 0.5) - q.t1); v[3] = relu0((q.t3 - (float)q.xcen) - 0.5f); }
      double c;
      if (q.br == 3) {
        if (y == q.ny && x == q.nx) c = 1.0;
        else {
          const double gg = ipow_kernel(y + 0.5, q.ny, a.spread) * ipow_kernel(x + 0.5, q.nx, a.spread);
          c = gg / (q.zy * q.zx);
        }
      } else if (q.br == 1) {
        c = (y == q.ny) ? 1.0 : ipow_kernel(y + 0.5, q.ny, a.spread) / q.zy;
      } else if (q.br == 2) {
        c = (x == q.nx) ? 1.0 : ipow_kernel(x + 0.5, q.nx, a.spread) / q.zx;
      } else {
        c = 1.0;
      }
      v[4] = (float)c;
    }
    float* o = a.out + ((size_t)b * cells + cell) * row;
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = v[k];
    for (int c = 0; c < a.C; ++c) o[5 + c] = ((bits[c >> 5] >> (c & 31)) & 1u) ? 1.0f : 0.0f;
  }
}

// ------------------------------------------------------------------------------------------------
// focal (alpha .25, gamma 2) on classes + smooth-L1 on 4 box channels masked by max(class) > 0,
// per image sums and gradients (CenterNet model_loss, RetinaNet train_loss per (level, anchor)).
// ------------------------------------------------------------------------------------------------
struct DetLossArgs {
  const float* reg;
  const float* cls;
  const float* tgt;
  double* partial;
  float* dreg;
  float* dcls;
  int ld_reg, ld_cls, P, C, tiles;
  float grad_scale_cls, grad_scale_reg;
};

// one focal-loss element (alpha .25, gamma 2, the stable form of retinanet_module.py:367-386 /
// fcos.py:443-462): returns the loss, *g = d loss / d logit
__device__ __forceinline__ float focal_elem(float y, float x, float* g) {
  const float e = expf(-fabsf(x));
  const float L = log1pf(e);
  const float p1 = x >= 0.f ? 1.0f / (1.0f + e) : e / (1.0f + e);
  const float q1 = x >= 0.f ? e / (1.0f + e) : 1.0f / (1.0f + e);
  const float nlp = L - fminf(x, 0.f), nlq = L + fmaxf(x, 0.f);
  *g = -y * 0.25f * q1 * q1 * (2.0f * p1 * nlp + q1) + (1.0f - y) * 0.75f * p1 * p1 * (2.0f * q1 * nlq + p1);
  return y * 0.25f * q1 * q1 * nlp + (1.0f - y) * 0.75f * p1 * p1 * nlq;
}

// one (discontinuous, Q8) smooth-L1 element, delta 1: returns the loss, *g = d loss / d pred
__device__ __forceinline__ float sl1_elem(float t, float x, float* g) {
  const float d = t - x;
  const float ad = fabsf(d);
  if (ad < 1.0f) { *g = -d; return 0.5f * d * d; }
  *g = d > 0.f ? -1.0f : (d < 0.f ? 1.0f : 0.0f);
  return ad;
}

__global__ void __launch_bounds__(NT) det_loss_kernel(DetLossArgs a) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * NT + threadIdx.x;
  float s_cls = 0.f, s_reg = 0.f;
  if (p < a.P) {
    const size_t cell = (size_t)b * a.P + p;
    const float* t = a.tgt + cell * (4 + a.C);
    const float* xr = a.reg + cell * a.ld_reg;
    const float* xc = a.cls + cell * a.ld_cls;
    float tmax = 0.f;
    for (int c = 0; c < a.C; ++c) {
      const float y = t[4 + c];
      tmax = fmaxf(tmax, y);
      float g;
      s_cls += focal_elem(y, xc[c], &g);
      if (a.dcls) a.dcls[cell * a.ld_cls + c] = g * a.grad_scale_cls;
    }
    const float mask = tmax > 0.f ? 1.0f : 0.0f;                 // max(class) > 0
    for (int j = 0; j < 4; ++j) {
      float g;
      s_reg += mask * sl1_elem(t[j], xr[j], &g);
      if (a.dreg) a.dreg[cell * a.ld_reg + j] = mask * g * a.grad_scale_reg;
    }
  }
  __shared__ double red[2][NT / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)b * a.tiles + blockIdx.x) * 2 + threadIdx.x] = s;
  }
}

// CenterNet training loss (tf_centernet_hourglass.py:492-505 inside train_step :537-545) straight
// off the output conv: pred [B*P][ld_pred] fp32 = [reg 0..3 | cls 4..4+C) (b_focal already in the
// conv bias), targets [B*P][4+C].  Writes the bf16 gradient of cls_scale*cls + reg_scale*reg as
// the output conv's backward operand [B*P][ld_d] (channels >= 4+C zeroed) and per-image sums.
struct CnLossArgs {
  const float* pred;
  const float* tgt;
  double* partial;
  cvl_bf16* d;
  int ld_pred, ld_d, P, C, tiles;
  float cls_scale, reg_scale;
};

__global__ void __launch_bounds__(NT) centernet_loss_kernel(CnLossArgs a) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * NT + threadIdx.x;
  float s_cls = 0.f, s_reg = 0.f;
  if (p < a.P) {
    const size_t cell = (size_t)b * a.P + p;
    const float* t = a.tgt + cell * (4 + a.C);
    const float* x = a.pred + cell * a.ld_pred;
    cvl_bf16* d = a.d + cell * a.ld_d;
    float tmax = 0.f;
    for (int c = 0; c < a.C; ++c) {
      const float y = t[4 + c];
      tmax = fmaxf(tmax, y);
      float g;
      s_cls += focal_elem(y, x[4 + c], &g);
      d[4 + c] = f32_to_bf16(g * a.cls_scale);
    }
    const float mask = tmax > 0.f ? 1.0f : 0.0f;
    for (int j = 0; j < 4; ++j) {
      float g;
      s_reg += mask * sl1_elem(t[j], x[j], &g);
      d[j] = f32_to_bf16(mask * g * a.reg_scale);
    }
    for (int c = 4 + a.C; c < a.ld_d; ++c) d[c] = 0;
  }
  __shared__ double red[2][NT / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)b * a.tiles + blockIdx.x) * 2 + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// CenterNet v2 (CenterNet/tf_hourglass_net.py) targets: the inline builder of
// CenterNet/train_hourglass_voc.py train() :96-160 for one batch.  boxes [B][n_max][5] are the
// dataset's corner rows (b0, b1, b2, b3, label), converted by utils.convert_to_xywh (:16-27) to
// (x_cen, y_cen, w, h); one (raw_dims, img_dims) per batch (the step's jitter scale), pad_dims =
// int((img_dims - raw_dims) / 2).  Output [B][S][S][4][5+C], S = img_dims / 8.  Boxes go in
// ascending w*h*100 order (stable on ties); each writes (y_off, x_off, h_reg, w_reg, 1) of its
// (cell, scale) -- the last writer wins -- and ORs its class bit.  fp32 sequences as the
// reference's numpy float32 scalars (NEP 50); negative cell indices wrap as numpy indexing does,
// cells past the map (an IndexError there) and labels outside [0, C) are skipped.
// ------------------------------------------------------------------------------------------------
struct Hg2Args {
  const float* boxes;
  const int32_t* nbox;
  float* out;
  int n_max, C, S, raw, img;
};

__global__ void __launch_bounds__(NT) hg2_assign_kernel(Hg2Args a) {
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  __shared__ int order[kMaxBox];
  __shared__ float area[kMaxBox];
  __shared__ int key[kMaxBox];                 // (row * S + col) * 4 + scale, -1 = no write
  __shared__ int cls[kMaxBox];
  __shared__ float val[kMaxBox][4];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const float* bx = a.boxes + (size_t)b * a.n_max * 5;
  for (int i = tid; i < n; i += NT) {
    const float* r = bx + i * 5;
    area[i] = ((r[2] - r[0]) * (r[3] - r[1])) * 100.0f;           // tmp_box_areas (:113-114)
  }
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    int rk = 0;
    for (int j = 0; j < n; ++j) rk += (area[j] < area[i]) || (area[j] == area[i] && j < i);
    order[rk] = i;
  }
  __syncthreads();
  const float rawf = (float)a.raw;
  const float padf = (float)((a.img - a.raw) / 2);
  float sc[4];                                                      // img_scale (:108-109)
#pragma unroll
  for (int k = 0; k < 4; ++k) sc[k] = (float)((double)a.img / (double)(1 << (3 - k)));
  for (int k = tid; k < n; k += NT) {
    const float* r = bx + order[k] * 5;
    const float x0 = (r[0] + r[2]) / 2.0f, y0 = (r[1] + r[3]) / 2.0f;
    const float bw = r[2] - r[0], bh = r[3] - r[1];
    const float xcen = padf + x0 * rawf, ycen = padf + y0 * rawf;  // :123-126
    const float width = bw * rawf, height = bh * rawf;
    int kk = -1;
    if (!(width < 0.f || height < 0.f)) {
      int id = 3;
      if (width < sc[0] && height < sc[0]) id = 0;
      else if (width < sc[1] && height < sc[1]) id = 1;
      else if (width < sc[2] && height < sc[2]) id = 2;
      const float bs = sc[id];
      const float wreg = width / bs, hreg = height / bs;              // :144-151
      int wc = (int)(xcen / 8.0f), hc = (int)(ycen / 8.0f);
      const float woff = (xcen - (float)(wc * 8)) / 8.0f;
      const float hoff = (ycen - (float)(hc * 8)) / 8.0f;
      if (wc < 0) wc += a.S;
      if (hc < 0) hc += a.S;
      if (wc >= 0 && wc < a.S && hc >= 0 && hc < a.S) {
        kk = (hc * a.S + wc) * 4 + id;
        val[k][0] = hoff; val[k][1] = woff; val[k][2] = hreg; val[k][3] = wreg;
      }
    }
    key[k] = kk;
    cls[k] = (int)r[4];
  }
  __syncthreads();
  const int R = 5 + a.C;
  const int rows = a.S * a.S * 4;
  for (int row = blockIdx.x * NT + tid; row < rows; row += gridDim.x * NT) {
    float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    uint32_t bits[kWords];
#pragma unroll
    for (int k = 0; k < kWords; ++k) bits[k] = 0u;
    for (int k = 0; k < n; ++k) {
      if (key[k] != row) continue;
      v[0] = val[k][0]; v[1] = val[k][1]; v[2] = val[k][2]; v[3] = val[k][3]; v[4] = 1.0f;
      if (cls[k] >= 0 && cls[k] < a.C) bits[cls[k] >> 5] |= 1u << (cls[k] & 31);
    }
    float* o = a.out + ((size_t)b * rows + row) * R;
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = v[k];
    for (int c = 0; c < a.C; ++c) o[5 + c] = ((bits[c >> 5] >> (c & 31)) & 1u) ? 1.0f : 0.0f;
  }
}

// CenterNet v2 model_loss (tf_hourglass_net.py:398-413) inside train_step (:415-447) straight off
// the head conv: pred [B*P][ld_pred] fp32 = the Conv2D(4*(5+C)) logits with b_focal folded into
// the class channels' bias (channel sc*(5+C) + j of cell p = row (p, sc) of the [S,S,4,5+C]
// reshape); targets [B*P][4][5+C].  reg = sum |t - sigmoid(x)| * mask (mask = t[4]); cls = focal
// (loss_type "focal") or sigmoid cross-entropy over channels 4..4+C (labels cast to int).  Writes
// the bf16 gradient of cls_scale*cls + reg_scale*reg [B*P][ld_d] (channels >= 4*(5+C) zeroed).
struct Hg2LossArgs {
  const float* pred;
  const float* tgt;
  double* partial;
  cvl_bf16* d;
  int ld_pred, ld_d, P, C, tiles, sce;
  float cls_scale, reg_scale;
};

__global__ void __launch_bounds__(NT) hg2_loss_kernel(Hg2LossArgs a) {
  const int b = blockIdx.y;
  const int row = blockIdx.x * NT + threadIdx.x;            // (pixel, scale)
  const int R = 5 + a.C;
  float s_cls = 0.f, s_reg = 0.f;
  if (row < a.P * 4) {
    const int p = row >> 2, sc = row & 3;
    const float* t = a.tgt + ((size_t)b * a.P * 4 + row) * R;
    const float* x = a.pred + ((size_t)b * a.P + p) * a.ld_pred + sc * R;
    cvl_bf16* d = a.d + ((size_t)b * a.P + p) * a.ld_d + sc * R;
    const float m = t[4];
    const bool prob = (a.sce & 2) != 0;                     // box channels already sigmoid'd
    for (int j = 0; j < 4; ++j) {
      const float s = prob ? x[j] : 1.0f / (1.0f + expf(-x[j]));
      const float df = t[j] - s;
      s_reg += fabsf(df) * m;
      const float sg = df > 0.f ? -1.0f : (df < 0.f ? 1.0f : 0.0f);
      d[j] = f32_to_bf16(m * sg * (prob ? 1.0f : s * (1.0f - s)) * a.reg_scale);
    }
    for (int j = 4; j < R; ++j) {
      const float y = (float)(int)t[j];
      const float xv = x[j];
      float g;
      if (a.sce & 1) {
        const float e = expf(-fabsf(xv));
        s_cls += (fmaxf(xv, 0.f) - xv * y) + log1pf(e);
        g = (xv >= 0.f ? 1.0f / (1.0f + e) : e / (1.0f + e)) - y;
      } else {
        s_cls += focal_elem(y, xv, &g);
      }
      d[j] = f32_to_bf16(g * a.cls_scale);
    }
    if (sc == 3)
      for (int c = 4 * R; c < a.ld_d; ++c) a.d[((size_t)b * a.P + p) * a.ld_d + c] = 0;
  }
  __shared__ double red[2][NT / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)b * a.tiles + blockIdx.x) * 2 + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// CenterNet ResNet stride-8 multi-scale targets: CenterNet/tf_centernet_resnet_s8.py format_data
// (:243-330) as train_centernet_crowdhuman.py (:64-104) calls it: gt_labels rows (y, x, h, w, cls)
// normalised, concatenated with the int64 class column, hence float64 arithmetic throughout
// (inputs are the float32 box values); img_dim [B][2] = the resized (raw) size, img_pad the padded
// size.  Output [B][pad_w/stride][pad_h/stride][n_scales][4+C] (h_max from img_pad[1], w_max from
// img_pad[0], kept): ascending area, each box writes (y_off, x_off, h/scale, w/scale) at its
// centre cell and first scale with max(h, w) < box_scales[sc], ORs its class bit.  Boxes with no
// such scale (a ValueError there) or a centre off the map are skipped.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxScales = 8;

struct S8Args {
  const float* boxes;
  const int32_t* nbox;
  const float* img_dim;
  float* out;
  int n_max, C, hm, wm, ns, stride;
  double pad_h, pad_w;
  double scales[kMaxScales];
};

__global__ void __launch_bounds__(NT) s8_assign_kernel(S8Args a) {
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  __shared__ int order[kMaxBox];
  __shared__ double dar[kMaxBox];
  __shared__ int key[kMaxBox];
  __shared__ int cls[kMaxBox];
  __shared__ float val[kMaxBox][4];
  int n = a.nbox[b];
  n = n < 0 ? 0 : (n > a.n_max ? a.n_max : n);
  const double D0 = (double)a.img_dim[2 * b], D1 = (double)a.img_dim[2 * b + 1];
  const float* bx = a.boxes + (size_t)b * a.n_max * 5;
  for (int i = tid; i < n; i += NT) dar[i] = ((double)bx[i * 5 + 2] * D0) * ((double)bx[i * 5 + 3] * D1);
  __syncthreads();
  for (int i = tid; i < n; i += NT) {
    int rk = 0;
    if (n > 1)
      for (int j = 0; j < n; ++j) rk += (dar[j] < dar[i]) || (dar[j] == dar[i] && j < i);
    else
      rk = i;
    order[rk] = i;
  }
  __syncthreads();
  const double st = (double)a.stride;
  const double py = (double)(int)((a.pad_w - D1) / 2.0), px = (double)(int)((a.pad_h - D0) / 2.0);
  for (int k = tid; k < n; k += NT) {
    const float* r = bx + order[k] * 5;
    const double y = r[0], x = r[1], h = r[2], w = r[3];
    const double c0 = (y - 0.5 * h) * D0, c1 = (x - 0.5 * w) * D1;
    const double c2 = (y + 0.5 * h) * D0, c3 = (x + 0.5 * w) * D1;
    const double bh = c2 - c0, bw = c3 - c1;
    const double bd = bh > bw ? bh : bw;                               // max(box_h, box_w)
    int id = -1;
    for (int s = 0; s < a.ns; ++s)
      if (bd < a.scales[s]) { id = s; break; }
    int kk = -1;
    if (id >= 0) {
      const double ryc = (c0 + c2) / 2.0, rxc = (c1 + c3) / 2.0;
      int yc = (int)((py + ryc) / st), xc = (int)((px + rxc) / st);
      const double yo = (py + ryc - (double)yc * st), xo = (px + rxc - (double)xc * st);
      val[k][0] = (float)(yo / st); val[k][1] = (float)(xo / st);
      val[k][2] = (float)(bh / a.scales[id]); val[k][3] = (float)(bw / a.scales[id]);
      if (yc < 0) yc += a.hm;
      if (xc < 0) xc += a.wm;
      if (yc >= 0 && yc < a.hm && xc >= 0 && xc < a.wm) kk = (yc * a.wm + xc) * a.ns + id;
    }
    key[k] = kk;
    cls[k] = (int)r[4];
  }
  __syncthreads();
  const int R = 4 + a.C;
  const int rows = a.hm * a.wm * a.ns;
  for (int row = blockIdx.x * NT + tid; row < rows; row += gridDim.x * NT) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    uint32_t bits[kWords];
#pragma unroll
    for (int k = 0; k < kWords; ++k) bits[k] = 0u;
    for (int k = 0; k < n; ++k) {
      if (key[k] != row) continue;
      v[0] = val[k][0]; v[1] = val[k][1]; v[2] = val[k][2]; v[3] = val[k][3];
      if (cls[k] >= 0 && cls[k] < a.C) bits[cls[k] >> 5] |= 1u << (cls[k] & 31);
    }
    float* o = a.out + ((size_t)b * rows + row) * R;
#pragma unroll
    for (int k = 0; k < 4; ++k) o[k] = v[k];
    for (int c = 0; c < a.C; ++c) o[4 + c] = ((bits[c >> 5] >> (c & 31)) & 1u) ? 1.0f : 0.0f;
  }
}

// tf_centernet_resnet_s8.model_loss (:368-385) in train_step (:387-444) off the two head convs:
// reg [B*P][ld_reg] fp32 holds the n_scales x 4 raw box logits of a cell (scale-major), cls
// [B*P][ld_cls] the n_scales x C class logits; targets [B*P][n_scales][4+C].  Per (cell, scale):
// focal on the classes, smooth-L1 (Q8) of sigmoid(box) masked by max(class target) > 0.
// Writes bf16 gradients of cls_scale*cls + reg_scale*reg into d_reg / d_cls (pads zeroed).
struct S8LossArgs {
  const float* reg;
  const float* cls;
  const float* tgt;
  double* partial;
  cvl_bf16* dreg;
  cvl_bf16* dcls;
  int ld_reg, ld_cls, ld_dreg, ld_dcls, P, C, ns, tiles;
  float cls_scale, reg_scale;
};

__global__ void __launch_bounds__(NT) s8_loss_kernel(S8LossArgs a) {
  const int b = blockIdx.y;
  const int row = blockIdx.x * NT + threadIdx.x;              // (cell, scale)
  const int R = 4 + a.C;
  float s_cls = 0.f, s_reg = 0.f;
  if (row < a.P * a.ns) {
    const int p = row / a.ns, sc = row - (row / a.ns) * a.ns;
    const size_t cell = (size_t)b * a.P + p;
    const float* t = a.tgt + ((size_t)b * a.P * a.ns + row) * R;
    const float* xr = a.reg + cell * a.ld_reg + sc * 4;
    const float* xc = a.cls + cell * a.ld_cls + sc * a.C;
    cvl_bf16* dr = a.dreg + cell * a.ld_dreg + sc * 4;
    cvl_bf16* dc = a.dcls + cell * a.ld_dcls + sc * a.C;
    float tmax = 0.f;
    for (int c = 0; c < a.C; ++c) {
      const float y = t[4 + c];
      tmax = fmaxf(tmax, y);
      float g;
      s_cls += focal_elem(y, xc[c], &g);
      dc[c] = f32_to_bf16(g * a.cls_scale);
    }
    const float mask = tmax > 0.f ? 1.0f : 0.0f;
    for (int j = 0; j < 4; ++j) {
      const float sg = 1.0f / (1.0f + expf(-xr[j]));
      float g;
      s_reg += mask * sl1_elem(t[j], sg, &g);
      dr[j] = f32_to_bf16(mask * g * (sg * (1.0f - sg)) * a.reg_scale);
    }
    if (sc == a.ns - 1) {
      for (int c = a.ns * 4; c < a.ld_dreg; ++c) a.dreg[cell * a.ld_dreg + c] = 0;
      for (int c = a.ns * a.C; c < a.ld_dcls; ++c) a.dcls[cell * a.ld_dcls + c] = 0;
    }
  }
  __shared__ double red[2][NT / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)b * a.tiles + blockIdx.x) * 2 + threadIdx.x] = s;
  }
}

// ------------------------------------------------------------------------------------------------
// CenterNet detection decode (tf_centernet_hourglass.py:576-650, the part before `nms`): corners
// from prediction_to_corners (:355-377: fp32 grid +- ltrb, then stride * in float64), sigmoid class
// probabilities (fp32; evaluated in float64 and rounded), per-cell max / first argmax, threshold,
// the image-ratio scaling, w/h clamps and x/y floors of :630-650, int(prob * 100).  Rows are
// emitted in np.nonzero (row-major cell) order: one 1024-thread workgroup scans the cells in
// chunks with a ballot prefix sum.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) centernet_decode_kernel(const float* pred, int ld, int H, int W, int C,
                                                                double stride, float thresh, double w_ratio,
                                                                double h_ratio, double img_w, double img_h,
                                                                double* rows, int32_t* count) {
  __shared__ int wtot[16];
  __shared__ int base_s;
  if (threadIdx.x == 0) base_s = 0;
  __syncthreads();
  const int n = H * W;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int cell = c0 + threadIdx.x;
    bool keep = false;
    float pmax = 0.f;
    int lab = 0;
    if (cell < n) {
      const float* p = pred + (size_t)cell * ld;
      for (int c = 0; c < C; ++c) {
        const float pr = (float)(1.0 / (1.0 + exp(-(double)p[4 + c])));
        if (c == 0 || pr > pmax) { pmax = pr; lab = c; }
      }
      keep = pmax >= thresh;
    }
    const unsigned long long m = __ballot(keep);
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wtot[wv] = __popcll(m);
    __syncthreads();
    int off = 0, tot = 0;
    for (int k = 0; k < 16; ++k) { off += k < wv ? wtot[k] : 0; tot += wtot[k]; }
    if (keep) {
      const float* p = pred + (size_t)cell * ld;
      const int y = cell / W, x = cell - (cell / W) * W;
      const float gy = (float)y + 0.5f, gx = (float)x + 0.5f;
      const double b0 = stride * (double)(gy - p[0]), b1 = stride * (double)(gx - p[2]);
      const double b2 = stride * (double)(gy + p[1]), b3 = stride * (double)(gx + p[3]);
      double x_low = h_ratio * b1, y_low = w_ratio * b0;
      const double x_upp = h_ratio * b3, y_upp = w_ratio * b2;
      double bw = x_upp - x_low, bh = y_upp - y_low;
      if (bw > img_w) bw = img_w;
      if (bh > img_h) bh = img_h;
      if (x_low < 0.0) x_low = 0.0;
      if (y_low < 0.0) y_low = 0.0;
      double* r = rows + (size_t)(base_s + off + pre) * 6;
      r[0] = x_low; r[1] = y_low; r[2] = bw; r[3] = bh;
      r[4] = (double)(int)(pmax * 100.0f);
      r[5] = (double)lab;
    }
    __syncthreads();
    if (threadIdx.x == 0) base_s += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = base_s;
}

// The per-scale decodes of the two variant CenterNets' obj_detect_results (the parts before the
// plotting; one image, scales in order, cells in np.nonzero (row-major) order within a scale):
// * mode 1, CenterNet/tf_centernet_resnet_s8.py:446-547: prediction_to_corners (:210-241: fp32
//   centre (grid + offset) * stride, size * box_scales[s] with the scale as an fp32 operand, corners
//   +- size / 2 in fp32, stored into float64), then the ltrb post-processing of :524-547 (image
//   ratios in float64, w / h clamps, x / y floors) -> the rows `nms` takes;
// * mode 2, CenterNet/tf_hourglass_net.py:517-578: centroid = ratio * (cell + offset) * 8 in float64
//   (np.nonzero's int64 index + a float32 output), size = float32(ratio * box_scale) * output in
//   fp32 (a python float times a numpy float32: NumPy >= 2 promotion, NEP 50, the numpy the goldens
//   ran under), clamps to the image size, corner = centroid - size / 2 floored at 0 -> the drawn
//   rectangles (no NMS in that decode).
// Probabilities: fp32 sigmoid of the class logits (float64, rounded), max / first argmax over the
// classes [cls0, cls0 + C) of the scale, kept when >= thresh; int(prob * 100) in fp32.
struct ScaleDecodeArgs {
  const float* pred;
  double* rows;
  int32_t* count;
  int ld, H, W, ns, chs, cls0, C, mode;
  float stride, thresh;
  double w_ratio, h_ratio, img_w, img_h;
  double scale[16];
};

__global__ void __launch_bounds__(1024) centernet_scale_decode_kernel(ScaleDecodeArgs a) {
  __shared__ int wtot[16];
  __shared__ int base_s;
  if (threadIdx.x == 0) base_s = 0;
  __syncthreads();
  const int n = a.H * a.W;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int s = 0; s < a.ns; ++s) {
    for (int c0 = 0; c0 < n; c0 += 1024) {
      const int cell = c0 + threadIdx.x;
      bool keep = false;
      float pmax = 0.f;
      int lab = 0;
      const float* p = a.pred + (size_t)cell * a.ld + s * a.chs;
      if (cell < n) {
        for (int c = 0; c < a.C; ++c) {
          const float pr = (float)(1.0 / (1.0 + exp(-(double)p[a.cls0 + c])));
          if (c == 0 || pr > pmax) { pmax = pr; lab = c; }
        }
        keep = pmax >= a.thresh;
      }
      const unsigned long long m = __ballot(keep);
      const int pre = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) wtot[wv] = __popcll(m);
      __syncthreads();
      int off = 0, tot = 0;
      for (int k = 0; k < 16; ++k) { off += k < wv ? wtot[k] : 0; tot += wtot[k]; }
      if (keep) {
        const int y = cell / a.W, x = cell - (cell / a.W) * a.W;
        double r0, r1, r2, r3;
        if (a.mode == 1) {
          const float sc = (float)a.scale[s];
          const float yc = ((float)y + p[0]) * a.stride, xc = ((float)x + p[1]) * a.stride;
          const float bh = p[2] * sc, bw = p[3] * sc;
          const double b0 = (double)(yc - bh / 2.0f), b2 = (double)(yc + bh / 2.0f);
          const double b1 = (double)(xc - bw / 2.0f), b3 = (double)(xc + bw / 2.0f);
          double x_low = a.h_ratio * b1, y_low = a.w_ratio * b0;
          const double x_upp = a.h_ratio * b3, y_upp = a.w_ratio * b2;
          double bw_ = x_upp - x_low, bh_ = y_upp - y_low;
          if (bw_ > a.img_w) bw_ = a.img_w;
          if (bh_ > a.img_h) bh_ = a.img_h;
          if (x_low < 0.0) x_low = 0.0;
          if (y_low < 0.0) y_low = 0.0;
          r0 = x_low; r1 = y_low; r2 = bw_; r3 = bh_;
        } else {
          const double xcen = a.w_ratio * ((double)y + (double)p[0]) * 8.0;
          const double ycen = a.h_ratio * ((double)x + (double)p[1]) * 8.0;
          const float bwf = (float)(a.w_ratio * a.scale[s]) * p[2];
          const float bhf = (float)(a.h_ratio * a.scale[s]) * p[3];
          const double bw_ = bwf > (float)a.img_w ? a.img_w : (double)bwf;
          const double bh_ = bhf > (float)a.img_h ? a.img_h : (double)bhf;
          double x_low = xcen - bw_ / 2.0, y_low = ycen - bh_ / 2.0;
          if (x_low < 0.0) x_low = 0.0;
          if (y_low < 0.0) y_low = 0.0;
          r0 = x_low; r1 = y_low; r2 = bw_; r3 = bh_;
        }
        double* r = a.rows + (size_t)(base_s + off + pre) * 6;
        r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3;
        r[4] = (double)(int)(pmax * 100.0f);
        r[5] = (double)lab;
      }
      __syncthreads();
      if (threadIdx.x == 0) base_s += tot;
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) *a.count = base_s;
}

// RetinaNet.train_loss (retinanet_module.py:403-426) over every (level, anchor) at once, fwd + bwd.
// Predictions come straight from the grouped head convs: row (level offset + cell) of [B][P][ld],
// class channels a*C + c, box channels a*4 + j.  Targets are cvl_retina_assign's [B][A*P][4+C] in
// (level, anchor, cell) order.  Gradients are written as bf16 (the head backward's operand);
// img_weight[b] (0/1, nullable) drops images the reference loop skipped (no matches,
// train_retinanet_coco.py:203-208) from both the loss and the gradient.
struct RetinaLossArgs {
  const float* reg;
  const float* cls;
  const float* tgt;
  const float* img_w;
  double* partial;
  cvl_bf16* dreg;
  cvl_bf16* dcls;
  int ld_reg, ld_cls, ld_dreg, ld_dcls, P, A, C, tiles;
  int off[6];          // per-image cell offsets of the 5 levels (+ P)
  float grad_scale;
  int grad_f32;        // 1: d_reg / d_cls are fp32 (the parity mode), 0: bf16
};

// A workgroup owns RL_ROWS consecutive target rows of one image (a contiguous [rows][4+C] slab):
// the slab is staged through LDS with coalesced loads, each row's (mask, prediction row, anchor)
// is resolved once, then the workgroup walks the slab element by element so that consecutive
// lanes touch consecutive classes of one prediction row (coalesced logit reads / gradient writes).
constexpr int RL_ROWS = 32;
constexpr int RL_MAXW = 4 + 128;     // row width bound held in LDS (C <= 128)

__global__ void __launch_bounds__(NT) retina_loss_kernel(RetinaLossArgs a) {
  const int b = blockIdx.y;
  const int W = 4 + a.C;
  const long T = (long)a.P * a.A;
  const long t0 = (long)blockIdx.x * RL_ROWS;
  const int nrow = (int)min((long)RL_ROWS, T - t0);
  __shared__ float tile[RL_ROWS * RL_MAXW];
  __shared__ long prow_s[RL_ROWS];
  __shared__ int an_s[RL_ROWS];
  __shared__ float mask_s[RL_ROWS];
  const float* src = a.tgt + ((size_t)b * T + t0) * W;
  for (int i = threadIdx.x; i < nrow * W; i += NT) tile[i] = src[i];
  if (threadIdx.x < nrow) {
    const long t = t0 + threadIdx.x;
    // (level, anchor, cell) of target row t
    int l = 0;
#pragma unroll
    for (int k = 1; k < 5; ++k)
      if (t >= (long)a.A * a.off[k]) l = k;
    const int S2 = a.off[l + 1] - a.off[l];
    const long r = t - (long)a.A * a.off[l];
    const int an = (int)(r / S2), cell = a.off[l] + (int)(r - (long)(r / S2) * S2);
    prow_s[threadIdx.x] = (long)b * a.P + cell;
    an_s[threadIdx.x] = an;
  }
  __syncthreads();
  if (threadIdx.x < nrow) {
    float tmax = 0.f;
    for (int c = 0; c < a.C; ++c) tmax = fmaxf(tmax, tile[threadIdx.x * W + 4 + c]);
    mask_s[threadIdx.x] = tmax > 0.f ? 1.0f : 0.0f;      // max(class) > 0
  }
  __syncthreads();
  const float wb = a.img_w ? a.img_w[b] : 1.0f;
  const float gs = a.grad_scale * wb;
  float s_cls = 0.f, s_reg = 0.f;
  for (int i = threadIdx.x; i < nrow * W; i += NT) {
    const int row = i / W, ch = i - (i / W) * W;
    const long prow = prow_s[row];
    const int an = an_s[row];
    const float y = tile[i];
    float g;
    if (ch < 4) {
      const float m = mask_s[row];
      s_reg += m * sl1_elem(y, a.reg[prow * a.ld_reg + an * 4 + ch], &g);
      if (a.dreg) {
        const long o = prow * a.ld_dreg + an * 4 + ch;
        if (a.grad_f32) reinterpret_cast<float*>(a.dreg)[o] = m * g * gs;
        else a.dreg[o] = f32_to_bf16(m * g * gs);
      }
    } else {
      const int c = ch - 4;
      s_cls += focal_elem(y, a.cls[prow * a.ld_cls + (long)an * a.C + c], &g);
      if (a.dcls) {
        const long o = prow * a.ld_dcls + (long)an * a.C + c;
        if (a.grad_f32) reinterpret_cast<float*>(a.dcls)[o] = g * gs;
        else a.dcls[o] = f32_to_bf16(g * gs);
      }
    }
  }
  __shared__ double red[2][NT / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    double s = 0.0;
    for (int k = 0; k < NT / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)b * a.tiles + blockIdx.x) * 2 + threadIdx.x] = s * (double)wb;
  }
}

// losses[b][k] = sum_i partial[b][i][k]: one 256-thread block per image; thread t sums tiles
// t, t + 256, ... (both terms), then a fixed-shape LDS tree (deterministic, no atomics)
constexpr int FIN_T = 256;
__global__ void __launch_bounds__(FIN_T) det_loss_finalize(const double* partial, float* losses, int tiles) {
  const int b = blockIdx.x, t = threadIdx.x;
  double s0 = 0.0, s1 = 0.0;
  for (int i = t; i < tiles; i += FIN_T) {
    s0 += partial[((size_t)b * tiles + i) * 2];
    s1 += partial[((size_t)b * tiles + i) * 2 + 1];
  }
  __shared__ double red[2][FIN_T];
  red[0][t] = s0;
  red[1][t] = s1;
  __syncthreads();
  for (int w = FIN_T / 2; w > 0; w >>= 1) {
    if (t < w) {
      red[0][t] += red[0][t + w];
      red[1][t] += red[1][t + w];
    }
    __syncthreads();
  }
  if (t < 2) losses[b * 2 + t] = (float)red[t][0];
}

// ------------------------------------------------------------------------------------------------
// Greedy per-class NMS with the reference's selection order: within a class, repeatedly take the
// first maximum score among the survivors and drop survivors with IoU > thr (bboxes_iou: float64,
// floor at fp32 eps).  One workgroup per class; candidates in input order; output = kept indices
// in the reference's emission order (classes in the caller-given order).
// ------------------------------------------------------------------------------------------------
__global__ void nms_kernel(const double* boxes /*[n][6] x1 y1 x2 y2 score cls*/, int n, const double* classes,
                           int ncls, double thr, int32_t* keep /*[ncls][n]*/, int32_t* nkeep /*[ncls]*/,
                           uint8_t* alive_ws /*[ncls][n]*/) {
  const int ci = blockIdx.x;
  if (ci >= ncls) return;
  const double cval = classes[ci];
  uint8_t* alive = alive_ws + (size_t)ci * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) alive[i] = boxes[i * 6 + 5] == cval ? 1 : 0;
  __shared__ double best_s[NT];
  __shared__ int best_i[NT];
  __shared__ int sel;
  int count = 0;
  __syncthreads();
  for (;;) {
    double bsc = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!alive[i]) continue;
      const double sc = boxes[i * 6 + 4];
      if (sc > bsc || (sc == bsc && i < bi)) { bsc = sc; bi = i; }
    }
    best_s[threadIdx.x] = bsc;
    best_i[threadIdx.x] = bi;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = -INFINITY;
      int i0 = 0x7fffffff;
      for (int k = 0; k < (int)blockDim.x; ++k)
        if (best_s[k] > s0 || (best_s[k] == s0 && best_i[k] < i0)) { s0 = best_s[k]; i0 = best_i[k]; }
      sel = (i0 == 0x7fffffff) ? -1 : i0;
      if (sel >= 0) { keep[(size_t)ci * n + count] = sel; alive[sel] = 0; }
    }
    __syncthreads();
    const int s = sel;
    if (s < 0) break;
    ++count;
    const double* q = boxes + s * 6;
    const double qa = (q[2] - q[0]) * (q[3] - q[1]);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!alive[i]) continue;
      const double* r = boxes + i * 6;
      const double ra = (r[2] - r[0]) * (r[3] - r[1]);
      const double l0 = q[0] > r[0] ? q[0] : r[0], l1 = q[1] > r[1] ? q[1] : r[1];
      const double h0 = q[2] < r[2] ? q[2] : r[2], h1 = q[3] < r[3] ? q[3] : r[3];
      const double w0 = h0 - l0 > 0.0 ? h0 - l0 : 0.0, w1 = h1 - l1 > 0.0 ? h1 - l1 : 0.0;
      const double inter = w0 * w1;
      double iou = 1.0 * inter / (qa + ra - inter);
      const double eps = 1.1920928955078125e-07;        // np.finfo(np.float32).eps
      iou = iou > eps ? iou : eps;
      if (iou > thr || !(r[4] * (iou > thr ? 0.0 : 1.0) > 0.0)) alive[i] = 0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) nkeep[ci] = count;
}

// Soft-NMS (tf_centernet_hourglass.py:44-85, method 'soft-nms', float64): per class, repeatedly
// emit the first maximum of the current (decayed) scores among the survivors with that score,
// then multiply every other survivor's score by exp(-(1.0 * iou^2 / sigma)) (bboxes_iou with the
// fp32-eps floor) and drop those whose score is no longer > 0.  One workgroup per class; the
// running scores live in the workspace.
__global__ void soft_nms_kernel(const double* boxes, int n, const double* classes, int ncls, double sigma,
                                int32_t* keep, double* keep_score, int32_t* nkeep, double* score_ws,
                                uint8_t* alive_ws) {
  const int ci = blockIdx.x;
  if (ci >= ncls) return;
  const double cval = classes[ci];
  uint8_t* alive = alive_ws + (size_t)ci * n;
  double* sc = score_ws + (size_t)ci * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    sc[i] = boxes[i * 6 + 4];
    alive[i] = boxes[i * 6 + 5] == cval ? 1 : 0;
  }
  __shared__ double best_s[NT];
  __shared__ int best_i[NT];
  __shared__ int sel;
  int count = 0;
  __syncthreads();
  for (;;) {
    double bsc = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!alive[i]) continue;
      if (sc[i] > bsc || (sc[i] == bsc && i < bi)) { bsc = sc[i]; bi = i; }
    }
    best_s[threadIdx.x] = bsc;
    best_i[threadIdx.x] = bi;
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = -INFINITY;
      int i0 = 0x7fffffff;
      for (int k = 0; k < (int)blockDim.x; ++k)
        if (best_s[k] > s0 || (best_s[k] == s0 && best_i[k] < i0)) { s0 = best_s[k]; i0 = best_i[k]; }
      sel = (i0 == 0x7fffffff) ? -1 : i0;
      if (sel >= 0) {
        keep[(size_t)ci * n + count] = sel;
        keep_score[(size_t)ci * n + count] = sc[sel];
        alive[sel] = 0;
      }
    }
    __syncthreads();
    const int s = sel;
    if (s < 0) break;
    ++count;
    const double* q = boxes + s * 6;
    const double qa = (q[2] - q[0]) * (q[3] - q[1]);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      if (!alive[i]) continue;
      const double* r = boxes + i * 6;
      const double ra = (r[2] - r[0]) * (r[3] - r[1]);
      const double l0 = q[0] > r[0] ? q[0] : r[0], l1 = q[1] > r[1] ? q[1] : r[1];
      const double h0 = q[2] < r[2] ? q[2] : r[2], h1 = q[3] < r[3] ? q[3] : r[3];
      const double w0 = h0 - l0 > 0.0 ? h0 - l0 : 0.0, w1 = h1 - l1 > 0.0 ? h1 - l1 : 0.0;
      const double inter = w0 * w1;
      double iou = 1.0 * inter / (qa + ra - inter);
      const double eps = 1.1920928955078125e-07;        // np.finfo(np.float32).eps
      iou = iou > eps ? iou : eps;
      const double wgt = exp(-(1.0 * (iou * iou) / sigma));
      sc[i] = sc[i] * wgt;
      if (!(sc[i] > 0.0)) alive[i] = 0;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) nkeep[ci] = count;
}

// tf_centernet.py:6-19 center_dist_1d / _2d on a grid of n points (float64): g = 1 / (x - mu_x)^p
// [* 1 / (y - mu_y)^p], divided by its maximum (tf.reduce_max).  One workgroup: pass 1 the values
// and a block max (NaN-propagating like reduce_max over inf/nan is not modelled: the reference grids
// never hit a pole), pass 2 the division.
__global__ void center_dist_kernel(const double* gx, const double* gy, int n, double mu_x, double mu_y,
                                   double spread, double* out) {
  __shared__ double red[NT];
  double m = -INFINITY;
  for (int i = threadIdx.x; i < n; i += NT) {
    double g = 1.0 / pow(gx[i] - mu_x, spread);
    if (gy) g = g * (1.0 / pow(gy[i] - mu_y, spread));
    out[i] = g;
    m = g > m ? g : m;
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w = NT / 2; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] = red[threadIdx.x + w] > red[threadIdx.x] ? red[threadIdx.x + w] : red[threadIdx.x];
    __syncthreads();
  }
  const double z = red[0];
  for (int i = threadIdx.x; i < n; i += NT) out[i] = out[i] / z;
}

}  // namespace

#define S_ ((hipStream_t)stream)

extern "C" int cvl_retina_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B, int n_max,
                                 int pad, int num_classes, const float* anchor_dims, int n_anchors,
                                 const int32_t* strides, float iou_thresh, float* targets, int32_t* num_targets,
                                 cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && img_dim && anchor_dims && strides && targets && num_targets);
  CVL_CHECK_ARG(B > 0 && n_max > 0 && n_max <= kMaxBox && pad > 0 && num_classes > 0 &&
                num_classes <= 32 * kWords && n_anchors > 0);
  RetinaArgs a;
  a.boxes = boxes; a.nbox = nbox; a.img_dim = img_dim; a.adims = anchor_dims; a.out = targets;
  a.ntgt = num_targets; a.n_max = n_max; a.C = num_classes; a.A = n_anchors; a.pad = pad;
  a.thresh = iou_thresh;
  a.off[0] = 0;
  for (int l = 0; l < 5; ++l) {
    CVL_CHECK_ARG(strides[l] > 0);
    a.stride[l] = strides[l];
    a.S[l] = pad / strides[l];
    a.off[l + 1] = a.off[l] + n_anchors * a.S[l] * a.S[l];
  }
  a.P = a.off[5];
  const size_t lds = (size_t)RT * (4 + num_classes) * sizeof(float);
  CVL_CHECK_ARG(lds <= 60 * 1024);
  hipError_t e = hipMemsetAsync(num_targets, 0, sizeof(int32_t) * B, S_);
  if (e != hipSuccess) return CVL_EHIP + (int)e;
  hipLaunchKernelGGL(retina_assign_kernel, dim3((a.P + RT - 1) / RT, B), dim3(RT), lds, S_, a);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B,
                                    int n_max, int pad_h, int pad_w, int num_classes, int stride,
                                    float* targets, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && img_dim && targets && B > 0 && n_max > 0 && n_max <= kMaxBox);
  CVL_CHECK_ARG(num_classes > 0 && num_classes <= 32 * kWords && stride > 0 && pad_h > 0 && pad_w > 0);
  CenterArgs a;
  a.boxes = boxes; a.nbox = nbox; a.img_dim = img_dim; a.out = targets; a.n_max = n_max;
  a.C = num_classes; a.stride = stride;
  // tf_centernet_hourglass.py:395-398: h_max uses img_pad[1], w_max img_pad[0] (swapped)
  a.hm = pad_w / stride;
  a.wm = pad_h / stride;
  a.pad_h = (float)pad_h; a.pad_w = (float)pad_w;
  const int cells = a.hm * a.wm;
  int gx = (cells + NT - 1) / NT;
  gx = gx > 64 ? 64 : gx;
  hipLaunchKernelGGL(centernet_assign_kernel, dim3(gx, B), dim3(NT), 0, S_, a);
  return cvl_launch_status();
}

extern "C" int cvl_center_dist(const double* grid_x, const double* grid_y, int n, double mu_x, double mu_y,
                               double spread, double* out, cvl_stream_t stream) {
  CVL_CHECK_ARG(grid_x && out && n > 0);
  hipLaunchKernelGGL(center_dist_kernel, dim3(1), dim3(NT), 0, S_, grid_x, grid_y, n, mu_x, mu_y, spread, out);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_splat(const float* boxes, const int32_t* nbox, const float* img_dim, int B,
                                   int n_max, int pad_h, int pad_w, int num_classes, int stride, float sigma,
                                   float* targets, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && img_dim && targets && B > 0 && n_max > 0 && n_max <= kMaxBox);
  CVL_CHECK_ARG(num_classes > 0 && num_classes <= 32 * kWords && stride > 0);
  SplatArgs a;
  a.boxes = boxes; a.nbox = nbox; a.img_dim = img_dim; a.out = targets; a.n_max = n_max;
  a.C = num_classes; a.Hs = pad_h / stride; a.Ws = pad_w / stride; a.stride = stride;
  a.sigma = sigma; a.spread = 8.0f;              // tmp_std forced to 8.0 (tf_centernet.py:206-207)
  const int cells = a.Hs * a.Ws;
  int gx = (cells + NT - 1) / NT;
  gx = gx > 64 ? 64 : gx;
  hipLaunchKernelGGL(centernet_splat_kernel, dim3(gx, B), dim3(NT), 0, S_, a);
  return cvl_launch_status();
}

extern "C" size_t cvl_det_loss_workspace_size(int B, int P) {
  return (size_t)B * ((P + NT - 1) / NT) * 2 * sizeof(double);
}

extern "C" int cvl_det_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                            const float* targets, int B, int P, int num_classes, float grad_scale_cls,
                            float grad_scale_reg, float* losses, float* d_reg, float* d_cls, void* workspace,
                            cvl_stream_t stream) {
  CVL_CHECK_ARG(reg_pred && cls_pred && targets && losses && workspace && ld_reg >= 4 && ld_cls >= num_classes);
  DetLossArgs a;
  a.reg = reg_pred; a.cls = cls_pred; a.tgt = targets; a.partial = (double*)workspace;
  a.dreg = d_reg; a.dcls = d_cls; a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.P = P; a.C = num_classes;
  a.tiles = (P + NT - 1) / NT;
  a.grad_scale_cls = grad_scale_cls; a.grad_scale_reg = grad_scale_reg;
  hipLaunchKernelGGL(det_loss_kernel, dim3(a.tiles, B), dim3(NT), 0, S_, a);
  hipLaunchKernelGGL(det_loss_finalize, dim3(B), dim3(FIN_T), 0, S_, (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

extern "C" size_t cvl_retina_loss_workspace_size(int B, int P, int n_anchors) {
  return (size_t)B * (((size_t)P * n_anchors + RL_ROWS - 1) / RL_ROWS) * 2 * sizeof(double);
}

static int retina_loss_impl(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                            const float* targets, int B, const int32_t* level_cells, int n_anchors,
                            int num_classes, const float* img_weight, float grad_scale, float* losses,
                            void* d_reg, int ld_dreg, void* d_cls, int ld_dcls, void* workspace,
                            cvl_stream_t stream, int grad_f32) {
  CVL_CHECK_ARG(reg_pred && cls_pred && targets && losses && workspace && level_cells && B > 0);
  CVL_CHECK_ARG(n_anchors > 0 && num_classes > 0 && ld_reg >= 4 * n_anchors && ld_cls >= n_anchors * num_classes);
  CVL_CHECK_ARG(!d_reg || ld_dreg >= 4 * n_anchors);
  CVL_CHECK_ARG(!d_cls || ld_dcls >= n_anchors * num_classes);
  RetinaLossArgs a;
  a.reg = reg_pred; a.cls = cls_pred; a.tgt = targets; a.img_w = img_weight;
  a.partial = (double*)workspace;
  a.dreg = (cvl_bf16*)d_reg; a.dcls = (cvl_bf16*)d_cls;
  a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.ld_dreg = ld_dreg; a.ld_dcls = ld_dcls;
  a.A = n_anchors; a.C = num_classes; a.grad_scale = grad_scale;
  a.grad_f32 = grad_f32;
  int o = 0;
  for (int l = 0; l < 5; ++l) {
    CVL_CHECK_ARG(level_cells[l] > 0);
    a.off[l] = o;
    o += level_cells[l];
  }
  a.off[5] = o;
  a.P = o;
  CVL_CHECK_ARG(4 + num_classes <= RL_MAXW);
  a.tiles = (int)(((long)a.P * a.A + RL_ROWS - 1) / RL_ROWS);
  hipLaunchKernelGGL(retina_loss_kernel, dim3(a.tiles, B), dim3(NT), 0, S_, a);
  hipLaunchKernelGGL(det_loss_finalize, dim3(B), dim3(FIN_T), 0, S_, (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

extern "C" int cvl_retina_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                               const float* targets, int B, const int32_t* level_cells, int n_anchors,
                               int num_classes, const float* img_weight, float grad_scale, float* losses,
                               void* d_reg, int ld_dreg, void* d_cls, int ld_dcls, void* workspace,
                               cvl_stream_t stream) {
  return retina_loss_impl(reg_pred, ld_reg, cls_pred, ld_cls, targets, B, level_cells, n_anchors, num_classes,
                          img_weight, grad_scale, losses, d_reg, ld_dreg, d_cls, ld_dcls, workspace, stream, 0);
}

extern "C" int cvl_retina_loss_f32(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                                   const float* targets, int B, const int32_t* level_cells, int n_anchors,
                                   int num_classes, const float* img_weight, float grad_scale, float* losses,
                                   float* d_reg, int ld_dreg, float* d_cls, int ld_dcls, void* workspace,
                                   cvl_stream_t stream) {
  return retina_loss_impl(reg_pred, ld_reg, cls_pred, ld_cls, targets, B, level_cells, n_anchors, num_classes,
                          img_weight, grad_scale, losses, d_reg, ld_dreg, d_cls, ld_dcls, workspace, stream, 1);
}

extern "C" size_t cvl_nms_workspace_size(int n, int ncls) { return (size_t)n * ncls + 16; }

extern "C" int cvl_nms(const double* boxes, int n, const double* classes, int ncls, double iou_threshold,
                       int32_t* keep, int32_t* nkeep, void* workspace, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && classes && keep && nkeep && workspace && n > 0 && ncls > 0);
  hipLaunchKernelGGL(nms_kernel, dim3(ncls), dim3(NT), 0, S_, boxes, n, classes, ncls, iou_threshold, keep,
                     nkeep, (uint8_t*)workspace);
  return cvl_launch_status();
}

extern "C" size_t cvl_soft_nms_workspace_size(int n, int ncls) {
  return (size_t)n * ncls * (sizeof(double) + 1) + 16;
}

extern "C" int cvl_soft_nms(const double* boxes, int n, const double* classes, int ncls, double sigma,
                            int32_t* keep, double* keep_score, int32_t* nkeep, void* workspace,
                            cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && classes && keep && keep_score && nkeep && workspace && n > 0 && ncls > 0 && sigma > 0.0);
  double* scw = reinterpret_cast<double*>(workspace);
  uint8_t* alive = reinterpret_cast<uint8_t*>(scw + (size_t)n * ncls);
  hipLaunchKernelGGL(soft_nms_kernel, dim3(ncls), dim3(NT), 0, S_, boxes, n, classes, ncls, sigma, keep, keep_score,
                     nkeep, scw, alive);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_loss(const float* pred, int ld_pred, const float* targets, int B, int P, int num_classes,
                                  float cls_scale, float reg_scale, float* losses, void* d_pred, int ld_d,
                                  void* workspace, cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && targets && losses && d_pred && workspace && B > 0 && P > 0 && num_classes > 0);
  CVL_CHECK_ARG(ld_pred >= 4 + num_classes && ld_d >= 4 + num_classes);
  CnLossArgs a;
  a.pred = pred; a.tgt = targets; a.partial = (double*)workspace; a.d = (cvl_bf16*)d_pred;
  a.ld_pred = ld_pred; a.ld_d = ld_d; a.P = P; a.C = num_classes; a.tiles = (P + NT - 1) / NT;
  a.cls_scale = cls_scale; a.reg_scale = reg_scale;
  hipLaunchKernelGGL(centernet_loss_kernel, dim3(a.tiles, B), dim3(NT), 0, S_, a);
  hipLaunchKernelGGL(det_loss_finalize, dim3(B), dim3(FIN_T), 0, S_, (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_decode(const float* pred, int ld, int H, int W, int num_classes, double stride,
                                    float thresh, double w_ratio, double h_ratio, double img_width,
                                    double img_height, double* rows, int32_t* count, cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && rows && count && H > 0 && W > 0 && num_classes > 0 && ld >= 4 + num_classes);
  hipLaunchKernelGGL(centernet_decode_kernel, dim3(1), dim3(1024), 0, S_, pred, ld, H, W, num_classes, stride, thresh,
                     w_ratio, h_ratio, img_width, img_height, rows, count);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_scale_decode(const float* pred, int ld, int H, int W, int n_scales, int ch_per_scale,
                                          int cls0, int num_classes, int box_mode, const double* box_scales,
                                          float stride, float thresh, double w_ratio, double h_ratio,
                                          double img_width, double img_height, double* rows, int32_t* count,
                                          cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && rows && count && box_scales && H > 0 && W > 0 && num_classes > 0);
  CVL_CHECK_ARG(n_scales > 0 && n_scales <= 16 && (box_mode == 1 || box_mode == 2));
  CVL_CHECK_ARG(cls0 >= 4 && ch_per_scale >= cls0 + num_classes && ld >= n_scales * ch_per_scale);
  ScaleDecodeArgs a;
  a.pred = pred; a.rows = rows; a.count = count;
  a.ld = ld; a.H = H; a.W = W; a.ns = n_scales; a.chs = ch_per_scale; a.cls0 = cls0; a.C = num_classes;
  a.mode = box_mode; a.stride = stride; a.thresh = thresh;
  a.w_ratio = w_ratio; a.h_ratio = h_ratio; a.img_w = img_width; a.img_h = img_height;
  for (int s = 0; s < 16; ++s) a.scale[s] = s < n_scales ? box_scales[s] : 0.0;
  hipLaunchKernelGGL(centernet_scale_decode_kernel, dim3(1), dim3(1024), 0, S_, a);
  return cvl_launch_status();
}

extern "C" int cvl_hourglass_v2_assign(const float* boxes, const int32_t* nbox, int B, int n_max, int raw_dims,
                                       int img_dims, int num_classes, float* targets, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && targets && B > 0 && n_max > 0 && n_max <= kMaxBox);
  CVL_CHECK_ARG(num_classes > 0 && num_classes <= 32 * kWords && raw_dims > 0 && img_dims >= raw_dims);
  CVL_CHECK_ARG(img_dims % 8 == 0);
  Hg2Args a;
  a.boxes = boxes; a.nbox = nbox; a.out = targets; a.n_max = n_max; a.C = num_classes;
  a.S = img_dims / 8; a.raw = raw_dims; a.img = img_dims;
  const int rows = a.S * a.S * 4;
  int gx = (rows + NT - 1) / NT;
  gx = gx > 64 ? 64 : gx;
  hipLaunchKernelGGL(hg2_assign_kernel, dim3(gx, B), dim3(NT), 0, S_, a);
  return cvl_launch_status();
}

extern "C" size_t cvl_hourglass_v2_loss_workspace_size(int B, int P) {
  return (size_t)B * ((4 * (size_t)P + NT - 1) / NT) * 2 * sizeof(double);
}

extern "C" int cvl_hourglass_v2_loss(const float* pred, int ld_pred, const float* targets, int B, int P,
                                     int num_classes, int loss_type, float cls_scale, float reg_scale, float* losses,
                                     void* d_pred, int ld_d, void* workspace, cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && targets && losses && d_pred && workspace && B > 0 && P > 0 && num_classes > 0);
  CVL_CHECK_ARG(ld_pred >= 4 * (5 + num_classes) && ld_d >= 4 * (5 + num_classes) && loss_type >= 0 && loss_type <= 3);
  Hg2LossArgs a;
  a.pred = pred; a.tgt = targets; a.partial = (double*)workspace; a.d = (cvl_bf16*)d_pred;
  a.ld_pred = ld_pred; a.ld_d = ld_d; a.P = P; a.C = num_classes; a.tiles = (4 * P + NT - 1) / NT;
  a.sce = loss_type; a.cls_scale = cls_scale; a.reg_scale = reg_scale;
  hipLaunchKernelGGL(hg2_loss_kernel, dim3(a.tiles, B), dim3(NT), 0, S_, a);
  hipLaunchKernelGGL(det_loss_finalize, dim3(B), dim3(FIN_T), 0, S_, (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

extern "C" int cvl_centernet_s8_assign(const float* boxes, const int32_t* nbox, const float* img_dim, int B,
                                       int n_max, int pad_h, int pad_w, int num_classes, const float* box_scales,
                                       int n_scales, int stride, float* targets, cvl_stream_t stream) {
  CVL_CHECK_ARG(boxes && nbox && img_dim && targets && box_scales && B > 0 && n_max > 0 && n_max <= kMaxBox);
  CVL_CHECK_ARG(num_classes > 0 && num_classes <= 32 * kWords && stride > 0 && n_scales > 0 &&
                n_scales <= kMaxScales);
  S8Args a;
  a.boxes = boxes; a.nbox = nbox; a.img_dim = img_dim; a.out = targets; a.n_max = n_max; a.C = num_classes;
  a.hm = (int)((double)pad_w / stride); a.wm = (int)((double)pad_h / stride);   // h_max from img_pad[1]
  a.ns = n_scales; a.stride = stride; a.pad_h = pad_h; a.pad_w = pad_w;
  for (int s = 0; s < kMaxScales; ++s) a.scales[s] = s < n_scales ? (double)box_scales[s] : 0.0;
  const int rows = a.hm * a.wm * a.ns;
  int gx = (rows + NT - 1) / NT;
  gx = gx > 64 ? 64 : gx;
  hipLaunchKernelGGL(s8_assign_kernel, dim3(gx, B), dim3(NT), 0, S_, a);
  return cvl_launch_status();
}

extern "C" size_t cvl_centernet_s8_loss_workspace_size(int B, int P, int n_scales) {
  return (size_t)B * (((size_t)P * n_scales + NT - 1) / NT) * 2 * sizeof(double);
}

extern "C" int cvl_centernet_s8_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                                     const float* targets, int B, int P, int n_scales, int num_classes,
                                     float cls_scale, float reg_scale, float* losses, void* d_reg, int ld_dreg,
                                     void* d_cls, int ld_dcls, void* workspace, cvl_stream_t stream) {
  CVL_CHECK_ARG(reg_pred && cls_pred && targets && losses && d_reg && d_cls && workspace && B > 0 && P > 0);
  CVL_CHECK_ARG(n_scales > 0 && num_classes > 0 && ld_reg >= 4 * n_scales && ld_cls >= num_classes * n_scales);
  CVL_CHECK_ARG(ld_dreg >= 4 * n_scales && ld_dcls >= num_classes * n_scales);
  S8LossArgs a;
  a.reg = reg_pred; a.cls = cls_pred; a.tgt = targets; a.partial = (double*)workspace;
  a.dreg = (cvl_bf16*)d_reg; a.dcls = (cvl_bf16*)d_cls;
  a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.ld_dreg = ld_dreg; a.ld_dcls = ld_dcls;
  a.P = P; a.C = num_classes; a.ns = n_scales; a.tiles = (P * n_scales + NT - 1) / NT;
  a.cls_scale = cls_scale; a.reg_scale = reg_scale;
  hipLaunchKernelGGL(s8_loss_kernel, dim3(a.tiles, B), dim3(NT), 0, S_, a);
  hipLaunchKernelGGL(det_loss_finalize, dim3(B), dim3(FIN_T), 0, S_, (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

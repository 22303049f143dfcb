// Depthwise convolution (Keras DepthwiseConv2D, depth_multiplier 1, no bias) on gfx950: the
// MobileNetV2 backbone's 3x3 stride-1 / stride-2 layers (tf.keras.applications.MobileNetV2, the
// `backbone_model="mobilenetv2"` branch of FCOS/fcos.py:36-41, RetinaNet/retinanet_module.py:68,
// CenterNet/tf_centernet*.py).  NHWC bf16 activations, fp32 HWC kernels [k][k][C], fp32
// accumulation.  Each op touches every activation element a bounded number of times and does
// k*k MACs per element: HBM-bound, so the kernels are 16-byte vector streams with the k*k-fold
// re-reads of the shifted taps served by L1 / L2:
//   * forward: one thread per (output pixel, 8 channels), k*k taps (zero padding by bounds);
//   * data gradient: one thread per (input pixel, 8 channels), the gather form of the transposed
//     conv (stride-aware), optional beta accumulate;
//   * weight gradient: per (row chunk, image-flat) block partial sums [k*k][C] over its output
//     pixels, reduced across the block's pixel lanes through LDS, then a fixed-order column
//     reduction over the blocks (deterministic, no atomics).
// Padding: explicit (pad_t, pad_l); TF "same" and Keras' ZeroPadding2D(correct_pad) + "valid" are
// both expressed this way by the caller.
#include "conv_common.h"

namespace {

constexpr int NT = 256;
constexpr int KMAX = 7;

__device__ __forceinline__ void unpack8(s16x8 v, float* f) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = bf16_to_f32((cvl_bf16)v[i]);
}
__device__ __forceinline__ s16x8 pack8(const float* f) {
  s16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (short)f32_to_bf16(f[i]);
  return v;
}

inline int grid_for(long n, int cap = 8192) {
  long b = (n + NT - 1) / NT;
  return (int)(b > cap ? cap : (b < 1 ? 1 : b));
}

struct DwGeo {
  int H, W, C, Ho, Wo, k, s, pt, pl;
};

template <int K>
__global__ void __launch_bounds__(NT) dw_fwd_kernel(const cvl_bf16* __restrict__ x, const float* __restrict__ w,
                                                    cvl_bf16* __restrict__ y, DwGeo g, long total) {
  const int C8 = g.C / 8;
  const int k = K > 0 ? K : g.k;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)g.Ho * g.Wo;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int oy = q / g.Wo, ox = q - (q / g.Wo) * g.Wo;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ky = 0; ky < k; ++ky) {
      const int iy = oy * g.s - g.pt + ky;
      if (iy < 0 || iy >= g.H) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int ix = ox * g.s - g.pl + kx;
        if (ix < 0 || ix >= g.W) continue;
        float v[8];
        unpack8(*reinterpret_cast<const s16x8*>(x + (((long)b * g.H + iy) * g.W + ix) * g.C + c0), v);
        const float4 w0 = *reinterpret_cast<const float4*>(w + ((long)ky * k + kx) * g.C + c0);
        const float4 w1 = *reinterpret_cast<const float4*>(w + ((long)ky * k + kx) * g.C + c0 + 4);
        acc[0] += v[0] * w0.x; acc[1] += v[1] * w0.y; acc[2] += v[2] * w0.z; acc[3] += v[3] * w0.w;
        acc[4] += v[4] * w1.x; acc[5] += v[5] * w1.y; acc[6] += v[6] * w1.z; acc[7] += v[7] * w1.w;
      }
    }
    *reinterpret_cast<s16x8*>(y + pix * g.C + c0) = pack8(acc);
  }
}

template <int K>
__global__ void __launch_bounds__(NT) dw_dgrad_kernel(const cvl_bf16* __restrict__ dy, const float* __restrict__ w,
                                                      cvl_bf16* __restrict__ dx, DwGeo g, long total, float beta) {
  const int C8 = g.C / 8;
  const int k = K > 0 ? K : g.k;
  for (long i = blockIdx.x * (long)NT + threadIdx.x; i < total; i += (long)gridDim.x * NT) {
    const long pix = i / C8;
    const int c0 = (int)(i - pix * C8) * 8;
    const long hw = (long)g.H * g.W;
    const int b = (int)(pix / hw);
    const int q = (int)(pix - (long)b * hw);
    const int iy = q / g.W, ix = q - (q / g.W) * g.W;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ky = 0; ky < k; ++ky) {
      const int ty = iy + g.pt - ky;
      if (ty < 0 || ty % g.s) continue;
      const int oy = ty / g.s;
      if (oy >= g.Ho) continue;
      for (int kx = 0; kx < k; ++kx) {
        const int tx = ix + g.pl - kx;
        if (tx < 0 || tx % g.s) continue;
        const int ox = tx / g.s;
        if (ox >= g.Wo) continue;
        float v[8];
        unpack8(*reinterpret_cast<const s16x8*>(dy + (((long)b * g.Ho + oy) * g.Wo + ox) * g.C + c0), v);
        const float4 w0 = *reinterpret_cast<const float4*>(w + ((long)ky * k + kx) * g.C + c0);
        const float4 w1 = *reinterpret_cast<const float4*>(w + ((long)ky * k + kx) * g.C + c0 + 4);
        acc[0] += v[0] * w0.x; acc[1] += v[1] * w0.y; acc[2] += v[2] * w0.z; acc[3] += v[3] * w0.w;
        acc[4] += v[4] * w1.x; acc[5] += v[5] * w1.y; acc[6] += v[6] * w1.z; acc[7] += v[7] * w1.w;
      }
    }
    if (beta != 0.f) {
      float o[8];
      unpack8(*reinterpret_cast<const s16x8*>(dx + pix * g.C + c0), o);
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += beta * o[u];
    }
    *reinterpret_cast<s16x8*>(dx + pix * g.C + c0) = pack8(acc);
  }
}

// partial[blk][t][c] = sum over this block's output pixels of x(tap t) * dy.  Threads own 8
// channels (tpr threads per pixel, rpp pixel lanes); pixels [p0, p1) of the flattened B*Ho*Wo.
template <int K>
__global__ void __launch_bounds__(NT) dw_wgrad_kernel(const cvl_bf16* __restrict__ x, const cvl_bf16* __restrict__ dy,
                                                      float* __restrict__ part, DwGeo g, long npix, int pix_per_blk) {
  constexpr int KK = K * K;
  constexpr int k = K;
  const int C8 = g.C / 8;
  const int tpr = C8 < NT ? C8 : NT;
  const int rpp = NT / tpr;
  const int cg = threadIdx.x % tpr, lane = threadIdx.x / tpr;
  const long p0 = (long)blockIdx.x * pix_per_blk;
  const long p1 = p0 + pix_per_blk < npix ? p0 + pix_per_blk : npix;
  const long hw = (long)g.Ho * g.Wo;
  __shared__ float red[NT][9];
  const int n_iter = (C8 + tpr - 1) / tpr;
  for (int itr = 0; itr < n_iter; ++itr) {
    const int cgb = itr * tpr + cg;
    const bool act = cgb < C8 && lane < rpp;
    const int c0 = (cgb < C8 ? cgb : C8 - 1) * 8;
    float acc[KK][8];
#pragma unroll
    for (int t = 0; t < KK; ++t)
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[t][u] = 0.f;
    if (act) {
      for (long p = p0 + lane; p < p1; p += rpp) {
        const int b = (int)(p / hw);
        const int q = (int)(p - (long)b * hw);
        const int oy = q / g.Wo, ox = q - (q / g.Wo) * g.Wo;
        float gd[8];
        unpack8(*reinterpret_cast<const s16x8*>(dy + p * g.C + c0), gd);
#pragma unroll
        for (int ky = 0; ky < k; ++ky) {
          const int iy = oy * g.s - g.pt + ky;
          if (iy < 0 || iy >= g.H) continue;
#pragma unroll
          for (int kx = 0; kx < k; ++kx) {
            const int ix = ox * g.s - g.pl + kx;
            if (ix < 0 || ix >= g.W) continue;
            float v[8];
            unpack8(*reinterpret_cast<const s16x8*>(x + (((long)b * g.H + iy) * g.W + ix) * g.C + c0), v);
            const int t = ky * k + kx;
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[t][u] += v[u] * gd[u];
          }
        }
      }
    }
    // reduce the rpp pixel lanes of each channel group, one tap at a time (fixed order)
#pragma unroll
    for (int t = 0; t < KK; ++t) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 8; ++u) red[threadIdx.x][u] = acc[t][u];
      __syncthreads();
      if (lane == 0 && cgb < C8) {
        float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int r = 0; r < rpp; ++r)
#pragma unroll
          for (int u = 0; u < 8; ++u) s[u] += red[r * tpr + cg][u];
        float* o = part + ((long)blockIdx.x * k * k + t) * g.C + c0;
        *reinterpret_cast<float4*>(o) = make_float4(s[0], s[1], s[2], s[3]);
        *reinterpret_cast<float4*>(o + 4) = make_float4(s[4], s[5], s[6], s[7]);
      }
    }
  }
}

// 3x3 / stride 1 weight gradient with a sliding tap window: a pixel lane walks a run of `seg`
// consecutive output pixels of one row, keeping the 3x3 window of x (3 rows x 3 columns x 8
// channels) in registers, so each step loads one new x column (3 rows) and one dy vector instead
// of 9 + 1 (the CenterNet hourglass's split separable convs at 256x256 / 128x128).  Same
// partial layout and fixed-order reductions as dw_wgrad_kernel.
__global__ void __launch_bounds__(NT) dw_wgrad_rows_kernel(const cvl_bf16* __restrict__ x,
                                                           const cvl_bf16* __restrict__ dy, float* __restrict__ part,
                                                           DwGeo g, int seg, int spr, long nseg) {
  const int C8 = g.C / 8;
  const int tpr = C8;                          // host: C8 <= NT
  const int rpp = NT / tpr;
  const int cg = threadIdx.x % tpr, lane = threadIdx.x / tpr;
  const int c0 = cg * 8;
  __shared__ float red[NT][9];
  float acc[9][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[t][u] = 0.f;
  const long sgi = (long)blockIdx.x * rpp + lane;
  if (lane < rpp && sgi < nseg) {
    const long row = sgi / spr;                          // b * Ho + oy
    const int x0 = (int)(sgi - row * spr) * seg;
    const int x1 = x0 + seg < g.Wo ? x0 + seg : g.Wo;
    const int b = (int)(row / g.Ho), oy = (int)(row - (long)b * g.Ho);
    const cvl_bf16* xb = x + (long)b * g.H * g.W * g.C + c0;
    bool rok[3];
    long roff[3];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int iy = oy - g.pt + ky;
      rok[ky] = iy >= 0 && iy < g.H;
      roff[ky] = (long)(rok[ky] ? iy : 0) * g.W;
    }
    auto ld = [&](int ky, int ix, float* v) {
      if (rok[ky] && ix >= 0 && ix < g.W) {
        unpack8(*reinterpret_cast<const s16x8*>(xb + (roff[ky] + ix) * g.C), v);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = 0.f;
      }
    };
    float win[3][3][8];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      ld(ky, x0 - g.pl, win[ky][0]);
      ld(ky, x0 - g.pl + 1, win[ky][1]);
    }
    const cvl_bf16* dyr = dy + row * g.Wo * g.C + c0;
    for (int ox = x0; ox < x1; ++ox) {
      float gd[8];
      unpack8(*reinterpret_cast<const s16x8*>(dyr + (long)ox * g.C), gd);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) ld(ky, ox - g.pl + 2, win[ky][2]);
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
          for (int u = 0; u < 8; ++u) acc[ky * 3 + kx][u] += win[ky][kx][u] * gd[u];
#pragma unroll
      for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int u = 0; u < 8; ++u) { win[ky][0][u] = win[ky][1][u]; win[ky][1][u] = win[ky][2][u]; }
    }
  }
  // reduce the rpp pixel lanes of each channel group, one tap at a time (fixed order)
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) red[threadIdx.x][u] = acc[t][u];
    __syncthreads();
    if (lane == 0) {
      float sm[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < rpp; ++r)
#pragma unroll
        for (int u = 0; u < 8; ++u) sm[u] += red[r * tpr + cg][u];
      float* o = part + ((long)blockIdx.x * 9 + t) * g.C + c0;
      *reinterpret_cast<float4*>(o) = make_float4(sm[0], sm[1], sm[2], sm[3]);
      *reinterpret_cast<float4*>(o + 4) = make_float4(sm[4], sm[5], sm[6], sm[7]);
    }
  }
}

// row-walk plan of dw_wgrad_rows_kernel: segment length, segments per row, blocks (0 = not taken)
inline int rows_plan(int B, int Ho, int Wo, int C, int k, int s, int* seg, int* spr) {
  if (k != 3 || s != 1 || C / 8 > NT || cvl_tune_flag("CVL_DW_NO_ROWS")) return 0;
  *seg = Wo >= 128 ? 32 : (Wo >= 32 ? 16 : 8);
  *spr = (Wo + *seg - 1) / *seg;
  const int rpp = NT / (C / 8);
  const long nseg = (long)B * Ho * *spr;
  return (int)((nseg + rpp - 1) / rpp);
}

// dw[i] = beta*dw[i] + sum_b part[b][i]: a block owns 32 consecutive outputs and 8 block lanes;
// lane l sums partials l, l+8, ... with 4 loads in flight, then the 8 lane sums are added in a
// fixed order (deterministic; hundreds of partials per output at large maps)
__global__ void __launch_bounds__(256) dw_wgrad_reduce_kernel(const float* __restrict__ part, float* __restrict__ dw,
                                                              long n, int nblk, float beta) {
  __shared__ float red[8][33];
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const long i = (long)blockIdx.x * 32 + col;
  float acc = 0.f;
  if (i < n) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int b = sl;
    for (; b + 24 < nblk; b += 32) {
      a0 += part[(long)b * n + i];
      a1 += part[(long)(b + 8) * n + i];
      a2 += part[(long)(b + 16) * n + i];
      a3 += part[(long)(b + 24) * n + i];
    }
    for (; b < nblk; b += 8) a0 += part[(long)b * n + i];
    acc = (a0 + a1) + (a2 + a3);
  }
  red[sl][col] = acc;
  __syncthreads();
  if (sl == 0 && i < n) {
    float s = red[0][col];
#pragma unroll
    for (int k = 1; k < 8; ++k) s += red[k][col];
    dw[i] = (beta != 0.f ? beta * dw[i] : 0.f) + s;
  }
}

inline int wgrad_pix_per_blk(long npix, int C) {
  const int C8 = C / 8;
  const int rpp = NT / (C8 < NT ? C8 : NT);
  long want = npix / 1024;                             // ~1024 blocks
  if (want < rpp * 8) want = rpp * 8;                  // >= 8 pixels per lane
  return (int)((want + rpp - 1) / rpp * rpp);
}

bool geo_ok(int B, int H, int W, int C, int k, int s, int pt, int pl, int Ho, int Wo) {
  return B > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && k > 0 && k <= KMAX && s > 0 && pt >= 0 && pl >= 0 &&
         Ho > 0 && Wo > 0;
}

}  // namespace

#define S_ ((hipStream_t)stream)

extern "C" int cvl_depthwise_fwd(const void* x, const float* w, void* y, int B, int H, int W, int C, int k, int stride,
                                 int pad_t, int pad_l, int Ho, int Wo, cvl_stream_t stream) {
  CVL_CHECK_ARG(x && w && y && geo_ok(B, H, W, C, k, stride, pad_t, pad_l, Ho, Wo));
  DwGeo g{H, W, C, Ho, Wo, k, stride, pad_t, pad_l};
  const long total = (long)B * Ho * Wo * (C / 8);
  if (k == 3)
    hipLaunchKernelGGL(dw_fwd_kernel<3>, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)x, w, (cvl_bf16*)y,
                       g, total);
  else
    hipLaunchKernelGGL(dw_fwd_kernel<0>, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)x, w, (cvl_bf16*)y,
                       g, total);
  return cvl_launch_status();
}

extern "C" int cvl_depthwise_dgrad(const void* dy, const float* w, void* dx, int B, int H, int W, int C, int k,
                                   int stride, int pad_t, int pad_l, int Ho, int Wo, float beta, cvl_stream_t stream) {
  CVL_CHECK_ARG(dy && w && dx && geo_ok(B, H, W, C, k, stride, pad_t, pad_l, Ho, Wo));
  DwGeo g{H, W, C, Ho, Wo, k, stride, pad_t, pad_l};
  const long total = (long)B * H * W * (C / 8);
  if (k == 3)
    hipLaunchKernelGGL(dw_dgrad_kernel<3>, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dy, w,
                       (cvl_bf16*)dx, g, total, beta);
  else
    hipLaunchKernelGGL(dw_dgrad_kernel<0>, dim3(grid_for(total)), dim3(NT), 0, S_, (const cvl_bf16*)dy, w,
                       (cvl_bf16*)dx, g, total, beta);
  return cvl_launch_status();
}

extern "C" size_t cvl_depthwise_wgrad_workspace_size(int B, int Ho, int Wo, int C, int k) {
  int seg, spr;
  const int rb = rows_plan(B, Ho, Wo, C, k, 1, &seg, &spr);   // (stride unknown here: size for both)
  const long npix = (long)B * Ho * Wo;
  const long nblk = (npix + wgrad_pix_per_blk(npix, C) - 1) / wgrad_pix_per_blk(npix, C);
  const long nb = rb > nblk ? rb : nblk;
  return (size_t)nb * k * k * C * sizeof(float);
}

extern "C" int cvl_depthwise_wgrad(const void* x, const void* dy, float* dw, float beta, int B, int H, int W, int C,
                                   int k, int stride, int pad_t, int pad_l, int Ho, int Wo, void* workspace,
                                   size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(x && dy && dw && workspace && geo_ok(B, H, W, C, k, stride, pad_t, pad_l, Ho, Wo));
  CVL_CHECK_ARG(k == 3);                       // the MobileNetV2 depthwise layers (register-resident taps)
  CVL_CHECK_ARG(workspace_bytes >= cvl_depthwise_wgrad_workspace_size(B, Ho, Wo, C, k));
  DwGeo g{H, W, C, Ho, Wo, k, stride, pad_t, pad_l};
  const long npix = (long)B * Ho * Wo;
  float* part = reinterpret_cast<float*>(workspace);
  int seg = 0, spr = 0;
  int nblk = rows_plan(B, Ho, Wo, C, k, stride, &seg, &spr);
  if (nblk > 0) {                              // stride 1: the sliding-window row walk
    hipLaunchKernelGGL(dw_wgrad_rows_kernel, dim3(nblk), dim3(NT), 0, S_, (const cvl_bf16*)x, (const cvl_bf16*)dy,
                       part, g, seg, spr, (long)B * Ho * spr);
  } else {
    const int ppb = wgrad_pix_per_blk(npix, C);
    nblk = (int)((npix + ppb - 1) / ppb);
    hipLaunchKernelGGL(dw_wgrad_kernel<3>, dim3(nblk), dim3(NT), 0, S_, (const cvl_bf16*)x, (const cvl_bf16*)dy, part,
                       g, npix, ppb);
  }
  const long n = (long)k * k * C;
  hipLaunchKernelGGL(dw_wgrad_reduce_kernel, dim3((unsigned)((n + 31) / 32)), dim3(256), 0, S_, (const float*)part, dw,
                     n, nblk, beta);
  return cvl_launch_status();
}

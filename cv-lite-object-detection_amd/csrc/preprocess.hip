// Input pipeline on MI355X (FCOS/data_preprocess.py:24-133): the
// per-image resize / normalise / pad / flip of `resize_and_pad_image` and
// `random_flip_horizontal`, one launch writing straight into a slot of the device batch.
//
//   out[y][x][c] = y < oh && x < ow ? bilinear(src', y, x, c) / 127.5 - 1 : 0      (pad value 0)
//   src'         = flip == 1 ? tf.image.flip_left_right(src) : src
//   flip == 2: the resize first, then the flip of its output (preprocess_data's pad_flag=False order,
//   :111-125): out[y][x] = resized[y][ow - 1 - x]
//
// bilinear = tf.image.resize(method="bilinear", antialias=False) of TF2, restated from TF's
// published kernel (TF is absent here, so parity is pinned to the numpy restatement, not TF):
// half-pixel centres, scale = in / out in fp32, in = (o + 0.5) * scale - 0.5, lower =
// max(floor(in), 0), upper = min(ceil(in), in - 1), lerp = in - floor(in);
// top = tl + (tr - tl) * xl, bottom = bl + (br - bl) * xl, v = top + (bottom - top) * yl, all fp32
// (built with -ffp-contract=off so no FMA changes the rounding).
#include "cvl_common.h"

namespace {

constexpr int PT = 256;

__global__ void __launch_bounds__(PT) resize_pad_kernel(const void* src, int src_u8, int H, int W, int C,
                                                        int flip, int oh, int ow, int ph, int pw, float* out) {
  const long i = (long)blockIdx.x * PT + threadIdx.x;
  if (i >= (long)ph * pw) return;
  const int y = (int)(i / pw), x = (int)(i - (long)(i / pw) * pw);
  float* o = out + i * C;
  if (y >= oh || x >= ow) {
    for (int c = 0; c < C; ++c) o[c] = 0.0f;
    return;
  }
  const float sy = (float)H / (float)oh, sx = (float)W / (float)ow;
  const int xs = flip == 2 ? ow - 1 - x : x;
  const float iny = ((float)y + 0.5f) * sy - 0.5f, inx = ((float)xs + 0.5f) * sx - 0.5f;
  const float fy = floorf(iny), fx = floorf(inx);
  const int y0 = fy > 0.f ? (int)fy : 0, x0 = fx > 0.f ? (int)fx : 0;
  const int y1 = (int)ceilf(iny) < H - 1 ? (int)ceilf(iny) : H - 1;
  const int x1 = (int)ceilf(inx) < W - 1 ? (int)ceilf(inx) : W - 1;
  const float yl = iny - fy, xl = inx - fx;
  const int c0 = flip == 1 ? W - 1 - x0 : x0, c1 = flip == 1 ? W - 1 - x1 : x1;
  for (int c = 0; c < C; ++c) {
    float tl, tr, bl, br;
    if (src_u8) {
      const uint8_t* s = (const uint8_t*)src;
      tl = s[((long)y0 * W + c0) * C + c]; tr = s[((long)y0 * W + c1) * C + c];
      bl = s[((long)y1 * W + c0) * C + c]; br = s[((long)y1 * W + c1) * C + c];
    } else {
      const float* s = (const float*)src;
      tl = s[((long)y0 * W + c0) * C + c]; tr = s[((long)y0 * W + c1) * C + c];
      bl = s[((long)y1 * W + c0) * C + c]; br = s[((long)y1 * W + c1) * C + c];
    }
    const float top = tl + (tr - tl) * xl;
    const float bot = bl + (br - bl) * xl;
    const float v = top + (bot - top) * yl;
    o[c] = v / 127.5f - 1.0f;
  }
}

}  // namespace

extern "C" int cvl_resize_pad_normalize(const void* src, int src_u8, int H, int W, int C, int flip, int out_h,
                                        int out_w, int pad_h, int pad_w, float* out, cvl_stream_t stream) {
  CVL_CHECK_ARG(src && out && H > 0 && W > 0 && C > 0 && C <= 4 && out_h > 0 && out_w > 0 && flip >= 0 && flip <= 2);
  CVL_CHECK_ARG(pad_h >= out_h && pad_w >= out_w && (long)pad_h * pad_w < (1L << 31));
  const long n = (long)pad_h * pad_w;
  hipLaunchKernelGGL(resize_pad_kernel, dim3((unsigned)((n + PT - 1) / PT)), dim3(PT), 0, (hipStream_t)stream, src,
                     src_u8, H, W, C, flip, out_h, out_w, pad_h, pad_w, out);
  return cvl_launch_status();
}

// ---------------------------------------------------------------------------------------------
// CenterNet v2 image_augment (CenterNet/train_hourglass_voc.py:24-67; restated in
// oracle/augment_ref.py): per image of a batch one of
//   0 none, 1 brightness x + delta, 2 contrast (x - mean_c) * f + mean_c (mean over the N x N pixels
//   of channel c), 3 flip left-right, 4 transpose, 5 transpose then flip up-down,
// applied to the padded image [N][N][3] fp32 and its target map [S][S][4][T] (T = 5 + C; the
// geometric ops move whole cells: 3 sets x-offset channel 1 to 1 - v, 4 / 5 write the transposed
// cell with channels 0 := 1 and 2 := 3 -- the reference's aliased swap -- and 5 then sets channel 0
// to 1 - v).  Two launches: the per-image channel sums of the contrast images (fixed-order partials,
// deterministic), then one launch doing every image's pixels and every target cell.  The pixel part
// moves 32 x 32-pixel tiles through LDS so both the (transposed) read and the write are coalesced.
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int AUG_T = 32;        // tile side, pixels
constexpr int AUG_PARTS = 64;    // partial-sum workgroups per contrast image
constexpr int AUG_TGT = 1024;    // target floats per workgroup

__global__ void __launch_bounds__(PT) augment_sums_kernel(const float* img, const int32_t* ops, int N,
                                                          double* part) {
  const int b = blockIdx.y;
  if (ops[b] != 2) return;
  const long npix = (long)N * N;
  const float* s = img + (long)b * npix * 3;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  for (long p = (long)blockIdx.x * PT + threadIdx.x; p < npix; p += (long)AUG_PARTS * PT) {
    a0 += s[p * 3];
    a1 += s[p * 3 + 1];
    a2 += s[p * 3 + 2];
  }
  __shared__ double red[3][PT];
  red[0][threadIdx.x] = a0;
  red[1][threadIdx.x] = a1;
  red[2][threadIdx.x] = a2;
  __syncthreads();
  for (int w = PT / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int c = 0; c < 3; ++c) red[c][threadIdx.x] += red[c][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x < 3) part[((long)b * AUG_PARTS + blockIdx.x) * 3 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void __launch_bounds__(PT) augment_apply_kernel(const float* img_src, float* img_dst, const float* tgt_src,
                                                           float* tgt_dst, const int32_t* ops, const float* params,
                                                           int N, int S, int T, int img_tiles, const double* part) {
  const int b = blockIdx.y;
  const int op = ops[b];
  const float prm = params[b];
  const int t = blockIdx.x;
  if (t >= img_tiles) {                          // target cells
    const long per = (long)S * S * 4 * T;
    const long e = (long)(t - img_tiles) * AUG_TGT;
    const float* src = tgt_src + (long)b * per;
    float* dst = tgt_dst + (long)b * per;
    for (int k = threadIdx.x; k < AUG_TGT; k += PT) {
      const long i = e + k;
      if (i >= per) break;
      const long q = i / (4 * T);
      const int w = (int)(i - q * 4 * T);
      const int j = w % T;
      const int y = (int)(q / S), x = (int)(q - (long)y * S);
      int sy = y, sx = x, sj = j;
      if (op == 3) sx = S - 1 - x;
      if (op == 4 || op == 5) {
        sy = x;
        sx = op == 5 ? S - 1 - y : y;
        sj = j == 0 ? 1 : (j == 2 ? 3 : j);
      }
      float v = src[((long)sy * S + sx) * 4 * T + (w - j + sj)];
      if ((op == 3 && j == 1) || (op == 5 && j == 0)) v = 1.0f - v;
      dst[i] = v;
    }
    return;
  }
  __shared__ float tile[AUG_T][AUG_T * 3 + 1];
  __shared__ float mean[3];
  if (op == 2 && threadIdx.x < 3) {
    double s = 0.0;
    for (int k = 0; k < AUG_PARTS; ++k) s += part[((long)b * AUG_PARTS + k) * 3 + threadIdx.x];
    mean[threadIdx.x] = (float)(s / ((double)N * (double)N));
  }
  const int ntx = (N + AUG_T - 1) / AUG_T;
  const int ty = t / ntx, tx = t - ty * ntx;
  // source region of this output tile: rows [r0, r0 + nr), columns [c0, c0 + nc)
  int r0 = ty * AUG_T, c0 = tx * AUG_T;
  if (op == 3) c0 = N - min(N, tx * AUG_T + AUG_T);
  if (op == 4) { r0 = tx * AUG_T; c0 = ty * AUG_T; }
  if (op == 5) { r0 = tx * AUG_T; c0 = N - min(N, ty * AUG_T + AUG_T); }
  const int nr = min(AUG_T, N - r0), nc = min(AUG_T, N - c0);
  const float* s = img_src + (long)b * N * N * 3;
  for (int i = threadIdx.x; i < AUG_T * AUG_T * 3; i += PT) {
    const int r = i / (AUG_T * 3), q = i - r * (AUG_T * 3);
    if (r < nr && q < nc * 3) tile[r][q] = s[((long)(r0 + r) * N + c0) * 3 + q];
  }
  __syncthreads();
  float* d = img_dst + (long)b * N * N * 3;
  for (int i = threadIdx.x; i < AUG_T * AUG_T * 3; i += PT) {
    const int yl = i / (AUG_T * 3), q = i - yl * (AUG_T * 3);
    const int xl = q / 3, ch = q - xl * 3;
    const int y = ty * AUG_T + yl, x = tx * AUG_T + xl;
    if (y >= N || x >= N) continue;
    int r = yl, c = xl;
    if (op == 3) c = N - 1 - x - c0;
    if (op == 4) { r = x - r0; c = y - c0; }
    if (op == 5) { r = x - r0; c = N - 1 - y - c0; }
    float v = tile[r][c * 3 + ch];
    if (op == 1) v = v + prm;
    if (op == 2) v = (v - mean[ch]) * prm + mean[ch];
    d[((long)y * N + x) * 3 + ch] = v;
  }
}

}  // namespace

extern "C" size_t cvl_image_augment_workspace_size(int B, int N) {
  (void)N;
  return B > 0 ? (size_t)B * AUG_PARTS * 3 * sizeof(double) : 0;
}

extern "C" int cvl_image_augment(const float* img_src, float* img_dst, const float* tgt_src, float* tgt_dst,
                                 const int32_t* ops, const float* params, int B, int N, int S, int T,
                                 void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(img_src && img_dst && ops && params && workspace && B > 0 && B < 65536 && N > 0 && N <= 16384);
  CVL_CHECK_ARG((tgt_src == nullptr) == (tgt_dst == nullptr));
  CVL_CHECK_ARG(!tgt_src || (S > 0 && T >= 4 && (long)S * S * 4 * T < (1L << 31)));
  CVL_CHECK_ARG(workspace_bytes >= cvl_image_augment_workspace_size(B, N));
  const hipStream_t s = (hipStream_t)stream;
  const int ntx = (N + AUG_T - 1) / AUG_T;
  const int img_tiles = ntx * ntx;
  const long tgt_per = tgt_src ? (long)S * S * 4 * T : 0;
  const int tgt_blocks = (int)((tgt_per + AUG_TGT - 1) / AUG_TGT);
  hipLaunchKernelGGL(augment_sums_kernel, dim3(AUG_PARTS, B), dim3(PT), 0, s, img_src, ops, N, (double*)workspace);
  hipLaunchKernelGGL(augment_apply_kernel, dim3(img_tiles + tgt_blocks, B), dim3(PT), 0, s, img_src, img_dst, tgt_src,
                     tgt_dst, ops, params, N, S, T, img_tiles, (const double*)workspace);
  return cvl_launch_status();
}

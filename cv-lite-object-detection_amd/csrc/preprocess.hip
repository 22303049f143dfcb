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

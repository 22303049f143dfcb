// ResNet stem convolution straight from the image (gfx950): Keras ResNet50 conv1 --
// ZeroPadding2D(3) + Conv2D(64, 7, strides=2) + bias -- the first layer of the backbones behind
// FCOS/fcos.py:30-46 and RetinaNet/retinanet_module.py:39-72.  Forward (with the conv1_bn
// statistics) and weight gradient; the input image has no gradient.
//
// The generic path materialised the im2col matrix of the 7x7x3 patches ([B*Ho*Wo][192] bf16, 403 MB
// at 512x512 bs 16), wrote it once and read it twice (forward GEMM and weight gradient).  Here each
// workgroup builds its patch tile in LDS from the fp32 image rows (which L1/L2 serve to the ~7
// workgroups that share them) and feeds the MFMAs from there: the HBM traffic is the image (50 MB)
// plus z / dz (134 MB), not the patch matrix.
//
// K order (both kernels, and the packed weights): k = ky * 24 + kx * 3 + c for kx < 7, c < 3 -- one
// image row's 21 consecutive floats per ky, padded to 24 -- then k in [168, 192) zero (the 32-deep
// MFMA step).  The packed forward weights are cvl_pack_conv_weights of the HWIO kernel viewed as
// KH = 7, KW = 1, Cin = 21, Cin_k = 24 (w_fwd [64][168]); the weight gradient is written in the same
// padded order, dw [192][64] fp32 (rows ky * 24 + kx * 3 + c; the pad rows come out 0).
//
// Numerics as the im2col path: the image rounded to bf16 (round to nearest even), bf16 MFMA with
// fp32 accumulation, bias added in fp32, the output rounded to bf16; BN statistics of the rounded
// output as exact accumulators (bn_acc.h).  Tile = 128 output pixels of one row.
#include "conv_common.h"

namespace {

constexpr int NT = 256;                  // 4 waves
constexpr int SP = 128;                  // output pixels per tile
constexpr int KR = 168, KP = 192;        // real (7 x 24) and MFMA-padded K
constexpr int KA = 200;                  // LDS pitch (elements) of the forward A / W rows
constexpr int PA = 136;                  // LDS pitch (elements) of the weight gradient's transposed rows
constexpr int CO = 64;

struct StemArgs {
  const float* img;       // [B][H][W][3] fp32
  const cvl_bf16* w;      // [64][168] bf16 (forward)
  const float* bias;      // [64] or null
  const cvl_bf16* dz;     // [B][Ho][Wo][64] bf16 (weight gradient)
  cvl_bf16* z;            // [B][Ho][Wo][64] bf16 (forward)
  acc_u64* stats;         // [B][64][2][8] or null
  float* out;             // weight gradient: slab [wgs][192][64] or dw
  int B, H, W, Ho, Wo, ntx, tiles, tiles_per_wg;
  float beta;
};

__device__ __forceinline__ s16x8 pack8f(const float* f) {
  s16x8 v;
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = (short)f32_to_bf16(f[u]);
  return v;
}

__device__ __forceinline__ void tile_coords(const StemArgs& g, int t, int* b, int* oy, int* x0) {
  const int xt = t % g.ntx, r = t / g.ntx;
  *oy = r % g.Ho;
  *b = r / g.Ho;
  *x0 = xt * SP;
}

// ---------------------------------------------------------------------------------------------
// forward: one workgroup per tile.  LDS: A [128 px][KA] (row = the pixel's 192 patch values) and
// W [64 co][KA]; 4 waves x (32 px x 64 co), 6 K-steps of v_mfma_f32_16x16x32_bf16.
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) stem_fwd_kernel(StemArgs g) {
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[SP * KA + CO * KA];
  cvl_bf16* A = lds;
  cvl_bf16* Wl = lds + SP * KA;
  const int tid = threadIdx.x;
  int b, oy, x0;
  tile_coords(g, blockIdx.x, &b, &oy, &x0);

  // weights: 64 rows x 24 chunks of 8 (chunks 21..23 = the zero K pad)
  for (int i = tid; i < CO * (KP / 8); i += NT) {
    const int co = i / (KP / 8), ch = i - (i / (KP / 8)) * (KP / 8);
    s16x8 v = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (ch < KR / 8) v = *reinterpret_cast<const s16x8*>(g.w + co * KR + ch * 8);
    *reinterpret_cast<s16x8*>(Wl + co * KA + ch * 8) = v;
  }
  // patches: item (ky, px) = 21 consecutive floats of image row 2*oy + ky - 3 from pixel 2*ox - 3
  const float* imgb = g.img + (long)b * g.H * g.W * 3;
  for (int it = tid; it < 7 * SP; it += NT) {
    const int ky = it / SP, px = it - (it / SP) * SP;
    const int iy = 2 * oy + ky - 3, ox = x0 + px;
    const int xs = 2 * ox - 3;
    const bool rok = (unsigned)iy < (unsigned)g.H && ox < g.Wo;
    const float* row = imgb + (long)iy * g.W * 3;
    float f[24];
#pragma unroll
    for (int j = 0; j < 21; ++j) {
      const int xx = xs + j / 3;
      f[j] = (rok && (unsigned)xx < (unsigned)g.W) ? row[xx * 3 + j % 3] : 0.f;
    }
    f[21] = f[22] = f[23] = 0.f;
    cvl_bf16* dst = A + px * KA + ky * 24;
#pragma unroll
    for (int q = 0; q < 3; ++q) *reinterpret_cast<s16x8*>(dst + q * 8) = pack8f(f + q * 8);
  }
  for (int i = tid; i < SP * 3; i += NT)           // K pad [168, 192)
    *reinterpret_cast<s16x8*>(A + (i / 3) * KA + KR + (i % 3) * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  __syncthreads();

  const int wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KP / 32; ++ks) {
    s16x8 fa[2], fb[4];
#pragma unroll
    for (int i = 0; i < 2; ++i) fa[i] = *reinterpret_cast<const s16x8*>(A + (wave * 32 + i * 16 + lr) * KA + ks * 32 + lg * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const s16x8*>(Wl + (j * 16 + lr) * KA + ks * 32 + lg * 8);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                             __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
  }
  // epilogue: C[px][co] (row px = wave*32 + i*16 + lg*4 + e, col co = j*16 + lr); + bias, bf16
  const int npx = g.Wo - x0 < SP ? g.Wo - x0 : SP;
  float s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float bj = g.bias ? g.bias[j * 16 + lr] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = bf16_to_f32(f32_to_bf16(acc[i][j][e] + bj));
        acc[i][j][e] = v;
        if (wave * 32 + i * 16 + lg * 4 + e < npx) { s1[j] += v; s2[j] += v * v; }
      }
  }
  __syncthreads();                                   // A / W no longer read: reuse the LDS
  float* red = reinterpret_cast<float*>(lds + SP * 72);    // [4 waves][64 co][2]
  if (g.stats) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a1 = s1[j], a2 = s2[j];
      a1 += __shfl_xor(a1, 16, 64); a1 += __shfl_xor(a1, 32, 64);
      a2 += __shfl_xor(a2, 16, 64); a2 += __shfl_xor(a2, 32, 64);
      if (lg == 0) {
        red[(wave * CO + j * 16 + lr) * 2] = a1;
        red[(wave * CO + j * 16 + lr) * 2 + 1] = a2;
      }
    }
  }
  cvl_bf16* Cs = lds;                                // [128 px][72] bf16
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        Cs[(wave * 32 + i * 16 + lg * 4 + e) * 72 + j * 16 + lr] = f32_to_bf16(acc[i][j][e]);   // exact
  __syncthreads();
  if (g.stats && tid < CO) {
    float a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { a1 += red[(w * CO + tid) * 2]; a2 += red[(w * CO + tid) * 2 + 1]; }
    acc_u64* st = g.stats + acc_idx((long)b * CO + tid, 0);
    acc_add(st, a1);
    acc_add(st + kAccSlots, a2);
  }
  cvl_bf16* zrow = g.z + ((long)(b * g.Ho + oy) * g.Wo + x0) * CO;
  for (int i = tid; i < npx * 8; i += NT) {
    const int px = i >> 3, c8 = (i & 7) * 8;
    *reinterpret_cast<s16x8*>(zrow + (long)px * CO + c8) = *reinterpret_cast<const s16x8*>(Cs + px * 72 + c8);
  }
}

// ---------------------------------------------------------------------------------------------
// weight gradient: dw[k][co] = sum over output pixels of A[px][k] * dz[px][co].  A workgroup loops
// over a contiguous range of tiles; per tile it builds A^T [192 k][128 px] and dz^T [64 co][128 px]
// in LDS (so both MFMA operands are plain 16-byte row reads), then 4 K-steps over the pixels.  4
// waves x (48 k x 64 co) accumulators; the partial [192][64] goes to the workgroup's fp32 slab,
// summed in a fixed order by the shared split reducer (deterministic).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) stem_wgrad_kernel(StemArgs g) {
  __shared__ __attribute__((aligned(16))) cvl_bf16 lds[KP * PA + CO * PA];
  cvl_bf16* At = lds;                      // [192][PA]
  cvl_bf16* Dt = lds + KP * PA;            // [64][PA]
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
  // zero K rows (the per-ky pad 21..23 and [168, 192)): never written by the builds below
  for (int i = tid; i < KP * (SP / 8); i += NT) {
    const int k = i / (SP / 8), pg = i - (i / (SP / 8)) * (SP / 8);
    if (k >= KR || k % 24 >= 21) *reinterpret_cast<s16x8*>(At + k * PA + pg * 8) = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  f32x4 acc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int t0 = blockIdx.x * g.tiles_per_wg;
  const int t1 = t0 + g.tiles_per_wg < g.tiles ? t0 + g.tiles_per_wg : g.tiles;
  for (int t = t0; t < t1; ++t) {
    int b, oy, x0;
    tile_coords(g, t, &b, &oy, &x0);
    const float* imgb = g.img + (long)b * g.H * g.W * 3;
    __syncthreads();                       // the previous tile's fragment reads are done
    // A^T: item (k < 168 with k % 24 < 21, px group of 8): 8 pixels 2 apart of one image row
    for (int it = tid; it < 7 * 21 * (SP / 8); it += NT) {
      const int kk = it / (SP / 8), pg = it - (it / (SP / 8)) * (SP / 8);
      const int ky = kk / 21, r = kk - (kk / 21) * 21;
      const int kx = r / 3, c = r - (r / 3) * 3;
      const int iy = 2 * oy + ky - 3;
      const bool rok = (unsigned)iy < (unsigned)g.H;
      const float* row = imgb + (long)iy * g.W * 3 + c;
      float f[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int ox = x0 + pg * 8 + q, xx = 2 * ox + kx - 3;
        f[q] = (rok && ox < g.Wo && (unsigned)xx < (unsigned)g.W) ? row[xx * 3] : 0.f;
      }
      *reinterpret_cast<s16x8*>(At + (ky * 24 + r) * PA + pg * 8) = pack8f(f);
    }
    // dz^T: lane = co, 8 pixel rows per 16-byte store (rows of 128 B read coalesced over the lanes)
    const cvl_bf16* dzr = g.dz + ((long)(b * g.Ho + oy) * g.Wo + x0) * CO;
    {
      const int co = tid & 63, pq = tid >> 6;
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int pg = pq * 4 + gg;
        s16x8 v;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int px = pg * 8 + q;
          v[q] = x0 + px < g.Wo ? (short)dzr[(long)px * CO + co] : (short)0;
        }
        *reinterpret_cast<s16x8*>(Dt + co * PA + pg * 8) = v;
      }
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < SP / 32; ++ks) {
      s16x8 fa[3], fb[4];
#pragma unroll
      for (int i = 0; i < 3; ++i)
        fa[i] = *reinterpret_cast<const s16x8*>(At + (wave * 48 + i * 16 + lr) * PA + ks * 32 + lg * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = *reinterpret_cast<const s16x8*>(Dt + (j * 16 + lr) * PA + ks * 32 + lg * 8);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                               __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
  }
  // C[k][co]: row k = wave*48 + i*16 + lg*4 + e, col co = j*16 + lr
  const bool direct = gridDim.x == 1;
  float* out = direct ? g.out : g.out + (size_t)blockIdx.x * KP * CO;
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float* po = out + (size_t)(wave * 48 + i * 16 + lg * 4 + e) * CO + j * 16 + lr;
        const float v = acc[i][j][e];
        *po = (direct && g.beta != 0.f) ? v + g.beta * *po : v;
      }
}

inline void stem_geometry(int H, int W, int* Ho, int* Wo) {
  *Ho = (H - 1) / 2 + 1;                  // (H + 6 - 7) / 2 + 1
  *Wo = (W - 1) / 2 + 1;
}

inline int stem_wgrad_wgs(int tiles) {
  static const int target = cvl_env_int("CVL_STEM_WGRAD_WGS", 512);
  int n = target < tiles ? target : tiles;
  return n < 1 ? 1 : n;
}

}  // namespace

extern "C" int cvl_stem_conv7x7s2(const float* img, int B, int H, int W, const void* w_packed, const float* bias,
                                  void* z, uint64_t* bn_stats, cvl_stream_t stream) {
  CVL_CHECK_ARG(img && w_packed && z && B > 0 && H > 0 && W > 0);
  CVL_CHECK_ARG((long)B * H * W * 3 < (1L << 31));
  StemArgs g{};
  g.img = img;
  g.w = reinterpret_cast<const cvl_bf16*>(w_packed);
  g.bias = bias;
  g.z = reinterpret_cast<cvl_bf16*>(z);
  g.stats = reinterpret_cast<acc_u64*>(bn_stats);
  g.B = B; g.H = H; g.W = W;
  stem_geometry(H, W, &g.Ho, &g.Wo);
  g.ntx = (g.Wo + SP - 1) / SP;
  g.tiles = B * g.Ho * g.ntx;
  hipLaunchKernelGGL(stem_fwd_kernel, dim3(g.tiles), dim3(NT), 0, (hipStream_t)stream, g);
  return cvl_launch_status();
}

extern "C" size_t cvl_stem_wgrad_workspace_size(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  int Ho, Wo;
  stem_geometry(H, W, &Ho, &Wo);
  const int tiles = B * Ho * ((Wo + SP - 1) / SP);
  const int tpw = (tiles + stem_wgrad_wgs(tiles) - 1) / stem_wgrad_wgs(tiles);
  const int wgs = (tiles + tpw - 1) / tpw;
  return wgs > 1 ? (size_t)wgs * KP * CO * sizeof(float) : 16;
}

extern "C" int cvl_stem_wgrad(const float* img, int B, int H, int W, const void* dz, float* dw, float beta,
                              void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(img && dz && dw && B > 0 && H > 0 && W > 0);
  CVL_CHECK_ARG((long)B * H * W * 3 < (1L << 31));
  CVL_CHECK_ARG(workspace && workspace_bytes >= cvl_stem_wgrad_workspace_size(B, H, W));
  hipStream_t s = (hipStream_t)stream;
  StemArgs g{};
  g.img = img;
  g.dz = reinterpret_cast<const cvl_bf16*>(dz);
  g.B = B; g.H = H; g.W = W;
  stem_geometry(H, W, &g.Ho, &g.Wo);
  g.ntx = (g.Wo + SP - 1) / SP;
  g.tiles = B * g.Ho * g.ntx;
  g.tiles_per_wg = (g.tiles + stem_wgrad_wgs(g.tiles) - 1) / stem_wgrad_wgs(g.tiles);
  const int wgs = (g.tiles + g.tiles_per_wg - 1) / g.tiles_per_wg;
  g.beta = beta;
  g.out = wgs > 1 ? reinterpret_cast<float*>(workspace) : dw;
  if (wgs == 1) {                                   // writes dW now: a queued reduction into it first
    const int gs = cvl_wgrad_defer_guard(dw, s);
    if (gs) return gs;
  }
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(wgs), dim3(NT), 0, s, g);
  const int st = cvl_launch_status();
  if (st || wgs == 1) return st;
  return cvl_wgrad_reduce(reinterpret_cast<const float*>(workspace), dw, dw, (long)KP * CO / 4, wgs, 1, beta, s);
}

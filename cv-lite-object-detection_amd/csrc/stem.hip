// ResNet stem convolution straight from the image (gfx950): Keras ResNet50 conv1 --
// ZeroPadding2D(3) + Conv2D(64, 7, strides=2) + bias -- the first layer of the backbones behind
// FCOS/fcos.py:30-46 and RetinaNet/retinanet_module.py:39-72.  Forward (with the conv1_bn
// statistics) and weight gradient; the input image has no gradient.
//
// The im2col form these kernels replaced materialised the 7x7x3 patch matrix ([B*Ho*Wo][192] bf16,
// 403 MB at 512x512 bs 16), wrote it once and read it twice (forward GEMM and weight gradient).  Here a
// workgroup walks a band of output rows of one image (and one 256-pixel column range) and keeps a
// ring of the image rows they need in LDS as bf16 -- each output row needs 7 image rows, the next
// one 2 more -- and the MFMA operands are read straight out of that ring: the patch of output pixel
// p, kernel row ky, is the 21 consecutive values of image row 2*oy + ky - 3 starting at element
// 6*p (pixel 2*p - 3 + 3 of the ring's row, 3 channels).  HBM traffic: the image (~1.4x, the bands'
// overlapping first rows) plus z / dz, no patch matrix.
//
// K order (both kernels, and the packed weights): k = ky * 24 + kx * 3 + c for kx < 7, c < 3 -- one
// image row's 21 consecutive values per ky, padded to 24 -- and k in [168, 192) for the last
// 32-deep MFMA step.  The packed forward weights are cvl_pack_conv_weights of the HWIO kernel viewed
// as KH = 7, KW = 1, Cin = 21, Cin_k = 24 (w_fwd [64][168]): their pad columns are zero, so the
// ring values a pad k reads (the next pixel's, or a ring row not yet loaded: finite, the ring is
// zeroed first) add nothing.  The weight gradient is written in the same padded order, dw [192][64]
// fp32 (rows ky * 24 + kx * 3 + c; the pad rows come out 0).
//
// Numerics as that im2col form: the image rounded to bf16 (round to nearest even), bf16 MFMA with
// fp32 accumulation, bias added in fp32, the output rounded to bf16; BN statistics of the rounded
// output as BN accumulators (bn_acc.h: float64 or the exact mode's bins), one add per (workgroup, channel).
#include "conv_common.h"

namespace {
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
constexpr int NT = 256;                  // 4 waves
constexpr int SPX = 256;                 // output pixels per column range
constexpr int RL = 1560;                 // ring row (bf16): (2 * SPX + 6) * 3 = 1554 values, padded
constexpr int NRING = 12;                // ring rows (7 in use + 2 prefetched + slack)
constexpr int KR = 168, KP = 192;        // real (7 x 24) and MFMA-padded K
constexpr int WA = 200;                  // LDS pitch (elements) of the weight rows (forward)
constexpr int CO = 64;
constexpr int DZP = CO + 8;              // LDS pitch (elements) of the dz row image [px][co] (weight gradient)
// output rows per workgroup (forward / weight gradient): 8 gives 512 units at 512x512 bs 16, exactly
// two resident per CU in one round (tools/stem_probe.py sweep, round 4: forward 82 us at 8 vs 101 /
// 109 at 4 / 16; weight gradient 74 us at 8 vs 102 at 16, 95 at 4 and 12, 170 at 32)
constexpr int RPW_F = 8, RPW_W = 8;
constexpr int RPT = (RL + NT - 1) / NT;  // ring values per thread per image row

struct StemArgs {
  const float* img;       // [B][H][W][3] fp32
  const cvl_bf16* w;      // [64][168] bf16 (forward)
  const float* bias;      // [64] or null
  const cvl_bf16* dz;     // [B][Ho][Wo][64] bf16 (weight gradient)
  cvl_bf16* z;            // [B][Ho][Wo][64] bf16 (forward)
  acc_u64* stats;         // [B][64][2][slots] or null
  int acc_slots;
  float* out;             // weight gradient: slab [units][192][64] or dw
  int B, H, W, Ho, Wo, ntx, nbands, rpw;
  float beta;
  unsigned long long* stamps;   // measurement builds (CVL_STEM_STAMPS=1): u64 [grid][8], else null
};

struct Unit {
  int b, x0, npx, oy0, oy1;
};

__device__ __forceinline__ Unit unit_of(const StemArgs& g, int u) {
  Unit t;
  const int band = u % g.nbands, r = u / g.nbands;
  const int xt = r % g.ntx;
  t.b = r / g.ntx;
  t.x0 = xt * SPX;
  t.npx = g.Wo - t.x0 < SPX ? g.Wo - t.x0 : SPX;
  t.oy0 = band * g.rpw;
  t.oy1 = t.oy0 + g.rpw < g.Ho ? t.oy0 + g.rpw : g.Ho;
  return t;
}

// image row iy of the unit as ring values (bf16; zero outside the image): thread part only
__device__ __forceinline__ void row_load(const StemArgs& g, const Unit& t, int iy, float (&v)[RPT]) {
  const int tid = threadIdx.x;
  const bool rok = (unsigned)iy < (unsigned)g.H;
  const long rowbase = ((long)t.b * g.H + iy) * g.W * 3;
  const int xs0 = 2 * t.x0 - 3;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int e = tid + q * NT;
    const int p = xs0 + e / 3;
    v[q] = (rok && e < (2 * SPX + 6) * 3 && (unsigned)p < (unsigned)g.W) ? g.img[rowbase + (long)p * 3 + e % 3] : 0.f;
  }
}
__device__ __forceinline__ void row_store(cvl_bf16* ring, int iy, const float (&v)[RPT]) {
  cvl_bf16* r = ring + ((iy + 3) % NRING) * RL;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int e = threadIdx.x + q * NT;
    if (e < RL) r[e] = f32_to_bf16(v[q]);
  }
}

// the unit's first 7 image rows into the ring, all loads in flight at once (one latency, not 7)
__device__ __forceinline__ void ring_prologue(const StemArgs& g, const Unit& t, cvl_bf16* ring) {
  float v[7][RPT];
#pragma unroll
  for (int r = 0; r < 7; ++r) row_load(g, t, 2 * t.oy0 - 3 + r, v[r]);
#pragma unroll
  for (int r = 0; r < 7; ++r) row_store(ring, 2 * t.oy0 - 3 + r, v[r]);
}

// 8 consecutive ring values (16 B at a 4-B aligned address) as an MFMA fragment
__device__ __forceinline__ s16x8 ring8(const cvl_bf16* p) {
  const unsigned* u = reinterpret_cast<const unsigned*>(p);
  const unsigned a = u[0], b = u[1], c = u[2], d = u[3];
  s16x8 v;
  v[0] = (short)(a & 0xffff); v[1] = (short)(a >> 16);
  v[2] = (short)(b & 0xffff); v[3] = (short)(b >> 16);
  v[4] = (short)(c & 0xffff); v[5] = (short)(c >> 16);
  v[6] = (short)(d & 0xffff); v[7] = (short)(d >> 16);
  return v;
}

// ---------------------------------------------------------------------------------------------
// forward: swapped operands D[co][px] = W[co][k] . patch[k][px], so a lane's accumulator quad is
// 4 consecutive channels of one pixel (8-byte stores straight from the registers).  4 waves x 64
// pixels x 64 channels, 6 K-steps per output row.  The next row's two image rows are loaded into
// registers before the row's MFMAs and stored to the ring after them.
// ---------------------------------------------------------------------------------------------
template <bool ST = false>
__global__ void __launch_bounds__(NT, 2) stem_fwd_kernel(StemArgs g) {
  __shared__ __attribute__((aligned(16))) cvl_bf16 Wl[CO * WA];
  __shared__ __attribute__((aligned(16))) cvl_bf16 ring[NRING * RL];
  __shared__ float red[4][CO][2];
  const int tid = threadIdx.x;
  // stamps (thread 0): wall clock at entry / prologue landed / rows done / exit, then shader-clock
  // ticks spent in the rows' MFMA phase, epilogue (stores + statistics) and ring refill
  unsigned long long* stamp = (ST && tid == 0) ? g.stamps + blockIdx.x * 8 : nullptr;
  unsigned long long t_mma = 0, t_epi = 0, t_ref = 0, c0 = 0;
  if (stamp) stamp[0] = wall_clock64();
  const Unit t = unit_of(g, blockIdx.x);
  if (t.oy0 >= g.Ho) return;
  // prologue, every load in flight at once: the weights, then the first 7 image rows; the weights
  // land in LDS and the ring is zeroed while the image rows are still in flight
  constexpr int WQ = CO * (KP / 8) / NT;
  s16x8 wv[WQ];
#pragma unroll
  for (int q = 0; q < WQ; ++q) {
    const int i = tid + q * NT, co = i / (KP / 8), ch = i - (i / (KP / 8)) * (KP / 8);
    wv[q] = ch < KR / 8 ? *reinterpret_cast<const s16x8*>(g.w + co * KR + ch * 8) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
  {
    float v[7][RPT];
#pragma unroll
    for (int r = 0; r < 7; ++r) row_load(g, t, 2 * t.oy0 - 3 + r, v[r]);
#pragma unroll
    for (int q = 0; q < WQ; ++q) {
      const int i = tid + q * NT, co = i / (KP / 8), ch = i - (i / (KP / 8)) * (KP / 8);
      *reinterpret_cast<s16x8*>(Wl + co * WA + ch * 8) = wv[q];
    }
    for (int i = tid; i < NRING * RL / 8; i += NT) reinterpret_cast<s16x8*>(ring)[i] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 7; ++r) row_store(ring, 2 * t.oy0 - 3 + r, v[r]);
  }
  __syncthreads();
  if (stamp) stamp[1] = wall_clock64();

  const int wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
  float bias[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[i][e] = g.bias ? g.bias[i * 16 + lg * 4 + e] : 0.f;
  f32x2 s1[4][2], s2[4][2];        // (channel i*16 + lg*4 + e) statistics, channel pairs packed
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 2; ++e) { s1[i][e] = f32x2{0.f, 0.f}; s2[i][e] = f32x2{0.f, 0.f}; }

  // per row: the next row's two image rows are loaded, the MFMAs issue, the two rows go into the
  // ring slots this row does not read ((2*oy + 7) % NRING is only its pad K, which the fragments
  // replace by zeros) while the MFMAs run, then the epilogue; ONE barrier per row, at its top
  for (int oy = t.oy0; oy < t.oy1; ++oy) {
    if (oy > t.oy0) __syncthreads();                // the previous row's ring stores are visible
    const bool more = oy + 1 < t.oy1;
    float n0[RPT], n1[RPT];
    if (more) {                                     // image rows 2*oy + 4, 2*oy + 5 for row oy + 1
      row_load(g, t, 2 * oy + 4, n0);
      row_load(g, t, 2 * oy + 5, n1);
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (stamp) c0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int s = 0; s < KP / 32; ++s) {
      const int k0 = s * 32 + lg * 8, ky = k0 / 24, off = k0 - ky * 24;
      const cvl_bf16* rr = ring + ((2 * oy + ky) % NRING) * RL + off;
      // pad K (kx*3 + c in 21..23 = the next pixel's values, or ky == 7 = the ring row being
      // rewritten) enters the MFMAs as exact zeros, not as data under zero weights: a non-finite pixel
      // then reaches only its own outputs, and the ky == 7 read's race with row_store is harmless
      const unsigned keep_hi = off == 16 ? 0x0000ffffu : 0xffffffffu;     // elements 5..7 of the chunk
      const bool padrow = ky >= 7;
      s16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const s16x8*>(Wl + (i * 16 + lr) * WA + k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        u32x4 v = __builtin_bit_cast(u32x4, ring8(rr + 6 * (wave * 64 + j * 16 + lr)));
        v[2] &= keep_hi;
        v[3] = off == 16 ? 0u : v[3];
        v = padrow ? u32x4{0u, 0u, 0u, 0u} : v;
        fb[j] = __builtin_bit_cast(s16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                               __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
    }
    if (stamp) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      t_mma += c1 - c0;
      c0 = c1;
    }
    if (more) {
      row_store(ring, 2 * oy + 4, n0);
      row_store(ring, 2 * oy + 5, n1);
    }
    if (stamp) {
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      t_ref += c1 - c0;
      c0 = c1;
    }
    // epilogue: D[co = i*16 + lg*4 + e][px = wave*64 + j*16 + lr]; one v_permlane16_swap per packed
    // register regroups channel blocks (2m, 2m+1) so a lane holds 8 consecutive channels of its pixel
    // (32 m + lgo ..): two 16-B stores per pixel instead of four 8-B ones
    cvl_bf16* zrow = g.z + ((long)(t.b * g.Ho + oy) * g.Wo + t.x0) * CO;
    const int lgo = ((lg & 1) ? 16 : 0) + ((lg & 2) ? 8 : 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int px = wave * 64 + j * 16 + lr;
      const bool ok = px < t.npx;
      unsigned pk[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float r[4];
#pragma unroll
        for (int e = 0; e < 4; e += 2) {            // one v_cvt_pk_bf16_f32 per channel pair (RNE)
          const bf16x2 h = __builtin_convertvector(
              (f32x2{acc[i][j][e] + bias[i][e], acc[i][j][e + 1] + bias[i][e + 1]}), bf16x2);
          const unsigned u = __builtin_bit_cast(unsigned, h);
          r[e] = __uint_as_float(u << 16);
          r[e + 1] = __uint_as_float(u & 0xffff0000u);
          pk[i][e >> 1] = u;
        }
        if (ok) {                                   // packed fp32 adds / fmas on channel pairs
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const f32x2 v = f32x2{r[2 * e], r[2 * e + 1]};
            s1[i][e] += v;
            s2[i][e] = __builtin_elementwise_fma(v, v, s2[i][e]);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[2 * m][h], pk[2 * m + 1][h], false, false);
          pk[2 * m][h] = sw[0];
          pk[2 * m + 1][h] = sw[1];
        }
        if (ok)
          *reinterpret_cast<u32x4*>(zrow + (long)px * CO + 32 * m + lgo) =
              u32x4{pk[2 * m][0], pk[2 * m][1], pk[2 * m + 1][0], pk[2 * m + 1][1]};
      }
    }
    if (stamp) t_epi += __builtin_amdgcn_s_memtime() - c0;
  }
  if (stamp) { stamp[2] = wall_clock64(); stamp[4] = t_mma; stamp[5] = t_epi; stamp[6] = t_ref; }
  if (g.stats) {              // the 16 pixel lanes, then the 4 waves, in a fixed order
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float a1 = s1[i][e >> 1][e & 1], a2 = s2[i][e >> 1][e & 1];
#pragma unroll
        for (int m = 1; m < 16; m <<= 1) { a1 += __shfl_xor(a1, m, 64); a2 += __shfl_xor(a2, m, 64); }
        if (lr == 0) { red[wave][i * 16 + lg * 4 + e][0] = a1; red[wave][i * 16 + lg * 4 + e][1] = a2; }
      }
    __syncthreads();
    if (tid < CO) {
      const float a1 = (red[0][tid][0] + red[1][tid][0]) + (red[2][tid][0] + red[3][tid][0]);
      const float a2 = (red[0][tid][1] + red[1][tid][1]) + (red[2][tid][1] + red[3][tid][1]);
      acc_u64* st = g.stats + acc_idx((long)t.b * CO + tid, 0, g.acc_slots);
      acc_add(st, a1, g.acc_slots);
      acc_add(st + g.acc_slots, a2, g.acc_slots);
    }
  }
  if (stamp) stamp[3] = wall_clock64();
}

// ---------------------------------------------------------------------------------------------
// weight gradient: D[co][k] = sum over the band's pixels of dz^T[co][px] . patch[px][k].  Per output
// row the dz row is transposed into LDS (dz^T[co][px]: plain 16-byte fragment reads) and the patch
// fragments are gathered from the ring (8 pixels 2 apart = stride 6 values).  4 waves x 48 k x 64
// co accumulators over the band, then the [192][64] partial goes to the unit's fp32 slab (summed in
// a fixed order by the shared split reducer: deterministic).
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(NT) stem_wgrad_kernel(StemArgs g) {
  __shared__ __attribute__((aligned(16))) cvl_bf16 ring[NRING * RL];
  __shared__ __attribute__((aligned(16))) cvl_bf16 dzl[SPX * DZP];
  const int tid = threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63, lr = lane & 15, lg = lane >> 4;
  const Unit t = unit_of(g, blockIdx.x);
  f32x4 acc[4][3];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's patch columns k = wave*48 + j*16 + lr: kernel row, offset in the ring row, valid
  int kyj[3], offj[3];
  bool kv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int k = wave * 48 + j * 16 + lr, r = k % 24;
    kv[j] = k < KR && r < 21;
    kyj[j] = k / 24;
    offj[j] = r;                                    // kx * 3 + c
  }
  if (t.oy0 < g.Ho) {
    for (int i = tid; i < NRING * RL / 8; i += NT) reinterpret_cast<s16x8*>(ring)[i] = s16x8{0, 0, 0, 0, 0, 0, 0, 0};
    __syncthreads();
    ring_prologue(g, t, ring);
    // dz row -> registers: thread owns 8 chunks (pixel, 8 channels) of the 256 x 64 row
    auto dz_load = [&](int oy, s16x8 (&d)[8]) {
      const cvl_bf16* zr = g.dz + ((long)(t.b * g.Ho + oy) * g.Wo + t.x0) * CO;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int idx = tid + q * NT, px = idx >> 3, c8 = (idx & 7) * 8;
        d[q] = px < t.npx ? *reinterpret_cast<const s16x8*>(zr + (long)px * CO + c8) : s16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    };
    s16x8 dcur[8];
    dz_load(t.oy0, dcur);
    // A fragments dz^T[co][px] by transposed reads of the row image [px][co]: rows p0 + 8*lg + q4
    // (+ 4), column chunk i*16 + 4*pp (the conv_wgrad_x dY pattern; padded pitch, no swizzle)
    const int q4 = lr >> 2, pp = lr & 3;
    const unsigned dz0 = lds_addr(dzl);
    for (int oy = t.oy0; oy < t.oy1; ++oy) {
      __syncthreads();                              // the previous row's fragment reads are done
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int idx = tid + q * NT, px = idx >> 3, c8 = (idx & 7) * 8;
        *reinterpret_cast<s16x8*>(dzl + px * DZP + c8) = dcur[q];
      }
      const bool more = oy + 1 < t.oy1;
      float n0[RPT], n1[RPT];
      s16x8 dnext[8];
      if (more) {
        row_load(g, t, 2 * oy + 4, n0);
        row_load(g, t, 2 * oy + 5, n1);
        dz_load(oy + 1, dnext);
      }
      __syncthreads();
#pragma unroll 2
      for (int s = 0; s < SPX / 32; ++s) {
        const int p0 = s * 32 + lg * 8;
        s16x4 al[4], ah[4];
        s16x8 fb[3];
        const unsigned rlo = dz0 + 2 * ((s * 32 + 8 * lg + q4) * DZP + 4 * pp);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          al[i] = ds_tr16(rlo + 2 * (i * 16));
          ah[i] = ds_tr16(rlo + 2 * (4 * DZP + i * 16));
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const cvl_bf16* rr = ring + ((2 * oy + kyj[j]) % NRING) * RL + offj[j] + 6 * p0;
          s16x8 v;
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = kv[j] ? (short)rr[6 * q] : (short)0;
          fb[j] = v;
        }
        lgkm_wait();
        s16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          tr_pin(al[i]);
          tr_pin(ah[i]);
          fa[i] = tr_join(al[i], ah[i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 3; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, fa[i]),
                                                                 __builtin_bit_cast(bf16x8, fb[j]), acc[i][j], 0, 0, 0);
      }
      if (more) {
        __syncthreads();
        row_store(ring, 2 * oy + 4, n0);
        row_store(ring, 2 * oy + 5, n1);
#pragma unroll
        for (int q = 0; q < 8; ++q) dcur[q] = dnext[q];
      }
    }
  }
  // D[co = i*16 + lg*4 + e][k = wave*48 + j*16 + lr] -> out[k][co], 16 bytes per accumulator
  const bool direct = gridDim.x == 1;
  float* out = direct ? g.out : g.out + (size_t)blockIdx.x * KP * CO;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f32x4 v = acc[i][j];
      f32x4* po = reinterpret_cast<f32x4*>(out + (size_t)(wave * 48 + j * 16 + lr) * CO + i * 16 + lg * 4);
      if (direct && g.beta != 0.f) v += g.beta * *po;
      *po = v;
    }
}

inline void stem_geometry(int H, int W, int* Ho, int* Wo) {
  *Ho = (H - 1) / 2 + 1;                  // (H + 6 - 7) / 2 + 1
  *Wo = (W - 1) / 2 + 1;
}

inline void stem_plan(StemArgs* g, int B, int H, int W, int rpw) {
  g->B = B; g->H = H; g->W = W;
  stem_geometry(H, W, &g->Ho, &g->Wo);
  g->ntx = (g->Wo + SPX - 1) / SPX;
  g->rpw = rpw;
  g->nbands = (g->Ho + rpw - 1) / rpw;
}

#ifdef CVL_MEASURE
// measurement builds: CVL_STEM_STAMPS=1 stamps every forward launch into this buffer
constexpr int kStemStampWgs = 4096;
__device__ unsigned long long g_stem_stamps[kStemStampWgs * 8];
int g_stem_stamp_grid = 0;
#endif

}  // namespace

#ifdef CVL_MEASURE
// Measurement hook: the stamps of the last stamped stem forward (CVL_STEM_STAMPS=1): u64 [grid][8] =
// wall clock at entry / prologue landed / rows done / exit, then shader-clock ticks in the rows' MFMA
// phase, epilogue and ring refill (thread 0 of each workgroup); returns the grid size (0: none).
extern "C" int cvl_debug_stem_stamps(uint64_t* host, int max_wgs) {
  const int n = g_stem_stamp_grid < max_wgs ? g_stem_stamp_grid : max_wgs;
  if (n <= 0 || !host) return g_stem_stamp_grid;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stem_stamps), (size_t)n * 64, 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return g_stem_stamp_grid;
}
#endif  // CVL_MEASURE

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
  g.acc_slots = cvl_bn_acc_slots();
  stem_plan(&g, B, H, W, RPW_F);
  const int grid = B * g.ntx * g.nbands;
#ifdef CVL_MEASURE
  static const bool stamps = cvl_tune_flag("CVL_STEM_STAMPS");
  if (stamps && grid <= kStemStampWgs) {
    void* sym = nullptr;
    if (hipGetSymbolAddress(&sym, HIP_SYMBOL(g_stem_stamps)) == hipSuccess) g.stamps = (unsigned long long*)sym;
    g_stem_stamp_grid = grid;
  }
  if (g.stamps) hipLaunchKernelGGL(stem_fwd_kernel<true>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, g);
  else
#endif
  hipLaunchKernelGGL(stem_fwd_kernel<false>, dim3(grid), dim3(NT), 0, (hipStream_t)stream, g);
  return cvl_launch_status();
}

extern "C" size_t cvl_stem_wgrad_workspace_size(int B, int H, int W) {
  if (B <= 0 || H <= 0 || W <= 0) return 0;
  StemArgs g{};
  stem_plan(&g, B, H, W, RPW_W);
  const long units = (long)B * g.ntx * g.nbands;
  return units > 1 ? (size_t)units * KP * CO * sizeof(float) : 16;
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
  g.beta = beta;
  stem_plan(&g, B, H, W, RPW_W);
  const int units = B * g.ntx * g.nbands;
  g.out = units > 1 ? reinterpret_cast<float*>(workspace) : dw;
  if (units == 1) {                                 // writes dW now: a queued reduction into it first
    const int gs = cvl_wgrad_defer_guard(dw, s);
    if (gs) return gs;
  }
  hipLaunchKernelGGL(stem_wgrad_kernel, dim3(units), dim3(NT), 0, s, g);
  const int st = cvl_launch_status();
  if (st || units == 1) return st;
  return cvl_wgrad_reduce(reinterpret_cast<const float*>(workspace), dw, dw, (long)KP * CO / 4, units, 1, beta, s);
}

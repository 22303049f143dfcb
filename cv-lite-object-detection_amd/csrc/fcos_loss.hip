// Fused FCOS loss forward + backward on gfx950 — restates FCOS/fcos.py:380-496.
//
//   cls = sum focal(targets[5:], cls_logits)            (fcos.py:443-462, alpha .25, gamma 2)
//   cen = sum smoothL1(targets[4], sigmoid(reg[4]))     over ALL cells (fcos.py:483-486, Q10)
//   reg = sum mask * smoothL1(targets[:4], reg[:4])     (l1)  or  -log IoU (iou, fcos.py:393-441)
//   mask = max(targets[5:]) >= 1                        (fcos.py:475-477)
// Variant flags (bits of reg_type above the reg kind in bits 0-1):
//   4  FOCAL_CEN  centerness as focal(targets[4], logit) (fcos_center.py:386-389, cen_type="focal";
//                 fcos_center_v1.py:305-307)
//   8  SIG_REG    smooth-L1 on sigmoid(reg[:4]) (fcos_center_v1.py:115 applies the sigmoid in the model)
//   16 CEN_IN_CLS the centerness logit (and its gradient) is column cc = round_up(C, 8) of the class
//                 rows (the centre variants' cen_output_l head sits on the cls tower,
//                 fcos_center.py:85-101; the 8-aligned column lets its weight gradient read it)
//   32 MASK_T5    the regression mask is the float value targets[5] itself (the drop-in
//                 smooth_l1_loss / iou_loss(mask=<float map>) of fcos.py:380-441; C = 1)
// cvl_fcos_loss_ex takes the focal alpha / gamma and the smooth-L1 delta (fcos.py:380, 443-444
// keywords); cvl_fcos_loss is it with the reference defaults 0.25 / 2 / 1.
// "smooth L1" is the reference's discontinuous 0.5 d^2 (|d|<1) / |d| (Q8).  One pass reads the
// predictions and targets once and writes the gradients once (HBM-bound); per-image sums are
// reduced deterministically (per-tile partials in float64, then a fixed-order second pass).
#include "cvl_common.h"

namespace {

constexpr int kThreads = 256;
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct LossArgs {
  const float* reg;
  const float* cls;
  const float* tgt;
  float* losses;
  void* dreg;
  void* dcls;
  double* partial;   // [B, tiles, 3]
  int ld_reg, ld_cls, ld_dreg, ld_dcls, dreg_bf16, dcls_bf16;
  int P, C, reg_type, tiles;
  float grad_scale;
  float alpha, gamma, delta;
};

__device__ __forceinline__ void store_g(void* base, size_t idx, float v, int is_bf16) {
  if (is_bf16) reinterpret_cast<cvl_bf16*>(base)[idx] = f32_to_bf16(v);
  else reinterpret_cast<float*>(base)[idx] = v;
}

__device__ __forceinline__ float sl1(float d, float delta, float* g) {
  // loss of d = t - x and its derivative w.r.t. x (TF gradient of the tf.where form)
  const float ad = fabsf(d);
  if (ad < delta) { *g = -d; return 0.5f * d * d; }
  *g = d > 0.f ? -1.0f : (d < 0.f ? 1.0f : 0.0f);
  return ad;
}

// q^gamma: the reference default gamma = 2 as a product (the values every training path uses)
__device__ __forceinline__ float powg(float q, float gamma) { return gamma == 2.0f ? q * q : powf(q, gamma); }

// focal loss term (the reference's stable form, fcos.py:443-462) and d/dx:
//   y a q^g (L - min(x,0)) + (1-y)(1-a) p^g (L + max(x,0)),  p = sigmoid(x), q = 1 - p, L = log(1+e^-|x|)
//   d/dx = -y a q^g (g p nlp + q) + (1-y)(1-a) p^g (g q nlq + p)
__device__ __forceinline__ float focal_term(float y, float x, float alpha, float gamma, float* g) {
  const float e = expf(-fabsf(x));
  const float L = log1pf(e);                       // log(1 + exp(-|x|))
  const float p1 = x >= 0.f ? 1.0f / (1.0f + e) : e / (1.0f + e);   // sigmoid(x)
  const float q1 = x >= 0.f ? e / (1.0f + e) : 1.0f / (1.0f + e);   // 1 - sigmoid(x)
  const float nlp = L - fminf(x, 0.f);             // -log p
  const float nlq = L + fmaxf(x, 0.f);             // -log(1-p)
  const float qg = powg(q1, gamma), pg = powg(p1, gamma);
  const float wpos = y * alpha * qg;
  const float wneg = (1.0f - y) * (1.0f - alpha) * pg;
  *g = -wpos * (gamma * p1 * nlp + q1) + wneg * (gamma * q1 * nlq + p1);
  return wpos * nlp + wneg * nlq;
}

// One cell's loss terms and gradients: t(i) targets[i], xc(c) class logit c, xr(j) box / centerness
// prediction j; putc(c, g) / putcen(g) / putr(j, g) receive the SCALED gradients (class c, the
// centerness column of the class rows, box j < 5).  Both kernels below run exactly this code.
// everything after the class loop: centerness and box terms of one cell, given its positive mask
template <class TF, class XCF, class XRF, class PCEN, class PR>
__device__ __forceinline__ void cell_rest(const LossArgs& a, TF t, XCF xc, XRF xr, PCEN putcen, PR putr, float mask,
                                          float& s_reg, float& s_cen) {
  const int kind = a.reg_type & 3;
  const bool focal_cen = a.reg_type & 4, sig_reg = a.reg_type & 8, cen_in_cls = a.reg_type & 16;
  const int cc = (a.C + 7) / 8 * 8;                // centerness column of the class rows (CEN_IN_CLS)
  float g[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  // centerness: smooth-L1 on sigmoid(logit) (fcos.py:483-486) or focal (centre variants), all cells
  {
    const float x = cen_in_cls ? xc(cc) : xr(4);
    float gc;
    if (focal_cen) {
      s_cen += focal_term(t(4), x, a.alpha, a.gamma, &gc);
    } else {
      const float sg = 1.0f / (1.0f + expf(-x));
      float gd;
      s_cen += sl1(t(4) - sg, a.delta, &gd);
      gc = gd * sg * (1.0f - sg);
    }
    if (cen_in_cls) {
      putcen(gc * a.grad_scale);
    } else {
      g[4] = gc;
    }
  }
  if (kind == 0) {
    for (int j = 0; j < 4; ++j) {
      float gd;
      if (sig_reg) {                             // fcos_center_v1.py:115: reg = sigmoid(conv)
        const float sg = 1.0f / (1.0f + expf(-xr(j)));
        const float l = sl1(t(j) - sg, a.delta, &gd);
        s_reg += mask * l;
        g[j] = mask * gd * sg * (1.0f - sg);
      } else {
        const float l = sl1(t(j) - xr(j), a.delta, &gd);
        s_reg += mask * l;
        g[j] = mask * gd;
      }
    }
  } else if (mask != 0.f) {
    // IoU of ltrb boxes about the same grid point (grid offsets cancel)
    const float t0 = t(0), t1 = t(1), t2 = t(2), t3 = t(3);
    const float p0 = xr(0), p1 = xr(1), p2 = xr(2), p3 = xr(3);
    const float th = t0 + t1, tw = t2 + t3, ph = p0 + p1, pw = p2 + p3;
    const float ihr = fminf(t1, p1) + fminf(t0, p0);
    const float iwr = fminf(t3, p3) + fminf(t2, p2);
    const float ih = fmaxf(ihr, 0.f), iw = fmaxf(iwr, 0.f);
    const float I = ih * iw;
    const float Ue = th * tw + ph * pw - I + 1.0e-12f;
    const float iou = I / Ue;
    s_reg += -logf(iou + 1.0e-12f) * mask;
    const float dL = -mask / (iou + 1.0e-12f);
    const float dI = (Ue + I) / (Ue * Ue);            // d iou / d I (U depends on -I)
    const float dph = -I * pw / (Ue * Ue), dpw = -I * ph / (Ue * Ue);
    const float gih = ihr > 0.f ? dI * iw : 0.f;
    const float giw = iwr > 0.f ? dI * ih : 0.f;
    g[0] = dL * ((p0 < t0 ? gih : 0.f) + dph);
    g[1] = dL * ((p1 < t1 ? gih : 0.f) + dph);
    g[2] = dL * ((p2 < t2 ? giw : 0.f) + dpw);
    g[3] = dL * ((p3 < t3 ? giw : 0.f) + dpw);
  }
  for (int j = 0; j < 5; ++j) putr(j, g[j] * a.grad_scale);
}

template <class TF, class XCF, class XRF, class PC, class PCEN, class PR>
__device__ __forceinline__ void cell_loss(const LossArgs& a, TF t, XCF xc, XRF xr, PC putc, PCEN putcen, PR putr,
                                          float& s_cls, float& s_reg, float& s_cen) {
  float tmax = 0.f;
  for (int c = 0; c < a.C; ++c) {
    const float y = t(5 + c);
    tmax = fmaxf(tmax, y);
    float g;
    s_cls += focal_term(y, xc(c), a.alpha, a.gamma, &g);
    putc(c, g * a.grad_scale);
  }
  const float mask = (a.reg_type & 32) ? t(5) : (tmax >= 1.0f ? 1.0f : 0.0f);
  cell_rest(a, t, xc, xr, putcen, putr, mask, s_reg, s_cen);
}

// deterministic block reduction of the three sums in float64 -> partial[b][tile][3]
template <int NTH>
__device__ __forceinline__ void block_partials(const LossArgs& a, float s_cls, float s_reg, float s_cen) {
  __shared__ double red[3][NTH / 64];
  double v0 = warp_sum_d((double)s_cls), v1 = warp_sum_d((double)s_reg), v2 = warp_sum_d((double)s_cen);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) { red[0][w] = v0; red[1][w] = v1; red[2][w] = v2; }
  __syncthreads();
  if (threadIdx.x < 3) {
    double s = 0.0;
    for (int k = 0; k < NTH / 64; ++k) s += red[threadIdx.x][k];
    a.partial[((size_t)blockIdx.y * a.tiles + blockIdx.x) * 3 + threadIdx.x] = s;
  }
}

// Row-pointer form (any layout): a thread walks its cell's rows in global memory.
__global__ void __launch_bounds__(kThreads) fcos_loss_kernel(LossArgs a) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * kThreads + threadIdx.x;
  float s_cls = 0.f, s_reg = 0.f, s_cen = 0.f;
  const int cc = (a.C + 7) / 8 * 8;
  if (p < a.P) {
    const size_t cell = (size_t)b * a.P + p;
    const float* t = a.tgt + cell * (5 + a.C);
    const float* xr = a.reg + cell * a.ld_reg;
    const float* xc = a.cls + cell * a.ld_cls;
    cell_loss(
        a, [&](int i) { return t[i]; }, [&](int c) { return xc[c]; }, [&](int j) { return xr[j]; },
        [&](int c, float v) {
          if (a.dcls) store_g(a.dcls, cell * a.ld_dcls + c, v, a.dcls_bf16);
        },
        [&](float v) {
          if (a.dcls) {
            for (int c = a.C; c < a.ld_dcls; ++c) store_g(a.dcls, cell * a.ld_dcls + c, 0.f, a.dcls_bf16);
            store_g(a.dcls, cell * a.ld_dcls + cc, v, a.dcls_bf16);
          }
        },
        [&](int j, float v) {
          if (a.dreg) store_g(a.dreg, cell * a.ld_dreg + j, v, a.dreg_bf16);
        },
        s_cls, s_reg, s_cen);
    if (a.dcls && !(a.reg_type & 16))
      for (int c = a.C; c < a.ld_dcls; ++c) store_g(a.dcls, cell * a.ld_dcls + c, 0.f, a.dcls_bf16);
    if (a.dreg)
      for (int j = 5; j < a.ld_dreg; ++j) store_g(a.dreg, cell * a.ld_dreg + j, 0.f, a.dreg_bf16);
  }
  block_partials<kThreads>(a, s_cls, s_reg, s_cen);
}

// LDS-staged form: the block's NTH cells' target, class and box rows are loaded cooperatively (every
// global load coalesced and issued before any math), each thread runs its cell from LDS (row pitch R
// odd: conflict-free) writing the scaled gradients back in place, and the gradient rows leave as
// 16-byte stores of whole rows (padding columns zero).  Same cell_loss, same per-thread and block
// sum order as fcos_loss_kernel at NTH = 256: bit-identical results.
template <int NTH>
__global__ void __launch_bounds__(NTH) fcos_loss_lds_kernel(LossArgs a, int R) {
  extern __shared__ float rows[];
  const int b = blockIdx.y, p0 = blockIdx.x * NTH;
  const int ncell = min(NTH, a.P - p0);
  const bool cen_in_cls = a.reg_type & 16;
  const int cc = (a.C + 7) / 8 * 8;
  const int T5 = 5 + a.C, ncc = cen_in_cls ? cc + 1 : a.C, nrg = cen_in_cls ? 4 : 5;
  const int OC = T5, OR = T5 + ncc;                   // row: targets | class logits | box (5 slots)
  const size_t cell0 = (size_t)b * a.P + p0;
  {
    // every global load of a batch issued before its LDS stores (a load -> store loop waited for
    // each load in turn): batches of 8 per thread
    const float* tg = a.tgt + cell0 * T5;
    const float* cg = a.cls + cell0 * a.ld_cls;
    const float* rg = a.reg + cell0 * a.ld_reg;
    auto stage = [&](int n, int width, int ld, const float* src, int col0) {
      for (int base = 0; base < n; base += 8 * NTH) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = base + (int)threadIdx.x + u * NTH;
          const int r = i / width;
          v[u] = i < n ? src[(size_t)r * ld + (i - r * width)] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int i = base + (int)threadIdx.x + u * NTH;
          const int r = i / width;
          if (i < n) rows[r * R + col0 + (i - r * width)] = v[u];
        }
      }
    };
    stage(ncell * T5, T5, T5, tg, 0);
    stage(ncell * ncc, ncc, a.ld_cls, cg, OC);
    stage(ncell * nrg, nrg, a.ld_reg, rg, OR);
  }
  __syncthreads();
  float s_cls = 0.f, s_reg = 0.f, s_cen = 0.f;
  if ((int)threadIdx.x < ncell) {
    float* row = rows + threadIdx.x * R;
    cell_loss(
        a, [&](int i) { return row[i]; }, [&](int c) { return row[OC + c]; }, [&](int j) { return row[OR + j]; },
        [&](int c, float v) { row[OC + c] = v; }, [&](float v) { row[OC + cc] = v; },
        [&](int j, float v) { row[OR + j] = v; }, s_cls, s_reg, s_cen);
  }
  __syncthreads();
  // gradient rows: whole rows in 16-byte pieces (8 bf16 or 4 fp32 columns), padding columns zero
  auto grad_rows = [&](void* dst, int ld, int is_bf16, int base, int ncol, int extra) {
    const int w = is_bf16 ? 8 : 4, npc = ld / w;
    for (int i = threadIdx.x; i < ncell * npc; i += NTH) {
      const int r = i / npc, c0 = (i - r * npc) * w;
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u;
        v[u] = (u < w && (c < ncol || c == extra)) ? rows[r * R + base + c] : 0.f;
      }
      if (is_bf16) {
        s16x8 o;
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = (short)f32_to_bf16(v[u]);
        *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(dst) + (cell0 + r) * ld + c0) = o;
      } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dst) + (cell0 + r) * ld + c0) = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
  };
  if (a.dcls) grad_rows(a.dcls, a.ld_dcls, a.dcls_bf16, OC, a.C, cen_in_cls ? cc : -1);
  if (a.dreg) grad_rows(a.dreg, a.ld_dreg, a.dreg_bf16, OR, 5, -1);
  block_partials<NTH>(a, s_cls, s_reg, s_cen);
}

// Four lanes per cell (round 6): the class terms -- 20 focal terms per cell, the kernel's VALU work --
// spread over the cell's 4 lanes (class c on lane c % 4), each term parked in the cell's target slot
// 5 + c once read, then the cell's owner lane sums them in class order (the same fp32 sequence as
// cell_loss) and runs the rest of the cell; the block's partial sums take the 256 owners' values in
// the fcos_loss_kernel lane order.  Bit-identical to fcos_loss_lds_kernel<256>; 4x the waves (one
// thread per cell left 1.4 waves per SIMD at 512 / bs 16).
template <int CPB>
__global__ void __launch_bounds__(4 * CPB) fcos_loss_lds4_kernel(LossArgs a, int R) {
  constexpr int NTH = 4 * CPB;
  extern __shared__ float rows[];
  float* csum = rows + CPB * R;                       // per-cell (s_cls, s_reg, s_cen)
  const int b = blockIdx.y, p0 = blockIdx.x * CPB;
  const int ncell = min(CPB, a.P - p0);
  const bool cen_in_cls = a.reg_type & 16;
  const int cc = (a.C + 7) / 8 * 8;
  const int T5 = 5 + a.C, ncc = cen_in_cls ? cc + 1 : a.C, nrg = cen_in_cls ? 4 : 5;
  const int OC = T5, OR = T5 + ncc;
  const size_t cell0 = (size_t)b * a.P + p0;
  {
    const float* tg = a.tgt + cell0 * T5;
    for (int i = threadIdx.x; i < ncell * T5; i += NTH) {
      const int r = i / T5;
      rows[r * R + (i - r * T5)] = tg[i];
    }
    const float* cg = a.cls + cell0 * a.ld_cls;
    for (int i = threadIdx.x; i < ncell * ncc; i += NTH) {
      const int r = i / ncc, c = i - r * ncc;
      rows[r * R + OC + c] = cg[(size_t)r * a.ld_cls + c];
    }
    const float* rg = a.reg + cell0 * a.ld_reg;
    for (int i = threadIdx.x; i < ncell * nrg; i += NTH) {
      const int r = i / nrg, j = i - r * nrg;
      rows[r * R + OR + j] = rg[(size_t)r * a.ld_reg + j];
    }
  }
  __syncthreads();
  const int cell = threadIdx.x >> 2, sub = threadIdx.x & 3;
  float tmax = 0.f, y0 = 0.f;
  if (cell < ncell) {
    float* row = rows + cell * R;
    y0 = row[5];
    for (int c = sub; c < a.C; c += 4) {
      const float y = row[5 + c];
      tmax = fmaxf(tmax, y);
      float g;
      row[5 + c] = focal_term(y, row[OC + c], a.alpha, a.gamma, &g);   // the term, in its target slot
      row[OC + c] = g * a.grad_scale;
    }
  }
  tmax = fmaxf(tmax, __shfl_xor(tmax, 1, 64));
  tmax = fmaxf(tmax, __shfl_xor(tmax, 2, 64));
  __syncthreads();
  if (sub == 0) {
    float s_cls = 0.f, s_reg = 0.f, s_cen = 0.f;
    if (cell < ncell) {
      float* row = rows + cell * R;
      for (int c = 0; c < a.C; ++c) s_cls += row[5 + c];
      const float mask = (a.reg_type & 32) ? y0 : (tmax >= 1.0f ? 1.0f : 0.0f);
      cell_rest(
          a, [&](int i) { return row[i]; }, [&](int c) { return row[OC + c]; }, [&](int j) { return row[OR + j]; },
          [&](float v) { row[OC + cc] = v; }, [&](int j, float v) { row[OR + j] = v; }, mask, s_reg, s_cen);
    }
    csum[cell * 3] = s_cls;
    csum[cell * 3 + 1] = s_reg;
    csum[cell * 3 + 2] = s_cen;
  }
  __syncthreads();
  auto grad_rows = [&](void* dst, int ld, int is_bf16, int base, int ncol, int extra) {
    const int w = is_bf16 ? 8 : 4, npc = ld / w;
    for (int i = threadIdx.x; i < ncell * npc; i += NTH) {
      const int r = i / npc, c0 = (i - r * npc) * w;
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int c = c0 + u;
        v[u] = (u < w && (c < ncol || c == extra)) ? rows[r * R + base + c] : 0.f;
      }
      if (is_bf16) {
        s16x8 o;
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = (short)f32_to_bf16(v[u]);
        *reinterpret_cast<s16x8*>(reinterpret_cast<cvl_bf16*>(dst) + (cell0 + r) * ld + c0) = o;
      } else {
        *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(dst) + (cell0 + r) * ld + c0) = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
  };
  if (a.dcls) grad_rows(a.dcls, a.ld_dcls, a.dcls_bf16, OC, a.C, cen_in_cls ? cc : -1);
  if (a.dreg) grad_rows(a.dreg, a.ld_dreg, a.dreg_bf16, OR, 5, -1);
  // lanes 0 .. CPB-1 carry cells 0 .. CPB-1 as fcos_loss_kernel's threads do; the other waves add zeros
  const bool own = (int)threadIdx.x < CPB;
  block_partials<NTH>(a, own ? csum[threadIdx.x * 3] : 0.f, own ? csum[threadIdx.x * 3 + 1] : 0.f,
                      own ? csum[threadIdx.x * 3 + 2] : 0.f);
}

__global__ void fcos_loss_finalize(const double* partial, float* losses, int tiles) {
  const int b = blockIdx.x;
  const int k = threadIdx.x;   // 0..2
  if (k < 3) {
    double s = 0.0;
    for (int i = 0; i < tiles; ++i) s += partial[((size_t)b * tiles + i) * 3 + k];
    losses[b * 3 + k] = (float)s;
  }
}

}  // namespace

extern "C" size_t cvl_fcos_loss_workspace_size(int B, int P) {
  const size_t tiles = (size_t)(P + 63) / 64;        // per-tile partials of the smallest (64-cell) tiles
  return (size_t)B * tiles * 3 * sizeof(double);
}

extern "C" int cvl_fcos_loss_ex(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                                const float* targets, int B, int P, int num_classes, int reg_type,
                                float grad_scale, float alpha, float gamma, float delta, float* losses,
                                void* d_reg, int ld_dreg, int dreg_dtype, void* d_cls, int ld_dcls, int dcls_dtype,
                                void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG(reg_pred && cls_pred && targets && losses && workspace);
  CVL_CHECK_ARG(B > 0 && P > 0 && num_classes > 0);
  CVL_CHECK_ARG(workspace_bytes >= cvl_fcos_loss_workspace_size(B, P));
  const int kind = reg_type & 3, cen_in_cls = (reg_type & 16) ? 1 : 0;
  CVL_CHECK_ARG((kind == 0 || kind == 1) && (reg_type & ~63) == 0 && !(kind == 1 && (reg_type & 8)));
  CVL_CHECK_ARG(!(reg_type & 32) || num_classes == 1);
  CVL_CHECK_ARG(gamma >= 0.f && delta > 0.f);
  const int ncls_cols = cen_in_cls ? (num_classes + 7) / 8 * 8 + 1 : num_classes;
  CVL_CHECK_ARG(ld_reg >= (cen_in_cls ? 4 : 5) && ld_cls >= ncls_cols);
  CVL_CHECK_ARG(!d_reg || ld_dreg >= 5);
  CVL_CHECK_ARG(!d_cls || ld_dcls >= ncls_cols);
  CVL_CHECK_ARG((dreg_dtype == 0 || dreg_dtype == 1) && (dcls_dtype == 0 || dcls_dtype == 1));
  LossArgs a;
  a.reg = reg_pred; a.cls = cls_pred; a.tgt = targets; a.losses = losses;
  a.dreg = d_reg; a.dcls = d_cls; a.partial = (double*)workspace;
  a.ld_reg = ld_reg; a.ld_cls = ld_cls; a.ld_dreg = ld_dreg; a.ld_dcls = ld_dcls;
  a.dreg_bf16 = dreg_dtype; a.dcls_bf16 = dcls_dtype;
  a.P = P; a.C = num_classes; a.reg_type = reg_type; a.grad_scale = grad_scale;
  a.alpha = alpha; a.gamma = gamma; a.delta = delta;
  // the LDS-staged form when its rows fit (pitch R floats, odd) and the gradient rows take 16-B stores
  const int ncc = cen_in_cls ? (num_classes + 7) / 8 * 8 + 1 : num_classes;
  const int R = (5 + num_classes + ncc + 5) | 1;
  auto vec_ok = [](const void* p, int ld, int bf16) {
    return !p || ((reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % (bf16 ? 8 : 4) == 0);
  };
  int nth = 0;
  if (vec_ok(d_reg, ld_dreg, dreg_dtype) && vec_ok(d_cls, ld_dcls, dcls_dtype) && !cvl_dispatch_flag("loss_rows"))
    for (int n = 256; n >= 64 && !nth; n /= 2)
      if ((size_t)n * R * sizeof(float) <= 64 * 1024) nth = n;
  a.tiles = (P + (nth ? nth : kThreads) - 1) / (nth ? nth : kThreads);
  const size_t lds = (size_t)nth * R * sizeof(float);
  if (nth == 256 && !cvl_dispatch_flag("loss_lds1") && lds + 256 * 3 * sizeof(float) <= 64 * 1024)
    hipLaunchKernelGGL((fcos_loss_lds4_kernel<256>), dim3(a.tiles, B), dim3(1024), lds + 256 * 3 * sizeof(float),
                       (hipStream_t)stream, a, R);
  else if (nth == 256) hipLaunchKernelGGL((fcos_loss_lds_kernel<256>), dim3(a.tiles, B), dim3(256), lds, (hipStream_t)stream, a, R);
  else if (nth == 128) hipLaunchKernelGGL((fcos_loss_lds_kernel<128>), dim3(a.tiles, B), dim3(128), lds, (hipStream_t)stream, a, R);
  else if (nth == 64) hipLaunchKernelGGL((fcos_loss_lds_kernel<64>), dim3(a.tiles, B), dim3(64), lds, (hipStream_t)stream, a, R);
  else hipLaunchKernelGGL(fcos_loss_kernel, dim3(a.tiles, B), dim3(kThreads), 0, (hipStream_t)stream, a);
  int st = cvl_launch_status();
  if (st) return st;
  hipLaunchKernelGGL(fcos_loss_finalize, dim3(B), dim3(64), 0, (hipStream_t)stream,
                     (const double*)workspace, losses, a.tiles);
  return cvl_launch_status();
}

extern "C" int cvl_fcos_loss(const float* reg_pred, int ld_reg, const float* cls_pred, int ld_cls,
                             const float* targets, int B, int P, int num_classes, int reg_type,
                             float grad_scale, float* losses, void* d_reg, int ld_dreg,
                             int dreg_dtype, void* d_cls, int ld_dcls, int dcls_dtype,
                             void* workspace, size_t workspace_bytes, cvl_stream_t stream) {
  CVL_CHECK_ARG((reg_type & 32) == 0);
  return cvl_fcos_loss_ex(reg_pred, ld_reg, cls_pred, ld_cls, targets, B, P, num_classes, reg_type, grad_scale,
                          0.25f, 2.0f, 1.0f, losses, d_reg, ld_dreg, dreg_dtype, d_cls, ld_dcls, dcls_dtype,
                          workspace, workspace_bytes, stream);
}

// ---------------------------------------------------------------------------------------------
// fcos.py:112-134 prediction_to_corners: fp32 (cell centre -/+ ltrb), then float64 * stride
// ---------------------------------------------------------------------------------------------
namespace {
__global__ void fcos_decode_kernel(const float* p, int ld, int S0, int S1, double stride, double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S0 * S1) return;
  const int y = i / S1, x = i - (i / S1) * S1;
  const float gy = (float)y + 0.5f, gx = (float)x + 0.5f;
  const float* q = p + (size_t)i * ld;
  out[i * 4 + 0] = stride * (double)(gy - q[0]);
  out[i * 4 + 1] = stride * (double)(gx - q[2]);
  out[i * 4 + 2] = stride * (double)(gy + q[1]);
  out[i * 4 + 3] = stride * (double)(gx + q[3]);
}

// fcos_center_v1.py:124-147 prediction_to_corners(xy_pred, box_sc, stride): fp32 centre
// (grid + offset) * stride (grid WITHOUT +0.5), size * box_sc, fp32 corners stored as float64
__global__ void fcos_v1_decode_kernel(const float* p, int ld, int S0, int S1, float box_sc, float stride,
                                      double* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= S0 * S1) return;
  const int y = i / S1, x = i - (i / S1) * S1;
  const float* q = p + (size_t)i * ld;
  const float yc = ((float)y + q[0]) * stride, xc = ((float)x + q[1]) * stride;
  const float bh = q[2] * box_sc, bw = q[3] * box_sc;
  out[i * 4 + 0] = (double)(yc - bh / 2.0f);            // TF fp32 ops, stored into float64
  out[i * 4 + 2] = (double)(yc + bh / 2.0f);
  out[i * 4 + 1] = (double)(xc - bw / 2.0f);
  out[i * 4 + 3] = (double)(xc + bw / 2.0f);
}
}  // namespace

extern "C" int cvl_fcos_decode(const float* pred, int ld, int S0, int S1, double stride, double* out,
                               cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && out && ld >= 4 && S0 > 0 && S1 > 0);
  hipLaunchKernelGGL(fcos_decode_kernel, dim3((S0 * S1 + 255) / 256), dim3(256), 0, (hipStream_t)stream, pred,
                     ld, S0, S1, stride, out);
  return cvl_launch_status();
}

extern "C" int cvl_fcos_v1_decode(const float* pred, int ld, int S0, int S1, float box_sc, float stride, double* out,
                                  cvl_stream_t stream) {
  CVL_CHECK_ARG(pred && out && ld >= 4 && S0 > 0 && S1 > 0);
  hipLaunchKernelGGL(fcos_v1_decode_kernel, dim3((S0 * S1 + 255) / 256), dim3(256), 0, (hipStream_t)stream, pred,
                     ld, S0, S1, box_sc, stride, out);
  return cvl_launch_status();
}

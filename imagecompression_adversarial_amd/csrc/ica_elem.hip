// Bandwidth-bound kernels of the attack step (HBM roofline), layout
// conversion, deterministic per-image reductions, and the eval-time entropy
// models.
//
// Reference anchors:
//   bounds / clamp pass-through       utils/ops.py:28-56 (Low_bound, Up_bound)
//   noise box + input clamp           attack_rd.py:507,517
//   L2 losses + branch                attack_rd.py:333-379 (attack_our)
//   Adam on the noise                 attack_rd.py:502,546-548 (torch.optim.Adam op order)
//   I-FGSM / MI-FGSM update           attack_ifgsm.py:348-362,393-419
//   EntropyBottleneck / GaussianConditional likelihoods, bpp
//                                     anchors/model.py:86-108, attack_rd.py:419 (CompressAI semantics)
#include "ica_common.h"

// ---------------------------------------------------------------------------
// Layout conversion  NCHW <-> nChw4c (padded channels are written as zero)
// ---------------------------------------------------------------------------
__global__ void nchw_to_nc4_kernel(const float* __restrict__ src, float* __restrict__ dst, int N, int C, int H,
                                   int W) {
  const int C4 = (C + 3) >> 2;
  const long HW = (long)H * W;
  const long total = (long)N * C4 * HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i % HW;
    const long t = i / HW;
    const int c4 = t % C4, n = t / C4;
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c4 * 4 + e;
      v[e] = c < C ? src[((long)n * C + c) * HW + pix] : 0.f;
    }
    st4(dst + i * 4, v);
  }
}

__global__ void nc4_to_nchw_kernel(const float* __restrict__ src, float* __restrict__ dst, int N, int C, int H,
                                   int W) {
  const int C4 = (C + 3) >> 2;
  const long HW = (long)H * W;
  const long total = (long)N * C4 * HW;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long pix = i % HW;
    const long t = i / HW;
    const int c4 = t % C4, n = t / C4;
    const f32x4 v = ld4(src + i * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = c4 * 4 + e;
      if (c < C) dst[((long)n * C + c) * HW + pix] = v[e];
    }
  }
}

// ---------------------------------------------------------------------------
// Deterministic per-image reduction: partial[b][k] for k < nblk -> out[b]
// (fixed order: each block reduces a strided slice, then a single-wave tree).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float block_sum_256(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float r = 0.f;
  if (threadIdx.x == 0) r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
  return r;
}

__global__ void reduce_rows_kernel(const float* __restrict__ part, float* __restrict__ out, int nblk, float scale) {
  __shared__ float sh[4];
  const int b = blockIdx.x;
  float v = 0.f;
  for (int k = threadIdx.x; k < nblk; k += 256) v += part[(long)b * nblk + k];
  const float r = block_sum_256(v, sh);
  if (threadIdx.x == 0) out[b] = r * scale;
}

// ---------------------------------------------------------------------------
// Attack step, per-image semantics (each image of the batch is an independent
// reference run; B == 1 reproduces attack_rd.py exactly).  Image tensors are
// NCHW [B][3][H][W]; network tensors nChw4c with C4 == 1.
// ---------------------------------------------------------------------------
constexpr int ELEM_BLOCKS_PER_IMAGE = 256;

// noise_c = Up(Low(noise,-eps),eps); im_in = Up(Low(im_s + noise_c, 0), 1)
// -> im_in (nChw4c, ch3 = 0) and partial sums of (im_s - im_in)^2.
__global__ void attack_prologue_kernel(const float* __restrict__ noise, const float* __restrict__ im_s,
                                       float* __restrict__ im_in4, float* __restrict__ part, long HW, float eps,
                                       int clamp_in) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const float* nz = noise + (long)b * 3 * HW;
  const float* is = im_s + (long)b * 3 * HW;
  float* o4 = im_in4 + (long)b * 4 * HW;
  float acc = 0.f;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float nc = fminf(fmaxf(nz[c * HW + pix], -eps), eps);
      const float s = is[c * HW + pix];
      const float u = fadd_rn(s, nc);
      const float ii = clamp_in ? fminf(fmaxf(u, 0.f), 1.f) : u;
      v[c] = ii;
      const float d = fsub_rn(s, ii);
      acc = fadd_rn(acc, fmul_rn(d, d));
    }
    st4(o4 + pix * 4, v);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// Expensive-branch L2 loss on the reconstruction.
// mode 0 (attack_rd.py:354,364): o = Up(Low(x_hat,0),1) if clamp; loss = 1 - mean((os-o)^2);
//        dL/dx_hat = bound-bwd( 2*fl(invN*(os-o)) )
// mode 1 (attack_ifgsm.py:396): o = x_hat; loss = mean((os-o)^2); dL/dx_hat = -2*fl(invN*(os-o))
__global__ void attack_loss_kernel(const float* __restrict__ xhat4, const float* __restrict__ out_s,
                                   float* __restrict__ grad4, float* __restrict__ part, long HW, float invN,
                                   int clamp, int mode) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const float* x4 = xhat4 + (long)b * 4 * HW;
  const float* os = out_s + (long)b * 3 * HW;
  float* g4 = grad4 + (long)b * 4 * HW;
  float acc = 0.f;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 xv = ld4(x4 + pix * 4);
    f32x4 gv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float xh = xv[c];
      const float lo = fmaxf(xh, 0.f);
      const float o = (clamp && mode == 0) ? fminf(lo, 1.f) : xh;
      const float d = fsub_rn(os[c * HW + pix], o);
      acc = fadd_rn(acc, fmul_rn(d, d));
      const float t = fmul_rn(invN, d);
      float g = mode == 0 ? fadd_rn(t, t) : -fadd_rn(t, t);
      if (clamp && mode == 0) {
        g = (lo <= 1.f || g > 0.f) ? g : g * 0.f;  // Up_bound backward
        g = (xh >= 0.f || g < 0.f) ? g : g * 0.f;  // Low_bound backward
      }
      gv[c] = g;
    }
    st4(g4 + pix * 4, gv);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// Targeted / ROI attack (semantics in DESIGN.md "Targeted / ROI attack"):
//   loss_i = mean_tar((s - ii)^2) + la_bkg_in * mean_bkg((s - ii)^2)              (box-weighted, per image)
//   loss_o = la_tar * mean_tar((ot - o)^2) + la_bkg_out * mean_bkg((os - o)^2)     (minimised)
// with o = Up(Low(x_hat, 0), 1) when clamping; ot = the codec's reconstruction of the target image.
__global__ void roi_prologue_kernel(const float* __restrict__ noise, const float* __restrict__ im_s,
                                    float* __restrict__ im_in4, float* __restrict__ part, long HW, long W, float eps,
                                    RoiBox roi) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const float* nz = noise + (long)b * 3 * HW;
  const float* is = im_s + (long)b * 3 * HW;
  float* o4 = im_in4 + (long)b * 4 * HW;
  float acc = 0.f;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const float w = roi_inside(roi, pix, W) ? roi.w_in_tar : roi.w_in_bkg;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float nc = fminf(fmaxf(nz[c * HW + pix], -eps), eps);
      const float s = is[c * HW + pix];
      const float u = fadd_rn(s, nc);
      const float ii = fminf(fmaxf(u, 0.f), 1.f);
      v[c] = ii;
      const float d = fsub_rn(s, ii);
      acc = fadd_rn(acc, fmul_rn(w, fmul_rn(d, d)));
    }
    st4(o4 + pix * 4, v);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

__global__ void roi_loss_kernel(const float* __restrict__ xhat4, const float* __restrict__ out_s,
                                const float* __restrict__ out_t, float* __restrict__ grad4, float* __restrict__ part,
                                long HW, long W, RoiBox roi, int clamp) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const float* x4 = xhat4 + (long)b * 4 * HW;
  const float* os = out_s + (long)b * 3 * HW;
  const float* ot = out_t + (long)b * 3 * HW;
  float* g4 = grad4 + (long)b * 4 * HW;
  float acc = 0.f;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const bool tar = roi_inside(roi, pix, W);
    const float w = tar ? roi.w_out_tar : roi.w_out_bkg;
    const float* ref = tar ? ot : os;
    const f32x4 xv = ld4(x4 + pix * 4);
    f32x4 gv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float xh = xv[c];
      const float lo = fmaxf(xh, 0.f);
      const float o = clamp ? fminf(lo, 1.f) : xh;
      const float d = fsub_rn(ref[c * HW + pix], o);
      acc = fadd_rn(acc, fmul_rn(w, fmul_rn(d, d)));
      const float t = fmul_rn(w, d);
      float g = -fadd_rn(t, t);
      if (clamp) {
        g = (lo <= 1.f || g > 0.f) ? g : g * 0.f;  // Up_bound backward
        g = (xh >= 0.f || g < 0.f) ? g : g * 0.f;  // Low_bound backward
      }
      gv[c] = g;
    }
    st4(g4 + pix * 4, gv);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// Branch select + bounds backward + torch Adam step on the noise (in place).
//   cheap[b] = loss_i[b] > thr  -> g = -2*fl(invN*(im_s - im_in))   (L2 input loss)
//   else                        -> g = g_net (nChw4c)               (network gradient)
// Adam (torch 2.x op order): m = fma(1-b1, g-m, m); v = v*b2 + ((1-b2)*g)*g;
// denom = sqrt(v)/bc2s + eps; p = p + neg_step*(m/denom)
// ROI (targeted / masked attack): the cheap-branch input loss is the box-weighted mean, so the
// per-element weight w_in(pixel) replaces invN (same op order: t = w*(s - ii), g = -(t + t)).
// gpos (optional): row of image b in gnet4 when the network ran on a compacted sub-batch of the expensive
// images (ica_branch_select); null = gnet4 is indexed by b.  census (optional): census[b] += cheap, the
// per-image count of cheap-branch steps (network FLOPs count only the expensive image-steps).
template <bool ROI>
__global__ void attack_adam_kernel(float* __restrict__ noise, const float* __restrict__ im_s,
                                   const float* __restrict__ gnet4, const float* __restrict__ loss_i,
                                   const float* __restrict__ cheap_grad, float* __restrict__ m,
                                   float* __restrict__ v, float* __restrict__ im_in_out, long HW, float eps,
                                   float thr, float invN, float bc2s, float neg_step, int* __restrict__ branch,
                                   RoiBox roi, long W, const int* __restrict__ gpos, int* __restrict__ census,
                                   int clamp_in) {
  const int b = blockIdx.y;
  const bool cheap = loss_i[b] > thr;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (branch) branch[b] = cheap ? 1 : 0;
    if (census) census[b] += cheap ? 1 : 0;
  }
  const long off = (long)b * 3 * HW;
  const long grow = cheap ? 0 : (gpos ? gpos[b] : b);   // the network gradient is read only when used
  // one pixel's update (the op order below is the pinned one); g_in: the network gradient of channel c
  auto update = [&](long pix, float nz, float s, float g_in, float cg, float mo, float vo, float& nz_out,
                    float& m_out, float& v_out, float& ii_out) {
    const float lowN = fmaxf(nz, -eps);
    const float nc = fminf(lowN, eps);
    const float u = fadd_rn(s, nc);
    const float lowU = clamp_in ? fmaxf(u, 0.f) : u;
    const float ii = clamp_in ? fminf(lowU, 1.f) : u;
    ii_out = ii;
    float g;
    if (cheap) {
      if (cheap_grad) {
        g = cg;
      } else {
        float w = invN;
        if constexpr (ROI) w = roi_inside(roi, pix, W) ? roi.w_in_tar : roi.w_in_bkg;
        const float t = fmul_rn(w, fsub_rn(s, ii));
        g = -fadd_rn(t, t);
      }
    } else {
      g = g_in;
    }
    if (clamp_in) {
      g = (lowU <= 1.f || g > 0.f) ? g : g * 0.f;
      g = (u >= 0.f || g < 0.f) ? g : g * 0.f;
    }
    g = (lowN <= eps || g > 0.f) ? g : g * 0.f;
    g = (nz >= -eps || g < 0.f) ? g : g * 0.f;
    const float mn = __fmaf_rn(0.1f, fsub_rn(g, mo), mo);
    const float vn = fadd_rn(fmul_rn(vo, 0.999f), fmul_rn(fmul_rn(0.001f, g), g));
    const float denom = fadd_rn(fdiv_rn(sqrtf(vn), bc2s), 1e-8f);
    m_out = mn;
    v_out = vn;
    nz_out = fadd_rn(nz, fmul_rn(neg_step, fdiv_rn(mn, denom)));
  };
  if ((HW & 3) == 0) {
    // four pixels per thread: 16-B loads / stores of every plane (same per-element ops, same bits; the kernel has
    // no reduction).  The per-channel 4-B form moved 3.4 GB in 0.84 ms (4.0 TB/s) at the config-5 shapes.
    const long HW4 = HW >> 2;
    for (long q = (long)blockIdx.x * 256 + threadIdx.x; q < HW4; q += (long)gridDim.x * 256) {
      const long pix0 = q * 4;
      f32x4 gn[4] = {};
      if (!cheap) {
#pragma unroll
        for (int k = 0; k < 4; ++k) gn[k] = ld4(gnet4 + (grow * HW + pix0 + k) * 4);
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const long i0 = off + c * HW + pix0;
        const f32x4 nz4 = ld4(noise + i0), s4 = ld4(im_s + i0), m4 = ld4(m + i0), v4 = ld4(v + i0);
        const f32x4 cg4 = (cheap && cheap_grad) ? ld4(cheap_grad + i0) : f32x4{0.f, 0.f, 0.f, 0.f};
        float no[4], mo4[4], vo4[4], io[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          update(pix0 + k, nz4[k], s4[k], gn[k][c], cg4[k], m4[k], v4[k], no[k], mo4[k], vo4[k], io[k]);
        if (im_in_out) st4(im_in_out + i0, f32x4{io[0], io[1], io[2], io[3]});
        st4(m + i0, f32x4{mo4[0], mo4[1], mo4[2], mo4[3]});
        st4(v + i0, f32x4{vo4[0], vo4[1], vo4[2], vo4[3]});
        st4(noise + i0, f32x4{no[0], no[1], no[2], no[3]});
      }
    }
    return;
  }
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    f32x4 gn = {0.f, 0.f, 0.f, 0.f};
    if (!cheap) gn = ld4(gnet4 + (grow * HW + pix) * 4);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long i = off + c * HW + pix;
      float no, mo, vo, io;
      update(pix, noise[i], im_s[i], gn[c], (cheap && cheap_grad) ? cheap_grad[i] : 0.f, m[i], v[i], no, mo, vo, io);
      if (im_in_out) im_in_out[i] = io;
      m[i] = mo;
      v[i] = vo;
      noise[i] = no;
    }
  }
}

// Branch compaction (attack_rd.py:334 decides per image whether the network runs at all).  One thread walks
// the batch in order: idx[0..E) = the expensive images (loss_i <= thr), gpos[b] = their row in the compacted
// sub-batch (-1 for cheap images), sel[0] = E.  The host reads sel (E + B ints) to size the sub-batch.
__global__ void branch_select_kernel(const float* __restrict__ loss_i, float thr, int B, int* __restrict__ sel,
                                     int* __restrict__ gpos) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  int e = 0;
  for (int b = 0; b < B; ++b) {
    const bool cheap = loss_i[b] > thr;
    gpos[b] = cheap ? -1 : e;
    if (!cheap) sel[1 + e++] = b;
  }
  sel[0] = e;
}

// dst[r] = src[idx[r]] for r < E: whole images of `quads` 16-byte vectors each (grid.y = E).
__global__ void gather_images_kernel(const f32x4* __restrict__ src, f32x4* __restrict__ dst,
                                     const int* __restrict__ idx, long quads) {
  const int r = blockIdx.y;
  const f32x4* s = src + (long)idx[r] * quads;
  f32x4* d = dst + (long)r * quads;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < quads; i += (long)gridDim.x * 256) d[i] = s[i];
}

// I-FGSM / MI-FGSM step (attack_ifgsm.py:348-362, 405-419), per image.
//   momentum: gacc = gacc + grad / l1[b]; x = clamp(x + alpha*sign(gacc), 0, 1)
//   plain:    x = x + alpha*sign(grad)
//   then project into [im_s - eps, im_s + eps] with torch.where semantics.
__global__ void ifgsm_kernel(float* __restrict__ x, const float* __restrict__ im_s, const float* __restrict__ grad4,
                             float* __restrict__ gacc, const float* __restrict__ l1, long HW, float alpha, float eps,
                             int momentum) {
  const int b = blockIdx.y;
  const long off = (long)b * 3 * HW;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 gv = ld4(grad4 + ((long)b * HW + pix) * 4);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const long i = off + c * HW + pix;
      float g = gv[c];
      float xn;
      if (momentum) {
        const float ga = fadd_rn(gacc[i], fdiv_rn(g, l1[b]));
        gacc[i] = ga;
        const float sg = ga > 0.f ? 1.f : (ga < 0.f ? -1.f : 0.f);
        xn = fminf(fmaxf(fadd_rn(x[i], fmul_rn(alpha, sg)), 0.f), 1.f);
      } else {
        const float sg = g > 0.f ? 1.f : (g < 0.f ? -1.f : 0.f);
        xn = fadd_rn(x[i], fmul_rn(alpha, sg));
      }
      const float s = im_s[i];
      const float hi = fadd_rn(s, eps), lo = fsub_rn(s, eps);
      xn = xn > hi ? hi : xn;
      xn = xn < lo ? lo : xn;
      x[i] = xn;
    }
  }
}

// per-image L1 partials of an nChw4c C4==1 tensor (channels 0..2)
__global__ void l1_partial_kernel(const float* __restrict__ g4, float* __restrict__ part, long HW) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  float acc = 0.f;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 v = ld4(g4 + ((long)b * HW + pix) * 4);
    acc += (fabsf(v[0]) + fabsf(v[1])) + fabsf(v[2]);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// ---------------------------------------------------------------------------
// Entropy models (eval / train forward).  Tensors nChw4c [N][C4][H][W][4].
// ---------------------------------------------------------------------------
// GaussianConditional: y_hat = round(y - mu) + mu (eval, rint = half-even) or
// y + noise (train); lik = max(Phi((.5-|v|)/s) - Phi((-.5-|v|)/s), 1e-9),
// s = max(scales, 0.11).  Also emits per-image partial sums of log(lik).
__global__ void gc_kernel(const float* __restrict__ y, const float* __restrict__ scales,
                          const float* __restrict__ means, const float* __restrict__ qnoise,
                          float* __restrict__ y_hat, float* __restrict__ lik, float* __restrict__ part, int C,
                          long per_image, int training) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const int C4 = (C + 3) >> 2;
  const long HW = per_image / (4L * C4);
  float acc = 0.f;
  for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < per_image; k += (long)gridDim.x * 256) {
    const long i = (long)b * per_image + k;
    const int e = (int)(k & 3);
    const int c4 = (int)((k >> 2) / HW);
    if (c4 * 4 + e >= C) {
      if (y_hat) y_hat[i] = 0.f;
      if (lik) lik[i] = 1.f;
      continue;
    }
    const float yv = y[i];
    const float mu = means ? means[i] : 0.f;
    float yh;
    if (training) yh = fadd_rn(yv, qnoise[i]);
    else yh = means ? fadd_rn(rintf(fsub_rn(yv, mu)), mu) : rintf(yv);
    const float sc = fmaxf(scales[i], 0.11f);
    const float val = fabsf(means ? fsub_rn(yh, mu) : yh);
    const float k2 = -0.70710678118654752f;
    const float up = 0.5f * erfcf(k2 * fdiv_rn(fsub_rn(0.5f, val), sc));
    const float lo = 0.5f * erfcf(k2 * fdiv_rn(fsub_rn(-0.5f, val), sc));
    const float l = fmaxf(fsub_rn(up, lo), 1e-9f);
    if (y_hat) y_hat[i] = yh;
    if (lik) lik[i] = l;
    acc += logf(l);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// EntropyBottleneck (filters (3,3,3,3)).  Per-channel packed parameters
// prm[c][58]: softplus(H0)[3], b0[3], tanh(a0)[3], softplus(H1)[9], b1[3], tanh(a1)[3],
//             softplus(H2)[9], b2[3], tanh(a2)[3], softplus(H3)[9], b3[3], tanh(a3)[3],
//             softplus(H4)[3], b4[1]   (= 3+3+3 + 3*(9+3+3) + 3+1 = 58)
__device__ __forceinline__ float eb_logit(const float* q, float u) {
  float l0[3], l1[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float t = fadd_rn(fmul_rn(q[k], u), q[3 + k]);
    l0[k] = fadd_rn(t, fmul_rn(q[6 + k], tanhf(t)));
  }
  const float* s = q + 9;
#pragma unroll
  for (int layer = 0; layer < 3; ++layer) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float t = fadd_rn(fadd_rn(fmul_rn(s[3 * k], l0[0]), fmul_rn(s[3 * k + 1], l0[1])), fmul_rn(s[3 * k + 2], l0[2]));
      t = fadd_rn(t, s[9 + k]);
      l1[k] = fadd_rn(t, fmul_rn(s[12 + k], tanhf(t)));
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) l0[k] = l1[k];
    s += 15;
  }
  const float t = fadd_rn(fadd_rn(fmul_rn(s[0], l0[0]), fmul_rn(s[1], l0[1])), fmul_rn(s[2], l0[2]));
  return fadd_rn(t, s[3]);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void eb_kernel(const float* __restrict__ z, const float* __restrict__ prm, const float* __restrict__ med,
                          const float* __restrict__ qnoise, float* __restrict__ z_hat, float* __restrict__ lik,
                          float* __restrict__ part, int C, long per_image, int training) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  const int C4 = (C + 3) >> 2;
  const long HW = per_image / (4L * C4);
  float acc = 0.f;
  for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < per_image; k += (long)gridDim.x * 256) {
    const long i = (long)b * per_image + k;
    const int e = (int)(k & 3);
    const int c = (int)((k >> 2) / HW) * 4 + e;
    if (c >= C) {
      if (z_hat) z_hat[i] = 0.f;
      if (lik) lik[i] = 1.f;
      continue;
    }
    const float zv = z[i];
    const float md = med[c];
    const float v = training ? fadd_rn(zv, qnoise[i]) : fadd_rn(rintf(fsub_rn(zv, md)), md);
    const float* q = prm + (long)c * 58;
    const float lower = eb_logit(q, fsub_rn(v, 0.5f));
    const float upper = eb_logit(q, fadd_rn(v, 0.5f));
    const float sm = fadd_rn(lower, upper);
    const float sg = sm > 0.f ? -1.f : (sm < 0.f ? 1.f : 0.f);
    const float l = fmaxf(fabsf(fsub_rn(sigmoidf_(sg * upper), sigmoidf_(sg * lower))), 1e-9f);
    if (z_hat) z_hat[i] = v;
    if (lik) lik[i] = l;
    acc += logf(l);
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// prm[c][58] from the EntropyBottleneck parameters (softplus / tanh applied once).
__device__ __forceinline__ float softplusf_(float x) { return x > 20.f ? x : log1pf(expf(x)); }

__global__ void pack_eb_kernel(const float* __restrict__ m0, const float* __restrict__ m1,
                               const float* __restrict__ m2, const float* __restrict__ m3,
                               const float* __restrict__ m4, const float* __restrict__ b0,
                               const float* __restrict__ b1, const float* __restrict__ b2,
                               const float* __restrict__ b3, const float* __restrict__ b4,
                               const float* __restrict__ f0, const float* __restrict__ f1,
                               const float* __restrict__ f2, const float* __restrict__ f3,
                               const float* __restrict__ quantiles, float* __restrict__ prm,
                               float* __restrict__ med, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float* q = prm + (long)c * 58;
  for (int k = 0; k < 3; ++k) {
    q[k] = softplusf_(m0[c * 3 + k]);
    q[3 + k] = b0[c * 3 + k];
    q[6 + k] = tanhf(f0[c * 3 + k]);
  }
  const float* ms[3] = {m1, m2, m3};
  const float* bs[3] = {b1, b2, b3};
  const float* fs[3] = {f1, f2, f3};
  for (int layer = 0; layer < 3; ++layer) {
    float* s = q + 9 + 15 * layer;
    for (int k = 0; k < 9; ++k) s[k] = softplusf_(ms[layer][c * 9 + k]);
    for (int k = 0; k < 3; ++k) {
      s[9 + k] = bs[layer][c * 3 + k];
      s[12 + k] = tanhf(fs[layer][c * 3 + k]);
    }
  }
  for (int k = 0; k < 3; ++k) q[54 + k] = softplusf_(m4[c * 3 + k]);
  q[57] = b4[c];
  med[c] = quantiles[c * 3 + 1];
}

__global__ void abs_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = fabsf(x[i]);
}

// fp32 <-> bf16 activation casts at the ends of the bf16 conv path (latent for the entropy models,
// y_hat into g_s): 4 values per thread, RNE (v_cvt_pk_bf16_f32) / exact widening.
__global__ void cast_f32_bf16_kernel(const f32x4* __restrict__ x, u32x2* __restrict__ y, long nq) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (long)gridDim.x * blockDim.x)
    y[i] = f4_to_bf4(x[i]);
}
__global__ void cast_bf16_f32_kernel(const u32x2* __restrict__ x, f32x4* __restrict__ y, long nq) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nq; i += (long)gridDim.x * blockDim.x)
    y[i] = bf4_to_f4(x[i]);
}

// round half to even (torch.round / quantize "dequantize" with means=None; SURVEY §8 a16: rintf)
__global__ void round_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = rintf(x[i]);
}

// per-image sum of squared differences (mse numerators) for nChw4c C4==1 tensors
// or plain NCHW float tensors: both given as [B][len] with stride.
__global__ void sqdiff_partial_kernel(const float* __restrict__ a, const float* __restrict__ b_,
                                      float* __restrict__ part, long len, int clamp_a) {
  __shared__ float sh[4];
  const int b = blockIdx.y;
  float acc = 0.f;
  for (long k = (long)blockIdx.x * 256 + threadIdx.x; k < len; k += (long)gridDim.x * 256) {
    float x = a[(long)b * len + k];
    if (clamp_a) x = fminf(fmaxf(x, 0.f), 1.f);
    const float d = fsub_rn(x, b_[(long)b * len + k]);
    acc = fadd_rn(acc, fmul_rn(d, d));
  }
  const float r = block_sum_256(acc, sh);
  if (threadIdx.x == 0) part[(long)b * gridDim.x + blockIdx.x] = r;
}

// out = Up(Low(x_hat,0),1) (or x_hat) written NCHW from an nChw4c tensor with C = 3.
__global__ void nc4_bound_to_nchw_kernel(const float* __restrict__ x4, float* __restrict__ out, long HW, int clamp) {
  const int b = blockIdx.y;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 v = ld4(x4 + ((long)b * HW + pix) * 4);
#pragma unroll
    for (int c = 0; c < 3; ++c) out[((long)b * 3 + c) * HW + pix] = clamp ? fminf(fmaxf(v[c], 0.f), 1.f) : v[c];
  }
}

// g4 = bound01-backward(g (NCHW, dL/dout)) at x_hat4, in nChw4c (C = 3).
__global__ void bound_bwd_nc4_kernel(const float* __restrict__ x4, const float* __restrict__ g,
                                     float* __restrict__ g4, long HW, int clamp) {
  const int b = blockIdx.y;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 v = ld4(x4 + ((long)b * HW + pix) * 4);
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float gg = g[((long)b * 3 + c) * HW + pix];
      if (clamp) {
        const float xh = v[c], lo = fmaxf(xh, 0.f);
        gg = (lo <= 1.f || gg > 0.f) ? gg : gg * 0.f;
        gg = (xh >= 0.f || gg < 0.f) ? gg : gg * 0.f;
      }
      o[c] = gg;
    }
    st4(g4 + ((long)b * HW + pix) * 4, o);
  }
}

__global__ void clamp01_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = fminf(fmaxf(x[i], 0.f), 1.f);
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
static inline int grid_1d(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

extern "C" {

int ica_elem_blocks_per_image() { return ELEM_BLOCKS_PER_IMAGE; }

int ica_nchw_to_nc4(const float* src, float* dst, int N, int C, int H, int W, hipStream_t st) {
  const long total = (long)N * ((C + 3) / 4) * H * W;
  ICA_LAUNCH(nchw_to_nc4_kernel, dim3(grid_1d(total)), dim3(256), 0, st, src, dst, N, C, H, W);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_nc4_to_nchw(const float* src, float* dst, int N, int C, int H, int W, hipStream_t st) {
  const long total = (long)N * ((C + 3) / 4) * H * W;
  ICA_LAUNCH(nc4_to_nchw_kernel, dim3(grid_1d(total)), dim3(256), 0, st, src, dst, N, C, H, W);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_reduce_rows(const float* part, float* out, int B, int nblk, float scale, hipStream_t st) {
  ICA_LAUNCH(reduce_rows_kernel, dim3(B), dim3(256), 0, st, part, out, nblk, scale);
  ICA_CHECK_LAUNCH();
  return 0;
}

// part must hold B * ica_elem_blocks_per_image() floats.
int ica_attack_prologue_ex(const float* noise, const float* im_s, float* im_in4, float* part, int B, int H, int W,
                           float eps, int clamp_in, hipStream_t st) {
  ICA_LAUNCH(attack_prologue_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, noise, im_s, im_in4,
                     part, (long)H * W, eps, clamp_in);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_attack_prologue(const float* noise, const float* im_s, float* im_in4, float* part, int B, int H, int W,
                        float eps, hipStream_t st) {
  return ica_attack_prologue_ex(noise, im_s, im_in4, part, B, H, W, eps, 1, st);
}

int ica_attack_loss(const float* xhat4, const float* out_s, float* grad4, float* part, int B, int H, int W,
                    float invN, int clamp, int mode, hipStream_t st) {
  ICA_LAUNCH(attack_loss_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, xhat4, out_s, grad4, part,
                     (long)H * W, invN, clamp, mode);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_attack_adam_ex(float* noise, const float* im_s, const float* gnet4, const float* loss_i,
                       const float* cheap_grad, float* m, float* v, float* im_in_out, int B, int H, int W, float eps,
                       float thr, float invN, float bc2s, float neg_step, int* branch, const int* gpos, int* census,
                       int clamp_in, hipStream_t st) {
  ICA_LAUNCH(attack_adam_kernel<false>, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, noise, im_s, gnet4,
                     loss_i, cheap_grad, m, v, im_in_out, (long)H * W, eps, thr, invN, bc2s, neg_step, branch,
                     RoiBox{}, (long)W, gpos, census, clamp_in);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_attack_adam(float* noise, const float* im_s, const float* gnet4, const float* loss_i, const float* cheap_grad,
                    float* m, float* v, float* im_in_out, int B, int H, int W, float eps, float thr, float invN,
                    float bc2s, float neg_step, int* branch, const int* gpos, int* census, hipStream_t st) {
  return ica_attack_adam_ex(noise, im_s, gnet4, loss_i, cheap_grad, m, v, im_in_out, B, H, W, eps, thr, invN, bc2s,
                            neg_step, branch, gpos, census, 1, st);
}

int ica_roi_prologue(const float* noise, const float* im_s, float* im_in4, float* part, int B, int H, int W, float eps,
                     int x0, int x1, int y0, int y1, float w_in_tar, float w_in_bkg, hipStream_t st) {
  const RoiBox roi{x0, x1, y0, y1, w_in_tar, w_in_bkg, 0.f, 0.f};
  ICA_LAUNCH(roi_prologue_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, noise, im_s, im_in4, part,
                     (long)H * W, (long)W, eps, roi);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_roi_loss(const float* xhat4, const float* out_s, const float* out_t, float* grad4, float* part, int B, int H,
                 int W, int x0, int x1, int y0, int y1, float w_out_tar, float w_out_bkg, int clamp, hipStream_t st) {
  const RoiBox roi{x0, x1, y0, y1, 0.f, 0.f, w_out_tar, w_out_bkg};
  ICA_LAUNCH(roi_loss_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, xhat4, out_s, out_t, grad4,
                     part, (long)H * W, (long)W, roi, clamp);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_roi_adam(float* noise, const float* im_s, const float* gnet4, const float* loss_i, float* m, float* v,
                 float* im_in_out, int B, int H, int W, float eps, float thr, float bc2s, float neg_step, int* branch,
                 int x0, int x1, int y0, int y1, float w_in_tar, float w_in_bkg, const int* gpos, int* census,
                 hipStream_t st) {
  const RoiBox roi{x0, x1, y0, y1, w_in_tar, w_in_bkg, 0.f, 0.f};
  ICA_LAUNCH(attack_adam_kernel<true>, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, noise, im_s, gnet4,
                     loss_i, nullptr, m, v, im_in_out, (long)H * W, eps, thr, 0.f, bc2s, neg_step, branch, roi,
                     (long)W, gpos, census, 1);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_branch_select(const float* loss_i, float thr, int B, int* sel, int* gpos, hipStream_t st) {
  ICA_LAUNCH(branch_select_kernel, dim3(1), dim3(64), 0, st, loss_i, thr, B, sel, gpos);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_gather_images(const float* src, float* dst, const int* idx, int E, long floats_per_image, hipStream_t st) {
  if (E <= 0) return 0;
  if (floats_per_image % 4) return (int)hipErrorInvalidValue;
  const long quads = floats_per_image / 4;
  const int gx = (int)((quads + 255) / 256 < 1024 ? (quads + 255) / 256 : 1024);
  ICA_LAUNCH(gather_images_kernel, dim3(gx, E), dim3(256), 0, st, reinterpret_cast<const f32x4*>(src),
                     reinterpret_cast<f32x4*>(dst), idx, quads);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_ifgsm_step(float* x, const float* im_s, const float* grad4, float* gacc, const float* l1, int B, int H,
                   int W, float alpha, float eps, int momentum, hipStream_t st) {
  ICA_LAUNCH(ifgsm_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, x, im_s, grad4, gacc, l1,
                     (long)H * W, alpha, eps, momentum);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_l1_partial(const float* g4, float* part, int B, int H, int W, hipStream_t st) {
  ICA_LAUNCH(l1_partial_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, g4, part, (long)H * W);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_gc_likelihood(const float* y, const float* scales, const float* means, const float* qnoise, float* y_hat,
                      float* lik, float* part, int B, int C, int H, int W, int training, hipStream_t st) {
  const long per_image = 4L * ((C + 3) / 4) * H * W;
  ICA_LAUNCH(gc_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, y, scales, means, qnoise, y_hat,
                     lik, part, C, per_image, training);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_eb_likelihood(const float* z, const float* prm, const float* med, const float* qnoise, float* z_hat,
                      float* lik, float* part, int B, int C, int H, int W, int training, hipStream_t st) {
  const long per_image = 4L * ((C + 3) / 4) * H * W;
  ICA_LAUNCH(eb_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, z, prm, med, qnoise, z_hat, lik,
                     part, C, per_image, training);
  ICA_CHECK_LAUNCH();
  return 0;
}

// params: the 14 EntropyBottleneck tensors in order
// _matrix0.._matrix4, _bias0.._bias4, _factor0.._factor3, then quantiles [C][1][3].
int ica_pack_eb(const float* const* params, float* prm, float* med, int C, hipStream_t st) {
  const float* const* p = params;
  ICA_LAUNCH(pack_eb_kernel, dim3((C + 63) / 64), dim3(64), 0, st, p[0], p[1], p[2], p[3], p[4], p[5], p[6],
                     p[7], p[8], p[9], p[10], p[11], p[12], p[13], p[14], prm, med, C);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_round(const float* x, float* y, long n, hipStream_t st) {
  ICA_LAUNCH(round_kernel, dim3(grid_1d(n)), dim3(256), 0, st, x, y, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

// n must be a multiple of 4 (nChw4c tensors)
int ica_cast_f32_bf16(const float* x, void* y, long n, hipStream_t st) {
  if (n % 4) return -2;
  ICA_LAUNCH(cast_f32_bf16_kernel, dim3(grid_1d(n / 4)), dim3(256), 0, st, reinterpret_cast<const f32x4*>(x),
                     reinterpret_cast<u32x2*>(y), n / 4);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_cast_bf16_f32(const void* x, float* y, long n, hipStream_t st) {
  if (n % 4) return -2;
  ICA_LAUNCH(cast_bf16_f32_kernel, dim3(grid_1d(n / 4)), dim3(256), 0, st, reinterpret_cast<const u32x2*>(x),
                     reinterpret_cast<f32x4*>(y), n / 4);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_abs(const float* x, float* y, long n, hipStream_t st) {
  ICA_LAUNCH(abs_kernel, dim3(grid_1d(n)), dim3(256), 0, st, x, y, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_nc4_bound_to_nchw(const float* x4, float* out, int B, int H, int W, int clamp, hipStream_t st) {
  ICA_LAUNCH(nc4_bound_to_nchw_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, x4, out, (long)H * W,
                     clamp);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_bound_bwd_nc4(const float* x4, const float* g, float* g4, int B, int H, int W, int clamp, hipStream_t st) {
  ICA_LAUNCH(bound_bwd_nc4_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, x4, g, g4, (long)H * W,
                     clamp);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_clamp01(const float* x, float* y, long n, hipStream_t st) {
  ICA_LAUNCH(clamp01_kernel, dim3(grid_1d(n)), dim3(256), 0, st, x, y, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_sqdiff_partial(const float* a, const float* b, float* part, int B, long len, int clamp_a, hipStream_t st) {
  ICA_LAUNCH(sqdiff_partial_kernel, dim3(ELEM_BLOCKS_PER_IMAGE, B), dim3(256), 0, st, a, b, part, len,
                     clamp_a);
  ICA_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// Shared pieces of the implicit-GEMM conv kernels (ica_conv.hip: fp32 / bf16 operands; ica_conv_x6.hip:
// fp32-accurate bf16x6 operands): epilogue kinds, feature flags, the launch parameter block and the fused
// epilogues (bias / ReLU / leaky ReLU, GDN / IGDN forward and backward, residual / PixelShuffle extras).
// Reference anchors: anchors/utils.py:112-130 (conv / deconv geometry), utils/ops.py:58-97 (GDN).
#pragma once
#include "ica_common.h"

// A/B builds only (scripts/build_variant.sh): 1 = the conv_epilogue x6 GDN / IGDN forward with the fp32 path's IEEE
// 1/sqrtf / sqrtf instead of v_rsq_f32 / v_sqrt_f32 (the cheng2020 k3 kernels)
#ifndef ICA_X6_IEEE_GDN
#define ICA_X6_IEEE_GDN 0
#endif

enum {
  EPI_BIAS = 0,      // y = acc + bias
  EPI_RELU = 1,      // y = relu(acc + bias)
  EPI_GDN = 2,       // x = acc + bias; y = x * rsqrt(beta' + gamma' x^2)
  EPI_IGDN = 3,      // x = acc + bias; y = x * sqrt(beta' + gamma' x^2)
  EPI_GDN_BWD = 4,   // acc = dL/dy of a GDN; emit dL/dx  (needs saved y, s)
  EPI_IGDN_BWD = 5,  // same for IGDN
  EPI_LRELU = 6,     // y = leaky_relu(acc + bias, 0.01)
  EPI_LRELU_BWD = 7, // y = acc * (m > 0 ? 1 : 0.01), m = in_x (the saved leaky-ReLU output)
};
// Compile-time feature flags (template parameter FX) so that plain layers compile to plain code:
enum { FX_RES = 1, FX_PS = 2, FX_MASK = 4, FX_UNSHUF = 8, FX_T = 16 };  // FX_T: GDN-bwd writes save_t
// Optional extras (present only in FX-enabled instantiations; res / save_x may still be null there):
//   res      forward epilogues: y = act(...) + res (residual add after the activation);
//            GDN_BWD/IGDN_BWD: acc += res before the GDN backward (gradient of out = gdn + skip)
//   save_x   forward: the activation output before the residual add (GDN: y = x*s; LRELU: a);
//            GDN_BWD/IGDN_BWD: the summed upstream gradient acc + res (feeds the skip branch)
//   ps       (BIAS/RELU/LRELU) PixelShuffle(2) store: MFMA row rho = 16*c4 + 4*q + e is output
//            channel 4*c4 + e at sub-pixel q = 2i + j of the (2 Hout) x (2 Wout) output
//            (the host packs weights / bias in rho order)

struct ConvParams {
  const float* x;     // input  nChw4c [N][ceil(Cin/4)][Hin][Win][4]
  float* y;           // output nChw4c [N][ceil(Cout/4)][Hout][Wout][4]
  const float* wp;    // packed weight fragments (ica_pack_conv_weight)
  const float* bias;  // [Cout] or null
  const float* gp;    // packed gamma' fragments (fwd: gamma', bwd: gamma'^T)
  const float* beta;  // beta' [Cout] (fwd GDN epilogues)
  float* save_x;      // fwd GDN: pre-normalisation activation (optional)
  float* save_s;      // fwd GDN: s = rsqrt(n) | sqrt(n)           (optional)
  const float* in_x;  // bwd GDN: saved GDN OUTPUT y = x*s (x is recovered as y/s)
  const float* in_s;  // bwd GDN: saved s
  int N, Cin, Hin, Win, Cout, Hout, Wout;
  float* save_t;      // bwd GDN (training): dL/dn per element, for the GDN parameter gradients
  const float* res;   // optional residual (output layout), see above
  const float* mask;  // conv_down fill_mode 1: leaky-ReLU mask source (input layout)
  int fill_mode;      // conv_down: 0 plain, 1 x * lrelu'(mask), 2 PixelUnshuffle(2) view of x
  int ps;             // PixelShuffle(2) store (BIAS/RELU/LRELU epilogues)
  int prec;           // 0: fp32 operands (v_mfma_f32_32x32x2_f32, exact fp32 products)
                      // 1: bf16 operands, fp32 accumulate (v_mfma_f32_32x32x16_bf16); wp / gp hold the
                      //    bf16 packs (ica_pack_conv_weight_bf16 / ica_pack_gdn_bf16)
                      // 2: fp32-accurate bf16x6 operands (ica_conv_x6.hip; wp = ica_pack_conv_weight_x6, fp32
                      //    activations and epilogues, gp = the fp32 gamma' pack)
  int pl;             // parity-split pixel order (pix_at): PL_IN = x, PL_OUT = every output-layout tensor (y,
                      // save_x / save_s, in_x / in_s, save_t, res); x6 k5 s2 kernels and the x6 conv_up3 only
};
enum { PL_IN = 1, PL_OUT = 2 };

// v -> (hi, mid, lo) bf16 quads, each stage round-to-nearest-even on the residual (exact: hi + mid + lo == v)
ICA_DEV void split3(f32x4 v, u32x2& hi, u32x2& mid, u32x2& lo) {
  bf16x4 a, b, c;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 h = (__bf16)v[e];
    const float r1 = v[e] - (float)h;
    const __bf16 m = (__bf16)r1;
    const float r2 = r1 - (float)m;
    a[e] = h;
    b[e] = m;
    c[e] = (__bf16)r2;
  }
  hi = __builtin_bit_cast(u32x2, a);
  mid = __builtin_bit_cast(u32x2, b);
  lo = __builtin_bit_cast(u32x2, c);
}

// the six products of one 16-deep k step (small terms first)
ICA_DEV f32x16 mfma_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  c = mfma32bf(a[2], b[0], c);
  c = mfma32bf(a[0], b[2], c);
  c = mfma32bf(a[1], b[1], c);
  c = mfma32bf(a[1], b[0], c);
  c = mfma32bf(a[0], b[1], c);
  c = mfma32bf(a[0], b[0], c);
  return c;
}
// NPL planes: 3 = the six x6 products; 1 = the hi planes alone (bf16 operands, RNE)
template <int NPL>
ICA_DEV f32x16 mfma_np(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 c) {
  if constexpr (NPL == 1) return mfma32bf(a[0], b[0], c);
  else return mfma_x6(a, b, c);
}

// channels c0..c0+3 of a per-channel vector (bias, beta'): one 16-B buffer load, no branch.  A null vector gets a
// zero-range descriptor and reads 0; the range is rounded up to whole quads (a quad that straddles C is read whole,
// inside the allocation's 512-B granule) and callers mask channels >= Cout themselves.  (Element loads guarded by
// p.bias / c < Cout compiled to one branch + s_waitcnt vmcnt(0) per element: serialised L2 round trips that made
// the bias epilogue of a 1-wave/SIMD kernel cost ~20 us per block.)
ICA_DEV __amdgpu_buffer_rsrc_t chan_rsrc(const float* v, int C) { return uniform_rsrc(v, v ? (unsigned)((C + 3) & ~3) * 4u : 0u); }
ICA_DEV f32x4 ld_chan4(__amdgpu_buffer_rsrc_t r, int c0) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, c0 * 4, 0, 0));
}

// eight fp32 values (already in registers) -> the three bf16x8 planes of one MFMA operand
ICA_DEV void split3x8(const float (&v)[8], bf16x8 (&o)[3]) {
  u32x2 a0, b0, c0, a1, b1, c1;
  split3(f32x4{v[0], v[1], v[2], v[3]}, a0, b0, c0);
  split3(f32x4{v[4], v[5], v[6], v[7]}, a1, b1, c1);
  o[0] = __builtin_bit_cast(bf16x8, u32x4_t{a0[0], a0[1], a1[0], a1[1]});
  o[1] = __builtin_bit_cast(bf16x8, u32x4_t{b0[0], b0[1], b1[0], b1[1]});
  o[2] = __builtin_bit_cast(bf16x8, u32x4_t{c0[0], c0[1], c1[0], c1[1]});
}

// --------------------------------------------------------------------------
// Epilogue parameters in LDS (bf16 kernels).  vmcnt counts loads and stores together in issue order, so every
// bias / beta' / gamma' load an epilogue issues after one of its own stores waits for that store to complete:
// the bf16 conv_up epilogues (one parameter load per channel quad or normaliser tile between stores) ran as a
// chain of store round trips, ~20-40k cycles per class (phase stamps, scripts/exp/bf_trace.py).  The block copies
// the parameters into LDS once, next to its patch fill; the epilogue then reads them with ds_read (lgkmcnt), which
// never waits on a store.  Layout in 16-B entries: [0, 8 IT) bias quads of channels co_base.., [8 IT, 16 IT)
// beta' quads (GDN / IGDN forward), then the bf16 gamma' (forward) / gamma'^T (backward) hi fragments,
// entry k * 64 + lane for k = (a * IT + b) * 2 + s (the global pack's 1-KB piece at byte k * 2048).
// --------------------------------------------------------------------------
template <int EPI>
constexpr bool epi_gdn() { return EPI == EPI_GDN || EPI == EPI_IGDN || EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD; }
template <int IT, int EPI>
constexpr int epi_lds_entries() { return 16 * IT + (epi_gdn<EPI>() ? IT * IT * 128 : 0); }

template <int IT, int EPI>
ICA_DEV void epi_params_to_lds(const ConvParams& p, f32x4* lp, int co_base) {
  constexpr int NG = epi_gdn<EPI>() ? IT * IT * 128 : 0, NP = 16 * IT;
  constexpr int NI = (NP + NG + 255) / 256;
  const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout);
  const __amdgpu_buffer_rsrc_t ers = chan_rsrc((EPI == EPI_GDN || EPI == EPI_IGDN) ? p.beta : nullptr, p.Cout);
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(epi_gdn<EPI>() ? p.gp : nullptr, epi_gdn<EPI>() ? IT * IT * 4096 : 0);
  f32x4 v[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (e < 8 * IT) v[i] = ld_chan4(brs, co_base + 4 * e);
    else if (e < NP) v[i] = ld_chan4(ers, 4 * (e - 8 * IT));
    else if (e < NP + NG) {   // gamma' pieces: byte (k * 2048 + l * 16) < IT * IT * 4096
      const int k = (e - NP) >> 6, l = (e - NP) & 63;
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(grs, k * 2048 + l * 16, 0, 0));
    } else {
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (e < NP + NG) lp[e] = v[i];
  }
}

// pixel (y, x) of an H x W activation plane -> its pixel index: row-major, or parity-split (split: the four
// (y & 1, x & 1) sub-planes of (H/2) x (W/2) pixels one after another, H and W even; ConvParams::pl).  A conv_up
// parity class then owns a dense sub-plane, so its 16-B stores (and the GDN-backward epilogue's saved (y, s) loads)
// fill whole cache lines instead of every other 16 B of each line
ICA_DEV unsigned pix_at(int y, int x, int H, int W, bool split) {
  return split ? ((unsigned)((((y & 1) << 1) | (x & 1)) * (H >> 1) + (y >> 1))) * (unsigned)(W >> 1) + (x >> 1)
               : (unsigned)y * W + x;
}

// --------------------------------------------------------------------------
// Epilogue: acc[it] holds channels co_base + it*32 + acc_row(r,h) of pixel
// (n, oy, ox) for this lane.  Register quad g (r = 4g..4g+3) of tile it is one
// float4 of channel group c4 = co_base/4 + it*8 + 2g + h.
// --------------------------------------------------------------------------
// X6 (fp32 operands only): the GDN / IGDN normaliser GEMMs run as bf16x6 MFMAs on the split x^2 / t values and
// the three-plane gamma' pack of ica_pack_gdn_x6 (p.gp).  X6 = 1 ("wide", for 1-wave/SIMD kernels with the whole
// register file): all IT output tiles at once, gamma' fragments one round ahead; X6 = 2 ("narrow", for kernels
// at 2 waves/SIMD, 256 registers): one output tile at a time, the other wave hides the fragment latency.
// the three-plane gamma' pack of ica_pack_gdn_x6 (p.gp), fp32-accurate like the main loop of the x6 kernels.
// LG: the epilogue parameters come from the block's epi_params_to_lds copy at lp (bf16 kernels); otherwise from
// global memory
// EAG (bf16 GDN backward): 1 = every (y, s) quad loaded before the first use (conv_down: igdn_bwd 2.17 -> 2.07 ms,
// RGB igdn_bwd 2.01 -> 1.60 ms at the config-5 shapes); 2 = a two-channel-tile ring (32 registers: channel tile
// it + 2's quads issued once tile it's are consumed), for conv_up at 252 registers, where the whole set measured
// 3.43 -> 3.63 ms and loads beside their use compiled to one s_waitcnt vmcnt(0) per quad pair (16 HBM round trips
// per tile, ~28k cycles per tile stamped at the config-5 shapes); 0 = beside their use
template <int IT, int EPI, int FX, bool BF = false, int X6 = 0, bool LG = false, int EAG = 1>
ICA_DEV void conv_epilogue(const ConvParams& p, f32x16 (&acc)[IT], int n, int oy, int ox,
                           bool valid, int co_base, const f32x4* lp = nullptr, float* lst = nullptr) {
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int C4o = (p.Cout + 3) >> 2;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const unsigned pix = valid ? pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u;
  const size_t img = (size_t)C4o * plane;  // channel quads per image of every output-layout tensor
  // channel group c4 = u + h (u = co_base/4 + it*8 + 2g, wave-uniform): quad offset = vo + so(u)
  // (BF: every activation tensor of the epilogue is bf16 nChw4c, Img4T<true>)
  using Img = Img4T<BF>;
  const unsigned vo = h * plane + pix;
  auto so = [&](int u) -> unsigned { return (unsigned)u * plane; };
  const int cu = co_base >> 2;

  if constexpr (EPI == EPI_BIAS || EPI == EPI_RELU || EPI == EPI_LRELU) {
    const Img Y(p.y, img, n);
    // PixelShuffle(2) store: output tensor [N][Cout/16][2 Hout][2 Wout][4]; rho-row quad (it, g, h) is
    // channel group c4 = (cu + it*8 + 2g) / 4 at sub-pixel q = 2(g&1) + h of the (2Hout)x(2Wout) plane
    const unsigned plane2 = 4u * plane;
    const unsigned vo_ps = valid ? ((unsigned)(2 * oy) * (2 * p.Wout) + 2 * ox + h) : 0u;
    auto so_ps = [&](int it, int g) -> unsigned {
      const int c4 = (cu + it * 8 + 2 * g) >> 2;
      return (unsigned)c4 * plane2 + (unsigned)(g & 1) * (2 * p.Wout);
    };
    // (the shuffled tensor holds the same Cout * Hout * Wout floats per image as the plain one)
    const Img SX((FX & FX_RES) ? p.save_x : nullptr, img, n);
    const Img RS((FX & FX_RES) ? p.res : nullptr, img, n);
    const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout);
    // x6 kernels (1 wave/SIMD, registers to spare): every bias quad loaded before the first store (a load issued
    // after a store waits for it: vmcnt is in order)
    constexpr bool PRE = X6 != 0 && !LG;
    f32x4 bvs[PRE ? IT : 1][4];
    if constexpr (PRE) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) bvs[it][g] = ld_chan4(brs, co_base + it * 32 + 8 * g + 4 * h);
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = co_base + it * 32 + 8 * g + 4 * h;
        const f32x4 bv = LG ? lp[it * 8 + 2 * g + h] : PRE ? bvs[PRE ? it : 0][g] : ld_chan4(brs, c0);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = c0 + e < p.Cout ? acc[it][4 * g + e] + bv[e] : 0.f;
          if constexpr (EPI == EPI_RELU) t = fmaxf(t, 0.f);
          if constexpr (EPI == EPI_LRELU) t = t > 0.f ? t : t * 0.01f;
          v[e] = t;
        }
        if (valid && c0 < p.Cout) {
          unsigned vv, ss;
          if constexpr ((FX & FX_PS) != 0) {
            vv = vo_ps;
            ss = so_ps(it, g);
          } else {
            vv = vo;
            ss = so(cu + it * 8 + 2 * g);
          }
          if constexpr ((FX & FX_RES) != 0) {
            if (p.save_x) SX.st(vv, ss, v);
            if (p.res) {
              const f32x4 r = RS.ld(vv, ss);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += r[e];
            }
          }
          Y.st(vv, ss, v);
        }
      }
    }
  } else if constexpr (EPI == EPI_LRELU_BWD) {
    const Img Y(p.y, img, n), M(p.in_x, img, n);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c0 = co_base + it * 32 + 8 * g + 4 * h;
        if (c0 >= p.Cout || !valid) continue;
        const unsigned ss = so(cu + it * 8 + 2 * g);
        const f32x4 m = M.ld(vo, ss);
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float t = acc[it][4 * g + e];
          v[e] = (c0 + e < p.Cout) ? (m[e] > 0.f ? t : t * 0.01f) : 0.f;
        }
        Y.st(vo, ss, v);
      }
    }
  } else if constexpr (EPI == EPI_GDN || EPI == EPI_IGDN) {
    // requires IT*32 == Cout, co_base == 0.  acc := x = conv + bias (kept intact
    // until every normaliser tile is done); one 32-channel tile of
    // n = beta' + gamma' x^2 at a time (16 accumulator registers live).
    const Img Y(p.y, img, n), SS(p.save_s, img, n);
    const Img SX((FX & FX_RES) ? p.save_x : nullptr, img, n), RS((FX & FX_RES) ? p.res : nullptr, img, n);
    const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout), ers = chan_rsrc(p.beta, p.Cout);
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bv = LG ? lp[it * 8 + 2 * g + h] : ld_chan4(brs, it * 32 + 8 * g + 4 * h);   // channels acc_row(4g + e, h)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += bv[e];
      }
    // bf16 path: x^2 (rounded to bf16) as the B operand of a bf16 GEMM with gamma' (its bf16 hi part; one
    // MFMA per k-step); the accumulator registers 8s..8s+7 of tile it are k-step s (pack_gdn_bf16_kernel gives
    // the matching gamma' order).  n = beta' + sum of non-negative terms then carries <= 2^-8 relative error,
    // s and y half of it: the size of the bf16 rounding of the stored y and s.
    bf16x8 xh[BF ? IT : 1][2];
    // x6: every normaliser tile at once.  Round k = (k-tile it, k-step s) splits x^2 of accumulator registers
    // 8s..8s+7 of tile it (fp32 square, exact 3-way split; the per-lane order of the fp32 gamma' pack that
    // ica_pack_gdn_x6 splits, plane stride IT*IT*2048 bytes) and feeds all IT output tiles; the gamma' fragments
    // of round k+1 are issued before round k's MFMAs (4 independent accumulation chains hide their latency).
    const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, X6 ? IT * IT * 6144 : IT * IT * 4096);
    // narrow x6: x^2 of every (tile, k-step) split into its three planes once, before the output tiles (the split
    // per output tile and k-step repeated it IT times: ~1.4k VALU instructions per tile at IT = 4)
    bf16x8 xs2[X6 == 2 ? IT : 1][2][3];
    if constexpr (X6 == 2) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          float v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = acc[it][8 * s + j] * acc[it][8 * s + j];
          split3x8(v, xs2[it][s]);
        }
    }
    f32x16 nx[X6 == 1 ? IT : 1];
    if constexpr (X6 == 1) {
      static_assert(!BF, "x6 epilogue: fp32 activations");
#pragma unroll
      for (int ct = 0; ct < IT; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 ev = ld_chan4(ers, ct * 32 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) nx[ct][4 * g + e] = ev[e];
        }
      bf16x8 ga[2][IT][3];
      auto ldg = [&](bf16x8 (&a)[IT][3], int k) {
#pragma unroll
        for (int ct = 0; ct < IT; ++ct)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            a[ct][q] = ld_bf8(grs, lane * 16, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
      };
      ldg(ga[0], 0);
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
        __builtin_amdgcn_sched_barrier(0);
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[k >> 1][8 * (k & 1) + j] * acc[k >> 1][8 * (k & 1) + j];
        bf16x8 xq[3];
        split3x8(v, xq);
#pragma unroll
        for (int ct = 0; ct < IT; ++ct) nx[ct] = mfma_x6(ga[k & 1][ct], xq, nx[ct]);
      }
    }
    if constexpr (BF) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float xv = acc[it][8 * s + j];
            xh[it][s][j] = (__bf16)(xv * xv);
          }
    }
#pragma unroll
    for (int ct = 0; ct < IT; ++ct) {
      // LDS parameters: one normaliser tile per scheduling region (hoisting every tile's gamma' reads spilled)
      if constexpr (LG) __builtin_amdgcn_sched_barrier(0);
      f32x16 nacc;
      if constexpr (X6 == 1) {
        nacc = nx[ct];
      } else {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 ev = LG ? lp[8 * IT + ct * 8 + 2 * g + h] : ld_chan4(ers, ct * 32 + 8 * g + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) nacc[4 * g + e] = ev[e];
        }
      }
      if constexpr (X6 == 2) {
        // narrow x6: the output tile's gamma' fragments in two bursts of IT*3 (left to itself the scheduler loaded
        // each next to its MFMA and waited out a full L2 round trip per fragment), x^2 split per k-step
        static_assert(X6 != 2 || IT % 2 == 0, "narrow x6 epilogue: even IT");
#pragma unroll
        for (int hb = 0; hb < 2; ++hb) {
          bf16x8 ga[IT / 2][2][3];
#pragma unroll
          for (int i2 = 0; i2 < IT / 2; ++i2)
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
              for (int q = 0; q < 3; ++q)
                ga[i2][s][q] = ld_bf8(grs, lane * 16,
                                      ((ct * IT + hb * (IT / 2) + i2) * 2 + s) * 1024 + q * IT * IT * 2048);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i2 = 0; i2 < IT / 2; ++i2)
#pragma unroll
            for (int s = 0; s < 2; ++s) nacc = mfma_x6(ga[i2][s], xs2[hb * (IT / 2) + i2][s], nacc);
        }
      }
#pragma unroll
      for (int it = 0; it < (X6 ? 0 : IT); ++it) {
        if constexpr (BF) {
          const int o = (ct * IT + it) * 4096, k0 = (ct * IT + it) * 2;
#pragma unroll
          for (int s = 0; s < 2; ++s)
            nacc = mfma32bf(LG ? f4_as_bf8(lp[16 * IT + (k0 + s) * 64 + lane]) : ld_bf8(grs, lane * 16, o + s * 2048),
                            xh[it][s], nacc);
        } else {
          const float* gq = p.gp + ((size_t)(ct * IT + it) * 64 + lane) * 16;
          const f32x4 g0 = ld4(gq), g1 = ld4(gq + 4), g2 = ld4(gq + 8), g3 = ld4(gq + 12);
          const float ga[16] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3],
                                g2[0], g2[1], g2[2], g2[3], g3[0], g3[1], g3[2], g3[3]};
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float xv = acc[it][r];
            nacc = mfma32(ga[r], xv * xv, nacc);
          }
        }
      }
      if (valid) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 yv, sv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float nv = nacc[4 * g + e];
            // bf16 path: v_rsq_f32 / v_sqrt_f32 (1 ulp; n >= beta' > 0), no IEEE division / sqrt fix-ups
            float s;
            // x6: the same 1-ulp instructions (1/sqrtf rounds twice, so the IEEE form is no closer; measured
            // 8-10k cycles per conv_up class of IEEE sqrt fix-ups)
            if constexpr (BF || (X6 && !ICA_X6_IEEE_GDN)) s = (EPI == EPI_GDN) ? __builtin_amdgcn_rsqf(nv) : __builtin_amdgcn_sqrtf(nv);
            else s = (EPI == EPI_GDN) ? (1.0f / sqrtf(nv)) : sqrtf(nv);
            sv[e] = s;
            yv[e] = acc[ct][4 * g + e] * s;
          }
          const unsigned ss = so(ct * 8 + 2 * g);
          if (p.save_s) SS.st(vo, ss, sv);
          if constexpr ((FX & FX_RES) != 0) {
            if (p.save_x) SX.st(vo, ss, yv);
            if (p.res) {
              const f32x4 r = RS.ld(vo, ss);
#pragma unroll
              for (int e = 0; e < 4; ++e) yv[e] += r[e];
            }
          }
          Y.st(vo, ss, yv);
        }
      }
    }
  } else {  // EPI_GDN_BWD / EPI_IGDN_BWD, requires IT*32 == Cout
    // acc = g = dL/dy.  t = (g x) dS/dn (GDN: -0.5 s^3, IGDN: 0.5/s) for all
    // channel tiles, then per output tile jt: u = gamma'^T t (16 live
    // accumulators) and dx = g s + 2 x u with x, s re-read (L2-hot).
    // Residual gradient: added unconditionally (r = 0 without one) so that the accumulators are
    // never live in two versions across a branch (that doubled the register footprint).
    const Img Y(p.y, img, n), IX(p.in_x, img, n), IS(p.in_s, img, n);
    if constexpr (BF) {
      // bf16 path (FX == 0): ONE pass over the saved (y, s) — the second read of them was the epilogue's latency
      // cost at 2 waves/SIMD (IT = 6, the C = 192 layers: one wave per SIMD, the whole register file).  Per element: t (-> a bf16 B fragment), g*s in place of g,
      // and 2x = 2 y rcp(s) kept as bf16 (the saved y and s are bf16 already); then per output tile
      // u = gamma'^T t (bf16 MFMAs, gamma' hi part) and dx = g s + 2x u, stores only.  t, gamma' and 2x rounded
      // to bf16 add 2^-9-relative errors, the size of the bf16 storage of y and s.
      static_assert(!BF || FX == 0, "bf16 GDN-bwd epilogue: plain layers");
      bf16x8 th[IT][2];
      u32x2 x2q[IT][4];
      // unconditional loads (one basic block, all in flight): a pixel outside the output reads past the
      // descriptor's range (returns 0); its MFMA column (lanes j, j+32 = one pixel) is never stored
      const unsigned vo_ld = valid ? vo : 0x1FFFFFF0u;
      __builtin_amdgcn_sched_barrier(0);  // not into the main loop (its weight ring is live there)
      // EAG: every (y, s) quad of the tile in flight before the first use (raw 8-B bf16 quads: 64 registers at IT = 4)
      u32x2 yq[EAG == 1 ? IT : 1][4], sq[EAG == 1 ? IT : 1][4];
      u32x2 ry[EAG == 2 ? 2 : 1][4], rq[EAG == 2 ? 2 : 1][4];   // EAG 2: the two-tile ring
      auto ring_ld = [&](int it) {
        if constexpr (EAG == 2) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int so8 = (int)(so(it * 8 + 2 * g) * 8u);
            ry[it & 1][g] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(IX.r, (int)(vo_ld * 8u), so8, 0));
            rq[it & 1][g] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(IS.r, (int)(vo_ld * 8u), so8, 0));
          }
        }
      };
      if constexpr (EAG == 2) {
        ring_ld(0);
        if (IT > 1) ring_ld(1);
      }
      if constexpr (EAG == 1) {
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int so8 = (int)(so(it * 8 + 2 * g) * 8u);
            yq[it][g] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(IX.r, (int)(vo_ld * 8u), so8, 0));
            sq[it][g] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(IS.r, (int)(vo_ld * 8u), so8, 0));
          }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const unsigned ss = so(it * 8 + 2 * g);
          const f32x4 yv = EAG == 1 ? bf4_to_f4(yq[EAG == 1 ? it : 0][g])
                         : EAG == 2 ? bf4_to_f4(ry[EAG == 2 ? (it & 1) : 0][g]) : IX.ld(vo_ld, ss);
          const f32x4 sv = EAG == 1 ? bf4_to_f4(sq[EAG == 1 ? it : 0][g])
                         : EAG == 2 ? bf4_to_f4(rq[EAG == 2 ? (it & 1) : 0][g]) : IS.ld(vo_ld, ss);
          f32x4 x2;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float gg = acc[it][4 * g + e], sg = sv[e], yg = yv[e];
            const float r = __builtin_amdgcn_rcpf(sg);
            const float t = (EPI == EPI_GDN_BWD) ? (-0.5f * (gg * yg)) * (sg * sg) : (0.5f * (gg * yg)) * (r * r);
            th[it][g >> 1][4 * (g & 1) + e] = (__bf16)t;
            float gs = gg * sg;
            asm volatile("" : "+v"(gs));  // materialise here: LLVM otherwise sinks g*s and y*rcp(s) into the
            acc[it][4 * g + e] = gs;      // stores after the GEMM, keeping g, s, y, r live (spills)
            x2[e] = 2.0f * (yg * r);
          }
          u32x2 q = f4_to_bf4(x2);
          asm volatile("" : "+v"(q));
          x2q[it][g] = q;
        }
        if constexpr (EAG == 2) {
          if (it + 2 < IT) ring_ld(it + 2);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // pack 2x here, do not sink y and rcp(s) into the second phase
      const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 4096);
#pragma unroll
      for (int jt = 0; jt < IT; ++jt) {
        // keep each output tile's gamma'^T fragment loads inside its tile (hoisting all of them spilled)
        __builtin_amdgcn_sched_barrier(0);
        f32x16 uacc = f32x16{0};
#pragma unroll
        for (int ct = 0; ct < IT; ++ct) {
          const int o = (jt * IT + ct) * 4096, k0 = (jt * IT + ct) * 2;
#pragma unroll
          for (int s = 0; s < 2; ++s)
            uacc = mfma32bf(LG ? f4_as_bf8(lp[16 * IT + (k0 + s) * 64 + lane]) : ld_bf8(grs, lane * 16, o + s * 2048),
                            th[ct][s], uacc);
        }
        if (valid) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 x2 = bf4_to_f4(x2q[jt][g]);
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[jt][4 * g + e] + x2[e] * uacc[4 * g + e];
            Y.st(vo, so(jt * 8 + 2 * g), v);
          }
        }
      }
    } else if constexpr (FX == 0 && IT <= 4) {
      // fp32, plain layers: one pass over the saved (y, s) as well.  x = y / s, t and g*s are formed with the
      // ops of the two-pass form below and kept in registers (gs in place of g), so dx needs no second read.
      f32x16 tt[X6 == 1 ? 1 : IT], xx[IT];
      bf16x8 tq[X6 == 1 ? IT : 1][2][3];   // wide x6: t split into three planes (k-step s = registers 8s..8s+7)
      const unsigned vo_ld = valid ? vo : 0x0FFFFFF0u;  // past the descriptor's range: loads return 0
      float tw[8];   // x6: t of register quads g = 2k, 2k+1 (one k-step) before the split
      __builtin_amdgcn_sched_barrier(0);
      // x6 (1 wave/SIMD): every (y, s) load of the tile in flight before the first use (left to itself the
      // scheduler issued them two at a time, each pair behind an s_waitcnt vmcnt(0): 16 serialised HBM round
      // trips per tile, ~35k cycles per conv_up class); the registers pass to t / 2x as the loads are consumed.
      // The fp32 kernels run 2 waves/SIMD (the other wave covers the latency; the 128 registers would spill).
      f32x4 yq[X6 ? IT : 1][4], sq[X6 ? IT : 1][4];
      if constexpr (X6 != 0) {
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            yq[it][g] = IX.ld(vo_ld, so(it * 8 + 2 * g));
            sq[it][g] = IS.ld(vo_ld, so(it * 8 + 2 * g));
          }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const unsigned ss = so(it * 8 + 2 * g);
          const f32x4 yv = X6 ? yq[X6 ? it : 0][g] : IX.ld(vo_ld, ss), sv = X6 ? sq[X6 ? it : 0][g] : IS.ld(vo_ld, ss);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            // x6: one v_rcp_f32 (1 ulp) replaces the two IEEE divisions (measured 2.7% on up.gdn_bwd)
            const float sg = sv[e], rs = X6 ? __builtin_amdgcn_rcpf(sg) : 0.f;
            const float xs = X6 ? yv[e] * rs : yv[e] / sg;
            const float gx = acc[it][4 * g + e] * xs;
            const float tv = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (sg * sg * sg)
                                                  : (X6 ? (0.5f * gx) * rs : gx / (2.0f * sg));
            if constexpr (X6 == 1) tw[4 * (g & 1) + e] = tv;
            else tt[it][4 * g + e] = tv;
            float gs = acc[it][4 * g + e] * sg;
            float x2 = 2.0f * xs;
            asm volatile("" : "+v"(gs), "+v"(x2));  // materialise (see the bf16 branch)
            acc[it][4 * g + e] = gs;
            xx[it][4 * g + e] = x2;
          }
          if constexpr (X6 == 1) {
            if (g & 1) split3x8(tw, tq[it][g >> 1]);
          }
          if constexpr (X6 == 2) {
            // narrow x6 (256 registers): g*s parked in the output (same-thread write, re-read at the end) so the
            // accumulator tiles are dead during the u GEMM
            if (valid) Y.st(vo, ss, f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]});
          }
        }
      __builtin_amdgcn_sched_barrier(0);
      // x6: u for every output tile at once; round k = (k-tile ct, k-step s) feeds all IT accumulators, the
      // gamma'^T fragments of round k+1 issued before round k's MFMAs (as in the forward GDN epilogue)
      f32x16 ux[X6 == 1 ? IT : 1];
      bf16x8 gn[X6 == 2 ? IT / 2 : 1][2][3];   // narrow x6: half an output tile's gamma'^T fragments
      if constexpr (X6 == 1) {
        const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
#pragma unroll
        for (int jt = 0; jt < IT; ++jt) ux[jt] = f32x16{0};
        bf16x8 ga[2][IT][3];
        auto ldg = [&](bf16x8 (&a)[IT][3], int k) {
#pragma unroll
          for (int jt = 0; jt < IT; ++jt)
#pragma unroll
            for (int q = 0; q < 3; ++q)
              a[jt][q] = ld_bf8(grs, lane * 16, (((jt * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
        };
        ldg(ga[0], 0);
#pragma unroll
        for (int k = 0; k < 2 * IT; ++k) {
          if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int jt = 0; jt < IT; ++jt) ux[jt] = mfma_x6(ga[k & 1][jt], tq[k >> 1][k & 1], ux[jt]);
        }
      }
#pragma unroll
      for (int jt = 0; jt < IT; ++jt) {
        __builtin_amdgcn_sched_barrier(0);
        f32x16 uacc = f32x16{0};
#pragma unroll
        for (int ct = 0; ct < IT; ++ct) {
          if constexpr (X6 == 1) {
            if (ct == 0) uacc = ux[jt];
          } else if constexpr (X6 == 2) {
            // narrow x6: the output tile's fragments in one burst at ct == 0 (see the forward epilogue), t of tile
            // ct split per k-step on the fly (no 96-register three-plane copy)
            if (ct % (IT / 2) == 0) {   // two bursts of IT*3 fragments per output tile
              const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
#pragma unroll
              for (int c2 = 0; c2 < IT / 2; ++c2)
#pragma unroll
                for (int s = 0; s < 2; ++s)
#pragma unroll
                  for (int q = 0; q < 3; ++q)
                    gn[c2][s][q] = ld_bf8(grs, lane * 16, ((jt * IT + ct + c2) * 2 + s) * 1024 + q * IT * IT * 2048);
              __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
              float v[8];
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = tt[ct][8 * s + e];
              bf16x8 tq2[3];
              split3x8(v, tq2);
              uacc = mfma_x6(gn[ct % (IT / 2)][s], tq2, uacc);
            }
          } else {
            const float* gq = p.gp + ((size_t)(jt * IT + ct) * 64 + lane) * 16;
            const f32x4 g0 = ld4(gq), g1 = ld4(gq + 4), g2 = ld4(gq + 8), g3 = ld4(gq + 12);
            const float ga[16] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3],
                                  g2[0], g2[1], g2[2], g2[3], g3[0], g3[1], g3[2], g3[3]};
#pragma unroll
            for (int r = 0; r < 16; ++r) uacc = mfma32(ga[r], tt[ct][r], uacc);
          }
        }
        if (valid) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            f32x4 v;
            const f32x4 gs = X6 == 2 ? Y.ld(vo, so(jt * 8 + 2 * g)) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              v[e] = (X6 == 2 ? gs[e] : acc[jt][4 * g + e]) + xx[jt][4 * g + e] * uacc[4 * g + e];
            Y.st(vo, so(jt * 8 + 2 * g), v);
          }
        }
      }
    } else if constexpr (X6 == 1) {
      // x6 with a residual gradient and / or C = 192 (the cheng2020 k3 s1 kernels, 1 wave/SIMD): ONE pass over the
      // saved (y, s) like the plain branch above.  g*s is parked in this wave's LDS slab lst (IT*16 floats per
      // lane: the kernel's patch, idle after its main loop), 2x replaces g in the accumulators and t goes straight
      // into its three bf16 planes; u = gamma'^T t runs in two halves of IT/2 output tiles (fragments a round
      // ahead), so neither y, s nor a parked g*s is read twice from memory.  Same per-element ops as the fp32 form.
      static_assert(!BF && (FX & ~FX_RES) == 0 && IT % 2 == 0, "x6 GDN-bwd epilogue: residual view, even IT");
      const unsigned vo_ld = valid ? vo : 0x0FFFFFF0u;   // past the descriptor's range: loads return 0
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((FX & FX_RES) != 0) {
        const Img SX(p.save_x, p.save_x ? img : 0, n), RS(p.res, p.res ? img : 0, n);   // absent: zero-size range
        f32x4 rq[IT][4];
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int g = 0; g < 4; ++g) rq[it][g] = RS.ld(vo_ld, so(it * 8 + 2 * g));
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += rq[it][g][e];
            if (p.save_x && valid)
              SX.st(vo, so(it * 8 + 2 * g),
                    f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]});
          }
        __builtin_amdgcn_sched_barrier(0);
      }
      f32x4 yq[IT][4], sq[IT][4];
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          yq[it][g] = IX.ld(vo_ld, so(it * 8 + 2 * g));
          sq[it][g] = IS.ld(vo_ld, so(it * 8 + 2 * g));
        }
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 tq[IT][2][3];
      float tw[8];
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sg = sq[it][g][e], xs = yq[it][g][e] / sg;
            const float gx = acc[it][4 * g + e] * xs;
            tw[4 * (g & 1) + e] = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (sg * sg * sg) : gx / (2.0f * sg);
            float gs = acc[it][4 * g + e] * sg;
            float x2 = 2.0f * xs;
            asm volatile("" : "+v"(gs), "+v"(x2));   // materialise (see the bf16 branch)
            lst[((it * 4 + g) * 4 + e) * 64 + lane] = gs;
            acc[it][4 * g + e] = x2;
          }
          if (g & 1) split3x8(tw, tq[it][g >> 1]);
        }
      __builtin_amdgcn_sched_barrier(0);
      const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
      constexpr int H2 = IT / 2;
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        f32x16 ux[H2];
#pragma unroll
        for (int j = 0; j < H2; ++j) ux[j] = f32x16{0};
        bf16x8 ga[2][H2][3];
        auto ldg = [&](bf16x8 (&a)[H2][3], int k) {
#pragma unroll
          for (int j = 0; j < H2; ++j)
#pragma unroll
            for (int q = 0; q < 3; ++q)
              a[j][q] = ld_bf8(grs, lane * 16,
                               ((((hb * H2 + j) * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
        };
        ldg(ga[0], 0);
#pragma unroll
        for (int k = 0; k < 2 * IT; ++k) {
          if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int j = 0; j < H2; ++j) ux[j] = mfma_x6(ga[k & 1][j], tq[k >> 1][k & 1], ux[j]);
        }
        if (valid) {
#pragma unroll
          for (int j = 0; j < H2; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int jt = hb * H2 + j;
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e)
                v[e] = lst[((jt * 4 + g) * 4 + e) * 64 + lane] + acc[jt][4 * g + e] * ux[j][4 * g + e];
              Y.st(vo, so(jt * 8 + 2 * g), v);
            }
        }
      }
    } else {
      static_assert(!X6, "x6 GDN-bwd epilogue: the single-pass branches above");
      if constexpr ((FX & FX_RES) != 0) {
        const Img SX(p.save_x, img, n), RS(p.res, img, n);
  #pragma unroll
        for (int it = 0; it < IT; ++it)
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            const unsigned ss = so(it * 8 + 2 * g);
            f32x4 r = {0.f, 0.f, 0.f, 0.f};
            if (p.res && valid) r = RS.ld(vo, ss);
  #pragma unroll
            for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += r[e];
            if (p.save_x && valid)
              SX.st(vo, ss, f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]});
          }
      }
      // IT > 4 (C = 192): g*s is parked in the output (same-thread global write, re-read below) so that
      // the 6 accumulator tiles are dead while the 6 t tiles and the u GEMM are live.
      constexpr bool STASH = IT > 4;
      if constexpr (STASH) {
        if (valid) {
  #pragma unroll
          for (int it = 0; it < IT; ++it)
  #pragma unroll
            for (int g = 0; g < 4; ++g) {
              const unsigned ss = so(it * 8 + 2 * g);
              const f32x4 sv = IS.ld(vo, ss);
              Y.st(vo, ss, f32x4{acc[it][4 * g] * sv[0], acc[it][4 * g + 1] * sv[1], acc[it][4 * g + 2] * sv[2],
                                 acc[it][4 * g + 3] * sv[3]});
            }
        }
      }
      // t = (g x) dS/dn with x = y / s (in_x holds the GDN output y).  fp32 path: IEEE divisions, the op order
      // the parity tests were pinned with.  bf16 path: GDN -0.5 g y s^2, IGDN 0.5 g y rcp(s)^2 (v_rcp_f32; the
      // epilogue was VALU-bound on division sequences), and t goes straight into its hi/lo B fragments
      // (register r = 4g+e is k-step r>>3, element r&7), no fp32 copy kept.
      f32x16 tt[BF ? 1 : IT];
      bf16x8 th[BF ? IT : 1][2], tl[BF ? IT : 1][2];
      const Img ST((FX & FX_T) ? p.save_t : nullptr, img, n);
  #pragma unroll
      for (int it = 0; it < IT; ++it)
  #pragma unroll
        for (int g = 0; g < 4; ++g) {
          const unsigned ss = so(it * 8 + 2 * g);
          f32x4 xv = {0.f, 0.f, 0.f, 0.f}, sv = {1.f, 1.f, 1.f, 1.f};
          if (valid) {
            xv = IX.ld(vo, ss);
            sv = IS.ld(vo, ss);
          }
          f32x4 tv;
  #pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float s = sv[e];
            float t;
            if constexpr (!BF) {
              const float gx = acc[it][4 * g + e] * (xv[e] / s);
              t = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (s * s * s) : gx / (2.0f * s);
            } else if constexpr (EPI == EPI_GDN_BWD) {
              t = (-0.5f * (acc[it][4 * g + e] * xv[e])) * (s * s);
            } else {
              const float r = __builtin_amdgcn_rcpf(s);
              t = (0.5f * (acc[it][4 * g + e] * xv[e])) * (r * r);
            }
            tv[e] = t;
            if constexpr (BF) {
              __bf16 hi, lo;
              split_bf(t, hi, lo);
              th[it][g >> 1][4 * (g & 1) + e] = hi;
              tl[it][g >> 1][4 * (g & 1) + e] = lo;
            } else {
              tt[it][4 * g + e] = t;
            }
          }
          if constexpr ((FX & FX_T) != 0) {
            if (valid) ST.st(vo, ss, tv);
          }
        }
      const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 4096);
  #pragma unroll
      for (int jt = 0; jt < IT; ++jt) {
        f32x16 uacc = f32x16{0};
  #pragma unroll
        for (int ct = 0; ct < IT; ++ct) {
          if constexpr (BF) {
            const int o = (jt * IT + ct) * 4096;
  #pragma unroll
            for (int s = 0; s < 2; ++s) {
              const bf16x8 ah = ld_bf8(grs, lane * 16, o + s * 2048), al = ld_bf8(grs, lane * 16, o + s * 2048 + 1024);
              uacc = mfma32bf(ah, th[ct][s], uacc);
              uacc = mfma32bf(al, th[ct][s], uacc);
              uacc = mfma32bf(ah, tl[ct][s], uacc);
            }
          } else {
            const float* gq = p.gp + ((size_t)(jt * IT + ct) * 64 + lane) * 16;
            const f32x4 g0 = ld4(gq), g1 = ld4(gq + 4), g2 = ld4(gq + 8), g3 = ld4(gq + 12);
            const float ga[16] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3],
                                  g2[0], g2[1], g2[2], g2[3], g3[0], g3[1], g3[2], g3[3]};
  #pragma unroll
            for (int r = 0; r < 16; ++r) uacc = mfma32(ga[r], tt[ct][r], uacc);
          }
        }
        if (valid) {
  #pragma unroll
          for (int g = 0; g < 4; ++g) {
            const unsigned ss = so(jt * 8 + 2 * g);
            const f32x4 xv = IX.ld(vo, ss), sv = IS.ld(vo, ss);
            f32x4 v;
            // dx = g s + 2 x u,  x = y / s (bf16 path: y * rcp(s))
            f32x4 xs;
  #pragma unroll
            for (int e = 0; e < 4; ++e) xs[e] = BF ? xv[e] * __builtin_amdgcn_rcpf(sv[e]) : xv[e] / sv[e];
            if constexpr (STASH) {
              const f32x4 gs = Y.ld(vo, ss);
  #pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = gs[e] + 2.0f * xs[e] * uacc[4 * g + e];
            } else {
  #pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int r = 4 * g + e;
                v[e] = acc[jt][r] * sv[e] + 2.0f * xs[e] * uacc[r];
              }
            }
            Y.st(vo, ss, v);
          }
        }
      }
    }
  }
}

// --------------------------------------------------------------------------
// GDN / IGDN forward epilogue of TWO pixel tiles of one wave (the x6 kernels' PT = 2), fp32 activations, x6
// normaliser GEMM: every gamma' fragment round feeds both tiles (2 x IT x 6 MFMAs per 3 x IT fragment loads, the
// next round's loads a whole round = 1.5k cycles ahead), which halves the fragment traffic of two single-tile
// epilogues and hides its L2 latency.  Requires IT*32 == Cout, co_base == 0, FX == 0.
// --------------------------------------------------------------------------
template <int IT, int EPI>
ICA_DEV void gdn_fwd_x6_pair(const ConvParams& p, f32x16 (&acc)[2][IT], int n, const int (&oy)[2],
                             const int (&ox)[2]) {
  static_assert(EPI == EPI_GDN || EPI == EPI_IGDN, "forward GDN epilogues only");
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int C4o = (p.Cout + 3) >> 2;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)C4o * plane;
  const Img4 Y(p.y, img, n), SS(p.save_s, img, n);
  const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout), ers = chan_rsrc(p.beta, p.Cout);
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
  f32x16 nx[2][IT];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = ld_chan4(brs, it * 32 + 8 * g + 4 * h), ev = ld_chan4(ers, it * 32 + 8 * g + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[0][it][4 * g + e] += bv[e];
        acc[1][it][4 * g + e] += bv[e];
        nx[0][it][4 * g + e] = ev[e];
        nx[1][it][4 * g + e] = ev[e];
      }
    }
  bf16x8 ga[2][IT][3];
  auto ldg = [&](bf16x8 (&a)[IT][3], int k) {
#pragma unroll
    for (int ct = 0; ct < IT; ++ct)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        a[ct][q] = ld_bf8(grs, lane * 16, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
  };
  ldg(ga[0], 0);
#pragma unroll
  for (int k = 0; k < 2 * IT; ++k) {
    if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[t][k >> 1][8 * (k & 1) + j] * acc[t][k >> 1][8 * (k & 1) + j];
      bf16x8 xq[3];
      split3x8(v, xq);
#pragma unroll
      for (int ct = 0; ct < IT; ++ct) nx[t][ct] = mfma_x6(ga[k & 1][ct], xq, nx[t][ct]);
    }
  }
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (oy[t] >= p.Hout || ox[t] >= p.Wout) continue;
    const unsigned vo = h * plane + pix_at(oy[t], ox[t], p.Hout, p.Wout, p.pl & PL_OUT);
#pragma unroll
    for (int ct = 0; ct < IT; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 yv, sv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float nv = nx[t][ct][4 * g + e];
          const float sc = (EPI == EPI_GDN) ? __builtin_amdgcn_rsqf(nv) : __builtin_amdgcn_sqrtf(nv);
          sv[e] = sc;
          yv[e] = acc[t][ct][4 * g + e] * sc;
        }
        const unsigned ss = (unsigned)(ct * 8 + 2 * g) * plane;
        if (p.save_s) SS.st(vo, ss, sv);
        Y.st(vo, ss, yv);
      }
  }
}

// --------------------------------------------------------------------------
// The wide x6 GDN / IGDN backward epilogue (conv_epilogue<.., X6 = 1> with FX == 0, IT <= 4) in two halves, so that
// a pipelined kernel can issue the saved (y, s) loads of a tile before its main loop:
//   gdn_bwd_x6_load  : every (y, s) quad of the lane's pixel (a pixel outside the output reads past the descriptor:
//                      0; its MFMA column is never stored)
//   gdn_bwd_x6_wide  : the X6 = 1 arithmetic with the two IEEE divisions per element (x = y / s and, IGDN,
//                      t = g x / (2 s)) replaced by one v_rcp_f32 (1 ulp): x = y rcp(s), t = 0.5 g x rcp(s).  The
//                      divisions were ~20 of the epilogue's ~35 VALU instructions per element, as many cycles as the
//                      kernel's MFMAs at one wave per SIMD; the x6 main loop's own error is ~17 ulps
// --------------------------------------------------------------------------
template <int IT>
ICA_DEV void gdn_bwd_x6_load(const ConvParams& p, int n, int oy, int ox, bool valid, f32x4 (&yq)[IT][4],
                             f32x4 (&sq)[IT][4]) {
  const int h = (threadIdx.x & 63) >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 IX(p.in_x, img, n), IS(p.in_s, img, n);
  const unsigned vo = valid ? h * plane + pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0x0FFFFFF0u;
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      yq[it][g] = IX.ld(vo, (unsigned)(it * 8 + 2 * g) * plane);
      sq[it][g] = IS.ld(vo, (unsigned)(it * 8 + 2 * g) * plane);
    }
}

template <int IT, int EPI>
ICA_DEV void gdn_bwd_x6_wide(const ConvParams& p, f32x16 (&acc)[IT], int n, int oy, int ox, bool valid,
                             const f32x4 (&yq)[IT][4], const f32x4 (&sq)[IT][4]) {
  static_assert(EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD, "GDN backward epilogues only");
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n);
  const unsigned vo = valid ? h * plane + pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u;
  f32x16 xx[IT];
  bf16x8 tq[IT][2][3];
  float tw[8];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 yv = yq[it][g], sv = sq[it][g];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sg = sv[e], rs = __builtin_amdgcn_rcpf(sg), xs = yv[e] * rs;
        const float gx = acc[it][4 * g + e] * xs;
        tw[4 * (g & 1) + e] = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (sg * sg * sg) : (0.5f * gx) * rs;
        float gs = acc[it][4 * g + e] * sg;
        float x2 = 2.0f * xs;
        asm volatile("" : "+v"(gs), "+v"(x2));
        acc[it][4 * g + e] = gs;
        xx[it][4 * g + e] = x2;
      }
      if (g & 1) split3x8(tw, tq[it][g >> 1]);
    }
  __builtin_amdgcn_sched_barrier(0);
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
  f32x16 ux[IT];
#pragma unroll
  for (int jt = 0; jt < IT; ++jt) ux[jt] = f32x16{0};
  bf16x8 ga[2][IT][3];
  auto ldg = [&](bf16x8 (&a)[IT][3], int k) {
#pragma unroll
    for (int jt = 0; jt < IT; ++jt)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        a[jt][q] = ld_bf8(grs, lane * 16, (((jt * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
  };
  ldg(ga[0], 0);
#pragma unroll
  for (int k = 0; k < 2 * IT; ++k) {
    if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jt = 0; jt < IT; ++jt) ux[jt] = mfma_x6(ga[k & 1][jt], tq[k >> 1][k & 1], ux[jt]);
  }
  if (valid) {
#pragma unroll
    for (int jt = 0; jt < IT; ++jt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[jt][4 * g + e] + xx[jt][4 * g + e] * ux[jt][4 * g + e];
        Y.st(vo, (unsigned)(jt * 8 + 2 * g) * plane, v);
      }
  }
}

// --------------------------------------------------------------------------
// x6 GDN / IGDN forward epilogue for kernels at TWO waves per SIMD (256 registers; conv_up_x6w): the two pixel
// tiles' 128 accumulator registers are live on entry, so the pair form's 2 x IT normaliser tiles do not fit.  One
// tile at a time (the other tile's 64 registers wait), one normaliser tile ct at a time (x^2 split per round, the
// gamma' fragments of round k+1 issued before round k's MFMAs): the arithmetic, MFMA order and bits of
// gdn_fwd_x6_pair.  (A GDN-backward counterpart at 256 registers -- t kept or split, g*s parked in the output, u
// per output tile -- measured 17-20 % slower than the 4-wave kernel's wide epilogue and is not built.)
// --------------------------------------------------------------------------
template <int IT, int EPI>
ICA_DEV void gdn_fwd_x6_tile_narrow(const ConvParams& p, f32x16 (&acc)[IT], int n, int oy, int ox) {
  static_assert(EPI == EPI_GDN || EPI == EPI_IGDN, "forward GDN epilogues only");
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n), SS(p.save_s, img, n);
  const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout), ers = chan_rsrc(p.beta, p.Cout);
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = ld_chan4(brs, it * 32 + 8 * g + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += bv[e];
    }
  }
  auto ldg = [&](bf16x8 (&a)[3], int ct, int k) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
      a[q] = ld_bf8(grs, lane * 16, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
  };
  const bool ok = oy < p.Hout && ox < p.Wout;
  const unsigned vo = h * plane + (ok ? pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u);
#pragma unroll
  for (int ct = 0; ct < IT; ++ct) {
    __builtin_amdgcn_sched_barrier(0);
    f32x16 nx;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 ev = ld_chan4(ers, ct * 32 + 8 * g + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) nx[4 * g + e] = ev[e];
    }
    bf16x8 ga[2][3];
    ldg(ga[0], ct, 0);
#pragma unroll
    for (int k = 0; k < 2 * IT; ++k) {
      if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], ct, k + 1);
      __builtin_amdgcn_sched_barrier(0);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = acc[k >> 1][8 * (k & 1) + j] * acc[k >> 1][8 * (k & 1) + j];
      bf16x8 xq[3];
      split3x8(v, xq);
      nx = mfma_x6(ga[k & 1], xq, nx);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (ok) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 yv, sv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float nv = nx[4 * g + e];
          const float sc = (EPI == EPI_GDN) ? __builtin_amdgcn_rsqf(nv) : __builtin_amdgcn_sqrtf(nv);
          sv[e] = sc;
          yv[e] = acc[ct][4 * g + e] * sc;
        }
        const unsigned ss = (unsigned)(ct * 8 + 2 * g) * plane;
        if (p.save_s) SS.st(vo, ss, sv);
        Y.st(vo, ss, yv);
      }
    }
  }
}

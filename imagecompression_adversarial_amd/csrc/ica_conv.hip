// Implicit-GEMM convolutions for the Balle2018 analysis/synthesis transforms on
// CDNA4 fp32 MFMA (v_mfma_f32_32x32x2_f32), with fused GDN/IGDN epilogues.
//
// Replaces (reference): the nn.Conv2d / nn.ConvTranspose2d layers built by
// anchors/utils.py:112-130 (conv k5 s2 p2, deconv k5 s2 p2 op1, and the k3 s1
// convs of h_a/h_s), their autograd input-gradients, and the GDN/IGDN layers of
// utils/ops.py:58-97 (== compressai.layers.GDN) fused into the producing conv.
//
// GEMM orientation: D[co][px] = sum_k W[co][k] * X[k][px].  Output channels are
// the MFMA rows (4 accumulator tiles = 128 channels per wave), pixels the MFMA
// columns (32 per wave).  Because a wave owns ALL channels of its pixels, the
// GDN normaliser  n = beta' + gamma' x^2  is a second in-register MFMA GEMM over
// the accumulator rows (no LDS transpose), and GDN backward
// u = gamma'^T (g x dS/dn) likewise.
//
//   conv_down : stride-S conv, KS x KS, pad KS/2.  Block = 4 waves x 32 px
//               (TH x TW output tile), all (IT*32) channels of a channel block.
//               K loop = channel chunks (LDS patch, CC channels) x taps.
//   conv_up   : transposed conv k5 s2 p2 op1, decomposed into the 4 output
//               parity classes (9/6/6/4 taps).  Block = 8x32 output pixels
//               (4x16 per class); the whole-Cin input patch lives in LDS; each
//               wave runs two class tiles paired 9+4 / 6+6 for balance.
#include <cxxabi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "ica_conv_epi.h"

// bf16 weight-fragment load of tile it at step g
#define ICA_WLOAD_BF(w, it, g) ((w)[(it) * 64])

// Load one (chunk, tap) weight fragment set: IT tiles x KH floats per lane.
template <int IT, int KH>
ICA_DEV void load_frag(float (&a)[IT][KH], const float* w) {
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if constexpr (KH == 8) {
      const f32x4 w0 = ld4(w + it * 64 * KH), w1 = ld4(w + it * 64 * KH + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a[it][e] = w0[e];
        a[it][4 + e] = w1[e];
      }
    } else {
      const f32x2 w0 = *reinterpret_cast<const f32x2*>(w + it * 64 * KH);
      a[it][0] = w0[0];
      a[it][1] = w0[1];
    }
  }
}

// --------------------------------------------------------------------------
// conv_down: stride-S KSxKS conv, pad KS/2.  Weight fragments packed as
// [cb][chunk][tap][it][lane][KH]  with  o = cb*IT*32 + it*32 + (lane&31),
// c = chunk*CC + (lane>>5)*KH + s.
// --------------------------------------------------------------------------
// pixel tiles (32 px each) per wave: the bf16 16-channel-chunk path runs 2, so each weight fragment (an
// L1 -> register stream of 4 KB per wave-step, the bf16 main loop's limit) feeds twice the MFMAs
template <int CC, bool BF>
constexpr int down_pt() { return (BF && CC == 16) ? 2 : 1; }
// the x6 k3 conv_down at two rows per wave on large grids (ICA_X6O_PT2=0 builds: one row; ICA_X6O_PT2_GDN=0: one row
// for the GDN / IGDN (backward) epilogues -- for A/B runs)
#ifndef ICA_X6O_PT2
#define ICA_X6O_PT2 1
#endif
#ifndef ICA_X6O_PT2_GDN
#define ICA_X6O_PT2_GDN 1
#endif

// occupancy target: 2 blocks/CU, except the k5 IT = 6 (C = 192, bmshj2018 q6-8) variants, whose 6-tile
// accumulators + fragment ring + GDN epilogue need the whole 512-register file (1 block/CU, no spills)
template <int KS, int IT>
constexpr int conv_min_blocks() { return (KS == 5 && IT == 6) ? 1 : 2; }

// the bf16 RGB-input GDN forward (g_a's first layer, store-bound) fits 128 VGPRs: 4 waves/SIMD (IT = 4; the
// C = 192 variant runs one wave per SIMD like every IT = 6 k5 kernel)
template <int KS, int IT, int CC, int EPI, bool BF>
constexpr int conv_down_waves() {
  return (BF && CC == 4 && EPI == EPI_GDN && IT <= 4) ? 4 : conv_min_blocks<KS, IT>();
}

// X6O: fp32-accurate bf16x6 operands (fp32 activations split into three bf16 planes as the patch is staged, the
// three-plane weight pack of ica_pack_conv_weight_x6, six MFMAs per 16-deep k step; x6 GDN epilogue GEMMs on the
// ica_pack_gdn_x6 pack): the k3 s1 layers of cheng2020 on the x6 ceiling.  One block per CU (512 registers); two for
// IT = 1 (g_s.7's 16 rho rows: 16 accumulators).
// XPT: 32-px rows per wave on the X6O path (2 at IT >= 4 on large grids, see pick_tw_down_x6o).
// NPL: bf16 planes of the X6O operands: 3 = x6 (six MFMAs per k step); 1 = bf16 operands over fp32 activations
// (ICA_PREC_B1: the hi plane alone, i.e. RNE bf16 of the activations and of the weights, one MFMA per k step, fp32
// accumulate; the GDN epilogue GEMMs stay x6) -- cheng2020's --precision bf16.
template <int KS, int S, int IT, int CC, int TW, int EPI, int FX, bool BF, bool X6O = false, int XPT = 1, int NPL = 3>
__global__ __launch_bounds__(256, X6O ? (IT == 1 ? 2 : 1) : (conv_down_waves<KS, IT, CC, EPI, BF>())) void conv_down_kernel(ConvParams p) {
  constexpr int PT = X6O ? XPT : down_pt<CC, BF>();
  static_assert(XPT == 1 || (X6O && XPT == 2 && (ICA_X6O_PT2_GDN || !epi_gdn<EPI>()) && IT >= 4), "x6 conv_down: two rows per wave at IT >= 4");
  constexpr int TH = PT * 128 / TW;
  constexpr int PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS;
  constexpr int NQ = CC / 4, KH = CC / 2, PLANE = PR * PC, PAD = KS / 2;
  constexpr int WSTEP = IT * 64 * KH;  // floats per (chunk, tap)
  // bf16 operands (BF): one 16-B LDS entry holds 8 channels of a pixel as bf16 (2 entries per
  // 16-channel chunk, entry h = channels 8h..8h+7 = the B fragment of lane half h)
  constexpr int NE = (BF && CC == 16) ? NQ / 2 : NQ;
  // bf16 with CC == 4 (an RGB conv input): K = 4 taps x 4 channels per MFMA ("tap groups"), fp32 LDS patch
  static_assert(!BF || CC == 16 || CC == 4, "bf16 conv_down: 16-channel chunks or 4-channel tap groups");
  static_assert(!X6O || (!BF && CC == 16), "x6 conv_down: fp32 fills of 16-channel chunks");
  static_assert(NPL == 3 || (NPL == 1 && X6O), "one-plane operands: the X6O kernel only");
  // X6O: [buffer][plane][half][pixel], 8 channels as bf16; the GDN-backward epilogues park g*s in it afterwards
  // (IT*16 floats per lane, one slab per wave)
  constexpr bool XST = X6O && (EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD) && !(FX == 0 && IT <= 4);
  __shared__ f32x4 patch[X6O ? (XST && IT * 1024 > 12 * PLANE ? IT * 1024 : 12 * PLANE) : NE * PLANE];
  // bf16 16-channel-chunk layers: the epilogue parameters in LDS (epi_params_to_lds), copied before the first
  // chunk fill, whose barriers publish them
  // The RGB-input GDN forward too (g_a.0: 1.65 -> 1.31 ms at the config-5 shapes, although its 46 KB of LDS take it
  // from 4 to 3 blocks per CU); the RGB GDN backward measured neutral and keeps the global loads.
  constexpr bool LG = BF && FX == 0 && (CC == 16 || (CC == 4 && (EPI == EPI_GDN || EPI == EPI_IGDN)));
  __shared__ f32x4 lpar[LG ? epi_lds_entries<IT, EPI>() : 1];

  const int tiles_x = (p.Wout + TW - 1) / TW, tiles_y = (p.Hout + TH - 1) / TH;
  int bid, cb;
  xcd_block<BF>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int Cin4 = (p.Cin + 3) >> 2;
  const int nch = (Cin4 * 4 + CC - 1) / CC;
  if constexpr (LG) epi_params_to_lds<IT, EPI>(p, lpar, cb * IT * 32);
  // pixel tile t of this wave: block pixels (wave*PT + t)*32 + j
  int oyl[PT], oxl[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int pl = (wave * PT + t) * 32 + j;
    oyl[t] = pl / TW;
    oxl[t] = pl % TW;
  }

  f32x16 acc[PT][IT];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};

  // one 4-channel group of the conv input at (iy, ix), with the fill-mode view applied
  auto ldc4 = [&](int c4, int iy, int ix) -> f32x4 {
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win) {
      if constexpr ((FX & FX_UNSHUF) != 0) {
        // PixelUnshuffle(2): rho channel 16*c4g + 4*q + e of pixel (iy, ix) is channel 4*c4g + e
        // of the (2 Hin) x (2 Win) tensor at sub-pixel q = 2i + j
        const int c4g = c4 >> 2, q = c4 & 3;
        v = ld4(p.x + ((((size_t)n * (Cin4 >> 2) + c4g) * (2 * p.Hin) + 2 * iy + (q >> 1)) * (2 * p.Win) +
                       2 * ix + (q & 1)) * 4);
      } else {
        const size_t xo = (((size_t)n * Cin4 + c4) * ((size_t)p.Hin * p.Win) + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 4;
        v = ld4(p.x + xo);
        if constexpr ((FX & FX_MASK) != 0) {
          const f32x4 m = ld4(p.mask + xo);
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) v[e2] = m[e2] > 0.f ? v[e2] : v[e2] * 0.01f;
        }
      }
      if constexpr (CC == 4) {
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2)
          if (c4 * 4 + e2 >= p.Cin) v[e2] = 0.f;
      }
    }
    return v;
  };
  auto fill = [&](int ch) {
    if constexpr (BF && CC == 16) {
      // bf16 activations: the chunk's loads are issued in two batches of NB rows per thread (registers), the
      // first one before the barrier that ends the previous chunk's reads: two memory latencies per fill
      // instead of one per 256-entry row of the patch (the whole chunk at once spilled)
      static_assert(!BF || FX == 0, "bf16 conv_down fill: plain view only");
      constexpr int NF = (NE * PLANE + 255) / 256, NB = (NF + 1) / 2;
      // buffer loads with 32-bit lane offsets into this image (no 64-bit address registers); padding and
      // entries past the patch read out of the descriptor's range, which returns zeros
      const unsigned xplane = (unsigned)p.Hin * p.Win;
      const __amdgpu_buffer_rsrc_t xr =
          uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 8, Cin4 * xplane * 8u);
      auto batch = [&](int i0, u32x2 (&va)[NB], u32x2 (&vb)[NB]) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int e = threadIdx.x + 256 * (i0 + i);
          const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
          const int iy = iy0 + pr, ix = ix0 + pc;
          const int c4 = ch * NQ + 2 * q;
          const bool ok = i0 + i < NF && e < NE * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 &&
                          ix < p.Win;
          const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 8u;
          va[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
          vb[i] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, ok ? vo + xplane * 8u : 0xFFFFFFF0u,
                                                                                 0, 0));
        }
      };
      auto put = [&](int i0, const u32x2 (&va)[NB], const u32x2 (&vb)[NB]) {
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int e = threadIdx.x + 256 * (i0 + i);
          if (i0 + i < NF && e < NE * PLANE)
            patch[e] = __builtin_bit_cast(f32x4, (u32x4_t){va[i][0], va[i][1], vb[i][0], vb[i][1]});
        }
      };
      u32x2 va[NB], vb[NB];
      batch(0, va, vb);
      __syncthreads();
      put(0, va, vb);
      batch(NB, va, vb);
      put(NB, va, vb);
      __syncthreads();
      return;
    }
    if constexpr (!BF && CC == 16 && (X6O || (FX & (FX_MASK | FX_UNSHUF)) == 0)) {
      // fp32 plain view (any epilogue extras): batches of FB 16-B buffer loads (32-bit offsets, out-of-image reads return zeros)
      // issued before their LDS writes, the first batch ahead of the barrier that ends the previous chunk's
      // reads.  FB is kept small: these kernels run 3 waves/SIMD at <= 168 VGPRs.  X6O also takes the
      // leaky-ReLU-masked view (the mask quads load beside the activations; one block per CU, VGPRs spare) and
      // the PixelUnshuffle(2) view here (same image extent, only the quad offsets differ).
      constexpr bool MK = (FX & FX_MASK) != 0, US = (FX & FX_UNSHUF) != 0;
      constexpr int NF = (NE * PLANE + 255) / 256, FB = 3;
      const unsigned xplane = (unsigned)p.Hin * p.Win;
      const __amdgpu_buffer_rsrc_t xr =
          uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
      const __amdgpu_buffer_rsrc_t mr =
          uniform_rsrc(reinterpret_cast<const char*>(MK ? p.mask : p.x) + (size_t)n * Cin4 * xplane * 16,
                       MK ? Cin4 * xplane * 16u : 0u);
      u32x4_t mv[MK ? FB : 1];
      auto batch = [&](int i0, u32x4_t (&v)[FB]) {
#pragma unroll
        for (int i = 0; i < FB; ++i) {
          const int e = threadIdx.x + 256 * (i0 + i);
          const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
          const int iy = iy0 + pr, ix = ix0 + pc;
          const int c4 = ch * NQ + q;
          const bool ok = i0 + i < NF && e < NE * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 &&
                          ix < p.Win;
          unsigned vo;
          if constexpr (US) {   // rho quad 4*c4g + sq of pixel (iy, ix): quad c4g of the 2x tensor at sub-pixel sq
            const int c4g = c4 >> 2, sq = c4 & 3;
            vo = (((unsigned)c4g * (2 * p.Hin) + 2 * iy + (sq >> 1)) * (2 * p.Win) + 2 * ix + (sq & 1)) * 16u;
          } else {
            vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
          }
          v[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
          if constexpr (MK)
            mv[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(mr, ok ? vo : 0xFFFFFFF0u, 0, 0));
        }
      };
      auto put = [&](int i0, const u32x4_t (&v)[FB]) {
#pragma unroll
        for (int i = 0; i < FB; ++i) {
          const int e = threadIdx.x + 256 * (i0 + i);
          if (i0 + i < NF && e < NE * PLANE) {
            if constexpr (X6O) {   // quad q of pixel pix -> three bf16 planes, half q >> 1, slot q & 1
              const int q = e / PLANE, pix = e - q * PLANE;
              f32x4 x = __builtin_bit_cast(f32x4, v[i]);
              if constexpr (MK) {   // the generic fill's leaky-ReLU view, same fp32 ops
                const f32x4 m = __builtin_bit_cast(f32x4, mv[i]);
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) x[e2] = m[e2] > 0.f ? x[e2] : x[e2] * 0.01f;
              }
              u32x2 a, b, c;
              split3(x, a, b, c);
              u32x2* p2 = reinterpret_cast<u32x2*>(patch);
              const int ent = (q >> 1) * PLANE + pix;
              p2[(0 * 2 * PLANE + ent) * 2 + (q & 1)] = a;
              p2[(1 * 2 * PLANE + ent) * 2 + (q & 1)] = b;
              p2[(2 * 2 * PLANE + ent) * 2 + (q & 1)] = c;
            } else {
              patch[e] = __builtin_bit_cast(f32x4, v[i]);
            }
          }
        }
      };
      u32x4_t v[FB];
      batch(0, v);
      __syncthreads();
      put(0, v);
#pragma unroll
      for (int i0 = FB; i0 < NF; i0 += FB) {
        batch(i0, v);
        put(i0, v);
      }
      __syncthreads();
      return;
    }
    if constexpr (CC == 4 && FX == 0) {
      // RGB input (one 4-channel plane, one fill per block): every entry of this thread (NF = 3 for the
      // k5 s2 tiles) is loaded up front with 16-B buffer loads (32-bit offsets; padding reads past the
      // descriptor and returns zeros), one memory latency instead of NF dependent rounds.
      constexpr int NF = (NE * PLANE + 255) / 256;
      const unsigned xplane = (unsigned)p.Hin * p.Win;
      const __amdgpu_buffer_rsrc_t xr =
          uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
      u32x4_t v[NF];
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int e = threadIdx.x + 256 * i;
        const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
        const int iy = iy0 + pr, ix = ix0 + pc;
        const int c4 = ch * NQ + q;
        const bool ok = e < NE * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
        v[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        const int e = threadIdx.x + 256 * i;
        if (e < NE * PLANE) {
          f32x4 f = __builtin_bit_cast(f32x4, v[i]);
          const int c4 = ch * NQ + e / PLANE;
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2)
            if (c4 * 4 + e2 >= p.Cin) f[e2] = 0.f;
          patch[e] = f;
        }
      }
      __syncthreads();
      return;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < NE * PLANE; e += 256) {
      const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      if constexpr (BF && CC == 16) {
        // bf16 activations: the two channel quads are two 8-B loads, concatenated as they are
        static_assert(!BF || FX == 0, "bf16 conv_down fill: plain view only");
        const int c4 = ch * NQ + 2 * q;
        u32x2 a = {0u, 0u}, b = {0u, 0u};
        if (c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win) {
          const u32x2* xb =
              reinterpret_cast<const u32x2*>(p.x) + ((size_t)n * Cin4 + c4) * ((size_t)p.Hin * p.Win) + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN);
          a = xb[0];
          b = xb[(size_t)p.Hin * p.Win];
        }
        patch[e] = __builtin_bit_cast(f32x4, (u32x4_t){a[0], a[1], b[0], b[1]});
      } else {
        patch[e] = ldc4(ch * NQ + q, iy, ix);
      }
    }
    __syncthreads();
  };

  constexpr int KK = KS * KS;
  const int total = nch * KK;
  int lb[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) lb[t] = (S * oyl[t]) * PC + S * oxl[t];
  const int lbase = lb[0];
  if constexpr (BF && CC == 4) {
    // bf16, 3-channel input: k = 8h + j of tap group tg is tap 4tg + 2h + (j>>2), channel j&3, so a lane's
    // B fragment is the f32x4 pixels of two taps (rounded to bf16); 7 MFMAs per tile cover the 25 taps
    // (fp32 CC = 4 needs 50).  Weights: [cb][tg][it][lane][8] bf16 (pack_conv_tg_kernel), 4-set ring.
    constexpr int TG = (KK + 3) / 4;
    fill(0);
    const bf16x8* wb = reinterpret_cast<const bf16x8*>(p.wp) + (size_t)cb * TG * IT * 64 + lane;
    bf16x8 fr[4][IT];
    auto ldw = [&](bf16x8 (&a)[IT], int g) {
      const bf16x8* w = wb + (size_t)min(g, TG - 1) * IT * 64;
#pragma unroll
      for (int it = 0; it < IT; ++it) a[it] = ICA_WLOAD_BF(w, it, g);
    };
    auto tapoff = [&](int t) {
      t = min(t, KK - 1);  // taps past KK carry zero weights; read any finite patch value
      const int ky = t / KS, kx = t - ky * KS;
      return lbase + ky * PC + kx;
    };
    auto step = [&](bf16x8 (&cur)[IT], bf16x8 (&nxt)[IT], int g) {
      ldw(nxt, g + 3);
      const int t0 = 4 * g + 2 * h;
      const bf16x8 b = to_bf8(patch[tapoff(t0)], patch[tapoff(t0 + 1)]);
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[0][it] = mfma32bf(cur[it], b, acc[0][it]);
    };
    ldw(fr[0], 0);
    ldw(fr[1], 1);
    ldw(fr[2], 2);
    int g = 0;
#pragma unroll 1
    for (; g + 4 <= TG; g += 4) {
      step(fr[0], fr[3], g);
      step(fr[1], fr[0], g + 1);
      step(fr[2], fr[1], g + 2);
      step(fr[3], fr[2], g + 3);
    }
    if (g < TG) step(fr[0], fr[3], g);
    if (g + 1 < TG) step(fr[1], fr[0], g + 1);
    if (g + 2 < TG) step(fr[2], fr[1], g + 2);
  } else if constexpr (BF) {
    // bf16: one v_mfma_f32_32x32x16_bf16 per (chunk, tap, tile) = 32 cycles, so the weight
    // fragments (16 B per lane per tile, L2-resident) are prefetched 3 steps ahead in a 4-set
    // register ring (indices compile-time via a 4x unrolled loop: no scratch, no copies).
    const bf16x8* wb = reinterpret_cast<const bf16x8*>(p.wp) + (size_t)cb * nch * KK * IT * 64 + lane;
    bf16x8 fr[4][IT];
    auto ldw = [&](bf16x8 (&a)[IT], int g) {
      const bf16x8* w = wb + (size_t)min(g, total - 1) * IT * 64;
#pragma unroll
      for (int it = 0; it < IT; ++it) a[it] = ICA_WLOAD_BF(w, it, g);
    };
    auto step = [&](bf16x8 (&cur)[IT], bf16x8 (&nxt)[IT], int g) {
      const int ch = g / KK, tap = g - ch * KK;
      if (tap == 0) fill(ch);
      ldw(nxt, g + 3);
      const int ky = tap / KS, kx = tap - (tap / KS) * KS;
      bf16x8 b[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) b[t] = f4_as_bf8(patch[h * PLANE + lb[t] + ky * PC + kx]);
#pragma unroll
      for (int t = 0; t < PT; ++t)
#pragma unroll
        for (int it = 0; it < IT; ++it) acc[t][it] = mfma32bf(cur[it], b[t], acc[t][it]);
    };
    ldw(fr[0], 0);
    ldw(fr[1], 1);
    ldw(fr[2], 2);
    int g = 0;
#pragma unroll 1
    for (; g + 4 <= total; g += 4) {
      step(fr[0], fr[3], g);
      step(fr[1], fr[0], g + 1);
      step(fr[2], fr[1], g + 2);
      step(fr[3], fr[2], g + 3);
    }
    if (g < total) step(fr[0], fr[3], g);
    if (g + 1 < total) step(fr[1], fr[0], g + 1);
    if (g + 2 < total) step(fr[2], fr[1], g + 2);
  } else if constexpr (CC == 4) {
    // fp32 RGB input, packed K (pack_conv_kernel, CC = 4): k-step m = 2g + s2 of step g takes the (tap,
    // channel) pair f = 2m + h from lane half h, f running over tap*Cin + channel.  With Cin = 3 that is
    // ceil(75/4) = 19 steps of 2 MFMA k-steps instead of 25 taps x (3 channels + 1 zero pad).
    fill(0);
    const int Cp = p.Cin;
    const int NS = (KK * Cp + 3) / 4;
    const float* wptr = p.wp + (size_t)cb * KK * WSTEP + (size_t)lane * KH;
    const float* pf = reinterpret_cast<const float*>(patch);
    auto bval = [&](int f) -> float {
      int tap = f / Cp;
      const int c = f - tap * Cp;
      tap = min(tap, KK - 1);  // past the list: zero weight, read any finite patch value
      const int ky = tap / KS, kx = tap - ky * KS;
      return pf[4 * (lbase + ky * PC + kx) + c];
    };
    auto step = [&](float (&cur)[IT][KH], float (&nxt)[IT][KH], int g) {
      load_frag<IT, KH>(nxt, wptr + (size_t)min(g + 1, NS - 1) * WSTEP);  // unconditional: no phi copies
      const float b[2] = {bval(4 * g + h), bval(4 * g + 2 + h)};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int it = 0; it < IT; ++it) acc[0][it] = mfma32(cur[it][s2], b[s2], acc[0][it]);
    };
    float fa[IT][KH], fb[IT][KH];
    load_frag<IT, KH>(fa, wptr);
    int g = 0;
#pragma unroll 1
    for (; g + 1 < NS; g += 2) {
      step(fa, fb, g);
      step(fb, fa, g + 1);
    }
    if (g < NS) step(fa, fb, g);
  } else if constexpr (X6O) {
    // x6 operands: three bf16 weight-fragment planes (plane stride ps fragments), one step ahead (ping-pong)
    const long ps = (long)((p.Cout + IT * 32 - 1) / (IT * 32)) * nch * KK * IT * 64;
    const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
    const int wbase = cb * nch * KK * IT * 64;
    auto ldw = [&](bf16x8 (&a)[IT][3], int g) {
      const int f = wbase + min(g, total - 1) * IT * 64;
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int q = 0; q < NPL; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + it * 64) * 16));
    };
    // Double-buffered patch (X6DB): chunk c + 1 is staged into the other 6-plane buffer while chunk c's taps run
    // -- its NF quads per thread are issued one per tap (taps 0..NF-1, after that tap's weight prefetch) and split
    // into the bf16 planes PUTD taps later -- so one barrier per chunk and no exposed fill latency.  The weights
    // run in a 3-set ring two taps ahead (KK = 9 = 3 rings, so a chunk always starts on set 0): a tap's fill load
    // is then younger than the weights consumed for the next three taps, and the in-order vmcnt never waits on it
    // before its own split.  Same MFMA order as the single-buffer loop (bit-identical results).
    static_assert(KK % 3 == 0, "x6 conv_down ring: KK a multiple of 3");
    constexpr bool MK = (FX & FX_MASK) != 0, US = (FX & FX_UNSHUF) != 0;
    // FPT quads per thread issued per tap (1 for the stride-1 patches; 2 for the stride-2 forward's 2.5x larger
    // patch, NF = 9-10), each split PUTD taps after its load
    constexpr int NF = (NE * PLANE + 255) / 256, PUTD = 3, FPT = (NF + KK - PUTD - 1) / (KK - PUTD);
    static_assert((NF + FPT - 1) / FPT + PUTD <= KK, "x6 conv_down: the chunk's fill must land inside its taps");
    const unsigned xplane = (unsigned)p.Hin * p.Win;
    const __amdgpu_buffer_rsrc_t xr =
        uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
    const __amdgpu_buffer_rsrc_t mr =
        uniform_rsrc(reinterpret_cast<const char*>(MK ? p.mask : p.x) + (size_t)n * Cin4 * xplane * 16,
                     MK ? Cin4 * xplane * 16u : 0u);
    // per-thread quad offsets (chunk 0) and validity: a quad's offset is linear in the chunk (4 quads a chunk) in
    // both views (plain: 4 channel planes; PixelUnshuffle(2): one quad plane of the 2x tensor = 4 Hin Win quads)
    unsigned fo[NF];
    int fq[NF];
    bool fok[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      fq[i] = q;
      fok[i] = e < NE * PLANE && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      if constexpr (US)
        fo[i] = (((unsigned)(2 * iy + (q >> 1))) * (2 * p.Win) + 2 * ix + (q & 1)) * 16u;
      else
        fo[i] = ((unsigned)q * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
    }
    u32x4_t fv[NF], fm[MK ? NF : 1];
    auto fload = [&](int ch, int i) {
      const bool ok = fok[i] && ch * NQ + fq[i] < Cin4;
      const unsigned vo = ok ? fo[i] + (unsigned)ch * 4u * xplane * 16u : 0xFFFFFFF0u;
      fv[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, vo, 0, 0));
      if constexpr (MK) fm[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(mr, vo, 0, 0));
    };
    auto fput = [&](f32x4* buf, int i) {
      const int e = threadIdx.x + 256 * i;
      if (e < NE * PLANE) {   // quad q of pixel pix -> three bf16 planes, half q >> 1, slot q & 1
        const int q = fq[i], pix = e - q * PLANE;
        f32x4 x = __builtin_bit_cast(f32x4, fv[i]);
        if constexpr (MK) {   // the generic fill's leaky-ReLU view, same fp32 ops
          const f32x4 m = __builtin_bit_cast(f32x4, fm[i]);
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) x[e2] = m[e2] > 0.f ? x[e2] : x[e2] * 0.01f;
        }
        u32x2 a, b, c;
        split3(x, a, b, c);
        u32x2* p2 = reinterpret_cast<u32x2*>(buf);
        const int ent = (q >> 1) * PLANE + pix;
        p2[(0 * 2 * PLANE + ent) * 2 + (q & 1)] = a;
        if constexpr (NPL == 3) {
          p2[(1 * 2 * PLANE + ent) * 2 + (q & 1)] = b;
          p2[(2 * 2 * PLANE + ent) * 2 + (q & 1)] = c;
        }
      }
    };
#pragma unroll
    for (int i = 0; i < NF; ++i) fload(0, i);
#pragma unroll
    for (int i = 0; i < NF; ++i) fput(patch, i);
    __syncthreads();
    if constexpr (PT == 2 || S == 2) {
      // (S = 2: the stride-2 forward's 10 fill quads per thread leave no room for a third weight set either)
      // Two 32-px rows per wave (the k3 layers on large grids): each weight fragment -- the main loop's
      // L1 -> register stream, ~37 B/cycle/CU at one row -- feeds twice the MFMAs.  The 2 x IT accumulators leave
      // room for two weight sets only, so the ring is a ping-pong one tap ahead; KK is odd, so a chunk's first set
      // is ch & 1 and the loop body runs a chunk pair.  A tap's fill load is issued after the next tap's weights,
      // so the in-order vmcnt waits on it only at its own split PUTD taps later.  Same MFMA order per output as
      // PT = 1 (bit-identical results).
      static_assert(KK % 2 == 1, "x6 conv_down ping-pong: KK odd");
      bf16x8 fr[2][IT][3];
      ldw(fr[0], 0);
      auto chunk = [&](int ch, auto r0) {
        constexpr int R0 = decltype(r0)::value;
        const f32x4* cur = patch + (ch & 1) * 6 * PLANE;
        f32x4* nxt = patch + ((ch & 1) ^ 1) * 6 * PLANE;
        bf16x8 bb[2][PT][3];
        auto ldb = [&](bf16x8 (&b)[PT][3], int tap) {
          const int ky = tap / KS, kx = tap - (tap / KS) * KS;
#pragma unroll
          for (int t = 0; t < PT; ++t) {
            const int o = h * PLANE + lb[t] + ky * PC + kx;
            b[t][0] = f4_as_bf8(cur[o]);
            if constexpr (NPL == 3) {
              b[t][1] = f4_as_bf8(cur[2 * PLANE + o]);
              b[t][2] = f4_as_bf8(cur[4 * PLANE + o]);
            }
          }
        };
        ldb(bb[0], 0);
#pragma unroll
        for (int tap = 0; tap < KK; ++tap) {
          ldw(fr[(R0 + tap + 1) & 1], ch * KK + tap + 1);
#pragma unroll
          for (int i = tap * FPT; i < (tap + 1) * FPT && i < NF; ++i) fload(ch + 1, i);
#pragma unroll
          for (int i = (tap - PUTD) * FPT; i >= 0 && i < (tap - PUTD + 1) * FPT && i < NF; ++i) fput(nxt, i);
          if (tap + 1 < KK) ldb(bb[(tap + 1) & 1], tap + 1);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int it = 0; it < IT; ++it)
#pragma unroll
            for (int t = 0; t < PT; ++t)
              acc[t][it] = mfma_np<NPL>(fr[(R0 + tap) & 1][it], bb[tap & 1][t], acc[t][it]);
        }
        __syncthreads();
      };
      using I0 = std::integral_constant<int, 0>;
      using I1 = std::integral_constant<int, 1>;
      int ch = 0;
#pragma unroll 1
      for (; ch + 1 < nch; ch += 2) {
        chunk(ch, I0{});
        chunk(ch + 1, I1{});
      }
      if (ch < nch) chunk(ch, I0{});
    } else {
      bf16x8 fr[3][IT][3];
      ldw(fr[0], 0);
      ldw(fr[1], 1);
  #pragma unroll 1
      for (int ch = 0; ch < nch; ++ch) {
        const f32x4* cur = patch + (ch & 1) * 6 * PLANE;
        f32x4* nxt = patch + ((ch & 1) ^ 1) * 6 * PLANE;
        // B operands: tap t + 1's three planes are read during tap t (tap 0's right after the barrier)
        bf16x8 bb[2][3];
        auto ldb = [&](bf16x8 (&b)[3], int tap) {
          const int ky = tap / KS, kx = tap - (tap / KS) * KS;
          const int o = h * PLANE + lbase + ky * PC + kx;
          b[0] = f4_as_bf8(cur[o]);
          if constexpr (NPL == 3) {
            b[1] = f4_as_bf8(cur[2 * PLANE + o]);
            b[2] = f4_as_bf8(cur[4 * PLANE + o]);
          }
        };
        ldb(bb[0], 0);
  #pragma unroll
        for (int tap = 0; tap < KK; ++tap) {
          ldw(fr[(tap + 2) % 3], ch * KK + tap + 2);
          // past the last chunk: c4 >= Cin4, zero reads into the idle buffer
#pragma unroll
          for (int i = tap * FPT; i < (tap + 1) * FPT && i < NF; ++i) fload(ch + 1, i);
#pragma unroll
          for (int i = (tap - PUTD) * FPT; i >= 0 && i < (tap - PUTD + 1) * FPT && i < NF; ++i) fput(nxt, i);
          if (tap + 1 < KK) ldb(bb[(tap + 1) & 1], tap + 1);
          __builtin_amdgcn_sched_barrier(0);
  #pragma unroll
          for (int it = 0; it < IT; ++it) acc[0][it] = mfma_np<NPL>(fr[tap % 3][it], bb[tap & 1], acc[0][it]);
        }
        __syncthreads();
      }
    }
  } else {
    // Weight fragments stream linearly through (chunk, tap); they are prefetched
    // one tap ahead into the other of two register sets (ping-pong, no copies)
    // so each tap's MFMAs cover the next tap's global (L2-resident) load latency.
    const float* wptr = p.wp + (size_t)cb * nch * KS * KS * WSTEP + (size_t)lane * KH;
    auto step = [&](float (&cur)[IT][KH], float (&nxt)[IT][KH], int g) {
      const int ch = g / KK, tap = g - ch * KK;
      if (tap == 0) fill(ch);
      load_frag<IT, KH>(nxt, wptr + (size_t)min(g + 1, total - 1) * WSTEP);  // unconditional: no phi copies
      const int ky = tap / KS, kx = tap - (tap / KS) * KS;
      const int lo = lbase + ky * PC + kx;
      float b[KH];
      if constexpr (CC == 16) {
        const f32x4 v0 = patch[(2 * h) * PLANE + lo];
        const f32x4 v1 = patch[(2 * h + 1) * PLANE + lo];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          b[e] = v0[e];
          b[4 + e] = v1[e];
        }
      } else {  // CC == 4
        const float* pf = reinterpret_cast<const float*>(&patch[lo]) + 2 * h;
        const f32x2 v = *reinterpret_cast<const f32x2*>(pf);
        b[0] = v[0];
        b[1] = v[1];
      }
#pragma unroll
      for (int s2 = 0; s2 < KH; ++s2)
#pragma unroll
        for (int it = 0; it < IT; ++it) acc[0][it] = mfma32(cur[it][s2], b[s2], acc[0][it]);
    };
    float fa[IT][KH], fb[IT][KH];
    load_frag<IT, KH>(fa, wptr);
    int g = 0;
#pragma unroll 1
    for (; g + 1 < total; g += 2) {
      step(fa, fb, g);
      step(fb, fa, g + 1);
    }
    if (g < total) step(fa, fb, g);
  }
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int oy = oy0 + oyl[t], ox = ox0 + oxl[t];
    // X6O: the GDN / IGDN (and backward) normaliser GEMMs on x6 operands too (wide form, 1 wave/SIMD; the gamma' pack
    // of ica_pack_gdn_x6)
    constexpr int EX6 = X6O && epi_gdn<EPI>() ? 1 : 0;
    conv_epilogue<IT, EPI, FX, BF, EX6, LG>(p, acc[t], n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32, lpar,
                                            X6O ? reinterpret_cast<float*>(patch) + wave * IT * 1024 : nullptr);
  }
}

// --------------------------------------------------------------------------
// Small-grid fp32 conv_down (16-channel chunks, plain view): the 4 waves of a block share ONE 32-pixel output
// tile (4 x 8) and split its taps (wave w: taps [w KK / 4, (w + 1) KK / 4)); the four partial accumulators are
// summed through LDS in wave order (deterministic) and wave 0 runs the epilogue.  4x the blocks of
// conv_down_kernel and a quarter of its serial MFMA chain per wave, for the layers whose plain grid leaves most
// CUs idle (the fine-tune's 256x256 crops: 16x16 .. 64x64 outputs, 32-256 blocks), where the plain kernel runs at
// the latency of one wave's K chain.  Weights: the conv_down pack ([cb][chunk][tap][it][lane][8]).
// --------------------------------------------------------------------------
constexpr int DS_TW = 8, DS_TH = 4;
template <int KS, int S, int IT, int EPI, int FX>
__global__ __launch_bounds__(256, 2) void conv_down_split_kernel(ConvParams p) {
  constexpr int PR = S * (DS_TH - 1) + KS, PC = S * (DS_TW - 1) + KS, PLANE = PR * PC, PAD = KS / 2;
  constexpr int KK = KS * KS, NQ = 4, KH = 8, WSTEP = IT * 64 * KH;
  constexpr int NF = (NQ * PLANE + 255) / 256;
  __shared__ f32x4 patch[NQ * PLANE];
  __shared__ f32x4 red[3 * IT * 4 * 64];   // partial accumulators of waves 1..3: [wave-1][it][quad][lane]
  const int tiles_x = (p.Wout + DS_TW - 1) / DS_TW, tiles_y = (p.Hout + DS_TH - 1) / DS_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5,
            j = lane & 31;
  const int oy0 = ty * DS_TH, ox0 = tx * DS_TW;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int Cin4 = (p.Cin + 3) >> 2, nch = (Cin4 * 4 + 15) / 16;
  const int oyl = j / DS_TW, oxl = j % DS_TW;
  const int lbase = S * oyl * PC + S * oxl;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  // chunk fill: every entry of this thread loaded before the barrier that ends the previous chunk's reads
  auto fill = [&](int ch) {
    u32x4_t v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc, c4 = ch * NQ + q;
      const bool ok = e < NQ * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
      v[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < NQ * PLANE) patch[e] = __builtin_bit_cast(f32x4, v[i]);
    }
    __syncthreads();
  };
  f32x16 acc[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) acc[it] = f32x16{0};
  const int t0 = wave * KK / 4, t1 = (wave + 1) * KK / 4, nt = t1 - t0;
  const float* wptr = p.wp + (size_t)cb * nch * KK * WSTEP + (size_t)lane * KH;
  // step u of this wave = (chunk u / nt, tap t0 + u % nt); weights one step ahead (ping-pong)
  auto goff = [&](int u) -> size_t {
    const int ch = u / nt, t = t0 + (u - ch * nt);
    return ((size_t)ch * KK + t) * WSTEP;
  };
  const int total = nch * nt;
  auto step = [&](float (&cur)[IT][KH], float (&nxt)[IT][KH], int u) {
    const int ch = u / nt, tap = t0 + (u - ch * nt);
    load_frag<IT, KH>(nxt, wptr + goff(min(u + 1, total - 1)));
    const int ky = tap / KS, kx = tap - (tap / KS) * KS;
    const int lo = lbase + ky * PC + kx;
    const f32x4 v0 = patch[(2 * h) * PLANE + lo], v1 = patch[(2 * h + 1) * PLANE + lo];
    const float b[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
    for (int s2 = 0; s2 < KH; ++s2)
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[it] = mfma32(cur[it][s2], b[s2], acc[it]);
  };
  float fa[IT][KH], fb[IT][KH];
  load_frag<IT, KH>(fa, wptr + goff(0));
  // every wave joins every chunk's fill (the barriers); a chunk is nt steps of this wave
  int u = 0;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    fill(ch);
    const int ue = u + nt;
#pragma unroll 1
    for (; u + 1 < ue; u += 2) {
      step(fa, fb, u);
      step(fb, fa, u + 1);
    }
    if (u < ue) {   // odd step count: swap the roles by copying the prefetched set (once per chunk)
      step(fa, fb, u);
      ++u;
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int k = 0; k < KH; ++k) fa[it][k] = fb[it][k];
    }
  }
  // fixed-order reduction: waves 1..3 park their partial sums, wave 0 adds them in wave order
  if (wave > 0) {
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        red[(((wave - 1) * IT + it) * 4 + g) * 64 + lane] =
            f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]};
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll 1
  for (int w = 0; w < 3; ++w) {   // one partial at a time (all LDS reads hoisted spilled)
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 r = red[((w * IT + it) * 4 + g) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += r[e];
      }
  }
  const int oy = oy0 + oyl, ox = ox0 + oxl;
  conv_epilogue<IT, EPI, FX, false>(p, acc, n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
}

// --------------------------------------------------------------------------
// conv_up: ConvTranspose2d k5 s2 p2 op1 (Hout = 2 Hin).  Output pixel
// y = 2a + PY uses taps ky = PY (mod 2) at input row iy = a + (PY + 2 - ky)/2.
// Weight fragments packed [cb][tap][chunk][it][lane][8] (CC = 16).
// --------------------------------------------------------------------------
// Block tile: UP_TH input rows x UP_TW input columns (4 parity classes of 2x as many output pixels).  The
// bf16 path doubles the rows: each wave then runs two 32-pixel tiles per class (up_pt), so a weight
// fragment feeds twice the MFMAs (as in conv_down).
constexpr int UP_TW = 16, UP_PC = UP_TW + 2;
#ifndef ICA_BF_UP3_OLD
#define ICA_BF_UP3_OLD 0   // A/B builds: 1 = the bf16 Z-gather on conv_up3_kernel<true> (rounds 1-5)
#endif
#ifndef ICA_BF_UP_PT
#define ICA_BF_UP_PT 2   // A/B builds: pixel tiles per wave and class of the bf16 conv_up (4: one block per CU)
#endif
template <bool BF>
constexpr int up_pt() { return BF ? ICA_BF_UP_PT : 1; }
template <bool BF>
constexpr int up_th() { return 4 * up_pt<BF>(); }
template <bool BF>
constexpr int up_plane() { return (up_th<BF>() + 2) * UP_PC; }

// bf16: the epilogue parameters (epi_params_to_lds) sit in LDS right after the whole-Cin patch (IT <= 4; the IT = 6
// kernels of the C = 192 layers run one wave per SIMD and load them from global memory: their 75 KB of gamma'
// fragments next to a 320-channel patch would not fit)
template <int IT, bool BF>
constexpr bool up_lg() { return BF && IT <= 4; }
template <int IT, bool BF>
ICA_DEV const f32x4* up_lpar(const f32x4* patch, int nch) {
  return up_lg<IT, BF>() ? patch + 2 * nch * up_plane<BF>() : nullptr;
}

// Generalised over the kernel size: ConvTranspose2d kKS s2 p(KS/2) op1, i.e. the input-gradient
// of a stride-2 KSxKS conv with pad KS/2 (KS = 5: g_s deconvs / g_a dgrad; KS = 3, 1: the dgrad of
// cheng2020's conv3x3 s2 and conv1x1 s2 skips).  Output y = 2a + PY uses taps
// ky = ky0 + 2i, ky0 = (PY + PAD) & 1, at input row iy = a + (PY + PAD - ky) / 2 in [a-1, a+1].
// TH: input rows of the block tile (the patch holds TH + 2 rows)
template <int KS, int PY, int PX, int IT, int EPI, int FX, bool BF, int TH = up_th<BF>()>
// c0, cn (fp32 only): accumulate input-channel chunks [c0, c0 + cn) of the nch (cn = 0: all of them)
ICA_DEV void conv_up_acc(const ConvParams& p, const f32x4* patch, int jt, int cb, int nch,
                         f32x16 (&acc)[up_pt<BF>()][IT], int c0 = 0, int cn = 0) {
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  constexpr int PT = up_pt<BF>(), UP_PLANE = (TH + 2) * UP_PC;
  // pixel tile t of this wave: input rows (jt*PT + t)*2 + (j>>4) of the block tile, columns j&15
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
  constexpr int WSTEP = IT * 64 * 8;
  constexpr int PAD = KS / 2;
  constexpr int KY0 = (PY + PAD) & 1, KX0 = (PX + PAD) & 1;
  constexpr int NY = (KS - KY0 + 1) / 2, NX = (KS - KX0 + 1) / 2;  // taps per axis
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
  // (tap, chunk) sequence flattened
  const int ncw = cn > 0 ? cn : nch;
  const int total = NY * NX * ncw;
  auto woff = [&](int u) -> size_t {
    const int ti = u / ncw, ch = c0 + (u - ti * ncw);
    const int ky = KY0 + 2 * (ti / (NX > 0 ? NX : 1)), kx = KX0 + 2 * (ti % (NX > 0 ? NX : 1));
    return (size_t)(ky * KS + kx) * nch + ch;
  };
  // LDS entry of (tap, chunk) step u for this lane: fp32 entries are 4 channels, bf16 entries 8
  auto poff = [&](int u) -> int {
    const int ti = u / ncw, ch = c0 + (u - ti * ncw);
    const int ky = KY0 + 2 * (ti / (NX > 0 ? NX : 1)), kx = KX0 + 2 * (ti % (NX > 0 ? NX : 1));
    const int pr = a_rel + 1 + (PY + PAD - ky) / 2, pc = b_rel + 1 + (PX + PAD - kx) / 2;
    return (BF ? (2 * ch + h) : (4 * ch + 2 * h)) * UP_PLANE + pr * UP_PC + pc;
  };
  if constexpr (NY * NX > 0) {
    if constexpr (BF) {
      // bf16: 4-set weight-fragment ring, prefetch distance 3 (see conv_down_kernel).  The (tap, chunk) walk
      // u -> (ti, ch) runs on scalar counters (no runtime division by nch: at one 32-cycle MFMA per tile that
      // scalar arithmetic was ~10 SALU per MFMA and kept the MFMA pipe a quarter busy); LDS address = a
      // per-lane base + a wave-uniform (tap, chunk) offset.
      constexpr int NT = NY * NX;
      const bf16x8* wb = reinterpret_cast<const bf16x8*>(p.wp) + (size_t)cb * KS * KS * nch * IT * 64 + lane;
      const int lane_off = h * UP_PLANE + (a_rel + 1) * UP_PC + (b_rel + 1);
      auto tap_lds = [&](int ti) -> int {
        const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
        return ((PY + PAD - ky) / 2) * UP_PC + (PX + PAD - kx) / 2;
      };
      auto tap_w = [&](int ti) -> int {
        const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
        return ky * KS + kx;
      };
      int ti_c = 0, ch_c = 0, ti_w = 0, ch_w = 0;
      auto adv = [&](int& ti, int& ch) {
        ch = ch + 1 == nch ? 0 : ch + 1;
        ti = ch == 0 ? ti + 1 : ti;
      };
      bf16x8 fr[4][IT];
      auto ldw = [&](bf16x8 (&a)[IT]) {   // the fragment set of step (ti_w, ch_w), clamped to the last step
        const bool past = ti_w >= NT;
        const int wo = tap_w(past ? NT - 1 : ti_w) * nch + (past ? nch - 1 : ch_w);
        const bf16x8* w = wb + (size_t)wo * IT * 64;
#pragma unroll
        for (int it = 0; it < IT; ++it) a[it] = ICA_WLOAD_BF(w, it, wo);
        adv(ti_w, ch_w);
      };
      auto step = [&](bf16x8 (&cur)[IT], bf16x8 (&nxt)[IT]) {
        // one scheduling region per step: the ring's loads stay 3 steps ahead of their MFMAs (without it the
        // scheduler sank one set next to its use, a full L2-latency wait per 4 steps)
        __builtin_amdgcn_sched_barrier(0);
        ldw(nxt);
        const int po = lane_off + 2 * ch_c * UP_PLANE + tap_lds(ti_c);
        adv(ti_c, ch_c);
        bf16x8 b[PT];
#pragma unroll
        for (int t = 0; t < PT; ++t) b[t] = f4_as_bf8(patch[po + t * 2 * UP_PC]);   // tile t: 2 rows down
#pragma unroll
        for (int t = 0; t < PT; ++t)
#pragma unroll
          for (int it = 0; it < IT; ++it) acc[t][it] = mfma32bf(cur[it], b[t], acc[t][it]);
      };
      ldw(fr[0]);
      ldw(fr[1]);
      ldw(fr[2]);
      int u = 0;
#pragma unroll 1
      for (; u + 4 <= total; u += 4) {
        step(fr[0], fr[3]);
        step(fr[1], fr[0]);
        step(fr[2], fr[1]);
        step(fr[3], fr[2]);
      }
      if (u < total) step(fr[0], fr[3]);
      if (u + 1 < total) step(fr[1], fr[0]);
      if (u + 2 < total) step(fr[2], fr[1]);
    } else {
      // weight fragments prefetched one step ahead into the other of two register sets (ping-pong)
      const float* wl = p.wp + (size_t)cb * KS * KS * nch * WSTEP + (size_t)lane * 8;
      auto step = [&](float (&cur)[IT][8], float (&nxt)[IT][8], int u) {
        load_frag<IT, 8>(nxt, wl + woff(min(u + 1, total - 1)) * WSTEP);  // unconditional: no phi copies
        const f32x4* pp = patch + poff(u);
        const f32x4 v0 = pp[0], v1 = pp[UP_PLANE];
        const float b[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
          for (int it = 0; it < IT; ++it) acc[0][it] = mfma32(cur[it][s2], b[s2], acc[0][it]);
      };
      float fa[IT][8], fb[IT][8];
      load_frag<IT, 8>(fa, wl + woff(0) * WSTEP);
      int u = 0;
#pragma unroll 1
      for (; u + 1 < total; u += 2) {
        step(fa, fb, u);
        step(fb, fa, u + 1);
      }
      if (u < total) step(fa, fb, u);
    }
  }
}

// the bf16 GDN-backward epilogue's (y, s) loads (conv_epilogue EAG): a two-channel-tile ring (ICA_UP_EAG=0 builds:
// beside their use, the round-4 form, for A/B runs)
#ifndef ICA_UP_EAG
#define ICA_UP_EAG 2
#endif
// the epilogue of class (PY, PX) for the pixel tiles of row group jt
template <int PY, int PX, int IT, int EPI, int FX, bool BF>
ICA_DEV void conv_up_store(const ConvParams& p, f32x16 (&acc)[up_pt<BF>()][IT], int n, int a0, int b0, int jt,
                           int cb, const f32x4* lp) {
  constexpr int PT = up_pt<BF>();
  const int j = threadIdx.x & 31;
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    const int oy = 2 * (a0 + a_rel + 2 * t) + PY, ox = 2 * (b0 + b_rel) + PX;
    conv_epilogue<IT, EPI, FX, BF, 0, up_lg<IT, BF>(), ICA_UP_EAG>(p, acc[t], n, oy, ox, oy < p.Hout && ox < p.Wout,
                                                               cb * IT * 32, lp);
  }
}

template <int KS, int PY, int PX, int IT, int EPI, int FX, bool BF>
ICA_DEV void conv_up_class(const ConvParams& p, const f32x4* patch, int n, int a0, int b0, int jt, int cb,
                           int nch, int tk) {
  f32x16 acc[up_pt<BF>()][IT];
  conv_up_acc<KS, PY, PX, IT, EPI, FX, BF>(p, patch, jt, cb, nch, acc);
  ICA_STAMP_AT(tk - 2);
  conv_up_store<PY, PX, IT, EPI, FX, BF>(p, acc, n, a0, b0, jt, cb, up_lpar<IT, BF>(patch, nch));
  ICA_STAMP_AT(tk - 1);
  (void)tk;
}

// fp32 forward epilogues (stores only): both classes' main loops first, then both epilogues.  The first class's
// output stores, issued before the second class's main loop, made that loop's weight-prefetch waits (vmcnt
// counts stores too) wait for the stores to drain.  The 64 extra accumulator registers fit the 2 waves/SIMD
// these kernels run at.
template <int KS, int IT, int EPI, int FX, bool BF>
constexpr bool up_defer() {
  return !BF && IT <= 4 && FX == 0 &&
         (EPI == EPI_BIAS || EPI == EPI_RELU || EPI == EPI_LRELU || EPI == EPI_IGDN || EPI == EPI_GDN);
}
template <int KS, int PY0, int PX0, int PY1, int PX1, int IT, int EPI, int FX, bool BF>
ICA_DEV void conv_up_pair(const ConvParams& p, const f32x4* patch, int n, int a0, int b0, int jt, int cb, int nch) {
  if constexpr (up_defer<KS, IT, EPI, FX, BF>()) {
    f32x16 acc0[up_pt<BF>()][IT], acc1[up_pt<BF>()][IT];
    conv_up_acc<KS, PY0, PX0, IT, EPI, FX, BF>(p, patch, jt, cb, nch, acc0);
    __builtin_amdgcn_sched_barrier(0);
    conv_up_acc<KS, PY1, PX1, IT, EPI, FX, BF>(p, patch, jt, cb, nch, acc1);
    __builtin_amdgcn_sched_barrier(0);
    conv_up_store<PY0, PX0, IT, EPI, FX, BF>(p, acc0, n, a0, b0, jt, cb, up_lpar<IT, BF>(patch, nch));
    conv_up_store<PY1, PX1, IT, EPI, FX, BF>(p, acc1, n, a0, b0, jt, cb, up_lpar<IT, BF>(patch, nch));
  } else {
    conv_up_class<KS, PY0, PX0, IT, EPI, FX, BF>(p, patch, n, a0, b0, jt, cb, nch, 2);
    __builtin_amdgcn_sched_barrier(0);  // keep the second class's prologue out of the first epilogue
    conv_up_class<KS, PY1, PX1, IT, EPI, FX, BF>(p, patch, n, a0, b0, jt, cb, nch, 4);
  }
}

template <int KS, int IT, int EPI, int FX, bool BF>
__global__ __launch_bounds__(256, ((BF && ICA_BF_UP_PT > 2) ? 1 : conv_min_blocks<KS, IT>())) void conv_up_kernel(ConvParams p) {
  ICA_STAMP_BEGIN();
  extern __shared__ f32x4 patch[];  // fp32: [Cin/4][TH+2][UP_PC] f32x4; bf16: [Cin/8][TH+2][UP_PC] bf16x8
  constexpr int UP_TH = up_th<BF>(), UP_PLANE = up_plane<BF>();
  const int Hh = p.Hin, Wh = p.Win;
  const int tiles_x = (Wh + UP_TW - 1) / UP_TW, tiles_y = (Hh + UP_TH - 1) / UP_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);  // both precisions: the fp32 GDN-bwd layer's HBM reads drop with the halo rows L2-shared
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * UP_TH, b0 = tx * UP_TW;
  const int Cin4 = p.Cin >> 2;  // Cin % 16 == 0 enforced by host
  const int total = (BF ? Cin4 / 2 : Cin4) * UP_PLANE;
  // The patch fill: batches of UP_FB entries per thread whose loads are all issued before their LDS writes
  // (buffer loads with 32-bit offsets into this image; padding pixels read past the descriptor and get
  // zeros), so the fill costs one memory latency per batch instead of one per entry.
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const unsigned qbytes = BF ? 8u : 16u;
  const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(
      reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * qbytes, Cin4 * xplane * qbytes);
  constexpr int UP_FB = 8;
  if constexpr (up_lg<IT, BF>()) epi_params_to_lds<IT, EPI>(p, patch + total, cb * IT * 32);   // published by the fill's barrier
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * UP_FB) {
    u32x4_t v[UP_FB];
#pragma unroll
    for (int i = 0; i < UP_FB; ++i) {
      const int e = e0 + 256 * i;
      const int q = e / UP_PLANE, rem = e - q * UP_PLANE, pr = rem / UP_PC, pc = rem - pr * UP_PC;
      const int iy = a0 - 1 + pr, ix = b0 - 1 + pc;
      const bool ok = e < total && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)(BF ? 2 * q : q) * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * qbytes;
      if constexpr (BF) {  // bf16 activations: two 8-B channel quads per 16-B LDS entry
        const u32x2 lo = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
        const u32x2 hi = __builtin_bit_cast(
            u32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, ok ? vo + xplane * 8u : 0xFFFFFFF0u, 0, 0));
        v[i] = (u32x4_t){lo[0], lo[1], hi[0], hi[1]};
      } else {
        v[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
      }
    }
#pragma unroll
    for (int i = 0; i < UP_FB; ++i) {
      const int e = e0 + 256 * i;
      if (e < total) patch[e] = __builtin_bit_cast(f32x4, v[i]);
    }
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int jt = wave & 1, nch = p.Cin / 16;
  // class pairs balance the tap counts: k5 9+4 | 6+6, k3 1+4 | 2+2
  if (wave < 2) {
    conv_up_pair<KS, 0, 0, 1, 1, IT, EPI, FX, BF>(p, patch, n, a0, b0, jt, cb, nch);
  } else {
    conv_up_pair<KS, 0, 1, 1, 0, IT, EPI, FX, BF>(p, patch, n, a0, b0, jt, cb, nch);
  }
  ICA_STAMP_END();
}

// --------------------------------------------------------------------------
// Small-grid fp32 conv_up: a block computes ONE output-parity class (9 / 6 / 6 / 4 taps) of ONE 32-pixel input
// tile (2 x 16), its 4 waves splitting the input-channel chunks (wave w: chunks [w nch / 4, (w + 1) nch / 4));
// the partial accumulators are summed through LDS in wave order (deterministic) and wave 0 runs the epilogue.
// 8x the blocks of conv_up_kernel (64-pixel tiles, two classes per wave) and 1/4-1/6 of its per-wave MFMA chain,
// for the layers whose plain grid leaves most CUs idle (the fine-tune's 256x256 crops: 16x16 .. 64x64 inputs,
// 32-512 blocks), where the plain kernel runs at the latency of one wave's K chain.
// --------------------------------------------------------------------------
constexpr int UPS_TH = 2, UPS_PLANE = (UPS_TH + 2) * UP_PC;
template <int IT>
constexpr int ups_red_entries() { return 3 * IT * 4 * 64; }   // partial sums of waves 1..3: [w-1][it][quad][lane]
template <int KS, int IT, int EPI, int FX>
__global__ __launch_bounds__(256, 2) void conv_up_small_kernel(ConvParams p) {
  extern __shared__ f32x4 patch[];  // [Cin/4][UPS_TH + 2][UP_PC]; then reused for the partial sums
  const int Hh = p.Hin, Wh = p.Win;
  const int tiles_x = (Wh + UP_TW - 1) / UP_TW, tiles_y = (Hh + UPS_TH - 1) / UPS_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int cls = bid & 3;   // the 4 classes of a tile are neighbouring blocks (shared patch rows in L2)
  bid >>= 2;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * UPS_TH, b0 = tx * UP_TW;
  const int Cin4 = p.Cin >> 2;  // Cin % 16 == 0 enforced by host
  const int total = Cin4 * UPS_PLANE;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  constexpr int FB = 8;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * FB) {
    u32x4_t v[FB];
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const int e = e0 + 256 * i;
      const int q = e / UPS_PLANE, rem = e - q * UPS_PLANE, pr = rem / UP_PC, pc = rem - pr * UP_PC;
      const int iy = a0 - 1 + pr, ix = b0 - 1 + pc;
      const bool ok = e < total && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)q * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
      v[i] = __builtin_bit_cast(u32x4_t, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const int e = e0 + 256 * i;
      if (e < total) patch[e] = __builtin_bit_cast(f32x4, v[i]);
    }
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nch = p.Cin / 16;
  const int lane = threadIdx.x & 63, c0 = wave * nch / 4, cn = (wave + 1) * nch / 4 - c0;
  auto run = [&](auto py_c, auto px_c) __attribute__((always_inline)) {
    constexpr int PY = decltype(py_c)::value, PX = decltype(px_c)::value;
    f32x16 acc[1][IT];
    conv_up_acc<KS, PY, PX, IT, EPI, FX, false, UPS_TH>(p, patch, 0, cb, nch, acc, c0, cn);   // cn >= 1 (host)
    __syncthreads();   // every wave is done with the patch: its LDS now takes the partial sums
    if (wave > 0) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          patch[(((wave - 1) * IT + it) * 4 + g) * 64 + lane] =
              f32x4{acc[0][it][4 * g], acc[0][it][4 * g + 1], acc[0][it][4 * g + 2], acc[0][it][4 * g + 3]};
    }
    __syncthreads();
    if (wave != 0) return;
#pragma unroll 1
    for (int w = 0; w < 3; ++w) {   // one partial at a time (all 48 LDS reads hoisted spilled)
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 r = patch[((w * IT + it) * 4 + g) * 64 + lane];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[0][it][4 * g + e] += r[e];
        }
    }
    const int j = threadIdx.x & 31;
    const int oy = 2 * (a0 + (j >> 4)) + PY, ox = 2 * (b0 + (j & 15)) + PX;
    conv_epilogue<IT, EPI, FX, false>(p, acc[0], n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  switch (cls) {
    case 0: run(I0{}, I0{}); break;
    case 1: run(I0{}, I1{}); break;
    case 2: run(I1{}, I0{}); break;
    default: run(I1{}, I1{}); break;
  }
}

// --------------------------------------------------------------------------
// conv_up to 3 channels (g_s last deconv k5 s2 128->3, and the input-gradient
// of g_a's first conv 3->128).  A naive class decomposition would pad the 3
// output channels to a 32-row MFMA tile (10.7x waste).  Instead:
//   Z[(co,ky,kx)][pixel] = sum_ci W[ci][co][ky][kx] * x[ci][pixel]   (75 x Cin dense GEMM)
//   out[co][2a+py][2b+px] = sum_{ky=py, kx=px (mod 2)} Z[(co,ky,kx)][a+dy, b+dx]
// The block owns a 5x32 input-pixel tile; Z is computed for its 7x34 halo
// tile into LDS (75 x 238 floats = 71400 B, so two blocks share a CU's 160 KB and one block's Z GEMM
// overlaps the other's gather and loads; the 8x32 tile's 102 KB Z allowed one block per CU, whose
// phases then ran back to back).  The 238 halo pixels are 8 MFMA column tiles, 2 per wave (6 rows:
// 9 tiles, 3/2/2/2; fp32 1.21 -> 1.19 ms).  Then each thread of the first 5 rows gathers the 12 outputs
// of one input pixel.  Weight fragments packed [it(3)][chunk][lane][8] with row
// o = it*32 + (lane&31) = co*25 + ky*5 + kx.
// --------------------------------------------------------------------------
constexpr int T3_TH = 5, T3_TW = 32, T3_HR = T3_TH + 2, T3_HC = T3_TW + 2, T3_NPX = T3_HR * T3_HC;  // 238
constexpr int T3_ROWS = 75, T3_JT = (T3_NPX + 31) / 32;                                                // 8
constexpr int T3_NCH_BF = 8;  // bf16 up-front-load path: Cin = 128
constexpr int T3_BLOCKS = (2 * T3_ROWS * T3_NPX * 4 <= 160 * 1024) ? 2 : 1;

// X6: fp32-accurate bf16x6 operands (weights from pack_up3_x6_kernel: three planes [plane][it][chunk][lane][8];
// activations split per chunk in registers), six 32x32x16 MFMAs per 16-channel chunk and row tile instead of
// eight 32x32x2 fp32 ones per 2 channels: the fp32 Z GEMM is MFMA-bound (~1 ms of the 1.3 ms kernel at 512x768)
template <bool BF, bool X6 = false>
__global__ __launch_bounds__(256, T3_BLOCKS) void conv_up3_kernel(ConvParams p) {
  __shared__ float zs[T3_ROWS * T3_NPX];
  const int tiles_x = (p.Win + T3_TW - 1) / T3_TW, tiles_y = (p.Hin + T3_TH - 1) / T3_TH;
  int bid, by;
  xcd_block<BF>(bid, by);
  (void)by;  // one channel block
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * T3_TH, b0 = tx * T3_TW;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Cin4 = p.Cin >> 2, nch = p.Cin / 16;
  const size_t plane = (size_t)p.Hin * p.Win;
  if constexpr (BF) {
    if (nch == T3_NCH_BF) {
      // bf16, Cin = 128 (the N = 128 models): the Z GEMM is latency-bound at one block per CU (the 102 KB Z
      // tile), so every load of the block is issued up front: all 24 weight fragments (once per block, L2) and
      // the 8 chunks of each of this wave's (<= 2) pixel tiles (HBM, buffer loads with 32-bit offsets;
      // out-of-image pixels read past the descriptor and get zeros), then the tiles' MFMAs and Z stores.
      constexpr int MJ = (T3_JT + 3) / 4;
      const bf16x8* wl = reinterpret_cast<const bf16x8*>(p.wp) + lane;
      bf16x8 wa[T3_NCH_BF][3];
#pragma unroll
      for (int ch = 0; ch < T3_NCH_BF; ++ch)
#pragma unroll
        for (int it = 0; it < 3; ++it) wa[ch][it] = wl[((size_t)it * T3_NCH_BF + ch) * 64];
      const unsigned img_bytes = (unsigned)(Cin4 * plane * 8);
      const __amdgpu_buffer_rsrc_t xr =
          uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * img_bytes, img_bytes);
      u32x2 xa[MJ][T3_NCH_BF][2];
#pragma unroll
      for (int k = 0; k < MJ; ++k) {
        const int q = (wave + 4 * k) * 32 + j;
        const int hr = q / T3_HC, hc = q - hr * T3_HC;
        const int iy = a0 - 1 + hr, ix = b0 - 1 + hc;
        const bool ok = wave + 4 * k < T3_JT && q < T3_NPX && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        const unsigned po = pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN) * 8u;
#pragma unroll
        for (int ch = 0; ch < T3_NCH_BF; ++ch)
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const unsigned vo = ok ? po + (unsigned)((4 * ch + 2 * h + e) * plane) * 8u : 0xFFFFFFF0u;
            xa[k][ch][e] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(xr, vo, 0, 0));
          }
      }
#pragma unroll
      for (int k = 0; k < MJ; ++k) {
        const int jt = wave + 4 * k;
        if (jt >= T3_JT) break;
        const int q = jt * 32 + j;
        f32x16 acc[3];
#pragma unroll
        for (int it = 0; it < 3; ++it) acc[it] = f32x16{0};
#pragma unroll
        for (int ch = 0; ch < T3_NCH_BF; ++ch) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, (u32x4_t){xa[k][ch][0][0], xa[k][ch][0][1], xa[k][ch][1][0],
                                                                 xa[k][ch][1][1]});
#pragma unroll
          for (int it = 0; it < 3; ++it) acc[it] = mfma32bf(wa[ch][it], b, acc[it]);
        }
        if (q < T3_NPX) {
#pragma unroll
          for (int it = 0; it < 3; ++it)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int row = it * 32 + acc_row(r, h);
              if (row < T3_ROWS) zs[row * T3_NPX + q] = acc[it][r];
            }
        }
      }
      goto gather;
    }
  }
  for (int jt = wave; jt < T3_JT; jt += 4) {
    const int q = jt * 32 + j;
    const int hr = q / T3_HC, hc = q - hr * T3_HC;
    const int iy = a0 - 1 + hr, ix = b0 - 1 + hc;
    const bool ok = q < T3_NPX && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
    const size_t pix = ok ? (size_t)pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN) : 0;
    const float* xp = p.x + (((size_t)n * Cin4) * plane + pix) * 4;
    f32x16 acc[3];
#pragma unroll
    for (int it = 0; it < 3; ++it) acc[it] = f32x16{0};
    if constexpr (BF) {
      // bf16: the 8 channels a lane loads are the k = 8h..8h+7 slice of ONE 32x32x16 MFMA per tile, so a
      // chunk is 3 MFMAs; the B loads (HBM) and A loads (L2) of 4 chunks are issued before their MFMAs.
      const bf16x8* wl = reinterpret_cast<const bf16x8*>(p.wp) + lane;
      const u32x2* xq = reinterpret_cast<const u32x2*>(p.x) + (((size_t)n * Cin4) * plane + pix);
#pragma unroll 1
      for (int ch0 = 0; ch0 < nch; ch0 += 4) {
        f32x4 v0[4];
        bf16x8 a[4][3];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int ch = min(ch0 + c, nch - 1);
          u32x2 qa = {0u, 0u}, qb = {0u, 0u};   // bf16 activations: 8-B channel quads
          if (ok) {
            qa = xq[(size_t)(4 * ch + 2 * h) * plane];
            qb = xq[(size_t)(4 * ch + 2 * h + 1) * plane];
          }
          v0[c] = __builtin_bit_cast(f32x4, (u32x4_t){qa[0], qa[1], qb[0], qb[1]});
#pragma unroll
          for (int it = 0; it < 3; ++it) a[c][it] = wl[((size_t)it * nch + ch) * 64];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (ch0 + c < nch) {
            const bf16x8 b = f4_as_bf8(v0[c]);
#pragma unroll
            for (int it = 0; it < 3; ++it) acc[it] = mfma32bf(a[c][it], b, acc[it]);
          }
        }
      }
    } else if constexpr (X6) {
      const long pst = 3L * nch * 64;   // fragments per plane
      const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * pst * 16));
      const __amdgpu_buffer_rsrc_t xr = uniform_rsrc(p.x + (size_t)n * Cin4 * plane * 4, (unsigned)(Cin4 * plane * 16));
      const unsigned po = ok ? (unsigned)pix * 16u : 0xFFFFFFF0u;
      auto load = [&](int ch, bf16x8 (&a)[3][3], f32x4& v0, f32x4& v1) {
#pragma unroll
        for (int it = 0; it < 3; ++it)
#pragma unroll
          for (int q = 0; q < 3; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * pst + ((long)it * nch + ch) * 64) * 16));
        const unsigned o0 = ok ? po + (unsigned)((4 * ch + 2 * h) * plane) * 16u : 0xFFFFFFF0u;
        v0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, o0, 0, 0));
        v1 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? o0 + (unsigned)plane * 16u
                                                                                     : 0xFFFFFFF0u, 0, 0));
      };
      auto compute = [&](const bf16x8 (&a)[3][3], const f32x4& v0, const f32x4& v1) {
        const float v[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        bf16x8 b[3];
        split3x8(v, b);
#pragma unroll
        for (int it = 0; it < 3; ++it) acc[it] = mfma_x6(a[it], b, acc[it]);
      };
      bf16x8 aa[3][3], ab[3][3];
      f32x4 xa0, xa1, xb0, xb1;
      load(0, aa, xa0, xa1);
      int ch = 0;
#pragma unroll 1
      for (; ch + 1 < nch; ch += 2) {
        load(ch + 1, ab, xb0, xb1);
        __builtin_amdgcn_sched_barrier(0);
        compute(aa, xa0, xa1);
        load(min(ch + 2, nch - 1), aa, xa0, xa1);
        __builtin_amdgcn_sched_barrier(0);
        compute(ab, xb0, xb1);
      }
      if (ch < nch) compute(aa, xa0, xa1);
    } else {
      const float* wl = p.wp + (size_t)lane * 8;
      // B (activations, straight from HBM: 32 consecutive pixels x 16 B per plane = 512 B
      // coalesced) and A (weights, L2) for chunk ch+1 are loaded while chunk ch computes.
      auto load = [&](int ch, f32x4& v0, f32x4& v1, float (&a)[3][8]) {
        v0 = f32x4{0.f, 0.f, 0.f, 0.f};
        v1 = v0;
        if (ok) {
          v0 = ld4(xp + (size_t)(4 * ch + 2 * h) * plane * 4);
          v1 = ld4(xp + (size_t)(4 * ch + 2 * h + 1) * plane * 4);
        }
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          const float* wt = wl + ((size_t)it * nch + ch) * 512;
          const f32x4 w0 = ld4(wt), w1 = ld4(wt + 4);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            a[it][e] = w0[e];
            a[it][4 + e] = w1[e];
          }
        }
      };
      auto compute = [&](const f32x4& v0, const f32x4& v1, const float (&a)[3][8]) {
        const float b[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
        for (int s2 = 0; s2 < 8; ++s2)
#pragma unroll
          for (int it = 0; it < 3; ++it) acc[it] = mfma32(a[it][s2], b[s2], acc[it]);
      };
      f32x4 pa0, pa1, pb0, pb1;
      float aa[3][8], ab[3][8];
      load(0, pa0, pa1, aa);
      int ch = 0;
#pragma unroll 1
      for (; ch + 1 < nch; ch += 2) {
        load(ch + 1, pb0, pb1, ab);
        compute(pa0, pa1, aa);
        load(min(ch + 2, nch - 1), pa0, pa1, aa);
        compute(pb0, pb1, ab);
      }
      if (ch < nch) compute(pa0, pa1, aa);
    }
    if (q < T3_NPX) {
#pragma unroll
      for (int it = 0; it < 3; ++it)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = it * 32 + acc_row(r, h);
          if (row < T3_ROWS) zs[row * T3_NPX + q] = acc[it][r];
        }
    }
  }
gather:
  __syncthreads();
  // gather: thread -> input pixel (a, b) of the owned tile, 4 classes x 3 channels
  const int al = threadIdx.x / T3_TW, bl = threadIdx.x % T3_TW;
  const int a = a0 + al, b = b0 + bl;
  if (al >= T3_TH || a >= p.Hin || b >= p.Win) return;
  const float bias0 = p.bias ? p.bias[0] : 0.f, bias1 = p.bias ? p.bias[1] : 0.f, bias2 = p.bias ? p.bias[2] : 0.f;
#pragma unroll
  for (int py = 0; py < 2; ++py) {
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      float o0 = 0.f, o1 = 0.f, o2 = 0.f;
#pragma unroll
      for (int ky = py; ky < 5; ky += 2) {
#pragma unroll
        for (int kx = px; kx < 5; kx += 2) {
          const int dy = (py + 2 - ky) / 2, dx = (px + 2 - kx) / 2;
          const int q = (al + 1 + dy) * T3_HC + (bl + 1 + dx);
          const int tap = ky * 5 + kx;
          o0 += zs[(0 * 25 + tap) * T3_NPX + q];
          o1 += zs[(1 * 25 + tap) * T3_NPX + q];
          o2 += zs[(2 * 25 + tap) * T3_NPX + q];
        }
      }
      const int y = 2 * a + py, x = 2 * b + px;
      if (y < p.Hout && x < p.Wout)
        st4(p.y + (((size_t)n * p.Hout + y) * p.Wout + x) * 4, f32x4{o0 + bias0, o1 + bias1, o2 + bias2, 0.f});
    }
  }
}

// --------------------------------------------------------------------------
// conv_up3 on x6 operands, persistent and pipelined (the default for Cin = 128 / 192).  A tile is R = 4 CT - 2 input
// rows x 30 columns; its Z = W^T x (75 x Cin, fp32-accurate bf16x6 MFMAs) covers the (R + 2) x 32 halo, i.e. exactly
// one 32-pixel MFMA column tile per halo row, CT rows per wave (Z in LDS: 75 x 4 CT x 32 floats; the halo costs
// (R + 2) x 32 / (R x 30) = 1.28x at CT = 3 instead of the 5 x 32 tile's 1.49x).  Each block walks its tiles (see the
// tile order below); the activations of its next tile are loaded into the registers of the current one's as each chunk is consumed (one whole
// tile of prefetch distance, no extra registers), so the kernel streams instead of waiting out one HBM round trip per
// chunk (the 5 x 32 kernel ran 8 dependent chunk loads per tile: latency-bound at 0.17 of the x6 ceiling).
// Weights: the pack_up3_x6 fragments, one chunk's 9 fragments a chunk ahead, shared by the CT column tiles.
// --------------------------------------------------------------------------
constexpr int U3_OW = 30, U3_HW = 32;
template <int CT>
constexpr int u3_rows() { return 4 * CT - 2; }
template <int CT>
constexpr int u3_npx() { return 4 * CT * U3_HW; }

// BF: the same persistent pipeline on bf16 operands (config 5's g_s.6 forward / g_a.0 input gradient; bf16 nChw4c
// activations, 8-B channel quads; the ica_pack_up3_bf16 fragments, one plane): one MFMA per chunk and row tile, no
// split.  It replaced conv_up3_kernel<true> (one block of 5 x 32 input pixels, loads up front, 1.2 ms per launch at
// the config-5 shapes).
template <int NCH, int CT, bool BF = false>
__global__ __launch_bounds__(256, 1) void conv_up3_x6p_kernel(ConvParams p) {
  constexpr int R = u3_rows<CT>(), NPX = u3_npx<CT>();
  __shared__ float zs[T3_ROWS * NPX];
  const int tiles_x = (p.Win + U3_OW - 1) / U3_OW, tiles_y = (p.Hin + R - 1) / R;
  const int total = tiles_x * tiles_y * p.N;
  // Tile order (speed only; every tile runs the same instructions whichever block takes it): the grid is 8 x nb
  // blocks, dealt round-robin over the XCDs, so block b runs on XCD b % 8.  XCD x owns one contiguous eighth of the
  // tiles and its nb blocks take them interleaved (block i: tiles i, i + nb, ...), so at any moment an XCD's blocks
  // work on ~nb NEIGHBOURING tiles: the halo lines two tiles share are fetched from HBM once and hit in that XCD's
  // L2 for the other.  (Contiguous runs per block put concurrent tiles ~40 tiles apart: every shared line came from
  // HBM twice, and the 30-column tiles' misaligned 256-B runs cost 1.79x the input bytes.)
  const int nb = (int)(gridDim.x >> 3), xcd = (int)(blockIdx.x & 7), bi = (int)(blockIdx.x >> 3);
  const int q8 = total >> 3, r8 = total & 7;
  const int t_end = xcd * q8 + min(xcd, r8) + q8 + (xcd < r8 ? 1 : 0);
  const int t_begin = xcd * q8 + min(xcd, r8) + bi;
  if (t_begin >= t_end) return;   // block-uniform
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Cin4 = p.Cin >> 2;
  const unsigned plane = (unsigned)p.Hin * p.Win;
  auto coords = [&](int t, int& n, int& a0, int& b0) {
    const int tx = t % tiles_x, r = t / tiles_x;
    a0 = (r % tiles_y) * R;
    b0 = tx * U3_OW;
    n = r / tiles_y;
  };
  // activations of (column tile ct, chunk ch): channels 16 ch + 8 h .. + 7 of halo pixel (row wave + 4 ct, col j).
  // Per tile, once: the image's descriptor and, per column tile, the byte offset of the lane's first quad (chunk 0,
  // quad 2h), or OOB for pixels outside the image and for the "next tile" past the block's run (the loads then
  // return zeros: no branches in the MFMA loop)
  const bool split_in = (p.pl & PL_IN) != 0;
  constexpr unsigned QB = BF ? 8u : 16u;             // bytes per channel quad
  const unsigned qs = plane * QB, cs = 4u * qs;      // second quad, next chunk (bytes)
  constexpr unsigned OOB = 0xFFFFFFF0u;
  auto prep = [&](int t, bool real, __amdgpu_buffer_rsrc_t& r, unsigned (&vb)[CT]) __attribute__((always_inline)) {
    int n, a0, b0;
    coords(real ? t : t_begin, n, a0, b0);
    r = uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * plane * QB, (unsigned)(Cin4 * plane * QB));
    const int ix = b0 - 1 + j;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int iy = a0 - 1 + wave + 4 * ct;
      const bool ok = real && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      vb[ct] = ok ? ((unsigned)(2 * h) * plane + pix_at(iy, ix, p.Hin, p.Win, split_in)) * QB : OOB;
    }
  };
  // fp32: two 16-B quads (8 channels) per (ct, ch); bf16: two 8-B quads, packed into the first
  f32x4 xa[CT][NCH][BF ? 1 : 2];
  auto load = [&](const __amdgpu_buffer_rsrc_t& r, const unsigned (&vb)[CT], int ct, int ch)
      __attribute__((always_inline)) {
    const bool ok = vb[ct] != OOB;
    const unsigned o = vb[ct] + (unsigned)ch * cs;
    if constexpr (BF) {
      const u32x2 lo = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, ok ? o : OOB, 0, 0));
      const u32x2 hi = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, ok ? o + qs : OOB, 0, 0));
      xa[ct][ch][0] = __builtin_bit_cast(f32x4, (u32x4_t){lo[0], lo[1], hi[0], hi[1]});
    } else {
      xa[ct][ch][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? o : OOB, 0, 0));
      xa[ct][ch][BF ? 0 : 1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? o + qs : OOB, 0, 0));
    }
  };
  __amdgpu_buffer_rsrc_t rn;
  unsigned vbn[CT];
  prep(t_begin, true, rn, vbn);
#pragma unroll
  for (int ct = 0; ct < CT; ++ct)
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) load(rn, vbn, ct, ch);
  constexpr long pst = 3L * NCH * 64;   // fragments per plane
  constexpr int NPL = BF ? 1 : 3;        // weight planes
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(NPL * pst * 16));
  int wz = 0;   // a per-tile "zero" (keeps the fragment offsets from being hoisted into SGPRs across the tile loop)
  auto ldw = [&](bf16x8 (&a)[3][3], int ch) {
#pragma unroll
    for (int it = 0; it < 3; ++it)
#pragma unroll
      for (int q = 0; q < NPL; ++q) a[it][q] = ld_bf8(wr, lane * 16, wz + (int)((q * pst + ((long)it * NCH + ch) * 64) * 16));
  };
  auto split = [&](int ct, int ch, bf16x8 (&b)[3]) __attribute__((always_inline)) {
    if constexpr (BF) {
      b[0] = f4_as_bf8(xa[ct][ch][0]);
    } else {
      const float v[8] = {xa[ct][ch][0][0], xa[ct][ch][0][1], xa[ct][ch][0][2], xa[ct][ch][0][3],
                          xa[ct][ch][BF ? 0 : 1][0], xa[ct][ch][BF ? 0 : 1][1], xa[ct][ch][BF ? 0 : 1][2],
                          xa[ct][ch][BF ? 0 : 1][3]};
      split3x8(v, b);
    }
  };
  const float bias0 = p.bias ? p.bias[0] : 0.f, bias1 = p.bias ? p.bias[1] : 0.f, bias2 = p.bias ? p.bias[2] : 0.f;
#pragma unroll 1
  for (int t = t_begin; t < t_end; t += nb) {
    wz = 0;
    asm volatile("" : "+s"(wz));
    prep(t + nb, t + nb < t_end, rn, vbn);
    f32x16 acc[CT][3];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int it = 0; it < 3; ++it) acc[ct][it] = f32x16{0};
    bf16x8 wa[2][3][3];
    ldw(wa[0], 0);
    // software pipeline: the B operand of step (ct, ch) is split during the MFMAs of the step before (interleaved
    // 3 VALU per MFMA); the step's registers then take tile t+1's chunk
    bf16x8 bc[3];
    split(0, 0, bc);
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      if (ch + 1 < NCH) ldw(wa[(ch + 1) & 1], ch + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int nct = ct + 1 < CT ? ct + 1 : 0, nch = ct + 1 < CT ? ch : ch + 1;
        bf16x8 bn[3];
        if (nch < NCH) split(nct, nch, bn);
#pragma unroll
        for (int it = 0; it < 3; ++it) {
          if constexpr (BF) acc[ct][it] = mfma32bf(wa[ch & 1][it][0], bc[0], acc[ct][it]);
          else acc[ct][it] = mfma_x6(wa[ch & 1][it], bc, acc[ct][it]);
        }
        load(rn, vbn, ct, ch);   // the registers just consumed take tile t+1's chunk
        if constexpr (!BF) {
#pragma unroll
          for (int k = 0; k < 18; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // one MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);   // up to three VALU (the next operand's split)
          }
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);     // the two activation loads
        }
        __builtin_amdgcn_sched_barrier(0);
        if (nch < NCH) {
#pragma unroll
          for (int q = 0; q < 3; ++q) bc[q] = bn[q];
        }
      }
    }
    __syncthreads();   // the previous tile's gather is done with zs
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int q = (wave + 4 * ct) * U3_HW + j;
#pragma unroll
      for (int it = 0; it < 3; ++it)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = it * 32 + acc_row(r, h);
          if (row < T3_ROWS) zs[row * NPX + q] = acc[ct][it][r];
        }
    }
    __syncthreads();
    // gather: owned pixel (al, bl) -> its 4 classes x 3 channels; both column parities of a row pair are stored as
    // one 32-B run
    int n, a0, b0;
    coords(t, n, a0, b0);
#pragma unroll 1
    for (int idx = threadIdx.x; idx < R * U3_OW; idx += 256) {
      const int al = idx / U3_OW, bl = idx - al * U3_OW;
      const int a = a0 + al, b = b0 + bl;
      if (a >= p.Hin || b >= p.Win) continue;
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        f32x4 o[2];
#pragma unroll
        for (int px = 0; px < 2; ++px) {
          float o0 = 0.f, o1 = 0.f, o2 = 0.f;
#pragma unroll
          for (int ky = py; ky < 5; ky += 2)
#pragma unroll
            for (int kx = px; kx < 5; kx += 2) {
              const int dy = (py + 2 - ky) / 2, dx = (px + 2 - kx) / 2;
              const int q = (al + 1 + dy) * U3_HW + (bl + 1 + dx);
              const int tap = ky * 5 + kx;
              o0 += zs[(0 * 25 + tap) * NPX + q];
              o1 += zs[(1 * 25 + tap) * NPX + q];
              o2 += zs[(2 * 25 + tap) * NPX + q];
            }
          o[px] = f32x4{o0 + bias0, o1 + bias1, o2 + bias2, 0.f};
        }
        const int y = 2 * a + py, x = 2 * b;
        float* dst = p.y + (((size_t)n * p.Hout + y) * p.Wout + x) * 4;
        if (y < p.Hout) {
          st4(dst, o[0]);
          if (x + 1 < p.Wout) st4(dst + 4, o[1]);
        }
      }
    }
  }
}

// x6 weights for conv_up3: the pack_up3_kernel fragment order, each value split exactly into three bf16 planes
__global__ void pack_up3_x6_kernel(const float* __restrict__ w, __bf16* __restrict__ dst, int Cin, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nch = Cin / 16;
  long t = i;
  const int s = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int ch = t % nch; t /= nch;
  const int row = (int)t * 32 + (lane & 31);
  const int c = ch * 16 + (lane >> 5) * 8 + s;
  float v = 0.f;
  if (row < T3_ROWS) v = w[((size_t)c * 3 + row / 25) * 25 + row % 25];
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  dst[total + i] = b;
  dst[2 * total + i] = (__bf16)(r1 - (float)b);
}

template <typename T>
__global__ void pack_up3_kernel(const float* __restrict__ w, T* __restrict__ dst, int Cin, long total) {
  // w: [Cin][3][5][5] (transposed-conv view); dst[it][chunk][lane][8]
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nch = Cin / 16;
  long t = i;
  const int s = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int ch = t % nch; t /= nch;
  const int it = (int)t;
  const int row = it * 32 + (lane & 31);
  const int c = ch * 16 + (lane >> 5) * 8 + s;
  float v = 0.f;
  if (row < T3_ROWS) {
    const int co = row / 25, tap = row % 25;
    v = w[((size_t)c * 3 + co) * 25 + tap];
  }
  dst[i] = (T)v;
}

// --------------------------------------------------------------------------
// Weight / GDN-parameter packing
// --------------------------------------------------------------------------
// dst fragment (cb, outer, inner, it, lane, s) with
//   order 0 (down): outer = chunk, inner = tap ; order 1 (up): outer = tap, inner = chunk
//   o = cb*IT*32 + it*32 + (lane&31) ; c = chunk*CC + (lane>>5)*KH + s
// value = w[o*so + c*sc + ky*KS + kx]  (0 outside O x C)
template <typename T>
__global__ void pack_conv_kernel(const float* __restrict__ w, T* __restrict__ dst, int O, int C, int KS,
                                 long so, long sc, int IT, int CC, int order, long total, int flip) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int KH = CC / 2, KK = KS * KS;
  const int C4 = (C + 3) / 4, nch = (C4 * 4 + CC - 1) / CC;
  long t = i;
  const int s = t % KH; t /= KH;
  const int lane = t % 64; t /= 64;
  const int it = t % IT; t /= IT;
  int inner, outer;
  if (order == 0) { inner = t % KK; t /= KK; outer = t % nch; t /= nch; }
  else { inner = t % nch; t /= nch; outer = t % KK; t /= KK; }
  const int cb = (int)t;
  const int chunk = order == 0 ? outer : inner;
  const int tap = order == 0 ? inner : outer;
  const int o = cb * IT * 32 + it * 32 + (lane & 31);
  int c = chunk * CC + (lane >> 5) * KH + s;
  int tp = tap;
  if (CC == 4) {
    // C <= 4 input channels (RGB), packed K: slot (step g = tap, s) of lane half h holds the (tap, channel)
    // pair f = 4g + 2s + h of the dense list f = tap*C + channel (zero past KK*C): no zero-padded 4th
    // channel, ceil(KK*C/4) steps instead of KK (conv_down_kernel's fp32 CC = 4 main loop)
    const int f = 4 * tap + 2 * s + (lane >> 5);
    tp = f / C;
    c = f - tp * C;
    if (tp >= KK) c = C;  // past the list: zero
  }
  float v = 0.f;
  const int wt = flip ? KK - 1 - tp : tp;  // flip: spatially reversed kernel (dgrad of a stride-1 conv)
  if (o < O && c < C) v = w[o * so + c * sc + (wt / KS) * KS + (wt % KS)];
  dst[i] = (T)v;
}

// gamma' = max(gamma, 2^-18)^2 - 2^-36 ; beta' = max(beta, bound)^2 - 2^-36
// (NonNegativeParametrizer; utils/ops.py:83-89).  Packed fragment
// G[a][b][lane][r] = M[a*32 + (lane&31)][b*32 + acc_row(r, lane>>5)],
// M = gamma' (transpose == 0) or gamma'^T (transpose == 1).
__global__ void pack_gdn_kernel(const float* __restrict__ gamma, const float* __restrict__ beta, float* __restrict__ gp,
                                float* __restrict__ beta_eff, int C, int transpose, float beta_bound) {
  const int T = C / 32;
  const long total = (long)T * T * 64 * 16;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const float ped = 1.4551915228366852e-11f;  // 2^-36
  const float gbound = 3.814697265625e-06f;   // 2^-18
  if (i < total) {
    long t = i;
    const int r = t % 16; t /= 16;
    const int lane = t % 64; t /= 64;
    const int b = t % T; t /= T;
    const int a = (int)t;
    const int row = a * 32 + (lane & 31), col = b * 32 + acc_row(r, lane >> 5);
    const int gi = transpose ? (col * C + row) : (row * C + col);
    const float g = fmaxf(gamma[gi], gbound);
    gp[i] = fsub_rn(fmul_rn(g, g), ped);
  }
  if (i < C) {
    const float bb = fmaxf(beta[i], beta_bound);
    beta_eff[i] = fsub_rn(fmul_rn(bb, bb), ped);
  }
}

// --------------------------------------------------------------------------
// Host launchers (C ABI)
// --------------------------------------------------------------------------
// Instantiated (geometry, channel tile, epilogue, features) combinations; others return -4/-5.
//   (5,2): bmshj2018 g_a / g_s-dgrad / h_a     (3,1): all 3x3 s1 convs and their dgrads
//   (3,2): cheng2020 strided 3x3               (1,2): cheng2020 strided 1x1 skips
//   (1,1): entropy_parameters 1x1 stack         (5,1): MaskedConv2d context model
template <int KS, int S, int IT, int EPI>
constexpr bool down_base() {
  constexpr bool it_ok = IT == 1 || IT == 3 || IT == 4 || IT == 6;
  constexpr bool gdn = EPI >= EPI_GDN && EPI <= EPI_IGDN_BWD;
  if (!it_ok) return false;
  if (KS == 5 && S == 2) {
    // IT = 6: the C = 192 GDN layers of bmshj2018 q6-8 (g_a forward, g_s input-gradient)
    if (IT == 6) return EPI == EPI_GDN || EPI == EPI_IGDN_BWD;
    // LReLU: the mbt2018 hyper-analysis (h_a.2, CompressAI JointAutoregressiveHierarchicalPriors)
    return gdn ? IT == 4 : (EPI == EPI_BIAS || EPI == EPI_RELU || EPI == EPI_LRELU);
  }
  if (KS == 3 && S == 1) return gdn ? (IT == 4 || IT == 6) : true;
  if (KS == 3 && S == 2) return EPI == EPI_BIAS || EPI == EPI_LRELU;
  if (KS == 1 && S == 2) return EPI == EPI_BIAS;
  if (KS == 1 && S == 1) return EPI == EPI_BIAS || EPI == EPI_LRELU;
  if (KS == 5 && S == 1) return EPI == EPI_BIAS;
  return false;
}
template <int KS, int S, int IT, int EPI, int FX>
constexpr bool down_variant() {
  if (!down_base<KS, S, IT, EPI>()) return false;
  if (FX == 0) return true;
  if (FX == FX_T) return KS == 5 && S == 2 && (EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD);  // bmshj2018 training
  if (!(KS == 3 && S == 1)) return false;
  switch (EPI) {
    case EPI_BIAS: return FX == FX_RES || FX == FX_UNSHUF || FX == (FX_UNSHUF | FX_RES) || FX == FX_PS;
    case EPI_LRELU: return FX == FX_RES || FX == FX_PS;
    case EPI_LRELU_BWD: return FX == FX_MASK;
    case EPI_GDN: case EPI_IGDN: case EPI_GDN_BWD: case EPI_IGDN_BWD: return FX == FX_RES;
    default: return false;
  }
}
// 4-channel chunks only where an RGB image is the conv input
template <int KS, int S>
constexpr bool down_cc4() { return (KS == 5 && S == 2) || (KS == 3 && S == 2) || (KS == 1 && S == 2); }

template <int KS, int S, int IT, int CC, int TW, int EPI, int FX, bool BF, bool X6O = false, int XPT = 1, int NPL = 3>
static int launch_down(const ConvParams& p, hipStream_t st) {
  constexpr int TH = (X6O ? XPT : down_pt<CC, BF>()) * 128 / TW;
  const int tiles = ((p.Wout + TW - 1) / TW) * ((p.Hout + TH - 1) / TH) * p.N;
  dim3 grid(tiles, (p.Cout + IT * 32 - 1) / (IT * 32));
  ICA_LAUNCH((conv_down_kernel<KS, S, IT, CC, TW, EPI, FX, BF, X6O, XPT, NPL>), grid, dim3(256), 0, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

// x6 operands for the k3 s1 conv_downs (cheng2020 g_a / g_s and their input gradients): plain, leaky-ReLU-mask and
// PixelUnshuffle fills with the residual / PixelShuffle extras, IT 4 / 6; the t output (FX_T) and other extras
// return -4 (nothing falls back here: engine_cheng._x6_ok keeps the fp32 pack for launches writing t)
template <int IT, int EPI, int FX, int NPL>
static int pick_tw_down_x6o(const ConvParams& p, hipStream_t st) {
  if constexpr (!down_variant<3, 1, IT, EPI, FX>()) {
    return -4;
  } else {
    // two rows per wave (half the weight-fragment stream per MFMA) where the halved grid still gives every CU
    // >= 4 blocks (k3 lrelu 9.66 -> 8.56 ms, gdn+res 12.05 -> 10.81 ms, gdn_bwd 12.2 -> 10.9 ms at the config-3
    // shapes; the GDN epilogues run tile by tile, the second tile's accumulators held)
    if constexpr (ICA_X6O_PT2 && (ICA_X6O_PT2_GDN || !epi_gdn<EPI>()) && IT >= 4) {
      const int cbs = (p.Cout + IT * 32 - 1) / (IT * 32);
      if (p.Wout >= 32 && p.Wout % 32 == 0) {
        if ((long)(p.Wout / 32) * ((p.Hout + 7) / 8) * p.N * cbs >= 1024)
          return launch_down<3, 1, IT, 16, 32, EPI, FX, false, true, 2, NPL>(p, st);
      } else if ((long)((p.Wout + 15) / 16) * ((p.Hout + 15) / 16) * p.N * cbs >= 1024) {
        return launch_down<3, 1, IT, 16, 16, EPI, FX, false, true, 2, NPL>(p, st);
      }
    }
    if (p.Wout >= 32 && p.Wout % 32 == 0) return launch_down<3, 1, IT, 16, 32, EPI, FX, false, true, 1, NPL>(p, st);
    return launch_down<3, 1, IT, 16, 16, EPI, FX, false, true, 1, NPL>(p, st);
  }
}
// x6 operands for the k3 s2 forwards (cheng2020 g_a.2 / g_a.4 conv1: leaky ReLU, and bias): one row per wave, the
// fill two quads per tap
template <int IT, int NPL>
static int pick_down_x6o_s2(const ConvParams& p, int epi, int fx, hipStream_t st) {
  if (fx != 0) return -4;
  const bool w32 = p.Wout >= 32 && p.Wout % 32 == 0;
  if (epi == EPI_LRELU)
    return w32 ? launch_down<3, 2, IT, 16, 32, EPI_LRELU, 0, false, true, 1, NPL>(p, st)
               : launch_down<3, 2, IT, 16, 16, EPI_LRELU, 0, false, true, 1, NPL>(p, st);
  if (epi == EPI_BIAS)
    return w32 ? launch_down<3, 2, IT, 16, 32, EPI_BIAS, 0, false, true, 1, NPL>(p, st)
               : launch_down<3, 2, IT, 16, 16, EPI_BIAS, 0, false, true, 1, NPL>(p, st);
  return -4;
}
template <int IT, int EPI, int NPL>
static int pick_fx_down_x6o(const ConvParams& p, int fx, hipStream_t st) {
  switch (fx) {
    case 0: return pick_tw_down_x6o<IT, EPI, 0, NPL>(p, st);
    case FX_RES: return pick_tw_down_x6o<IT, EPI, FX_RES, NPL>(p, st);
    case FX_PS: return pick_tw_down_x6o<IT, EPI, FX_PS, NPL>(p, st);
    case FX_MASK: return pick_tw_down_x6o<IT, EPI, FX_MASK, NPL>(p, st);
    case FX_UNSHUF: return pick_tw_down_x6o<IT, EPI, FX_UNSHUF, NPL>(p, st);
    case FX_UNSHUF | FX_RES: return pick_tw_down_x6o<IT, EPI, FX_UNSHUF | FX_RES, NPL>(p, st);
    default: return -4;
  }
}
template <int IT, int NPL>
static int pick_epi_down_x6o(const ConvParams& p, int epi, int fx, hipStream_t st) {
  switch (epi) {
    case EPI_BIAS: return pick_fx_down_x6o<IT, EPI_BIAS, NPL>(p, fx, st);
    case EPI_RELU: return pick_fx_down_x6o<IT, EPI_RELU, NPL>(p, fx, st);
    case EPI_LRELU: return pick_fx_down_x6o<IT, EPI_LRELU, NPL>(p, fx, st);
    case EPI_LRELU_BWD: return pick_fx_down_x6o<IT, EPI_LRELU_BWD, NPL>(p, fx, st);
    case EPI_GDN: return pick_fx_down_x6o<IT, EPI_GDN, NPL>(p, fx, st);
    case EPI_IGDN: return pick_fx_down_x6o<IT, EPI_IGDN, NPL>(p, fx, st);
    case EPI_GDN_BWD: return pick_fx_down_x6o<IT, EPI_GDN_BWD, NPL>(p, fx, st);
    case EPI_IGDN_BWD: return pick_fx_down_x6o<IT, EPI_IGDN_BWD, NPL>(p, fx, st);
    default: return -5;
  }
}
template <int NPL>
static int pick_down_x6o(const ConvParams& p, int it, int epi, int fx, hipStream_t st) {
  if (p.Cin < 16) return -4;
  switch (it) {
    case 1:   // cheng2020 g_s.7, subpel_conv3x3(N, 3, 2): 16 rho rows, PixelShuffle store
      return epi == EPI_BIAS && fx == FX_PS ? pick_tw_down_x6o<1, EPI_BIAS, FX_PS, NPL>(p, st) : -4;
    case 4: return pick_epi_down_x6o<4, NPL>(p, epi, fx, st);
    case 6: return pick_epi_down_x6o<6, NPL>(p, epi, fx, st);
    default: return -4;
  }
}
// the k3 conv_downs on X6O operands: NPL = 3 (x6) or 1 (ICA_PREC_B1)
template <int NPL>
static int pick_x6o(const ConvParams& p, int kind, int KS, int S, int epi, int it, int fx, hipStream_t st) {
  if (kind == 0 && KS == 3 && S == 1) return pick_down_x6o<NPL>(p, it, epi, fx, st);
  if (kind == 0 && KS == 3 && S == 2 && p.fill_mode == 0 && !p.ps) {
    if (it == 6) return pick_down_x6o_s2<6, NPL>(p, epi, fx, st);
    if (it == 4) return pick_down_x6o_s2<4, NPL>(p, epi, fx, st);
  }
  return -4;
}

// small-grid variant (conv_down_split_kernel): outputs of at most 64 x 64 pixels per image.  A per-image
// criterion, so image b of a batch runs the same kernel (and rounds identically) at any batch size.
constexpr int DOWN_SMALL_PX = 64 * 64, UP_SMALL_PX = 64 * 64;
template <int KS, int S, int IT, int EPI, int FX>
static int launch_down_split(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Wout + DS_TW - 1) / DS_TW) * ((p.Hout + DS_TH - 1) / DS_TH) * p.N;
  dim3 grid(tiles, (p.Cout + IT * 32 - 1) / (IT * 32));
  ICA_LAUNCH((conv_down_split_kernel<KS, S, IT, EPI, FX>), grid, dim3(256), 0, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int KS, int S, int IT, int CC, int EPI, int FX, bool BF = false>
static int pick_tw_down(const ConvParams& p, hipStream_t st) {
  if constexpr (!BF && CC == 16 && KS == 5 && S == 2 && (FX == 0 || FX == FX_T) && (IT == 3 || IT == 4 || IT == 6)) {
    if (p.Hout * p.Wout <= DOWN_SMALL_PX) return launch_down_split<KS, S, IT, EPI, FX>(p, st);
  }
  if (p.Wout >= 32 && p.Wout % 32 == 0) return launch_down<KS, S, IT, CC, 32, EPI, FX, BF>(p, st);
  return launch_down<KS, S, IT, CC, 16, EPI, FX, BF>(p, st);
}

// bf16-operand variants: the bmshj2018 g_a forward / g_s input-gradient layers (k5 s2, 16-channel chunks); IT = 6:
// the C = 192 GDN / IGDN-backward layers of q6-8 (one wave per SIMD, the whole register file)
template <int KS, int S, int IT, int EPI, int FX>
constexpr bool down_bf() {
  return KS == 5 && S == 2 && FX == 0 &&
         (((IT == 3 || IT == 4) && (EPI == EPI_BIAS || EPI == EPI_GDN || EPI == EPI_IGDN_BWD)) ||
          (IT == 6 && (EPI == EPI_GDN || EPI == EPI_IGDN_BWD)));
}
// ... and the RGB-input ones (g_a.0 forward, g_s.6 input-gradient): 4-channel tap groups
template <int KS, int S, int IT, int EPI, int FX>
constexpr bool down_bf4() {
  return KS == 5 && S == 2 && FX == 0 && (IT == 4 || IT == 6) && (EPI == EPI_GDN || EPI == EPI_IGDN_BWD);
}

template <int KS, int S, int IT, int EPI, int FX>
static int pick_cc_down(const ConvParams& p, hipStream_t st) {
  if constexpr (!down_variant<KS, S, IT, EPI, FX>()) {
    return -4;
  } else {
    if (p.prec == 1) {
      if (p.Cin <= 4) {
        if constexpr (down_bf4<KS, S, IT, EPI, FX>()) return pick_tw_down<KS, S, IT, 4, EPI, FX, true>(p, st);
        return -4;
      }
      if constexpr (down_bf<KS, S, IT, EPI, FX>()) return pick_tw_down<KS, S, IT, 16, EPI, FX, true>(p, st);
      return -4;
    }
    if (p.Cin <= 4) {
      if constexpr (down_cc4<KS, S>() && (FX == 0 || FX == FX_T)) return pick_tw_down<KS, S, IT, 4, EPI, FX>(p, st);
      return -2;
    }
    // any Cin: the fill zeroes channel groups past Cin/4 and the packer zero-pads weight columns
    // (nChw4c padding lanes are zero), so only the unshuffled view needs whole 16-channel chunks
    if ((FX & FX_UNSHUF) != 0 && p.Cin % 16 != 0) return -2;
    return pick_tw_down<KS, S, IT, 16, EPI, FX>(p, st);
  }
}

template <int KS, int S, int EPI, int FX>
static int pick_it_down(const ConvParams& p, int it, hipStream_t st) {
  switch (it) {
    case 1: return pick_cc_down<KS, S, 1, EPI, FX>(p, st);
    case 3: return pick_cc_down<KS, S, 3, EPI, FX>(p, st);
    case 4: return pick_cc_down<KS, S, 4, EPI, FX>(p, st);
    case 6: return pick_cc_down<KS, S, 6, EPI, FX>(p, st);
    default: return -3;
  }
}

template <int KS, int S, int EPI>
static int pick_fx_down(const ConvParams& p, int it, int fx, hipStream_t st) {
  switch (fx) {
    case 0: return pick_it_down<KS, S, EPI, 0>(p, it, st);
    case FX_RES: return pick_it_down<KS, S, EPI, FX_RES>(p, it, st);
    case FX_PS: return pick_it_down<KS, S, EPI, FX_PS>(p, it, st);
    case FX_MASK: return pick_it_down<KS, S, EPI, FX_MASK>(p, it, st);
    case FX_UNSHUF: return pick_it_down<KS, S, EPI, FX_UNSHUF>(p, it, st);
    case FX_UNSHUF | FX_RES: return pick_it_down<KS, S, EPI, FX_UNSHUF | FX_RES>(p, it, st);
    case FX_T: return pick_it_down<KS, S, EPI, FX_T>(p, it, st);
    default: return -4;
  }
}

template <int KS, int S>
static int pick_epi_down(const ConvParams& p, int it, int epi, int fx, hipStream_t st) {
  switch (epi) {
    case EPI_BIAS: return pick_fx_down<KS, S, EPI_BIAS>(p, it, fx, st);
    case EPI_RELU: return pick_fx_down<KS, S, EPI_RELU>(p, it, fx, st);
    case EPI_GDN: return pick_fx_down<KS, S, EPI_GDN>(p, it, fx, st);
    case EPI_IGDN: return pick_fx_down<KS, S, EPI_IGDN>(p, it, fx, st);
    case EPI_GDN_BWD: return pick_fx_down<KS, S, EPI_GDN_BWD>(p, it, fx, st);
    case EPI_IGDN_BWD: return pick_fx_down<KS, S, EPI_IGDN_BWD>(p, it, fx, st);
    case EPI_LRELU: return pick_fx_down<KS, S, EPI_LRELU>(p, it, fx, st);
    case EPI_LRELU_BWD: return pick_fx_down<KS, S, EPI_LRELU_BWD>(p, it, fx, st);
    default: return -5;
  }
}

static int pick_down(const ConvParams& p, int KS, int S, int it, int epi, int fx, hipStream_t st) {
  if (KS == 5 && S == 2) return pick_epi_down<5, 2>(p, it, epi, fx, st);
  if (KS == 3 && S == 1) return pick_epi_down<3, 1>(p, it, epi, fx, st);
  if (KS == 3 && S == 2) return pick_epi_down<3, 2>(p, it, epi, fx, st);
  if (KS == 1 && S == 2) return pick_epi_down<1, 2>(p, it, epi, fx, st);
  if (KS == 1 && S == 1) return pick_epi_down<1, 1>(p, it, epi, fx, st);
  if (KS == 5 && S == 1) return pick_epi_down<5, 1>(p, it, epi, fx, st);
  return -6;
}

template <int KS, int IT, int EPI, int FX>
static int launch_up_small(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Win + UP_TW - 1) / UP_TW) * ((p.Hin + UPS_TH - 1) / UPS_TH) * p.N;
  dim3 grid(4 * tiles, (p.Cout + IT * 32 - 1) / (IT * 32));
  const size_t lds = (size_t)std::max((p.Cin / 4) * UPS_PLANE, ups_red_entries<IT>()) * sizeof(f32x4);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_small_kernel<KS, IT, EPI, FX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_small_kernel<KS, IT, EPI, FX>), grid, dim3(256), lds, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int KS, int IT, int EPI, int FX, bool BF = false>
static int launch_up(const ConvParams& p, hipStream_t st) {
  if (p.Cin % 16 != 0 || p.Hout != 2 * p.Hin || p.Wout != 2 * p.Win) return -2;
  // small grids (inputs of at most 64 x 64 pixels per image): one class per block over 32-pixel tiles, the
  // input-channel chunks split over the 4 waves (each needs one: Cin >= 64)
  if constexpr (!BF && KS == 5 && (FX == 0 || FX == FX_T) && (IT == 4 || IT == 6)) {
    if (p.Hin * p.Win <= UP_SMALL_PX && p.Cin >= 64) return launch_up_small<KS, IT, EPI, FX>(p, st);
  }
  constexpr int UP_TH = up_th<BF>();
  const int tiles = ((p.Win + UP_TW - 1) / UP_TW) * ((p.Hin + UP_TH - 1) / UP_TH) * p.N;
  dim3 grid(tiles, (p.Cout + IT * 32 - 1) / (IT * 32));
  const size_t lds = ((size_t)(p.Cin / (BF ? 8 : 4)) * up_plane<BF>() +
                      (up_lg<IT, BF>() ? epi_lds_entries<IT, EPI>() : 0)) * sizeof(f32x4);
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_kernel<KS, IT, EPI, FX, BF>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_kernel<KS, IT, EPI, FX, BF>), grid, dim3(256), lds, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

static int pick_up(const ConvParams& p, int KS, int it, int epi, int fx, hipStream_t st) {
  if (p.prec == 1) {  // bf16 operands: the bmshj2018 g_s forward / g_a input-gradient layers
    if (KS != 5 || fx != 0 || (it != 4 && it != 6)) return -4;
    if (it == 6) {   // C = 192 (q6-8): the IGDN forward and GDN input-gradient layers
      switch (epi) {
        case EPI_IGDN: return launch_up<5, 6, EPI_IGDN, 0, true>(p, st);
        case EPI_GDN_BWD: return launch_up<5, 6, EPI_GDN_BWD, 0, true>(p, st);
        default: return -5;
      }
    }
    switch (epi) {
      case EPI_BIAS: return launch_up<5, 4, EPI_BIAS, 0, true>(p, st);
      case EPI_IGDN: return launch_up<5, 4, EPI_IGDN, 0, true>(p, st);
      case EPI_GDN_BWD: return launch_up<5, 4, EPI_GDN_BWD, 0, true>(p, st);
      default: return -5;
    }
  }
  if (KS == 5) {
    if (fx == FX_T && it == 4) {
      if (epi == EPI_GDN_BWD) return launch_up<5, 4, EPI_GDN_BWD, FX_T>(p, st);
      if (epi == EPI_IGDN_BWD) return launch_up<5, 4, EPI_IGDN_BWD, FX_T>(p, st);
    }
    // bmshj2018 q6-8 training (C = 192): the g_a GDN input-gradients with t = dL/dn for the parameter grads
    if (fx == FX_T && it == 6 && epi == EPI_GDN_BWD) return launch_up<5, 6, EPI_GDN_BWD, FX_T>(p, st);
    if (fx != 0) return -4;
    if (it == 1) {
      if (epi == EPI_BIAS) return launch_up<5, 1, EPI_BIAS, 0>(p, st);
      if (epi == EPI_RELU) return launch_up<5, 1, EPI_RELU, 0>(p, st);
      if (epi == EPI_LRELU) return launch_up<5, 1, EPI_LRELU, 0>(p, st);
      return -4;
    }
    if (it == 6) {  // C = 192 (bmshj2018 q6-8: g_s IGDN layers, g_a GDN input-gradients, h_s ReLU deconvs)
      switch (epi) {
        case EPI_BIAS: return launch_up<5, 6, EPI_BIAS, 0>(p, st);
        case EPI_RELU: return launch_up<5, 6, EPI_RELU, 0>(p, st);
        case EPI_LRELU: return launch_up<5, 6, EPI_LRELU, 0>(p, st);  // mbt2018 h_s.0 (M = 192)
        case EPI_IGDN: return launch_up<5, 6, EPI_IGDN, 0>(p, st);
        case EPI_GDN_BWD: return launch_up<5, 6, EPI_GDN_BWD, 0>(p, st);
        default: return -5;
      }
    }
    if (it == 4) {
      switch (epi) {
        case EPI_BIAS: return launch_up<5, 4, EPI_BIAS, 0>(p, st);
        case EPI_RELU: return launch_up<5, 4, EPI_RELU, 0>(p, st);
        case EPI_LRELU: return launch_up<5, 4, EPI_LRELU, 0>(p, st);  // mbt2018 h_s (M = 320, 3M/2)
        case EPI_GDN: return launch_up<5, 4, EPI_GDN, 0>(p, st);
        case EPI_IGDN: return launch_up<5, 4, EPI_IGDN, 0>(p, st);
        case EPI_GDN_BWD: return launch_up<5, 4, EPI_GDN_BWD, 0>(p, st);
        case EPI_IGDN_BWD: return launch_up<5, 4, EPI_IGDN_BWD, 0>(p, st);
        default: return -5;
      }
    }
    return -3;
  }
  if (epi != EPI_BIAS || (fx & ~FX_RES) != 0) return -4;
  if (KS == 3) {
    if (fx == 0) {
      if (it == 1) return launch_up<3, 1, EPI_BIAS, 0>(p, st);
      if (it == 4) return launch_up<3, 4, EPI_BIAS, 0>(p, st);
      if (it == 6) return launch_up<3, 6, EPI_BIAS, 0>(p, st);
    } else {
      if (it == 1) return launch_up<3, 1, EPI_BIAS, FX_RES>(p, st);
      if (it == 4) return launch_up<3, 4, EPI_BIAS, FX_RES>(p, st);
      if (it == 6) return launch_up<3, 6, EPI_BIAS, FX_RES>(p, st);
    }
    return -3;
  }
  if (KS == 1) {
    if (fx != 0) return -4;
    if (it == 1) return launch_up<1, 1, EPI_BIAS, 0>(p, st);
    if (it == 4) return launch_up<1, 4, EPI_BIAS, 0>(p, st);
    if (it == 6) return launch_up<1, 6, EPI_BIAS, 0>(p, st);
    return -3;
  }
  return -6;
}

// fp32-accurate bf16x6 operand kernels (ica_conv_x6.hip)
int ica_conv_x6_dispatch(const ConvParams& p, int kind, int KS, int S, int it, int epi, int fx, hipStream_t st);
int ica_rgb5_bf16_dispatch(const ConvParams& p, int epi, hipStream_t st);
int ica_pack_rgb5_planes(const float* w, void* dst, int O, int C, long so, long sc, int it, int planes, hipStream_t st);

// C-ABI argument block of ica_conv_ex (mirrors include/ica_hip.h)
extern "C" {
#ifdef ICA_CLOCK_STAMP
// diagnostic builds only (scripts/clock_probe.py --bf16): where the stamped kernels of this file put their stamps
int ica_diag_stamp_buffer(unsigned long long* buf, unsigned slots) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(ica_stamp_buf), &buf, sizeof(buf)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(ica_stamp_slots), &slots, sizeof(slots)) != hipSuccess) return -1;
  return 0;
}
#endif

int ica_last_launch(char* name, int cap, unsigned long long* threads) {
  const IcaLaunchRec r = ica_launch_rec();
  ica_launch_rec() = IcaLaunchRec{nullptr, 0, 0};   // consumed: the next query sees only later launches
  if (!r.fn) return 0;
  if (threads) *threads = r.threads;
  if (name && cap > 0) {
    const char* m = hipKernelNameRefByPtr(r.fn, nullptr);
    int st = -1;
    char* d = m ? abi::__cxa_demangle(m, nullptr, nullptr, &st) : nullptr;
    const char* src = (st == 0 && d) ? d : (m ? m : "");
    std::snprintf(name, (size_t)cap, "%s", src);
    std::free(d);
  }
  return r.count;
}

typedef struct ica_conv_args {
  const float* x;
  float* y;
  const float* wp;
  const float* bias;
  const float* gp;
  const float* beta;
  float* save_x;
  float* save_s;
  const float* in_x;
  const float* in_s;
  float* save_t;
  const float* res;
  const float* mask;
  int N, Cin, Hin, Win, Cout, Hout, Wout;
  int kind, KS, S, epi, it, fill_mode, ps;
  int prec;   /* 0 fp32 operands, 1 bf16 operands (fp32 accumulate), 2 bf16x6 (fp32-accurate) */
  int layout; /* parity-split tensors: 1 = x, 2 = the output-layout tensors (ConvParams::pl) */
} ica_conv_args;

// Channel tile (IT = number of 32-channel MFMA row tiles per wave) the conv
// launchers use for a given output-channel count; the packer must agree.
int ica_conv_it(int cout) {
  if (cout <= 32) return 1;
  if (cout % 128 == 0) return 4;
  if (cout % 96 == 0) return 3;
  return 4;
}

static inline int resolve_it(int O, int it) { return it > 0 ? it : ica_conv_it(O); }

size_t ica_pack_conv_weight_size(int O, int C, int KS, int CC, int it) {
  const int IT = resolve_it(O, it);
  const int ncb = (O + IT * 32 - 1) / (IT * 32);
  const int C4 = (C + 3) / 4, nch = (C4 * 4 + CC - 1) / CC;
  return (size_t)ncb * nch * KS * KS * IT * 64 * (CC / 2);
}

int ica_pack_conv_weight(const float* w, float* dst, int O, int C, int KS, long so, long sc, int CC, int order,
                         int flip, int it, hipStream_t st) {
  const int IT = resolve_it(O, it);
  const long total = (long)ica_pack_conv_weight_size(O, C, KS, CC, IT);
  ICA_LAUNCH(pack_conv_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, st, w, dst, O, C, KS, so, sc,
                     IT, CC, order, total, flip);
  ICA_CHECK_LAUNCH();
  return 0;
}

// bf16 tap-group fragments for a conv_down with C <= 4 input channels: [cb][tg][it][lane][8] with
// o = cb*IT*32 + it*32 + (lane&31), tap = 4 tg + 2 (lane>>5) + (s>>2), c = s & 3 (0 past KS*KS or C).
__global__ void pack_conv_tg_kernel(const float* __restrict__ w, __bf16* __restrict__ dst, int O, int C, int KS,
                                    long so, long sc, int IT, long total, int flip) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int KK = KS * KS, TG = (KK + 3) / 4;
  long t = i;
  const int s = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int it = t % IT; t /= IT;
  const int tg = t % TG; t /= TG;
  const int cb = (int)t;
  const int o = cb * IT * 32 + it * 32 + (lane & 31);
  const int tap = 4 * tg + 2 * (lane >> 5) + (s >> 2), c = s & 3;
  float v = 0.f;
  if (o < O && c < C && tap < KK) {
    const int wt = flip ? KK - 1 - tap : tap;
    v = w[o * so + c * sc + (wt / KS) * KS + (wt % KS)];
  }
  dst[i] = (__bf16)v;
}

// bf16 values ica_pack_conv_weight_bf16 writes for W[O][C][KS][KS] (C <= 4: tap groups, else CC = 16 chunks)
size_t ica_pack_conv_weight_bf16_size(int O, int C, int KS, int it) {
  if (C > 4) return ica_pack_conv_weight_size(O, C, KS, 16, it);
  const int IT = resolve_it(O, it);
  const int ncb = (O + IT * 32 - 1) / (IT * 32);
  return (size_t)ncb * ((KS * KS + 3) / 4) * IT * 64 * 8;
}

// bf16 fragments for prec = 1 launches: the same [cb][outer][inner][it][lane][8] order as the fp32 pack
// with CC = 16 (lane half h holds channels 8h..8h+7 of the chunk = the bf16 MFMA k map), each element
// rounded to nearest-even bf16.  dst holds ica_pack_conv_weight_size(O, C, KS, 16, it) bf16 values.
int ica_pack_conv_weight_bf16(const float* w, void* dst, int O, int C, int KS, long so, long sc, int order, int flip,
                              int it, hipStream_t st) {
  const int IT = resolve_it(O, it);
  if (C <= 4) {  // conv_down tap groups (RGB input)
    if (order == 2) {   // the dense tap-row pack of conv_rgb5_bf16 (C <= 3, KS = 5, no flip): one bf16 plane
      if (KS != 5 || flip) return -4;
      return ica_pack_rgb5_planes(w, dst, O, C, so, sc, IT, 1, st);
    }
    if (order != 0) return -4;
    const long tot = (long)ica_pack_conv_weight_bf16_size(O, C, KS, IT);
    ICA_LAUNCH(pack_conv_tg_kernel, dim3((tot + 255) / 256), dim3(256), 0, st, w, reinterpret_cast<__bf16*>(dst),
                       O, C, KS, so, sc, IT, tot, flip);
    ICA_CHECK_LAUNCH();
    return 0;
  }
  const long total = (long)ica_pack_conv_weight_size(O, C, KS, 16, IT);
  ICA_LAUNCH(pack_conv_kernel<__bf16>, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     reinterpret_cast<__bf16*>(dst), O, C, KS, so, sc, IT, 16, order, total, flip);
  ICA_CHECK_LAUNCH();
  return 0;
}

size_t ica_pack_up3_size(int Cin) { return (size_t)3 * (Cin / 16) * 64 * 8; }

// w: transposed-conv weight view [Cin][3][5][5] contiguous (ConvTranspose2d(Cin,3) weight,
// or Conv2d(3,Cin) weight [Cin_out=Cin][3][5][5] used for its input-gradient).
int ica_pack_up3(const float* w, float* dst, int Cin, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  const long total = (long)ica_pack_up3_size(Cin);
  ICA_LAUNCH(pack_up3_kernel<float>, dim3((total + 255) / 256), dim3(256), 0, st, w, dst, Cin, total);
  ICA_CHECK_LAUNCH();
  return 0;
}

// layout: PL_IN = x parity-split (the 3-channel output, the image, is always row-major)
static int up3_layout_ok(int layout, int Hin, int Win) {
  if (layout & ~PL_IN) return -4;
  if ((layout & PL_IN) && ((Hin | Win) & 1)) return -2;
  return 0;
}

int ica_conv_up3(const float* x, float* y, const float* wp, const float* bias, int N, int Cin, int Hin, int Win,
                 int layout, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  if (const int rc = up3_layout_ok(layout, Hin, Win)) return rc;
  ConvParams p{x, y, wp, bias, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, N, Cin, Hin, Win, 3,
               2 * Hin, 2 * Win, nullptr};
  p.pl = layout;
  const int tiles = ((Win + T3_TW - 1) / T3_TW) * ((Hin + T3_TH - 1) / T3_TH) * N;
  ICA_LAUNCH(conv_up3_kernel<false>, dim3(tiles), dim3(256), 0, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

// fp32-accurate bf16x6 variants (prec = 2): three bf16 planes of the fp32 fragment order (3 * ica_pack_up3_size(Cin)
// values)
int ica_pack_up3_x6(const float* w, void* dst, int Cin, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  const long total = (long)ica_pack_up3_size(Cin);
  ICA_LAUNCH(pack_up3_x6_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     reinterpret_cast<__bf16*>(dst), Cin, total);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_conv_up3_x6(const float* x, float* y, const void* wp, const float* bias, int N, int Cin, int Hin, int Win,
                    int layout, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  if (const int rc = up3_layout_ok(layout, Hin, Win)) return rc;
  ConvParams p{x, y, reinterpret_cast<const float*>(wp), bias, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
               N, Cin, Hin, Win, 3, 2 * Hin, 2 * Win, nullptr};
  p.pl = layout;
  auto persistent = [&](auto kern, int R) {   // 8 x nb blocks: nb per XCD, at most one per CU
    const int tiles = ((Win + U3_OW - 1) / U3_OW) * ((Hin + R - 1) / R) * N;
    const int nb = std::max(1, std::min((tiles + 7) / 8, ica_cu_count() / 8));
    ICA_LAUNCH(kern, dim3(8 * nb), dim3(256), 0, st, p);
  };
  if (Cin == 128) {
    persistent(conv_up3_x6p_kernel<8, 3>, u3_rows<3>());
  } else if (Cin == 192) {
    persistent(conv_up3_x6p_kernel<12, 2>, u3_rows<2>());
  } else {
    const int tiles = ((Win + T3_TW - 1) / T3_TW) * ((Hin + T3_TH - 1) / T3_TH) * N;
    ICA_LAUNCH((conv_up3_kernel<false, true>), dim3(tiles), dim3(256), 0, st, p);
  }
  ICA_CHECK_LAUNCH();
  return 0;
}

// bf16-operand variants (prec = 1): fragments in the fp32 order rounded to bf16 (ica_pack_up3_size(Cin) values)
int ica_pack_up3_bf16(const float* w, void* dst, int Cin, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  const long total = (long)ica_pack_up3_size(Cin);
  ICA_LAUNCH(pack_up3_kernel<__bf16>, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     reinterpret_cast<__bf16*>(dst), Cin, total);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_conv_up3_bf16(const float* x, float* y, const void* wp, const float* bias, int N, int Cin, int Hin, int Win,
                      int layout, hipStream_t st) {
  if (Cin % 16 != 0) return -2;
  if (const int rc = up3_layout_ok(layout, Hin, Win)) return rc;
  ConvParams p{x, y, reinterpret_cast<const float*>(wp), bias, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
               N, Cin, Hin, Win, 3, 2 * Hin, 2 * Win, nullptr};
  p.pl = layout;
  if (Cin == 128 && !ICA_BF_UP3_OLD) {   // the persistent pipeline (conv_up3_x6p_kernel<.., BF>)
    const int tiles = ((Win + U3_OW - 1) / U3_OW) * ((Hin + u3_rows<3>() - 1) / u3_rows<3>()) * N;
    const int nb = std::max(1, std::min((tiles + 7) / 8, ica_cu_count() / 8));
    ICA_LAUNCH((conv_up3_x6p_kernel<8, 3, true>), dim3(8 * nb), dim3(256), 0, st, p);
    ICA_CHECK_LAUNCH();
    return 0;
  }
  const int tiles = ((Win + T3_TW - 1) / T3_TW) * ((Hin + T3_TH - 1) / T3_TH) * N;
  ICA_LAUNCH(conv_up3_kernel<true>, dim3(tiles), dim3(256), 0, st, p);
  ICA_CHECK_LAUNCH();
  return 0;
}

// bf16 GDN fragments (prec = 1; the epilogues read the hi part, lo is kept for a bf16x3 variant):
// for channel tiles (a, b), k-step s, part hl (0 = hi, 1 = lo), lane l:
// element j = part of M[a*32 + (l&31)][b*32 + 16s + 8(j>>2) + 4(l>>5) + (j&3)], the k order in which the
// accumulator registers 8s..8s+7 of a 32x32 tile serve as the B operand.  M = gamma' or gamma'^T;
// hi = bf16(g), lo = bf16(g - hi).  gpb holds (C/32)^2 * 2048 bf16; beta_eff as ica_pack_gdn.
__global__ void pack_gdn_bf16_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                     __bf16* __restrict__ gp, float* __restrict__ beta_eff, int C, int transpose,
                                     float beta_bound) {
  const int T = C / 32;
  const long total = (long)T * T * 2048;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const float ped = 1.4551915228366852e-11f;  // 2^-36
  const float gbound = 3.814697265625e-06f;   // 2^-18
  if (i < total) {
    long t = i;
    const int j = t % 8; t /= 8;
    const int lane = t % 64; t /= 64;
    const int hl = t % 2; t /= 2;
    const int s = t % 2; t /= 2;
    const int b = t % T; t /= T;
    const int a = (int)t;
    const int row = a * 32 + (lane & 31), col = b * 32 + 16 * s + 8 * (j >> 2) + 4 * (lane >> 5) + (j & 3);
    const int gi = transpose ? (col * C + row) : (row * C + col);
    const float g0 = fmaxf(gamma[gi], gbound);
    const float g = fsub_rn(fmul_rn(g0, g0), ped);
    __bf16 hi, lo;
    split_bf(g, hi, lo);
    gp[i] = hl ? lo : hi;
  }
  if (i < C) {
    const float bb = fmaxf(beta[i], beta_bound);
    beta_eff[i] = fsub_rn(fmul_rn(bb, bb), ped);
  }
}

int ica_pack_gdn_bf16(const float* gamma, const float* beta, void* gpb, float* beta_eff, int C, int transpose,
                      float beta_bound, hipStream_t st) {
  if (C % 32 != 0) return -2;
  const long total = (long)(C / 32) * (C / 32) * 2048;
  ICA_LAUNCH(pack_gdn_bf16_kernel, dim3((total + 255) / 256), dim3(256), 0, st, gamma, beta,
                     reinterpret_cast<__bf16*>(gpb), beta_eff, C, transpose, beta_bound);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_pack_gdn(const float* gamma, const float* beta, float* gp, float* beta_eff, int C, int transpose,
                 float beta_bound, hipStream_t st) {
  if (C % 32 != 0) return -2;
  const long total = (long)(C / 32) * (C / 32) * 64 * 16;
  ICA_LAUNCH(pack_gdn_kernel, dim3((total + 255) / 256), dim3(256), 0, st, gamma, beta, gp, beta_eff, C,
                     transpose, beta_bound);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_conv_down(const float* x, float* y, const float* wp, const float* bias, int N, int Cin, int Hin, int Win,
                  int Cout, int Hout, int Wout, int KS, int S, int epi, const float* gp, const float* beta,
                  float* save_x, float* save_s, const float* in_x, const float* in_s, float* save_t,
                  hipStream_t st) {
  ConvParams p{x, y, wp, bias, gp, beta, save_x, save_s, in_x, in_s, N, Cin, Hin, Win, Cout, Hout, Wout, save_t};
  const int it = ica_conv_it(Cout);
  if (epi >= EPI_GDN && epi <= EPI_IGDN_BWD && Cout != it * 32) return -4;
  const int fx = (save_x ? FX_RES : 0) | (save_t ? FX_T : 0);
  return pick_down(p, KS, S, it, epi, fx, st);
}

int ica_conv_up(const float* x, float* y, const float* wp, const float* bias, int N, int Cin, int Hin, int Win,
                int Cout, int Hout, int Wout, int epi, const float* gp, const float* beta, float* save_x,
                float* save_s, const float* in_x, const float* in_s, float* save_t, hipStream_t st) {
  ConvParams p{x, y, wp, bias, gp, beta, save_x, save_s, in_x, in_s, N, Cin, Hin, Win, Cout, Hout, Wout, save_t};
  const int it = ica_conv_it(Cout);
  if (epi >= EPI_GDN && epi <= EPI_IGDN_BWD && Cout != it * 32) return -4;
  const int fx = (save_x ? FX_RES : 0) | (save_t ? FX_T : 0);
  return pick_up(p, 5, it, epi, fx, st);
}

int ica_conv_ex(const ica_conv_args* a, hipStream_t st) {
  ConvParams p{a->x,    a->y,    a->wp,   a->bias, a->gp,   a->beta, a->save_x, a->save_s, a->in_x, a->in_s,
               a->N,    a->Cin,  a->Hin,  a->Win,  a->Cout, a->Hout, a->Wout,   a->save_t, a->res,  a->mask,
               a->fill_mode, a->ps, a->prec, a->layout};
  if (a->prec < 0 || a->prec > 3) return -4;
  // parity-split tensors: the k5 s2 layers of the bmshj2018 transforms (plain fill, no PixelShuffle), even planes
  if (a->layout & ~(PL_IN | PL_OUT)) return -4;
  if (a->layout && (a->KS != 5 || a->S != 2 || a->fill_mode != 0 || a->ps)) return -4;
  if (((a->layout & PL_IN) && ((a->Hin | a->Win) & 1)) || ((a->layout & PL_OUT) && ((a->Hout | a->Wout) & 1)))
    return -2;
  const int it = resolve_it(a->Cout, a->it);
  if (a->epi >= EPI_GDN && a->epi <= EPI_IGDN_BWD && a->Cout != it * 32) return -4;
  if (a->ps && (a->Cout % 16 != 0 || !(a->epi == EPI_BIAS || a->epi == EPI_RELU || a->epi == EPI_LRELU))) return -4;
  if (a->fill_mode == 1 && !a->mask) return -4;
  if (a->fill_mode == 2 && a->Cin % 16 != 0) return -2;
  if (a->epi == EPI_LRELU_BWD && !a->in_x) return -4;
  const int fx = ((a->res || a->save_x) ? FX_RES : 0) | (a->ps ? FX_PS : 0) | (a->fill_mode == 1 ? FX_MASK : 0) |
                 (a->fill_mode == 2 ? FX_UNSHUF : 0) | (a->save_t ? FX_T : 0);
  if (a->prec == 2) {
    if (a->kind == 0 && a->KS == 3) return pick_x6o<3>(p, a->kind, a->KS, a->S, a->epi, it, fx, st);
    return ica_conv_x6_dispatch(p, a->kind, a->KS, a->S, it, a->epi, fx, st);
  }
  // bf16 operands over fp32 activations: the k3 conv_downs only, on the x6 pack's hi plane (cheng2020 bf16)
  if (a->prec == 3) return pick_x6o<1>(p, a->kind, a->KS, a->S, a->epi, it, fx, st);
  // bf16 RGB-side conv_down with the dense tap-row pack (hip_ops packs order 2 for exactly these layers)
  if (a->prec == 1 && a->kind == 0 && a->KS == 5 && a->S == 2 && a->Cin <= 3 && a->Cout == 128 && it == 4 && fx == 0 &&
      a->fill_mode == 0 && (a->epi == EPI_BIAS || a->epi == EPI_GDN || a->epi == EPI_IGDN_BWD))
    return ica_rgb5_bf16_dispatch(p, a->epi, st);
  if (a->kind == 0) return pick_down(p, a->KS, a->S, it, a->epi, fx, st);
  if (a->kind == 1) return a->S == 2 ? pick_up(p, a->KS, it, a->epi, fx, st) : -6;
  return -6;
}

}  // extern "C"

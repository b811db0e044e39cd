// fp32-accurate convolutions on the bf16 matrix cores ("x6" operands), for the k5 s2 layers of the bmshj2018
// analysis / synthesis transforms (anchors/utils.py:112-130) and their input gradients.
//
// CDNA4's fp32 MFMA (v_mfma_f32_32x32x2_f32) runs at 1/16 of the bf16 rate.  Every fp32 operand is split exactly
// into three bf16 parts, v = v_hi + v_mid + v_lo (each a round-to-nearest residual: 8 + 8 + 8 significant bits =
// the fp32 significand), and a product is the six partial products with combined weight >= 2^-16:
//     a*b ~ ah*bh + ah*bm + am*bh + ah*bl + al*bh + am*bm
// (dropped: am*bl + al*bm + al*bl, below 2^-24 relative, the size of one fp32 rounding).  bf16 x bf16 products are
// exact in the fp32 accumulator, which adds them as the fp32 MFMA adds its own products, so the result has fp32
// accuracy (measured in round 2: max |err| vs float64 2.3e-6 where a sequential fp32 FMA chain gives 3.1e-6).
// Six v_mfma_f32_32x32x16_bf16 replace eight v_mfma_f32_32x32x2_f32 per 16-deep k step: 192 instead of 512 cycles.
//
// Storage stays fp32 (activations, saved tensors, gradients): the split happens when an input patch is staged into
// LDS (three bf16 planes, 16-B entries of 8 channels) and, for the weights, once per weight version
// (ica_pack_conv_weight_x6: three bf16 fragment planes).  The epilogues are the fp32 ones of ica_conv_epi.h, with
// their GDN normaliser GEMMs on x6 operands as well (gamma' from ica_pack_gdn_x6).
//
//   conv_down_x6 : stride-2 5x5 conv.  Block = 4 waves x 2 pixel tiles x 32 px (8 x 32 outputs), IT x 32 output
//                  channels; K loop = 16-channel LDS chunks x 25 taps, 6 x IT x 2 MFMAs per (chunk, tap).
//   conv_up_x6   : ConvTranspose2d k5 s2 p2 op1 as 4 output-parity classes (9/6/6/4 taps).  Block = 8 x 16 input
//                  pixels (16 x 32 outputs); the channel group (all of Cin, or 64-channel groups) lives in LDS;
//                  each wave runs two classes (9 + 4 or 6 + 6 taps) over 2 pixel tiles.
// One block per CU (the 3-plane patches take 122 / 138 KB of LDS), so each wave has the whole 512-register file.
#include <algorithm>
#include <type_traits>

#include "ica_conv_epi.h"

namespace {

constexpr int X6_PT = 2;                 // 32-pixel tiles per wave
constexpr int XD_TW = 32;
// conv_down_x6 rows per block: 4 waves x PT tiles of one 32-pixel row each.  PT = 1 (128-pixel blocks, 71 KB of LDS)
// where the PT = 2 grid (256-pixel blocks, one per CU) would leave CUs idle (the fine-tune's 64 x 64 layers: 128
// blocks for 256 CUs).  Both run the same MFMA sequence per output.
template <int PT>
constexpr int xd_th() { return 4 * PT; }

// --------------------------------------------------------------------------------------------------------------
// conv_down_x6: weights [plane][cb][chunk][tap][it][lane] bf16x8 (plane stride ps fragments)
// --------------------------------------------------------------------------------------------------------------
template <int IT, int EPI, int PT = X6_PT>
__global__ __launch_bounds__(256, 1) void conv_down_x6_kernel(ConvParams p, long ps) {
  ICA_STAMP_BEGIN();
  constexpr int KS = 5, S = 2, PAD = 2, KK = 25, TW = XD_TW, TH = xd_th<PT>();
  constexpr int PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;
  constexpr int NF = (4 * PLANE + 255) / 256, NB = (NF + 1) / 2;  // fill items per thread, in two batches
  __shared__ f32x4 patch[3 * 2 * PLANE];                          // [plane][half][pixel]: 8 channels as bf16
  const int tiles_x = (p.Wout + TW - 1) / TW, tiles_y = (p.Hout + TH - 1) / TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int Cin4 = (p.Cin + 3) >> 2, nch = (Cin4 * 4 + 15) / 16;
  f32x16 acc[PT][IT];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};

  // patch fill: 16-B buffer loads (32-bit offsets into this image; padding and channel quads past Cin read out of
  // the descriptor's range and return zeros), split into the three planes.  The first batch is issued before the
  // barrier that ends the previous chunk's reads.
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* p2 = reinterpret_cast<u32x2*>(patch);
  auto batch = [&](int ch, int i0, f32x4 (&v)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = threadIdx.x + 256 * (i0 + i);
      const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc, c4 = ch * 4 + q;
      const bool ok = i0 + i < NF && e < 4 * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
  };
  auto put = [&](int i0, const f32x4 (&v)[NB]) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int e = threadIdx.x + 256 * (i0 + i);
      if (i0 + i < NF && e < 4 * PLANE) {
        const int q = e / PLANE, pix = e - q * PLANE;
        u32x2 a, b, c;
        split3(v[i], a, b, c);
        const int ent = (q >> 1) * PLANE + pix;
        p2[(0 * 2 * PLANE + ent) * 2 + (q & 1)] = a;
        p2[(1 * 2 * PLANE + ent) * 2 + (q & 1)] = b;
        p2[(2 * 2 * PLANE + ent) * 2 + (q & 1)] = c;
      }
    }
  };
  const int total = nch * KK;
  // weight fragments through one buffer descriptor: a per-lane byte offset and a wave-uniform (scalar) one
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * total * IT * 64;
  auto ldw = [&](bf16x8 (&a)[IT][3], int g) {
    const int f = wbase + min(g, total - 1) * IT * 64;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int q = 0; q < 3; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + it * 64) * 16));
  };
  // one (chunk, tap) step: the next step's fragments are issued first, a whole step (48 MFMAs) ahead of their use
  // (the barrier keeps the scheduler from sinking them to their first use); hook() issues patch loads after them
  auto step = [&](bf16x8 (&cur)[IT][3], bf16x8 (&nxt)[IT][3], int g, int tap, auto hook) __attribute__((always_inline)) {
    ldw(nxt, g + 1);
    hook();
    __builtin_amdgcn_sched_barrier(0);
    const int ky = tap / 5, kx = tap - ky * 5;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int o = h * PLANE + (S * (wave * PT + t) + ky) * PC + S * j + kx;
      const bf16x8 b[3] = {f4_as_bf8(patch[o]), f4_as_bf8(patch[2 * PLANE + o]), f4_as_bf8(patch[4 * PLANE + o])};
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[t][it] = mfma_x6(cur[it], b, acc[t][it]);
    }
  };
  auto none = []() {};
  // the next chunk's patch is loaded into registers during the last KK - TPF taps of the current one (both
  // batches, a straight-line tail so the waits stay exact) and staged into LDS between two barriers at the chunk
  // boundary: only the split and the LDS writes remain exposed (the fill's HBM latency was ~30 % of the loop)
  constexpr int TPF = 20;
  f32x4 v1[NB], v2[NB];
  auto chunk = [&](bf16x8 (&fa)[IT][3], bf16x8 (&fb)[IT][3], int ch) __attribute__((always_inline)) {
    batch(ch, NB, v2);
    __syncthreads();
    put(0, v1);
    put(NB, v2);
    __syncthreads();
    const int g0 = ch * KK, cn = min(ch + 1, nch - 1);
#pragma unroll 1
    for (int tp = 0; tp < TPF; tp += 2) {
      step(fa, fb, g0 + tp, tp, none);
      step(fb, fa, g0 + tp + 1, tp + 1, none);
    }
    step(fa, fb, g0 + TPF, TPF, [&]() { batch(cn, 0, v1); });
#pragma unroll
    for (int tp = TPF + 1; tp < KK; ++tp) {
      if ((tp - TPF) & 1) step(fb, fa, g0 + tp, tp, none);
      else step(fa, fb, g0 + tp, tp, none);
    }
  };
  static_assert(TPF % 2 == 0 && KK % 2 == 1, "chunk parity: a chunk starting on fa ends with the next fragments in fb");
  bf16x8 fa[IT][3], fb[IT][3];
  batch(0, 0, v1);
  ldw(fa, 0);
  int ch = 0;
#pragma unroll 1
  for (; ch + 1 < nch; ch += 2) {
    chunk(fa, fb, ch);
    chunk(fb, fa, ch + 1);
  }
  if (ch < nch) chunk(fa, fb, ch);
  if constexpr ((EPI == EPI_GDN || EPI == EPI_IGDN) && PT == 2) {
    const int oy[2] = {oy0 + wave * PT, oy0 + wave * PT + 1}, ox[2] = {ox0 + j, ox0 + j};
    gdn_fwd_x6_pair<IT, EPI>(p, acc, n, oy, ox);
  } else {
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int oy = oy0 + wave * PT + t, ox = ox0 + j;
      conv_epilogue<IT, EPI, 0, false, 1>(p, acc[t], n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
    }
  }
  ICA_STAMP_END();
}

// --------------------------------------------------------------------------------------------------------------
// conv_down_x6w: the k5 s2 conv of 128 output channels (IT = 4) on EIGHT waves, two per SIMD.  Block = 4 PT x 32
// output pixels (as conv_down_x6); wave w owns output rows PT (w & 3) .. + PT - 1 and output channels
// 64 (w >> 2) .. + 63, so the SIMD partners w, w + 4 share the pixels and split the channels.
//   * K order: 8-channel chunks x tap PAIRS: a 16-deep MFMA k step is channels 8 c .. 8 c + 7 of taps 2 s (lane
//     half h = 0) and 2 s + 1 (h = 1).  Chunks run in pairs whose two taps 24 form one cross step (lane half h =
//     chunk 2 cp + h), so a pair of 8-channel chunks is 25 steps, as many as one 16-channel chunk x 25 taps.
//   * An 8-channel patch is 61 KB (three bf16 planes), so two fit in LDS: the next chunk's loads are issued at the
//     start of a chunk's 12 steps and split into the other buffer in the middle of them (waves 0-3 after step 3,
//     waves 4-7 after step 8, so the partners' VALU never coincide); three barriers per chunk pair (the cross step
//     reads both buffers).  At one wave per SIMD the 16-channel patch (122 KB, single buffer) was refilled between
//     two barriers, ~11 % of conv_down_x6's time.
//   Measured (kbench_x6, same box): bias 2.82 -> 2.59 ms, GDN 2.92 -> 2.73, IGDN backward 2.94 -> 2.80.  Without
//   the cross step (13 steps per chunk, tap 25 a zero weight: +4 % MFMAs) the same kernel only matched
//   conv_down_x6: its MFMA-busy fraction rose 0.67 -> 0.72-0.76 but the chip held a lower clock.
//   * Patch rows hold their even columns, then their odd ones: the stride-2 pixel reads of 32 lanes are 32
//     consecutive 16-B entries (conflict-free ds_read_b128).
//   * Epilogues: after the last chunk the whole LDS is free; each wave publishes what its partner's channels need
//     (GDN: x = conv + bias; IGDN backward: t) and reads the partner's, so the GDN GEMMs over all 128 channels run
//     with the arithmetic, MFMA order and bits of the single-wave epilogues (gdn_fwd_x6_pair / the wide backward).
// Weights: the tap-pair pack that ica_pack_conv_weight_x6 appends to the order-0 pack for KS = 5, IT = 4:
// [plane][cb][chunk8][step][it][lane] bf16x8, plane stride ps2 fragments, starting 3 ps fragments in.
// --------------------------------------------------------------------------------------------------------------
constexpr int XW_NS = 13;   // tap pairs per 8-channel chunk
__device__ __forceinline__ int xw_pos(int pr, int pc) {   // LDS entry of patch pixel (pr, pc): even columns first
  constexpr int PC = 2 * 31 + 5, PCE = (PC + 1) / 2;
  return pr * PC + ((pc & 1) ? PCE + (pc >> 1) : (pc >> 1));
}
// Epilogue of the 8-wave x6 conv_down (conv_down_x6w): this wave's PT pixel tiles x 64 output channels
// (half chh; the SIMD partner wave ^ 4 holds the other half of the same pixels).  The block's LDS, free by now,
// is the exchange area [wave][t][it][g][lane]: each wave publishes what the partner's channels need (GDN / IGDN:
// x = conv + bias; the GDN / IGDN backward: t) and reads the partner's, so the normaliser GEMMs over all 128
// channels run with the arithmetic and MFMA order of the single-wave epilogues (gdn_fwd_x6_pair / the wide
// backward).  All waves of the block call it (it holds a block barrier).  (The same epilogue behind a conv_up whose
// SIMD partners split the output channels, both classes accumulated first, measured 2-4 % slower than
// conv_up_x6w / conv_up_x6 on every layer: conv_up has no patch refill for a double buffer to hide.)
template <int EPI, int PT>
ICA_DEV void xw_epilogue(const ConvParams& p, f32x16 (&acc)[PT][2], int n, const int (&oy)[PT], int ox,
                         const bool (&ok)[PT], int chh, int wave, int cb, f32x4* lds) {
  constexpr int IT = 4, ITW = 2;
  const int lane = threadIdx.x & 63, h = lane >> 5;
if constexpr (EPI == EPI_BIAS) {
#pragma unroll
  for (int t = 0; t < PT; ++t)
    conv_epilogue<ITW, EPI, 0, false, 2>(p, acc[t], n, oy[t], ox, ok[t], cb * IT * 32 + chh * ITW * 32);
} else {
  static_assert(EPI == EPI_GDN || EPI == EPI_IGDN_BWD || EPI == EPI_GDN_BWD || EPI == EPI_IGDN,
                "conv_down_x6w epilogues: bias, GDN / IGDN, GDN / IGDN backward");
  auto xch = [&](int wv, int t, int it, int g) -> f32x4& { return lds[(((wv * PT + t) * ITW + it) * 4 + g) * 64 + lane]; };
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
  auto ldg = [&](bf16x8 (&a)[3], int ct, int k) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
      a[q] = ld_bf8(grs, lane * 16, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
  };
  unsigned vo[PT], vl[PT];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    vo[t] = ok[t] ? h * plane + pix_at(oy[t], ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u;
    vl[t] = ok[t] ? vo[t] : 0x0FFFFFF0u;   // past the descriptor's range: loads return 0 (never stored)
  }
  // the 8 values (registers 8s..8s+7) of global channel tile itg, k-step s, pixel tile t: this wave's own
  // channel tile from registers, the partner's from the exchange area
  auto kvals = [&](int t, int k, float (&v)[8]) {
    const int itg = k >> 1, s = k & 1, hw = itg / ITW, il = itg - hw * ITW;
    if (hw == chh) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = acc[t][il][8 * s + e];
    } else {
      const f32x4 a = xch(wave ^ 4, t, il, 2 * s), b = xch(wave ^ 4, t, il, 2 * s + 1);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
      v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    }
  };
  if constexpr (EPI == EPI_GDN || EPI == EPI_IGDN) {
    const Img4 Y(p.y, img, n), SS(p.save_s, img, n);
    const __amdgpu_buffer_rsrc_t brs = chan_rsrc(p.bias, p.Cout), ers = chan_rsrc(p.beta, p.Cout);
#pragma unroll
    for (int it = 0; it < ITW; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 bv = ld_chan4(brs, (chh * ITW + it) * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int t = 0; t < PT; ++t) {
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[t][it][4 * g + e] += bv[e];
          xch(wave, t, it, g) = f32x4{acc[t][it][4 * g], acc[t][it][4 * g + 1], acc[t][it][4 * g + 2],
                                      acc[t][it][4 * g + 3]};
        }
      }
    __syncthreads();
#pragma unroll
    for (int il = 0; il < ITW; ++il) {   // this wave's output channel tiles
      const int ct = chh * ITW + il;
      __builtin_amdgcn_sched_barrier(0);
      f32x16 nx[PT];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 ev = ld_chan4(ers, ct * 32 + 8 * g + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int t = 0; t < PT; ++t) nx[t][4 * g + e] = ev[e];
      }
      bf16x8 ga[2][3];
      ldg(ga[0], ct, 0);
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], ct, k + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < PT; ++t) {
          float v[8];
          kvals(t, k, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * v[e];
          bf16x8 xq[3];
          split3x8(v, xq);
          nx[t] = mfma_x6(ga[k & 1], xq, nx[t]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        if (!ok[t]) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 yv, sv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float nv = nx[t][4 * g + e];
            const float sc = (EPI == EPI_GDN) ? __builtin_amdgcn_rsqf(nv) : __builtin_amdgcn_sqrtf(nv);
            sv[e] = sc;
            yv[e] = acc[t][il][4 * g + e] * sc;
          }
          const unsigned ss = (unsigned)(ct * 8 + 2 * g) * plane;
          if (p.save_s) SS.st(vo[t], ss, sv);
          Y.st(vo[t], ss, yv);
        }
      }
    }
  } else {
    const Img4 Y(p.y, img, n), IX(p.in_x, img, n), IS(p.in_s, img, n);
    // pass 1: t of this wave's channels into the exchange area, g*s in place of g
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int it = 0; it < ITW; ++it) {
        __builtin_amdgcn_sched_barrier(0);
        const int itg = chh * ITW + it;
        f32x4 yq[4], sq[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          yq[g] = IX.ld(vl[t], (unsigned)(itg * 8 + 2 * g) * plane);
          sq[g] = IS.ld(vl[t], (unsigned)(itg * 8 + 2 * g) * plane);
        }
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 tv;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float sg = sq[g][e], rs = __builtin_amdgcn_rcpf(sg), xs = yq[g][e] * rs;
            const float gx = acc[t][it][4 * g + e] * xs;
            tv[e] = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (sg * sg * sg) : (0.5f * gx) * rs;
            float gs = acc[t][it][4 * g + e] * sg;
            asm volatile("" : "+v"(gs));   // g*s rounded on its own: never contracted into dx's fma
            acc[t][it][4 * g + e] = gs;
          }
          xch(wave, t, it, g) = tv;
        }
      }
    __syncthreads();
    // pass 2: u for this wave's output channel tiles over all 128 channels of t (exchange area), then
    // dx = g*s + 2 y rcp(s) u
#pragma unroll
    for (int il = 0; il < ITW; ++il) {
      const int jt = chh * ITW + il;
      __builtin_amdgcn_sched_barrier(0);
      f32x16 ux[PT];
#pragma unroll
      for (int t = 0; t < PT; ++t) ux[t] = f32x16{0};
      bf16x8 ga[2][3];
      ldg(ga[0], jt, 0);
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], jt, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        const int itg = k >> 1, s = k & 1, hw = itg / ITW, ilk = itg - hw * ITW;
#pragma unroll
        for (int t = 0; t < PT; ++t) {
          const f32x4 a = xch(hw == chh ? wave : (wave ^ 4), t, ilk, 2 * s),
                      b = xch(hw == chh ? wave : (wave ^ 4), t, ilk, 2 * s + 1);
          const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
          bf16x8 tq[3];
          split3x8(v, tq);
          ux[t] = mfma_x6(ga[k & 1], tq, ux[t]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        if (!ok[t]) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const unsigned ss = (unsigned)(jt * 8 + 2 * g) * plane;
          const f32x4 yv = IX.ld(vo[t], ss), sv = IS.ld(vo[t], ss);
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x2 = 2.0f * (yv[e] * __builtin_amdgcn_rcpf(sv[e]));
            asm volatile("" : "+v"(x2));   // as in the wide form: 2x materialised, then one fma with u
            o[e] = acc[t][il][4 * g + e] + x2 * ux[t][4 * g + e];
          }
          Y.st(vo[t], ss, o);
        }
      }
    }
  }
}
}

// PT = 2: 8 x 32 output pixels per block, two rows per wave; PT = 1 (4 x 32, one row per wave) where the PT = 2 grid
// leaves CUs idle.  Both run the same MFMA and epilogue sequence per output (same bits at any batch size).

template <int EPI, int PT>
__global__ __launch_bounds__(512, 1) void conv_down_x6w_kernel(ConvParams p, long ps2) {
  ICA_STAMP_BEGIN();
  constexpr int IT = 4, ITW = 2, KS = 5, S = 2, PAD = 2, TW = 32, TH = 4 * PT, NS = XW_NS;
  constexpr int PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;   // 19 x 67
  constexpr int PCE = (PC + 1) / 2;
  constexpr int NF = (2 * PLANE + 511) / 512;                                       // fill entries per thread
  constexpr int BUF = 3 * PLANE;                                                    // entries per buffer
  constexpr int XCH = 8 * PT * ITW * 4 * 64;                                        // epilogue exchange entries
  __shared__ f32x4 lds[(2 * BUF > XCH) ? 2 * BUF : XCH];
  const int tiles_x = (p.Wout + TW - 1) / TW, tiles_y = (p.Hout + TH - 1) / TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rp = wave & 3, chh = wave >> 2;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int Cin4 = (p.Cin + 3) >> 2, nch = (Cin4 + 1) >> 1;   // 8-channel chunks
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* l2 = reinterpret_cast<u32x2*>(lds);
  // fill: entry e = (quad q of the chunk, patch pixel); padding and quads past Cin read out of range (zeros)
  auto fill_load = [&](int ch, f32x4 (&v)[NF]) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 512 * i;
      const int q = e >= PLANE ? 1 : 0, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc, c4 = 2 * ch + q;
      const bool ok = e < 2 * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
  };
  auto fill_put = [&](int buf, const f32x4 (&v)[NF]) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 512 * i;
      if (e < 2 * PLANE) {
        const int q = e >= PLANE ? 1 : 0, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
        u32x2 a, b, c;
        split3(v[i], a, b, c);
        const int ent = buf * BUF + xw_pos(pr, pc);
        l2[(ent + 0 * PLANE) * 2 + q] = a;
        l2[(ent + 1 * PLANE) * 2 + q] = b;
        l2[(ent + 2 * PLANE) * 2 + q] = c;
      }
    }
  };
  const int total = (nch >> 1) * 25 + (nch & 1) * NS;   // global K steps (chunk pairs, then a lone chunk)
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps2 * 16));
  const int wbase = cb * total * IT * 64 + chh * ITW * 64;
  auto ldw = [&](bf16x8 (&a)[3], int g, int it) {   // output tile it (of this wave's two) at step g
    const int f = wbase + min(g, total - 1) * IT * 64 + it * 64;
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = ld_bf8(wr, lane * 16, (int)((q * ps2 + f) * 16));
  };
  auto ldb = [&](bf16x8 (&b)[PT][3], int buf, int s) {
    const int tap = min(2 * s + h, KS * KS - 1);   // tap 25: any finite operand (its weights are zero)
    const int ky = tap / KS, kx = tap - ky * KS;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int o = buf * BUF + (S * (PT * rp + t) + ky) * PC + (kx & 1) * PCE + j + (kx >> 1);
      b[t][0] = f4_as_bf8(lds[o]);
      b[t][1] = f4_as_bf8(lds[o + PLANE]);
      b[t][2] = f4_as_bf8(lds[o + 2 * PLANE]);
    }
  };
  f32x16 acc[PT][ITW];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < ITW; ++it) acc[t][it] = f32x16{0};
  bf16x8 w[ITW][3], bq[2][PT][3];
  f32x4 v[NF];
  // one K step: the MFMAs of both pixel tiles per output tile, each tile's fragment set refilled for step g + 1
  // right after its last use (a ring: one step of prefetch distance)
  auto mm = [&](const bf16x8 (&b)[PT][3], int g) __attribute__((always_inline)) {
#pragma unroll
    for (int it = 0; it < ITW; ++it) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < PT; ++t) acc[t][it] = mfma_x6(w[it], b[t], acc[t][it]);
      ldw(w[it], g + 1, it);
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // the 12 tap-pair steps (taps 2 s, 2 s + 1) of the chunk in buffer buf, global steps g0 .. g0 + 11; the other
  // buffer's next chunk (loaded into v beforehand) is split into LDS after step 3 (waves 0-3) or 8 (waves 4-7)
  auto run12 = [&](int buf, int g0, bool put, int pbuf) __attribute__((always_inline)) {
    ldb(bq[0], buf, 0);
#pragma unroll
    for (int s = 0; s < 12; ++s) {
      if (s + 1 < 12) ldb(bq[(s + 1) & 1], buf, s + 1);
      mm(bq[s & 1], g0 + s);
      if (s == 3 && chh == 0 && put) fill_put(pbuf, v);   // the partners split at different steps
      if (s == 8 && chh == 1 && put) fill_put(pbuf, v);
    }
  };
  fill_load(0, v);
#pragma unroll
  for (int it = 0; it < ITW; ++it) ldw(w[it], 0, it);
  fill_put(0, v);
  __syncthreads();
  // K order: chunk PAIRS (2 cp in buffer 0, 2 cp + 1 in buffer 1): 12 tap pairs of the first, the cross step (tap
  // 24 of both chunks, lane half h = chunk), 12 tap pairs of the second -- 25 steps per 16 channels, as many as
  // 16-channel chunks x 25 taps (no zero tap)
  const int npair = nch >> 1;
#pragma unroll 1
  for (int cp = 0; cp < npair; ++cp) {
    const int g0 = cp * 25;
    fill_load(2 * cp + 1, v);
    run12(0, g0, true, 1);
    __syncthreads();                      // chunk 2 cp + 1 is in buffer 1
    {
      bf16x8 bx[PT][3];
#pragma unroll
      for (int t = 0; t < PT; ++t) {      // the cross step: buffer h, tap 24 = (4, 4)
        const int o = h * BUF + (S * (PT * rp + t) + 4) * PC + j + 2;   // ky = kx = 4: even column half
        bx[t][0] = f4_as_bf8(lds[o]);
        bx[t][1] = f4_as_bf8(lds[o + PLANE]);
        bx[t][2] = f4_as_bf8(lds[o + 2 * PLANE]);
      }
      mm(bx, g0 + 12);
    }
    __syncthreads();                      // every wave is done with buffer 0
    const bool more = 2 * cp + 2 < nch;
    if (more) fill_load(2 * cp + 2, v);
    run12(1, g0 + 13, more, 0);
    __syncthreads();                      // chunk 2 cp + 2 is in buffer 0
  }
  if (nch & 1) {                          // a lone last chunk (buffer 0): 13 tap pairs, tap 25 a zero weight
    const int g0 = npair * 25;
    ldb(bq[0], 0, 0);
#pragma unroll
    for (int s = 0; s < 13; ++s) {
      if (s + 1 < 13) ldb(bq[(s + 1) & 1], 0, s + 1);
      mm(bq[s & 1], g0 + s);
    }
    __syncthreads();
  }
  // epilogue: the patch is dead, the LDS is the exchange area [wave][t][it][g][lane]
  int oy[PT];
  bool ok[PT];
  const int ox = ox0 + j;
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    oy[t] = oy0 + PT * rp + t;
    ok[t] = oy[t] < p.Hout && ox < p.Wout;
  }
  xw_epilogue<EPI, PT>(p, acc, n, oy, ox, ok, chh, wave, cb, lds);
  ICA_STAMP_END();
}

// --------------------------------------------------------------------------------------------------------------
// conv_rgb5_x6: the k5 s2 conv whose input is a 3-channel map (g_a.0 forward, the g_s.6 input gradient; 128 output
// channels), with its 75 (tap, channel) pairs packed densely into K: 5 steps of 16, one per tap row ky (the
// PixelUnshuffle(2) k3 view of rounds 2-5 ran 9 steps of 16 for the same 75 pairs: 1.92x the MFMA work).  k = 8 h + e
// of step ky is
//     h = 0: e 0-5 -> (kx 0, c 0-2), (kx 1, c 0-2);   e 6, 7 -> (kx 4, c 0), (kx 4, c 1)
//     h = 1: e 0-5 -> (kx 2, c 0-2), (kx 3, c 0-2);   e 6    -> (kx 4, c 2);  e 7: zero weight
// so the B fragment of lane (h, j) (output pixel ox = ox0 + j) is built in registers from three RGB quads of input
// row 2 oy + ky - 2: columns 2 ox - 2 + 2 h, 2 ox - 1 + 2 h and 2 ox + 2 (one 16-B load each; padding reads past
// the descriptor and returns zeros), split into its three bf16 planes.  A wave computes one 32-pixel output row.
//   Everything the tiles share lives in LDS for the whole launch: the conv weight fragments (3 planes x 5 steps x 4
// row tiles, 60 KB), the x6 gamma' / gamma'^T pack (96 KB), bias and beta' (1 KB) -- 157 KB, one persistent block
// per CU walking a contiguous run of row tiles.  Streamed from L2 per tile instead, those 156 KB of fragments per
// 32-pixel row outran the vector L1 (the per-tile form ran 1.31 / 1.65 ms at the config-2 shapes).
// Weights: [plane][ky][it][lane][e] (pack_conv_rgb5_x6_kernel, ica_pack_conv_weight_x6 order 2), plane stride ps.
// --------------------------------------------------------------------------------------------------------------
constexpr int RGB5_KY = 5, RGB5_IT = 4;
#ifndef RGB5_STAGGER
#define RGB5_STAGGER 0
#endif
#ifndef RGB5_PRIO
#define RGB5_PRIO 0
#endif
#ifndef RGB5_W
#define RGB5_W 0    // 1: the GDN / IGDN forward on the one-wave-per-SIMD kernel (conv_rgb5w_x6_kernel)
#endif
#ifndef RGB5_BJ
#define RGB5_BJ 1   // 1: the backward epilogue's gamma'^T fragments one MFMA group ahead
#endif
#ifndef RGB5_AB
#define RGB5_AB 0   // timing-only A/B builds (scripts/build_variant.sh): 1 = 1/16 of the forward stores, 2 = no GDN GEMM
#endif
constexpr int RGB5_W_BYTES = 3 * RGB5_KY * RGB5_IT * 64 * 16;            // 61440
constexpr int RGB5_G_BYTES = 3 * RGB5_IT * RGB5_IT * 2048;               // 98304
constexpr int RGB5_LDS = RGB5_W_BYTES + RGB5_G_BYTES + 2 * 128 * 4;      // + bias, beta': 160768

// the 15 input quads of one output pixel's 5 tap rows (lane half h's columns)
ICA_DEV void rgb5_load(const ConvParams& p, int n, int oy, int ox, bool valid, f32x4 (&q)[RGB5_KY][3]) {
  const int h = (threadIdx.x & 63) >> 5;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * p.Hin * p.Win * 16, (unsigned)p.Hin * p.Win * 16u);
  const int c0 = 2 * ox - 2 + 2 * h, c2 = 2 * ox + 2;
  const int cols[3] = {c0, c0 + 1, c2};
#pragma unroll
  for (int ky = 0; ky < RGB5_KY; ++ky) {
    const int iy = 2 * oy + ky - 2;
    const bool rok = valid && iy >= 0 && iy < p.Hin;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const bool ok = rok && cols[k] >= 0 && cols[k] < p.Win;
      const unsigned vo = ((unsigned)iy * p.Win + cols[k]) * 16u;
      q[ky][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
  }
}

ICA_DEV bf16x8 lds_frag(const char* lds, int off) { return *reinterpret_cast<const bf16x8*>(lds + off); }

// block prologue: the weight planes, the gamma' pack (GDN epilogues), bias and beta' into LDS (layout above)
template <bool GDN>
ICA_DEV void rgb5_stage(const ConvParams& p, long ps, char* lds) {
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const __amdgpu_buffer_rsrc_t gr = uniform_rsrc(GDN ? p.gp : nullptr, GDN ? RGB5_G_BYTES : 0);
  const __amdgpu_buffer_rsrc_t br = chan_rsrc(p.bias, p.Cout), er = chan_rsrc(GDN ? p.beta : nullptr, p.Cout);
  constexpr int NW = RGB5_W_BYTES / 16, NG = GDN ? RGB5_G_BYTES / 16 : 0, NE = NW + RGB5_G_BYTES / 16 + 64;
  for (int e = threadIdx.x; e < NE; e += blockDim.x) {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
    if (e < NW) {   // plane pl, byte b of the plane
      const int pl = e / (NW / 3), b = (e - pl * (NW / 3)) * 16;
      v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, (int)(pl * ps * 16) + b, 0, 0));
    } else if (e < NW + RGB5_G_BYTES / 16) {
      if (NG) v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(gr, (e - NW) * 16, 0, 0));
    } else {
      const int k = e - NW - RGB5_G_BYTES / 16;   // 0-31 bias quads, 32-63 beta' quads
      v = k < 32 ? ld_chan4(br, 4 * k) : ld_chan4(er, 4 * (k - 32));
    }
    *reinterpret_cast<f32x4*>(lds + (size_t)e * 16) = v;
  }
  __syncthreads();
}

// the 5-step main loop, weight fragments from LDS one step ahead
ICA_DEV void rgb5_main(const char* lds, const f32x4 (&q)[RGB5_KY][3], f32x16 (&acc)[RGB5_IT]) {
  constexpr int IT = RGB5_IT, PS = RGB5_W_BYTES / 3;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  auto ldw = [&](bf16x8 (&a)[IT][3], int g) {
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[it][pl] = lds_frag(lds, pl * PS + ((g * IT + it) * 64 + lane) * 16);
  };
  bf16x8 fa[IT][3], fb[IT][3];
  ldw(fa, 0);
  auto step = [&](bf16x8 (&cur)[IT][3], bf16x8 (&nxt)[IT][3], int ky) __attribute__((always_inline)) {
    if (ky + 1 < RGB5_KY) ldw(nxt, ky + 1);
    __builtin_amdgcn_sched_barrier(0);   // the scheduler otherwise hoists every step's LDS reads (spills)
    const f32x4 a = q[ky][0], b = q[ky][1], c = q[ky][2];
    const float v[8] = {a[0], a[1], a[2], b[0], b[1], b[2], h ? c[2] : c[0], h ? 0.f : c[1]};
    bf16x8 bs[3];
    split3x8(v, bs);
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[it] = mfma_x6(cur[it], bs, acc[it]);
  };
#pragma unroll
  for (int ky = 0; ky < RGB5_KY; ++ky) {
    if (ky & 1) step(fb, fa, ky);
    else step(fa, fb, ky);
  }
}

// bias / GDN / IGDN forward epilogue of one row tile, parameters from LDS (narrow: 256 registers, one normaliser
// tile at a time, x^2 split once per k-step; the ops and MFMA order of gdn_fwd_x6_tile_narrow)
template <int EPI>
ICA_DEV void rgb5_epi_fwd(const ConvParams& p, const char* lds, f32x16 (&acc)[RGB5_IT], int n, int oy, int ox,
                          bool valid) {
  constexpr int IT = RGB5_IT;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n), SS(p.save_s, img, n);
  const f32x4* bq = reinterpret_cast<const f32x4*>(lds + RGB5_W_BYTES + RGB5_G_BYTES);   // [32 bias][32 beta'] quads
  const unsigned vo = h * plane + (valid ? pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u);
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = bq[it * 8 + 2 * g + h];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += bv[e];
    }
  if constexpr (EPI == EPI_BIAS) {
    if (valid) {
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int g = 0; g < 4; ++g)
          Y.st(vo, (unsigned)(it * 8 + 2 * g) * plane,
               f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]});
    }
    return;
  } else {
    const char* gl = lds + RGB5_W_BYTES;
    bf16x8 xs2[IT][2][3];
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = acc[it][8 * s + j] * acc[it][8 * s + j];
        split3x8(v, xs2[it][s]);
      }
    auto ldg = [&](bf16x8 (&a)[3], int ct, int k) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[pl] = lds_frag(gl, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + pl * IT * IT * 2048 + lane * 16);
    };
#pragma unroll
    for (int ct = 0; ct < IT; ++ct) {
      __builtin_amdgcn_sched_barrier(0);
      f32x16 nx;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 ev = bq[32 + ct * 8 + 2 * g + h];
#pragma unroll
        for (int e = 0; e < 4; ++e) nx[4 * g + e] = ev[e];
      }
      bf16x8 ga[2][3];
#if RGB5_AB != 2 && RGB5_AB != 3
      ldg(ga[0], ct, 0);
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], ct, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        nx = mfma_x6(ga[k & 1], xs2[k >> 1][k & 1], nx);
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
      if (valid) {
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
#if RGB5_AB == 1
          if (ct == 0 && g == 0) {
            if (p.save_s) SS.st(vo, ss, sv);
            Y.st(vo, ss, yv);
          }
#else
          if (p.save_s) SS.st(vo, ss, sv);
          Y.st(vo, ss, yv);
#endif
        }
      }
    }
  }
}

// the same epilogue at one wave per SIMD (512 registers): every normaliser tile at once (4 accumulation chains), x^2
// split one k-step at a time (the round's 8 values feed all 4 output tiles), gamma' fragments from LDS one output
// tile ahead; the ops of the narrow form, the MFMA order of gdn_fwd_x6_pair
template <int EPI>
ICA_DEV void rgb5_epi_fwd_wide(const ConvParams& p, const char* lds, f32x16 (&acc)[RGB5_IT], int n, int oy, int ox,
                               bool valid) {
  constexpr int IT = RGB5_IT;
  static_assert(EPI == EPI_GDN || EPI == EPI_IGDN, "forward GDN epilogues");
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n), SS(p.save_s, img, n);
  const f32x4* bq = reinterpret_cast<const f32x4*>(lds + RGB5_W_BYTES + RGB5_G_BYTES);   // [32 bias][32 beta'] quads
  const unsigned vo = h * plane + (valid ? pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u);
  const char* gl = lds + RGB5_W_BYTES;
  f32x16 nx[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 bv = bq[it * 8 + 2 * g + h], ev = bq[32 + it * 8 + 2 * g + h];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[it][4 * g + e] += bv[e];
        nx[it][4 * g + e] = ev[e];
      }
    }
  auto ldg = [&](bf16x8 (&a)[3], int ct, int k) {
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      a[pl] = lds_frag(gl, (((ct * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + pl * IT * IT * 2048 + lane * 16);
  };
  bf16x8 ga[2][3];
  ldg(ga[0], 0, 0);
#pragma unroll
  for (int k = 0; k < 2 * IT; ++k) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = acc[k >> 1][8 * (k & 1) + j] * acc[k >> 1][8 * (k & 1) + j];
    bf16x8 xq[3];
    split3x8(v, xq);
#pragma unroll
    for (int ct = 0; ct < IT; ++ct) {
      const int r = k * IT + ct;
      if (r + 1 < 2 * IT * IT) ldg(ga[(r + 1) & 1], (r + 1) % IT, (r + 1) / IT);
      __builtin_amdgcn_sched_barrier(0);
      nx[ct] = mfma_x6(ga[r & 1], xq, nx[ct]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  if (valid) {
#pragma unroll
    for (int ct = 0; ct < IT; ++ct)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 yv, sv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float nv = nx[ct][4 * g + e];
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

// GDN / IGDN backward epilogue of one row tile (the wide form of gdn_bwd_x6_wide, 512 registers), gamma'^T
// fragments from LDS one round ahead
template <int EPI>
ICA_DEV void rgb5_epi_bwd(const ConvParams& p, const char* lds, f32x16 (&acc)[RGB5_IT], int n, int oy, int ox,
                          bool valid, const f32x4 (&yq)[RGB5_IT][4], const f32x4 (&sq)[RGB5_IT][4]) {
  constexpr int IT = RGB5_IT;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n);
  const unsigned vo = valid ? h * plane + pix_at(oy, ox, p.Hout, p.Wout, p.pl & PL_OUT) : 0u;
  f32x16 xx[IT];
  bf16x8 tq[IT][2][3];
  float tw[8];
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
  const char* gl = lds + RGB5_W_BYTES;
  f32x16 ux[IT];
#pragma unroll
  for (int jt = 0; jt < IT; ++jt) ux[jt] = f32x16{0};
  __builtin_amdgcn_sched_barrier(0);
#if RGB5_BJ
  // fragments one MFMA group (k, jt) ahead: 24 registers instead of two rounds' 96
  bf16x8 ga[2][3];
  auto ldg = [&](bf16x8 (&a)[3], int r) {
    const int k = r / IT, jt = r % IT;
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
      a[pl] = lds_frag(gl, (((jt * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + pl * IT * IT * 2048 + lane * 16);
  };
  ldg(ga[0], 0);
#pragma unroll
  for (int r = 0; r < 2 * IT * IT; ++r) {
    if (r + 1 < 2 * IT * IT) ldg(ga[(r + 1) & 1], r + 1);
    __builtin_amdgcn_sched_barrier(0);
    const int k = r / IT, jt = r % IT;
    ux[jt] = mfma_x6(ga[r & 1], tq[k >> 1][k & 1], ux[jt]);
  }
#else
  bf16x8 ga[2][IT][3];
  auto ldg = [&](bf16x8 (&a)[IT][3], int k) {
#pragma unroll
    for (int jt = 0; jt < IT; ++jt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[jt][pl] = lds_frag(gl, (((jt * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + pl * IT * IT * 2048 + lane * 16);
  };
  ldg(ga[0], 0);
#pragma unroll
  for (int k = 0; k < 2 * IT; ++k) {
    if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], k + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jt = 0; jt < IT; ++jt) ux[jt] = mfma_x6(ga[k & 1][jt], tq[k >> 1][k & 1], ux[jt]);
  }
#endif
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

// forward (bias / GDN / IGDN): 8 waves (two per SIMD: one wave's loads and stores overlap the other's MFMAs), each
// wave a sequence of row tiles
template <int EPI>
__global__ __launch_bounds__(512, 1) void conv_rgb5_x6_kernel(ConvParams p, long ps, int nblk) {
  extern __shared__ __attribute__((aligned(16))) char rgb5_lds[];
  constexpr bool GDN = EPI == EPI_GDN || EPI == EPI_IGDN;
  rgb5_stage<GDN>(p, ps, rgb5_lds);
  const int tiles_x = (p.Wout + 31) / 32, total = tiles_x * p.Hout * p.N, per = (total + nblk - 1) / nblk;
  int b, cb;
  xcd_block<true>(b, cb);
  const int t_end = min(total, b * per + per), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#if RGB5_STAGGER > 0
  // the SIMD partners (waves w, w + 4) run the same tile program and would stay in lockstep, both in their MFMA
  // phase, then both in their store phase; waves 4-7 start RGB5_STAGGER x 4096 cycles late
  if (wave >= 4) {
#pragma unroll 1
    for (int i = 0; i < RGB5_STAGGER; ++i) __builtin_amdgcn_s_sleep(64);
  }
#endif
#if RGB5_PRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll 1
  for (int t = b * per + wave; t < t_end; t += 8) {
    const int tx = t % tiles_x, r = t / tiles_x;
    const int oy = r % p.Hout, n = r / p.Hout, ox = tx * 32 + (threadIdx.x & 31);
    const bool valid = ox < p.Wout;
    f32x4 q[RGB5_KY][3];
    rgb5_load(p, n, oy, ox, valid, q);
    f32x16 acc[RGB5_IT];
#pragma unroll
    for (int it = 0; it < RGB5_IT; ++it) acc[it] = f32x16{0};
#if RGB5_AB == 3
#pragma unroll
    for (int it = 0; it < RGB5_IT; ++it) acc[it] = f32x16{q[it][0][0] + q[4][1][1]};
#else
    rgb5_main(rgb5_lds, q, acc);
#endif
    rgb5_epi_fwd<EPI>(p, rgb5_lds, acc, n, oy, ox, valid);
  }
}

// GDN / IGDN forward at one wave per SIMD: tile i+1's input quads are issued before tile i's epilogue, so the wait
// for them does not include tile i's stores (vmcnt counts loads and stores together, in order: loaded after the
// stores, every tile start waited for the previous tile's stores to complete, and the stores never overlapped the
// MFMAs)
template <int EPI>
__global__ __launch_bounds__(256, 1) void conv_rgb5w_x6_kernel(ConvParams p, long ps, int nblk) {
  extern __shared__ __attribute__((aligned(16))) char rgb5_lds[];
  rgb5_stage<true>(p, ps, rgb5_lds);
  const int tiles_x = (p.Wout + 31) / 32, total = tiles_x * p.Hout * p.N, per = (total + nblk - 1) / nblk;
  int b, cb;
  xcd_block<true>(b, cb);
  const int t_end = min(total, b * per + per), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto coords = [&](int t, int& n, int& oy, int& ox) {
    const int tx = t % tiles_x, r = t / tiles_x;
    oy = r % p.Hout;
    n = r / p.Hout;
    ox = tx * 32 + (threadIdx.x & 31);
  };
  int t = b * per + wave;
  if (t >= t_end) return;   // wave-uniform; no barrier follows
  f32x4 q[RGB5_KY][3];
  {
    int n, oy, ox;
    coords(t, n, oy, ox);
    rgb5_load(p, n, oy, ox, ox < p.Wout, q);
  }
#pragma unroll 1
  for (; t < t_end; t += 4) {
    int n, oy, ox;
    coords(t, n, oy, ox);
    const bool valid = ox < p.Wout;
    f32x16 acc[RGB5_IT];
#pragma unroll
    for (int it = 0; it < RGB5_IT; ++it) acc[it] = f32x16{0};
    rgb5_main(rgb5_lds, q, acc);
    if (t + 4 < t_end) {
      int n1, oy1, ox1;
      coords(t + 4, n1, oy1, ox1);
      rgb5_load(p, n1, oy1, ox1, ox1 < p.Wout, q);
    }
    rgb5_epi_fwd_wide<EPI>(p, rgb5_lds, acc, n, oy, ox, valid);
  }
}

// bf16 operands (config 5's RGB end, the targeted ROI attack's g_a.0 forward / g_s.6 input gradient): the same dense
// tap-row K and persistent row-tile walk; B = the 8 RGB values rounded to bf16 (one plane), weights one bf16 plane
// (plane 0 of the x6 split = round-to-nearest bf16(w)), the bf16 conv path's epilogues (bf16 y / s / dx nChw4c;
// bias, beta' and the gamma' / gamma'^T hi fragments from LDS: epi_params_to_lds).  7 tap-group MFMAs per tile
// (pack_conv_tg_kernel) become 5; the per-tile weight fragment loads become one LDS copy per CU.
constexpr int RGB5B_W_BYTES = RGB5_KY * RGB5_IT * 64 * 16;   // 20480

template <int EPI>
constexpr int rgb5b_lds_bytes() { return RGB5B_W_BYTES + epi_lds_entries<RGB5_IT, EPI>() * 16; }

template <int EPI>
__global__ __launch_bounds__(512, 1) void conv_rgb5_bf16_kernel(ConvParams p, int nblk) {
  extern __shared__ __attribute__((aligned(16))) char rgb5_lds[];
  constexpr int IT = RGB5_IT;
  {
    const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)RGB5B_W_BYTES);
    for (int e = threadIdx.x; e < RGB5B_W_BYTES / 16; e += blockDim.x)
      *reinterpret_cast<f32x4*>(rgb5_lds + (size_t)e * 16) =
          __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, e * 16, 0, 0));
  }
  const f32x4* lp = reinterpret_cast<const f32x4*>(rgb5_lds + RGB5B_W_BYTES);
  if (threadIdx.x < 256) epi_params_to_lds<IT, EPI>(p, reinterpret_cast<f32x4*>(rgb5_lds + RGB5B_W_BYTES), 0);
  __syncthreads();
  const int tiles_x = (p.Wout + 31) / 32, total = tiles_x * p.Hout * p.N, per = (total + nblk - 1) / nblk;
  int b, cb;
  xcd_block<true>(b, cb);
  const int t_end = min(total, b * per + per), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, h = lane >> 5;
#pragma unroll 1
  for (int t = b * per + wave; t < t_end; t += 8) {
    const int tx = t % tiles_x, r = t / tiles_x;
    const int oy = r % p.Hout, n = r / p.Hout, ox = tx * 32 + (threadIdx.x & 31);
    const bool valid = ox < p.Wout;
    f32x4 q[RGB5_KY][3];
    rgb5_load(p, n, oy, ox, valid, q);
    f32x16 acc[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[it] = f32x16{0};
    auto ldw = [&](bf16x8 (&a)[IT], int g) {
#pragma unroll
      for (int it = 0; it < IT; ++it) a[it] = lds_frag(rgb5_lds, ((g * IT + it) * 64 + lane) * 16);
    };
    bf16x8 fa[IT], fb[IT];
    ldw(fa, 0);
    auto step = [&](bf16x8 (&cur)[IT], bf16x8 (&nxt)[IT], int ky) __attribute__((always_inline)) {
      if (ky + 1 < RGB5_KY) ldw(nxt, ky + 1);
      __builtin_amdgcn_sched_barrier(0);
      const f32x4 a = q[ky][0], bq = q[ky][1], c = q[ky][2];
      const bf16x8 bs = {(__bf16)a[0], (__bf16)a[1], (__bf16)a[2], (__bf16)bq[0], (__bf16)bq[1], (__bf16)bq[2],
                         (__bf16)(h ? c[2] : c[0]), (__bf16)(h ? 0.f : c[1])};
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[it] = mfma32bf(cur[it], bs, acc[it]);
    };
#pragma unroll
    for (int ky = 0; ky < RGB5_KY; ++ky) {
      if (ky & 1) step(fb, fa, ky);
      else step(fa, fb, ky);
    }
    __builtin_amdgcn_sched_barrier(0);
    conv_epilogue<IT, EPI, 0, true, 0, true, 1>(p, acc, n, oy, ox, valid, 0, lp);
  }
}

// GDN / IGDN backward (g_s.6 input gradient): 4 waves (one per SIMD: the wide epilogue needs the 512-register file),
// each a sequence of row tiles; tile i's saved (y, s) loads are issued before its main loop and tile i+1's input
// quads before tile i's epilogue, so their HBM latency hides behind MFMAs.  Every tile runs the same instruction
// sequence whichever wave takes it (batch-independent bits).
template <int EPI>
__global__ __launch_bounds__(256, 1) void conv_rgb5_bwd_x6_kernel(ConvParams p, long ps, int nblk) {
  extern __shared__ __attribute__((aligned(16))) char rgb5_lds[];
  static_assert(EPI == EPI_IGDN_BWD || EPI == EPI_GDN_BWD, "GDN-backward epilogues");
  rgb5_stage<true>(p, ps, rgb5_lds);
  const int tiles_x = (p.Wout + 31) / 32, total = tiles_x * p.Hout * p.N, per = (total + nblk - 1) / nblk;
  int b, cb;
  xcd_block<true>(b, cb);
  const int t_end = min(total, b * per + per), wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto coords = [&](int t, int& n, int& oy, int& ox) {
    const int tx = t % tiles_x, r = t / tiles_x;
    oy = r % p.Hout;
    n = r / p.Hout;
    ox = tx * 32 + (threadIdx.x & 31);
  };
  int t = b * per + wave;
  if (t >= t_end) return;   // wave-uniform; no barrier follows
  f32x4 q[RGB5_KY][3];
  {
    int n, oy, ox;
    coords(t, n, oy, ox);
    rgb5_load(p, n, oy, ox, ox < p.Wout, q);
  }
#pragma unroll 1
  for (; t < t_end; t += 4) {
    int n, oy, ox;
    coords(t, n, oy, ox);
    const bool valid = ox < p.Wout;
    f32x4 yq[RGB5_IT][4], sq[RGB5_IT][4];
    gdn_bwd_x6_load<RGB5_IT>(p, n, oy, ox, valid, yq, sq);
    f32x16 acc[RGB5_IT];
#pragma unroll
    for (int it = 0; it < RGB5_IT; ++it) acc[it] = f32x16{0};
    rgb5_main(rgb5_lds, q, acc);
    if (t + 4 < t_end) {
      int n1, oy1, ox1;
      coords(t + 4, n1, oy1, ox1);
      rgb5_load(p, n1, oy1, ox1, ox1 < p.Wout, q);
    }
    rgb5_epi_bwd<EPI>(p, rgb5_lds, acc, n, oy, ox, valid, yq, sq);
  }
}

// --------------------------------------------------------------------------------------------------------------
// conv_up_x6: weights [plane][cb][tap][chunk][it][lane] bf16x8.  Output y = 2a + PY uses taps ky = ky0 + 2i,
// ky0 = (PY + 2) & 1, at input row a + (PY + 2 - ky) / 2 (conv_up_kernel's decomposition).
// --------------------------------------------------------------------------------------------------------------
// Block tile: 4 PT input rows x 16 columns; PT = 1 (64-pixel blocks) where the PT = 2 grid would end in a
// partly-filled round of the 256 CUs (launch_up_x6): the same MFMA and epilogue sequence per output, so the same bits
constexpr int XU_TW = 16, XU_PC = XU_TW + 2;
template <int PT>
constexpr int xu_th() { return 4 * PT; }
template <int PT>
constexpr int xu_plane() { return (xu_th<PT>() + 2) * XU_PC; }   // 180 px (PT = 2)

template <int CG, int PT>
constexpr int xu_lds_bytes() { return 3 * (CG / 8) * xu_plane<PT>() * 16; }

// KS = 3 (cheng2020's conv3x3 stride-2 input gradients, pad 1): the same decomposition, 1 / 2 / 2 / 4 taps per class
template <int PY, int PX, int IT, int CG, int PT, int KS = 5>
ICA_DEV void conv_up_x6_class(const ConvParams& p, const f32x4* patch, int jt, int cb, int nch, int grp, long ps,
                              f32x16 (&acc)[PT][IT]) {
  constexpr int PAD = KS / 2, XU_PLANE = xu_plane<PT>();
  constexpr int KY0 = (PY + PAD) & 1, KX0 = (PX + PAD) & 1;
  constexpr int NY = (KS - KY0 + 1) / 2, NX = (KS - KX0 + 1) / 2, NT = NY * NX;
  constexpr int NCG = CG / 16;   // 16-channel chunks per LDS group
  if constexpr (NT == 0) return;  // KS = 1: only class (0, 0) has a tap (the others' outputs are the epilogue's alone)
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * KS * KS * nch * IT * 64;
  const int total = NT * NCG;
  auto wofs = [&](int u) -> int {   // fragment set of (tap ti, chunk c) of this group
    const int ti = u / NCG, c = u - ti * NCG;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    return (ky * KS + kx) * nch + grp * NCG + c;
  };
  auto ldw = [&](bf16x8 (&a)[IT][3], int u) {
    const int f = wbase + wofs(min(u, total - 1)) * IT * 64;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int q = 0; q < 3; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + it * 64) * 16));
  };
  // the B operands (three LDS planes per pixel tile) of step u
  auto ldb = [&](bf16x8 (&b)[PT][3], int u) {
    u = min(u, total - 1);
    const int ti = u / NCG, c = u - ti * NCG;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    const int pr = a_rel + 1 + (PY + PAD - ky) / 2, pc = b_rel + 1 + (PX + PAD - kx) / 2;
    const int e = (2 * c + h) * XU_PLANE + pr * XU_PC + pc;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int o = e + t * 2 * XU_PC;   // tile t: 2 input rows down
      b[t][0] = f4_as_bf8(patch[o]);
      b[t][1] = f4_as_bf8(patch[(CG / 8) * XU_PLANE + o]);
      b[t][2] = f4_as_bf8(patch[2 * (CG / 8) * XU_PLANE + o]);
    }
  };
  // one step: the next step's weight fragments AND LDS operands are issued first, a whole step (48 MFMAs) ahead of
  // their use (without the barrier the scheduler sank the fragment loads next to their first use and waited on L2
  // latency every few MFMAs; the LDS reads issued at the step's start exposed their latency to its first MFMA)
  auto step = [&](bf16x8 (&cur)[IT][3], bf16x8 (&nxt)[IT][3], bf16x8 (&bc)[PT][3], bf16x8 (&bn)[PT][3], int u) {
    ldw(nxt, u + 1);
    ldb(bn, u + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[t][it] = mfma_x6(cur[it], bc[t], acc[t][it]);
  };
  bf16x8 fa[IT][3], fb[IT][3], ba[PT][3], bb[PT][3];
  ldw(fa, 0);
  ldb(ba, 0);
  int u = 0;
#pragma unroll 1
  for (; u + 1 < total; u += 2) {
    step(fa, fb, ba, bb, u);
    step(fb, fa, bb, ba, u + 1);
  }
  if (u < total) step(fa, fb, ba, bb, u);
}

#ifdef ICA_MFMA16_AB
// A/B experiment (timing only; variant builds, scripts/build_variant.sh -DICA_MFMA16_AB): the conv_up_x6 class main
// loop on v_mfma_f32_16x16x32_bf16.  A K step is 32 deep (a chunk PAIR of one tap); the wave's 128-channel x 64-pixel
// tile is 8 x 4 blocks of 16 x 16, 6 MFMAs of 16 cycles per block and step: the cycles, operand bytes and register
// blocking of the 32x32x16 loop (8 row blocks x 3 planes x 1 KB of weights and 4 column blocks x 3 planes of LDS
// reads per 32 channels).  The weight bytes are the product pack's entries of the two chunks (same addresses, not
// the 16x16 fragment order) and the accumulators reach the epilogue in the 16x16 block layout: the instruction
// stream and the traffic are the product's, the values are not.
ICA_DEV f32x4 mfma16_x6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}

template <int PY, int PX, int IT, int CG, int PT, int KS = 5>
ICA_DEV void conv_up_x6_class16(const ConvParams& p, const f32x4* patch, int jt, int cb, int nch, int grp, long ps,
                                f32x16 (&acc)[PT][IT]) {
  constexpr int PAD = KS / 2, XU_PLANE = xu_plane<PT>();
  constexpr int KY0 = (PY + PAD) & 1, KX0 = (PX + PAD) & 1;
  constexpr int NY = (KS - KY0 + 1) / 2, NX = (KS - KX0 + 1) / 2, NT = NY * NX;
  constexpr int NCG = CG / 16, NCP = NCG / 2, RB = 2 * IT, CB = 2 * PT;
  const int lane = threadIdx.x & 63, q4 = lane >> 4, j16 = lane & 15;
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * KS * KS * nch * IT * 64;
  const int total = NT * NCP;
  f32x4 a4[RB][CB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int t = c >> 1, it = rb >> 1, k = 2 * (rb & 1) + (c & 1);
      a4[rb][c] = f32x4{acc[t][it][4 * k], acc[t][it][4 * k + 1], acc[t][it][4 * k + 2], acc[t][it][4 * k + 3]};
    }
  auto ldw = [&](bf16x8 (&a)[RB][3], int u) {
    u = min(u, total - 1);
    const int ti = u / NCP, cp = u - ti * NCP;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    const int f = wbase + ((ky * KS + kx) * nch + grp * NCG + 2 * cp) * IT * 64;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int q = 0; q < 3; ++q)
        a[rb][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + (rb & 1) * IT * 64 + (rb >> 1) * 64) * 16));
  };
  auto ldb = [&](bf16x8 (&b)[CB][3], int u) {
    u = min(u, total - 1);
    const int ti = u / NCP, cp = u - ti * NCP;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    const int pc = j16 + 1 + (PX + PAD - kx) / 2;
    const int e = (4 * cp + q4) * XU_PLANE + (jt * 2 * PT + 1 + (PY + PAD - ky) / 2) * XU_PC + pc;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int o = e + c * XU_PC;
      b[c][0] = f4_as_bf8(patch[o]);
      b[c][1] = f4_as_bf8(patch[(CG / 8) * XU_PLANE + o]);
      b[c][2] = f4_as_bf8(patch[2 * (CG / 8) * XU_PLANE + o]);
    }
  };
  auto step = [&](bf16x8 (&cur)[RB][3], bf16x8 (&nxt)[RB][3], bf16x8 (&bc)[CB][3], bf16x8 (&bn)[CB][3], int u) {
    ldw(nxt, u + 1);
    ldb(bn, u + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) a4[rb][c] = mfma16_x6(cur[rb], bc[c], a4[rb][c]);
  };
  bf16x8 fa[RB][3], fb[RB][3], ba[CB][3], bb[CB][3];
  ldw(fa, 0);
  ldb(ba, 0);
  int u = 0;
#pragma unroll 1
  for (; u + 1 < total; u += 2) {
    step(fa, fb, ba, bb, u);
    step(fb, fa, bb, ba, u + 1);
  }
  if (u < total) step(fa, fb, ba, bb, u);
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      const int t = c >> 1, it = rb >> 1, k = 2 * (rb & 1) + (c & 1);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[t][it][4 * k + i] = a4[rb][c][i];
    }
}
#endif

template <int IT, int EPI, int CG, int PT = X6_PT, int KS = 5, int FX = 0>
__global__ __launch_bounds__(256, 1) void conv_up_x6_kernel(ConvParams p, long ps) {
  ICA_STAMP_BEGIN();
  constexpr int NQ = CG / 4, XU_TH = xu_th<PT>(), XU_PLANE = xu_plane<PT>();
  extern __shared__ f32x4 patch[];   // [plane][CG/8][XU_PLANE]
  const int tiles_x = (p.Win + XU_TW - 1) / XU_TW, tiles_y = (p.Hin + XU_TH - 1) / XU_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * XU_TH, b0 = tx * XU_TW;
  const int Cin4 = p.Cin >> 2, nch = p.Cin / 16, ngrp = p.Cin / CG;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* p2 = reinterpret_cast<u32x2*>(patch);
  // one channel group into LDS: NQ quads x XU_PLANE pixels, batches of 8 loads per thread (forced inline: as a
  // call it kept the whole register file live across an s_swappc)
  auto fill = [&](int grp) __attribute__((always_inline)) {
    constexpr int FB = 8, TOT = NQ * XU_PLANE;
    __syncthreads();
    for (int e0 = threadIdx.x; e0 < TOT; e0 += 256 * FB) {
      f32x4 v[FB];
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 256 * i;
        const int q = e / XU_PLANE, rem = e - q * XU_PLANE, pr = rem / XU_PC, pc = rem - pr * XU_PC;
        const int iy = a0 - 1 + pr, ix = b0 - 1 + pc;
        const bool ok = e < TOT && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        const unsigned vo = ((unsigned)(grp * NQ + q) * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 256 * i;
        if (e < TOT) {
          const int q = e / XU_PLANE, pix = e - q * XU_PLANE;
          u32x2 a, b, c;
          split3(v[i], a, b, c);
          const int ent = (q >> 1) * XU_PLANE + pix;
          p2[(0 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = a;
          p2[(1 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = b;
          p2[(2 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = c;
        }
      }
    }
    __syncthreads();
  };
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int jt = wave & 1;
  const int j = threadIdx.x & 31;
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
  // one class of the wave's pair: all channel groups (a group is re-staged per class when Cin > CG), then its
  // epilogue; classes pair 9 + 4 and 6 + 6 taps for balance
  auto run_class = [&](auto py_c, auto px_c, bool refill, int tk) __attribute__((always_inline)) {
    constexpr int PY = decltype(py_c)::value, PX = decltype(px_c)::value;
    f32x16 acc[PT][IT];
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
    for (int grp = 0; grp < ngrp; ++grp) {
      if (refill) fill(grp);
#ifdef ICA_MFMA16_AB
      if constexpr (KS == 5 && PT == 2 && IT == 4)
        conv_up_x6_class16<PY, PX, IT, CG, PT, KS>(p, patch, jt, cb, nch, grp, ps, acc);
      else
#endif
      conv_up_x6_class<PY, PX, IT, CG, PT, KS>(p, patch, jt, cb, nch, grp, ps, acc);
    }
    ICA_STAMP_AT(tk - 2);
    if constexpr ((EPI == EPI_GDN || EPI == EPI_IGDN) && PT == 2) {
      const int oy[2] = {2 * (a0 + a_rel) + PY, 2 * (a0 + a_rel + 2) + PY};
      const int ox[2] = {2 * (b0 + b_rel) + PX, 2 * (b0 + b_rel) + PX};
      gdn_fwd_x6_pair<IT, EPI>(p, acc, n, oy, ox);
    } else {
#pragma unroll
      for (int t = 0; t < PT; ++t) {
        const int oy = 2 * (a0 + a_rel + 2 * t) + PY, ox = 2 * (b0 + b_rel) + PX;
        conv_epilogue<IT, EPI, FX, false, 1>(p, acc[t], n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
      }
    }
    ICA_STAMP_AT(tk - 1);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  const bool multi = ngrp > 1;
  if (!multi) fill(0);
  // every wave joins every fill barrier: both classes of every wave run the same group sequence
  if (wave < 2) {
    run_class(I0{}, I0{}, multi, 2);
    run_class(I1{}, I1{}, multi, 4);
  } else {
    run_class(I0{}, I1{}, multi, 2);
    run_class(I1{}, I0{}, multi, 4);
  }
  ICA_STAMP_END();
}

// --------------------------------------------------------------------------------------------------------------
// conv_up_x6w: the conv_up_x6 block (8 x 16 input pixels, the channel group in LDS) on EIGHT waves, one output-parity
// class per wave, two waves per SIMD (waves w and w + 4 share one).  The partners run complementary classes (9 + 4 or
// 6 + 6 taps), so while one wave is in its epilogue (saved (y, s) reads, VALU, stores) or waits on a load, the
// other's MFMAs keep the SIMD's matrix pipe busy; at one wave per SIMD (conv_up_x6) every epilogue and wait left it
// idle.  256 registers per wave: the weight fragments of output tile it are refilled right after that tile's MFMAs
// of the step (a ring, one step of prefetch distance, instead of two whole fragment sets), one B operand set, and the
// GDN forward epilogue is the tile-serial narrow form.  Each output runs the same MFMA and epilogue arithmetic as in
// conv_up_x6: same bits (scripts/gpu_ab_bits.sh).  Forward layers only (launch_up_x6): bias 2.98 -> 2.73 ms, IGDN
// 3.66 -> 3.44 ms at the config-2 shapes (row-major, same box).
// --------------------------------------------------------------------------------------------------------------
template <int PY, int PX, int IT, int CG, int PT>
ICA_DEV void conv_up_x6w_class(const ConvParams& p, const f32x4* patch, int jt, int cb, int nch, int grp, long ps,
                               f32x16 (&acc)[PT][IT]) {
  constexpr int KS = 5, PAD = 2, XU_PLANE = xu_plane<PT>();
  constexpr int KY0 = (PY + PAD) & 1, KX0 = (PX + PAD) & 1;
  constexpr int NY = (KS - KY0 + 1) / 2, NX = (KS - KX0 + 1) / 2, NT = NY * NX;
  constexpr int NCG = CG / 16;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * KS * KS * nch * IT * 64;
  const int total = NT * NCG;
  auto ldw = [&](bf16x8 (&a)[3], int u, int it) {   // output tile it's fragments of step u
    u = min(u, total - 1);
    const int ti = u / NCG, c = u - ti * NCG;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    const int f = wbase + ((ky * KS + kx) * nch + grp * NCG + c) * IT * 64 + it * 64;
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = ld_bf8(wr, lane * 16, (int)((q * ps + f) * 16));
  };
  auto ldb = [&](bf16x8 (&b)[PT][3], int u) {
    u = min(u, total - 1);
    const int ti = u / NCG, c = u - ti * NCG;
    const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
    const int pr = a_rel + 1 + (PY + PAD - ky) / 2, pc = b_rel + 1 + (PX + PAD - kx) / 2;
    const int e = (2 * c + h) * XU_PLANE + pr * XU_PC + pc;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int o = e + t * 2 * XU_PC;
      b[t][0] = f4_as_bf8(patch[o]);
      b[t][1] = f4_as_bf8(patch[(CG / 8) * XU_PLANE + o]);
      b[t][2] = f4_as_bf8(patch[2 * (CG / 8) * XU_PLANE + o]);
    }
  };
  // one B set: the next step's LDS operands are read after this step's last MFMA (the SIMD partner's MFMAs cover
  // their latency)
  bf16x8 w[IT][3], b[PT][3];
#pragma unroll
  for (int it = 0; it < IT; ++it) ldw(w[it], 0, it);
  ldb(b, 0);
#pragma unroll 1
  for (int u = 0; u < total; ++u) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < PT; ++t) acc[t][it] = mfma_x6(w[it], b[t], acc[t][it]);
      ldw(w[it], u + 1, it);   // after this step's last use: one step ahead of the next
    }
    __builtin_amdgcn_sched_barrier(0);
    ldb(b, u + 1);
  }
}

// GDN / IGDN backward epilogue of the 8-wave conv_up (two waves per SIMD, 256 registers): this wave's PT pixel
// tiles x IT * 32 channels (all of Cout).  The wide form's t (IT * 16 registers) and 2x (IT * 16) do not fit next
// to the accumulators, so t goes through this wave's LDS slab (4 IT x 64 entries: the block's LDS, free after the
// barrier that ends every wave's main loop):
//   pass 1 (per channel tile it): the saved (y, s) quads -> t into the slab (k-step order), g*s in place of g;
//   pass 2 (per output tile jt): u = gamma'^T t on x6 MFMAs over the k-steps of the slab (each split on the fly),
//   dx = g*s + 2x u.  PT = 2: 2x is formed again from the (y, s) quads of jt, re-read before the GEMM (the SIMD
//   partner's MFMAs cover the latency); PT = 1 (64 accumulator registers): 2x is kept from pass 1, (y, s) read once.
// Pass 1's (y, s) quads run in a two-channel-tile ring (64 registers): the first two tiles' loads of pixel tile 0
// are issued before the block barrier, which waits for LDS operations only (barrier_lds_only), so they stay in
// flight through it; each later tile's loads go out two tiles ahead of their use.
// Every output gets the arithmetic and MFMA order of gdn_bwd_x6_wide, at PT = 1 and 2 alike.
// Measured and not kept (profiles/r05): t parked in the output tensor instead of LDS, no barrier, the shorter classes
// on the waves the SIMD arbiter favours (so their epilogues run under the partners' main loops): 4.23 -> 5.14 ms, the
// early epilogues' memory traffic delayed the partners' weight loads (their main loops ended 70k cycles later).
struct X6wPix {
  unsigned vo[2], vl[2];
  bool valid[2];
};
template <int IT>
ICA_DEV X6wPix x6w_pix(const ConvParams& p, const int (&oy)[2], const int (&ox)[2]) {
  const int h = (threadIdx.x & 63) >> 5;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  X6wPix r;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    r.valid[t] = oy[t] < p.Hout && ox[t] < p.Wout;
    r.vo[t] = r.valid[t] ? h * plane + pix_at(oy[t], ox[t], p.Hout, p.Wout, p.pl & PL_OUT) : 0u;
    r.vl[t] = r.valid[t] ? r.vo[t] : 0x0FFFFFF0u;   // past the descriptor's range: loads return 0 (never stored)
  }
  return r;
}
// the (y, s) quads of channel tile it at lane offset vl (x6w_pix)
ICA_DEV void x6w_ys(const ConvParams& p, int n, unsigned vl, int it, f32x4 (&yq)[4], f32x4 (&sq)[4]) {
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 IX(p.in_x, img, n), IS(p.in_s, img, n);
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    yq[g] = IX.ld(vl, (unsigned)(it * 8 + 2 * g) * plane);
    sq[g] = IS.ld(vl, (unsigned)(it * 8 + 2 * g) * plane);
  }
}

template <int IT, int EPI, int PT>
ICA_DEV void gdn_bwd_x6w_slab(const ConvParams& p, f32x16 (&acc)[PT][IT], int n, const X6wPix& px,
                              f32x4 (&ry)[2][4], f32x4 (&rs)[2][4], f32x4* slab) {
  static_assert(EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD, "GDN backward epilogues only");
  static_assert(IT >= 2, "x6w GDN backward: a two-tile (y, s) ring");
  const int lane = threadIdx.x & 63;
  const unsigned plane = (unsigned)p.Hout * p.Wout;
  const size_t img = (size_t)((p.Cout + 3) >> 2) * plane;
  const Img4 Y(p.y, img, n);
  const __amdgpu_buffer_rsrc_t grs = uniform_rsrc(p.gp, IT * IT * 6144);
  auto ldg = [&](bf16x8 (&a)[3], int jt, int k) {
#pragma unroll
    for (int q = 0; q < 3; ++q)
      a[q] = ld_bf8(grs, lane * 16, (((jt * IT + (k >> 1)) * 2 + (k & 1)) * 1024) + q * IT * IT * 2048);
  };
  f32x16 xx[PT == 1 ? IT : 1];
#pragma unroll
  for (int t = 0; t < PT; ++t) {
    if (t == 1) {   // pixel tile 1: its ring starts here
      x6w_ys(p, n, px.vl[1], 0, ry[0], rs[0]);
      x6w_ys(p, n, px.vl[1], 1, ry[1], rs[1]);
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        f32x4 tv;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float sg = rs[it & 1][g][e], rc = __builtin_amdgcn_rcpf(sg), xs = ry[it & 1][g][e] * rc;
          const float gx = acc[t][it][4 * g + e] * xs;
          tv[e] = (EPI == EPI_GDN_BWD) ? (-0.5f * gx) * (sg * sg * sg) : (0.5f * gx) * rc;
          float gs = acc[t][it][4 * g + e] * sg;
          float x2 = 2.0f * xs;
          asm volatile("" : "+v"(gs), "+v"(x2));   // rounded on their own: never contracted into dx's fma
          acc[t][it][4 * g + e] = gs;
          if constexpr (PT == 1) xx[it][4 * g + e] = x2;
        }
        slab[((2 * it + (g >> 1)) * 2 + (g & 1)) * 64 + lane] = tv;   // k-step 2 it + g / 2, half g & 1
      }
      if (it + 2 < IT) x6w_ys(p, n, px.vl[t], it + 2, ry[it & 1], rs[it & 1]);
    }
#pragma unroll
    for (int jt = 0; jt < IT; ++jt) {
      __builtin_amdgcn_sched_barrier(0);
      f32x4 yq[4], sq[4];
      if constexpr (PT != 1) x6w_ys(p, n, px.vl[t], jt, yq, sq);
      f32x16 ux = f32x16{0};
      bf16x8 ga[2][3];
      ldg(ga[0], jt, 0);
#pragma unroll
      for (int k = 0; k < 2 * IT; ++k) {
        if (k + 1 < 2 * IT) ldg(ga[(k + 1) & 1], jt, k + 1);
        __builtin_amdgcn_sched_barrier(0);
        const f32x4 a = slab[(2 * k) * 64 + lane], b = slab[(2 * k + 1) * 64 + lane];
        const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        bf16x8 tq[3];
        split3x8(v, tq);
        ux = mfma_x6(ga[k & 1], tq, ux);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (px.valid[t]) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float x2;
            if constexpr (PT == 1) {
              x2 = xx[jt][4 * g + e];
            } else {
              x2 = 2.0f * (yq[g][e] * __builtin_amdgcn_rcpf(sq[g][e]));
              asm volatile("" : "+v"(x2));   // as in the wide form: 2x materialised, then one fma with u
            }
            o[e] = acc[t][jt][4 * g + e] + x2 * ux[4 * g + e];
          }
          Y.st(px.vo[t], (unsigned)(jt * 8 + 2 * g) * plane, o);
        }
      }
    }
    ICA_STAMP_AT(2 + t);
  }
}

// a block barrier that waits only for this wave's LDS operations (the waves' patch reads), not for its global loads:
// the (y, s) loads issued before it stay in flight through the wait
ICA_DEV void barrier_lds_only() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <int IT, int EPI, int CG, int PT = 2>
__global__ __launch_bounds__(512, 1) void conv_up_x6w_kernel(ConvParams p, long ps) {
  ICA_STAMP_BEGIN();
  constexpr int NQ = CG / 4, XU_TH = xu_th<PT>(), XU_PLANE = xu_plane<PT>();
  extern __shared__ f32x4 patch[];   // [plane][CG/8][XU_PLANE]
  const int tiles_x = (p.Win + XU_TW - 1) / XU_TW, tiles_y = (p.Hin + XU_TH - 1) / XU_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * XU_TH, b0 = tx * XU_TW;
  const int Cin4 = p.Cin >> 2, nch = p.Cin / 16, ngrp = p.Cin / CG;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* p2 = reinterpret_cast<u32x2*>(patch);
  auto fill = [&](int grp) __attribute__((always_inline)) {
    constexpr int FB = 6, TOT = NQ * XU_PLANE;
    __syncthreads();
    for (int e0 = threadIdx.x; e0 < TOT; e0 += 512 * FB) {
      f32x4 v[FB];
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 512 * i;
        const int q = e / XU_PLANE, rem = e - q * XU_PLANE, pr = rem / XU_PC, pc = rem - pr * XU_PC;
        const int iy = a0 - 1 + pr, ix = b0 - 1 + pc;
        const bool ok = e < TOT && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        const unsigned vo = ((unsigned)(grp * NQ + q) * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 512 * i;
        if (e < TOT) {
          const int q = e / XU_PLANE, pix = e - q * XU_PLANE;
          u32x2 a, b, c;
          split3(v[i], a, b, c);
          const int ent = (q >> 1) * XU_PLANE + pix;
          p2[(0 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = a;
          p2[(1 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = b;
          p2[(2 * (CG / 8) * XU_PLANE + ent) * 2 + (q & 1)] = c;
        }
      }
    }
    __syncthreads();
  };
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int jt = wave & 1;
  const int j = threadIdx.x & 31;
  const int a_rel = jt * 2 * PT + (j >> 4), b_rel = j & 15;
  auto run_class = [&](auto py_c, auto px_c, bool refill) __attribute__((always_inline)) {
    constexpr int PY = decltype(py_c)::value, PX = decltype(px_c)::value;
    f32x16 acc[PT][IT];
#pragma unroll
    for (int t = 0; t < PT; ++t)
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
    for (int grp = 0; grp < ngrp; ++grp) {
      if (refill) fill(grp);
      conv_up_x6w_class<PY, PX, IT, CG, PT>(p, patch, jt, cb, nch, grp, ps, acc);
    }
    int oy[2], ox[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {   // (PT = 1 uses entry 0 only)
      oy[t] = 2 * (a0 + a_rel + 2 * t) + PY;
      ox[t] = 2 * (b0 + b_rel) + PX;
    }
    static_assert(EPI == EPI_BIAS || EPI == EPI_GDN || EPI == EPI_IGDN || EPI == EPI_GDN_BWD ||
                      EPI == EPI_IGDN_BWD, "conv_up_x6w: bias, GDN / IGDN and their backward epilogues");
    if constexpr (EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD) {
      const X6wPix px = x6w_pix<IT>(p, oy, ox);
      f32x4 ry[2][4], rs[2][4];   // pass 1's (y, s) ring: channel tiles 0 and 1 of pixel tile 0 issued here
      x6w_ys(p, n, px.vl[0], 0, ry[0], rs[0]);
      x6w_ys(p, n, px.vl[0], 1, ry[1], rs[1]);
      ICA_STAMP_AT(0);
      ICA_STAMP_WAVE();
      barrier_lds_only();   // every wave's main loop is done with the patch: the LDS becomes the waves' t slabs
      ICA_STAMP_AT(1);
      gdn_bwd_x6w_slab<IT, EPI, PT>(p, acc, n, px, ry, rs, patch + wave * (4 * IT * 64));
    } else if constexpr (EPI == EPI_GDN || EPI == EPI_IGDN) {
#pragma unroll
      for (int t = 0; t < PT; ++t) gdn_fwd_x6_tile_narrow<IT, EPI>(p, acc[t], n, oy[t], ox[t]);
    } else {
#pragma unroll
      for (int t = 0; t < PT; ++t)
        conv_epilogue<IT, EPI, 0, false, 2>(p, acc[t], n, oy[t], ox[t], oy[t] < p.Hout && ox[t] < p.Wout,
                                            cb * IT * 32);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  const bool multi = ngrp > 1;
  if (!multi) fill(0);
  // SIMD partners (w, w + 4): (0,0) 9 taps with (1,1) 4 taps; (0,1) with (1,0), 6 + 6.  Every wave joins every
  // fill barrier (one class each, the same group sequence)
  switch (wave >> 1) {
    case 0: run_class(I0{}, I0{}, multi); break;
    case 1: run_class(I0{}, I1{}, multi); break;
    case 2: run_class(I1{}, I1{}, multi); break;
    default: run_class(I1{}, I0{}, multi); break;
  }
  ICA_STAMP_END();
}

// --------------------------------------------------------------------------------------------------------------
// Small-grid x6 kernels (layers whose low-resolution side is <= 32 x 32 per image: the fine-tune's 256x256 crops).
// The structure of the fp32 small-grid kernels of ica_conv.hip on x6 operands: a 32-pixel tile per
// block, the K loop split over the 4 waves, partial sums reduced through LDS in wave order (deterministic), wave 0
// runs the (narrow) x6 epilogue.  Six 32-cycle bf16 MFMAs per 16-deep k step instead of eight 64-cycle fp32 ones:
// the per-wave chain that bounds these latency-bound launches is 2.7x shorter.
// --------------------------------------------------------------------------------------------------------------
constexpr int XSD_TW = 8, XSD_TH = 4;   // conv_down: 4 x 8 output pixels per block
template <int IT>
constexpr int xs_red_entries() { return 3 * IT * 4 * 64; }

// partial sums of waves 1..3 into red, wave 0 adds them in wave order; returns true on wave 0
template <int IT>
ICA_DEV bool xs_reduce(f32x16 (&acc)[IT], f32x4* red, int wave, int lane) {
  if (wave > 0) {
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        red[(((wave - 1) * IT + it) * 4 + g) * 64 + lane] =
            f32x4{acc[it][4 * g], acc[it][4 * g + 1], acc[it][4 * g + 2], acc[it][4 * g + 3]};
  }
  __syncthreads();
  if (wave != 0) return false;
#pragma unroll 1
  for (int w = 0; w < 3; ++w) {   // one partial at a time (hoisting every LDS read spilled)
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 r = red[((w * IT + it) * 4 + g) * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[it][4 * g + e] += r[e];
      }
  }
  return true;
}

// conv_down (k5 s2): the 4 waves share one 4 x 8 output tile and split its 25 taps
template <int IT, int EPI>
__global__ __launch_bounds__(256, 2) void conv_down_small_x6_kernel(ConvParams p, long ps) {
  constexpr int KS = 5, S = 2, PAD = 2, KK = 25, TW = XSD_TW, TH = XSD_TH;
  constexpr int PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;   // 11 x 19
  constexpr int NF = (4 * PLANE + 255) / 256;
  __shared__ f32x4 patch[3 * 2 * PLANE];   // [plane][half][pixel]: 8 channels as bf16
  __shared__ f32x4 red[xs_red_entries<IT>()];
  const int tiles_x = (p.Wout + TW - 1) / TW, tiles_y = (p.Hout + TH - 1) / TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5,
            j = lane & 31;
  const int oy0 = ty * TH, ox0 = tx * TW, iy0 = oy0 * S - PAD, ix0 = ox0 * S - PAD;
  const int Cin4 = (p.Cin + 3) >> 2, nch = (Cin4 * 4 + 15) / 16;
  const int oyl = j / TW, oxl = j % TW, lbase = S * oyl * PC + S * oxl;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* p2 = reinterpret_cast<u32x2*>(patch);
  auto fill = [&](int ch) {
    f32x4 v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int q = e / PLANE, rem = e - q * PLANE, pr = rem / PC, pc = rem - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc, c4 = ch * 4 + q;
      const bool ok = e < 4 * PLANE && c4 < Cin4 && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
      const unsigned vo = ((unsigned)c4 * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
      v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < 4 * PLANE) {
        const int q = e / PLANE, pix = e - q * PLANE;
        u32x2 a, b, c;
        split3(v[i], a, b, c);
        const int ent = (q >> 1) * PLANE + pix;
        p2[(0 * 2 * PLANE + ent) * 2 + (q & 1)] = a;
        p2[(1 * 2 * PLANE + ent) * 2 + (q & 1)] = b;
        p2[(2 * 2 * PLANE + ent) * 2 + (q & 1)] = c;
      }
    }
    __syncthreads();
  };
  const int t0 = wave * KK / 4, nt = (wave + 1) * KK / 4 - t0, total = nch * nt;
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * nch * KK * IT * 64;
  auto ldw = [&](bf16x8 (&a)[IT][3], int u) {
    u = min(u, total - 1);
    const int ch = u / nt, tap = t0 + (u - ch * nt);
    const int f = wbase + (ch * KK + tap) * IT * 64;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int q = 0; q < 3; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + it * 64) * 16));
  };
  f32x16 acc[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) acc[it] = f32x16{0};
  auto step = [&](bf16x8 (&cur)[IT][3], bf16x8 (&nxt)[IT][3], int u) __attribute__((always_inline)) {
    ldw(nxt, u + 1);
    __builtin_amdgcn_sched_barrier(0);
    const int ch = u / nt, tap = t0 + (u - ch * nt);
    const int ky = tap / KS, kx = tap - ky * KS;
    const int o = h * PLANE + lbase + ky * PC + kx;
    const bf16x8 b[3] = {f4_as_bf8(patch[o]), f4_as_bf8(patch[2 * PLANE + o]), f4_as_bf8(patch[4 * PLANE + o])};
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[it] = mfma_x6(cur[it], b, acc[it]);
  };
  bf16x8 fa[IT][3], fb[IT][3];
  ldw(fa, 0);
  int u = 0;
#pragma unroll 1
  for (int ch = 0; ch < nch; ++ch) {
    fill(ch);   // every wave joins every chunk's barriers
    const int ue = u + nt;
#pragma unroll 1
    for (; u + 1 < ue; u += 2) {
      step(fa, fb, u);
      step(fb, fa, u + 1);
    }
    if (u < ue) {   // odd step count: the prefetched set moves to fa (once per chunk)
      step(fa, fb, u);
      ++u;
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int q = 0; q < 3; ++q) fa[it][q] = fb[it][q];
    }
  }
  if (!xs_reduce<IT>(acc, red, wave, lane)) return;
  const int oy = oy0 + oyl, ox = ox0 + oxl;
  conv_epilogue<IT, EPI, 0, false, 2>(p, acc, n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
}

// conv_up (k5 s2 p2 op1): one block = one output-parity class of one 2 x 16 input tile, the input-channel chunks
// split over the 4 waves; the whole-Cin patch as three bf16 planes
constexpr int XSU_TH = 2, XSU_PC = 18, XSU_PLANE = (XSU_TH + 2) * XSU_PC;   // 72 pixels
template <int IT, int EPI>
__global__ __launch_bounds__(256, 2) void conv_up_small_x6_kernel(ConvParams p, long ps) {
  constexpr int KS = 5, PAD = 2, TW = 16;
  extern __shared__ f32x4 patch[];   // [plane][Cin/8][XSU_PLANE]; then the partial sums
  const int tiles_x = (p.Win + TW - 1) / TW, tiles_y = (p.Hin + XSU_TH - 1) / XSU_TH;
  int bid, cb;
  xcd_block<true>(bid, cb);
  const int cls = bid & 3;
  bid >>= 2;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * XSU_TH, b0 = tx * TW;
  const int Cin4 = p.Cin >> 2, nch = p.Cin / 16, NQ8 = p.Cin / 8;
  const unsigned xplane = (unsigned)p.Hin * p.Win;
  const __amdgpu_buffer_rsrc_t xr =
      uniform_rsrc(reinterpret_cast<const char*>(p.x) + (size_t)n * Cin4 * xplane * 16, Cin4 * xplane * 16u);
  u32x2* p2 = reinterpret_cast<u32x2*>(patch);
  {
    constexpr int FB = 8;
    const int TOT = Cin4 * XSU_PLANE;
    for (int e0 = threadIdx.x; e0 < TOT; e0 += 256 * FB) {
      f32x4 v[FB];
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 256 * i;
        const int q = e / XSU_PLANE, rem = e - q * XSU_PLANE, pr = rem / XSU_PC, pc = rem - pr * XSU_PC;
        const int iy = a0 - 1 + pr, ix = b0 - 1 + pc;
        const bool ok = e < TOT && iy >= 0 && iy < p.Hin && ix >= 0 && ix < p.Win;
        const unsigned vo = ((unsigned)q * xplane + pix_at(iy, ix, p.Hin, p.Win, p.pl & PL_IN)) * 16u;
        v[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < FB; ++i) {
        const int e = e0 + 256 * i;
        if (e < TOT) {
          const int q = e / XSU_PLANE, pix = e - q * XSU_PLANE;
          u32x2 a, b, c;
          split3(v[i], a, b, c);
          const int ent = (q >> 1) * XSU_PLANE + pix;
          p2[(0 * NQ8 * XSU_PLANE + ent) * 2 + (q & 1)] = a;
          p2[(1 * NQ8 * XSU_PLANE + ent) * 2 + (q & 1)] = b;
          p2[(2 * NQ8 * XSU_PLANE + ent) * 2 + (q & 1)] = c;
        }
      }
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h = lane >> 5,
            j = lane & 31;
  const int c0 = wave * nch / 4, cn = (wave + 1) * nch / 4 - c0;   // cn >= 1: Cin >= 64 (host)
  const int a_rel = j >> 4, b_rel = j & 15;
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(p.wp, (unsigned)(3 * ps * 16));
  const int wbase = cb * KS * KS * nch * IT * 64;
  auto run = [&](auto py_c, auto px_c) __attribute__((always_inline)) {
    constexpr int PY = decltype(py_c)::value, PX = decltype(px_c)::value;
    constexpr int KY0 = (PY + PAD) & 1, KX0 = (PX + PAD) & 1;
    constexpr int NY = (KS - KY0 + 1) / 2, NX = (KS - KX0 + 1) / 2, NT = NY * NX;
    const int total = NT * cn;
    auto ldw = [&](bf16x8 (&a)[IT][3], int u) {
      u = min(u, total - 1);
      const int ti = u / cn, c = c0 + (u - ti * cn);
      const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
      const int f = wbase + ((ky * KS + kx) * nch + c) * IT * 64;
#pragma unroll
      for (int it = 0; it < IT; ++it)
#pragma unroll
        for (int q = 0; q < 3; ++q) a[it][q] = ld_bf8(wr, lane * 16, (int)((q * ps + f + it * 64) * 16));
    };
    f32x16 acc[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[it] = f32x16{0};
    auto step = [&](bf16x8 (&cur)[IT][3], bf16x8 (&nxt)[IT][3], int u) __attribute__((always_inline)) {
      ldw(nxt, u + 1);
      __builtin_amdgcn_sched_barrier(0);
      const int ti = u / cn, c = c0 + (u - ti * cn);
      const int ky = KY0 + 2 * (ti / NX), kx = KX0 + 2 * (ti % NX);
      const int pr = a_rel + 1 + (PY + PAD - ky) / 2, pc = b_rel + 1 + (PX + PAD - kx) / 2;
      const int o = (2 * c + h) * XSU_PLANE + pr * XSU_PC + pc;
      const bf16x8 b[3] = {f4_as_bf8(patch[o]), f4_as_bf8(patch[NQ8 * XSU_PLANE + o]),
                           f4_as_bf8(patch[2 * NQ8 * XSU_PLANE + o])};
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[it] = mfma_x6(cur[it], b, acc[it]);
    };
    bf16x8 fa[IT][3], fb[IT][3];
    ldw(fa, 0);
    int u = 0;
#pragma unroll 1
    for (; u + 1 < total; u += 2) {
      step(fa, fb, u);
      step(fb, fa, u + 1);
    }
    if (u < total) step(fa, fb, u);
    __syncthreads();   // every wave is done with the patch: its LDS takes the partial sums
    if (!xs_reduce<IT>(acc, patch, wave, lane)) return;
    const int oy = 2 * (a0 + a_rel) + PY, ox = 2 * (b0 + b_rel) + PX;
    conv_epilogue<IT, EPI, 0, false, 2>(p, acc, n, oy, ox, oy < p.Hout && ox < p.Wout, cb * IT * 32);
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

// (cb, outer, inner, it, lane, s) fragment index of pack_conv_kernel (CC = 16) -> three split planes
__global__ void pack_conv_x6_kernel(const float* __restrict__ w, __bf16* __restrict__ dst, int O, int C, int KS,
                                    long so, long sc, int IT, int order, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int KK = KS * KS;
  const int nch = (((C + 3) / 4) * 4 + 15) / 16;
  long t = i;
  const int s = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int it = t % IT; t /= IT;
  int inner, outer;
  if (order == 0) { inner = t % KK; t /= KK; outer = t % nch; t /= nch; }
  else { inner = t % nch; t /= nch; outer = t % KK; t /= KK; }
  const int cb = (int)t;
  const int chunk = order == 0 ? outer : inner;
  const int tap = order == 0 ? inner : outer;
  const int o = cb * IT * 32 + it * 32 + (lane & 31);
  const int c = chunk * 16 + (lane >> 5) * 8 + s;
  float v = 0.f;
  if (o < O && c < C) v = w[o * so + c * sc + (tap / KS) * KS + (tap % KS)];
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  dst[total + i] = b;
  dst[2 * total + i] = (__bf16)(r1 - (float)b);
}

// tap-pair fragments of conv_down_x6w, [cb][chunk8][step][it][lane][e] (three split planes): lane (h, r) supplies
// A[r][k = 8 h + e] = W[o][c = 8 chunk8 + e][tap = 2 step + h], 0 past C and for tap 25
__global__ void pack_conv_x6w_kernel(const float* __restrict__ w, __bf16* __restrict__ dst, int O, int C, long so,
                                     long sc, int IT, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int nch8 = ((C + 3) / 4 + 1) / 2, npair = nch8 >> 1;
  const int nsteps = npair * 25 + (nch8 & 1) * XW_NS;
  long t = i;
  const int e = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int it = t % IT; t /= IT;
  const int g = t % nsteps;
  const int cb = (int)(t / nsteps);
  const int h = lane >> 5;
  // step g -> (8-channel chunk, tap) of lane half h: chunk pairs of 25 steps (12 tap pairs of chunk 2 cp, the cross
  // step = tap 24 of chunk 2 cp + h, 12 tap pairs of chunk 2 cp + 1), then a lone chunk's 13 tap pairs
  int c8, tap;
  if (g < npair * 25) {
    const int cp = g / 25, sl = g - cp * 25;
    if (sl < 12) { c8 = 2 * cp; tap = 2 * sl + h; }
    else if (sl == 12) { c8 = 2 * cp + h; tap = 24; }
    else { c8 = 2 * cp + 1; tap = 2 * (sl - 13) + h; }
  } else {
    c8 = nch8 - 1;
    tap = 2 * (g - npair * 25) + h;
  }
  const int o = cb * IT * 32 + it * 32 + (lane & 31), c = c8 * 8 + e;
  float v = 0.f;
  if (o < O && c < C && tap < 25) v = w[o * so + c * sc + tap];
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  dst[total + i] = b;
  dst[2 * total + i] = (__bf16)(r1 - (float)b);
}

// dense tap-row fragments of conv_rgb5_x6, [cb][ky][it][lane][e] (three split planes): lane (h, r) supplies
// A[r][k = 8 h + e] = W[o][c][ky][kx] with (kx, c) of the conv_rgb5_x6 K map (0 for c >= C and for h = 1, e = 7)
__global__ void pack_conv_rgb5_x6_kernel(const float* __restrict__ w, __bf16* __restrict__ dst, int O, int C, long so,
                                         long sc, int IT, long total, int planes) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  long t = i;
  const int e = t % 8; t /= 8;
  const int lane = t % 64; t /= 64;
  const int it = t % IT; t /= IT;
  const int ky = t % RGB5_KY;
  const int cb = (int)(t / RGB5_KY);
  const int h = lane >> 5;
  int kx, c;
  if (e < 6) {
    kx = 2 * h + e / 3;
    c = e % 3;
  } else {
    kx = 4;
    c = h ? (e == 6 ? 2 : 3) : e - 6;   // c = 3: the zero slot
  }
  const int o = cb * IT * 32 + it * 32 + (lane & 31);
  float v = 0.f;
  if (o < O && c < C && c < 3) v = w[o * so + c * sc + ky * 5 + kx];
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  if (planes == 3) {
    dst[total + i] = b;
    dst[2 * total + i] = (__bf16)(r1 - (float)b);
  }
}

// the fp32 gamma' pack of ica_pack_gdn ([a][b][lane][r]) -> three bf16 planes [plane][a][b][s][lane][e], r = 8s + e
// (the epilogue's k-step s of tile b, lane order unchanged)
__global__ void pack_gdn_x6_kernel(const float* __restrict__ gp, __bf16* __restrict__ dst, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = i % 8, lane = (i / 8) % 64, s = (i / 512) % 2;
  const long ab = i / 1024;
  const float v = gp[(ab * 64 + lane) * 16 + 8 * s + e];
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  dst[total + i] = b;
  dst[2 * total + i] = (__bf16)(r1 - (float)b);
}

// --------------------------------------------------------------------------------------------------------------
// cheng2020 g_a.0 input gradient (ResidualBlockWithStride(3, N): conv1 = conv3x3(3, N, s2) and skip = conv1x1(3, N,
// s2), both read the image): dx = conv1^T g1 + skip^T gs in ONE pass.  A 3-channel output is a poor MFMA row tile
// (the two fp32 conv_up launches computed 32 rows for 3 and read their inputs separately: 6.7 ms at the config-3
// shapes), so the kernel runs the Z-gather of conv_up3: Z = Wt^T [g1; gs] for every gradient pixel (rows 0-26:
// (c, ky, kx) of conv1 over the g1 channels, rows 27-29: c of the skip over the gs channels; K = 2 Cg), on x6
// operands, into LDS, then each output pixel sums its 1, 2 or 4 conv1 taps and (even pixels) the skip row.
// Tile: UK_ZR = 16 gradient rows x 32 columns of Z (4 rows per wave), outputs for the first 15 x 31 of them (the
// transposed k3 s2 conv reads rows a, a + 1 and columns b, b + 1 of g for output row 2a + 1 / column 2b + 1).
// --------------------------------------------------------------------------------------------------------------
constexpr int UK_ZR = 16, UK_R = UK_ZR - 1, UK_OW = 31, UK_NPX = UK_ZR * 32;

// [plane][chunk][lane][e] (K = 2 Cg, chunk = 16 channels): lane (h, row) holds A[row][k = 16 chunk + 8 h + e]
__global__ void pack_up3k3_x6_kernel(const float* __restrict__ w1, const float* __restrict__ ws, __bf16* __restrict__ dst,
                                     int Cg, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int e = i % 8, lane = (i / 8) % 64, chunk = (int)(i / 512);
  const int row = lane & 31, k = chunk * 16 + (lane >> 5) * 8 + e;
  float v = 0.f;
  if (row < 27 && k < Cg) v = w1[((long)k * 3 + row / 9) * 9 + row % 9];               // conv1 [Cg][3][3][3]
  else if (row >= 27 && row < 30 && k >= Cg) v = ws[(long)(k - Cg) * 3 + (row - 27)];   // skip [Cg][3][1][1]
  const __bf16 a = (__bf16)v;
  const float r1 = v - (float)a;
  const __bf16 b = (__bf16)r1;
  dst[i] = a;
  dst[total + i] = b;
  dst[2 * total + i] = (__bf16)(r1 - (float)b);
}

__global__ __launch_bounds__(256, 2) void conv_up3k3_x6_kernel(const float* __restrict__ g1, const float* __restrict__ gs,
                                                                const void* __restrict__ wp, float* __restrict__ dx,
                                                                int Cg, int Hin, int Win, int Hout, int Wout) {
  __shared__ float zs[32 * UK_NPX];
  const int tiles_x = (Win + UK_OW - 1) / UK_OW, tiles_y = (Hin + UK_R - 1) / UK_R;
  int bid = blockIdx.x;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int a0 = ty * UK_R, b0 = tx * UK_OW;
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int Cg4 = Cg >> 2, nchg = Cg >> 4, nch = 2 * nchg;
  const unsigned plane = (unsigned)Hin * Win;
  const __amdgpu_buffer_rsrc_t r1 = uniform_rsrc(g1 + (size_t)n * Cg4 * plane * 4, (unsigned)(Cg4 * plane * 16));
  const __amdgpu_buffer_rsrc_t r2 = uniform_rsrc(gs + (size_t)n * Cg4 * plane * 4, (unsigned)(Cg4 * plane * 16));
  constexpr unsigned OOB = 0xFFFFFFF0u;
  // Z tile k of this wave: gradient row a0 + wave + 4k, column b0 + j; the lane's quads 2h, 2h + 1 of each chunk
  unsigned po[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int iy = a0 + wave + 4 * k, ix = b0 + j;
    po[k] = iy < Hin && ix < Win ? ((unsigned)(2 * h) * plane + (unsigned)iy * Win + ix) * 16u : OOB;
  }
  const long pst = (long)nch * 64;   // fragments per plane
  const __amdgpu_buffer_rsrc_t wr = uniform_rsrc(wp, (unsigned)(3 * pst * 16));
  auto ldw = [&](bf16x8 (&a)[3], int ch) {
#pragma unroll
    for (int q = 0; q < 3; ++q) a[q] = ld_bf8(wr, lane * 16, (int)((q * pst + (long)ch * 64) * 16));
  };
  auto ldx = [&](f32x4 (&v)[4][2], int ch) {
    const bool second = ch >= nchg;   // wave-uniform: chunks 0..nchg-1 read g1, the rest gs
    const __amdgpu_buffer_rsrc_t r = second ? r2 : r1;
    const unsigned co = (unsigned)(second ? ch - nchg : ch) * 4u * plane * 16u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool ok = po[k] != OOB;
      v[k][0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? po[k] + co : OOB, 0, 0));
      v[k][1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, ok ? po[k] + co + plane * 16u : OOB,
                                                                                 0, 0));
    }
  };
  f32x16 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f32x16{0};
  auto compute = [&](const bf16x8 (&a)[3], const f32x4 (&v)[4][2]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x[8] = {v[k][0][0], v[k][0][1], v[k][0][2], v[k][0][3], v[k][1][0], v[k][1][1], v[k][1][2], v[k][1][3]};
      bf16x8 b[3];
      split3x8(x, b);
      acc[k] = mfma_x6(a, b, acc[k]);
    }
  };
  // chunk ch + 1's weights and gradients in flight during chunk ch's MFMAs (ping-pong; nch is even)
  bf16x8 wa[3], wb[3];
  f32x4 xa[4][2], xb[4][2];
  ldw(wa, 0);
  ldx(xa, 0);
#pragma unroll 1
  for (int ch = 0; ch < nch; ch += 2) {
    ldw(wb, ch + 1);
    ldx(xb, ch + 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(wa, xa);
    if (ch + 2 < nch) {
      ldw(wa, ch + 2);
      ldx(xa, ch + 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    compute(wb, xb);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = acc_row(r, h);
      if (row < 30) zs[row * UK_NPX + (wave + 4 * k) * 32 + j] = acc[k][r];
    }
  __syncthreads();
  // gather: thread -> output row 2 al + py, columns 2 bl, 2 bl + 1 (32 contiguous bytes per thread)
  for (int e = threadIdx.x; e < 2 * UK_R * UK_OW; e += 256) {
    const int yl = e / UK_OW, bl = e - yl * UK_OW;
    const int al = yl >> 1, py = yl & 1;
    const int a = a0 + al, b = b0 + bl;
    if (a >= Hin || b >= Win) continue;
    f32x4 o[2];
#pragma unroll
    for (int px = 0; px < 2; ++px) {
      float s[3] = {0.f, 0.f, 0.f};
      // taps of output parity (py, px): ky = 1 (row a) for py = 0; ky = 0 (row a + 1), 2 (row a) for py = 1
#pragma unroll
      for (int ky = 0; ky < 3; ++ky) {
        if ((ky & 1) == py) continue;   // ky = 1 <-> py = 0
        const int dr = (py + 1 - ky) >> 1;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
          if ((kx & 1) == px) continue;
          const int dc = (px + 1 - kx) >> 1;
          const int q = (al + dr) * 32 + bl + dc;
#pragma unroll
          for (int c = 0; c < 3; ++c) s[c] += zs[(c * 9 + ky * 3 + kx) * UK_NPX + q];
        }
      }
      if (py == 0 && px == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) s[c] += zs[(27 + c) * UK_NPX + al * 32 + bl];
      }
      o[px] = f32x4{s[0], s[1], s[2], 0.f};
    }
    const int y = 2 * a + py, x = 2 * b;
    if (y < Hout) {
      float* d = dx + (((size_t)n * Hout + y) * Wout + x) * 4;
      if (x + 1 < Wout) {
        st4(d, o[0]);
        st4(d + 4, o[1]);
      } else if (x < Wout) {
        st4(d, o[0]);
      }
    }
  }
}

template <int IT, int EPI, int PT>
int launch_down_x6_pt(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Wout + XD_TW - 1) / XD_TW) * ((p.Hout + xd_th<PT>() - 1) / xd_th<PT>()) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * ((((p.Cin + 3) / 4) * 4 + 15) / 16) * 25 * IT * 64;
  ICA_LAUNCH((conv_down_x6_kernel<IT, EPI, PT>), dim3(tiles, ncb), dim3(256), 0, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}

// fragments of the order-0 x6 pack per plane, and of the tap-pair extension conv_down_x6w reads (KS = 5, IT = 4)
static inline long x6_plane_frags(int O, int C, int KS, int IT) {
  return (long)((O + IT * 32 - 1) / (IT * 32)) * ((((C + 3) / 4) * 4 + 15) / 16) * KS * KS * IT * 64;
}
static inline long x6w_plane_frags(int O, int C) {
  const int nch8 = ((C + 3) / 4 + 1) / 2;
  return (long)((O + 127) / 128) * ((nch8 >> 1) * 25 + (nch8 & 1) * XW_NS) * 4 * 64;
}

template <int EPI, int PT>
int launch_down_x6w(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Wout + XD_TW - 1) / XD_TW) * ((p.Hout + 4 * PT - 1) / (4 * PT)) * p.N;
  const int ncb = (p.Cout + 127) / 128;
  ConvParams q = p;
  q.wp = reinterpret_cast<const float*>(reinterpret_cast<const char*>(p.wp) +
                                        3 * x6_plane_frags(p.Cout, p.Cin, 5, 4) * 16);
  ICA_LAUNCH((conv_down_x6w_kernel<EPI, PT>), dim3(tiles, ncb), dim3(512), 0, st, q, x6w_plane_frags(p.Cout, p.Cin));
  ICA_CHECK_LAUNCH();
  return 0;
}

constexpr int XS_SMALL_PX = 32 * 32;   // the small-grid x6 kernels: low-resolution side <= 32 x 32 per image

template <int IT, int EPI>
int launch_down_small_x6(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Wout + XSD_TW - 1) / XSD_TW) * ((p.Hout + XSD_TH - 1) / XSD_TH) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * ((((p.Cin + 3) / 4) * 4 + 15) / 16) * 25 * IT * 64;
  ICA_LAUNCH((conv_down_small_x6_kernel<IT, EPI>), dim3(tiles, ncb), dim3(256), 0, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}

// Small grids (<= 32 x 32 outputs per image, a per-image rule: image b of a batch runs the same kernel at any
// batch size) take the small-grid kernel.  Otherwise PT = 1 when the PT = 2 grid would leave CUs idle (fewer
// blocks than the 256 CUs): PT = 1 and PT = 2 run the same MFMA and epilogue sequence per output (same bits), so
// this batch-dependent choice keeps every image's result.
template <int IT, int EPI>
int launch_down_x6(const ConvParams& p, hipStream_t st) {
  if (p.Hout * p.Wout <= XS_SMALL_PX) return launch_down_small_x6<IT, EPI>(p, st);
  const int blocks2 = ((p.Wout + XD_TW - 1) / XD_TW) * ((p.Hout + xd_th<X6_PT>() - 1) / xd_th<X6_PT>()) * p.N *
                      ((p.Cout + IT * 32 - 1) / (IT * 32));
  if constexpr (IT == 4) {   // 128 output channels: the 8-wave kernel
    if (blocks2 < 256) return launch_down_x6w<EPI, 1>(p, st);
    return launch_down_x6w<EPI, 2>(p, st);
  }
  if (blocks2 < 256) return launch_down_x6_pt<IT, EPI, 1>(p, st);
  return launch_down_x6_pt<IT, EPI, X6_PT>(p, st);
}

static inline long rgb5_plane_frags(int O, int IT) { return (long)((O + IT * 32 - 1) / (IT * 32)) * RGB5_KY * IT * 64; }

template <int EPI>
int launch_rgb_x6(const ConvParams& p, hipStream_t st) {
  if (p.Cout != 32 * RGB5_IT) return -3;   // the LDS-resident weights: one 128-row block
  const long ps = rgb5_plane_frags(p.Cout, RGB5_IT);
  const int total = ((p.Wout + 31) / 32) * p.Hout * p.N;
  constexpr bool BWD = EPI == EPI_IGDN_BWD || EPI == EPI_GDN_BWD;
  // one persistent block per CU; its waves take consecutive row tiles of a contiguous run
  const int nblk = std::max(1, std::min(ica_cu_count(), (total + (BWD ? 3 : 7)) / (BWD ? 4 : 8)));
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(BWD ? reinterpret_cast<const void*>(&conv_rgb5_bwd_x6_kernel<BWD ? EPI : EPI_IGDN_BWD>)
                                  : reinterpret_cast<const void*>(&conv_rgb5_x6_kernel<BWD ? EPI_GDN : EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, RGB5_LDS);
    attr_set = true;
  }
  if constexpr (BWD) {
    ICA_LAUNCH((conv_rgb5_bwd_x6_kernel<EPI>), dim3(nblk), dim3(256), RGB5_LDS, st, p, ps, nblk);
  } else if constexpr (RGB5_W && EPI != EPI_BIAS) {
    const int nb4 = std::max(1, std::min(ica_cu_count(), (total + 3) / 4));
    static bool attr_w = false;
    if (!attr_w) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_rgb5w_x6_kernel<EPI>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, RGB5_LDS);
      attr_w = true;
    }
    ICA_LAUNCH((conv_rgb5w_x6_kernel<EPI>), dim3(nb4), dim3(256), RGB5_LDS, st, p, ps, nb4);
  } else {
    ICA_LAUNCH((conv_rgb5_x6_kernel<EPI>), dim3(nblk), dim3(512), RGB5_LDS, st, p, ps, nblk);
  }
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int EPI>
int launch_rgb5_bf16(const ConvParams& p, hipStream_t st) {
  const int total = ((p.Wout + 31) / 32) * p.Hout * p.N;
  const int nblk = std::max(1, std::min(ica_cu_count(), (total + 7) / 8));
  constexpr int lds = rgb5b_lds_bytes<EPI>();
  static_assert(lds <= 160 * 1024, "conv_rgb5_bf16 LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_rgb5_bf16_kernel<EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_set = true;
  }
  ICA_LAUNCH((conv_rgb5_bf16_kernel<EPI>), dim3(nblk), dim3(512), lds, st, p, nblk);
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int IT, int EPI, int CG, int PT>
int launch_up_x6_pt(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<PT>() - 1) / xu_th<PT>()) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * 25 * (p.Cin / 16) * IT * 64;
  constexpr size_t lds = xu_lds_bytes<CG, PT>();
  static_assert(lds <= 160 * 1024, "conv_up_x6 channel group exceeds LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_x6_kernel<IT, EPI, CG, PT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_x6_kernel<IT, EPI, CG, PT>), dim3(tiles, ncb), dim3(256), lds, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int IT, int EPI, int CG, int PT = 2>
int launch_up_x6w(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<PT>() - 1) / xu_th<PT>()) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * 25 * (p.Cin / 16) * IT * 64;
  // the GDN backward's t slabs (8 waves x 4 IT x 64 entries) reuse the patch LDS
  constexpr bool BWD = EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD;
  constexpr size_t slabs = BWD ? (size_t)8 * 4 * IT * 64 * sizeof(f32x4) : 0;
  constexpr size_t lds = std::max((size_t)xu_lds_bytes<CG, PT>(), slabs);
  static_assert(lds <= 160 * 1024, "conv_up_x6w LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_x6w_kernel<IT, EPI, CG, PT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_x6w_kernel<IT, EPI, CG, PT>), dim3(tiles, ncb), dim3(512), lds, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}

// fraction of the launch's last round of 256 one-per-CU blocks that is busy, over all rounds
static inline double x6_round_fill(long blocks) {
  const long rounds = (blocks + 255) / 256;
  return rounds ? (double)blocks / (double)(rounds * 256) : 1.0;
}

// PT = 1 when the PT = 2 grid leaves a partly-empty last round and halving the blocks fills the rounds clearly
// better (config 2's 32x48-input layers: 384 blocks = 1.5 rounds -> 768 = 3 rounds); same bits either way
template <int IT, int EPI, int CG>
int launch_up_x6(const ConvParams& p, hipStream_t st) {
  const long ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long b2 = (long)((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<2>() - 1) / xu_th<2>()) * p.N * ncb;
  const long b1 = (long)((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<1>() - 1) / xu_th<1>()) * p.N * ncb;
  constexpr bool BWD = EPI == EPI_GDN_BWD || EPI == EPI_IGDN_BWD;
  // The GDN backward: the 4-wave kernel (one (y, s) read per output, its wide epilogue) for 128-channel inputs, the
  // 8-wave slab kernel for 64-channel groups (Cin = 192: g_a.6's input gradient).  At config 2 the 8-wave slab kernel
  // of round 5 took g_a.2.dgrad 3.56 -> 3.63-3.67 ms and 5.83 -> 8.84 GB per launch ((y, s) read twice at PT = 2);
  // for the 32 x 48-input g_a.6.dgrad it is the faster one (0.335 vs 0.41 ms).  PT follows the round fill; each
  // family's PT = 1 and PT = 2 forms give the same bits, and the family depends on the layer only (batch-independent
  // bits).  ICA_UPW_BWD_ALL builds put every GDN backward on the slab kernel (round 5) for A/B runs.
#ifdef ICA_UPW_BWD_ALL
  constexpr bool SLAB = BWD && IT == 4;
#else
  constexpr bool SLAB = BWD && IT == 4 && CG == 64;
#endif
  if (x6_round_fill(b1) > x6_round_fill(b2) + 0.15) {
    if constexpr (SLAB) return launch_up_x6w<IT, EPI, CG, 1>(p, st);
    return launch_up_x6_pt<IT, EPI, CG, 1>(p, st);
  }
  // the 8-wave class-per-wave kernel: forward layers (bias / IGDN) and the slab GDN backward
  if constexpr (SLAB) return launch_up_x6w<IT, EPI, CG, 2>(p, st);
  if constexpr (IT == 4 && !BWD) return launch_up_x6w<IT, EPI, CG>(p, st);
  return launch_up_x6_pt<IT, EPI, CG, X6_PT>(p, st);
}

// the k3 s2 input gradients of cheng2020's stride-2 residual blocks (conv_ex kind 1, x6): bias (+ residual) epilogue;
// KS = 1: the 1x1 stride-2 skips' input gradients (one tap in class (0, 0), zeros elsewhere)
template <int IT, int FX, int CG, int PT, int KS = 3>
int launch_up3s2_x6_pt(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<PT>() - 1) / xu_th<PT>()) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * KS * KS * (p.Cin / 16) * IT * 64;
  constexpr size_t lds = xu_lds_bytes<CG, PT>();
  static_assert(lds <= 160 * 1024, "conv_up_x6 channel group exceeds LDS");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_x6_kernel<IT, EPI_BIAS, CG, PT, KS, FX>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_x6_kernel<IT, EPI_BIAS, CG, PT, KS, FX>), dim3(tiles, ncb), dim3(256), lds, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}
template <int IT, int FX, int CG>
int launch_up3s2_x6(const ConvParams& p, hipStream_t st) {
  const long ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long b2 = (long)((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<2>() - 1) / xu_th<2>()) * p.N * ncb;
  const long b1 = (long)((p.Win + XU_TW - 1) / XU_TW) * ((p.Hin + xu_th<1>() - 1) / xu_th<1>()) * p.N * ncb;
  if (x6_round_fill(b1) > x6_round_fill(b2) + 0.15) return launch_up3s2_x6_pt<IT, FX, CG, 1>(p, st);
  return launch_up3s2_x6_pt<IT, FX, CG, 2>(p, st);
}
static int pick_up3s2_x6(const ConvParams& p, int it, int epi, int fx, hipStream_t st) {
  if (epi != EPI_BIAS || (fx != 0 && fx != FX_RES) || p.Cout % 32 != 0) return -4;
  if (p.Hout != 2 * p.Hin || p.Wout != 2 * p.Win || (p.pl & (PL_IN | PL_OUT))) return -2;
  const bool res = fx == FX_RES;
  // Cin = 192: the whole channel range in LDS at PT = 1 (124 KB), one fill per block -- in 64-channel groups each
  // class re-staged a group for 1-4 taps (g_a.2.conv1.dgrad 4.33 ms at the config-3 shapes)
  if (it == 6 && p.Cin == 192)
    return res ? launch_up3s2_x6_pt<6, FX_RES, 192, 1>(p, st) : launch_up3s2_x6_pt<6, 0, 192, 1>(p, st);
  if (it == 4 && p.Cin == 128)
    return res ? launch_up3s2_x6<4, FX_RES, 128>(p, st) : launch_up3s2_x6<4, 0, 128>(p, st);
  return -3;
}

template <int IT, int EPI>
int launch_up_small_x6(const ConvParams& p, hipStream_t st) {
  const int tiles = ((p.Win + 15) / 16) * ((p.Hin + XSU_TH - 1) / XSU_TH) * p.N;
  const int ncb = (p.Cout + IT * 32 - 1) / (IT * 32);
  const long ps = (long)ncb * 25 * (p.Cin / 16) * IT * 64;
  const size_t lds = (size_t)std::max(3 * (p.Cin / 8) * XSU_PLANE, xs_red_entries<IT>()) * 16;
  if (lds > 160 * 1024) return -2;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&conv_up_small_x6_kernel<IT, EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  ICA_LAUNCH((conv_up_small_x6_kernel<IT, EPI>), dim3(4 * tiles, ncb), dim3(256), lds, st, p, ps);
  ICA_CHECK_LAUNCH();
  return 0;
}

template <int IT, int EPI>
int pick_up_x6(const ConvParams& p, hipStream_t st) {
  if (p.Hin * p.Win <= XS_SMALL_PX && p.Cin >= 64 && p.Cin % 16 == 0) return launch_up_small_x6<IT, EPI>(p, st);
  if (p.Cin <= 128 && p.Cin % 16 == 0) {
    if (p.Cin == 128) return launch_up_x6<IT, EPI, 128>(p, st);
    if (p.Cin == 64) return launch_up_x6<IT, EPI, 64>(p, st);
    return -2;
  }
  if (p.Cin % 64 == 0) return launch_up_x6<IT, EPI, 64>(p, st);
  return -2;
}

}  // namespace

// bf16 RGB-side conv_down (ica_conv_ex prec = 1, kind 0, k5 s2, Cin <= 3, 128 outputs, plain fill, row-major input;
// ica_conv.hip routes here): conv_rgb5_bf16_kernel on the order-2 pack of ica_pack_conv_weight_bf16
int ica_rgb5_bf16_dispatch(const ConvParams& p, int epi, hipStream_t st) {
  if (p.Cin > 3 || p.Cout != 32 * RGB5_IT || (p.pl & PL_IN)) return -3;
  if (p.Hout * 2 != p.Hin + (p.Hin & 1) || p.Wout * 2 != p.Win + (p.Win & 1)) return -2;
  switch (epi) {
    case EPI_BIAS: return launch_rgb5_bf16<EPI_BIAS>(p, st);
    case EPI_GDN: return launch_rgb5_bf16<EPI_GDN>(p, st);
    case EPI_IGDN_BWD: return launch_rgb5_bf16<EPI_IGDN_BWD>(p, st);
    default: return -5;
  }
}

// the dense tap-row pack in `planes` split planes (3: x6; 1: bf16 = the round-to-nearest hi plane)
int ica_pack_rgb5_planes(const float* w, void* dst, int O, int C, long so, long sc, int it, int planes,
                         hipStream_t st) {
  if (C > 3 || C <= 0 || it <= 0 || (planes != 1 && planes != 3)) return -2;
  const long t3 = rgb5_plane_frags(O, it) * 8;
  ICA_LAUNCH(pack_conv_rgb5_x6_kernel, dim3((t3 + 255) / 256), dim3(256), 0, st, w, reinterpret_cast<__bf16*>(dst),
             O, C, so, sc, it, t3, planes);
  ICA_CHECK_LAUNCH();
  return 0;
}

// x6 launches (ica_conv_ex with prec = 2): the k5 s2 conv (kind 0) and transposed conv (kind 1) layers of the
// bmshj2018 transforms.  Returns -4 / -3 / -2 / -5 for shapes / epilogues without an x6 kernel: nothing falls back
// here; hip_ops.x6_ok restates this coverage so that PackedConv keeps the fp32 pack for such layers.
int ica_conv_x6_dispatch(const ConvParams& p, int kind, int KS, int S, int it, int epi, int fx, hipStream_t st) {
  if (kind == 1 && KS == 3 && S == 2) return pick_up3s2_x6(p, it, epi, fx, st);
  if (kind == 1 && KS == 1 && S == 2) {   // cheng2020's 1x1 stride-2 skips (no residual)
    if (epi != EPI_BIAS || fx != 0 || p.Cout % 32 != 0) return -4;
    if (p.Hout != 2 * p.Hin || p.Wout != 2 * p.Win || (p.pl & (PL_IN | PL_OUT))) return -2;
    if (it == 6 && p.Cin == 192) return launch_up3s2_x6_pt<6, 0, 192, 1, 1>(p, st);
    if (it == 4 && p.Cin == 128) return launch_up3s2_x6_pt<4, 0, 128, 2, 1>(p, st);
    return -3;
  }
  if (KS != 5 || S != 2 || fx != 0) return -4;
  if (p.Cout % 32 != 0) return -4;
  if (kind == 0) {
    if (p.Hout * 2 != p.Hin + (p.Hin & 1) || p.Wout * 2 != p.Win + (p.Win & 1)) return -2;
    if (p.Cin <= 4) {   // RGB-sized input: conv_rgb5_x6 on the dense tap-row pack (ica_pack_conv_weight_x6 order 2)
      if (it != 4 || p.Cin > 3) return -3;
      if (p.pl & PL_IN) return -2;   // the image side stays row-major
      switch (epi) {
        case EPI_BIAS: return launch_rgb_x6<EPI_BIAS>(p, st);
        case EPI_GDN: return launch_rgb_x6<EPI_GDN>(p, st);
        case EPI_IGDN_BWD: return launch_rgb_x6<EPI_IGDN_BWD>(p, st);
        default: return -5;
      }
    }
    if (p.Cin < 16) return -2;
    if (it == 4) {
      switch (epi) {
        case EPI_BIAS: return launch_down_x6<4, EPI_BIAS>(p, st);
        case EPI_GDN: return launch_down_x6<4, EPI_GDN>(p, st);
        case EPI_IGDN_BWD: return launch_down_x6<4, EPI_IGDN_BWD>(p, st);
        default: return -5;
      }
    }
    if (it == 3 && epi == EPI_BIAS) return launch_down_x6<3, EPI_BIAS>(p, st);
    return -3;
  }
  if (kind == 1) {
    if (p.Hout != 2 * p.Hin || p.Wout != 2 * p.Win) return -2;
    if (it == 4) {
      switch (epi) {
        case EPI_BIAS: return pick_up_x6<4, EPI_BIAS>(p, st);
        case EPI_IGDN: return pick_up_x6<4, EPI_IGDN>(p, st);
        case EPI_GDN_BWD: return pick_up_x6<4, EPI_GDN_BWD>(p, st);
        default: return -5;
      }
    }
    return -3;
  }
  return -6;
}

extern "C" {

size_t ica_pack_conv_weight_x6_size(int O, int C, int KS, int IT) {
  // the 16-channel-chunk pack, plus (KS = 5, IT = 4) the tap-pair pack of conv_down_x6w behind it
  return (size_t)3 * 8 * (x6_plane_frags(O, C, KS, IT) + (KS == 5 && IT == 4 ? x6w_plane_frags(O, C) : 0));
}

size_t ica_pack_gdn_x6_size(int C) { return (size_t)3 * (C / 32) * (C / 32) * 2048; }

// three bf16 planes of an fp32 gamma' / gamma'^T pack (ica_pack_gdn output) for the x6 GDN epilogues
int ica_pack_gdn_x6(const float* gp, void* dst, int C, hipStream_t st) {
  if (C % 32 != 0) return -2;
  const long total = (long)(C / 32) * (C / 32) * 1024;
  ICA_LAUNCH(pack_gdn_x6_kernel, dim3((total + 255) / 256), dim3(256), 0, st, gp,
                     reinterpret_cast<__bf16*>(dst), total);
  ICA_CHECK_LAUNCH();
  return 0;
}

// three bf16 planes (hi, mid, lo) of the 16-channel-chunk fragment pack; order 0: conv_down [cb][chunk][tap],
// order 1: conv_up [cb][tap][chunk]; order 2: the dense tap-row pack of a k5 conv_down with C <= 3 input channels
// (conv_rgb5_x6: g_a.0 forward, g_s.6 input gradient), [cb][ky][it] (smaller than the size above)
int ica_pack_conv_weight_x6(const float* w, void* dst, int O, int C, int KS, long so, long sc, int order, int it,
                            hipStream_t st) {
  if (it <= 0) return -3;
  if (order == 2) {
    if (KS != 5 || C > 3 || C <= 0) return -2;
    return ica_pack_rgb5_planes(w, dst, O, C, so, sc, it, 3, st);
  }
  if (order != 0 && order != 1) return -2;
  const long total = x6_plane_frags(O, C, KS, it) * 8;
  ICA_LAUNCH(pack_conv_x6_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w,
                     reinterpret_cast<__bf16*>(dst), O, C, KS, so, sc, it, order, total);
  ICA_CHECK_LAUNCH();
  if (KS == 5 && it == 4 && order == 0) {   // conv_down_x6w's tap-pair pack (conv_up packs leave it unused)
    const long t2 = x6w_plane_frags(O, C) * 8;
    ICA_LAUNCH(pack_conv_x6w_kernel, dim3((t2 + 255) / 256), dim3(256), 0, st, w,
               reinterpret_cast<__bf16*>(dst) + 3 * total, O, C, so, sc, it, t2);
    ICA_CHECK_LAUNCH();
  }
  return 0;
}

size_t ica_pack_up3k3_x6_size(int Cg) { return (size_t)3 * (2 * Cg / 16) * 64 * 16; }

// the fused g_a.0 input-gradient pack: conv1 [Cg][3][3][3] and skip [Cg][3][1][1] weights -> three bf16 planes
int ica_pack_up3k3_x6(const float* w1, const float* ws, void* dst, int Cg, hipStream_t st) {
  if (Cg <= 0 || Cg % 16 != 0) return -2;
  const long total = (long)(2 * Cg / 16) * 512;
  ICA_LAUNCH(pack_up3k3_x6_kernel, dim3((total + 255) / 256), dim3(256), 0, st, w1, ws, reinterpret_cast<__bf16*>(dst),
             Cg, total);
  ICA_CHECK_LAUNCH();
  return 0;
}

// dx [N][1][Hout][Wout][4] = conv3x3_s2^T(g1) + conv1x1_s2^T(gs); g1, gs [N][Cg/4][Hin][Win][4] row-major,
// Hin = ceil(Hout / 2), Win = ceil(Wout / 2)
int ica_conv_up3k3_x6(const float* g1, const float* gs, const void* wp, float* dx, int N, int Cg, int Hin, int Win,
                      int Hout, int Wout, hipStream_t st) {
  if (Cg <= 0 || Cg % 16 != 0 || N <= 0) return -2;
  if (Hin != (Hout + 1) / 2 || Win != (Wout + 1) / 2) return -3;
  const long blocks = (long)((Win + UK_OW - 1) / UK_OW) * ((Hin + UK_R - 1) / UK_R) * N;
  ICA_LAUNCH(conv_up3k3_x6_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g1, gs, wp, dx, Cg, Hin, Win, Hout, Wout);
  ICA_CHECK_LAUNCH();
  return 0;
}

#ifdef ICA_CLOCK_STAMP
// diagnostic builds only (scripts/clock_probe.py): where the x6 kernels put their entry / exit stamps
int ica_diag_stamp_buffer(unsigned long long* buf, unsigned slots) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(ica_stamp_buf), &buf, sizeof(buf)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(ica_stamp_slots), &slots, sizeof(slots)) != hipSuccess) return -1;
  return 0;
}
#endif

}  // extern "C"

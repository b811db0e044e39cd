// Experiment v2: fp32-accurate conv_down (k5 s2) on bf16 MFMA, exact 3-way splits (6 products per k-step), with
//   * 8-channel chunks and tap PAIRS as the 16-deep MFMA k (lane half h = tap 2tp + h), 13 pairs cover 25 taps;
//   * a double-buffered LDS patch (3 bf16 planes per buffer): the next chunk's HBM loads and splits are spread
//     over the current chunk's steps (one barrier per chunk, no fill stall);
//   * PT = 2 pixel tiles per wave (256 px per block), one block per CU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/x6_down2.cpp -o scripts/exp/x6_down2
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <random>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void split3(f32x4 v, u32x2& h, u32x2& m, u32x2& l) {
  bf16x4 bh, bm, bl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const __bf16 a = (__bf16)v[e];
    const float r1 = v[e] - (float)a;
    const __bf16 b = (__bf16)r1;
    const float r2 = r1 - (float)b;
    bh[e] = a;
    bm[e] = b;
    bl[e] = (__bf16)r2;
  }
  h = __builtin_bit_cast(u32x2, bh);
  m = __builtin_bit_cast(u32x2, bm);
  l = __builtin_bit_cast(u32x2, bl);
}

constexpr int KS = 5, S = 2, TW = 32, IT = 4, KK = KS * KS, NTP = (KK + 1) / 2;  // 13 tap pairs

template <int PT, int LAG>
__global__ __launch_bounds__(256, 1) void down_v2(const float* __restrict__ x, float* __restrict__ y,
                                                  const bf16x8* __restrict__ wp, const float* __restrict__ bias,
                                                  int N, int Cin, int Hin, int Win, int Cout, int Hout, int Wout) {
  constexpr int TH = 4 * PT, PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;
  constexpr int NQ = 2;                          // channel quads per 8-channel chunk
  constexpr int NF = (NQ * PLANE + 255) / 256;   // fill items per thread per chunk
  static_assert(NF + LAG <= NTP, "the fill of the next chunk must fit in one chunk's steps");
  // [buf][plane][pixel] 16-B entries = 8 channels as bf16
  __shared__ u32x4 patch[2 * 3 * PLANE];
  const int tiles_x = Wout / TW, tiles_y = Hout / TH;
  int bid = blockIdx.x;
  const int cb = blockIdx.y;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 2, ix0 = ox0 * S - 2;
  const int Cin4 = Cin >> 2, nch = Cin / 8;
  f32x16 acc[PT][IT];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
  const unsigned xplane = (unsigned)Hin * Win;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x) + (size_t)n * Cin4 * xplane * 4, 0, (int)(Cin4 * xplane * 16), 0x00020000);
  auto load_item = [&](int ch, int i) -> f32x4 {
    const int e = threadIdx.x + 256 * i;
    const int q = e / PLANE, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
    const int iy = iy0 + pr, ix = ix0 + pc;
    const bool ok = e < NQ * PLANE && ch < nch && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
    const unsigned vo = ((unsigned)(ch * NQ + q) * xplane + (unsigned)iy * Win + ix) * 16u;
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
  };
  auto put_item = [&](int buf, int i, f32x4 v) {
    const int e = threadIdx.x + 256 * i;
    if (e < NQ * PLANE) {
      const int q = e / PLANE, pix = e - q * PLANE;
      u32x2 hh, mm, ll;
      split3(v, hh, mm, ll);
      u32x2* p2 = reinterpret_cast<u32x2*>(patch);
      p2[((buf * 3 + 0) * PLANE + pix) * 2 + q] = hh;
      p2[((buf * 3 + 1) * PLANE + pix) * 2 + q] = mm;
      p2[((buf * 3 + 2) * PLANE + pix) * 2 + q] = ll;
    }
  };
  // chunk 0, synchronously
  {
    f32x4 v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) v[i] = load_item(0, i);
#pragma unroll
    for (int i = 0; i < NF; ++i) put_item(0, i, v[i]);
    __syncthreads();
  }
  const int total = nch * NTP;
  const bf16x8* wb = wp + (size_t)cb * nch * NTP * 3 * IT * 64 + lane;
  auto ldw = [&](bf16x8 (&a)[3][IT], int g) {
    const bf16x8* w = wb + (size_t)min(g, total - 1) * 3 * IT * 64;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int it = 0; it < IT; ++it) a[p][it] = w[(p * IT + it) * 64];
  };
  f32x4 ring[LAG];   // fill loads in flight (item i loaded at step i, written at step i + LAG)
  // LDS entry offset of tap t for pixel tile tt of this lane (buffer/plane base added later)
  auto tap_off = [&](int tt, int t) {
    t = min(t, KK - 1);   // tap 25 (pad) carries zero weights
    const int ky = t / KS, kx = t - ky * KS;
    return (S * (wave * PT + tt) + ky) * PC + S * j + kx;
  };
  auto step = [&](bf16x8 (&cur)[3][IT], bf16x8 (&nxt)[3][IT], int g) {
    const int ch = g / NTP, tp = g - ch * NTP;
    const int buf = ch & 1;
    __builtin_amdgcn_sched_barrier(0);
    ldw(nxt, g + 1);
    __builtin_amdgcn_sched_barrier(0);
    // spread fill of chunk ch + 1 into the other buffer: item s - LAG is written, item s loaded
    if (tp >= LAG && tp < NF + LAG) put_item(buf ^ 1, tp - LAG, ring[LAG - 1]);
#pragma unroll
    for (int r = LAG - 1; r > 0; --r) ring[r] = ring[r - 1];
    if (tp < NF) ring[0] = load_item(ch + 1, tp);
    __builtin_amdgcn_sched_barrier(0);
    const int t = 2 * tp + h;
#pragma unroll
    for (int tt = 0; tt < PT; ++tt) {
      const int o = tap_off(tt, t);
      const bf16x8 b0 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 0) * PLANE + o]);
      const bf16x8 b1 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 1) * PLANE + o]);
      const bf16x8 b2 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 2) * PLANE + o]);
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        acc[tt][it] = mfma(cur[2][it], b0, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b2, acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b1, acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b0, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b1, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b0, acc[tt][it]);
      }
    }
    if (tp == NTP - 1) __syncthreads();   // chunk done: its buffer is free, the next one is complete
  };
  bf16x8 fa[3][IT], fb[3][IT];
  ldw(fa, 0);
  int g = 0;
#pragma unroll 1
  for (; g + 1 < total; g += 2) {
    step(fa, fb, g);
    step(fb, fa, g + 1);
  }
  if (g < total) step(fa, fb, g);
  const int C4o = (Cout + 3) >> 2;
#pragma unroll
  for (int tt = 0; tt < PT; ++tt) {
    const int oy = oy0 + wave * PT + tt, ox = ox0 + j;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int c0 = cb * IT * 32 + it * 32 + 8 * gq + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[tt][it][4 * gq + e] + bias[c0 + e];
        *reinterpret_cast<f32x4*>(y + ((((size_t)n * C4o + (c0 >> 2)) * Hout + oy) * Wout + ox) * 4) = v;
      }
  }
}

// v3: 8 waves (2 per SIMD); wave w: pixel tiles of row group (w & 3) (PT tiles), output-channel half (w >> 2)
// (ITW = 2 tiles of 32 channels); same double-buffered 8-channel tap-pair patch as v2.
template <int PT, int LAG>
__global__ __launch_bounds__(512, 1) void down_v3(const float* __restrict__ x, float* __restrict__ y,
                                                  const bf16x8* __restrict__ wp, const float* __restrict__ bias,
                                                  int N, int Cin, int Hin, int Win, int Cout, int Hout, int Wout) {
  constexpr int ITW = 2;
  constexpr int TH = 4 * PT, PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;
  constexpr int NQ = 2;
  constexpr int NF = (NQ * PLANE + 511) / 512;
  static_assert(NF + LAG <= NTP, "fill must fit in one chunk");
  __shared__ u32x4 patch[2 * 3 * PLANE];
  const int tiles_x = Wout / TW, tiles_y = Hout / TH;
  int bid = blockIdx.x;
  const int cb = blockIdx.y;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int wr = wave & 3, wc = wave >> 2;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 2, ix0 = ox0 * S - 2;
  const int Cin4 = Cin >> 2, nch = Cin / 8;
  f32x16 acc[PT][ITW];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < ITW; ++it) acc[t][it] = f32x16{0};
  const unsigned xplane = (unsigned)Hin * Win;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x) + (size_t)n * Cin4 * xplane * 4, 0, (int)(Cin4 * xplane * 16), 0x00020000);
  auto load_item = [&](int ch, int i) -> f32x4 {
    const int e = threadIdx.x + 512 * i;
    const int q = e / PLANE, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
    const int iy = iy0 + pr, ix = ix0 + pc;
    const bool ok = e < NQ * PLANE && ch < nch && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
    const unsigned vo = ((unsigned)(ch * NQ + q) * xplane + (unsigned)iy * Win + ix) * 16u;
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
  };
  auto put_item = [&](int buf, int i, f32x4 v) {
    const int e = threadIdx.x + 512 * i;
    if (e < NQ * PLANE) {
      const int q = e / PLANE, pix = e - q * PLANE;
      u32x2 hh, mm, ll;
      split3(v, hh, mm, ll);
      u32x2* p2 = reinterpret_cast<u32x2*>(patch);
      p2[((buf * 3 + 0) * PLANE + pix) * 2 + q] = hh;
      p2[((buf * 3 + 1) * PLANE + pix) * 2 + q] = mm;
      p2[((buf * 3 + 2) * PLANE + pix) * 2 + q] = ll;
    }
  };
  {
    f32x4 v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) v[i] = load_item(0, i);
#pragma unroll
    for (int i = 0; i < NF; ++i) put_item(0, i, v[i]);
    __syncthreads();
  }
  const int total = nch * NTP;
  // weights packed [cb][chunk8][tp][plane][it(4)][lane]: this wave uses tiles 2 wc, 2 wc + 1
  const bf16x8* wb = wp + (size_t)cb * nch * NTP * 3 * IT * 64 + lane + wc * ITW * 64;
  auto ldw = [&](bf16x8 (&a)[3][ITW], int g) {
    const bf16x8* w = wb + (size_t)min(g, total - 1) * 3 * IT * 64;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int it = 0; it < ITW; ++it) a[p][it] = w[(p * IT + it) * 64];
  };
  f32x4 ring[LAG];
  auto tap_off = [&](int tt, int t) {
    t = min(t, KK - 1);
    const int ky = t / KS, kx = t - ky * KS;
    return (S * (wr * PT + tt) + ky) * PC + S * j + kx;
  };
  auto step = [&](bf16x8 (&cur)[3][ITW], bf16x8 (&nxt)[3][ITW], int g) {
    const int ch = g / NTP, tp = g - ch * NTP;
    const int buf = ch & 1;
    ldw(nxt, g + 1);
    if (tp >= LAG && tp < NF + LAG) put_item(buf ^ 1, tp - LAG, ring[LAG - 1]);
#pragma unroll
    for (int r = LAG - 1; r > 0; --r) ring[r] = ring[r - 1];
    if (tp < NF) ring[0] = load_item(ch + 1, tp);
    const int t = 2 * tp + h;
#pragma unroll
    for (int tt = 0; tt < PT; ++tt) {
      const int o = tap_off(tt, t);
      const bf16x8 b0 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 0) * PLANE + o]);
      const bf16x8 b1 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 1) * PLANE + o]);
      const bf16x8 b2 = __builtin_bit_cast(bf16x8, patch[(buf * 3 + 2) * PLANE + o]);
#pragma unroll
      for (int it = 0; it < ITW; ++it) {
        acc[tt][it] = mfma(cur[2][it], b0, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b2, acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b1, acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b0, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b1, acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b0, acc[tt][it]);
      }
    }
    if (tp == NTP - 1) __syncthreads();
  };
  bf16x8 fa[3][ITW], fb[3][ITW];
  ldw(fa, 0);
  int g = 0;
#pragma unroll 1
  for (; g + 1 < total; g += 2) {
    step(fa, fb, g);
    step(fb, fa, g + 1);
  }
  if (g < total) step(fa, fb, g);
  const int C4o = (Cout + 3) >> 2;
#pragma unroll
  for (int tt = 0; tt < PT; ++tt) {
    const int oy = oy0 + wr * PT + tt, ox = ox0 + j;
#pragma unroll
    for (int it = 0; it < ITW; ++it)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int c0 = cb * IT * 32 + (wc * ITW + it) * 32 + 8 * gq + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[tt][it][4 * gq + e] + bias[c0 + e];
        *reinterpret_cast<f32x4*>(y + ((((size_t)n * C4o + (c0 >> 2)) * Hout + oy) * Wout + ox) * 4) = v;
      }
  }
}

// v4: v2 (4 waves, PT tiles x 4 channel tiles per wave, double-buffered 8-channel tap-pair patch) with an explicit
// software pipeline: weights issued WD steps ahead (ring of WD + 1 sets), the B operands read from LDS one step
// ahead, the fill's split + LDS stores in the MFMA region.
template <int PT, int LAG, int WD>
__global__ __launch_bounds__(256, 1) void down_v4(const float* __restrict__ x, float* __restrict__ y,
                                                  const bf16x8* __restrict__ wp, const float* __restrict__ bias,
                                                  int N, int Cin, int Hin, int Win, int Cout, int Hout, int Wout) {
  constexpr int TH = 4 * PT, PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;
  constexpr int NQ = 2;
  constexpr int NF = (NQ * PLANE + 255) / 256;
  constexpr int NR = WD + 1;   // weight ring sets
  static_assert(NF + LAG <= NTP, "fill must fit in one chunk");
  __shared__ u32x4 patch[2 * 3 * PLANE];
  const int tiles_x = Wout / TW, tiles_y = Hout / TH;
  int bid = blockIdx.x;
  const int cb = blockIdx.y;
  const int tx = bid % tiles_x;
  bid /= tiles_x;
  const int ty = bid % tiles_y;
  const int n = bid / tiles_y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, j = lane & 31;
  const int oy0 = ty * TH, ox0 = tx * TW;
  const int iy0 = oy0 * S - 2, ix0 = ox0 * S - 2;
  const int Cin4 = Cin >> 2, nch = Cin / 8;
  f32x16 acc[PT][IT];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
  const unsigned xplane = (unsigned)Hin * Win;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x) + (size_t)n * Cin4 * xplane * 4, 0, (int)(Cin4 * xplane * 16), 0x00020000);
  auto load_item = [&](int ch, int i) -> f32x4 {
    const int e = threadIdx.x + 256 * i;
    const int q = e / PLANE, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
    const int iy = iy0 + pr, ix = ix0 + pc;
    const bool ok = e < NQ * PLANE && ch < nch && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
    const unsigned vo = ((unsigned)(ch * NQ + q) * xplane + (unsigned)iy * Win + ix) * 16u;
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
  };
  auto put_item = [&](int buf, int i, f32x4 v) {
    const int e = threadIdx.x + 256 * i;
    if (e < NQ * PLANE) {
      const int q = e / PLANE, pix = e - q * PLANE;
      u32x2 hh, mm, ll;
      split3(v, hh, mm, ll);
      u32x2* p2 = reinterpret_cast<u32x2*>(patch);
      p2[((buf * 3 + 0) * PLANE + pix) * 2 + q] = hh;
      p2[((buf * 3 + 1) * PLANE + pix) * 2 + q] = mm;
      p2[((buf * 3 + 2) * PLANE + pix) * 2 + q] = ll;
    }
  };
  {
    f32x4 v[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) v[i] = load_item(0, i);
#pragma unroll
    for (int i = 0; i < NF; ++i) put_item(0, i, v[i]);
    __syncthreads();
  }
  const int total = nch * NTP;
  const bf16x8* wb = wp + (size_t)cb * nch * NTP * 3 * IT * 64 + lane;
  auto ldw = [&](bf16x8 (&a)[3][IT], int g) {
    const bf16x8* w = wb + (size_t)min(g, total - 1) * 3 * IT * 64;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int it = 0; it < IT; ++it) a[p][it] = w[(p * IT + it) * 64];
  };
  auto tap_off = [&](int tt, int t) {
    t = min(t, KK - 1);
    const int ky = t / KS, kx = t - ky * KS;
    return (S * (wave * PT + tt) + ky) * PC + S * j + kx;
  };
  auto ldb = [&](bf16x8 (&b)[PT][3], int g) {
    const int gg = min(g, total - 1);
    const int ch = gg / NTP, tp = gg - ch * NTP;
    const int buf = ch & 1;
#pragma unroll
    for (int tt = 0; tt < PT; ++tt) {
      const int o = tap_off(tt, 2 * tp + h);
#pragma unroll
      for (int p = 0; p < 3; ++p) b[tt][p] = __builtin_bit_cast(bf16x8, patch[(buf * 3 + p) * PLANE + o]);
    }
  };
  f32x4 ring[LAG + 1];   // after the shift at step tp, ring[k] = fill item tp - k
  bf16x8 W[NR][3][IT];
  bf16x8 Bc[PT][3], Bn[PT][3];
  auto step = [&](bf16x8 (&cur)[3][IT], bf16x8 (&far)[3][IT], bf16x8 (&b)[PT][3], bf16x8 (&bn)[PT][3], int g) {
    const int ch = g / NTP, tp = g - ch * NTP;
    const int buf = ch & 1;
    __builtin_amdgcn_sched_barrier(0);
    ldw(far, g + WD);
#pragma unroll
    for (int r = LAG; r > 0; --r) ring[r] = ring[r - 1];
    if (tp < NF) ring[0] = load_item(ch + 1, tp);
    // next step's B operands (the last step of a chunk: the next chunk's buffer is not complete until the barrier)
    if (tp != NTP - 1) ldb(bn, g + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int tt = 0; tt < PT; ++tt)
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        acc[tt][it] = mfma(cur[2][it], b[tt][0], acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b[tt][2], acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b[tt][1], acc[tt][it]);
        acc[tt][it] = mfma(cur[1][it], b[tt][0], acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b[tt][1], acc[tt][it]);
        acc[tt][it] = mfma(cur[0][it], b[tt][0], acc[tt][it]);
      }
    if (tp >= LAG && tp < NF + LAG) put_item(buf ^ 1, tp - LAG, ring[LAG]);
    if (tp == NTP - 1) {
      __syncthreads();
      ldb(bn, g + 1);
    }
  };
#pragma unroll
  for (int r = 0; r < WD; ++r) ldw(W[r], r);
  ldb(Bc, 0);
  int g = 0;
  static_assert(NR == 3, "ring of 3");
#pragma unroll 1
  for (; g + 5 < total; g += 6) {
    step(W[0], W[2], Bc, Bn, g);
    step(W[1], W[0], Bn, Bc, g + 1);
    step(W[2], W[1], Bc, Bn, g + 2);
    step(W[0], W[2], Bn, Bc, g + 3);
    step(W[1], W[0], Bc, Bn, g + 4);
    step(W[2], W[1], Bn, Bc, g + 5);
  }
  for (; g < total; ++g) {   // tail (< 6 steps): same ring order
    const int k = g % 6;
    if (k == 0) step(W[0], W[2], Bc, Bn, g);
    else if (k == 1) step(W[1], W[0], Bn, Bc, g);
    else if (k == 2) step(W[2], W[1], Bc, Bn, g);
    else if (k == 3) step(W[0], W[2], Bn, Bc, g);
    else step(W[1], W[0], Bc, Bn, g);
  }
  const int C4o = (Cout + 3) >> 2;
#pragma unroll
  for (int tt = 0; tt < PT; ++tt) {
    const int oy = oy0 + wave * PT + tt, ox = ox0 + j;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int c0 = cb * IT * 32 + it * 32 + 8 * gq + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[tt][it][4 * gq + e] + bias[c0 + e];
        *reinterpret_cast<f32x4*>(y + ((((size_t)n * C4o + (c0 >> 2)) * Hout + oy) * Wout + ox) * 4) = v;
      }
  }
}

static uint16_t bf_rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

struct Ctx {
  int N, Cin, Cout, Hin, Win, Hout, Wout;
  float *dx, *dy, *db;
  bf16x8* dw;
  std::vector<float> hx, hw, hb;
};

template <int V, int PT, int LAG>
void run(Ctx& c, const char* name) {
  constexpr int TH = 4 * PT;
  dim3 grid((c.Wout / TW) * (c.Hout / TH) * c.N, c.Cout / (IT * 32));
  auto launch = [&]() {
    if constexpr (V == 2)
      hipLaunchKernelGGL((down_v2<PT, LAG>), grid, dim3(256), 0, 0, c.dx, c.dy, c.dw, c.db, c.N, c.Cin, c.Hin, c.Win,
                         c.Cout, c.Hout, c.Wout);
    else if constexpr (V == 3)
      hipLaunchKernelGGL((down_v3<PT, LAG>), grid, dim3(512), 0, 0, c.dx, c.dy, c.dw, c.db, c.N, c.Cin, c.Hin, c.Win,
                         c.Cout, c.Hout, c.Wout);
    else
      hipLaunchKernelGGL((down_v4<PT, LAG, 2>), grid, dim3(256), 0, 0, c.dx, c.dy, c.dw, c.db, c.N, c.Cin, c.Hin,
                         c.Win, c.Cout, c.Hout, c.Wout);
  };
  CHECK(hipMemset(c.dy, 0, (size_t)c.N * (c.Cout / 4) * c.Hout * c.Wout * 16));
  launch();
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 10;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const double flops = 2.0 * c.Cout * c.Cin * KK * (double)c.Hout * c.Wout * c.N;
  printf("%-28s %.3f ms  %6.1f TFLOP/s (fp32-equivalent algorithmic)\n", name, ms, flops / (ms * 1e-3) / 1e12);
  const size_t yn = (size_t)c.N * (c.Cout / 4) * c.Hout * c.Wout * 4;
  std::vector<float> hy(yn);
  CHECK(hipMemcpy(hy.data(), c.dy, yn * 4, hipMemcpyDeviceToHost));
  double max_err = 0, max_err32 = 0, max_ref = 0;
  std::mt19937 r2(7);
  const int Cin4 = c.Cin / 4;
  for (int s = 0; s < 2000; ++s) {
    const int nn = r2() % c.N, co = r2() % c.Cout, oy = r2() % c.Hout, ox = r2() % c.Wout;
    double ref = c.hb[co];
    float f32 = c.hb[co];
    for (int ci = 0; ci < c.Cin; ++ci)
      for (int t = 0; t < KK; ++t) {
        const int iy = oy * 2 - 2 + t / 5, ix = ox * 2 - 2 + t % 5;
        if (iy < 0 || iy >= c.Hin || ix < 0 || ix >= c.Win) continue;
        const float xv = c.hx[((((size_t)nn * Cin4 + ci / 4) * c.Hin + iy) * c.Win + ix) * 4 + (ci & 3)];
        const float wv = c.hw[((size_t)co * c.Cin + ci) * KK + t];
        ref += (double)xv * wv;
        f32 = fmaf(xv, wv, f32);
      }
    const float got = hy[((((size_t)nn * (c.Cout / 4) + co / 4) * c.Hout + oy) * c.Wout + ox) * 4 + (co & 3)];
    max_err = fmax(max_err, fabs(got - ref));
    max_err32 = fmax(max_err32, fabs(f32 - ref));
    max_ref = fmax(max_ref, fabs(ref));
  }
  printf("  vs float64: max abs err %.3e, sequential-fp32 max abs err %.3e (max |ref| %.3f)\n", max_err, max_err32,
         max_ref);
}

int main(int argc, char** argv) {
  Ctx c;
  c.N = argc > 1 ? atoi(argv[1]) : 32;
  c.Cin = 128, c.Cout = 128, c.Hin = 256, c.Win = 384;
  c.Hout = c.Hin / 2, c.Wout = c.Win / 2;
  const int Cin4 = c.Cin / 4, nch = c.Cin / 8;
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  const size_t xn = (size_t)c.N * Cin4 * c.Hin * c.Win * 4;
  c.hx.resize(xn);
  c.hw.resize((size_t)c.Cout * c.Cin * KK);
  c.hb.resize(c.Cout);
  for (auto& v : c.hx) v = U(rng);
  const float wsc = 1.f / sqrtf((float)c.Cin * KK);
  for (auto& v : c.hw) v = U(rng) * wsc;
  for (auto& v : c.hb) v = U(rng) * 0.1f;
  const int ncb = c.Cout / (IT * 32);
  // pack [cb][chunk8][tap pair][plane][it][lane][8]: lane half h = tap 2tp + h, element jj = channel 8*chunk + jj
  std::vector<uint16_t> hp((size_t)ncb * nch * NTP * 3 * IT * 64 * 8, 0);
  for (int cb = 0; cb < ncb; ++cb)
    for (int ch = 0; ch < nch; ++ch)
      for (int tp = 0; tp < NTP; ++tp)
        for (int it = 0; it < IT; ++it)
          for (int l = 0; l < 64; ++l)
            for (int jj = 0; jj < 8; ++jj) {
              const int t = 2 * tp + (l >> 5);
              if (t >= KK) continue;
              const int co = cb * IT * 32 + it * 32 + (l & 31), ci = ch * 8 + jj;
              const float w = c.hw[((size_t)co * c.Cin + ci) * KK + t];
              const uint16_t a = bf_rne(w);
              const float r1 = w - bf2f(a);
              const uint16_t b = bf_rne(r1);
              const float r2 = r1 - bf2f(b);
              const uint16_t cc = bf_rne(r2);
              const uint16_t pl[3] = {a, b, cc};
              for (int p = 0; p < 3; ++p)
                hp[(((((((size_t)cb * nch + ch) * NTP + tp) * 3 + p) * IT + it) * 64 + l) * 8) + jj] = pl[p];
            }
  const size_t yn = (size_t)c.N * (c.Cout / 4) * c.Hout * c.Wout * 4;
  CHECK(hipMalloc(&c.dx, xn * 4));
  CHECK(hipMalloc(&c.dy, yn * 4));
  CHECK(hipMalloc(&c.db, c.Cout * 4));
  CHECK(hipMalloc(&c.dw, hp.size() * 2));
  CHECK(hipMemcpy(c.dx, c.hx.data(), xn * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(c.db, c.hb.data(), c.Cout * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(c.dw, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
  run<2, 2, 2>(c, "v2 PT2 lag2");
  run<4, 2, 2>(c, "v4 PT2 lag2 wd2");
  run<4, 2, 3>(c, "v4 PT2 lag3 wd2");
  return 0;
}

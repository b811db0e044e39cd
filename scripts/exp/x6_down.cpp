// Experiment: fp32-accurate conv_down (k5 s2) main loop on bf16 MFMA with exact 3-way bf16 operand splits
// (6 products per k-step: hh, hm, mh, hl, lh, mm).  Standalone: times launch variants on one shape and checks
// a sample of outputs against a float64 CPU conv, next to the same sample computed in plain fp32.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/exp/x6_down.cpp -o scripts/exp/x6_down && ./x6_down
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

// exact split v = hi + mid + lo (round-to-nearest-even at each stage)
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

constexpr int KS = 5, S = 2, TW = 32, IT = 4, KK = KS * KS;

// PT: 32-pixel tiles per wave (block = 4 waves x PT x 32 px, TH = 4 * PT rows of TW = 32)
// PREF: 1 = next chunk's global loads held in registers through the current chunk; 0 = one batch at the fill
// NB: blocks per CU (launch bound)
// EO: patch columns stored even/odd-split (the stride-2 tap reads of consecutive output columns hit consecutive
// entries: conflict-free ds_read_b128); PREF = tap of a chunk at which the next chunk's global loads issue (-1: one
// batch at the fill)
template <int MODE, int PT, int PREF, int NB, int EO = 0, int ABL = 0>
__global__ __launch_bounds__(256, NB) void down_x6(const float* __restrict__ x, float* __restrict__ y,
                                                   const bf16x8* __restrict__ wp, const float* __restrict__ bias,
                                                   int N, int Cin, int Hin, int Win, int Cout, int Hout, int Wout) {
  constexpr int TH = 4 * PT, PR = S * (TH - 1) + KS, PC = S * (TW - 1) + KS, PLANE = PR * PC;
  constexpr int PCE = (PC + 1) / 2;   // even columns first, then odd (EO layout)
  auto col = [&](int pc) { return EO ? ((pc & 1) * PCE + (pc >> 1)) : pc; };
  __shared__ u32x4 patch[3 * 2 * PLANE];
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
  const int Cin4 = Cin >> 2, nch = Cin / 16;
  f32x16 acc[PT][IT];
#pragma unroll
  for (int t = 0; t < PT; ++t)
#pragma unroll
    for (int it = 0; it < IT; ++it) acc[t][it] = f32x16{0};
  const size_t xplane = (size_t)Hin * Win;
  constexpr int NF = (4 * PLANE + 255) / 256;
  f32x4 pf[NF];
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(x) + (size_t)n * Cin4 * xplane * 4, 0, (int)(Cin4 * xplane * 16), 0x00020000);
  auto fetch = [&](int ch) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      const int q = e / PLANE, pix = e - q * PLANE, pr = pix / PC, pc = pix - pr * PC;
      const int iy = iy0 + pr, ix = ix0 + pc;
      const bool ok = e < 4 * PLANE && ch < nch && iy >= 0 && iy < Hin && ix >= 0 && ix < Win;
      const unsigned vo = ((unsigned)(ch * 4 + q) * (unsigned)xplane + (unsigned)iy * Win + ix) * 16u;
      pf[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, ok ? vo : 0xFFFFFFF0u, 0, 0));
    }
  };
  auto put = [&]() {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int e = threadIdx.x + 256 * i;
      if (e < 4 * PLANE) {
        const int q = e / PLANE, pix0 = e - q * PLANE, pr0 = pix0 / PC, pix = pr0 * PC + col(pix0 - pr0 * PC);
        u32x2 hh, mm, ll;
        split3(pf[i], hh, mm, ll);
        u32x2* p2 = reinterpret_cast<u32x2*>(patch);
        const int half = q >> 1, sub = q & 1;
        p2[((0 * 2 + half) * PLANE + pix) * 2 + sub] = hh;
        p2[((1 * 2 + half) * PLANE + pix) * 2 + sub] = mm;
        p2[((2 * 2 + half) * PLANE + pix) * 2 + sub] = ll;
      }
    }
    __syncthreads();
  };
  auto fill = [&](int ch) {
    if constexpr ((ABL & 4) != 0) return;
    if constexpr (PREF >= 0) {
      if (ch == 0) fetch(0);
      put();
    } else {
      fetch(ch);
      put();
    }
  };
  const int total = nch * KK;
  const bf16x8* wb = wp + (size_t)cb * nch * KK * 3 * IT * 64 + lane;
  auto ldw = [&](bf16x8 (&a)[3][IT], int g) {
    const bf16x8* w = wb + (size_t)min(g, total - 1) * 3 * IT * 64;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        if constexpr ((ABL & 1) != 0) {
          a[p][it] = __builtin_bit_cast(bf16x8, (u32x4){0x3c003c00u + (unsigned)((g + it + p) & 7), 0x3c003c00u,
                                                         0x3c003c00u, 0x3c003c00u + (unsigned)(threadIdx.x & 3)});
        } else {
          a[p][it] = w[(p * IT + it) * 64];
        }
      }
  };
  auto step = [&](bf16x8 (&cur)[3][IT], bf16x8 (&nxt)[3][IT], int g) {
    const int ch = g / KK, tap = g - ch * KK;
    if (tap == 0) fill(ch);
    if constexpr (PREF >= 0) {
      if (tap == PREF) fetch(ch + 1);
    }
    __builtin_amdgcn_sched_barrier(0);
    ldw(nxt, g + 1);
    __builtin_amdgcn_sched_barrier(0);   // the next step's fragments issue before this step's MFMAs
    const int ky = tap / KS, kx = tap - ky * KS;
#pragma unroll
    for (int t = 0; t < PT; ++t) {
      const int o = (S * (wave * PT + t) + ky) * PC + (EO ? ((kx & 1) * PCE + j + (kx >> 1)) : S * j + kx);
      bf16x8 b0, b1, b2;
      if constexpr ((ABL & 2) != 0) {
        b0 = cur[0][t & 3]; b1 = cur[1][(t + 1) & 3]; b2 = cur[2][(t + 2) & 3];
        (void)o;
      } else {
        b0 = __builtin_bit_cast(bf16x8, patch[(0 * 2 + h) * PLANE + o]);
        b1 = __builtin_bit_cast(bf16x8, patch[(1 * 2 + h) * PLANE + o]);
        b2 = __builtin_bit_cast(bf16x8, patch[(2 * 2 + h) * PLANE + o]);
      }
#pragma unroll
      for (int it = 0; it < IT; ++it) {
        if constexpr (MODE == 6) {
          acc[t][it] = mfma(cur[2][it], b0, acc[t][it]);
          acc[t][it] = mfma(cur[0][it], b2, acc[t][it]);
          acc[t][it] = mfma(cur[1][it], b1, acc[t][it]);
          acc[t][it] = mfma(cur[1][it], b0, acc[t][it]);
          acc[t][it] = mfma(cur[0][it], b1, acc[t][it]);
          acc[t][it] = mfma(cur[0][it], b0, acc[t][it]);
        } else {
          acc[t][it] = mfma(cur[0][it], b0, acc[t][it]);
        }
      }
    }
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
  for (int t = 0; t < PT; ++t) {
    const int oy = oy0 + wave * PT + t, ox = ox0 + j;
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int c0 = cb * IT * 32 + it * 32 + 8 * gq + 4 * h;
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[t][it][4 * gq + e] + bias[c0 + e];
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

template <int MODE, int PT, int PREF, int NB, int EO = 0, int ABL = 0>
void run(Ctx& c, const char* name, bool check) {
  constexpr int TH = 4 * PT;
  dim3 grid((c.Wout / TW) * (c.Hout / TH) * c.N, c.Cout / (IT * 32));
  auto launch = [&]() {
    hipLaunchKernelGGL((down_x6<MODE, PT, PREF, NB, EO, ABL>), grid, dim3(256), 0, 0, c.dx, c.dy, c.dw, c.db, c.N, c.Cin,
                       c.Hin, c.Win, c.Cout, c.Hout, c.Wout);
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
  if (!check) return;
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
  const int Cin4 = c.Cin / 4, nch = c.Cin / 16;
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
  std::vector<uint16_t> hp((size_t)ncb * nch * KK * 3 * IT * 64 * 8);
  for (int cb = 0; cb < ncb; ++cb)
    for (int ch = 0; ch < nch; ++ch)
      for (int t = 0; t < KK; ++t)
        for (int it = 0; it < IT; ++it)
          for (int l = 0; l < 64; ++l)
            for (int jj = 0; jj < 8; ++jj) {
              const int co = cb * IT * 32 + it * 32 + (l & 31), ci = ch * 16 + 8 * (l >> 5) + jj;
              const float w = c.hw[((size_t)co * c.Cin + ci) * KK + t];
              const uint16_t a = bf_rne(w);
              const float r1 = w - bf2f(a);
              const uint16_t b = bf_rne(r1);
              const float r2 = r1 - bf2f(b);
              const uint16_t cc = bf_rne(r2);
              const uint16_t pl[3] = {a, b, cc};
              for (int p = 0; p < 3; ++p)
                hp[(((((((size_t)cb * nch + ch) * KK + t) * 3 + p) * IT + it) * 64 + l) * 8) + jj] = pl[p];
            }
  const size_t yn = (size_t)c.N * (c.Cout / 4) * c.Hout * c.Wout * 4;
  CHECK(hipMalloc(&c.dx, xn * 4));
  CHECK(hipMalloc(&c.dy, yn * 4));
  CHECK(hipMalloc(&c.db, c.Cout * 4));
  CHECK(hipMalloc(&c.dw, hp.size() * 2));
  CHECK(hipMemcpy(c.dx, c.hx.data(), xn * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(c.db, c.hb.data(), c.Cout * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(c.dw, hp.data(), hp.size() * 2, hipMemcpyHostToDevice));
  run<6, 2, -1, 1, 0>(c, "x6 PT2 batch nb1", true);
  run<6, 2, -1, 1, 0, 1>(c, "  abl: no weight loads", false);
  run<6, 2, -1, 1, 0, 2>(c, "  abl: no LDS B reads", false);
  run<6, 2, -1, 1, 0, 4>(c, "  abl: no fill", false);
  run<6, 2, -1, 1, 0, 7>(c, "  abl: MFMA only", false);
  run<6, 1, -1, 2, 0, 7>(c, "  abl PT1 nb2: MFMA only", false);
  return 0;
}

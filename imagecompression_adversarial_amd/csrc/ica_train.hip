// Training-side kernels for the adversarial fine-tune (train.py:335-366, adv_train.py:166-192):
// weight gradients of the conv/deconv layers, GDN / EntropyBottleneck / GaussianConditional
// parameter gradients, and the small elementwise backward pieces (ReLU, |.|, bounds, losses).
// All reductions are deterministic (fixed-order split reduction, no float atomics).
//
// Weight gradient (one kernel for conv k5s2 / k3s1 / k1 and deconv k5s2):
//   out[a][b][tap] = sum_{n, p in small grid} Sm[n][a][p] * Lg[n][b][S*p + tap - P]
//     conv   (W[o][c]):  Sm = dL/dy (a = o), Lg = x      (b = c)
//     deconv (W[c][o]):  Sm = x      (a = c), Lg = dL/dy (b = o)
//   MFMA 32x32x2 with the pixel as the reduction index; block = (a-tile, b-tile, pixel split),
//   wave w owns taps w, w+4, ...; operands staged in LDS per 32-pixel row segment.
#include "ica_common.h"

constexpr int WG_PX = 32;  // small-grid pixels per chunk (one row segment)

template <int KS, int S>
__global__ __launch_bounds__(256) void wgrad_kernel(const float* __restrict__ Sm, const float* __restrict__ Lg,
                                                    float* __restrict__ ws, int N, int A, int Bc, int Hs, int Ws_,
                                                    int Hb, int Wb, int P, int nsplit) {
  constexpr int KK = KS * KS;
  constexpr int PC = S * (WG_PX - 1) + KS;
  constexpr int NT = (KK + 3) / 4;  // taps per wave (max)
  __shared__ float s_sm[32][WG_PX + 1];       // [a][px]
  __shared__ float s_lg[KS][PC][33];          // [row][col][b]
  const int a0 = blockIdx.x * 32, b0 = blockIdx.y * 32, split = blockIdx.z;
  const int lane = threadIdx.x & 63, h = lane >> 5, l31 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int A4 = (A + 3) >> 2, B4 = (Bc + 3) >> 2;
  const int segs_per_row = (Ws_ + WG_PX - 1) / WG_PX;
  const long nchunks = (long)N * Hs * segs_per_row;
  const long c_begin = nchunks * split / nsplit, c_end = nchunks * (split + 1) / nsplit;
  f32x16 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x16{0};
  for (long c = c_begin; c < c_end; ++c) {
    const int seg = c % segs_per_row;
    const long rc = c / segs_per_row;
    const int ys = rc % Hs, n = rc / Hs;
    const int xs0 = seg * WG_PX;
    __syncthreads();
    // small tile: 32 channels x 32 px
    for (int e = threadIdx.x; e < 32 * WG_PX; e += 256) {
      const int a = e / WG_PX, px = e % WG_PX;
      const int ch = a0 + a, xs = xs0 + px;
      float v = 0.f;
      if (ch < A && xs < Ws_) v = Sm[((((size_t)n * A4 + (ch >> 2)) * Hs + ys) * Ws_ + xs) * 4 + (ch & 3)];
      s_sm[a][px] = v;
    }
    // big patch: KS rows x PC cols x 32 channels
    const int yb0 = S * ys - P, xb0 = S * xs0 - P;
    for (int e = threadIdx.x; e < KS * PC * 32; e += 256) {
      const int b = e % 32, rest = e / 32, col = rest % PC, row = rest / PC;
      const int ch = b0 + b, yb = yb0 + row, xb = xb0 + col;
      float v = 0.f;
      if (ch < Bc && yb >= 0 && yb < Hb && xb >= 0 && xb < Wb)
        v = Lg[((((size_t)n * B4 + (ch >> 2)) * Hb + yb) * Wb + xb) * 4 + (ch & 3)];
      s_lg[row][col][b] = v;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int tap = wave + 4 * t;
      if (tap < KK) {
        const int ky = tap / KS, kx = tap % KS;
#pragma unroll 4
        for (int s2 = 0; s2 < WG_PX / 2; ++s2) {
          const int px = 2 * s2 + h;
          const float av = s_sm[l31][px];
          const float bv = s_lg[ky][S * px + kx][l31];
          acc[t] = mfma32(av, bv, acc[t]);
        }
      }
    }
  }
  // D[i = a][j = b]: lane l reg r -> a = acc_row(r, h), b = l31
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tap = wave + 4 * t;
    if (tap >= KK) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int a = a0 + acc_row(r, h), b = b0 + l31;
      if (a < A && b < Bc) ws[(((size_t)split * A + a) * Bc + b) * KK + tap] = acc[t][r];
    }
  }
}

__global__ void split_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, long n, int nsplit,
                                    int accumulate) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < nsplit; ++k) s += ws[(size_t)k * n + i];
    out[i] = accumulate ? out[i] + s : s;
  }
}

// per-channel sum over (n, pixels) of an nChw4c tensor (bias grads, GDN beta grads);
// one block per channel, fixed-order tree.
__global__ void channel_sum_kernel(const float* __restrict__ x, float* __restrict__ out, int N, int C, long HW,
                                   int accumulate) {
  __shared__ float sh[4];
  const int c = blockIdx.x;
  const int C4 = (C + 3) >> 2;
  float acc = 0.f;
  for (long k = threadIdx.x; k < (long)N * HW; k += 256) {
    const long n = k / HW, p = k % HW;
    acc += x[(((size_t)n * C4 + (c >> 2)) * HW + p) * 4 + (c & 3)];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float r = (sh[0] + sh[1]) + (sh[2] + sh[3]);
    out[c] = accumulate ? out[c] + r : r;
  }
}

// elementwise helpers -------------------------------------------------------
__global__ void relu_bwd_kernel(float* __restrict__ g, const float* __restrict__ y, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    if (!(y[i] > 0.f)) g[i] = 0.f;
}

__global__ void abs_bwd_kernel(float* __restrict__ g, const float* __restrict__ x, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = x[i];
    g[i] = v > 0.f ? g[i] : (v < 0.f ? -g[i] : 0.f);
  }
}

// leaky-ReLU backward into a separate tensor (the pre-activation gradient a weight gradient reads): a is the layer's
// saved output (same sign as its input), slope 0.01 -- the same select as the conv fills / EPI_LRELU_BWD
__global__ void lrelu_bwd_kernel(const float* __restrict__ g, const float* __restrict__ a, float* __restrict__ out,
                                 long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float v = g[i];
    out[i] = a[i] > 0.f ? v : v * 0.01f;
  }
}

// t = dL/dn of a GDN / IGDN layer from g = dL/dy and its saved (y, s), y = x s:  GDN (s = n^-1/2) t = -0.5 g y s^2,
// IGDN (s = n^1/2) t = 0.5 g y / s^2 -- the arithmetic of the fused GDN-backward epilogues (ica_conv_epi.h), for the
// layers whose backward launch cannot write t (the k3 residual layers of cheng2020)
__global__ void gdn_t_kernel(const float* __restrict__ g, const float* __restrict__ y, const float* __restrict__ s,
                             float* __restrict__ t, long n, int inverse) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float sv = s[i], gy = g[i] * y[i];
    t[i] = inverse ? (sv != 0.f ? 0.5f * gy / (sv * sv) : 0.f) : -0.5f * gy * (sv * sv);
  }
}

// x^2 with x = y / s (GDN input recovered from the saved output y and s)
__global__ void gdn_xsq_kernel(const float* __restrict__ y, const float* __restrict__ s, float* __restrict__ out,
                               long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = y[i] / s[i];
    out[i] = x * x;
  }
}

// Reparam chain: p' = max(p, bound)^2 - ped  ->  dp = dp' * 2 * max(p, bound) gated by LowerBound's
// pass-through rule (x >= bound | g < 0).
__global__ void reparam_bwd_kernel(const float* __restrict__ p, const float* __restrict__ gprime,
                                   float* __restrict__ gout, long n, float bound, int accumulate) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = p[i];
    const float lb = fmaxf(x, bound);
    float g = gprime[i] * 2.0f * lb;  // d(lb^2)/dlb
    g = (x >= bound || g < 0.f) ? g : 0.f;
    gout[i] = accumulate ? gout[i] + g : g;
  }
}

// d bpp-term / d lik for RateDistortionLoss (train.py:60-64): L += sum log(clamp(lik, 1/65536)) / (-ln2 * npx)
// -> dL/dlik = scale / lik where lik >= 1/65536 else 0 (torch.clamp backward), then the
// likelihood LowerBound(1e-9) pass-through: rows where lik_raw < 1e-9 keep g only if g < 0.
// (lik here is the bounded likelihood the forward returned.)
__global__ void bpp_grad_kernel(const float* __restrict__ lik, float* __restrict__ g, long n, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float l = lik[i];
    g[i] = l >= (1.0f / 65536.0f) ? scale / l : 0.f;
  }
}

// GaussianConditional backward (train mode, means = None): lik = max(Phi((.5-|v|)/s) - Phi((-.5-|v|)/s), 1e-9)
// with s = max(sigma, 0.11) (LowerBound pass-through), v = y_tilde.  In: dL/dlik (gl).  Out: dL/dy, dL/dsigma.
__global__ void gc_bwd_kernel(const float* __restrict__ yt, const float* __restrict__ sigma,
                              const float* __restrict__ gl, float* __restrict__ gy, float* __restrict__ gs, int C,
                              long per_image, int B) {
  const long total = per_image * B;
  const int C4 = (C + 3) >> 2;
  const long HW = per_image / (4L * C4);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long k = i % per_image;
    const int c = (int)((k >> 2) / HW) * 4 + (int)(k & 3);
    if (c >= C) {
      gy[i] = 0.f;
      gs[i] = 0.f;
      continue;
    }
    const float v = yt[i], sr = sigma[i];
    const float s = fmaxf(sr, 0.11f);
    const float av = fabsf(v);
    const float k2 = -0.70710678118654752f;
    const float zu = (0.5f - av) / s, zl = (-0.5f - av) / s;
    const float up = 0.5f * erfcf(k2 * zu), lo = 0.5f * erfcf(k2 * zl);
    float g = gl[i];
    const float lraw = up - lo;
    g = (lraw >= 1e-9f || g < 0.f) ? g : 0.f;  // likelihood LowerBound
    const float inv_sqrt2pi = 0.3989422804014327f;
    const float pu = inv_sqrt2pi * expf(-0.5f * zu * zu), pl = inv_sqrt2pi * expf(-0.5f * zl * zl);
    // d lraw / d av = (-pu + pl) / s ; d lraw / d s = (-pu * zu + pl * zl) / s
    const float dav = g * (pl - pu) / s;
    float dsv = g * (pl * zl - pu * zu) / s;
    gy[i] = v > 0.f ? dav : (v < 0.f ? -dav : 0.f);
    dsv = (sr >= 0.11f || dsv < 0.f) ? dsv : 0.f;  // scale LowerBound
    gs[i] = dsv;
  }
}

// EntropyBottleneck backward (train mode): per channel c (one block), over all elements v of that
// channel: lik = |sig(s*F(v+.5)) - sig(s*F(v-.5))|, s = -sign(F(v-.5)+F(v+.5)) (detached),
// LowerBound(1e-9).  Writes dL/dv per element and accumulates dL/d{matrix,bias,factor} (58 per channel,
// raw-parameter space: softplus / tanh chain applied) into gparam[c][58] in fixed order.
struct EbLayerGrad {
  float m[9], b[3], f[3];
};

__device__ __forceinline__ float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

// forward of one logistic MLP branch keeping activations for backward
__device__ __forceinline__ float eb_fwd_keep(const float* q, float u, float (&pre)[4][3], float (&th)[4][3],
                                            float (&act)[5][3]) {
  // layer 0: 1 -> 3
  act[0][0] = u;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float t = q[k] * u + q[3 + k];
    pre[0][k] = t;
    th[0][k] = tanhf(t);
    act[1][k] = t + q[6 + k] * th[0][k];
  }
  const float* s = q + 9;
#pragma unroll
  for (int layer = 1; layer < 4; ++layer) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float t = s[3 * k] * act[layer][0] + s[3 * k + 1] * act[layer][1] + s[3 * k + 2] * act[layer][2] + s[9 + k];
      pre[layer][k] = t;
      th[layer][k] = tanhf(t);
      act[layer + 1][k] = t + s[12 + k] * th[layer][k];
    }
    s += 15;
  }
  return s[0] * act[4][0] + s[1] * act[4][1] + s[2] * act[4][2] + s[3];
}

// backward of one branch: gout = dL/dF; accumulates param grads (in effective-param space) into G
// (58 layout like q) and returns dL/du
__device__ __forceinline__ float eb_bwd(const float* q, float gout, const float (&pre)[4][3], const float (&th)[4][3],
                                        const float (&act)[5][3], float (&G)[58]) {
  const float* s4 = q + 54;
  float ga[3];
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    G[54 + l] += gout * act[4][l];
    ga[l] = gout * s4[l];
  }
  G[57] += gout;
#pragma unroll
  for (int layer = 3; layer >= 1; --layer) {
    const float* s = q + 9 + 15 * (layer - 1);
    float* Gs = G + 9 + 15 * (layer - 1);
    float gt[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      // act = t + f*tanh(t): dact/dt = 1 + f*(1 - tanh^2); dact/df = tanh(t)
      Gs[12 + k] += ga[k] * th[layer][k];
      gt[k] = ga[k] * (1.0f + s[12 + k] * (1.0f - th[layer][k] * th[layer][k]));
      Gs[9 + k] += gt[k];
    }
    float gprev[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int l = 0; l < 3; ++l) {
        Gs[3 * k + l] += gt[k] * act[layer][l];
        gprev[l] += gt[k] * s[3 * k + l];
      }
#pragma unroll
    for (int l = 0; l < 3; ++l) ga[l] = gprev[l];
  }
  float gu = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    G[6 + k] += ga[k] * th[0][k];
    const float gt = ga[k] * (1.0f + q[6 + k] * (1.0f - th[0][k] * th[0][k]));
    G[3 + k] += gt;
    G[k] += gt * act[0][0];
    gu += gt * q[k];
  }
  return gu;
}

__global__ __launch_bounds__(256) void eb_bwd_kernel(const float* __restrict__ v4, const float* __restrict__ gl4,
                                                     const float* __restrict__ prm, float* __restrict__ gv4,
                                                     float* __restrict__ gprm, int N, int C, long HW) {
  __shared__ float red[4][58];
  const int c = blockIdx.x;
  const int C4 = (C + 3) >> 2;
  const float* q = prm + (size_t)c * 58;
  float G[58];
#pragma unroll
  for (int k = 0; k < 58; ++k) G[k] = 0.f;
  for (long k = threadIdx.x; k < (long)N * HW; k += 256) {
    const long n = k / HW, p = k % HW;
    const size_t i = (((size_t)n * C4 + (c >> 2)) * HW + p) * 4 + (c & 3);
    const float v = v4[i];
    float preL[4][3], thL[4][3], actL[5][3], preU[4][3], thU[4][3], actU[5][3];
    const float lower = eb_fwd_keep(q, v - 0.5f, preL, thL, actL);
    const float upper = eb_fwd_keep(q, v + 0.5f, preU, thU, actU);
    const float sm = lower + upper;
    const float sg = sm > 0.f ? -1.f : (sm < 0.f ? 1.f : 0.f);
    const float su = sigm(sg * upper), sl = sigm(sg * lower);
    const float diff = su - sl;
    const float lraw = fabsf(diff);
    float g = gl4[i];
    g = (lraw >= 1e-9f || g < 0.f) ? g : 0.f;
    const float gd = diff > 0.f ? g : (diff < 0.f ? -g : 0.f);
    const float gU = gd * sg * su * (1.f - su);
    const float gL = -gd * sg * sl * (1.f - sl);
    const float gu = eb_bwd(q, gU, preU, thU, actU, G) + eb_bwd(q, gL, preL, thL, actL, G);
    gv4[i] = gu;
  }
  // block reduce G (fixed order)
#pragma unroll
  for (int k = 0; k < 58; ++k) {
    float t = wave_sum(G[k]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][k] = t;
  }
  __syncthreads();
  if (threadIdx.x < 58) {
    const int k = threadIdx.x;
    gprm[(size_t)c * 58 + k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  }
}

// map effective-parameter grads back to the raw EntropyBottleneck parameters:
// softplus(H) -> dH = g * sigmoid(H) ; tanh(a) -> da = g * (1 - tanh(a)^2) ; biases identity.
struct EbPtrs {
  const float* raw[14];
  float* grad[14];
};

__global__ void eb_param_scatter_kernel(const float* __restrict__ gprm, EbPtrs P, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float* const* raw = P.raw;
  float* const* graw = P.grad;
  const float* G = gprm + (size_t)c * 58;
  // raw order: m0..m4 (0-4), b0..b4 (5-9), f0..f3 (10-13)
  auto sp_grad = [](float g, float h) { return g * (1.0f / (1.0f + expf(-h))); };
  auto th_grad = [](float g, float a) { const float t = tanhf(a); return g * (1.0f - t * t); };
  for (int k = 0; k < 3; ++k) {
    graw[0][c * 3 + k] += sp_grad(G[k], raw[0][c * 3 + k]);
    graw[5][c * 3 + k] += G[3 + k];
    graw[10][c * 3 + k] += th_grad(G[6 + k], raw[10][c * 3 + k]);
  }
  for (int layer = 0; layer < 3; ++layer) {
    const float* Gs = G + 9 + 15 * layer;
    for (int k = 0; k < 9; ++k) graw[1 + layer][c * 9 + k] += sp_grad(Gs[k], raw[1 + layer][c * 9 + k]);
    for (int k = 0; k < 3; ++k) {
      graw[6 + layer][c * 3 + k] += Gs[9 + k];
      graw[11 + layer][c * 3 + k] += th_grad(Gs[12 + k], raw[11 + layer][c * 3 + k]);
    }
  }
  for (int k = 0; k < 3; ++k) graw[4][c * 3 + k] += sp_grad(G[54 + k], raw[4][c * 3 + k]);
  graw[9][c] += G[57];
}

// dL/dx_hat of lambda*255^2*mean((x_hat - x)^2) (+= into g), x_hat nChw4c C=3, x NCHW
__global__ void mse_grad_kernel(const float* __restrict__ xh4, const float* __restrict__ x, float* __restrict__ g4,
                                long HW, float scale) {
  const int b = blockIdx.y;
  for (long pix = (long)blockIdx.x * 256 + threadIdx.x; pix < HW; pix += (long)gridDim.x * 256) {
    const f32x4 v = ld4(xh4 + ((long)b * HW + pix) * 4);
    f32x4 o = ld4(g4 + ((long)b * HW + pix) * 4);
#pragma unroll
    for (int c = 0; c < 3; ++c) o[c] += scale * (v[c] - x[((long)b * 3 + c) * HW + pix]);
    st4(g4 + ((long)b * HW + pix) * 4, o);
  }
}

static inline int g1d(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

extern "C" {

size_t ica_wgrad_ws_size(int A, int Bc, int KS, int nsplit) { return (size_t)nsplit * A * Bc * KS * KS; }

int ica_wgrad_nsplit(int A, int Bc, long nchunks) {
  const int nab = ((A + 31) / 32) * ((Bc + 31) / 32);
  long s = (512 + nab - 1) / nab;
  if (s > nchunks) s = nchunks;
  if (s < 1) s = 1;
  return (int)s;
}

// out[a][b][ky][kx] (+)= sum Sm[n][a][p] * Lg[n][b][S*p + k - P]   (see header comment)
int ica_wgrad(const float* Sm, const float* Lg, float* ws, float* out, int N, int A, int Bc, int Hs, int Ws_, int Hb,
              int Wb, int KS, int S, int P, int nsplit, int accumulate, hipStream_t st) {
  dim3 grid((A + 31) / 32, (Bc + 31) / 32, nsplit);
  if (KS == 5 && S == 2)
    ICA_LAUNCH((wgrad_kernel<5, 2>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else if (KS == 3 && S == 1)
    ICA_LAUNCH((wgrad_kernel<3, 1>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else if (KS == 1 && S == 1)
    ICA_LAUNCH((wgrad_kernel<1, 1>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else if (KS == 3 && S == 2)   // cheng2020: the strided residual-block convs and h_a
    ICA_LAUNCH((wgrad_kernel<3, 2>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else if (KS == 1 && S == 2)   // cheng2020: the 1x1 stride-2 skips
    ICA_LAUNCH((wgrad_kernel<1, 2>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else if (KS == 5 && S == 1)   // the masked 5x5 context model (cheng2020, mbt2018)
    ICA_LAUNCH((wgrad_kernel<5, 1>), grid, dim3(256), 0, st, Sm, Lg, ws, N, A, Bc, Hs, Ws_, Hb, Wb, P, nsplit);
  else
    return -6;
  ICA_CHECK_LAUNCH();
  const long n = (long)A * Bc * KS * KS;
  ICA_LAUNCH(split_reduce_kernel, dim3(g1d(n)), dim3(256), 0, st, ws, out, n, nsplit, accumulate);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_channel_sum(const float* x, float* out, int N, int C, int H, int W, int accumulate, hipStream_t st) {
  ICA_LAUNCH(channel_sum_kernel, dim3(C), dim3(256), 0, st, x, out, N, C, (long)H * W, accumulate);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_relu_bwd(float* g, const float* y, long n, hipStream_t st) {
  ICA_LAUNCH(relu_bwd_kernel, dim3(g1d(n)), dim3(256), 0, st, g, y, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_abs_bwd(float* g, const float* x, long n, hipStream_t st) {
  ICA_LAUNCH(abs_bwd_kernel, dim3(g1d(n)), dim3(256), 0, st, g, x, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_lrelu_bwd(const float* g, const float* a, float* out, long n, hipStream_t st) {
  ICA_LAUNCH(lrelu_bwd_kernel, dim3(g1d(n)), dim3(256), 0, st, g, a, out, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_gdn_t(const float* g, const float* y, const float* s, float* t, long n, int inverse, hipStream_t st) {
  ICA_LAUNCH(gdn_t_kernel, dim3(g1d(n)), dim3(256), 0, st, g, y, s, t, n, inverse);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_gdn_xsq(const float* y, const float* s, float* out, long n, hipStream_t st) {
  ICA_LAUNCH(gdn_xsq_kernel, dim3(g1d(n)), dim3(256), 0, st, y, s, out, n);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_reparam_bwd(const float* p, const float* gprime, float* gout, long n, float bound, int accumulate,
                    hipStream_t st) {
  ICA_LAUNCH(reparam_bwd_kernel, dim3(g1d(n)), dim3(256), 0, st, p, gprime, gout, n, bound, accumulate);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_bpp_grad(const float* lik, float* g, long n, float scale, hipStream_t st) {
  ICA_LAUNCH(bpp_grad_kernel, dim3(g1d(n)), dim3(256), 0, st, lik, g, n, scale);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_gc_bwd(const float* yt, const float* sigma, const float* gl, float* gy, float* gs, int B, int C, int H, int W,
               hipStream_t st) {
  const long per_image = 4L * ((C + 3) / 4) * H * W;
  ICA_LAUNCH(gc_bwd_kernel, dim3(g1d(per_image * B)), dim3(256), 0, st, yt, sigma, gl, gy, gs, C, per_image,
                     B);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_eb_bwd(const float* v4, const float* gl4, const float* prm, float* gv4, float* gprm, int N, int C, int H, int W,
               hipStream_t st) {
  ICA_LAUNCH(eb_bwd_kernel, dim3(C), dim3(256), 0, st, v4, gl4, prm, gv4, gprm, N, C, (long)H * W);
  ICA_CHECK_LAUNCH();
  return 0;
}

// raw / graw: host arrays of 14 device pointers (_matrix0..4, _bias0..4, _factor0..3); graw accumulated.
int ica_eb_param_scatter(const float* gprm, const float* const* raw, float* const* graw, int C, hipStream_t st) {
  EbPtrs P;  // pointer tables passed by value as kernel arguments
  for (int i = 0; i < 14; ++i) {
    P.raw[i] = raw[i];
    P.grad[i] = graw[i];
  }
  ICA_LAUNCH(eb_param_scatter_kernel, dim3((C + 63) / 64), dim3(64), 0, st, gprm, P, C);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_mse_grad(const float* xh4, const float* x, float* g4, int B, int H, int W, float scale, hipStream_t st) {
  ICA_LAUNCH(mse_grad_kernel, dim3(256, B), dim3(256), 0, st, xh4, x, g4, (long)H * W, scale);
  ICA_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

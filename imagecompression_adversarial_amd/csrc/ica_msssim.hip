// MS-SSIM on HIP: LDS-staged separable Gaussian window, the five local
// moments (mu_x, mu_y, E[x^2], E[y^2], E[xy]) in one pass, per-(image,
// channel) partial sums of the SSIM and CS maps, 2x2 average pooling between
// levels, and the weighted product.  Forward AND backward.
//
// Variants:
//   valid (mode 0)  pytorch_msssim.ms_ssim  (attack_rd.py:336,362; self_ensemble.py:225,228)
//                   11-tap sigma 1.5 VALID conv, per-(N,C) means, relu(cs|ssim),
//                   avg_pool2d(2, padding = s % 2)
//   same  (mode 1)  utils/torch_msssim.py:26-71 (adv_train.py:92,170): window min(H,W,11),
//                   zero "same" padding, global mean, no relu, avg_pool2d(2, 2)
//
// Backward: with S = mean(ssim_map) (or CS), dS/dmu_x etc. are per-pixel maps;
// the gradient wrt x is the (transposed) Gaussian filter of those maps:
//   dL/dx = G^T * (dmu1) + 2 x G^T * (ds11) + y G^T * (ds12)   (and sym. for y)
// computed by the same tiled filter kernel applied to the 3 coefficient maps.
#include "ica_common.h"

constexpr int MS_T = 16;      // output tile (MS_T x MS_T per block)
constexpr int MS_MAXW = 11;   // max window taps

struct MsWin {
  float w[MS_MAXW];
  int ws;
};

// ---------------------------------------------------------------------------
// Level kernel: for plane (b, c) and a 16x16 output tile, compute
//   ssim_map, cs_map ; accumulate their sums into part[(plane)*nblk + blk][2]
// and (if maps != null) store per-pixel coefficient maps for backward:
//   A1 = dS/dmu1, A2 = dS/dmu2, B11 = dS/dsigma11-part..., see below.
// Output geometry: valid -> (H-ws+1) x (W-ws+1); same -> H x W (pad ws/2).
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(256) void msssim_level_kernel(const float* __restrict__ X, const float* __restrict__ Y,
                                                           int H, int W, MsWin win, float C1, float C2,
                                                           float* __restrict__ part, float* __restrict__ maps,
                                                           const float* __restrict__ wgt) {
  const int ws = win.ws;
  const int pad = MODE == 1 ? ws / 2 : 0;
  const int Ho = H + 2 * pad - ws + 1, Wo = W + 2 * pad - ws + 1;
  const int tiles_x = (Wo + MS_T - 1) / MS_T;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  const int plane = blockIdx.y;
  const float* x = X + (size_t)plane * H * W;
  const float* y = Y + (size_t)plane * H * W;
  constexpr int IN = MS_T + MS_MAXW - 1;  // 26
  __shared__ float sx[IN][IN + 1], sy[IN][IN + 1];
  __shared__ float v[5][MS_T][IN + 1];
  __shared__ float red[2][4];
  const int oy0 = ty * MS_T, ox0 = tx * MS_T;
  const int iy0 = oy0 - pad, ix0 = ox0 - pad;
  const int rows = MS_T + ws - 1;
  for (int e = threadIdx.x; e < rows * rows; e += 256) {
    const int r = e / rows, c = e % rows;
    const int iy = iy0 + r, ix = ix0 + c;
    float a = 0.f, b = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
      a = x[(size_t)iy * W + ix];
      b = y[(size_t)iy * W + ix];
    }
    sx[r][c] = a;
    sy[r][c] = b;
  }
  __syncthreads();
  // vertical pass (pytorch_msssim filters along H first): v[q][r][c] for r < MS_T, c < rows
  for (int e = threadIdx.x; e < MS_T * rows; e += 256) {
    const int r = e / rows, c = e % rows;
    float m1 = 0.f, m2 = 0.f, s11 = 0.f, s22 = 0.f, s12 = 0.f;
    for (int k = 0; k < ws; ++k) {
      const float wk = win.w[k];
      const float a = sx[r + k][c], b = sy[r + k][c];
      m1 += wk * a;
      m2 += wk * b;
      s11 += wk * (a * a);
      s22 += wk * (b * b);
      s12 += wk * (a * b);
    }
    v[0][r][c] = m1;
    v[1][r][c] = m2;
    v[2][r][c] = s11;
    v[3][r][c] = s22;
    v[4][r][c] = s12;
  }
  __syncthreads();
  const int r = threadIdx.x / MS_T, c = threadIdx.x % MS_T;
  const int oy = oy0 + r, ox = ox0 + c;
  float ssim = 0.f, cs = 0.f;
  if (oy < Ho && ox < Wo) {
    float m[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < ws; ++k) {
      const float wk = win.w[k];
#pragma unroll
      for (int q = 0; q < 5; ++q) m[q] += wk * v[q][r][c + k];
    }
    const float mu1 = m[0], mu2 = m[1];
    const float mu1sq = mu1 * mu1, mu2sq = mu2 * mu2, mu12 = mu1 * mu2;
    const float s1 = m[2] - mu1sq, s2 = m[3] - mu2sq, s12 = m[4] - mu12;
    const float V1 = 2.f * s12 + C2, V2 = s1 + s2 + C2;
    const float L1 = 2.f * mu12 + C1, L2 = mu1sq + mu2sq + C1;
    cs = V1 / V2;
    ssim = (MODE == 1) ? (L1 * V1) / (L2 * V2) : (L1 / L2) * cs;
    // (mode 1's ssim = L1 V1 / (L2 V2) == l * cs analytically; same derivative below)
    if (maps) {
      const float w_ssim = wgt[plane * 2], w_cs = wgt[plane * 2 + 1];
      // Objective per pixel: w_ssim*ssim + w_cs*cs (weights already / N_out).  Derivatives wrt the local
      // moments mu1, mu2, E11 = G*x^2, E22 = G*y^2, E12 = G*xy:
      const float l = L1 / L2;
      const float dcs_dV1 = 1.f / V2, dcs_dV2 = -V1 / (V2 * V2);
      const float dl_dL1 = 1.f / L2, dl_dL2 = -L1 / (L2 * L2);
      // ssim = l * cs
      const float gL1 = w_ssim * cs * dl_dL1, gL2 = w_ssim * cs * dl_dL2;
      const float gcs = w_ssim * l + w_cs;
      const float gV1 = gcs * dcs_dV1, gV2 = gcs * dcs_dV2;
      // L1 = 2 mu1 mu2 + C1 ; L2 = mu1^2 + mu2^2 + C1 ; V1 = 2 (E12 - mu1 mu2) + C2 ;
      // V2 = (E11 - mu1^2) + (E22 - mu2^2) + C2
      const float dE11 = gV2, dE22 = gV2, dE12 = 2.f * gV1;
      const float dmu1 = gL1 * 2.f * mu2 + gL2 * 2.f * mu1 - 2.f * gV1 * mu2 - 2.f * gV2 * mu1;
      const float dmu2 = gL1 * 2.f * mu1 + gL2 * 2.f * mu2 - 2.f * gV1 * mu1 - 2.f * gV2 * mu2;
      const size_t o = ((size_t)plane * Ho + oy) * Wo + ox;
      const size_t ps = (size_t)gridDim.y * Ho * Wo;
      maps[o] = dmu1;
      maps[ps + o] = dmu2;
      maps[2 * ps + o] = dE11;
      maps[3 * ps + o] = dE22;
      maps[4 * ps + o] = dE12;
    }
  }
  // block sums (fixed order)
  float a = wave_sum(ssim), b = wave_sum(cs);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[0][wv] = a;
    red[1][wv] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const size_t k = ((size_t)plane * gridDim.x + blockIdx.x) * 2;
    part[k] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[k + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// Transposed filter of the coefficient maps back to input pixels:
//   gx = G^T dmu1 + 2 x G^T dE11 + y G^T dE12 ; gy = G^T dmu2 + 2 y G^T dE22 + x G^T dE12
// accumulated (+=) into gX / gY at level resolution.
template <int MODE>
__global__ __launch_bounds__(256) void msssim_bwd_kernel(const float* __restrict__ X, const float* __restrict__ Y,
                                                         const float* __restrict__ maps, int H, int W, MsWin win,
                                                         float* __restrict__ gX, float* __restrict__ gY) {
  const int ws = win.ws;
  const int pad = MODE == 1 ? ws / 2 : 0;
  const int Ho = H + 2 * pad - ws + 1, Wo = W + 2 * pad - ws + 1;
  const int tiles_x = (W + MS_T - 1) / MS_T;
  const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
  const int plane = blockIdx.y;
  const size_t ps = (size_t)gridDim.y * Ho * Wo;
  constexpr int IN = MS_T + MS_MAXW - 1;
  __shared__ float sm[5][IN][IN + 1];
  __shared__ float v[5][MS_T][IN + 1];
  // input pixel i receives from output o where o = i + pad - k, k in [0, ws)
  const int iy0 = ty * MS_T, ix0 = tx * MS_T;
  const int oy0 = iy0 + pad - (ws - 1), ox0 = ix0 + pad - (ws - 1);
  const int rows = MS_T + ws - 1;
  for (int e = threadIdx.x; e < rows * rows; e += 256) {
    const int r = e / rows, c = e % rows;
    const int oy = oy0 + r, ox = ox0 + c;
    const bool ok = oy >= 0 && oy < Ho && ox >= 0 && ox < Wo;
    const size_t o = ((size_t)plane * Ho + (ok ? oy : 0)) * Wo + (ok ? ox : 0);
#pragma unroll
    for (int q = 0; q < 5; ++q) sm[q][r][c] = ok ? maps[q * ps + o] : 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < MS_T * rows; e += 256) {
    const int r = e / rows, c = e % rows;
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < ws; ++k) {
      const float wk = win.w[ws - 1 - k];
#pragma unroll
      for (int q = 0; q < 5; ++q) acc[q] += wk * sm[q][r + k][c];
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) v[q][r][c] = acc[q];
  }
  __syncthreads();
  const int r = threadIdx.x / MS_T, c = threadIdx.x % MS_T;
  const int iy = iy0 + r, ix = ix0 + c;
  if (iy < H && ix < W) {
    float t[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < ws; ++k) {
      const float wk = win.w[ws - 1 - k];
#pragma unroll
      for (int q = 0; q < 5; ++q) t[q] += wk * v[q][r][c + k];
    }
    const size_t i = ((size_t)plane * H + iy) * W + ix;
    const float xv = X[i], yv = Y[i];
    gX[i] += t[0] + 2.f * xv * t[2] + yv * t[4];
    gY[i] += t[1] + 2.f * yv * t[3] + xv * t[4];
  }
}

// avg_pool2d(kernel 2, stride 2, padding (ph, pw), count_include_pad) and its backward.
__global__ void avgpool2_kernel(const float* __restrict__ X, float* __restrict__ Yo, int P, int H, int W, int ph,
                                int pw) {
  const int Ho = (H + 2 * ph - 2) / 2 + 1, Wo = (W + 2 * pw - 2) / 2 + 1;
  const long total = (long)P * Ho * Wo;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ox = i % Wo;
    const long t = i / Wo;
    const int oy = t % Ho, p = t / Ho;
    float s = 0.f;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy)
#pragma unroll
      for (int dx = 0; dx < 2; ++dx) {
        const int iy = 2 * oy - ph + dy, ix = 2 * ox - pw + dx;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) s += X[((size_t)p * H + iy) * W + ix];
      }
    Yo[i] = s / 4.f;
  }
}

__global__ void avgpool2_bwd_kernel(const float* __restrict__ gO, float* __restrict__ gX, int P, int H, int W, int ph,
                                    int pw) {
  const int Ho = (H + 2 * ph - 2) / 2 + 1, Wo = (W + 2 * pw - 2) / 2 + 1;
  const long total = (long)P * H * W;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ix = i % W;
    const long t = i / W;
    const int iy = t % H, p = t / H;
    const int oy = (iy + ph) / 2, ox = (ix + pw) / 2;
    float g = 0.f;
    if (oy < Ho && ox < Wo) g = gO[((size_t)p * Ho + oy) * Wo + ox] / 4.f;
    gX[i] += g;
  }
}

__global__ void msssim_sum_kernel(const float* __restrict__ part, float* __restrict__ out, int nblk, float scale) {
  // out[plane][2] = sum over blocks of part[plane][blk][2] * scale
  const int plane = blockIdx.x;
  __shared__ float sh[2][4];
  float a = 0.f, b = 0.f;
  for (int k = threadIdx.x; k < nblk; k += 256) {
    a += part[((size_t)plane * nblk + k) * 2];
    b += part[((size_t)plane * nblk + k) * 2 + 1];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    sh[0][wv] = a;
    sh[1][wv] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[plane * 2] = ((sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3])) * scale;
    out[plane * 2 + 1] = ((sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3])) * scale;
  }
}

__global__ void scale_kernel(float* x, long n, float s) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= s;
}

// lvl[l][p][2] = per-plane means (ssim, cs) of level l.  mode 0: per group of G
// planes (an image), val = mean_p prod_l relu(v_lp)^w_l with v = cs (l<4), ssim (l=4).
// mode 1 (G = all planes): m_l = mean_p v_lp, val = prod_l m_l^w_l (no relu).
// If dval != null, writes wgt[l][p][2] = dL/dmean_{l,p}(ssim, cs) / nout[l].
__global__ void msssim_combine_kernel(const float* __restrict__ lvl, int P, int G, int mode, const float* __restrict__ dval,
                                      float* __restrict__ val, float* __restrict__ wgt, float n0, float n1, float n2,
                                      float n3, float n4) {
  const float w[5] = {0.0448f, 0.2856f, 0.3001f, 0.2363f, 0.1333f};
  const float nout[5] = {n0, n1, n2, n3, n4};
  const int grp = blockIdx.x * blockDim.x + threadIdx.x;
  if (grp * G >= P) return;
  auto v_of = [&](int l, int p) { return lvl[((size_t)l * P + p) * 2 + (l == 4 ? 0 : 1)]; };
  if (mode == 0) {
    float acc = 0.f;
    for (int p = grp * G; p < grp * G + G; ++p) {
      float prod = 1.f;
      for (int l = 0; l < 5; ++l) prod *= powf(fmaxf(v_of(l, p), 0.f), w[l]);
      acc += prod;
    }
    val[grp] = acc / (float)G;
    if (dval) {
      const float up = dval[grp] / (float)G;
      for (int p = grp * G; p < grp * G + G; ++p) {
        float vv[5], prod = 1.f;
        for (int l = 0; l < 5; ++l) {
          vv[l] = fmaxf(v_of(l, p), 0.f);
          prod *= powf(vv[l], w[l]);
        }
        for (int l = 0; l < 5; ++l) {
          const float d = (v_of(l, p) > 0.f) ? up * prod * w[l] / vv[l] : 0.f;
          float* o = wgt + ((size_t)l * P + p) * 2;
          o[0] = (l == 4 ? d : 0.f) / nout[l];
          o[1] = (l == 4 ? 0.f : d) / nout[l];
        }
      }
    }
  } else {
    float m[5];
    for (int l = 0; l < 5; ++l) {
      float acc = 0.f;
      for (int p = grp * G; p < grp * G + G; ++p) acc += v_of(l, p);
      m[l] = acc / (float)G;
    }
    float prod = 1.f;
    for (int l = 0; l < 5; ++l) prod *= powf(m[l], w[l]);
    val[grp] = prod;
    if (dval) {
      for (int l = 0; l < 5; ++l) {
        const float d = dval[grp] * prod * w[l] / m[l] / (float)G;
        for (int p = grp * G; p < grp * G + G; ++p) {
          float* o = wgt + ((size_t)l * P + p) * 2;
          o[0] = (l == 4 ? d : 0.f) / nout[l];
          o[1] = (l == 4 ? 0.f : d) / nout[l];
        }
      }
    }
  }
}

static MsWin make_win(const float* w, int ws) {
  MsWin m;
  for (int i = 0; i < MS_MAXW; ++i) m.w[i] = i < ws ? w[i] : 0.f;
  m.ws = ws;
  return m;
}

extern "C" {

// One level: X, Y are [P][H][W] planes (P = B*C).  part must hold
// P * ica_msssim_blocks(H, W, ws, mode) * 2 floats; out[P][2] = (mean ssim, mean cs)
// over the level's output pixels (per plane).  maps (optional) [5][P][Ho][Wo]
// receives the per-pixel derivative maps of  w_ssim*ssim + w_cs*cs  for backward.
int ica_msssim_blocks(int H, int W, int ws, int mode) {
  const int pad = mode == 1 ? ws / 2 : 0;
  const int Ho = H + 2 * pad - ws + 1, Wo = W + 2 * pad - ws + 1;
  return ((Wo + MS_T - 1) / MS_T) * ((Ho + MS_T - 1) / MS_T);
}

int ica_msssim_level(const float* X, const float* Y, int P, int H, int W, const float* win, int ws, int mode, float C1,
                     float C2, float* part, float* out, float* maps, const float* wgt, hipStream_t st) {
  if (maps && !wgt) return -4;
  if (ws > MS_MAXW || ws < 1) return -2;
  const int nblk = ica_msssim_blocks(H, W, ws, mode);
  if (nblk <= 0) return -3;
  const int pad = mode == 1 ? ws / 2 : 0;
  const int Ho = H + 2 * pad - ws + 1, Wo = W + 2 * pad - ws + 1;
  MsWin m = make_win(win, ws);
  dim3 grid(nblk, P);
  if (mode == 1)
    ICA_LAUNCH(msssim_level_kernel<1>, grid, dim3(256), 0, st, X, Y, H, W, m, C1, C2, part, maps, wgt);
  else
    ICA_LAUNCH(msssim_level_kernel<0>, grid, dim3(256), 0, st, X, Y, H, W, m, C1, C2, part, maps, wgt);
  ICA_CHECK_LAUNCH();
  ICA_LAUNCH(msssim_sum_kernel, dim3(P), dim3(256), 0, st, part, out, nblk, 1.0f / ((float)Ho * (float)Wo));
  ICA_CHECK_LAUNCH();
  return 0;
}

// maps (from ica_msssim_level with wgt) already carry the upstream gradient; accumulates into gX, gY.
int ica_msssim_level_bwd(const float* X, const float* Y, const float* maps, int P, int H, int W, const float* win,
                         int ws, int mode, float* gX, float* gY, hipStream_t st) {
  MsWin m = make_win(win, ws);
  dim3 grid(((W + MS_T - 1) / MS_T) * ((H + MS_T - 1) / MS_T), P);
  if (mode == 1)
    ICA_LAUNCH(msssim_bwd_kernel<1>, grid, dim3(256), 0, st, X, Y, maps, H, W, m, gX, gY);
  else
    ICA_LAUNCH(msssim_bwd_kernel<0>, grid, dim3(256), 0, st, X, Y, maps, H, W, m, gX, gY);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_avgpool2(const float* X, float* Yo, int P, int H, int W, int ph, int pw, hipStream_t st) {
  const int Ho = (H + 2 * ph - 2) / 2 + 1, Wo = (W + 2 * pw - 2) / 2 + 1;
  const long total = (long)P * Ho * Wo;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  ICA_LAUNCH(avgpool2_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, st, X, Yo, P, H, W, ph, pw);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_avgpool2_bwd(const float* gO, float* gX, int P, int H, int W, int ph, int pw, hipStream_t st) {
  const long total = (long)P * H * W;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  ICA_LAUNCH(avgpool2_bwd_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, st, gO, gX, P, H, W, ph, pw);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_msssim_combine(const float* lvl, int P, int G, int mode, const float* dval, float* val, float* wgt,
                       const float* nout, hipStream_t st) {
  const int groups = (P + G - 1) / G;
  ICA_LAUNCH(msssim_combine_kernel, dim3((groups + 63) / 64), dim3(64), 0, st, lvl, P, G, mode, dval, val, wgt,
                     nout[0], nout[1], nout[2], nout[3], nout[4]);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_scale(float* x, long n, float s, hipStream_t st) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  ICA_LAUNCH(scale_kernel, dim3((int)(g < 1 ? 1 : g)), dim3(256), 0, st, x, n, s);
  ICA_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

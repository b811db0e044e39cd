// Autoregressive (context-model) coding of the mbt2018 / cheng2020 latents (the models of
// anchors/model.py:74-77 whose y likelihood needs the masked 5x5 context model, anchors/model.py:97-106).
//
// The restated algorithm is CompressAI's JointAutoregressiveHierarchicalPriors._compress_ar / _decompress_ar
// (compressai 1.x, not vendored in the reference): latent positions in raster order; at each
// position the masked ("A") 5x5 context conv over the already-coded neighbours (12 causal taps of the zero-padded
// y_hat), entropy_parameters (1x1 convs 4M -> 10M/3 -> 8M/3 -> 2M with LeakyReLU 0.01) on cat(h_s params, ctx),
// scales = first M outputs, means = last M; index = the scale-table row of max(scale, 0.11), symbol =
// round(y - mean) (round half to even), y_hat = symbol + mean.  Symbols and indexes are emitted position-major,
// channel-minor: the order the bitstream holds.
//
// MI355X mapping: the chain over positions is sequential per image, so one workgroup runs one image's whole
// raster (encode: one launch), its four matrix-vector products per position spread over the 4 waves (lanes
// stride the reduction dimension: coalesced weight rows out of L2, a butterfly reduction per row); a batch of
// images runs in parallel on as many CUs.  Decoding needs the symbols of position p before the context of p + 1:
// the host's rANS decoder (ica_codec.hip) decodes one position of every image between two launches of the
// step kernel (mode 1: apply the previous position's symbols, then emit the next position's indexes / means).
#include "ica_common.h"

#include <cstring>

namespace {

// out[o] = bias[o] + sum_k W[o][k] v[k]  (o < O; v in LDS), LeakyReLU(0.01) when LR; four rows per wave pass,
// lanes over k, then a fixed butterfly reduction (deterministic: the encoder and the decoder run this same code)
template <bool LR>
ICA_DEV void ar_matvec(const float* __restrict__ w, const float* __restrict__ bias, const float* v, int K, int O,
                       float* dst) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int o0 = wave * 4; o0 < O; o0 += 16) {
    const float* r0 = w + (size_t)min(o0, O - 1) * K;
    const float* r1 = w + (size_t)min(o0 + 1, O - 1) * K;
    const float* r2 = w + (size_t)min(o0 + 2, O - 1) * K;
    const float* r3 = w + (size_t)min(o0 + 3, O - 1) * K;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
    for (int k = lane; k < K; k += 64) {
      const float x = v[k];
      a0 = fmaf(r0[k], x, a0);
      a1 = fmaf(r1[k], x, a1);
      a2 = fmaf(r2[k], x, a2);
      a3 = fmaf(r3[k], x, a3);
    }
#pragma unroll
    for (int s = 32; s > 0; s >>= 1) {
      a0 += __shfl_xor(a0, s, 64);
      a1 += __shfl_xor(a1, s, 64);
      a2 += __shfl_xor(a2, s, 64);
      a3 += __shfl_xor(a3, s, 64);
    }
    if (lane < 4 && o0 + lane < O) {
      float t = (lane == 0 ? a0 : lane == 1 ? a1 : lane == 2 ? a2 : a3) + bias[o0 + lane];
      if (LR) t = t > 0.f ? t : 0.01f * t;
      dst[o0 + lane] = t;
    }
  }
}

struct ArArgs {
  const float* y;          // mode 0: the latents, nChw4c [B][M/4][H][W][4]
  const float* params;     // h_s(z_hat), nChw4c [B][2M/4][H][W][4]
  float* yhat;             // [B][M][H + 4][W + 4], zero-initialised: CompressAI's padded y_hat
  int32_t* sym;            // mode 0: [B][H W M] symbols (position-major)
  int32_t* idx;            // mode 0: [B][H W M] CDF rows; mode 1: [B][M] rows of the position just computed
  const int32_t* sym_in;   // mode 1: [B][M] decoded symbols of the previous position
  float* means;            // mode 1: [B][M] means of the position just computed (kept for the next launch)
  const float* wc;         // [2M][12 M] masked-conv weight over the 12 causal taps (k = tap * M + c)
  const float* bc;         // [2M]
  const float* w1;         // [E1][4M]
  const float* b1;
  const float* w2;         // [E2][E1]
  const float* b2;
  const float* w3;         // [2M][E2]
  const float* b3;
  const float* table;      // [T] scale table
  int T;
  float bound;             // scale lower bound (0.11)
  int B, M, H, W, E1, E2;
};

__global__ __launch_bounds__(256) void ar_step_kernel(ArArgs a, int p0, int p1, int mode) {
  extern __shared__ float lds[];
  const int b = blockIdx.x, M = a.M, H = a.H, W = a.W, tid = threadIdx.x;
  float* in = lds;             // 4M: params (2M), then ctx (2M): torch.cat((params, ctx), dim=1)
  float* nb = in + 4 * M;      // 12M causal neighbours
  float* e1 = nb + 12 * M;     // E1
  float* e2 = e1 + a.E1;       // E2
  float* gp = e2 + a.E2;       // 2M: scales, means
  const int HP = H + 4, WP = W + 4;
  float* yh = a.yhat + (size_t)b * M * HP * WP;
  const int C4p = (2 * M + 3) >> 2, C4y = (M + 3) >> 2;
  if (mode == 1 && p0 > 0) {   // the previous position's decoded symbols: y_hat = symbol + mean
    const int h = (p0 - 1) / W, w = (p0 - 1) - ((p0 - 1) / W) * W;
    for (int c = tid; c < M; c += 256)
      yh[((size_t)c * HP + h + 2) * WP + w + 2] =
          __fadd_rn((float)a.sym_in[(size_t)b * M + c], a.means[(size_t)b * M + c]);
    __syncthreads();
  }
  for (int p = p0; p < p1; ++p) {
    const int h = p / W, w = p - h * W;
    // the 12 causal taps of the type-A mask: rows 0-1 of the 5x5 window, then columns 0-1 of row 2
    for (int e = tid; e < 12 * M; e += 256) {
      const int t = e / M, c = e - t * M;
      const int ky = t < 10 ? t / 5 : 2, kx = t < 10 ? t - 5 * (t / 5) : t - 10;
      nb[e] = yh[((size_t)c * HP + h + ky) * WP + w + kx];
    }
    for (int e = tid; e < 2 * M; e += 256)
      in[e] = a.params[((((size_t)b * C4p + (e >> 2)) * H + h) * W + w) * 4 + (e & 3)];
    __syncthreads();
    ar_matvec<false>(a.wc, a.bc, nb, 12 * M, 2 * M, in + 2 * M);
    __syncthreads();
    ar_matvec<true>(a.w1, a.b1, in, 4 * M, a.E1, e1);
    __syncthreads();
    ar_matvec<true>(a.w2, a.b2, e1, a.E1, a.E2, e2);
    __syncthreads();
    ar_matvec<false>(a.w3, a.b3, e2, a.E2, 2 * M, gp);
    __syncthreads();
    for (int c = tid; c < M; c += 256) {
      const float s = fmaxf(gp[c], a.bound);   // LowerBound(scale_bound)
      int k = a.T - 1;
      for (int j = 0; j < a.T - 1; ++j) k -= (s <= a.table[j]) ? 1 : 0;
      const float mean = gp[M + c];
      if (mode == 0) {
        const float yv = a.y[((((size_t)b * C4y + (c >> 2)) * H + h) * W + w) * 4 + (c & 3)];
        const float q = rintf(__fsub_rn(yv, mean));
        yh[((size_t)c * HP + h + 2) * WP + w + 2] = __fadd_rn(q, mean);
        const size_t o = ((size_t)b * H * W + p) * M + c;
        a.sym[o] = (int32_t)q;
        a.idx[o] = k;
      } else {
        a.idx[(size_t)b * M + c] = k;
        a.means[(size_t)b * M + c] = mean;
      }
    }
    __syncthreads();   // this position's y_hat before the next position's context loads
  }
}

}  // namespace

extern "C" {

// C-ABI mirror of ArArgs (include/ica_hip.h ica_ar_args)
typedef struct ica_ar_args {
  const float* y;
  const float* params;
  float* yhat;
  int32_t* sym;
  int32_t* idx;
  const int32_t* sym_in;
  float* means;
  const float* wc;
  const float* bc;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
  const float* w3;
  const float* b3;
  const float* table;
  int T;
  float bound;
  int B, M, H, W, E1, E2;
} ica_ar_args;

size_t ica_ar_lds_bytes(int M, int E1, int E2) { return (size_t)(18 * M + E1 + E2) * sizeof(float); }

// Positions [p0, p1) of every image (one workgroup each).  mode 0: encode (y -> symbols, indexes, y_hat);
// mode 1: decode step (apply sym_in to position p0 - 1 when p0 > 0, then indexes / means of p0 .. p1 - 1;
// the caller passes p1 <= p0 + 1).  Returns 0, -2 on bad sizes, -4 on a bad mode.
int ica_ar_step(const ica_ar_args* a, int p0, int p1, int mode, hipStream_t st) {
  if (mode != 0 && mode != 1) return -4;
  if (a->B <= 0 || a->M <= 0 || a->M % 4 || a->H <= 0 || a->W <= 0 || a->E1 <= 0 || a->E2 <= 0 || a->T < 1)
    return -2;
  if (p0 < 0 || p1 < p0 || p1 > a->H * a->W || (mode == 1 && p1 > p0 + 1)) return -2;
  const size_t lds = ica_ar_lds_bytes(a->M, a->E1, a->E2);
  if (lds > 64 * 1024) return -2;
  ArArgs k;
  static_assert(sizeof(ArArgs) == sizeof(ica_ar_args), "ArArgs mirrors ica_ar_args");
  std::memcpy(&k, a, sizeof(k));
  ICA_LAUNCH(ar_step_kernel, dim3(a->B), dim3(256), lds, st, k, p0, p1, mode);
  ICA_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// Real entropy coding of the latents: CompressAI's EntropyBottleneck /
// GaussianConditional compress() / decompress() around a 64-bit rANS coder with 16-bit CDFs and
// 4-bit bypass coding of out-of-range values (the CompressAI coder the reference's models carry:
// `_quantized_cdf` / `_offset` / `_cdf_length` buffers, anchors/balle.py:57-72, anchors/utils.py:74-109).
//
// Split of the work:
//   device  symbols + CDF indexes straight from the nChw4c latents (NCHW order out, the order the
//           bitstream uses), and the dequantisation of decoded symbols back into nChw4c;
//   host    the rANS coder itself.  One bitstream per image is a single sequential rANS state (the
//           format CompressAI readers expect), so it runs on a CPU core; the caller encodes the images
//           of a batch on parallel host threads (the C ABI holds no global state).
//   host    pmf_to_quantized_cdf (once per model update).
#include "ica_common.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

// ---------------------------------------------------------------------------
// Device: symbols / indexes / dequantisation (NCHW index t <-> nChw4c element)
// ---------------------------------------------------------------------------
ICA_DEV long nc4_off(long t, int C, int H, int W) {
  const long hw = (long)H * W;
  const long n = t / ((long)C * hw);
  const long r = t - n * (long)C * hw;
  const int c = (int)(r / hw);
  const long p = r - (long)c * hw;
  const int C4 = (C + 3) >> 2;
  return (((long)n * C4 + (c >> 2)) * hw + p) * 4 + (c & 3);
}

// GaussianConditional.build_indexes + quantize(y, "symbols", means):
//   s = max(scale, bound); index = T-1 - #{j < T-1 : s <= table[j]};  symbol = int(round(y - mean))
__global__ void gc_symbols_kernel(const float* __restrict__ y4, const float* __restrict__ s4,
                                  const float* __restrict__ m4, const float* __restrict__ table, int T, float bound,
                                  int32_t* __restrict__ sym, int32_t* __restrict__ idx, long total, int C, int H,
                                  int W) {
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long o = nc4_off(t, C, H, W);
    const float s = fmaxf(s4[o], bound);
    int k = T - 1;
    for (int j = 0; j < T - 1; ++j) k -= (s <= table[j]) ? 1 : 0;
    const float v = m4 ? __fsub_rn(y4[o], m4[o]) : y4[o];
    sym[t] = (int32_t)rintf(v);
    idx[t] = k;
  }
}

// EntropyBottleneck.compress: symbol = int(round(z - median[c])), index = c
__global__ void eb_symbols_kernel(const float* __restrict__ z4, const float* __restrict__ med,
                                  int32_t* __restrict__ sym, int32_t* __restrict__ idx, long total, int C, int H,
                                  int W) {
  const long hw = (long)H * W;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int c = (int)((t / hw) % C);
    sym[t] = (int32_t)rintf(__fsub_rn(z4[nc4_off(t, C, H, W)], med[c]));
    idx[t] = c;
  }
}

// dequantize: out = float(symbol) + mean (mean4: nChw4c means, or med[c] per channel, or none)
__global__ void dequantize_kernel(const int32_t* __restrict__ sym, const float* __restrict__ m4,
                                  const float* __restrict__ med, float* __restrict__ out4, long total, int C, int H,
                                  int W) {
  const long hw = (long)H * W;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const long o = nc4_off(t, C, H, W);
    float v = (float)sym[t];
    if (m4) v = __fadd_rn(v, m4[o]);
    else if (med) v = __fadd_rn(v, med[(int)((t / hw) % C)]);
    out4[o] = v;
  }
}

// ---------------------------------------------------------------------------
// Host: 64-bit rANS (32-bit renormalisation words, state in [2^31, 2^63)), 16-bit frequencies
// ---------------------------------------------------------------------------
namespace {
constexpr int kPrec = 16;
constexpr uint32_t kBypassBits = 4;
constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;
constexpr uint64_t kRansL = 1ull << 31;

struct Sym {
  uint32_t start, freq;
  bool bypass;
};

inline void enc_put(uint64_t& x, uint32_t*& p, uint32_t start, uint32_t freq) {
  const uint64_t x_max = ((kRansL >> kPrec) << 32) * freq;
  if (x >= x_max) {
    *--p = (uint32_t)x;
    x >>= 32;
  }
  x = ((x / freq) << kPrec) + (x % freq) + start;
}
// raw bits: the same renormalisation as a symbol of frequency 2^(16 - nbits), then x = x * 2^nbits + val
inline void enc_put_bits(uint64_t& x, uint32_t*& p, uint32_t val, uint32_t nbits) {
  const uint64_t x_max = ((kRansL >> kPrec) << 32) * (1u << (kPrec - nbits));
  if (x >= x_max) {
    *--p = (uint32_t)x;
    x >>= 32;
  }
  x = (x << nbits) | val;
}

// The coding sequence of symbol i: its CDF slot, then for an escape (the tail slot max_value) the
// count of 4-bit groups in unary-ish 15-chunks and the raw groups, least significant first.
inline int expand(int32_t s, const int32_t* cdf, int32_t max_value, int32_t offset, Sym* out) {
  int32_t value = s - offset;
  uint32_t raw = 0;
  if (value < 0) {
    raw = (uint32_t)(-2 * (int64_t)value - 1);
    value = max_value;
  } else if (value >= max_value) {
    raw = (uint32_t)(2 * (int64_t)(value - max_value));
    value = max_value;
  }
  int n = 0;
  out[n++] = {(uint32_t)cdf[value], (uint32_t)(cdf[value + 1] - cdf[value]), false};
  if (value == max_value) {
    int32_t nb = 0;
    while (nb < 8 && (raw >> (nb * kBypassBits)) != 0) ++nb;
    int32_t v = nb;
    while (v >= (int32_t)kBypassMax) {
      out[n++] = {kBypassMax, 0, true};
      v -= kBypassMax;
    }
    out[n++] = {(uint32_t)v, 0, true};
    for (int32_t j = 0; j < nb; ++j) out[n++] = {(raw >> (j * kBypassBits)) & kBypassMax, 0, true};
  }
  return n;
}

inline bool table_ok(int32_t k, int n_cdfs, const int32_t* sizes, int stride) {
  return k >= 0 && k < n_cdfs && sizes[k] >= 3 && sizes[k] <= stride;
}
}  // namespace

extern "C" {

static inline int grid_1d_codec(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 16384 ? 16384 : (g < 1 ? 1 : g));
}

int ica_gc_symbols(const float* y4, const float* scales4, const float* means4, const float* table, int T, float bound,
                   int32_t* symbols, int32_t* indexes, int B, int C, int H, int W, hipStream_t st) {
  if (T < 1) return -5;
  const long total = (long)B * C * H * W;
  ICA_LAUNCH(gc_symbols_kernel, dim3(grid_1d_codec(total)), dim3(256), 0, st, y4, scales4, means4, table, T,
                     bound, symbols, indexes, total, C, H, W);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_eb_symbols(const float* z4, const float* medians, int32_t* symbols, int32_t* indexes, int B, int C, int H,
                   int W, hipStream_t st) {
  const long total = (long)B * C * H * W;
  ICA_LAUNCH(eb_symbols_kernel, dim3(grid_1d_codec(total)), dim3(256), 0, st, z4, medians, symbols, indexes,
                     total, C, H, W);
  ICA_CHECK_LAUNCH();
  return 0;
}

int ica_dequantize(const int32_t* symbols, const float* means4, const float* medians, float* out4, int B, int C, int H,
                   int W, hipStream_t st) {
  const long total = (long)B * C * H * W;
  ICA_LAUNCH(dequantize_kernel, dim3(grid_1d_codec(total)), dim3(256), 0, st, symbols, means4, medians, out4,
                     total, C, H, W);
  ICA_CHECK_LAUNCH();
  return 0;
}

// pmf (n float32 probabilities) -> n + 1 cumulative 16-bit frequencies, every symbol at least 1
// (round(p * 2^16), rescale by the total, prefix sum, then steal one count from the smallest
// frequency > 1 for each empty slot).  Returns 0, -1 for a negative / non-finite pmf, -2 for an
// all-zero pmf, -3 when no frequency can be stolen.
int ica_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int32_t* cdf_out) {
  if (n < 1 || precision < 1 || precision > 24) return -5;
  std::vector<uint32_t> cdf(n + 1);
  cdf[0] = 0;
  for (int i = 0; i < n; ++i) {
    const float p = pmf[i];
    if (p < 0 || !std::isfinite(p)) return -1;
    cdf[i + 1] = (uint32_t)std::round(p * (float)(1 << precision));
  }
  uint32_t total = 0;
  for (uint32_t v : cdf) total += v;
  if (total == 0) return -2;
  for (auto& v : cdf) v = (uint32_t)(((uint64_t)(1u << precision) * v) / total);
  for (int i = 1; i <= n; ++i) cdf[i] += cdf[i - 1];
  cdf[n] = 1u << precision;
  for (int i = 0; i < n; ++i) {
    if (cdf[i] != cdf[i + 1]) continue;
    uint32_t best_freq = ~0u;
    int best = -1;
    for (int j = 0; j < n; ++j) {
      const uint32_t f = cdf[j + 1] - cdf[j];
      if (f > 1 && f < best_freq) {
        best_freq = f;
        best = j;
      }
    }
    if (best < 0) return -3;
    if (best < i) {
      for (int j = best + 1; j <= i; ++j) cdf[j]--;
    } else {
      for (int j = i + 1; j <= best; ++j) cdf[j]++;
    }
  }
  for (int i = 0; i <= n; ++i) cdf_out[i] = (int32_t)cdf[i];
  return 0;
}

// Encode n symbols of one image: symbol i with CDF row indexes[i] (cdfs: n_cdfs rows of `stride`
// int32, row k valid for cdf_sizes[k] entries, offsets[k] = value of slot 0).  Writes the bitstream
// (32-bit little-endian words) into out; returns its length in bytes, -7 with *needed set when cap is
// too small, -5 on a bad index / table.
long ica_rans_encode(const int32_t* symbols, const int32_t* indexes, long n, const int32_t* cdfs, int stride,
                     const int32_t* cdf_sizes, const int32_t* offsets, int n_cdfs, uint8_t* out, long cap,
                     long* needed) {
  // worst case per symbol: 1 slot + 1 count group + 8 raw groups, one word each, plus the 2-word flush
  std::vector<uint32_t> buf((size_t)n * 10 + 2);
  uint32_t* const end = buf.data() + buf.size();
  uint32_t* p = end;
  uint64_t x = kRansL;
  Sym seq[12];
  for (long i = n - 1; i >= 0; --i) {
    const int32_t k = indexes[i];
    if (!table_ok(k, n_cdfs, cdf_sizes, stride)) return -5;
    const int m = expand(symbols[i], cdfs + (long)k * stride, cdf_sizes[k] - 2, offsets[k], seq);
    for (int j = m - 1; j >= 0; --j) {
      if (seq[j].bypass) enc_put_bits(x, p, seq[j].start, kBypassBits);
      else {
        if (seq[j].freq == 0) return -5;
        enc_put(x, p, seq[j].start, seq[j].freq);
      }
    }
  }
  p -= 2;
  p[0] = (uint32_t)x;
  p[1] = (uint32_t)(x >> 32);
  const long nbytes = (long)(end - p) * 4;
  if (needed) *needed = nbytes;
  if (nbytes > cap) return -7;
  std::memcpy(out, p, (size_t)nbytes);
  return nbytes;
}

// One bitstream's decoder state: the words, the read position and the 64-bit rANS state.  Decoding can stop after
// any symbol and resume with the next call (the context models decode one latent position at a time, because the
// next position's CDF rows depend on the symbols just decoded).
struct RansDec {
  std::vector<uint32_t> words;
  size_t pos = 0;
  uint64_t x = 0;
};

static int rans_dec_init(RansDec& d, const uint8_t* data, long nbytes) {
  if (nbytes < 8 || (nbytes & 3)) return -8;
  d.words.resize((size_t)nbytes / 4);
  std::memcpy(d.words.data(), data, (size_t)nbytes);
  d.x = (uint64_t)d.words[0] | ((uint64_t)d.words[1] << 32);
  d.pos = 2;
  return 0;
}

static int rans_dec_run(RansDec& d, const int32_t* indexes, long n, const int32_t* cdfs, int stride,
                        const int32_t* cdf_sizes, const int32_t* offsets, int n_cdfs, int32_t* symbols) {
  const size_t end = d.words.size();
  const uint32_t mask = (1u << kPrec) - 1;
  uint64_t x = d.x;
  size_t p = d.pos;
  auto get_bits = [&](uint32_t nb, uint32_t& v) -> bool {
    v = (uint32_t)(x & ((1u << nb) - 1));
    x >>= nb;
    if (x < kRansL) {
      if (p >= end) return false;
      x = (x << 32) | d.words[p++];
    }
    return true;
  };
  for (long i = 0; i < n; ++i) {
    const int32_t k = indexes[i];
    if (!table_ok(k, n_cdfs, cdf_sizes, stride)) return -5;
    const int32_t* cdf = cdfs + (long)k * stride;
    const int32_t size = cdf_sizes[k];
    const int32_t max_value = size - 2;
    const uint32_t cum = (uint32_t)(x & mask);
    // first slot whose upper bound exceeds cum (the table is strictly increasing)
    const int32_t* it = std::upper_bound(cdf, cdf + size, (int32_t)cum);
    const int32_t s = (int32_t)(it - cdf) - 1;
    if (s < 0 || s >= size - 1) return -8;
    const uint32_t start = (uint32_t)cdf[s], freq = (uint32_t)(cdf[s + 1] - cdf[s]);
    x = freq * (x >> kPrec) + (x & mask) - start;
    if (x < kRansL) {
      if (p >= end) return -8;
      x = (x << 32) | d.words[p++];
    }
    int32_t value = s;
    if (value == max_value) {
      uint32_t v;
      if (!get_bits(kBypassBits, v)) return -8;
      int32_t nb = (int32_t)v;
      while (v == kBypassMax) {
        if (!get_bits(kBypassBits, v)) return -8;
        nb += (int32_t)v;
      }
      if (nb > 8) return -8;
      uint32_t raw = 0;
      for (int32_t j = 0; j < nb; ++j) {
        if (!get_bits(kBypassBits, v)) return -8;
        raw |= v << (j * kBypassBits);
      }
      value = (int32_t)(raw >> 1);
      value = (raw & 1) ? -value - 1 : value + max_value;
    }
    symbols[i] = value + offsets[k];
  }
  d.x = x;
  d.pos = p;
  return 0;
}

// Decode n symbols (the inverse of ica_rans_encode with the same indexes / tables).  Returns 0, -5 on a
// bad index / table, -8 when the stream ends early (truncated or corrupt input).
int ica_rans_decode(const uint8_t* data, long nbytes, const int32_t* indexes, long n, const int32_t* cdfs, int stride,
                    const int32_t* cdf_sizes, const int32_t* offsets, int n_cdfs, int32_t* symbols) {
  RansDec d;
  if (const int rc = rans_dec_init(d, data, nbytes)) return rc;
  return rans_dec_run(d, indexes, n, cdfs, stride, cdf_sizes, offsets, n_cdfs, symbols);
}

// Incremental decoding (the context models): open a decoder on one bitstream (*decoder = NULL and -8 for a
// malformed one), decode n symbols of each of B open decoders per call (indexes / symbols [B][n]; returns 0 or the
// first error, the failing image in *bad), close.
int ica_rans_dec_open(const uint8_t* data, long nbytes, void** decoder) {
  RansDec* d = new RansDec;
  if (const int rc = rans_dec_init(*d, data, nbytes)) {
    delete d;
    *decoder = nullptr;
    return rc;
  }
  *decoder = d;
  return 0;
}

int ica_rans_dec_step(void* const* decoders, int B, const int32_t* indexes, long n, const int32_t* cdfs, int stride,
                      const int32_t* cdf_sizes, const int32_t* offsets, int n_cdfs, int32_t* symbols, int* bad) {
  for (int b = 0; b < B; ++b) {
    RansDec* d = static_cast<RansDec*>(decoders[b]);
    const int rc = d ? rans_dec_run(*d, indexes + (long)b * n, n, cdfs, stride, cdf_sizes, offsets, n_cdfs,
                                    symbols + (long)b * n)
                     : -8;
    if (rc != 0) {
      if (bad) *bad = b;
      return rc;
    }
  }
  return 0;
}

int ica_rans_dec_close(void* decoder) {
  delete static_cast<RansDec*>(decoder);
  return 0;
}

}  // extern "C"

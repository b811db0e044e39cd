// Shared device helpers for libica_hip (gfx950 / CDNA4 only).
//
// Activation layout on the hot path is nChw4c: [N][ceil(C/4)][H][W][4] fp32.
// Four consecutive channels of one pixel are one 16-byte vector, so the
// MFMA accumulator rows (4 consecutive output channels per register quad)
// store as one dwordx4 per lane and 32 lanes cover 512 contiguous bytes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define ICA_DEV __device__ __forceinline__

// v_mfma_f32_32x32x2_f32: lane l supplies A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
// D lane l, reg r = D[i=(r&3)+8*(r>>2)+4*(l>>5)][j=l&31].
ICA_DEV f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// Row index (within a 32-row tile) held by accumulator register r of lane half h.
ICA_DEV constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

ICA_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
ICA_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

// Round-to-nearest, no contraction (used where the reference's op order matters).
ICA_DEV float fmul_rn(float a, float b) { return __fmul_rn(a, b); }
ICA_DEV float fadd_rn(float a, float b) { return __fadd_rn(a, b); }
ICA_DEV float fsub_rn(float a, float b) { return __fsub_rn(a, b); }
ICA_DEV float fdiv_rn(float a, float b) { return __fdiv_rn(a, b); }

// Wave-level sum (64 lanes), deterministic order.
ICA_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

#define ICA_CHECK_LAUNCH()                          \
  do {                                              \
    hipError_t _e = hipGetLastError();              \
    if (_e != hipSuccess) return (int)_e;           \
  } while (0)

// Targeted / ROI attack weights: box [y0, y1) x [x0, x1) is the target region.
// Per-element loss weights: input term  w_in  = tar ? 1/cnt_tar : la_bkg_in/cnt_bkg,
//                           output term w_out = tar ? la_tar/cnt_tar : la_bkg_out/cnt_bkg
// (cnt = 3 * pixels of the region; a zero count gives weight 0).
struct RoiBox {
  int x0, x1, y0, y1;
  float w_in_tar, w_in_bkg, w_out_tar, w_out_bkg;
};
ICA_DEV bool roi_inside(const RoiBox& r, long pix, long W) {
  const long y = pix / W, x = pix - y * W;
  return x >= r.x0 && x < r.x1 && y >= r.y0 && y < r.y1;
}

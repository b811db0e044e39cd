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

// v_mfma_f32_32x32x16_bf16: lane l (r = l&31, h = l>>5) supplies A[r][k = 8h + j], B[k = 8h + j][r]
// in element j = 0..7; the D layout is that of the f32 form (dtype-independent on gfx950).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
ICA_DEV f32x16 mfma32bf(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// 8 fp32 -> 8 bf16 (round to nearest even: v_cvt_pk_bf16_f32)
ICA_DEV bf16x8 to_bf8(f32x4 lo, f32x4 hi) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    r[e] = (__bf16)lo[e];
    r[4 + e] = (__bf16)hi[e];
  }
  return r;
}
// v = hi + lo + O(2^-16 |v|): the two-term bf16 split of a fp32 operand (bf16x3 products)
ICA_DEV void split_bf(float v, __bf16& hi, __bf16& lo) {
  hi = (__bf16)v;
  lo = (__bf16)(v - (float)hi);
}
// Buffer-descriptor loads of wave-uniform tables (32-bit lane offset + scalar/immediate offset, so
// the compiler keeps no per-fragment 64-bit address registers live).
ICA_DEV __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
ICA_DEV bf16x8 ld_bf8(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
ICA_DEV f32x4 bf4_to_f4(u32x2 raw) {
  const bf16x4 b = __builtin_bit_cast(bf16x4, raw);
  return f32x4{(float)b[0], (float)b[1], (float)b[2], (float)b[3]};
}
ICA_DEV u32x2 f4_to_bf4(f32x4 v) {
  const bf16x4 b = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  return __builtin_bit_cast(u32x2, b);
}

// Per-image view of an nChw4c tensor through a buffer descriptor (n is block-uniform): a 32-bit lane
// offset (vq) plus a wave-uniform scalar offset (sq), both in channel quads (4 channels of one pixel:
// 16 B fp32, 8 B when B16 = the bf16 activations of the bf16 conv path), so an epilogue keeps no 64-bit
// per-element address registers live (those spilled in the GDN-backward epilogue).  Loads return and
// stores take fp32 (bf16 round-to-nearest-even on store).  One image must be < 4 GiB.
template <bool B16 = false>
struct Img4T {
  static constexpr unsigned ESZ = B16 ? 8u : 16u;
  __amdgpu_buffer_rsrc_t r;
  ICA_DEV Img4T(const void* base, size_t img_quads, int n)
      : r(uniform_rsrc(base ? static_cast<const char*>(base) + (size_t)n * img_quads * ESZ : base,
                       (unsigned)(img_quads * ESZ))) {}
  ICA_DEV f32x4 ld(unsigned vq, unsigned sq) const {
    if constexpr (B16) {
      return bf4_to_f4(__builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(vq * ESZ),
                                                                                      (int)(sq * ESZ), 0)));
    } else {
      return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(vq * ESZ), (int)(sq * ESZ), 0));
    }
  }
  // Stores fold the scalar offset into the lane offset and pass a constant soffset 0.  With an SGPR
  // soffset, hipcc (ROCm 7.2) omits the wait state between a >8-byte buffer store and a VALU overwrite of
  // its data registers (LLVM models that hazard only for a constant soffset); on gfx950 the overwrite
  // then corrupted dword 1 of lanes 12-15 of each 16-lane group (measured: conv_up IGDN save_s).
  ICA_DEV void st(unsigned vq, unsigned sq, f32x4 v) const {
    if constexpr (B16) {
      __builtin_amdgcn_raw_buffer_store_b64(f4_to_bf4(v), r, (int)((vq + sq) * ESZ), 0, 0);
    } else {
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)((vq + sq) * ESZ), 0, 0);
    }
  }
};
typedef Img4T<false> Img4;
ICA_DEV f32x4 bf8_as_f4(bf16x8 v) { return __builtin_bit_cast(f32x4, v); }
ICA_DEV bf16x8 f4_as_bf8(f32x4 v) { return __builtin_bit_cast(bf16x8, v); }

// Row index (within a 32-row tile) held by accumulator register r of lane half h.
ICA_DEV constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// XCD-aware block order (a speed choice only; used by the bf16 conv kernels, +2-3 % on config 5, while the
// MFMA-bound fp32 kernels measured neutral to -1 % and keep the plain order).  Workgroups are dealt
// round-robin over the 8 XCDs by linear id, so neighbouring conv tiles (which share patch halo rows) land
// on different private L2s.  Remap the linear id so each XCD gets one contiguous run of (tile,
// channel-block) ids: q = total/8, r = total%8, XCD x = lin%8 takes ids [x*q + min(x,r), ... + q + (x<r))
// in dispatch order (a bijection for any total).
template <bool REMAP>
ICA_DEV void xcd_block(int& bx, int& by) {
  const unsigned nx = gridDim.x, total = nx * gridDim.y;
  const unsigned lin = blockIdx.y * nx + blockIdx.x;
  unsigned L = lin;
  if constexpr (REMAP) {
    const unsigned q = total >> 3, r = total & 7, x = lin & 7;
    L = x * q + (x < r ? x : r) + (lin >> 3);
  }
  bx = (int)(L % nx);
  by = (int)(L / nx);
}

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

// Compute units of the current device (host side; persistent launches size their grid to it).
inline int ica_cu_count() {
  static int cus = 0;
  if (cus <= 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      cus = v;
    else
      cus = 256;
  }
  return cus;
}

// Every launcher records the kernel and grid of its last launch and counts launches (ICA_LAUNCH), so that a host
// that just timed a tagged launch can ask which kernel that was and whether it was the only one (ica_last_launch
// consumes the record): bench.py checks its PMC traffic stamps with it.
struct IcaLaunchRec {
  const void* fn;
  unsigned long long threads;   // grid x block, as rocprofv3's Grid_Size
  int count;                    // launches since the record was last consumed, saturated at 2 (callers need 0 / 1 /
                                // many; a hook-less run never consumes it)
};
inline IcaLaunchRec& ica_launch_rec() {
  static thread_local IcaLaunchRec r{nullptr, 0, 0};
  return r;
}
template <typename F>
inline const void* ica_fnptr(F* f) {   // a kernel (function designator or pointer variable) -> its host stub
  return reinterpret_cast<const void*>(f);
}
#define ICA_LAUNCH(kern, grid, block, lds, st, ...)                                                           \
  do {                                                                                                       \
    const dim3 ica_g_ = (grid), ica_b_ = (block);                                                                \
    IcaLaunchRec& ica_r_ = ica_launch_rec();                                                                 \
    ica_r_ = IcaLaunchRec{ica_fnptr(kern),                                                                   \
                          (unsigned long long)ica_g_.x * ica_g_.y * ica_g_.z * ica_b_.x * ica_b_.y * ica_b_.z, \
                          ica_r_.count < 2 ? ica_r_.count + 1 : 2};                                          \
    hipLaunchKernelGGL(kern, ica_g_, ica_b_, lds, st, __VA_ARGS__);                                          \
  } while (0)

// In-kernel clock (diagnostic builds only, -DICA_CLOCK_STAMP via scripts/build_variant.sh; the product library
// compiles these to nothing).  Wave 0 of each block stamps the shader clock (s_memtime) and the 100 MHz real-time
// counter at kernel entry (record words 0, 1) and exit (words 6, 7), and optionally the shader clock at phase
// boundaries (ICA_STAMP_AT(k), words 2..5) and per wave (ICA_STAMP_WAVE, words 8..15), into a buffer of its own
// (ica_diag_stamp_buffer): 16 words per block,
// slot = linear block id.  clock = d(memtime) / d(memrealtime) * 100 MHz (MI355X_MICROARCH.md, DVFS give-back
// item 6).  No output element reads or depends on a stamp.
#ifdef ICA_CLOCK_STAMP
__device__ unsigned long long* ica_stamp_buf;   // one definition per translation unit built with the flag
__device__ unsigned ica_stamp_slots;
ICA_DEV void ica_stamp_put(int w, unsigned long long v, bool any_wave = false) {   // lane 0: one vector store
  const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  if ((any_wave ? (threadIdx.x & 63) : threadIdx.x) == 0 && ica_stamp_buf && b < ica_stamp_slots) {
    unsigned long long vv = v;
    asm volatile("" : "+v"(vv));
    ica_stamp_buf[(size_t)b * 16 + w] = vv;
  }
}
#define ICA_STAMP_BEGIN()                                                  \
  const unsigned long long ica_t0_ = __builtin_amdgcn_s_memtime();         \
  const unsigned long long ica_r0_ = __builtin_amdgcn_s_memrealtime()
#define ICA_STAMP_AT(k) ica_stamp_put(2 + (k), __builtin_amdgcn_s_memtime())
// every wave (up to 8) stamps word 8 + wave: e.g. where each wave's main loop ends
#define ICA_STAMP_WAVE() ica_stamp_put(8 + (int)(threadIdx.x >> 6), __builtin_amdgcn_s_memtime(), true)
#define ICA_STAMP_END()                                                      \
  do {                                                                       \
    const unsigned long long ica_t1_ = __builtin_amdgcn_s_memtime();         \
    const unsigned long long ica_r1_ = __builtin_amdgcn_s_memrealtime();     \
    ica_stamp_put(0, ica_t0_);                                               \
    ica_stamp_put(1, ica_r0_);                                               \
    ica_stamp_put(6, ica_t1_);                                               \
    ica_stamp_put(7, ica_r1_);                                               \
  } while (0)
#else
#define ICA_STAMP_BEGIN() ((void)0)
#define ICA_STAMP_AT(k) ((void)0)
#define ICA_STAMP_WAVE() ((void)0)
#define ICA_STAMP_END() ((void)0)
#endif

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

// fp8 (OCP e4m3) operands of the forward convolutions (BASELINE.json configs[4]
// "Wide U-Net fp8 MFMA im2col-GEMM conv").
//
// Per-tensor power-of-two scaling with a delayed amax (the scale of step t
// comes from the amax measured while quantizing step t-1, with 2x headroom):
//   q = sat_448(v * 2^e),  e = the largest integer with 2 * amax * 2^e <= 448,
// so dequantization is exact (x = q * 2^-e) and is done by the MFMA itself:
// v_mfma_scale_f32_16x16x128_f8f6f4 takes e8m0 block scales, code = 127 - e.
// Each tensor has an F8State {amax of the previous step, amax accumulating
// this step, e8m0 code in use}.  A plan's first fp8 forward calibrates: an
// amax pass over the tensor fills `prev` before the quantizer reads it.  Every
// later forward starts with one f8_roll over all states (prev <- cur, cur <- 0;
// a tensor quantized in no step keeps its prev), so the sequence replays
// unchanged inside a HIP graph.
#include "common.h"
#include "kernels.h"

namespace unet {

__device__ __forceinline__ int f8_exponent(unsigned prev_bits) {
  const float amax = __uint_as_float(prev_bits);
  if (!(amax > 0.f) || !(amax < 3.0e38f)) return 0;
  int e = (int)floorf(log2f(224.f / amax));
  while (e > -120 && ldexpf(2.f * amax, e) > 448.f) --e;  // log2f rounding at exact powers
  return max(-120, min(120, e));
}

__device__ __forceinline__ float f8_sat(float v) { return fminf(fmaxf(v, -448.f), 448.f); }

// 4 floats -> 4 e4m3 bytes (round to nearest even; operands pre-saturated)
__device__ __forceinline__ unsigned f8_pack4(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(a), f8_sat(b), 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(c), f8_sat(d), w, true);
  return (unsigned)w;
}

__device__ __forceinline__ void f8_amax_commit(float m, unsigned* dst) {
  m = wave_max(m);
  __shared__ float part[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) part[wave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, part[w]);
    if (r > 0.f) atomicMax(dst, __float_as_uint(r));  // non-negative floats order as their bits
  }
}

__global__ void f8_roll_kernel(F8State* s, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F8State v = s[i];
  if (v.cur_bits) v.prev_bits = v.cur_bits;
  v.cur_bits = 0;
  s[i] = v;
}

// amax of a bf16 [npix][C] tensor (channel stride ld) into prev (calibration)
__global__ void __launch_bounds__(256) f8_amax_act_kernel(const bf16_t* x, int ld, int C, int64_t npix, F8State* s) {
  const int cpr = C >> 3;  // 8-channel units per pixel
  const int64_t units = npix * cpr;
  float m = 0.f;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < units; u += (int64_t)gridDim.x * blockDim.x) {
    const int64_t px = u / cpr;
    const int c = (int)(u - px * cpr) << 3;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + px * ld + c), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
  }
  f8_amax_commit(m, &s->prev_bits);
}

__global__ void __launch_bounds__(256) f8_amax_f32_kernel(const float* w, int64_t n, F8State* s) {
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(w[i]));
  f8_amax_commit(m, &s->prev_bits);
}

// q[px][c] = e4m3(x[px*ld + c] * 2^e), dense [npix][C]; 8 channels per thread
// iteration; this step's amax accumulates into cur (commit != 0; an eval
// forward quantizes with the scale in use and leaves the training amax alone)
__global__ void __launch_bounds__(256) f8_quant_act_kernel(const bf16_t* x, int ld, int C, int64_t npix,
                                                           uint8_t* q, F8State* s, int commit) {
  const int e = f8_exponent(s->prev_bits);
  if (blockIdx.x == 0 && threadIdx.x == 0) s->code = 127 - e;
  const unsigned cpr = (unsigned)C >> 3;
  const unsigned units = (unsigned)(npix * cpr);  // < 2^31 (launcher)
  float m = 0.f;
  for (unsigned u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const unsigned px = u / cpr;
    const unsigned c = (u - px * cpr) << 3;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(x + (size_t)px * ld + c), f);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m = fmaxf(m, fabsf(f[k]));
      f[k] = ldexpf(f[k], e);
    }
    uint2 o;
    o.x = f8_pack4(f[0], f[1], f[2], f[3]);
    o.y = f8_pack4(f[4], f[5], f[6], f[7]);
    *reinterpret_cast<uint2*>(q + (size_t)px * C + c) = o;
  }
  if (commit) f8_amax_commit(m, &s->cur_bits);  // kernel-uniform: the barrier inside is reached by all
}

// conv weights fp32 [Co][Ci][RS] -> e4m3 [Co][RS][Ci] (the forward pack layout
// of PK_CONV_FWD): one thread per (co, ci) reads its RS taps (a contiguous run;
// neighbouring threads' runs are adjacent) and writes one byte per tap
// (neighbouring threads: neighbouring bytes)
__global__ void __launch_bounds__(256) f8_pack_w_kernel(const float* w, int Co, int Ci, int RS, uint8_t* dst,
                                                        F8State* s, int commit) {
  const int e = f8_exponent(s->prev_bits);
  if (blockIdx.x == 0 && threadIdx.x == 0) s->code = 127 - e;
  const unsigned units = (unsigned)Co * Ci;
  float m = 0.f;
  for (unsigned u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const unsigned co = u / Ci, ci = u - co * Ci;
    const float* src = w + (size_t)u * RS;
    uint8_t* d = dst + (size_t)co * RS * Ci + ci;
    for (int t = 0; t < RS; ++t) {
      const float v = src[t];
      m = fmaxf(m, fabsf(v));
      d[(size_t)t * Ci] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f8_sat(ldexpf(v, e)), 0.f, 0, false) & 0xff);
    }
  }
  if (commit) f8_amax_commit(m, &s->cur_bits);
}

static int grid_for(int64_t units) {
  int64_t g = (units + 255) / 256;
  if (g > 2048) g = 2048;
  return (int)(g < 1 ? 1 : g);
}

hipError_t launch_f8_roll(F8State* s, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(f8_roll_kernel, dim3((n + 255) / 256), dim3(256), 0, st, s, n);
  return hipGetLastError();
}

hipError_t launch_f8_quant_act(const bf16_t* x, int ld, int C, int64_t npix, uint8_t* q, F8State* s, int calibrate,
                               hipStream_t st) {
  if (C % 16 || ld % 8 || npix * (C >> 3) >= 0x7fffffffLL) return hipErrorInvalidValue;
  const int g = grid_for(npix * (C >> 3));
  const int commit = calibrate & F8_FROZEN ? 0 : 1;
  if (calibrate & F8_CALIBRATE) {
    hipLaunchKernelGGL(f8_amax_act_kernel, dim3(g), dim3(256), 0, st, x, ld, C, npix, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(f8_quant_act_kernel, dim3(g), dim3(256), 0, st, x, ld, C, npix, q, s, commit);
  return hipGetLastError();
}

hipError_t launch_f8_pack_w(const float* w, int Co, int Ci, int R, int S, uint8_t* dst, F8State* s, int calibrate,
                            hipStream_t st) {
  if (Ci % 16) return hipErrorInvalidValue;
  const int64_t n = (int64_t)Co * Ci * R * S;
  if (n >= 0x7fffffffLL) return hipErrorInvalidValue;
  const int commit = calibrate & F8_FROZEN ? 0 : 1;
  if (calibrate & F8_CALIBRATE) {
    hipLaunchKernelGGL(f8_amax_f32_kernel, dim3(grid_for(n)), dim3(256), 0, st, w, n, s);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(f8_pack_w_kernel, dim3(grid_for((int64_t)Co * Ci)), dim3(256), 0, st, w, Co, Ci, R * S, dst, s, commit);
  return hipGetLastError();
}

}  // namespace unet

// Fused Adam (coupled L2 weight decay) over flat fp32 buffers — the optimizer the
// reference builds in train.py:331-335 (torch.optim.Adam(model.parameters(),
// lr, weight_decay)).  torch's foreach Adam on ROCm is ~300 small launches per
// step (≈2.1 ms at 24.3 M params); this is two launches: a one-thread prologue
// that advances the step counter and derives the bias corrections in fp64, and
// one HBM-bound streaming pass (28 B per parameter: param r/w, grad r, m r/w,
// v r/w).  Per element it follows torch/optim/adam.py `_single_tensor_adam`:
//   g  = grad + wd * p                      (grad.add(param, alpha=wd))
//   m  = m + (1 - b1) * (g - m)             (exp_avg.lerp_(g, 1 - b1))
//   v  = v * b2 + (1 - b2) * g * g          (mul_(b2).addcmul_(g, g, 1 - b2))
//   p  = p - step_size * m / (sqrt(v) / sqrt(bc2) + eps)
#include "common.h"

namespace unet {

// coef[0] = step (float, torch's state['step']); coef[1] = step_size; coef[2] = sqrt(bc2)
__global__ void adam_prologue_kernel(float* coef, float lr, float beta1, float beta2) {
  const float step = coef[0] + 1.f;
  coef[0] = step;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  coef[1] = (float)((double)lr / bc1);
  coef[2] = (float)sqrt(bc2);
}

struct AdamConst { float b1, b2, omb1, omb2, eps, wd; };

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamConst& k,
                                          float step_size, float bc2s) {
  if (k.wd != 0.f) g = g + k.wd * p;
  m = m + k.omb1 * (g - m);
  v = v * k.b2 + k.omb2 * (g * g);
  const float denom = __fsqrt_rn(v) / bc2s + k.eps;
  p = p - step_size * (m / denom);
}

template <bool VEC>
__global__ void __launch_bounds__(256) adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   const float* __restrict__ coef, AdamConst k) {
  const float step_size = coef[1], bc2s = coef[2];
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (VEC) {
    const int64_t n4 = n >> 2;
    float4* p4 = reinterpret_cast<float4*>(p);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    for (int64_t i = tid; i < n4; i += stride) {
      float4 pp = p4[i], gg = g4[i], mm = m4[i], vv = v4[i];
      adam_elem(pp.x, gg.x, mm.x, vv.x, k, step_size, bc2s);
      adam_elem(pp.y, gg.y, mm.y, vv.y, k, step_size, bc2s);
      adam_elem(pp.z, gg.z, mm.z, vv.z, k, step_size, bc2s);
      adam_elem(pp.w, gg.w, mm.w, vv.w, k, step_size, bc2s);
      p4[i] = pp; m4[i] = mm; v4[i] = vv;
    }
    for (int64_t i = (n4 << 2) + tid; i < n; i += stride) {
      float pp = p[i], mm = m[i], vv = v[i];
      adam_elem(pp, g[i], mm, vv, k, step_size, bc2s);
      p[i] = pp; m[i] = mm; v[i] = vv;
    }
  } else {
    for (int64_t i = tid; i < n; i += stride) {
      float pp = p[i], mm = m[i], vv = v[i];
      adam_elem(pp, g[i], mm, vv, k, step_size, bc2s);
      p[i] = pp; m[i] = mm; v[i] = vv;
    }
  }
}

hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float* coef, float lr,
                       float beta1, float beta2, float eps, float wd, int advance_step, hipStream_t st) {
  if (advance_step) hipLaunchKernelGGL(adam_prologue_kernel, dim3(1), dim3(1), 0, st, coef, lr, beta1, beta2);
  if (n <= 0) return hipGetLastError();
  const AdamConst k{beta1, beta2, 1.f - beta1, 1.f - beta2, eps, wd};
  const bool vec = ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0;
  const int64_t work = vec ? (n + 3) / 4 : n;
  // 8 resident 256-thread blocks per CU on 256 CUs; each thread streams a few float4s
  int64_t blocks = (work + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  if (vec)
    hipLaunchKernelGGL(adam_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, coef, k);
  else
    hipLaunchKernelGGL(adam_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, coef, k);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// bf16 gradient exchange (opt-in, ddp.enable_data_parallel(grad_dtype="bf16")):
// the bucket is rounded to bf16 (RNE) before the all-reduce, which halves the
// xGMI bytes, and widened back to fp32 (times `scale`, 1/world for a SUM
// collective) after it.  The reference all-reduces nothing (single process);
// torch DDP's bf16 compress hook is the semantics this mirrors.
// ---------------------------------------------------------------------------
template <bool VEC>
__global__ void __launch_bounds__(256) grad_to_bf16_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                           int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n8 = VEC ? n >> 3 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(src)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(src)[2 * i + 1];
    reinterpret_cast<uint4*>(dst)[i] =
        make_uint4(pack_bf2(a.x, a.y), pack_bf2(a.z, a.w), pack_bf2(b.x, b.y), pack_bf2(b.z, b.w));
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = f2bf(src[i]);
}

template <bool VEC>
__global__ void __launch_bounds__(256) grad_from_bf16_kernel(const bf16_t* __restrict__ src, float* __restrict__ dst,
                                                             int64_t n, float scale) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n8 = VEC ? n >> 3 : 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float f[8];
    unpack8(reinterpret_cast<const uint4*>(src)[i], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) f[k] *= scale;
    reinterpret_cast<float4*>(dst)[2 * i] = make_float4(f[0], f[1], f[2], f[3]);
    reinterpret_cast<float4*>(dst)[2 * i + 1] = make_float4(f[4], f[5], f[6], f[7]);
  }
  for (int64_t i = (n8 << 3) + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = bf2f(src[i]) * scale;
}

static unsigned stream_blocks(int64_t n) {
  int64_t b = (n / 8 + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

hipError_t launch_grad_to_bf16(const float* src, bf16_t* dst, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (((uintptr_t)src | (uintptr_t)dst) % 16 == 0)
    hipLaunchKernelGGL(grad_to_bf16_kernel<true>, dim3(stream_blocks(n)), dim3(256), 0, st, src, dst, n);
  else
    hipLaunchKernelGGL(grad_to_bf16_kernel<false>, dim3(stream_blocks(8 * n)), dim3(256), 0, st, src, dst, n);
  return hipGetLastError();
}

hipError_t launch_grad_from_bf16(const bf16_t* src, float* dst, int64_t n, float scale, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (((uintptr_t)src | (uintptr_t)dst) % 16 == 0)
    hipLaunchKernelGGL(grad_from_bf16_kernel<true>, dim3(stream_blocks(n)), dim3(256), 0, st, src, dst, n, scale);
  else
    hipLaunchKernelGGL(grad_from_bf16_kernel<false>, dim3(stream_blocks(8 * n)), dim3(256), 0, st, src, dst, n,
                       scale);
  return hipGetLastError();
}

}  // namespace unet

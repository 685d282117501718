// Shared device helpers for the gfx950 U-Net kernels (bf16 NHWC activations,
// fp32 accumulation, 64-wide wavefronts).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

using unet::bf16_t;  // raw bf16 storage
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// In-kernel phase timing (debug build, -DUNET_TIMING: `make timing` builds
// libunet_hip_timing.so): thread 0 of block b < kTimBlocks writes the shader
// clock (s_memtime) of phase k to T[b * kTimSlots + k] of its launch's slot of a
// debug buffer that nothing else reads.  Compiled out of the product library.
using unet::kTimBlocks;
using unet::kTimSlots;
#ifdef UNET_TIMING
#define TSTAMP(T, k)                                                                      \
  do {                                                                                    \
    if ((T) && threadIdx.x == 0 && blockIdx.x < (unsigned)kTimBlocks)                     \
      (T)[blockIdx.x * kTimSlots + (k)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
#define TSTAMP_RT(T, k)                                                                   \
  do {                                                                                    \
    if ((T) && threadIdx.x == 0 && blockIdx.x < (unsigned)kTimBlocks)                     \
      (T)[blockIdx.x * kTimSlots + (k)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
// the same from thread `th` (a wave other than wave 0)
#define TSTAMP_TH(T, k, th)                                                               \
  do {                                                                                    \
    if ((T) && threadIdx.x == (th) && blockIdx.x < (unsigned)kTimBlocks)                  \
      (T)[blockIdx.x * kTimSlots + (k)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)
#define TSTAMP_RT_TH(T, k, th)                                                            \
  do {                                                                                    \
    if ((T) && threadIdx.x == (th) && blockIdx.x < (unsigned)kTimBlocks)                  \
      (T)[blockIdx.x * kTimSlots + (k)] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#else
#define TSTAMP(T, k) ((void)0)
#define TSTAMP_RT(T, k) ((void)0)
#define TSTAMP_TH(T, k, th) ((void)0)
#define TSTAMP_RT_TH(T, k, th) ((void)0)
#endif

// Phase ablation (debug builds only, `make abl`: -DUNET_TIMING -DUNET_ABL=n):
// 1 = the halo conv / weight-gradient kernels skip their MFMA work, 2 = they
// stage only the pipeline's first stages (later stages compute on stale LDS).
// Outputs are garbage; only the phase stamps mean anything.
#ifndef UNET_ABL
#define UNET_ABL 0
#endif

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}
// round-to-nearest-even, NaN preserving (v_cvt_pk_bf16_f32)
__device__ __forceinline__ bf16_t f2bf(float f) {
  return __builtin_bit_cast(bf16_t, (__bf16)f);
}
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
}
__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16); f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16); f[7] = __uint_as_float(u.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]),
                    pack_bf2(f[6], f[7]));
}

// ---- LDS-DMA staging (buffer_load ... lds): lane l of one wave instruction
// writes 16 B at lds_wave_base + 16*l; an offset >= num_records (kOOB) reads
// as zeros (conv padding, tile tails) ----
constexpr unsigned kOOB = 0x80000000u;

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, 0,
                                           0, 0);
}

// same, with a wave-uniform byte offset added to voff after the range check
// (raw buffer: soffset is not part of the num_records test), so a kOOB lane
// stays zero-filled whatever the stage offset
__device__ __forceinline__ void glds16s(__amdgpu_buffer_rsrc_t r, char* lds_wave_base, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff,
                                           0, 0);
}

// The same LDS-DMA as an inline-asm statement (cdna_hip_programming.md "What
// hipcc does not do" / LDS-DMA recipe: M0 written and restored in the same
// statement).  hipcc's waitcnt pass then never sees an LDS write on the VM
// counter, so it cannot insert the s_waitcnt vmcnt(0) it otherwise puts in
// front of the first ds_read_b64_tr_b16 of every k-step (draining the whole
// multi-stage pipeline); the kernel counts its DMA completions itself.
typedef int i32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4 make_rsrc_sgpr(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;  // make_rsrc's V#: base, stride 0, num_records, flags
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)p);
  r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ void glds16_asm(const i32x4& r, char* lds_wave_base, unsigned voff, unsigned soff) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(char, lds_wave_base));
  const unsigned so = __builtin_amdgcn_readfirstlane(soff);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(lds), "s"(so)
      : "memory");
}

// the same with the LDS destination as a byte address (lds_addr(smem) + an
// integer offset): no generic-pointer round trip, whose folded form
// (readfirstlane of a flat pointer cast back to LDS) hit an instruction-selection
// error in conv3x3_ws2_kernel
__device__ __forceinline__ unsigned lds_addr(const char* p) { return (unsigned)(size_t)LDS_PTR(const char, p); }
__device__ __forceinline__ void glds16_asm_at(const i32x4& r, unsigned lds_byte, unsigned voff, unsigned soff) {
  const unsigned lds = __builtin_amdgcn_readfirstlane(lds_byte);
  const unsigned so = __builtin_amdgcn_readfirstlane(soff);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %4 offen lds\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(r), "s"(lds), "s"(so)
      : "memory");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that the dispatcher deals to one XCD get consecutive ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// Last-arriver election across the blocks of one launch
// (cdna_hip_programming.md §6 Guideline 16, counter form): every wave drains
// its own atomics/stores, one lane releases at agent scope and takes a ticket;
// the block that draws total-1 acquires and may read everybody's results.
// `flag` must be a word of the DYNAMIC LDS region (no second __shared__ object
// beside an LDS-DMA staging array: §5 trap 4(a)).
// The published data are device-scope fp64 atomic adds, which execute at the
// memory side ("8-B agent atomics both sides", MI355X_MICROARCH.md Valid
// forms): the waves that issued them only drain their own vmcnt — no L2
// write-back release fence per block.
__device__ __forceinline__ bool last_block_arrive(unsigned* ticket, unsigned total, int* flag,
                                                  bool issued_atomics) {
  if (issued_atomics) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == total - 1 ? 1 : 0;
  }
  __syncthreads();
  const bool last = *flag != 0;
  if (last) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
  return last;
}

// BatchNorm per-channel statistics are fp64 sums (sum, sumsq) so that
// var = E[y^2]-mean^2 does not cancel: stats[0..C) = sum, stats[C..2C) = sumsq.
// Per-channel affine form of BN: y_hat*gamma+beta == y*scale + shift.
__device__ __forceinline__ void bn_scale_shift(const unet::BnLaunch& p, int c, float& scale,
                                               float& shift, float& mean_out, float& invstd_out,
                                               float& var_out) {
  float mean, var;
  if (p.training) {
    double s = 0.0, q = 0.0;
#pragma unroll
    for (int r = 0; r < unet::kStatRep; ++r) {
      s += p.stats[(size_t)r * 2 * p.C + c];
      q += p.stats[(size_t)r * 2 * p.C + p.C + c];
    }
    const double m = s / p.count;
    double v = q / p.count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
  } else {
    mean = p.run_mean[c];
    var = p.run_var[c];
  }
  const float inv = 1.0f / sqrtf(var + p.eps);
  scale = p.gamma[c] * inv;
  shift = p.beta[c] - mean * scale;
  mean_out = mean;
  invstd_out = inv;
  var_out = var;
}

// Training-mode finalisation of one BN layer (run by ONE block): scale/shift
// for the consumers, batch mean/invstd for the backward, running stats with
// momentum and the unbiased variance (torch.nn.BatchNorm2d semantics).
__device__ __forceinline__ void bn_finalize(const unet::BnLaunch& p) {
  for (int c = threadIdx.x; c < p.C; c += blockDim.x) {
    float sc, sh, m, inv, var;
    bn_scale_shift(p, c, sc, sh, m, inv, var);
    if (p.ss) {
      p.ss[c] = sc;
      p.ss[p.C + c] = sh;
    }
    if (p.training) {
      p.save_mean[c] = m;
      p.save_invstd[c] = inv;
      const double n = p.count;
      const float unb = (float)((double)var * (n / (n > 1.0 ? n - 1.0 : 1.0)));
      p.run_mean[c] = (1.f - p.momentum) * p.run_mean[c] + p.momentum * m;
      p.run_var[c] = (1.f - p.momentum) * p.run_var[c] + p.momentum * unb;
      if (c == 0 && p.nbt) *p.nbt += 1;  // exactly once per training forward, like the running stats
    }
  }
}

// Per-channel BN-backward apply coefficients from the replica sums:
// dY = A dZ + B y + C, A = k1 = gamma invstd, B = -k1 invstd m2,
// C = k1 (invstd m2 mu - m1), m1 = mean dZ, m2 = mean dZ xhat.  Shared by
// bn_bwd_apply_kernel (both coefficient sources: replica sums, or the
// finalised k1 / m1 / m2 of a ticket), the BN-fused weight gradients and the
// stem's fused apply (side products must be bit-identical to the apply
// pass): no contraction, fixed order (bn_bwd_coef_abc).
__device__ __forceinline__ void bn_bwd_coef_abc(float k1, float m1, float m2, float is, float mu, float& A, float& B,
                                                float& C) {
  // explicit round-to-nearest operations: no context-dependent contraction
  A = k1;
  B = __fmul_rn(__fmul_rn(-k1, is), m2);
  C = __fmul_rn(k1, __fsub_rn(__fmul_rn(__fmul_rn(is, m2), mu), m1));
}
__device__ __forceinline__ void bn_bwd_apply_coef(const unet::BnBwdArgs& a, int ch, double inv_n, float& A,
                                                  float& B, float& C, double& s1, double& s2) {
#pragma clang fp contract(off)
  s1 = 0.0;
  s2 = 0.0;
  for (int r = 0; r < unet::kStatRep; ++r) {
    const size_t rep = (size_t)r * 2 * a.C;
    s1 += a.sums[rep + ch];
    s2 += a.sums[rep + a.C + ch];
  }
  const float k1 = __fmul_rn(a.gamma[ch], a.invstd[ch]);
  const float m1 = (float)__dmul_rn(s1, inv_n), m2 = (float)__dmul_rn(s2, inv_n);
  bn_bwd_coef_abc(k1, m1, m2, a.invstd[ch], a.mean[ch], A, B, C);
}

// Last block of a BN-backward reduction (bn_bwd_reduce_kernel or a fused
// conv-dgrad epilogue): per-channel coefficients of the apply pass and the
// parameter gradients dgamma = sum dZ*xhat, dbeta = sum dZ.
__device__ __forceinline__ void bn_bwd_finalize(const unet::BnBwdArgs& a) {
  const bool two = a.y2 != nullptr;
  const double inv_n = 1.0 / (double)a.npix;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    double s1 = 0.0, s2 = 0.0, t2 = 0.0;
    for (int r = 0; r < unet::kStatRep; ++r) {
      const size_t rep = (size_t)r * 2 * a.C;
      s1 += a.sums[rep + c];
      s2 += a.sums[rep + a.C + c];
      if (two) t2 += a.sums2[rep + a.C + c];
    }
    a.coef[c] = a.gamma[c] * a.invstd[c];
    a.coef[a.C + c] = (float)(s1 * inv_n);
    a.coef[2 * a.C + c] = (float)(s2 * inv_n);
    a.dgamma[c] = (float)s2;
    a.dbeta[c] = (float)s1;
    if (two) {
      a.coef[3 * a.C + c] = a.gamma2[c] * a.invstd2[c];
      a.coef[4 * a.C + c] = (float)(t2 * inv_n);
      a.dgamma2[c] = (float)t2;
      a.dbeta2[c] = (float)s1;  // same dZ feeds both BNs
    }
  }
}

// dW index of element e of slab unit u (SlabLayout), -1 if that accumulator
// lane holds no dW element (tile tails, the idle half of a CO32 block)
__device__ __forceinline__ long long slab_dw_index(const unet::SlabLayout& L, long long u, int e) {
  const int lane = (int)(u & 63);
  long long r = u >> 6;
  const int frag = (int)(r % L.nf);
  r /= L.nf;
  const int wave = (int)(r % L.nw);
  const int blk = (int)(r / L.nw);
  const int g = lane >> 4, li = lane & 15;
  if (L.kind == unet::SLAB_HALO) {
    // CO32 slabs hold only the wm = 0 waves (wave slot = wn)
    const int t = frag >> 1, i = frag & 1, wm = L.co32 ? 0 : (wave & 1), wn = L.co32 ? wave : (wave >> 1);
    const int cob = blk % L.co_blocks, cib = blk / L.co_blocks;
    if (frag >= 18) {  // folded downsample: dW2 [Cout][C]
      const int co = cob * 64 + wm * 32 + i * 16 + 4 * g + e;
      if (co >= L.Cout) return -1;
      return L.dw2_off + (long long)co * L.C + cib * L.ci + wn * 16 + li;
    }
    const int co = cob * (L.co32 ? 32 : 64) + (L.co32 ? 0 : wm * 32) + i * 16 + 4 * g + e;
    const int c = cib * L.ci + wn * 16 + li;
    if (co >= L.Cout) return -1;
    return (long long)co * L.Krow + t * L.C + c;
  }
  if (L.kind == unet::SLAB_GEMM) {
    const int i = frag / L.fn, j = frag % L.fn;
    const int wm = wave % L.wm, wn = wave / L.wm;
    const int cob = blk % L.co_blocks, rest = blk / L.co_blocks;
    const int cblk = rest % L.c_blocks, tap = rest / L.c_blocks;
    const int co = cob * L.bmo + wm * (L.bmo / L.wm) + i * 16 + 4 * g + e;
    const int c = cblk * L.bnc + wn * (L.bnc / L.wn) + j * 16 + li;
    if (c >= L.cmax || co >= L.Cout) return -1;
    return (long long)co * L.Krow + (long long)tap * L.C + c;
  }
  // SLAB_STEM: one block per (split, 64-channel group blk), 4 waves of 32 co x 32 k
  const int i = frag >> 1, j = frag & 1, wm = wave & 1, wn = wave >> 1;
  return (long long)(blk * 64 + wm * 32 + i * 16 + 4 * g + e) * 64 + wn * 32 + j * 16 + li;
}

// dW = sum over the splits of the slab, bit-reproducible: a block covers
// 256/T consecutive units x T split lanes (lane-major over units, so every wave
// instruction reads whole runs of 16-B units); split lane r sums splits r, r+T,
// r+2T, ... in that order (eight loads in flight), then the T partials are
// added in r order through LDS.  The partition and both orders are fixed, so
// the result does not depend on timing.  Every dW element is written once.
__device__ __forceinline__ void slab_reduce_block(const f32x4* __restrict__ slab, float* __restrict__ dw,
                                                  const unet::SlabLayout& L, int T, int blk, f32x4* part) {
  const int tid = threadIdx.x;
  const int per = 256 / T;
  const int ul = tid % per, r = tid / per;
  const long long u = (long long)blk * per + ul;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (u < L.units) {
    int k = r;
    for (; k + 7 * T < L.splits; k += 8 * T) {
      f32x4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = slab[(long long)(k + q * T) * L.units + u];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc += v[q];
    }
    for (; k < L.splits; k += T) acc += slab[(long long)k * L.units + u];
  }
  part[tid] = acc;
  __syncthreads();
  if (r != 0 || u >= L.units) return;
  for (int j = 1; j < T; ++j) acc += part[j * per + ul];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const long long idx = slab_dw_index(L, u, e);
    if (idx >= 0) dw[idx] = acc[e];
  }
}

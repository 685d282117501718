// HBM-bound kernels of the U-Net hot path (gfx950): BatchNorm apply / backward,
// residual add + ReLU, maxpool 3/2/1, the fused upconv0+conv_final head, the
// pixel-wise BCE/Dice loss + mask metrics, and weight (un)packing.
//
// Every activation access is 16 B per lane (8 bf16 channels, NHWC) so one
// wave instruction moves 1 KiB; per-channel reductions are kept in registers
// per thread (each thread owns one 8-channel chunk for its whole pixel loop),
// folded through LDS once per block and published with fp64 atomics.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace unet {

constexpr float kMaskThreshold = 8.94069742685133e-08f;  // 0x33C00001, SURVEY.md §0

// grid cap of the BN apply kernels (each block recomputes the per-channel
// coefficients in its prologue; fewer, longer blocks amortise that and keep
// the next pass's loads in flight).  256 = 1 block per CU: since split-K
// reductions ride as trailing blocks of the backward apply, the smaller apply
// grid leaves the other CU slots to them (A/B on one box: bn_bwd 0.85 -> 0.81
// ms, 2445 -> 2466 img/s; 128 and 192 were slower, 512 was best before the
// reductions were merged)
static int g_apply_cap = std::getenv("UNET_APPLY_CAP") ? std::atoi(std::getenv("UNET_APPLY_CAP")) : 256;

static inline int grid_for(int64_t work, int per_block, int cap = 2048) {
  int64_t g = (work + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---------------------------------------------------------------------------
// BN apply (+ residual) (+ ReLU), forward.  Block 0 also finalises the batch
// statistics: save_mean/save_invstd for the backward and the running stats
// (momentum 0.1, unbiased variance), matching torch.nn.BatchNorm2d training.
// ---------------------------------------------------------------------------
__device__ void bn_finalize_block0(const BnLaunch& p, int tid, int nthreads, int cbeg, int cend) {
  for (int c = cbeg + tid; c < cend; c += nthreads) {
    float sc, sh, m, inv, var;
    bn_scale_shift(p, c, sc, sh, m, inv, var);
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

// Thread layout of the per-channel BN kernels: a block covers one group of
// CG channels (blockIdx.y; CG = 64 when C % 64 == 0, else C) so its
// coefficient prologue reads CG channels' replica sums, not C; inside the
// group chunk = tid % CC (8 channels = one 16-B access), row = tid / CC, and a
// thread keeps its chunk for the whole grid-stride pixel loop (coefficients in
// registers).  kBnPPT pixels per thread per pass; the first pass's loads are
// issued BEFORE the coefficient prologue so the two latencies overlap.
constexpr int kBnCG = 64;
#ifndef UNET_BN_PPT
#define UNET_BN_PPT 2
#endif
constexpr int kBnPPT = UNET_BN_PPT;  // (variant builds: make variant VDEF=-DUNET_BN_PPT=n)
__host__ __device__ __forceinline__ int bn_group(int C) { return C % kBnCG == 0 ? kBnCG : C; }

template <int RES, bool RELU>
__global__ void __launch_bounds__(256) bn_apply_kernel(BnApplyArgs a) {
  const int CG = bn_group(a.C);
  const int CC = CG >> 3;
  const int rows = blockDim.x / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int cg0 = blockIdx.y * CG;
  const int c8 = cg0 + (chunk << 3);
  constexpr int PPT = kBnPPT;
  const int64_t stride = (int64_t)gridDim.x * rows;
  uint4 uy[PPT], ur[PPT];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int64_t pix = base + u * stride;
      uy[u] = pix < a.npix ? *reinterpret_cast<const uint4*>(a.y + pix * a.ldy + c8) : make_uint4(0, 0, 0, 0);
      if constexpr (RES != 0)
        ur[u] = pix < a.npix ? *reinterpret_cast<const uint4*>(a.res + pix * a.ldr + c8) : make_uint4(0, 0, 0, 0);
    }
  };
  int64_t base = (int64_t)blockIdx.x * rows + row;
  if (row < rows) load(base);
  // per-channel affine coefficients of the group into LDS, then 8 per thread
  // into registers
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [4][CG]
  for (int c = threadIdx.x; c < CG; c += blockDim.x) {
    const int ch = cg0 + c;
    float m, inv, var;
    if (a.bn.training && a.bn.ss) {  // finalised by the producing conv's last block
      coef[c] = a.bn.ss[ch];
      coef[CG + c] = a.bn.ss[a.C + ch];
    } else {
      bn_scale_shift(a.bn, ch, coef[c], coef[CG + c], m, inv, var);
    }
    if (RES == 2) {
      if (a.bn2.training && a.bn2.ss) {
        coef[2 * CG + c] = a.bn2.ss[ch];
        coef[3 * CG + c] = a.bn2.ss[a.C + ch];
      } else {
        bn_scale_shift(a.bn2, ch, coef[2 * CG + c], coef[3 * CG + c], m, inv, var);
      }
    }
  }
  __syncthreads();
  float sc1[8], sh1[8], sc2[RES == 2 ? 8 : 1], sh2[RES == 2 ? 8 : 1];
  const int l8 = chunk << 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sc1[k] = coef[l8 + k];
    sh1[k] = coef[CG + l8 + k];
    if constexpr (RES == 2) {
      sc2[k] = coef[2 * CG + l8 + k];
      sh2[k] = coef[3 * CG + l8 + k];
    }
  }
  if (row < rows) {
    for (; base < a.npix; base += PPT * stride) {
      // this pass's operands; the next pass's loads go out before the math
      uint4 cy[PPT], cr[PPT];
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        cy[u] = uy[u];
        if constexpr (RES != 0) cr[u] = ur[u];
      }
      if (base + PPT * stride < a.npix) load(base + PPT * stride);
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int64_t pix = base + u * stride;
        if (pix >= a.npix) break;
        float v[8];
        unpack8(cy[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * sc1[k] + sh1[k];
        if constexpr (RES != 0) {
          float r[8];
          unpack8(cr[u], r);
          if constexpr (RES == 2) {
#pragma unroll
            for (int k = 0; k < 8; ++k) r[k] = r[k] * sc2[k] + sh2[k];
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += r[k];
        }
        if constexpr (RELU) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
        }
        *reinterpret_cast<uint4*>(a.out + pix * a.ldo + c8) = pack8(v);
      }
    }
  }
  // standalone use (no producer finalised the stats): block (0, g) finalises
  // its channel group
  if (blockIdx.x == 0) {
    if (!a.bn.ss) bn_finalize_block0(a.bn, threadIdx.x, blockDim.x, cg0, cg0 + CG);
    if (RES == 2 && !a.bn2.ss) bn_finalize_block0(a.bn2, threadIdx.x, blockDim.x, cg0, cg0 + CG);
  }
}

static inline dim3 chunk_block(int C) {
  const int CC = C / 8;
  return dim3((256 / CC) * CC);
}

// grid of the grouped BN kernels: x = pixel blocks (kBnPPT pixels per thread
// per pass, capped so that x * groups <= g_apply_cap), y = channel groups
static inline dim3 bn_grid(int64_t npix, int C) {
  const int CG = bn_group(C), groups = C / CG;
  const int rows = 256 / (CG / 8);
  const int cap = g_apply_cap / groups > 0 ? g_apply_cap / groups : 1;
  return dim3(grid_for(npix, rows * kBnPPT, cap), groups);
}

static inline bool bn_group_ok(int C) {
  return C % 8 == 0 && bn_group(C) / 8 <= 256;  // rows = 256 / CC, threads past rows*CC idle
}

hipError_t launch_bn_apply(const BnApplyArgs& a, hipStream_t st) {
  if (!bn_group_ok(a.C)) return hipErrorInvalidValue;
  const dim3 g = bn_grid(a.npix, a.C), b = chunk_block(bn_group(a.C));
  const size_t lds = 4 * bn_group(a.C) * sizeof(float);
  switch (a.res_mode * 2 + (a.relu ? 1 : 0)) {
    case 0: hipLaunchKernelGGL((bn_apply_kernel<0, false>), g, b, lds, st, a); break;
    case 1: hipLaunchKernelGGL((bn_apply_kernel<0, true>), g, b, lds, st, a); break;
    case 2: hipLaunchKernelGGL((bn_apply_kernel<1, false>), g, b, lds, st, a); break;
    case 3: hipLaunchKernelGGL((bn_apply_kernel<1, true>), g, b, lds, st, a); break;
    case 4: hipLaunchKernelGGL((bn_apply_kernel<2, false>), g, b, lds, st, a); break;
    case 5: hipLaunchKernelGGL((bn_apply_kernel<2, true>), g, b, lds, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// BN backward.  Thread layout: chunk = tid % CC (8 channels), row = tid / CC;
// each thread keeps its channel sums in registers over its pixel stride.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_dz(const BnBwdArgs& a, int64_t pix, int c8, float* dz) {
  unpack8(*reinterpret_cast<const uint4*>(a.da + pix * a.ldda + c8), dz);
  if (a.relu) {
    float av[8];
    unpack8(*reinterpret_cast<const uint4*>(a.act + pix * a.ldact + c8), av);
#pragma unroll
    for (int k = 0; k < 8; ++k) dz[k] = av[k] > 0.f ? dz[k] : 0.f;
  }
}

__global__ void __launch_bounds__(256) bn_bwd_reduce_kernel(BnBwdArgs a) {
  const int CC = a.C >> 3;
  const int rows = blockDim.x / CC;
  const int chunk = threadIdx.x % CC;
  const int row = threadIdx.x / CC;
  const int c8 = chunk << 3;
  const bool two = a.y2 != nullptr;
  float s1[8], s2[8], t2[8];
  float mu[8], is[8], mu2[8], is2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[k] = s2[k] = t2[k] = 0.f;
    mu[k] = a.mean[c8 + k]; is[k] = a.invstd[c8 + k];
    mu2[k] = two ? a.mean2[c8 + k] : 0.f; is2[k] = two ? a.invstd2[c8 + k] : 0.f;
  }
  constexpr int PPT = 4;
  if (row < rows) {
    const int64_t stride = (int64_t)gridDim.x * rows;
    for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.npix; base += PPT * stride) {
      uint4 uda[PPT], uact[PPT], uy[PPT], uy2[PPT];
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int64_t pix = base + u * stride;
        const bool in = pix < a.npix;
        const uint4 z = make_uint4(0, 0, 0, 0);
        uda[u] = in ? *reinterpret_cast<const uint4*>(a.da + pix * a.ldda + c8) : z;
        uact[u] = (in && a.relu) ? *reinterpret_cast<const uint4*>(a.act + pix * a.ldact + c8) : z;
        uy[u] = in ? *reinterpret_cast<const uint4*>(a.y + pix * a.ldy + c8) : z;
        uy2[u] = (in && two) ? *reinterpret_cast<const uint4*>(a.y2 + pix * a.ldy2 + c8) : z;
      }
#pragma unroll
      for (int u = 0; u < PPT; ++u) {  // out-of-range pixels load zeros: dz = 0 adds nothing
        float dz[8], y[8];
        unpack8(uda[u], dz);
        if (a.relu) {
          float av[8];
          unpack8(uact[u], av);
#pragma unroll
          for (int k = 0; k < 8; ++k) dz[k] = av[k] > 0.f ? dz[k] : 0.f;
        }
        unpack8(uy[u], y);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += dz[k]; s2[k] += dz[k] * (y[k] - mu[k]) * is[k]; }
        if (two) {
          unpack8(uy2[u], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) t2[k] += dz[k] * (y[k] - mu2[k]) * is2[k];
        }
      }
    }
  }
  // fold rows through LDS: red[row][C]
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int nsum = two ? 3 : 2;
  for (int q = 0; q < nsum; ++q) {
    const float* src = q == 0 ? s1 : (q == 1 ? s2 : t2);
    if (row < rows) {
#pragma unroll
      for (int k = 0; k < 8; ++k) red[row * a.C + c8 + k] = src[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      float acc = 0.f;
      for (int r = 0; r < rows; ++r) acc += red[r * a.C + c];
      const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.C;
      double* dst = q == 0 ? a.sums + rep : (q == 1 ? a.sums + rep + a.C : a.sums2 + rep + a.C);
      atomicAdd(dst + c, (double)acc);
    }
    __syncthreads();
  }
  if (a.ticket && last_block_arrive(a.ticket, gridDim.x, reinterpret_cast<int*>(red), true)) bn_bwd_finalize(a);
}

hipError_t launch_bn_bwd_reduce(const BnBwdArgs& a, hipStream_t st) {
  if (a.C % 8 || a.C / 8 > 256) return hipErrorInvalidValue;
  const int CC = a.C / 8;
  const int rows = 256 / CC;
  // <= 2048 blocks (fp64 atomics spread over kStatRep replicas), 8 pixels per thread
  const int g = grid_for(a.npix, rows * 8, 2048);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(g), chunk_block(a.C), (size_t)rows * a.C * sizeof(float), st, a);
  return hipGetLastError();
}

// dY = k1 (dZ - mean dZ - xhat mean(dZ xhat)), xhat = (y - mu) invstd, folded
// per channel into dY = A dZ + B y + Cc (A = k1, B = -k1 invstd m2,
// Cc = k1 (invstd m2 mu - m1)): 3 coefficients (6 with TWO) per channel in
// registers.  RELU: dZ = dA * (act > 0) (unfused path; the fused producers
// store dZ itself).  Blocks grid-stride over passes of kBnPPT pixels per
// thread with the next pass's loads issued before the current pass's math.
// RED: a deferred split-K reduction (ReduceTail) rides as trailing blocks of a
// 1-D grid: flat block ids [0, gx * gy) are the apply's (bx, by), the rest
// reduce (256-thread blocks; the coefficient LDS doubles as the reduction's)
template <bool TWO, bool RELU, bool RED>
__global__ void __launch_bounds__(256) bn_bwd_apply_kernel(BnBwdArgs a, double inv_n, ReduceTail rt, int gxa,
                                                           int gya) {
  extern __shared__ __attribute__((aligned(16))) float coef[];  // [6][CG]
  int bx, by, gx;
  if constexpr (RED) {
    const int flat = blockIdx.x;
    if (flat >= gxa * gya) {
      slab_reduce_block(reinterpret_cast<const f32x4*>(rt.slab), rt.dw, rt.L, rt.T, flat - gxa * gya,
                        reinterpret_cast<f32x4*>(coef));
      return;
    }
    bx = flat % gxa; by = flat / gxa; gx = gxa;
  } else {
    bx = blockIdx.x; by = blockIdx.y; gx = gridDim.x;
  }
  const int CG = bn_group(a.C);
  const int CC = CG >> 3;
  const int rows = blockDim.x / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int cg0 = by * CG;
  const int c8 = cg0 + (chunk << 3);
  constexpr int PPT = kBnPPT;
  const int64_t stride = (int64_t)gx * rows;
  uint4 uda[PPT], uact[PPT], uy[PPT], uy2[PPT];
  auto load = [&](int64_t base) {
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int64_t pix = base + u * stride;
      const bool in = pix < a.npix;
      const uint4 z = make_uint4(0, 0, 0, 0);
      uda[u] = in ? *reinterpret_cast<const uint4*>(a.da + pix * a.ldda + c8) : z;
      if constexpr (RELU) uact[u] = in ? *reinterpret_cast<const uint4*>(a.act + pix * a.ldact + c8) : z;
      uy[u] = in ? *reinterpret_cast<const uint4*>(a.y + pix * a.ldy + c8) : z;
      if constexpr (TWO) uy2[u] = in ? *reinterpret_cast<const uint4*>(a.y2 + pix * a.ldy2 + c8) : z;
    }
  };
  int64_t base = (int64_t)bx * rows + row;
  if (row < rows) load(base);  // first pass in flight during the prologue
  for (int c = threadIdx.x; c < CG; c += blockDim.x) {
    const int ch = cg0 + c;
    float k1, m1, m2, k1b = 0.f, m2b = 0.f;
    if (a.coef) {  // finalised by the reduce's (or fused producer's) last block
      k1 = a.coef[ch];
      m1 = a.coef[a.C + ch];
      m2 = a.coef[2 * a.C + ch];
      if (TWO) { k1b = a.coef[3 * a.C + ch]; m2b = a.coef[4 * a.C + ch]; }
    } else {
      double s1, s2, t2 = 0.0;
      float cA, cB, cC;
      bn_bwd_apply_coef(a, ch, inv_n, cA, cB, cC, s1, s2);
      if (TWO) {
        for (int r = 0; r < kStatRep; ++r) t2 += a.sums2[(size_t)r * 2 * a.C + a.C + ch];
        k1b = __fmul_rn(a.gamma2[ch], a.invstd2[ch]);
        m2b = (float)__dmul_rn(t2, inv_n);
      }
      if (bx == 0) {
        a.dgamma[ch] = (float)s2;
        a.dbeta[ch] = (float)s1;
        if (TWO) {
          a.dgamma2[ch] = (float)t2;
          a.dbeta2[ch] = (float)s1;  // same dZ feeds both BNs
        }
      }
      coef[c] = cA;
      coef[CG + c] = cB;
      coef[2 * CG + c] = cC;
      m1 = (float)__dmul_rn(s1, inv_n);
      if (TWO) {
        const float isb = a.invstd2[ch], mub = a.mean2[ch];
        bn_bwd_coef_abc(k1b, m1, m2b, isb, mub, coef[3 * CG + c], coef[4 * CG + c], coef[5 * CG + c]);
      }
      continue;
    }
    bn_bwd_coef_abc(k1, m1, m2, a.invstd[ch], a.mean[ch], coef[c], coef[CG + c], coef[2 * CG + c]);
    if (TWO) bn_bwd_coef_abc(k1b, m1, m2b, a.invstd2[ch], a.mean2[ch], coef[3 * CG + c], coef[4 * CG + c], coef[5 * CG + c]);
  }
  __syncthreads();
  float cA[8], cB[8], cC[8], dA[TWO ? 8 : 1], dB[TWO ? 8 : 1], dC[TWO ? 8 : 1];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = (chunk << 3) + k;
    cA[k] = coef[c];
    cB[k] = coef[CG + c];
    cC[k] = coef[2 * CG + c];
    if constexpr (TWO) {
      dA[k] = coef[3 * CG + c];
      dB[k] = coef[4 * CG + c];
      dC[k] = coef[5 * CG + c];
    }
  }
  if (row >= rows) return;
  for (; base < a.npix; base += PPT * stride) {
    uint4 cda[PPT], cact[PPT], cy[PPT], cy2[PPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      cda[u] = uda[u]; cy[u] = uy[u];
      if constexpr (RELU) cact[u] = uact[u];
      if constexpr (TWO) cy2[u] = uy2[u];
    }
    if (base + PPT * stride < a.npix) load(base + PPT * stride);
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int64_t pix = base + u * stride;
      if (pix >= a.npix) break;
      float dz[8], y[8], o[8];
      unpack8(cda[u], dz);
      if constexpr (RELU) {
        float av[8];
        unpack8(cact[u], av);
#pragma unroll
        for (int k = 0; k < 8; ++k) dz[k] = av[k] > 0.f ? dz[k] : 0.f;
      }
      unpack8(cy[u], y);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(cA[k], dz[k], fmaf(cB[k], y[k], cC[k]));
      *reinterpret_cast<uint4*>(a.dy + pix * a.lddy + c8) = pack8(o);
      if constexpr (TWO) {
        unpack8(cy2[u], y);
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = fmaf(dA[k], dz[k], fmaf(dB[k], y[k], dC[k]));
        *reinterpret_cast<uint4*>(a.dy2 + pix * a.lddy2 + c8) = pack8(o);
      }
      if (RELU && a.dres) *reinterpret_cast<uint4*>(a.dres + pix * a.lddres + c8) = pack8(dz);
    }
  }
}

hipError_t launch_bn_bwd_apply(const BnBwdArgs& a, hipStream_t st) {
  if (!bn_group_ok(a.C)) return hipErrorInvalidValue;
  if (!a.relu && a.dres) return hipErrorInvalidValue;  // dZ is dA itself: nothing to store
  const dim3 g = bn_grid(a.npix, a.C), b = chunk_block(bn_group(a.C));
  const size_t lds = 6 * bn_group(a.C) * sizeof(float);
  const double inv_n = 1.0 / (double)a.npix;
  const bool two = a.y2 != nullptr;
  const ReduceTail r = {};
  if (two && a.relu) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true, false>), g, b, lds, st, a, inv_n, r, 0, 0);
  else if (two) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, false>), g, b, lds, st, a, inv_n, r, 0, 0);
  else if (a.relu) hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true, false>), g, b, lds, st, a, inv_n, r, 0, 0);
  else hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false, false>), g, b, lds, st, a, inv_n, r, 0, 0);
  return hipGetLastError();
}

hipError_t launch_bn_bwd_apply_reduce(const BnBwdArgs& a, const ReduceTail& r, hipStream_t st) {
  if (!bn_group_ok(a.C)) return hipErrorInvalidValue;
  if (!a.relu && a.dres) return hipErrorInvalidValue;
  const dim3 g = bn_grid(a.npix, a.C), b = chunk_block(bn_group(a.C));
  if (b.x != 256 || r.blocks <= 0) return hipErrorNotSupported;  // the reduction's block shape
  const size_t lds = std::max<size_t>(6 * bn_group(a.C) * sizeof(float), 256 * 16);
  const double inv_n = 1.0 / (double)a.npix;
  const bool two = a.y2 != nullptr;
  const dim3 g1(g.x * g.y + r.blocks);
  if (two && a.relu) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, true, true>), g1, b, lds, st, a, inv_n, r, g.x, g.y);
  else if (two) hipLaunchKernelGGL((bn_bwd_apply_kernel<true, false, true>), g1, b, lds, st, a, inv_n, r, g.x, g.y);
  else if (a.relu) hipLaunchKernelGGL((bn_bwd_apply_kernel<false, true, true>), g1, b, lds, st, a, inv_n, r, g.x, g.y);
  else hipLaunchKernelGGL((bn_bwd_apply_kernel<false, false, true>), g1, b, lds, st, a, inv_n, r, g.x, g.y);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// MaxPool2d(3, 2, 1): torch CPU semantics — first maximum in (kh, kw) scan
// order wins (strict >), NaN propagates.  Index 0..8 kept as uint8.
//
// Both directions walk whole image rows: block b owns rows [b*rpb, (b+1)*rpb)
// of the output (forward) or input (backward) grid, and a thread keeps one
// 8-channel chunk (blockDim % CC == 0) while it strides over the row's
// pixels, so all address math is 32-bit with no per-element division chains;
// every tap's 16-B load is issued before any is consumed.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(MaxPoolArgs a, int rpb) {
  const int CC = a.C >> 3;
  const int chunk = threadIdx.x % CC;
  const int c8 = chunk << 3;
  const int per_row = a.Q * CC;
  const int nrows = a.N * a.P;
  for (int rr = 0; rr < rpb; ++rr) {
    const int orow = blockIdx.x * rpb + rr;
    if (orow >= nrows) break;
    const int n = orow / a.P, p = orow - n * a.P;
    const bf16_t* xrow[3];
    bool rok[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * p - 1 + kh;
      rok[kh] = ih >= 0 && ih < a.H;
      xrow[kh] = a.x + (size_t)(n * a.H + (rok[kh] ? ih : 0)) * a.W * a.ldx + c8;
    }
    for (int e = threadIdx.x; e < per_row; e += blockDim.x) {
      const int q = e / CC;
      uint4 u[9];
      bool ok[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int kh = t / 3, kw = t % 3;
        const int iw = 2 * q - 1 + kw;
        ok[t] = rok[kh] && iw >= 0 && iw < a.W;
        u[t] = ok[t] ? *reinterpret_cast<const uint4*>(xrow[kh] + (size_t)iw * a.ldx) : make_uint4(0, 0, 0, 0);
      }
      float best[8];
      int bi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = -1; }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
        float v[8];
        unpack8(u[t], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool take = bi[k] < 0 || v[k] > best[k] || (v[k] != v[k] && best[k] == best[k]);
          best[k] = take ? v[k] : best[k];
          bi[k] = take ? t : bi[k];
        }
      }
      const size_t opix = (size_t)orow * a.Q + q;
      *reinterpret_cast<uint4*>(a.y + opix * a.ldy + c8) = pack8(best);
      uint2 ix;
      ix.x = (unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16) | ((unsigned)bi[3] << 24);
      ix.y = (unsigned)bi[4] | ((unsigned)bi[5] << 8) | ((unsigned)bi[6] << 16) | ((unsigned)bi[7] << 24);
      *reinterpret_cast<uint2*>(a.idx + opix * a.C + c8) = ix;
    }
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(MaxPoolArgs a, int rpb) {
  const int CC = a.C >> 3;
  const int chunk = threadIdx.x % CC;
  const int c8 = chunk << 3;
  const BnBwdArgs& bb = a.bb;
  const bool fz = bb.sums != nullptr;  // launcher: 256 % CC == 0, so c8 is fixed per thread
  float s1[8], s2[8], mu[8], is[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[k] = s2[k] = 0.f;
    mu[k] = fz ? bb.mean[c8 + k] : 0.f;
    is[k] = fz ? bb.invstd[c8 + k] : 0.f;
  }
  const int per_row = a.W * CC;
  const int nrows = a.N * a.H;
  for (int rr = 0; rr < rpb; ++rr) {
    const int irow = blockIdx.x * rpb + rr;
    if (irow >= nrows) break;
    const int n = irow / a.H, h = irow - n * a.H;
    // output rows whose window covers h (2p-1 <= h <= 2p+1): p_lo and p_lo+1
    const int p_lo = h >= 1 ? h / 2 : 0;
    const int p_hi = min((h + 1) / 2, a.P - 1);
    for (int e = threadIdx.x; e < per_row; e += blockDim.x) {
      const int w = e / CC;
      const size_t ipix = (size_t)irow * a.W + w;
      const int q0 = w >= 1 ? w / 2 : 0;
      const int q1 = min((w + 1) / 2, a.Q - 1);
      uint2 ix[4];
      uint4 g[4];
      int want[4];
      bool ok[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = p_lo + (j >> 1);
        const int q = q0 + (j & 1);
        const int kh = h - (2 * p - 1), kw = w - (2 * q - 1);
        ok[j] = p <= p_hi && q <= q1 && kh >= 0 && kh <= 2 && kw >= 0 && kw <= 2;
        want[j] = kh * 3 + kw;
        const size_t opix = ((size_t)n * a.P + (ok[j] ? p : 0)) * a.Q + (ok[j] ? q : 0);
        ix[j] = ok[j] ? *reinterpret_cast<const uint2*>(a.idx + opix * a.C + c8) : make_uint2(0, 0);
        g[j] = ok[j] ? *reinterpret_cast<const uint4*>(a.dy + opix * a.lddy + c8) : make_uint4(0, 0, 0, 0);
      }
      uint4 addv = make_uint4(0, 0, 0, 0), actv = make_uint4(0, 0, 0, 0), yv = make_uint4(0, 0, 0, 0);
      if (a.add) addv = *reinterpret_cast<const uint4*>(a.add + ipix * a.ldadd + c8);
      if (fz) {
        actv = *reinterpret_cast<const uint4*>(bb.act + ipix * bb.ldact + c8);
        yv = *reinterpret_cast<const uint4*>(bb.y + ipix * bb.ldy + c8);
      }
      float acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (!ok[j]) continue;
        float gv[8];
        unpack8(g[j], gv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned word = k < 4 ? ix[j].x : ix[j].y;
          const int b = (word >> ((k & 3) * 8)) & 0xff;
          if (b == want[j]) acc[k] += gv[k];
        }
      }
      if (a.add) {
        float r[8];
        unpack8(addv, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += r[k];
      }
      if (fz) {
        float av[8];
        unpack8(actv, av);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = av[k] > 0.f ? acc[k] : 0.f;
      }
      const uint4 o = pack8(acc);
      *reinterpret_cast<uint4*>(a.dx + ipix * a.lddx + c8) = o;
      if (fz) {
        float dz[8], y[8];
        unpack8(o, dz);
        unpack8(yv, y);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += dz[k]; s2[k] += dz[k] * (y[k] - mu[k]) * is[k]; }
      }
    }
  }
  if (!fz) return;
  // fold the block's per-thread channel sums (thread t holds chunk t % CC)
  __shared__ float red[256 * 8];
  __shared__ int flag;
  for (int q = 0; q < 2; ++q) {
    const float* src = q == 0 ? s1 : s2;
#pragma unroll
    for (int k = 0; k < 8; ++k) red[threadIdx.x * 8 + k] = src[k];
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
      const int ch = c >> 3, k = c & 7;
      float acc = 0.f;
      for (int t = ch; t < (int)blockDim.x; t += CC) acc += red[t * 8 + k];
      const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.C;
      atomicAdd(bb.sums + rep + q * a.C + c, (double)acc);
    }
    __syncthreads();
  }
  if (bb.ticket && last_block_arrive(bb.ticket, gridDim.x, &flag, (int)threadIdx.x < a.C)) bn_bwd_finalize(bb);
}

// Stem forward tail in one pass: act = relu(bn(x)) (x = raw 7x7 conv output)
// and MaxPool2d(3,2,1) of act.  Pooled pixel (p, q) owns act pixels
// (2p + a, 2q + b), a, b in {0, 1} (H, W even), so every act pixel is written
// exactly once; the pooling compares the bf16-ROUNDED act values, exactly as
// the unfused maxpool reading act back from HBM would.  Replaces bn_apply +
// maxpool_fwd (act is read back 2.3x by the unfused pooling, PMC).
__global__ void __launch_bounds__(256) bn_relu_maxpool_fwd_kernel(MaxPoolArgs a, int rpb) {
  const int CC = a.C >> 3;
  const int chunk = threadIdx.x % CC;
  const int c8 = chunk << 3;
  const int per_row = a.Q * CC;
  const int nrows = a.N * a.P;
  __shared__ float coef[2][256];
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float m, inv, var;
    if (a.bn.training && a.bn.ss) { coef[0][c] = a.bn.ss[c]; coef[1][c] = a.bn.ss[a.C + c]; }
    else bn_scale_shift(a.bn, c, coef[0][c], coef[1][c], m, inv, var);
  }
  __syncthreads();
  float sc[8], sh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { sc[k] = coef[0][c8 + k]; sh[k] = coef[1][c8 + k]; }
  for (int rr = 0; rr < rpb; ++rr) {
    const int orow = blockIdx.x * rpb + rr;
    if (orow >= nrows) break;
    const int n = orow / a.P, p = orow - n * a.P;
    const bf16_t* xrow[3];
    bf16_t* arow[3];
    bool rok[3];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * p - 1 + kh;
      rok[kh] = ih >= 0 && ih < a.H;
      const size_t base = (size_t)(n * a.H + (rok[kh] ? ih : 0)) * a.W;
      xrow[kh] = a.x + base * a.ldx + c8;
      arow[kh] = a.act + base * a.ldact + c8;
    }
    for (int e = threadIdx.x; e < per_row; e += blockDim.x) {
      const int q = e / CC;
      uint4 u[9];
      bool ok[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int kh = t / 3, kw = t % 3;
        const int iw = 2 * q - 1 + kw;
        ok[t] = rok[kh] && iw >= 0 && iw < a.W;
        u[t] = ok[t] ? *reinterpret_cast<const uint4*>(xrow[kh] + (size_t)iw * a.ldx) : make_uint4(0, 0, 0, 0);
      }
      float best[8];
      int bi[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = -1; }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (!ok[t]) continue;
        float v[8];
        unpack8(u[t], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float z = v[k] * sc[k] + sh[k];
          v[k] = z > 0.f ? z : 0.f;
        }
        const uint4 r = pack8(v);  // the stored act value
        unpack8(r, v);
        const int kh = t / 3, kw = t % 3;
        if (kh >= 1 && kw >= 1) *reinterpret_cast<uint4*>(arow[kh] + (size_t)(2 * q - 1 + kw) * a.ldact) = r;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool take = bi[k] < 0 || v[k] > best[k] || (v[k] != v[k] && best[k] == best[k]);
          best[k] = take ? v[k] : best[k];
          bi[k] = take ? t : bi[k];
        }
      }
      const size_t opix = (size_t)orow * a.Q + q;
      *reinterpret_cast<uint4*>(a.y + opix * a.ldy + c8) = pack8(best);
      uint2 ix;
      ix.x = (unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16) | ((unsigned)bi[3] << 24);
      ix.y = (unsigned)bi[4] | ((unsigned)bi[5] << 8) | ((unsigned)bi[6] << 16) | ((unsigned)bi[7] << 24);
      *reinterpret_cast<uint2*>(a.idx + opix * a.C + c8) = ix;
    }
  }
  // batch statistics of the BN (save_mean/invstd, running stats): block 0
  if (blockIdx.x == 0 && !a.bn.ss) bn_finalize_block0(a.bn, threadIdx.x, blockDim.x, 0, a.C);
}

static inline int rows_per_block(int nrows, int target_blocks) {
  return (nrows + target_blocks - 1) / target_blocks;
}

hipError_t launch_maxpool_fwd(const MaxPoolArgs& a, hipStream_t st) {
  if (a.C % 8 || 256 % (a.C / 8)) return hipErrorInvalidValue;
  const int nrows = a.N * a.P;
  const int rpb = rows_per_block(nrows, 2048);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((nrows + rpb - 1) / rpb), dim3(256), 0, st, a, rpb);
  return hipGetLastError();
}
hipError_t launch_bn_relu_maxpool_fwd(const MaxPoolArgs& a, hipStream_t st) {
  if (a.C % 8 || 256 % (a.C / 8) || a.C > 256 || a.H != 2 * a.P || a.W != 2 * a.Q) return hipErrorInvalidValue;
  const int nrows = a.N * a.P;
  const int rpb = rows_per_block(nrows, 2048);
  hipLaunchKernelGGL(bn_relu_maxpool_fwd_kernel, dim3((nrows + rpb - 1) / rpb), dim3(256), 0, st, a, rpb);
  return hipGetLastError();
}

// blocks of the maxpool backward (tuning; its fused BN-backward sums end in
// fp64 replica atomics, blocks / kStatRep per address)
static int g_mp_blocks = std::getenv("UNET_MP_BLOCKS") ? std::atoi(std::getenv("UNET_MP_BLOCKS")) : 2048;

hipError_t launch_maxpool_bwd(const MaxPoolArgs& a, hipStream_t st) {
  if (a.C % 8 || 256 % (a.C / 8)) return hipErrorInvalidValue;
  if (a.bb.sums && a.bb.y2) return hipErrorInvalidValue;
  const int nrows = a.N * a.H;
  const int rpb = rows_per_block(nrows, g_mp_blocks);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((nrows + rpb - 1) / rpb), dim3(256), 0, st, a, rpb);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Fused head: upconv0 (ConvTranspose2d k2s2, Cin->Co) + conv_final (1x1, Co->1).
// No non-linearity sits between the two (advanced_models.py:337-350), so the
// pair contracts to V[c][ab] = sum_o Wf[o] W0[c][o][ab] and a constant.
// ---------------------------------------------------------------------------
constexpr int kHeadMaxCin = 64;

__device__ void head_contract(const HeadArgs& a, float* V, float* cst) {
  for (int t = threadIdx.x; t < a.Cin * 4; t += blockDim.x) {
    const int c = t >> 2, ab = t & 3;
    float v = 0.f;
    for (int o = 0; o < a.Co; ++o) v += a.wf[o] * a.w0[((size_t)c * a.Co + o) * 4 + ab];
    V[t] = v;
  }
  if (threadIdx.x == 0) {
    float c0 = a.bf[0];
    for (int o = 0; o < a.Co; ++o) c0 += a.wf[o] * a.b0[o];
    *cst = c0;
  }
  __syncthreads();
}

// Both head passes are HBM streams (decoder1's output, 32 or 64 bf16 channels
// per pixel, against fp32 logits).  Round 6: the channel count is a template
// argument, pixel indices are 32-bit (the launcher checks the range), and every
// thread issues the loads of HP pixels before using any of them; the grid is a
// few blocks per CU so the per-block prologue (the contraction V) amortises
// (round 5: one pixel's loads in flight and 64-bit index divisions per pixel,
// 2.2-2.7 TB/s).
constexpr int kHeadHP = 4;  // pixels in flight per thread (Cin = 32: 16 x 16 B of loads)

// Round 6: decoder1's last BN + ReLU folded into the head (a.bn_fold): the
// head reads the raw conv output y and forms act = bf16(relu(y * sc + sh)),
// the value bn_apply_kernel would have stored, in both passes (fmaf: the same
// bits in the forward and the backward).  sc / sh per channel into LDS as
// bn_apply_kernel computes them (the producer's finalised ss, or the replica
// sums).
__device__ __forceinline__ float head_act(float y, float sc, float sh) {
  const float v = fmaf(y, sc, sh);
  return bf2f(f2bf(v > 0.f ? v : 0.f));
}
__device__ void head_bn_coef(const HeadArgs& a, float2* ss) {
  for (int c = threadIdx.x; c < a.Cin; c += blockDim.x) {
    float sc, sh, m, inv, var;
    if (a.bn.training && a.bn.ss) {
      sc = a.bn.ss[c];
      sh = a.bn.ss[a.Cin + c];
    } else {
      bn_scale_shift(a.bn, c, sc, sh, m, inv, var);
    }
    ss[c] = make_float2(sc, sh);
  }
}

template <int CIN>
__global__ void __launch_bounds__(256) head_fwd_kernel(HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float V[kHeadMaxCin * 4];
  __shared__ __attribute__((aligned(8))) float2 bss[kHeadMaxCin];
  __shared__ float cst;
  const bool fold = a.bn_fold != 0;
  if (fold) head_bn_coef(a, bss);  // (head_contract's barrier publishes it)
  head_contract(a, V, &cst);
  constexpr int CC = CIN / 8;
  const float c0 = cst;
  const int total = a.N * a.H * a.W, HW = a.H * a.W, W2 = 2 * a.W;
  const int stride = gridDim.x * blockDim.x;
  for (int p0 = blockIdx.x * blockDim.x + threadIdx.x; p0 < total; p0 += kHeadHP * stride) {
    asm volatile("" ::: "memory");  // V is re-read from LDS per pixel (not hoisted into 4*CIN registers)
    uint4 xv[kHeadHP][CC];
#pragma unroll
    for (int u = 0; u < kHeadHP; ++u) {
      const int pix = p0 + u * stride;
#pragma unroll
      for (int q = 0; q < CC; ++q)
        xv[u][q] = pix < total ? *reinterpret_cast<const uint4*>(a.x + (size_t)pix * a.ldx + q * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kHeadHP; ++u) {
      const int pix = p0 + u * stride;
      if (pix >= total) break;
      float o[4] = {c0, c0, c0, c0};
#pragma unroll
      for (int q = 0; q < CC; ++q) {
        float x[8];
        unpack8(xv[u][q], x);
        if (fold) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float2 s = bss[q * 8 + k];
            x[k] = head_act(x[k], s.x, s.y);
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {  // V from LDS (a broadcast read: every lane the same address)
          const float4 v = *reinterpret_cast<const float4*>(V + (q * 8 + k) * 4);
          o[0] += x[k] * v.x; o[1] += x[k] * v.y; o[2] += x[k] * v.z; o[3] += x[k] * v.w;
        }
      }
      const int n = pix / HW, r = pix - n * HW, i = r / a.W, j = r - i * a.W;
      float* row0 = a.logits + ((size_t)n * 2 * a.H + 2 * i) * W2 + 2 * j;
      *reinterpret_cast<float2*>(row0) = make_float2(o[0], o[1]);
      *reinterpret_cast<float2*>(row0 + W2) = make_float2(o[2], o[3]);
    }
  }
  // the folded BN's statistics: save_mean / save_invstd and the running stats
  // (bn_apply_kernel's block 0 in the unfolded path)
  if (fold && blockIdx.x == 0 && !a.bn.ss) bn_finalize_block0(a.bn, threadIdx.x, blockDim.x, 0, a.Cin);
}

// thread = (8-channel chunk, pixel row); U[c][ab] partials live in registers;
// kHeadHP pixels' operands (dlogits, x, the fused BN's y) are loaded before use.
template <int CIN>
__global__ void __launch_bounds__(256) head_bwd_kernel(HeadArgs a) {
  __shared__ float V[kHeadMaxCin * 4];
  __shared__ __attribute__((aligned(8))) float2 bss[kHeadMaxCin];
  __shared__ float cst;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [rows][Cin*4 + 1]
  const bool fold = a.bn_fold != 0;  // x = y: act recomputed (the launcher checks bb.y == x)
  if (fold) head_bn_coef(a, bss);
  head_contract(a, V, &cst);
  constexpr int CC = CIN / 8;
  constexpr int rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int c8 = chunk << 3;
  const int total = a.N * a.H * a.W, HW = a.H * a.W;
  const BnBwdArgs& bb = a.bb;
  const bool fz = bb.sums != nullptr;
  float s1[8], s2[8], mu[8], is[8], bsc[8], bsh[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s1[k] = s2[k] = 0.f;
    mu[k] = fz ? bb.mean[c8 + k] : 0.f;
    is[k] = fz ? bb.invstd[c8 + k] : 0.f;
    bsc[k] = fold ? bss[c8 + k].x : 0.f;
    bsh[k] = fold ? bss[c8 + k].y : 0.f;
  }
  float U[8][4];
  float S = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) U[k][ab] = 0.f;
  float Vl[8][4];
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) Vl[k][ab] = V[(c8 + k) * 4 + ab];
  const int W2 = 2 * a.W;
  const int stride = gridDim.x * rows;
  for (int p0 = blockIdx.x * rows + row; p0 < total; p0 += kHeadHP * stride) {
    float2 d01[kHeadHP], d23[kHeadHP];
    uint4 xv[kHeadHP], yv[kHeadHP];
#pragma unroll
    for (int u = 0; u < kHeadHP; ++u) {
      const int pix = p0 + u * stride;
      const bool ok = pix < total;
      const int pc = ok ? pix : 0;
      const int n = pc / HW, r = pc - n * HW, i = r / a.W, j = r - i * a.W;
      const float* row0 = a.dl + ((size_t)n * 2 * a.H + 2 * i) * W2 + 2 * j;
      d01[u] = ok ? *reinterpret_cast<const float2*>(row0) : make_float2(0.f, 0.f);
      d23[u] = ok ? *reinterpret_cast<const float2*>(row0 + W2) : make_float2(0.f, 0.f);
      xv[u] = (ok && !fold) ? *reinterpret_cast<const uint4*>(a.x + (size_t)pc * a.ldx + c8) : make_uint4(0, 0, 0, 0);
      yv[u] = (ok && fz) ? *reinterpret_cast<const uint4*>(bb.y + (size_t)pc * bb.ldy + c8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kHeadHP; ++u) {
      const int pix = p0 + u * stride;
      if (pix >= total) break;
      const float d[4] = {d01[u].x, d01[u].y, d23[u].x, d23[u].y};
      if (chunk == 0) S += (d[0] + d[1]) + (d[2] + d[3]);
      float x[8], g[8];
      if (fold) {
        unpack8(yv[u], x);
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = head_act(x[k], bsc[k], bsh[k]);
      } else {
        unpack8(xv[u], x);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        g[k] = d[0] * Vl[k][0] + d[1] * Vl[k][1] + d[2] * Vl[k][2] + d[3] * Vl[k][3];
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) U[k][ab] += x[k] * d[ab];
      }
      if (fz) {  // x IS the BN+ReLU output (act): ReLU mask, then the BN-backward sums
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = x[k] > 0.f ? g[k] : 0.f;
      }
      const uint4 o = pack8(g);
      *reinterpret_cast<uint4*>(a.dx + (size_t)pix * a.lddx + c8) = o;
      if (fz) {
        float dz[8], y[8];
        unpack8(o, dz);  // sums of the stored bf16 dZ, as bn_bwd_reduce_kernel would read them
        unpack8(yv[u], y);
#pragma unroll
        for (int k = 0; k < 8; ++k) { s1[k] += dz[k]; s2[k] += dz[k] * (y[k] - mu[k]) * is[k]; }
      }
    }
  }
  // red[row][L]: U (Cin*4) | S | fused BN sums dZ (Cin) | dZ*xhat (Cin)
  const int LU = CIN * 4 + 1;
  const int L = LU + (fz ? 2 * CIN : 0);
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) red[row * L + (c8 + k) * 4 + ab] = U[k][ab];
  if (chunk == 0) red[row * L + CIN * 4] = S;
  if (fz) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[row * L + LU + c8 + k] = s1[k];
      red[row * L + LU + CIN + c8 + k] = s2[k];
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    float v = 0.f;
    for (int r = 0; r < rows; ++r) v += red[r * L + t];
    if (t < LU) {  // [kStatRep][Cin*4 + 1] replicas (head_grads_kernel sums them in order)
      atomicAdd(a.usum + (size_t)(blockIdx.x % kStatRep) * LU + t, (double)v);
    } else {  // [kStatRep][2][C] replica layout of the BN-backward sums
      const int q = (t - LU) / CIN, c = (t - LU) - q * CIN;
      atomicAdd(bb.sums + (size_t)(blockIdx.x % kStatRep) * 2 * CIN + q * CIN + c, (double)v);
    }
  }
  if (fz && bb.ticket) {
    __shared__ int flag;
    if (last_block_arrive(bb.ticket, gridDim.x, &flag, true)) bn_bwd_finalize(bb);
  }
}

constexpr int kHeadMaxW0 = kHeadMaxCin * 32 * 4;  // Cin x Co x 4 (Wide: 64 x 32)
__global__ void __launch_bounds__(256) head_grads_kernel(HeadArgs a) {
  // usum and w0 staged in LDS first: the serial per-output loops below then
  // read LDS instead of one dependent global load per term (same order, same
  // arithmetic as before)
  __shared__ double us[kHeadMaxCin * 4 + 1];
  __shared__ float w0s[kHeadMaxW0];
  const int nw = a.Cin * a.Co * 4;
  for (int t = threadIdx.x; t <= a.Cin * 4; t += blockDim.x) {
    double v = 0.0;
    for (int r = 0; r < kStatRep; ++r) v += a.usum[(size_t)r * (a.Cin * 4 + 1) + t];
    us[t] = v;
  }
  for (int t = threadIdx.x; t < nw; t += blockDim.x) w0s[t] = a.w0[t];
  __syncthreads();
  const double S = us[a.Cin * 4];
  for (int t = threadIdx.x; t < nw; t += blockDim.x) {
    const int ab = t & 3, o = (t >> 2) % a.Co, c = (t >> 2) / a.Co;
    a.gw0[t] = (float)((double)a.wf[o] * us[c * 4 + ab]);
  }
  for (int o = threadIdx.x; o < a.Co; o += blockDim.x) {
    a.gb0[o] = (float)((double)a.wf[o] * S);
    double g = (double)a.b0[o] * S;
    for (int c = 0; c < a.Cin; ++c)
      for (int ab = 0; ab < 4; ++ab) g += (double)w0s[(c * a.Co + o) * 4 + ab] * us[c * 4 + ab];
    a.gwf[o] = (float)g;
  }
  if (threadIdx.x == 0) a.gbf[0] = (float)S;
}

// the head's pixel range in 32-bit indices (decoder1 output pixels, and the
// 4x as many logits)
static bool head_ok(const HeadArgs& a) {
  return (a.Cin == 32 || a.Cin == 64) && (int64_t)a.N * a.H * a.W * 4 < 0x7fffffffLL;
}
hipError_t launch_head_fwd(const HeadArgs& a, hipStream_t st) {
  if (!head_ok(a) || (a.bn_fold && (a.bn.C != a.Cin || !a.bn.stats))) return hipErrorInvalidValue;
  const int64_t total = (int64_t)a.N * a.H * a.W;
  const int grid = grid_for(total, 256 * kHeadHP * 2, 1024);
  if (a.Cin == 32) hipLaunchKernelGGL(head_fwd_kernel<32>, dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(head_fwd_kernel<64>, dim3(grid), dim3(256), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_head_bwd(const HeadArgs& a, hipStream_t st) {
  if (!head_ok(a)) return hipErrorInvalidValue;
  const int64_t total = (int64_t)a.N * a.H * a.W;
  const int CC = a.Cin / 8, rows = 256 / CC;
  if (a.bb.sums && (a.bb.C != a.Cin || a.bb.y2)) return hipErrorInvalidValue;
  // the folded BN: act is recomputed from bb.y, which must be the head's x
  if (a.bn_fold && (!a.bb.sums || a.bb.y != a.x || a.bb.ldy != a.ldx || a.bn.C != a.Cin || !a.bn.stats))
    return hipErrorInvalidValue;
  const size_t lds = (size_t)rows * (a.Cin * 4 + 1 + (a.bb.sums ? 2 * a.Cin : 0)) * sizeof(float);
  // 512 blocks: each adds Cin*4 + 1 fp64 partials (16 replicas) at its end;
  // 1024 blocks onto one copy serialised ~1k same-address atomics per word
  const int grid = grid_for(total, rows * kHeadHP * 4, 512);
  if (a.Cin == 32) hipLaunchKernelGGL(head_bwd_kernel<32>, dim3(grid), dim3(256), lds, st, a);
  else hipLaunchKernelGGL(head_bwd_kernel<64>, dim3(grid), dim3(256), lds, st, a);
  return hipGetLastError();
}
hipError_t launch_head_grads(const HeadArgs& a, hipStream_t st) {
  if (a.Cin > kHeadMaxCin || a.Cin * a.Co * 4 > kHeadMaxW0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(head_grads_kernel, dim3(1), dim3(256), 0, st, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// per-channel sums (ConvTranspose bias gradients; the replicas are summed into
// the fp32 gradient by bucket 0's unpack launch, UP_D2F)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) channel_sum_kernel(const bf16_t* x, int ldx, int64_t npix, int C,
                                                         double* acc) {
  const int CC = C >> 3;
  const int rows = blockDim.x / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int c8 = chunk << 3;
  float s[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = 0.f;
  if (row < rows) {
    constexpr int PPT = 4;
    const int64_t stride = (int64_t)gridDim.x * rows;
    for (int64_t base = (int64_t)blockIdx.x * rows + row; base < npix; base += PPT * stride) {
      uint4 u[PPT];
#pragma unroll
      for (int j = 0; j < PPT; ++j) {
        const int64_t pix = base + j * stride;
        u[j] = pix < npix ? *reinterpret_cast<const uint4*>(x + pix * ldx + c8) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int j = 0; j < PPT; ++j) {
        float v[8];
        unpack8(u[j], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += v[k];
      }
    }
  }
  extern __shared__ __attribute__((aligned(16))) float red[];
  if (row < rows) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[row * C + c8 + k] = s[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float t = 0.f;
    for (int r = 0; r < rows; ++r) t += red[r * C + c];
    atomicAdd(acc + (size_t)(blockIdx.x % kStatRep) * C + c, (double)t);  // replica: no hot address
  }
}

// grid cap of the channel sums (tuning): each fp64 replica address takes
// blocks / kStatRep atomics
static int g_chsum_cap = std::getenv("UNET_CHSUM_CAP") ? std::atoi(std::getenv("UNET_CHSUM_CAP")) : 2048;

hipError_t launch_channel_sum(const bf16_t* x, int ldx, int64_t npix, int C, double* acc, hipStream_t st) {
  if (C % 8 || C / 8 > 256) return hipErrorInvalidValue;
  const int CC = C / 8, rows = 256 / CC;
  hipLaunchKernelGGL(channel_sum_kernel, dim3(grid_for(npix, rows * 8, g_chsum_cap)), dim3(rows * CC),
                     (size_t)rows * C * sizeof(float), st, x, ldx, npix, C, acc);
  return hipGetLastError();
}

// dst[i] = sum of the kStatRep replicas src[r][i]
__global__ void d2f_kernel(const double* s, float* d, int n, int stride) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = 0.0;
  for (int r = 0; r < kStatRep; ++r) v += s[(size_t)r * stride + i];
  d[i] = (float)v;
}
hipError_t launch_d2f(const double* src, float* dst, int n, hipStream_t st) {
  return launch_d2f_strided(src, dst, n, n, st);
}
hipError_t launch_d2f_strided(const double* src, float* dst, int n, int stride, hipStream_t st) {
  hipLaunchKernelGGL(d2f_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, n, stride);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// weight packing: fp32 torch layouts -> bf16 kernel layouts (one launch)
// ---------------------------------------------------------------------------
// Every layout change is a transpose of src viewed as [A][B][T] (T = R*S taps):
//   inner:  dst[a][t][b] = src[a][b][t]   conv fwd (A=Co,B=Ci), convT dgrad (A=Ci,B=Co)
//   full:   dst[b][t][a] = src[a][b][t]   conv dgrad (A=Co,B=Ci), convT fwd (A=Ci,B=Co)
// staged through LDS so that both the fp32 reads and the bf16 writes are
// contiguous runs (the direct gather reads one element per 36-B..18-KB stride).
constexpr int kPkTA = 64, kPkTB = 16, kPkTmax = 9;
__global__ void __launch_bounds__(256) pack_kernel(PackTable t) {
  const PackEntry e = t.e[blockIdx.y];
  // one LDS buffer for either path: [kPkTB*T][kPkTA+1] tile or a [B*T] row
  __shared__ float lds[kPkTB * kPkTmax * (kPkTA + 1)];
  static_assert(512 * kPkTmax <= kPkTB * kPkTmax * (kPkTA + 1), "row fits");
  if (e.kind == PK_ZERO) {
    uint4* d = reinterpret_cast<uint4*>(e.dst);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < e.Co; i += gridDim.x * blockDim.x)
      d[i] = make_uint4(0, 0, 0, 0);
    return;
  }
  if (e.kind == PK_STEM) {  // dst[co][k], k = kr*8 + ks -> W[co][0][kr][ks] (kr, ks < 7; else 0)
    const int total = e.Co * 64;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
      const int kr = (i >> 3) & 7, ks = i & 7, co = i >> 6;
      e.dst[i] = f2bf(kr < 7 && ks < 7 ? e.src[co * 49 + kr * 7 + ks] : 0.f);
    }
    return;
  }
  const bool convt = e.kind == PK_CONVT_FWD || e.kind == PK_CONVT_DGRAD;
  const int A = convt ? e.Ci : e.Co, B = convt ? e.Co : e.Ci, T = e.R * e.S;
  const bool full = e.kind == PK_CONV_DGRAD || e.kind == PK_CONVT_FWD || e.kind == PK_CONV_DGRAD_CH;
  // chunk-major 3x3 packs (conv3x3_fl_kernel): fwd dst[b/32][t][a][b%32],
  // dgrad dst[a/32][t][b][a%32]
  const bool chunk = e.kind == PK_CONV_FWD_CH || e.kind == PK_CONV_DGRAD_CH;
  // every load of a pass is issued before the first LDS store (no per-load
  // round trip to L2)
  if (!full) {  // one a-row [B][T] -> [T][B] per block iteration, in b-chunks of <= 512
    constexpr int kMaxPer = 512 * kPkTmax / 256;
    const int n = B * T;
    for (int a = blockIdx.x; a < A; a += gridDim.x) {
      for (int b0 = 0; b0 < B; b0 += 512) {  // rows wider than 512 b (Wide config, Ci = 1536)
        const int nb = min(512, B - b0), m = nb * T;
        const float* src = e.src + (size_t)a * n + (size_t)b0 * T;
        float v[kMaxPer];
#pragma unroll
        for (int k = 0; k < kMaxPer; ++k) {
          const int i = threadIdx.x + 256 * k;
          v[k] = i < m ? src[i] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < kMaxPer; ++k) {
          const int i = threadIdx.x + 256 * k;
          if (i < m) lds[i] = v[k];
        }
        __syncthreads();
        if (chunk) {
          for (int tt = 0; tt < T; ++tt)
            for (int b = threadIdx.x; b < nb; b += blockDim.x) {
              const int bg = b0 + b;
              e.dst[((size_t)((bg >> 5) * T + tt) * A + a) * 32 + (bg & 31)] = f2bf(lds[b * T + tt]);
            }
        } else {
          bf16_t* dst = e.dst + (size_t)a * n + b0;
          for (int tt = 0; tt < T; ++tt)
            for (int b = threadIdx.x; b < nb; b += blockDim.x) dst[tt * B + b] = f2bf(lds[b * T + tt]);
        }
        __syncthreads();
      }
    }
    return;
  }
  // full transpose in (kPkTA a) x (kPkTB b) x T tiles; tile row j = bl*T + t
  // maps to dst row b0*T + j, so no index needs a division
  constexpr int LD = kPkTA + 1;
  const int ta = (A + kPkTA - 1) / kPkTA, tb = (B + kPkTB - 1) / kPkTB;
  const int lane = threadIdx.x & 63, sub = threadIdx.x >> 6;  // 4 waves
  for (int tile_id = blockIdx.x; tile_id < ta * tb; tile_id += gridDim.x) {
    const int a0 = (tile_id % ta) * kPkTA, b0 = (tile_id / ta) * kPkTB;
    const int run = min(kPkTB, B - b0) * T;  // valid contiguous floats per a (<= 144)
    float v[16][3];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int al = sub + 4 * k;
      const float* src = e.src + ((size_t)(a0 + al) * B + b0) * T;
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int j = lane + 64 * m;
        v[k][m] = (j < run && a0 + al < A) ? src[j] : 0.f;
      }
    }
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const int j = lane + 64 * m;
        if (j < run) lds[j * LD + sub + 4 * k] = v[k][m];
      }
    __syncthreads();
    if (a0 + lane < A) {
      if (chunk) {
        const int ag = a0 + lane;
        bf16_t* dst = e.dst + (size_t)(ag >> 5) * T * B * 32 + (ag & 31);
        for (int j = sub; j < run; j += 4) {
          const int bl = j / T, t = j - bl * T;
          dst[((size_t)t * B + b0 + bl) * 32] = f2bf(lds[j * LD + lane]);
        }
      } else {
        bf16_t* dst = e.dst + (size_t)b0 * T * A + a0 + lane;
        for (int j = sub; j < run; j += 4) dst[(size_t)j * A] = f2bf(lds[j * LD + lane]);
      }
    }
    if (e.dst2) {  // forward layout from the same tile: element (a0+al, b0+bl, t) = lds[(bl*T + t)*LD + al]
      const int nb = min(kPkTB, B - b0), na = min(kPkTA, A - a0);
      const bool ch2 = e.kind2 == PK_CONV_FWD_CH;
      const int bl = threadIdx.x % kPkTB, b = b0 + bl;  // 16 lanes write 16 consecutive b (32 B)
      if (bl < nb)
        for (int al = threadIdx.x / kPkTB; al < na; al += blockDim.x / kPkTB) {
          const int a = a0 + al;
          // fwd dst[b/32][t][a][b%32] (chunk-major) or dst[a][t][b]
          bf16_t* d = ch2 ? e.dst2 + ((size_t)(b >> 5) * T * A + a) * 32 + (b & 31) : e.dst2 + (size_t)a * T * B + b;
          const size_t dt = ch2 ? (size_t)A * 32 : (size_t)B;
          for (int t = 0; t < T; ++t) d[t * dt] = f2bf(lds[(bl * T + t) * LD + al]);
        }
    }
    __syncthreads();
  }
}

hipError_t launch_pack(const PackTable& t, hipStream_t st) {
  if (t.n <= 0) return hipSuccess;
  for (int i = 0; i < t.n; ++i) {
    const PackEntry& e = t.e[i];
    if (e.kind != PK_STEM && e.R * e.S > kPkTmax) return hipErrorInvalidValue;
    if (e.dst2 && (!(e.kind == PK_CONV_DGRAD || e.kind == PK_CONV_DGRAD_CH) ||
                   !(e.kind2 == PK_CONV_FWD || e.kind2 == PK_CONV_FWD_CH)))
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(pack_kernel, dim3(256, t.n), dim3(256), 0, st, t);
  return hipGetLastError();
}

// Kernel-layout accumulators -> torch layout.  Conv [Co][T][Ci] -> [Co][Ci][T]
// and convT [Ci][T][Co] -> [Ci][Co][T] (T = R*S) are per-row [T][K] -> [K][T]
// transposes: a block stages <= 512 columns of a row in LDS with contiguous
// reads and writes the transposed run contiguously (row stride 513: no bank
// conflicts on the transposed read).  Stem [64][64] (k = r*8+s) keeps the
// element map; UP_ZERO writes zeros.
constexpr int kUpK = 512, kUpT = 9;
__global__ void __launch_bounds__(256) unpack_kernel(UnpackTable t) {
  const UnpackEntry e = t.e[blockIdx.y];
  if (e.kind == UP_D2F) {  // dst[i] = sum of the kStatRep fp64 replicas acc[r][i] (as d2f_kernel)
    const double* s = reinterpret_cast<const double*>(e.acc);
    for (int i = (int)blockIdx.x * blockDim.x + threadIdx.x; i < e.Co; i += (int)gridDim.x * blockDim.x) {
      double v = 0.0;
      for (int r = 0; r < kStatRep; ++r) v += s[(size_t)r * e.Co + i];
      e.dst[i] = (float)v;
    }
    return;
  }
  if (e.kind == UP_ZERO || e.kind == UP_STEM) {
    const int total = e.kind == UP_ZERO ? e.Co : e.Co * 49;
    for (int i = (int)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int)gridDim.x * blockDim.x) {
      float v = 0.f;  // UP_ZERO: a gradient that is exactly 0 (bias feeding a training-mode BN)
      if (e.kind == UP_STEM) {  // dst[co][0][r][s] <- acc[co][r*8+s] (row length 64)
        const int k = i % 49, co = i / 49;
        const int r = k / 7, ss = k - r * 7;
        v = e.acc[co * 64 + r * 8 + ss];
      }
      e.dst[i] = v;
    }
    return;
  }
  __shared__ float lds[kUpT * (kUpK + 1)];
  const bool convt = e.kind == UP_CONVT;
  const int rows = convt ? e.Ci : e.Co, K = convt ? e.Co : e.Ci, T = e.R * e.S;
  for (int a = blockIdx.x; a < rows; a += gridDim.x) {
    const float* src = e.acc + (size_t)a * K * T;
    float* dst = e.dst + (size_t)a * K * T;
    for (int k0 = 0; k0 < K; k0 += kUpK) {
      const int nk = min(kUpK, K - k0);
      // 16-B loads / stores (all of a thread's loads in flight before the LDS
      // stores) when both rows are 16-B aligned (a parameter after an odd-sized
      // one may not be)
      const bool v4 = (K & 3) == 0 && ((reinterpret_cast<uintptr_t>(e.acc) | reinterpret_cast<uintptr_t>(e.dst)) & 15) == 0;
      if (v4) {
        const int n4 = T * nk / 4, q4 = nk / 4;
        constexpr int kPer = (kUpT * kUpK / 4 + 255) / 256;  // <= 5 float4 per thread
        float4 v[kPer];
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int i = threadIdx.x + 256 * u;
          if (i < n4) {
            const int tt = i / q4, k = (i - tt * q4) * 4;
            v[u] = *reinterpret_cast<const float4*>(src + (size_t)tt * K + k0 + k);
          }
        }
#pragma unroll
        for (int u = 0; u < kPer; ++u) {
          const int i = threadIdx.x + 256 * u;
          if (i < n4) {
            const int tt = i / q4, k = (i - tt * q4) * 4;
            float* l = lds + tt * (kUpK + 1) + k;
            l[0] = v[u].x; l[1] = v[u].y; l[2] = v[u].z; l[3] = v[u].w;
          }
        }
        __syncthreads();
        float* d = dst + (size_t)k0 * T;  // the run [k0*T, (k0+nk)*T) is contiguous, 16-B aligned
        for (int i = threadIdx.x; i < n4; i += blockDim.x) {
          float o[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            const int j = 4 * i + c, k = j / T, tt = j - k * T;
            o[c] = lds[tt * (kUpK + 1) + k];
          }
          *reinterpret_cast<float4*>(d + 4 * i) = make_float4(o[0], o[1], o[2], o[3]);
        }
        __syncthreads();
        continue;
      }
      for (int i = threadIdx.x; i < T * nk; i += blockDim.x) {
        const int tt = i / nk, k = i - tt * nk;
        lds[tt * (kUpK + 1) + k] = src[(size_t)tt * K + k0 + k];
      }
      __syncthreads();
      for (int i = threadIdx.x; i < T * nk; i += blockDim.x) {
        const int k = i / T, tt = i - k * T;
        dst[(size_t)(k0 + k) * T + tt] = lds[tt * (kUpK + 1) + k];
      }
      __syncthreads();
    }
  }
}

hipError_t launch_unpack(const UnpackTable& t, hipStream_t st) {
  if (t.n <= 0) return hipSuccess;
  for (int i = 0; i < t.n; ++i)
    if ((t.e[i].kind == UP_CONV || t.e[i].kind == UP_CONVT) && t.e[i].R * t.e[i].S > kUpT) return hipErrorInvalidValue;
  hipLaunchKernelGGL(unpack_kernel, dim3(512, t.n), dim3(256), 0, st, t);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// pixel-wise loss and mask metrics (losses.py:13-37,161-171; utils.py:120-151)
// ---------------------------------------------------------------------------
// One pass over the pixels: 8 per-thread fp32 sums, folded per block in fp64
// into the block's partial slot (loss_reduce_kernel adds the slots in order).
// One block per CU (256 blocks); float4 loads (4 in flight per thread) when both
// operands are 16-B aligned.  The pass is VALU-bound, not HBM-bound: libm
// expf + log1pf + expf + an IEEE divide per pixel compiled to ~175 VALU
// instructions (26.7 us for 4 M pixels, 1.2 TB/s), so the terms share one
// exponential e = exp(-|v|) and one reciprocal of 1 + e on the hardware
// v_exp_f32 / v_log_f32 / v_rcp_f32 (~1 ulp each):
//   log1p(e) = log(u) * e / (u - 1), u = 1 + e  (exact-rounding correction; e when u == 1)
//   sigma(v) = (v >= 0 ? 1 : e) / u
__device__ __forceinline__ void loss_accum(float v, float y, int from_prob, float (&s)[8]) {
  float pred;
  if (!from_prob) {
    // torch: (1 - y) * x - log_sigmoid(x),  log_sigmoid(x) = min(x,0) - log1p(exp(-|x|))
    const float e = __expf(-fabsf(v));
    const float u = 1.f + e;
    const float ru = __builtin_amdgcn_rcpf(u);
    const float um1 = u - 1.f;
    const float l1p = um1 == 0.f ? e : __logf(u) * (e * __builtin_amdgcn_rcpf(um1));
    // (1 - y) v - log_sigmoid(v) = max(v, 0) - y v + log1p(e): the same value as
    // torch's formulation without its cancellation for confident logits
    // (e.g. v = -10, y = 0: -10 - (-10 - 4.5e-5) loses ~1 % in fp32)
    s[0] += (fmaxf(v, 0.f) - y * v) + l1p;
    const float sg = (v >= 0.f ? 1.f : e) * ru;
    s[1] += sg * y;
    s[2] += sg;
    s[3] += y;
    pred = v >= kMaskThreshold ? 1.f : 0.f;  // == (sigmoid_cpu(v) > 0.5)
  } else {
    pred = v > 0.5f ? 1.f : 0.f;
  }
  s[4] += pred * y;
  s[5] += pred * (1.f - y);
  s[6] += (1.f - pred) * y;
  s[7] += (1.f - pred) * (1.f - y);
}

// 1024 threads per block: 16 waves per CU hide the exp/log chains of the BCE
// terms (at 4 waves the kernel took 37 us for 4.2 M pixels); the block count
// stays at <= 256 (same-address fp64 atomics are serialised)
constexpr int kLossNT = 1024;
__global__ void __launch_bounds__(kLossNT) loss_sums_kernel(const float* x, const float* t, int64_t n,
                                                            double* part, int from_prob) {
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t done = 0;
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(t)) & 15) == 0) {
    const int64_t n4 = n >> 2;
    const float4* x4 = reinterpret_cast<const float4*>(x);
    const float4* t4 = reinterpret_cast<const float4*>(t);
    constexpr int U = 4;
    for (int64_t i = tid; i < n4; i += U * nthr) {
      float4 xv[U], tv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = i + u * nthr;
        xv[u] = j < n4 ? x4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
        tv[u] = j < n4 ? t4[j] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i + u * nthr >= n4) break;
        loss_accum(xv[u].x, tv[u].x, from_prob, s);
        loss_accum(xv[u].y, tv[u].y, from_prob, s);
        loss_accum(xv[u].z, tv[u].z, from_prob, s);
        loss_accum(xv[u].w, tv[u].w, from_prob, s);
      }
    }
    done = n4 << 2;
  }
  for (int64_t i = done + tid; i < n; i += nthr) loss_accum(x[i], t[i], from_prob, s);
  __shared__ double red[kLossNT / 64][8];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double v = wave_sum_d((double)s[k]);
    if (lane == 0) red[wave][k] = v;
  }
  __syncthreads();
  // this block's partial sums (fixed wave order) go to its own slot: the 8
  // totals are summed in block order by loss_reduce_kernel.  One fp64 atomic
  // per block and value on a single 64-B line serialised ~256 device-scope
  // atomics per address (the kernel measured 37 us for 32 MB, r04 profiles)
  // and made the sums depend on block arrival order.
  if (threadIdx.x < 8) {
    const int k = threadIdx.x;
    double v = 0.0;
    for (int w = 0; w < kLossNT / 64; ++w) v += red[w][k];
    part[blockIdx.x * 8 + k] = v;
  }
}

// s[k] = sum over blocks b (in order, 64 lanes then a fixed butterfly) of
// the partial part[8 b + k]; wave k owns value k.  Thread 0 then writes the
// loss value when `out` is given.
__global__ void __launch_bounds__(512) loss_reduce_kernel(double* s, const double* part, int nblk, int64_t n,
                                                          int kind, float alpha, float smooth, float* out) {
  __shared__ double tot[8];
  const int k = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double v = 0.0;
  for (int b = lane; b < nblk; b += 64) v += part[b * 8 + k];
  v = wave_sum_d(v);
  if (lane == 0) {
    s[k] = v;
    tot[k] = v;
  }
  __syncthreads();
  if (out == nullptr || threadIdx.x != 0) return;
  const double bce = tot[0] / (double)n;
  const double dice = 1.0 - (2.0 * tot[1] + smooth) / (tot[2] + tot[3] + smooth);
  double r;
  if (kind == LOSS_BCE) r = bce;
  else if (kind == LOSS_DICE) r = dice;
  else r = alpha * bce + (1.0 - alpha) * dice;
  *out = (float)r;
}

hipError_t launch_loss_sums(const float* logits, const float* target, int64_t n, double* sums, double* part,
                            int from_prob, int kind, float alpha, float smooth, float* out, hipStream_t st) {
  const int nblk = grid_for(n, kLossNT * 16, kLossBlocks);
  if (nblk > kLossBlocks) return hipErrorInvalidValue;  // part holds kLossBlocks slots
  hipLaunchKernelGGL(loss_sums_kernel, dim3(nblk), dim3(kLossNT), 0, st, logits, target, n, part, from_prob);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(512), 0, st, sums, part, nblk, n, kind, alpha, smooth, out);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) loss_grad_kernel(const float* x, const float* t, int64_t n, const double* s,
                                                       int kind, float alpha, float smooth, const float* gscale,
                                                       float* dl) {
  const float g = gscale ? *gscale : 1.f;
  const float wb = kind == LOSS_BCE ? 1.f : (kind == LOSS_COMBO ? alpha : 0.f);
  const float wd = kind == LOSS_DICE ? 1.f : (kind == LOSS_COMBO ? 1.f - alpha : 0.f);
  const double U = s[2] + s[3] + smooth;
  const float inv_u2 = (float)(1.0 / (U * U));
  const float twoI = (float)(2.0 * s[1] + smooth);
  const float Uf = (float)U;
  const float inv_n = (float)(1.0 / (double)n);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i], y = t[i];
    const float sg = 1.f / (1.f + expf(-v));
    float d = wb * (sg - y) * inv_n;
    if (wd != 0.f) {
      const float dds = -(2.f * y * Uf - twoI) * inv_u2;  // d(1 - dice)/d sigma_i
      d += wd * dds * sg * (1.f - sg);
    }
    dl[i] = g * d;
  }
}
hipError_t launch_loss_grad(const float* logits, const float* target, int64_t n, const double* sums, int kind,
                            float alpha, float smooth, const float* gscale, float* dl, hipStream_t st) {
  hipLaunchKernelGGL(loss_grad_kernel, dim3(grid_for(n, 256 * 4, 4096)), dim3(256), 0, st, logits, target, n, sums,
                     kind, alpha, smooth, gscale, dl);
  return hipGetLastError();
}

}  // namespace unet

// ConvTranspose2d(kernel 2, stride 2) forward and data gradient for the
// narrow decoder up-convs (advanced_models.py:96-99
// upconv2 128->64 and upconv1 64->32, applied at :305,315; Wide: upconv1
// 128->64) as weight-stationary GEMMs over the INPUT-resolution pixel grid:
//
//   forward    Y[n, 2h+a, 2w+b, co] = bias[co] + sum_ci W[ci][co][a][b] X[n,h,w,ci]
//   data grad  dX[n,h,w,ci] = sum_(a,b,co) W[ci][co][a][b] dY[n, 2h+a, 2w+b, co]
//
// Both are GEMMs with K <= 256 whose per-pixel K-vector is contiguous in HBM
// (X[m][0:Ci], or the four dY pixels of m with Co channels each), so the work
// is HBM-bound (≈ 100 MB per launch at upconv1, 5 TB/s -> 20 us) and the
// generic implicit GEMM (LDS-staged 128 x 128 tiles, the weights re-fetched
// by each of 2048 blocks, one K step each) ran at ≈ 1.7 TB/s.  Here:
//  * a persistent block stages its weights ONCE into LDS ([NN][K] rows, 16-B
//    chunks XOR-swizzled by row so the 16 rows of an A fragment hit distinct
//    bank groups) -- NN * K * 2 <= 64 KB, 2 blocks per CU;
//  * the pixel operand goes straight from HBM into the MFMA B fragments
//    (lane & 15 = pixel, lane >> 4 = 8-channel chunk: 16 B per lane, a pixel's
//    64 B of one 32-wide K step per lane quad);
//  * D = W^T X^T: a lane's 4 accumulator rows are 4 consecutive output
//    channels of one pixel -> one 8-B store each;
//  * the waves of a block are independent (no barrier in the pixel loop).
// Data-gradient epilogue: the fused BN(+ReLU) backward of the BN that produced
// the up-conv's input (dZ stored, sum dZ and sum dZ * xhat from the stored
// bf16 dZ, exactly conv_epilogue's), and the up-conv's BIAS gradient, the sum
// of dY over pixels and taps, taken from the B fragments themselves (every dY
// element is read exactly once) -- the separate channel_sum pass disappears.
#include <algorithm>
#include <cstdio>

#include "common.h"
#include "kernels.h"

namespace unet {

void conv_kernel_tag(const char* tag);  // conv_kernels.hip: per-launch profiler column

constexpr int kCtWaves = 4;

// byte offset of 16-B chunk c of LDS weight row r (rows of KB bytes): chunk
// XOR (r mod the row's chunk count, at most 8), so it stays inside the row
__device__ __forceinline__ int ct_off(int r, int c, int KB) {
  const int m = (KB >> 4) >= 8 ? 7 : (KB >> 4) - 1;
  return r * KB + ((c ^ (r & m)) << 4);
}

__device__ __forceinline__ void unpack4(uint2 u, float* f) {
  f[0] = __uint_as_float(u.x << 16); f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16); f[3] = __uint_as_float(u.y & 0xffff0000u);
}

// MODE 0 forward: NN = 4 Co output columns (tap-major: column t * Co + co),
// K = Ci.  MODE 1 data gradient: NN = Ci, K = 4 Co (k = t * Co + co).  MT
// 16-pixel tiles per wave and group; FB: fused BN backward (MODE 1).  A wave
// loads its next group once this one is stored; the other resident waves
// cover that latency (a register prefetch one group ahead and MT = 2 measured
// no faster, scripts/micro/convt_bench.py).
template <int MODE, int NT, int KS, int MT, bool FB>
__global__ void __launch_bounds__(kCtWaves * 64) convt2x2_kernel(ConvFwdArgs a, int ngroups) {
  constexpr int NN = NT * 16, K = KS * 32, KB = K * 2;
  constexpr int Co = MODE == 0 ? NN / 4 : K / 4;
  constexpr int NBS = MODE == 1 ? Co / 32 : 1;  // bias-sum channel sets per lane (8 channels each)
  static_assert(MODE == 0 || Co % 32 == 0, "a 32-wide K step stays inside one tap");
  static_assert(MODE == 1 || Co % 16 == 0, "a lane's 4 columns share one tap");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;                                         // [NN][K] bf16
  float* cst = reinterpret_cast<float*>(smem + NN * KB);  // MODE 0: bias [Co]; MODE 1: mean | invstd [2][NN]
  float* red = cst + 2 * NN;                               // [kCtWaves][NN][2], then bias sums [kCtWaves][Co]
  float* redb = red + kCtWaves * NN * 2;
  int* flag = reinterpret_cast<int*>(redb + kCtWaves * Co);
  float* xss = reinterpret_cast<float*>(flag + 4);  // MODE 0 xform: [2][K] scale | shift
  const bool xf = MODE == 0 && a.xform != 0;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pl = lane & 15, kq = lane >> 4;
  const bool bsum = MODE == 1 && a.bias_acc != nullptr;
  // FB operands with the pixel operand (one round trip per group) when they
  // fit; the 8-tile (128-channel) form loads them per tile in the epilogue
  constexpr bool FBTOP = FB && NT <= 4;

  const int Wd = a.W, HW = a.H * a.W, Q = 2 * a.W;
  // pixel operand of group g: MT tiles of 16 input-grid pixels
  auto load_b = [&](int g, bf16x8 (&B)[MT][KS]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = (g * MT + mt) * 16 + pl;
      if constexpr (MODE == 0) {
        const bf16_t* src = a.x + (size_t)m * a.ldx + kq * 8;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) B[mt][ks] = *reinterpret_cast<const bf16x8*>(src + ks * 32);
      } else {
        const int n = m / HW, r = m - n * HW, h = r / Wd, w = r - h * Wd;
        const size_t p00 = ((size_t)n * (2 * a.H) + 2 * h) * Q + 2 * w;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int k0 = ks * 32 + kq * 8, t = k0 / Co, co = k0 - t * Co;
          const size_t pix = p00 + (size_t)(t >> 1) * Q + (t & 1);
          B[mt][ks] = *reinterpret_cast<const bf16x8*>(a.x + pix * a.ldx + co);
        }
      }
    }
  };
  // FB: the BN's forward output (ReLU mask) and raw conv output at group g
  auto load_bn = [&](int g, uint2 (&ua)[MT][NT], uint2 (&uy)[MT][NT]) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const size_t m = (size_t)(g * MT + mt) * 16 + pl;
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const int ci = nt * 16 + kq * 4;
        ua[mt][nt] = *reinterpret_cast<const uint2*>(a.bb.act + m * a.bb.ldact + ci);
        uy[mt][nt] = *reinterpret_cast<const uint2*>(a.bb.y + m * a.bb.ldy + ci);
      }
    }
  };

  // the first group's operands go out before the weight staging (independent)
  const int nw = gridDim.x * kCtWaves;
  int g = blockIdx.x * kCtWaves + wave;
  bf16x8 Bc[MT][KS];
  uint2 uac[MT][NT], uyc[MT][NT];
  if (g < ngroups) {
    load_b(g, Bc);
    if constexpr (FBTOP) load_bn(g, uac, uyc);
  }

  // weights, once per block.  MODE 0: pack [Co][4][Ci] row co * 4 + t -> LDS
  // row t * Co + co; MODE 1: pack [Ci][4][Co] = [Ci][K] as is
  for (int idx = tid; idx < NN * KS * 4; idx += kCtWaves * 64) {
    const int r = idx / (KS * 4), c = idx - r * (KS * 4);
    const int gr = MODE == 0 ? (r % Co) * 4 + r / Co : r;
    *reinterpret_cast<uint4*>(wl + ct_off(r, c, KB)) = *reinterpret_cast<const uint4*>(a.w + (size_t)gr * K + c * 8);
  }
  if constexpr (MODE == 0) {
    for (int c = tid; c < Co; c += kCtWaves * 64) cst[c] = a.bias ? a.bias[c] : 0.f;
    if (xf) {  // the previous BN's affine map (bn_apply's coefficients, as the ws xform)
      for (int c = tid; c < K; c += kCtWaves * 64) {
        float m, is, var;
        bn_scale_shift(a.xbn, c, xss[c], xss[K + c], m, is, var);
      }
      if (blockIdx.x == 0) bn_finalize(a.xbn);  // saved mean / invstd, running statistics
    }
  } else if constexpr (FB) {
    for (int c = tid; c < NN; c += kCtWaves * 64) {
      cst[c] = a.bb.mean[c];
      cst[NN + c] = a.bb.invstd[c];
    }
  }
  __syncthreads();

  float q0[NT][4], q1[NT][4], bs[NBS][8];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = 0.f;
#pragma unroll
  for (int j = 0; j < NBS; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) bs[j][e] = 0.f;

  for (; g < ngroups; g += nw) {
    if (xf) {  // B holds the raw y: relu(y * scale + shift) in place, stored as the activation
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = (g * MT + mt) * 16 + pl;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int c0 = ks * 32 + kq * 8;
          float v[8];
          unpack8(__builtin_bit_cast(uint4, Bc[mt][ks]), v);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            v[k] = v[k] * xss[c0 + k] + xss[K + c0 + k];
            v[k] = v[k] > 0.f ? v[k] : 0.f;
          }
          const uint4 o = pack8(v);
          Bc[mt][ks] = __builtin_bit_cast(bf16x8, o);
          *reinterpret_cast<uint4*>(a.xh + (size_t)m * a.ldxh + c0) = o;
        }
      }
    }
    if (bsum) {  // bias gradient: lane's channels (ks % NBS) * 32 + 8 kq + e, every tap
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          float v[8];
          unpack8(__builtin_bit_cast(uint4, Bc[mt][ks]), v);
#pragma unroll
          for (int e = 0; e < 8; ++e) bs[ks % NBS][e] += v[e];
        }
    }
    // pixel coordinates of the lane's MT pixels (forward: the output quad)
    size_t pbase[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int m = (g * MT + mt) * 16 + pl;
      if constexpr (MODE == 0) {
        const int n = m / HW, r = m - n * HW, h = r / Wd, w = r - h * Wd;
        pbase[mt] = ((size_t)n * (2 * a.H) + 2 * h) * Q + 2 * w;
      } else {
        pbase[mt] = (size_t)m;
      }
    }
    // one output-channel tile at a time: its MFMAs, then its epilogue (4
    // accumulator registers per pixel tile live, one tile's weight fragments)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 A = *reinterpret_cast<const bf16x8*>(wl + ct_off(nt * 16 + pl, ks * 4 + kq, KB));
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, Bc[mt][ks], acc[mt], 0, 0, 0);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        if constexpr (MODE == 0) {
          const int nn = nt * 16 + kq * 4, t = nn / Co, co = nn - t * Co;
          const f32x4 b = *reinterpret_cast<const f32x4*>(cst + co);
          const size_t op = pbase[mt] + (size_t)(t >> 1) * Q + (t & 1);
          uint2 o;
          o.x = pack_bf2(acc[mt][0] + b[0], acc[mt][1] + b[1]);
          o.y = pack_bf2(acc[mt][2] + b[2], acc[mt][3] + b[3]);
          *reinterpret_cast<uint2*>(a.y + op * a.ldy + co) = o;
        } else {
          const int ci = nt * 16 + kq * 4;
          float v[4] = {acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]};
          if constexpr (FB && !FBTOP) {
            const size_t m = pbase[mt];
            uac[mt][nt] = *reinterpret_cast<const uint2*>(a.bb.act + m * a.bb.ldact + ci);
            uyc[mt][nt] = *reinterpret_cast<const uint2*>(a.bb.y + m * a.bb.ldy + ci);
          }
          if constexpr (FB) {
            float av[4];
            unpack4(uac[mt][nt], av);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (!(av[e] > 0.f)) v[e] = 0.f;
          }
          uint2 o;
          o.x = pack_bf2(v[0], v[1]);
          o.y = pack_bf2(v[2], v[3]);
          *reinterpret_cast<uint2*>(a.y + pbase[mt] * a.ldy + ci) = o;
          if constexpr (FB) {
            float dz[4], yv[4];
            unpack4(o, dz);
            unpack4(uyc[mt][nt], yv);
            const f32x4 mu = *reinterpret_cast<const f32x4*>(cst + ci);
            const f32x4 is = *reinterpret_cast<const f32x4*>(cst + NN + ci);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              q0[nt][e] += dz[e];
              q1[nt][e] += dz[e] * (yv[e] - mu[e]) * is[e];
            }
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (g + nw < ngroups) {
      load_b(g + nw, Bc);
      if constexpr (FBTOP) load_bn(g + nw, uac, uyc);
    }
  }
  if (!FB && !bsum) return;

  // block reduction: 16 pixel lanes, then the waves through LDS; fp64 atomics
  // into replica blockIdx.x % kStatRep (the layouts bn_bwd_reduce_kernel and
  // channel_sum_kernel publish)
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    if constexpr (FB) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          q0[i][e] += __shfl_xor(q0[i][e], o, 64);
          q1[i][e] += __shfl_xor(q1[i][e], o, 64);
        }
    }
    if (bsum) {
#pragma unroll
      for (int j = 0; j < NBS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) bs[j][e] += __shfl_xor(bs[j][e], o, 64);
    }
  }
  if (pl == 0) {
    if constexpr (FB) {
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = i * 16 + kq * 4 + e;
          red[(wave * NN + c) * 2] = q0[i][e];
          red[(wave * NN + c) * 2 + 1] = q1[i][e];
        }
    }
    if (bsum) {
#pragma unroll
      for (int j = 0; j < NBS; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) redb[wave * Co + j * 32 + kq * 8 + e] = bs[j][e];
    }
  }
  __syncthreads();
  const int rep = blockIdx.x % kStatRep;
  if constexpr (FB) {
    for (int c = tid; c < NN; c += kCtWaves * 64) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < kCtWaves; ++w) {
        s0 += red[(w * NN + c) * 2];
        s1 += red[(w * NN + c) * 2 + 1];
      }
      atomicAdd(a.bb.sums + (size_t)rep * 2 * NN + c, (double)s0);
      atomicAdd(a.bb.sums + (size_t)rep * 2 * NN + NN + c, (double)s1);
    }
  }
  if (bsum) {
    for (int c = tid; c < Co; c += kCtWaves * 64) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kCtWaves; ++w) s += redb[w * Co + c];
      atomicAdd(a.bias_acc + (size_t)rep * Co + c, (double)s);
    }
  }
  if constexpr (FB) {
    if (a.bb.ticket && last_block_arrive(a.bb.ticket, gridDim.x, flag, true)) bn_bwd_finalize(a.bb);
  }
}

template <int MODE, int NT, int KS, int MT, bool FB>
static hipError_t convt_cfg(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int NN = NT * 16, K = KS * 32, Co = MODE == 0 ? NN / 4 : K / 4;
  const long long M = (long long)a.N * a.H * a.W;
  if (M % (16 * MT)) return hipErrorNotSupported;
  const int ngroups = (int)(M / (16 * MT));
  const size_t lds = (size_t)NN * K * 2 + 2 * NN * 4 + kCtWaves * NN * 2 * 4 + kCtWaves * Co * 4 + 16 +
                     (MODE == 0 && a.xform ? 2 * K * 4 : 0);
  // the fused form keeps one block per CU: its per-block reduction and fp64
  // atomics amortise over more groups (micro: upconv1 38.6 -> 34.8 us,
  // upconv2 43.8 -> 34.1 us); otherwise as many as LDS allows, up to 4
  const int per_cu = FB ? 1 : std::max(1, std::min(4, (int)((160 * 1024) / lds)));
  int grid = std::min((ngroups + kCtWaves - 1) / kCtWaves, per_cu * device_cu_count());
  if (a.grid_cap > 0) grid = std::min(grid, a.grid_cap);
  char tag[64];
  std::snprintf(tag, sizeof(tag), "convt2x2_kernel<%d, %d, %d, %d, %d>", MODE, NT, KS, MT, FB ? 1 : 0);
  conv_kernel_tag(tag);
  hipLaunchKernelGGL((convt2x2_kernel<MODE, NT, KS, MT, FB>), dim3(grid), dim3(kCtWaves * 64), lds, st, a, ngroups);
  return hipGetLastError();
}

template <int MODE, int NT, int KS>
static hipError_t convt_fb(const ConvFwdArgs& a, hipStream_t st) {
  if constexpr (MODE == 1) {  // the fused BN backward exists in the data gradient only
    if (a.bb.sums) return convt_cfg<MODE, NT, KS, 1, true>(a, st);
  }
  return convt_cfg<MODE, NT, KS, 1, false>(a, st);
}

static bool al16(const void* p) { return ((size_t)p & 15) == 0; }
static bool al8(const void* p) { return ((size_t)p & 7) == 0; }

static bool convt_fwd_covered(int Ci, int Co) {
  return (Ci == 64 && Co == 32) || (Ci == 64 && Co == 64) || (Ci == 128 && Co == 64);
}

// forward with the previous BN + ReLU applied to the pixel operand (xform):
// the shapes and strides launch_convt2x2 takes for it (pointers are checked there)
bool convt2x2_xform_ok(const ConvFwdArgs& a) {
  return convt_fwd_covered(a.C, a.Cout) && (long long)a.N * a.H * a.W % 16 == 0 && a.ldx % 8 == 0 &&
         a.ldxh % 8 == 0 && a.ldy % 4 == 0 && a.N > 0 && a.H > 0 && a.W > 0;
}

hipError_t launch_convt2x2(const ConvFwdArgs& a, int mode, hipStream_t st) {
  if (mode != 0 && mode != 1) return hipErrorInvalidValue;
  if (a.add || a.stats || a.x2 || a.ysplit || a.fold_on || a.bb.y2 || a.wch) return hipErrorNotSupported;
  if (a.xform) {  // forward only, every operand of the fold in place (no fallback takes it)
    if (mode != 0 || !convt2x2_xform_ok(a) || !al16(a.xh) || !a.xbn.stats || a.xbn.C != a.C || a.xbn.ss)
      return hipErrorInvalidValue;
  }
  if (mode == 0 && (a.bb.sums || a.bias_acc)) return hipErrorInvalidValue;
  if (a.N <= 0 || a.H <= 0 || a.W <= 0) return hipErrorInvalidValue;
  // 16-B pixel-operand loads, 8-B result (and BN operand) accesses
  if (!al16(a.x) || !al16(a.w) || a.ldx % 8 || !al8(a.y) || a.ldy % 4) return hipErrorNotSupported;
  if (a.bb.sums && (!al8(a.bb.act) || !al8(a.bb.y) || a.bb.ldact % 4 || a.bb.ldy % 4 || a.bb.C != a.C))
    return hipErrorNotSupported;
  const int Ci = a.C, Co = a.Cout;
  if (mode == 0 && !convt_fwd_covered(Ci, Co)) return hipErrorNotSupported;
  if (mode == 0) {  // NN = 4 Co columns, K = Ci
    if (Ci == 64 && Co == 32) return convt_fb<0, 8, 2>(a, st);
    if (Ci == 64 && Co == 64) return convt_fb<0, 16, 2>(a, st);
    if (Ci == 128 && Co == 64) return convt_fb<0, 16, 4>(a, st);
  } else {  // NN = Ci, K = 4 Co
    if (Ci == 64 && Co == 32) return convt_fb<1, 4, 4>(a, st);
    if (Ci == 64 && Co == 64) return convt_fb<1, 4, 8>(a, st);
    if (Ci == 128 && Co == 64) return convt_fb<1, 8, 8>(a, st);
  }
  return hipErrorNotSupported;
}

// ---------------------------------------------------------------------------
// 1 x 1 / stride-1 convs of the narrow full-resolution attention gates
// (AttentionGate W_g / W_x, advanced_models.py:10-18, applied at :30-31 on the
// 128^2 / 256^2 decoder levels) with the same structure: weights [NN][K]
// staged once per block, the pixel operand straight into the B fragments,
// independent waves.  These launches move 0.1-0.3 GB at K, NN <= 64: the
// implicit-GEMM tiles ran them at 1.5-2.5 TB/s.
//   MODE 0 forward:        Y[m][co] = bias[co] + sum_ci W[co][ci] X[m][ci];
//                          stats != null: BN sums of the fp32 values
//                          (conv_epilogue's), last block finalises with a ticket
//   MODE 1 data gradient:  dX[m][ci] = sum_co W[co][ci] dY[m][co] (+ add[m][ci])
// Both read their pack ([Cout][Ci] forward, [Ci][Cout] dgrad) as [NN][K] rows.
// ---------------------------------------------------------------------------
template <int NT, int KS>
__global__ void __launch_bounds__(kCtWaves * 64) conv1x1_kernel(ConvFwdArgs a, int ngroups) {
  constexpr int NN = NT * 16, K = KS * 32, KB = K * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;                                         // [NN][K] bf16
  float* cst = reinterpret_cast<float*>(smem + NN * KB);  // bias [NN]
  float* red = cst + NN;                                   // [kCtWaves][NN][2]
  int* flag = reinterpret_cast<int*>(red + kCtWaves * NN * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pl = lane & 15, kq = lane >> 4;
  const bool stats = a.stats != nullptr, add = a.add != nullptr;

  // the group's pixel operand and (data gradient) its addend: one round trip
  auto load_b = [&](int g, bf16x8 (&B)[KS], uint2 (&ad)[NT]) {
    const size_t m = (size_t)g * 16 + pl;
    const bf16_t* src = a.x + m * a.ldx + kq * 8;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) B[ks] = *reinterpret_cast<const bf16x8*>(src + ks * 32);
    if (add) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) ad[nt] = *reinterpret_cast<const uint2*>(a.add + m * a.ldadd + nt * 16 + kq * 4);
    }
  };
  const int nw = gridDim.x * kCtWaves;
  int g = blockIdx.x * kCtWaves + wave;
  bf16x8 B[KS];
  uint2 ad[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) ad[nt] = make_uint2(0u, 0u);
  if (g < ngroups) load_b(g, B, ad);  // before the weight staging (independent)
  for (int idx = tid; idx < NN * KS * 4; idx += kCtWaves * 64) {
    const int r = idx / (KS * 4), c = idx - r * (KS * 4);
    *reinterpret_cast<uint4*>(wl + ct_off(r, c, KB)) = *reinterpret_cast<const uint4*>(a.w + (size_t)r * K + c * 8);
  }
  for (int c = tid; c < NN; c += kCtWaves * 64) cst[c] = a.bias ? a.bias[c] : 0.f;
  __syncthreads();

  float q0[NT][4], q1[NT][4];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = 0.f;
  for (; g < ngroups; g += nw) {
    const size_t m = (size_t)g * 16 + pl;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 A = *reinterpret_cast<const bf16x8*>(wl + ct_off(nt * 16 + pl, ks * 4 + kq, KB));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A, B[ks], acc, 0, 0, 0);
      }
      const int c = nt * 16 + kq * 4;
      const f32x4 b = *reinterpret_cast<const f32x4*>(cst + c);
      float v[4] = {acc[0] + b[0], acc[1] + b[1], acc[2] + b[2], acc[3] + b[3]};
      if (add) {
        float r[4];
        unpack4(ad[nt], r);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += r[e];
      }
      uint2 o;
      o.x = pack_bf2(v[0], v[1]);
      o.y = pack_bf2(v[2], v[3]);
      *reinterpret_cast<uint2*>(a.y + m * a.ldy + c) = o;
      if (stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          q0[nt][e] += v[e];
          q1[nt][e] += v[e] * v[e];
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (g + nw < ngroups) load_b(g + nw, B, ad);
  }
  if (!stats) return;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1)
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q0[i][e] += __shfl_xor(q0[i][e], o, 64);
        q1[i][e] += __shfl_xor(q1[i][e], o, 64);
      }
  if (pl == 0) {
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = i * 16 + kq * 4 + e;
        red[(wave * NN + c) * 2] = q0[i][e];
        red[(wave * NN + c) * 2 + 1] = q1[i][e];
      }
  }
  __syncthreads();
  const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * NN;
  for (int c = tid; c < NN; c += kCtWaves * 64) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int w = 0; w < kCtWaves; ++w) {
      s0 += red[(w * NN + c) * 2];
      s1 += red[(w * NN + c) * 2 + 1];
    }
    atomicAdd(a.stats + rep + c, (double)s0);
    atomicAdd(a.stats + rep + NN + c, (double)s1);
  }
  if (a.bn.ticket && last_block_arrive(a.bn.ticket, gridDim.x, flag, true)) bn_finalize(a.bn);
}

template <int NT, int KS>
static hipError_t conv1x1_cfg(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int NN = NT * 16, K = KS * 32;
  const long long M = (long long)a.N * a.H * a.W;
  if (M % 16) return hipErrorNotSupported;
  const int ngroups = (int)(M / 16);
  const size_t lds = (size_t)NN * K * 2 + NN * 4 + kCtWaves * NN * 2 * 4 + 16;
  // with statistics two blocks per CU instead of four: the per-block
  // reduction and its atomics amortise over more groups
  const int per_cu = a.stats ? 2 : 4;
  int grid = std::min((ngroups + kCtWaves - 1) / kCtWaves, per_cu * device_cu_count());
  if (a.grid_cap > 0) grid = std::min(grid, a.grid_cap);
  char tag[48];
  std::snprintf(tag, sizeof(tag), "conv1x1_kernel<%d, %d>", NT, KS);
  conv_kernel_tag(tag);
  hipLaunchKernelGGL((conv1x1_kernel<NT, KS>), dim3(grid), dim3(kCtWaves * 64), lds, st, a, ngroups);
  return hipGetLastError();
}

hipError_t launch_conv1x1(const ConvFwdArgs& a, int mode, hipStream_t st) {
  if (mode != 0 && mode != 1) return hipErrorInvalidValue;
  if (a.R != 1 || a.S != 1 || a.stride != 1 || a.pad != 0 || a.H != a.P || a.W != a.Q) return hipErrorNotSupported;
  if (a.bb.sums || a.x2 || a.ysplit || a.fold_on || a.xform || a.wch || a.wds || a.stride_w) return hipErrorNotSupported;
  if (mode == 1 && (a.stats || a.bias)) return hipErrorNotSupported;
  if (mode == 0 && a.add) return hipErrorNotSupported;
  if (!al16(a.x) || !al16(a.w) || a.ldx % 8 || !al8(a.y) || a.ldy % 4 || (a.add && (!al8(a.add) || a.ldadd % 4)))
    return hipErrorNotSupported;
  // NN = Cout (forward) / the dgrad's output channels; K = the reduction
  const int NN = a.Cout, K = a.C;
  if (NN == 32 && K == 32) return conv1x1_cfg<2, 1>(a, st);
  if (NN == 32 && K == 64) return conv1x1_cfg<2, 2>(a, st);
  if (NN == 64 && K == 32) return conv1x1_cfg<4, 1>(a, st);
  if (NN == 64 && K == 64) return conv1x1_cfg<4, 2>(a, st);
  return hipErrorNotSupported;
}

}  // namespace unet

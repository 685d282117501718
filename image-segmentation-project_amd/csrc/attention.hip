// Attention decoder of UNetWithBackbone(use_attention=True) (SURVEY.md §8(f)
// row 2): the per-pixel / per-channel parts that are not convolutions.
//
//  * AttentionGate (advanced_models.py:7-40): W_g / W_x are 1x1 convs on the
//    implicit-GEMM kernel and relu(BN_g + BN_x) is the two-BN bn_apply_kernel;
//    here: psi = conv1x1(F_int -> 1) with its BN(1) batch sums
//    (att_psi_fwd_kernel), the gate x * sigmoid(BN(psi)) written into the
//    concat slice (att_gate_fwd_kernel), and their backward.
//  * ChannelAttention (advanced_models.py:43-61): per-(n, c) average and max
//    (first-occurrence argmax, as torch's adaptive max pool) pooling, the
//    shared C -> C/16 -> C MLP, sigmoid, channel scale; and their backward.
//
// All of it is HBM-bound elementwise / reduction work: 16-B NHWC accesses
// (8 bf16 channels per lane), per-thread partial sums folded through LDS once
// per block, fp64 atomics for the BN(1) batch sums, fp32 atomics for the
// per-(n, c) pools and the weight gradients.
#include "common.h"
#include "kernels.h"

namespace unet {

namespace {

// sum of two doubles over the 256 threads of a block; result in thread 0
__device__ void block_sum2(double& a, double& b, double* red) {
  const int t = threadIdx.x;
  red[t] = a;
  red[256 + t] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) {
      red[t] += red[t + s];
      red[256 + t] += red[256 + t + s];
    }
    __syncthreads();
  }
  a = red[0];
  b = red[256];
}

__device__ __forceinline__ float sigmoidf(float z) { return 1.f / (1.f + expf(-z)); }

// float -> order-preserving u32 (larger float, larger key); every non-NaN key > 0
__device__ __forceinline__ unsigned ord_key(float f) {
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_value(unsigned long long k) {
  const unsigned o = (unsigned)(k >> 32);
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}
__device__ __forceinline__ unsigned key_index(unsigned long long k) {
  return 0xFFFFFFFFu - (unsigned)(k & 0xFFFFFFFFull);
}

__device__ void bn1_coef(const AttGateArgs& a, float& scale, float& shift, float& mean, float& inv, float& var) {
  if (a.training) {
    const double m = a.pst[0] / a.count;
    double v = a.pst[1] / a.count - m * m;
    if (v < 0.0) v = 0.0;
    mean = (float)m;
    var = (float)v;
  } else {
    mean = a.run_mean[0];
    var = a.run_var[0];
  }
  inv = 1.0f / sqrtf(var + a.eps);
  scale = a.gamma[0] * inv;
  shift = a.beta[0] - mean * scale;
}

}  // namespace

// pixels per lane group and loop pass in the gate kernels: their loads are all
// issued before the pass's math (one pixel per pass kept one load in flight)
constexpr int kAttU = 4;

// sum over the CC lanes of one pixel group (CC | 64, groups lane-aligned)
__device__ __forceinline__ float group_sum(float v, int CC) {
  for (int o = CC >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// p[px] = psi.0(s[px]) = b + sum_c w[c] s[px][c]; BN(1) batch sums (training).
// CC = F_int/8 consecutive lanes share a pixel (one 16-B chunk each, so a
// wave's loads are contiguous rows) and reduce the dot product by shuffles.
__global__ void __launch_bounds__(256) att_psi_fwd_kernel(AttGateArgs a) {
  __shared__ double red[512];
  double ls = 0.0, lq = 0.0;
  const int CC = a.Fi >> 3, ppb = 256 / CC;
  const int chunk = threadIdx.x % CC, prow = threadIdx.x / CC;
  float w[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = a.psi_w[chunk * 8 + k];
  const float bias = a.psi_b[0];
  const int64_t stride = (int64_t)gridDim.x * ppb;
  for (int64_t base = (int64_t)blockIdx.x * ppb + prow; base < a.npix; base += kAttU * stride) {
    uint4 sv[kAttU];  // kAttU pixels' loads in flight before any math
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      sv[u] = px < a.npix ? *reinterpret_cast<const uint4*>(a.s + px * a.lds + chunk * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      float v[8];
      unpack8(sv[u], v);
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) t += v[k] * w[k];
      const float acc = group_sum(t, CC) + bias;  // the whole lane group shares px
      if (chunk == 0 && px < a.npix) {
        a.p[px] = acc;
        ls += acc;
        lq += (double)acc * acc;
      }
    }
  }
  if (!a.training) return;
  block_sum2(ls, lq, red);
  if (threadIdx.x == 0) {
    atomicAdd(a.pst, ls);
    atomicAdd(a.pst + 1, lq);
  }
}

// psi = sigmoid(BN(p)); x_att[px][c] = x[px][c] * psi[px] (into the concat
// slice); block 0 saves mean/invstd and updates the running statistics
__global__ void __launch_bounds__(256) att_gate_fwd_kernel(AttGateArgs a) {
  float sc, sh, mean, inv, var;
  bn1_coef(a, sc, sh, mean, inv, var);
  const int CC = a.Fl >> 3, ppb = 256 / CC;
  const int chunk = threadIdx.x % CC, prow = threadIdx.x / CC;
  const int64_t stride = (int64_t)gridDim.x * ppb;
  for (int64_t base = (int64_t)blockIdx.x * ppb + prow; base < a.npix; base += kAttU * stride) {
    float pv[kAttU];
    uint4 xv[kAttU];
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      const bool in = px < a.npix;
      pv[u] = in ? a.p[px] : 0.f;
      xv[u] = in ? *reinterpret_cast<const uint4*>(a.x + px * a.ldx + chunk * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      if (px >= a.npix) break;
      const float ps = sigmoidf(pv[u] * sc + sh);
      if (chunk == 0) a.psi[px] = ps;
      float v[8];
      unpack8(xv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= ps;
      *reinterpret_cast<uint4*>(a.xatt + px * a.ldxatt + chunk * 8) = pack8(v);
    }
  }
  if (a.training && blockIdx.x == 0 && threadIdx.x == 0) {
    a.save[0] = mean;
    a.save[1] = inv;
    const double n = a.count;
    const float unb = (float)((double)var * (n / (n > 1.0 ? n - 1.0 : 1.0)));
    a.run_mean[0] = (1.f - a.momentum) * a.run_mean[0] + a.momentum * mean;
    a.run_var[0] = (1.f - a.momentum) * a.run_var[0] + a.momentum * unb;
    if (a.nbt) *a.nbt += 1;
  }
}

// backward, pass 1: d_psi = sum_c dXatt x; dZ = d_psi psi (1 - psi) (into
// dbnp); dX (gate path) = dXatt psi; BN(1) sums (sum dZ, sum dZ phat).
// CC = F_l/8 lanes per pixel, as in att_psi_fwd_kernel.
__global__ void __launch_bounds__(256) att_gate_bwd_reduce_kernel(AttGateArgs a) {
  __shared__ double red[512];
  const float mean = a.save[0], inv = a.save[1];
  const int CC = a.Fl >> 3, ppb = 256 / CC;
  const int chunk = threadIdx.x % CC, prow = threadIdx.x / CC;
  double s1 = 0.0, s2 = 0.0;
  const int64_t stride = (int64_t)gridDim.x * ppb;
  for (int64_t base = (int64_t)blockIdx.x * ppb + prow; base < a.npix; base += kAttU * stride) {
    float psv[kAttU], pv[kAttU];
    uint4 dv[kAttU], xv[kAttU];
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      const bool in = px < a.npix;
      psv[u] = in ? a.psi[px] : 0.f;
      pv[u] = in ? a.p[px] : 0.f;
      dv[u] = in ? *reinterpret_cast<const uint4*>(a.dxatt + px * a.lddxatt + chunk * 8) : make_uint4(0, 0, 0, 0);
      xv[u] = in ? *reinterpret_cast<const uint4*>(a.x + px * a.ldx + chunk * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      const bool in = px < a.npix;
      const float ps = psv[u];
      float d[8], v[8];
      unpack8(dv[u], d);
      unpack8(xv[u], v);
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        t += d[k] * v[k];
        d[k] *= ps;
      }
      if (in) *reinterpret_cast<uint4*>(a.dxpsi + px * a.lddxpsi + chunk * 8) = pack8(d);
      const float dpsi = group_sum(t, CC);  // the whole lane group shares px
      if (chunk == 0 && in) {
        const float dz = dpsi * ps * (1.f - ps);
        a.dbnp[px] = dz;
        s1 += dz;
        s2 += (double)dz * ((pv[u] - mean) * inv);
      }
    }
  }
  block_sum2(s1, s2, red);
  if (threadIdx.x == 0) {
    atomicAdd(a.pbs, s1);
    atomicAdd(a.pbs + 1, s2);
  }
}

// backward, pass 2: dp = gamma invstd (dZ - mean dZ - phat mean(dZ phat));
// dS[px][c] = dp w[c] (dA of relu(BN_g + BN_x)); dW_psi[c] = sum dp s[px][c].
// Thread = (8-channel chunk, pixel row) so each keeps 8 weight-gradient partials.
__global__ void __launch_bounds__(256) att_gate_bwd_apply_kernel(AttGateArgs a) {
  extern __shared__ float wred[];  // [rows][Fi]
  const int CC = a.Fi >> 3, rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int c8 = chunk * 8;
  const float mean = a.save[0], inv = a.save[1];
  const double M = a.count;
  const float m1 = (float)(a.pbs[0] / M), m2 = (float)(a.pbs[1] / M);
  const float k1 = a.gamma[0] * inv;
  // fused: dS is stored as dZ = dS * (s > 0) and the BN_g / BN_x backward sums
  // (sum dZ, sum dZ xhat_g, sum dZ xhat_x) are reduced here
  const BnBwdArgs& bb = a.bb;
  const bool fuse = bb.sums != nullptr;
  float w[8], gw[8], s1[8], s2[8], t2[8], mu[8], is[8], mu2[8], is2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[k] = a.psi_w[c8 + k];
    gw[k] = s1[k] = s2[k] = t2[k] = 0.f;
    mu[k] = fuse ? bb.mean[c8 + k] : 0.f;
    is[k] = fuse ? bb.invstd[c8 + k] : 0.f;
    mu2[k] = fuse ? bb.mean2[c8 + k] : 0.f;
    is2[k] = fuse ? bb.invstd2[c8 + k] : 0.f;
  }
  if (row < rows) {
    const int64_t stride = (int64_t)gridDim.x * rows;
    for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.npix; base += kAttU * stride) {
    float pv[kAttU], dbv[kAttU];
    uint4 sv[kAttU], gv[kAttU], xav[kAttU];
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {  // kAttU pixels' operands in flight before any math
      const int64_t px = base + u * stride;
      const bool in = px < a.npix;
      const uint4 z = make_uint4(0, 0, 0, 0);
      pv[u] = in ? a.p[px] : 0.f;
      dbv[u] = in ? a.dbnp[px] : 0.f;
      sv[u] = in ? *reinterpret_cast<const uint4*>(a.s + px * a.lds + c8) : z;
      gv[u] = (in && fuse) ? *reinterpret_cast<const uint4*>(bb.y + px * bb.ldy + c8) : z;
      xav[u] = (in && fuse) ? *reinterpret_cast<const uint4*>(bb.y2 + px * bb.ldy2 + c8) : z;
    }
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t px = base + u * stride;
      if (px >= a.npix) break;
      const float phat = (pv[u] - mean) * inv;
      const float dp = k1 * (dbv[u] - m1 - phat * m2);
      float v[8], o[8];
      unpack8(sv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        gw[k] += dp * v[k];
        o[k] = dp * w[k];
      }
      if (fuse) {
        float g[8], xa[8];
        unpack8(gv[u], g);
        unpack8(xav[u], xa);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          o[k] = v[k] > 0.f ? o[k] : 0.f;
          s1[k] += o[k];
          s2[k] += o[k] * (g[k] - mu[k]) * is[k];
          t2[k] += o[k] * (xa[k] - mu2[k]) * is2[k];
        }
      }
      *reinterpret_cast<uint4*>(a.dS + px * a.lddS + c8) = pack8(o);
    }
    }
  }
  const int nq = fuse ? 4 : 1;
  for (int q = 0; q < nq; ++q) {
    const float* src = q == 0 ? gw : (q == 1 ? s1 : (q == 2 ? s2 : t2));
    if (row < rows) {
#pragma unroll
      for (int k = 0; k < 8; ++k) wred[row * a.Fi + c8 + k] = src[k];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < a.Fi; c += 256) {
      float t = 0.f;
      for (int r = 0; r < rows; ++r) t += wred[r * a.Fi + c];
      if (q == 0) {
        atomicAdd(a.gpsi_acc + (size_t)(blockIdx.x % kStatRep) * a.Fi + c, (double)t);
      } else {
        const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.Fi;
        double* dst = q == 1 ? bb.sums + rep : (q == 2 ? bb.sums + rep + a.Fi : bb.sums2 + rep + a.Fi);
        atomicAdd(dst + c, (double)t);
      }
    }
    __syncthreads();
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    a.ggamma[0] = (float)a.pbs[1];
    a.gbeta[0] = (float)a.pbs[0];
  }
}

// ChannelAttention pooling: per (n, c) sum and (max, first argmax) key
__global__ void __launch_bounds__(256) ch_pool_kernel(ChAttArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int CC = a.C >> 3, rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int n = blockIdx.y;
  unsigned long long* kred = reinterpret_cast<unsigned long long*>(smem);  // [rows][C]
  float* sred = reinterpret_cast<float*>(smem + (size_t)rows * a.C * 8);  // [rows][C]
  if (row < rows) {
    float sum[8], mx[8];
    unsigned arg[8];
    bool any = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) { sum[k] = 0.f; mx[k] = 0.f; arg[k] = 0; }
    const int64_t stride = (int64_t)gridDim.x * rows;
    for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.HW; base += kAttU * stride) {
      uint4 yv[kAttU];  // the pass's loads first; the scan order (hw ascending) is unchanged
#pragma unroll
      for (int u = 0; u < kAttU; ++u) {
        const int64_t hw = base + u * stride;
        yv[u] = hw < a.HW ? *reinterpret_cast<const uint4*>(a.y + (n * a.HW + hw) * a.ldy + chunk * 8)
                          : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kAttU; ++u) {
        const int64_t hw = base + u * stride;
        if (hw >= a.HW) break;
        float v[8];
        unpack8(yv[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          sum[k] += v[k];
          if (!any || v[k] > mx[k]) { mx[k] = v[k]; arg[k] = (unsigned)hw; }
        }
        any = true;
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = chunk * 8 + k;
      sred[row * a.C + c] = sum[k];
      kred[row * a.C + c] = any ? (((unsigned long long)ord_key(mx[k]) << 32) | (0xFFFFFFFFu - arg[k])) : 0ull;
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.C; c += 256) {
    float t = 0.f;
    unsigned long long kk = 0ull;
    for (int r = 0; r < rows; ++r) {
      t += sred[r * a.C + c];
      kk = kk > kred[r * a.C + c] ? kk : kred[r * a.C + c];
    }
    atomicAdd(a.psum + n * a.C + c, (double)t);
    if (kk) atomicMax(a.pkey + n * a.C + c, kk);
  }
}

// the shared MLP on the pooled vectors (one block per image):
// gate = sigmoid(W2 relu(W1 avg) + W2 relu(W1 max))
__global__ void __launch_bounds__(256) ch_mlp_fwd_kernel(ChAttArgs a) {
  extern __shared__ float sm[];  // avg[C] | max[C] | h[2 Cr]
  const int n = blockIdx.x, C = a.C, Cr = a.Cr;
  float* av = sm;
  float* mv = sm + C;
  float* hh = sm + 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    av[c] = (float)a.psum[n * C + c] * a.inv_hw;
    mv[c] = key_value(a.pkey[n * C + c]);
    a.am[(size_t)n * 2 * C + c] = av[c];
    a.am[(size_t)n * 2 * C + C + c] = mv[c];
  }
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * Cr; j += 256) {
    const float* src = j < Cr ? av : mv;
    const float* w1 = a.w1 + (size_t)(j % Cr) * C;
    float t = 0.f;
    for (int c = 0; c < C; ++c) t += w1[c] * src[c];
    t = t > 0.f ? t : 0.f;
    hh[j] = t;
    a.h[(size_t)n * 2 * Cr + j] = t;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const float* w2 = a.w2 + (size_t)c * Cr;
    float o1 = 0.f, o2 = 0.f;
    for (int j = 0; j < Cr; ++j) {
      o1 += w2[j] * hh[j];
      o2 += w2[j] * hh[Cr + j];
    }
    a.gate[n * C + c] = sigmoidf(o1 + o2);
  }
}

// out2 = y * gate[n][c]; grid (blocks, N), a thread keeps one 8-channel chunk
__global__ void __launch_bounds__(256) ch_scale_kernel(ChAttArgs a) {
  const int CC = a.C >> 3, rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int n = blockIdx.y;
  float g[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) g[k] = a.gate[n * a.C + chunk * 8 + k];
  const int64_t stride = (int64_t)gridDim.x * rows;
  for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.HW; base += kAttU * stride) {
    uint4 yv[kAttU];
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t hw = base + u * stride;
      yv[u] = hw < a.HW ? *reinterpret_cast<const uint4*>(a.y + (n * a.HW + hw) * a.ldy + chunk * 8)
                        : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kAttU; ++u) {
      const int64_t hw = base + u * stride;
      if (hw >= a.HW) break;
      float v[8];
      unpack8(yv[u], v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= g[k];
      *reinterpret_cast<uint4*>(a.out + (n * a.HW + hw) * a.ldo + chunk * 8) = pack8(v);
    }
  }
}

// backward: dgate[n][c] = sum_hw dOut2 y
__global__ void __launch_bounds__(256) ch_bwd_reduce_kernel(ChAttArgs a) {
  extern __shared__ float sred[];  // [rows][C]
  const int CC = a.C >> 3, rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int n = blockIdx.y;
  if (row < rows) {
    float t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = 0.f;
    const int64_t stride = (int64_t)gridDim.x * rows;
    for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.HW; base += kAttU * stride) {
      uint4 dv[kAttU], yv[kAttU];
#pragma unroll
      for (int u = 0; u < kAttU; ++u) {
        const int64_t hw = base + u * stride;
        const bool in = hw < a.HW;
        dv[u] = in ? *reinterpret_cast<const uint4*>(a.dout2 + (n * a.HW + hw) * a.lddo2 + chunk * 8) : make_uint4(0, 0, 0, 0);
        yv[u] = in ? *reinterpret_cast<const uint4*>(a.y + (n * a.HW + hw) * a.ldy + chunk * 8) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kAttU; ++u) {  // out-of-range pixels loaded zeros: adding 0 * 0
        float d[8], v[8];
        unpack8(dv[u], d);
        unpack8(yv[u], v);
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] += d[k] * v[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) sred[row * a.C + chunk * 8 + k] = t[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.C; c += 256) {
    float t = 0.f;
    for (int r = 0; r < rows; ++r) t += sred[r * a.C + c];
    atomicAdd(a.dgate + n * a.C + c, (double)t);
  }
}

// backward of the MLP (one block per image): weight gradients (fp32 atomics
// over images) and dL/d(avg | max)
__global__ void __launch_bounds__(256) ch_mlp_bwd_kernel(ChAttArgs a) {
  extern __shared__ float sm[];  // do[C] | dh[2 Cr]
  const int n = blockIdx.x, C = a.C, Cr = a.Cr;
  float* dov = sm;
  float* dh = sm + C;
  const float* h = a.h + (size_t)n * 2 * Cr;
  const float* am = a.am + (size_t)n * 2 * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    const float g = a.gate[n * C + c];
    dov[c] = (float)a.dgate[n * C + c] * g * (1.f - g);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < Cr; j += 256) {
    float t = 0.f;
    for (int c = 0; c < C; ++c) t += a.w2[(size_t)c * Cr + j] * dov[c];
    dh[j] = h[j] > 0.f ? t : 0.f;
    dh[Cr + j] = h[Cr + j] > 0.f ? t : 0.f;
  }
  __syncthreads();
  // per-image weight-gradient terms, fp64 adds into replica n % kStatRep
  // (summed and rounded to fp32 once by d2f: independent of the add order)
  double* acc = a.gw_acc + (size_t)(n % kStatRep) * 2 * C * Cr;
  for (int i = threadIdx.x; i < C * Cr; i += 256) {
    const int c = i / Cr, j = i - c * Cr;
    atomicAdd(acc + i, (double)(dov[c] * (h[j] + h[Cr + j])));                               // W2 [C][Cr]
    atomicAdd(acc + C * Cr + (size_t)j * C + c, (double)(dh[j] * am[c] + dh[Cr + j] * am[C + c]));  // W1 [Cr][C]
  }
  for (int c = threadIdx.x; c < C; c += 256) {
    float ta = 0.f, tm = 0.f;
    for (int j = 0; j < Cr; ++j) {
      const float w = a.w1[(size_t)j * C + c];
      ta += w * dh[j];
      tm += w * dh[Cr + j];
    }
    a.dam[(size_t)n * 2 * C + c] = ta;
    a.dam[(size_t)n * 2 * C + C + c] = tm;
  }
}

// dOut = dOut2 gate + davg / HW + [hw == argmax] dmax; layout as ch_scale_kernel.
// Fused (bb.sums): dOut is dA of the decoder's last BN + ReLU, so store
// dZ = dOut * (out > 0) and reduce (sum dZ, sum dZ xhat) for its backward.
__global__ void __launch_bounds__(256) ch_bwd_apply_kernel(ChAttArgs a) {
  extern __shared__ float red[];  // [rows][C] (fused only)
  const int CC = a.C >> 3, rows = 256 / CC;
  const int chunk = threadIdx.x % CC, row = threadIdx.x / CC;
  const int c8 = chunk * 8;
  const int n = blockIdx.y;
  const BnBwdArgs& bb = a.bb;
  const bool fuse = bb.sums != nullptr;
  float g[8], da[8], dm[8], mu[8], is[8], s1[8], s2[8];
  unsigned arg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int c = c8 + k;
    g[k] = a.gate[n * a.C + c];
    da[k] = a.dam[(size_t)n * 2 * a.C + c] * a.inv_hw;
    dm[k] = a.dam[(size_t)n * 2 * a.C + a.C + c];
    arg[k] = key_index(a.pkey[n * a.C + c]);
    mu[k] = fuse ? bb.mean[c] : 0.f;
    is[k] = fuse ? bb.invstd[c] : 0.f;
    s1[k] = s2[k] = 0.f;
  }
  const int64_t stride = (int64_t)gridDim.x * rows;
  for (int64_t base = (int64_t)blockIdx.x * rows + row; base < a.HW; base += kAttU * stride) {
  uint4 dv[kAttU], av[kAttU], yv[kAttU];
#pragma unroll
  for (int u = 0; u < kAttU; ++u) {  // the pass's operands first
    const int64_t hw = base + u * stride, px = n * a.HW + hw;
    const bool in = hw < a.HW;
    const uint4 z = make_uint4(0, 0, 0, 0);
    dv[u] = in ? *reinterpret_cast<const uint4*>(a.dout2 + px * a.lddo2 + c8) : z;
    av[u] = (in && fuse) ? *reinterpret_cast<const uint4*>(bb.act + px * bb.ldact + c8) : z;
    yv[u] = (in && fuse) ? *reinterpret_cast<const uint4*>(bb.y + px * bb.ldy + c8) : z;
  }
#pragma unroll
  for (int u = 0; u < kAttU; ++u) {
    const int64_t hw = base + u * stride, px = n * a.HW + hw;
    if (hw >= a.HW) break;
    float d[8];
    unpack8(dv[u], d);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = d[k] * g[k] + da[k] + (arg[k] == (unsigned)hw ? dm[k] : 0.f);
    if (fuse) {
      float act[8], y[8];
      unpack8(av[u], act);
      unpack8(yv[u], y);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        d[k] = act[k] > 0.f ? d[k] : 0.f;
        s1[k] += d[k];
        s2[k] += d[k] * (y[k] - mu[k]) * is[k];
      }
    }
    *reinterpret_cast<uint4*>(a.dout + px * a.lddo + c8) = pack8(d);
  }
  }
  if (!fuse) return;
  const size_t rep = (size_t)((blockIdx.y * gridDim.x + blockIdx.x) % kStatRep) * 2 * a.C;
  for (int q = 0; q < 2; ++q) {
    const float* src = q == 0 ? s1 : s2;
#pragma unroll
    for (int k = 0; k < 8; ++k) red[row * a.C + c8 + k] = src[k];
    __syncthreads();
    for (int c = threadIdx.x; c < a.C; c += 256) {
      float t = 0.f;
      for (int r = 0; r < rows; ++r) t += red[r * a.C + c];
      atomicAdd(bb.sums + rep + q * a.C + c, (double)t);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int grid_of(int64_t work, int cap = 2048) {
  int64_t g = (work + 255) / 256;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

hipError_t launch_att_gate(const AttGateArgs& a, int pass, hipStream_t st) {
  // lane groups of F/8 lanes per pixel must tile a wave
  if (a.Fi % 8 || a.Fl % 8 || 64 % (a.Fi / 8) || 64 % (a.Fl / 8) || a.npix <= 0) return hipErrorInvalidValue;
  switch (pass) {
    case 0: hipLaunchKernelGGL(att_psi_fwd_kernel, dim3(grid_of(a.npix * (a.Fi / 8))), dim3(256), 0, st, a); break;
    case 1: hipLaunchKernelGGL(att_gate_fwd_kernel, dim3(grid_of(a.npix * (a.Fl / 8))), dim3(256), 0, st, a); break;
    case 2:
      hipLaunchKernelGGL(att_gate_bwd_reduce_kernel, dim3(grid_of(a.npix * (a.Fl / 8))), dim3(256), 0, st, a);
      break;
    case 3: {
      const int rows = 256 / (a.Fi / 8);
      const int g = (int)std::min<int64_t>(1024, (a.npix + rows * 8 - 1) / (rows * 8));
      hipLaunchKernelGGL(att_gate_bwd_apply_kernel, dim3(g), dim3(256), (size_t)rows * a.Fi * sizeof(float), st, a);
      if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
      return launch_d2f(a.gpsi_acc, a.gpsi_w, a.Fi, st);
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_ch_att(const ChAttArgs& a, int pass, hipStream_t st) {
  if (a.C % 8 || a.C / 8 > 256 || 256 % (a.C / 8) || a.Cr <= 0 || a.HW <= 0 || a.N <= 0) return hipErrorInvalidValue;
  if ((int64_t)a.HW > 0xFFFFFFFEll) return hipErrorInvalidValue;
  const int rows = 256 / (a.C / 8);
  const int per_img = (int)std::min<int64_t>(64, (a.HW + rows * 16 - 1) / (rows * 16));
  // elementwise passes: ~4 pixel rows per thread, <= 2048 blocks in total
  const int ew_img = (int)std::max<int64_t>(1, std::min<int64_t>(2048 / a.N, (a.HW + rows * 4 - 1) / (rows * 4)));
  switch (pass) {
    case 0:
      hipLaunchKernelGGL(ch_pool_kernel, dim3(per_img, a.N), dim3(256), (size_t)rows * a.C * 12, st, a);
      break;
    case 1:
      hipLaunchKernelGGL(ch_mlp_fwd_kernel, dim3(a.N), dim3(256), (size_t)(2 * a.C + 2 * a.Cr) * sizeof(float), st, a);
      break;
    case 2: hipLaunchKernelGGL(ch_scale_kernel, dim3(ew_img, a.N), dim3(256), 0, st, a); break;
    case 3:
      hipLaunchKernelGGL(ch_bwd_reduce_kernel, dim3(per_img, a.N), dim3(256), (size_t)rows * a.C * sizeof(float), st, a);
      break;
    case 4: {
      hipLaunchKernelGGL(ch_mlp_bwd_kernel, dim3(a.N), dim3(256), (size_t)(a.C + 2 * a.Cr) * sizeof(float), st, a);
      if (hipGetLastError() != hipSuccess) return hipErrorLaunchFailure;
      // d2f sums kStatRep replicas of stride n: run it over the [2][C*Cr] pair as one array
      // and split the result into fc.2 and fc.0 -- they are separate tensors, so two launches
      const int n2 = a.C * a.Cr;
      hipError_t e = launch_d2f_strided(a.gw_acc, a.gw2, n2, 2 * n2, st);
      if (e != hipSuccess) return e;
      return launch_d2f_strided(a.gw_acc + n2, a.gw1, n2, 2 * n2, st);
    }
    case 5:
      hipLaunchKernelGGL(ch_bwd_apply_kernel, dim3(ew_img, a.N), dim3(256), a.bb.sums ? (size_t)rows * a.C * 4 : 0, st,
                         a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace unet

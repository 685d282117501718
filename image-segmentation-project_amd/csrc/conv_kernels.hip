// Implicit-GEMM convolution kernels for gfx950 (CDNA4), bf16 NHWC, fp32 accumulate.
//
// One template covers every conv-shaped op on the U-Net hot path
// (SURVEY.md §8(a) rows a2-a6):
//   MODE_FWD   y[n,oh,ow,:] = sum_{r,s} x[n, oh*st-pad+r, ow*st-pad+s, :] . W[:,r,s,:]
//              (3x3 s1/s2 encoder+decoder convs, 1x1 s2 downsample, and the
//              k2s2 convT *dgrad*, which is an ordinary k2s2 conv of dY)
//   MODE_TRANS the transposed (gather) form, output split into stride^2 parity
//              classes so that every tap inside a class is dense (no zero MACs):
//              3x3 s1/s2 conv *dgrad* and the ConvTranspose2d(k2,s2) *forward*.
//   ALOAD_STEM the 7x7/s2 stem: im2col of the fp32 single-channel image built in
//              the loader (K = 49 taps padded to 64).
// GEMM view: D[co][pixel] = sum_k Wp[co][k] * X[pixel][k]; the MFMA A operand
// is the packed weight tile (rows = output channels), B the activation tile
// (cols = pixels), so each lane's accumulator holds 4 consecutive channels of
// one pixel -> 8-byte NHWC stores and per-channel BN sums in the epilogue.
//
// Weight-gradient kernel (conv_wgrad): dW[co][tap][c] = sum_px dY[px][co] *
// X_tap[px][c]; both operands are pixel-major in HBM, so they are staged as
// [pixel][channel] LDS tiles and fed to the MFMA with ds_read_b64_tr_b16
// (hardware transpose, cdna_hip_programming.md T10); split-K over pixels with
// fp32 atomics into a [Cout][R*S*C] accumulator.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace unet {

// template instance of the last conv launch ("name<args>", as rocprofv3 prints
// the kernel symbol) for the per-launch profiler's kernel column
static thread_local char g_kernel_tag[96];
template <typename... T>
static void set_kernel_tag(const char* fmt, T... v) {
  std::snprintf(g_kernel_tag, sizeof(g_kernel_tag), fmt, v...);
}
static void set_kernel_tag(const char* tag) { std::snprintf(g_kernel_tag, sizeof(g_kernel_tag), "%s", tag); }
void conv_kernel_tag(const char* tag) { set_kernel_tag(tag); }
const char* last_kernel_tag() { return g_kernel_tag; }

// ---------------------------------------------------------------------------
// LDS swizzles (cdna_hip_programming.md §2/T2) for ds_read_b128 fragment reads
// of the 16x16x32 MFMA: lane l reads row (l&15), 16-B chunk (l>>4) [+4*kk].
// gfx950 serves ds_read_b128 in four non-contiguous 16-lane groups; both
// swizzles put every group's 16 addresses on 16 distinct 16-B bank slots.
// ---------------------------------------------------------------------------
template <int BK>
__device__ __forceinline__ int frag_off(int row, int chunk) {
  if constexpr (BK == 64) {  // 128-B rows, 8 chunks
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  } else {  // 64-B rows, 4 chunks; g = (0,2,3,1) packed as 0x78
    return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3)) << 4);
  }
}

struct TapIter {
  // MODE_FWD: all R*S taps.  MODE_TRANS: taps r = r0 + st*j valid for class py.
  int r0, s0, nr, ns, st;
};

template <int MODE, int BN, int WM, int WN, int FM, int FN>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs& a, f32x4 (&acc)[FN][FM], char* smem, int m0,
                                              int n0, int Mtot, int py, int px_);

template <int MODE, int ALOAD, int BM, int BN, int BK, int WM, int WN>
__global__ void __launch_bounds__(256)
conv_fwd_kernel(ConvFwdArgs a) {
  constexpr int WTM = BM / WM;  // pixels per wave
  constexpr int WTN = BN / WN;  // channels per wave
  constexpr int FM = WTM / 16;
  constexpr int FN = WTN / 16;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(FM >= 1 && FN >= 1, "fragment tiling");
  constexpr int CPR = BK / 8;                       // 16-B chunks per LDS row
  constexpr int ROWB = BK * 2;                      // bytes per LDS row
  constexpr int A_ROWS_PER_PASS = 256 / CPR;
  constexpr int A_PASSES = (BM + A_ROWS_PER_PASS - 1) / A_ROWS_PER_PASS;
  constexpr int B_PASSES = (BN + A_ROWS_PER_PASS - 1) / A_ROWS_PER_PASS;
  constexpr int A_BYTES = BM * ROWB;
  constexpr int B_BYTES = BN * ROWB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave % WM;
  const int wn = wave / WM;

  // ---- tile coordinates ----
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int nblk = bid % a.nblocks;
  const int mblk = bid / a.nblocks;
  const int cls = blockIdx.z;
  const int st = a.stride;
  const int py = (MODE == MODE_TRANS) ? cls / st : 0;
  const int px_ = (MODE == MODE_TRANS) ? cls % st : 0;
  const int Pc = a.Pc, Qc = a.Qc;
  const int Mtot = a.N * Pc * Qc;
  const int m0 = mblk * BM;
  const int n0 = nblk * BN;

  TapIter ti;
  if constexpr (MODE == MODE_TRANS) {
    ti.st = st;
    ti.r0 = (py + a.pad) % st;
    ti.s0 = (px_ + a.pad) % st;
    ti.nr = (a.R - ti.r0 + st - 1) / st;
    ti.ns = (a.S - ti.s0 + st - 1) / st;
  } else if constexpr (ALOAD == ALOAD_STEM) {
    ti.st = 1; ti.r0 = 0; ti.s0 = 0; ti.nr = 1; ti.ns = 1;  // one K step of 64 taps
  } else {
    ti.st = 1; ti.r0 = 0; ti.s0 = 0; ti.nr = a.R; ti.ns = a.S;
  }
  const int cchunks = (ALOAD == ALOAD_STEM) ? 1 : a.C / BK;
  const int KT = ti.nr * ti.ns * cchunks;
  const int Ktot = (ALOAD == ALOAD_STEM) ? 64 : a.R * a.S * a.C;  // packed weight row length

  // ---- per-thread A-row bookkeeping (fixed rows across K steps) ----
  const int ach = tid % CPR;
  int an[A_PASSES], aa[A_PASSES], ab[A_PASSES];
#pragma unroll
  for (int i = 0; i < A_PASSES; ++i) {
    const int row = tid / CPR + i * A_ROWS_PER_PASS;
    const int m = m0 + row;
    if (row < BM && m < Mtot) {
      const int n = m / (Pc * Qc);
      const int rem = m - n * (Pc * Qc);
      an[i] = n;
      aa[i] = rem / Qc;
      ab[i] = rem - aa[i] * Qc;
    } else {
      an[i] = -1; aa[i] = 0; ab[i] = 0;
    }
  }

  uint4 ra[A_PASSES];
  uint4 rb[B_PASSES];

  auto load_tiles = [&](int kt) {
    const int cc = kt % cchunks;
    const int tap = kt / cchunks;
    const int jr = tap / ti.ns, js = tap - jr * ti.ns;
    const int r = ti.r0 + ti.st * jr;
    const int s = ti.s0 + ti.st * js;
    const int c0 = cc * BK;
    // activations
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      const int row = tid / CPR + i * A_ROWS_PER_PASS;
      if (row < BM && an[i] >= 0) {
        if constexpr (ALOAD == ALOAD_STEM) {
          // im2col of the fp32 image: k = ach*8 + e -> (kr, ks) = (ach, e), ks < 7
          const float* img = reinterpret_cast<const float*>(a.x);
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int kr = ach, ks = e;
            const int ih = aa[i] * st - a.pad + kr;
            const int iw = ab[i] * st - a.pad + ks;
            f[e] = (kr < 7 && ks < 7 && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                       ? img[((size_t)an[i] * a.H + ih) * a.W + iw] : 0.f;
          }
          v = pack8(f);
        } else {
          int ih, iw;
          if constexpr (MODE == MODE_FWD) {
            ih = aa[i] * st - a.pad + r;
            iw = ab[i] * st - a.pad + s;
          } else {
            ih = aa[i] + (py + a.pad - r) / st;
            iw = ab[i] + (px_ + a.pad - s) / st;
          }
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
            const bf16_t* p = a.x + ((size_t)(an[i] * a.H + ih) * a.W + iw) * a.ldx + c0 + ach * 8;
            v = *reinterpret_cast<const uint4*>(p);
          }
        }
      }
      ra[i] = v;
    }
    // packed weights [Cout][Ktot], k = (r*S + s)*C + c
    const int kbase = (ALOAD == ALOAD_STEM) ? 0 : (r * a.S + s) * a.C + c0;
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      const int row = tid / CPR + i * A_ROWS_PER_PASS;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (row < BN && n0 + row < a.Cout) {
        v = *reinterpret_cast<const uint4*>(a.w + (size_t)(n0 + row) * Ktot + kbase + ach * 8);
      }
      rb[i] = v;
    }
  };

  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PASSES; ++i) {
      const int row = tid / CPR + i * A_ROWS_PER_PASS;
      if (row < BM) *reinterpret_cast<uint4*>(As + frag_off<BK>(row, ach)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PASSES; ++i) {
      const int row = tid / CPR + i * A_ROWS_PER_PASS;
      if (row < BN) *reinterpret_cast<uint4*>(Bs + frag_off<BK>(row, ach)) = rb[i];
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (KT > 0) {  // KT == 0: a stride-2 parity class with no taps (1x1 s2 dgrad)
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();

  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tiles(kt + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 wf[FN], xf[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        wf[i] = *reinterpret_cast<const bf16x8*>(Bs + frag_off<BK>(wn * WTN + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < FM; ++j)
        xf[j] = *reinterpret_cast<const bf16x8*>(As + frag_off<BK>(wm * WTM + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_tiles(buf ^ 1);
    __syncthreads();
  }
  conv_epilogue<MODE, BN, WM, WN, FM, FN>(a, acc, smem, m0, n0, Mtot, py, px_);
}

// ---- epilogue: bias, addend, bf16 NHWC store, BN partial sums (fp64 atomics) ----
// Forward (a.stats): per-channel (sum y, sum y^2) of the stored values' fp32
// source.  Fused BN backward (a.bb.sums, dgrad producing dA of a BN+ReLU):
// dZ = dA * (act > 0) is stored instead of dA and (sum dZ, sum dZ*xhat[,
// sum dZ*xhat2]) are accumulated from the stored bf16 dZ, exactly what
// bn_bwd_reduce_kernel would read back.  Either way the block's partials are
// folded over its 16 pixel lanes and WM waves, added into replica
// blockIdx.x % kStatRep, and the last block finalises the BN.
template <int MODE, int BN, int WM, int WN, int FM, int FN>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs& a, f32x4 (&acc)[FN][FM], char* smem, int m0,
                                              int n0, int Mtot, int py, int px_) {
  constexpr int WTM = FM * 16, WTN = FN * 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int st = a.stride, Pc = a.Pc, Qc = a.Qc;
  if constexpr (MODE == MODE_SHUF) {
    // column j = t*Co + co of input pixel (n, pa, pb) -> y[n, 2pa + t/2, 2pb + t%2, co]
    // (+ bias[co]); a lane's 4 consecutive columns share t (Co % 4 == 0)
    const int Co = a.Cout >> 2;
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = m0 + wm * WTM + j * 16 + (lane & 15);
      if (m >= Mtot) continue;
      const int n = m / (Pc * Qc);
      const int rem = m - n * (Pc * Qc);
      const int pa = rem / Qc, pb = rem - pa * Qc;
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int jj = n0 + wn * WTN + i * 16 + ((lane >> 4) << 2);
        if (jj >= a.Cout) continue;
        const int t = jj / Co, co = jj - t * Co;
        const size_t pix = (size_t)(n * a.P + 2 * pa + (t >> 1)) * a.Q + 2 * pb + (t & 1);
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += a.bias[co + e];
        }
        uint2 o;
        o.x = pack_bf2(v[0], v[1]);
        o.y = pack_bf2(v[2], v[3]);
        *reinterpret_cast<uint2*>(a.y + pix * a.ldy + co) = o;
      }
    }
    return;
  }
  const BnBwdArgs& bb = a.bb;
  const bool fbwd = bb.sums != nullptr;
  const bool two = fbwd && bb.y2 != nullptr;
  float q0[FN][4], q1[FN][4], q2[FN][4];
  float mu[FN][4], is[FN][4], mu2[FN][4], is2[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q0[i][e] = q1[i][e] = q2[i][e] = 0.f;
      mu[i][e] = is[i][e] = mu2[i][e] = is2[i][e] = 0.f;
    }
  if (fbwd) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int co = n0 + wn * WTN + i * 16 + ((lane >> 4) << 2);
      if (co < a.Cout) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          mu[i][e] = bb.mean[co + e];
          is[i][e] = bb.invstd[co + e];
          if (two) { mu2[i][e] = bb.mean2[co + e]; is2[i][e] = bb.invstd2[co + e]; }
        }
      }
    }
  }

#pragma unroll
  for (int j = 0; j < FM; ++j) {
    const int m = m0 + wm * WTM + j * 16 + (lane & 15);
    const bool mvalid = m < Mtot;
    size_t pix = 0;
    if (mvalid) {
      const int n = m / (Pc * Qc);
      const int rem = m - n * (Pc * Qc);
      const int pa = rem / Qc, pb = rem - pa * Qc;
      const int oh = (MODE == MODE_TRANS) ? pa * st + py : pa;
      const int ow = (MODE == MODE_TRANS) ? pb * st + px_ : pb;
      pix = (size_t)(n * a.P + oh) * a.Q + ow;
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int co = n0 + wn * WTN + i * 16 + ((lane >> 4) << 2);
      if (mvalid && co < a.Cout) {
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if (a.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += a.bias[co + e];
        }
        if (a.fold_on) {  // eval BN folded into the epilogue (running statistics)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float sc, sh, m_, is_, var_;
            bn_scale_shift(a.fold, co + e, sc, sh, m_, is_, var_);
            v[e] = v[e] * sc + sh;
          }
        }
        if (a.add) {
          const uint2 u = *reinterpret_cast<const uint2*>(a.add + pix * a.ldadd + co);
          v[0] += __uint_as_float(u.x << 16); v[1] += __uint_as_float(u.x & 0xffff0000u);
          v[2] += __uint_as_float(u.y << 16); v[3] += __uint_as_float(u.y & 0xffff0000u);
        }
        if (a.fold_relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        if (fbwd) {  // ReLU mask of the BN's forward output
          const uint2 u = *reinterpret_cast<const uint2*>(bb.act + pix * bb.ldact + co);
          if (!(__uint_as_float(u.x << 16) > 0.f)) v[0] = 0.f;
          if (!(__uint_as_float(u.x & 0xffff0000u) > 0.f)) v[1] = 0.f;
          if (!(__uint_as_float(u.y << 16) > 0.f)) v[2] = 0.f;
          if (!(__uint_as_float(u.y & 0xffff0000u) > 0.f)) v[3] = 0.f;
        }
        uint2 o;
        o.x = pack_bf2(v[0], v[1]);
        o.y = pack_bf2(v[2], v[3]);
        if (a.ysplit && co >= a.csplit) *reinterpret_cast<uint2*>(a.ysplit + pix * a.ldysplit + co - a.csplit) = o;
        else *reinterpret_cast<uint2*>(a.y + pix * a.ldy + co) = o;
        if (fbwd) {
          const float dz[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                               __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
          const uint2 u = *reinterpret_cast<const uint2*>(bb.y + pix * bb.ldy + co);
          const float yv[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                               __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
#pragma unroll
          for (int e = 0; e < 4; ++e) { q0[i][e] += dz[e]; q1[i][e] += dz[e] * (yv[e] - mu[i][e]) * is[i][e]; }
          if (two) {
            const uint2 w = *reinterpret_cast<const uint2*>(bb.y2 + pix * bb.ldy2 + co);
            const float y2[4] = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                 __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
#pragma unroll
            for (int e = 0; e < 4; ++e) q2[i][e] += dz[e] * (y2[e] - mu2[i][e]) * is2[i][e];
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) { q0[i][e] += v[e]; q1[i][e] += v[e] * v[e]; }
        }
      }
    }
  }

  if (a.stats || fbwd) {
    // reduce over the 16 pixel lanes sharing (lane>>4), then over the WM waves
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          q0[i][e] += __shfl_xor(q0[i][e], o, 64);
          q1[i][e] += __shfl_xor(q1[i][e], o, 64);
          if (two) q2[i][e] += __shfl_xor(q2[i][e], o, 64);
        }
      }
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][3]
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int cl = wn * WTN + i * 16 + ((lane >> 4) << 2) + e;
          red[(wm * BN + cl) * 3 + 0] = q0[i][e];
          red[(wm * BN + cl) * 3 + 1] = q1[i][e];
          red[(wm * BN + cl) * 3 + 2] = q2[i][e];
        }
    }
    __syncthreads();
    for (int cl = tid; cl < BN; cl += blockDim.x) {
      const int co = n0 + cl;
      if (co < a.Cout) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int w = 0; w < WM; ++w) {
          s0 += red[(w * BN + cl) * 3];
          s1 += red[(w * BN + cl) * 3 + 1];
          s2 += red[(w * BN + cl) * 3 + 2];
        }
        const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout;
        double* dst = fbwd ? bb.sums + rep : a.stats + rep;
        atomicAdd(dst + co, (double)s0);
        atomicAdd(dst + a.Cout + co, (double)s1);
        if (two) atomicAdd(bb.sums2 + rep + a.Cout + co, (double)s2);
      }
    }
    unsigned* ticket = fbwd ? bb.ticket : a.bn.ticket;
    if (ticket) {
      const unsigned total = gridDim.x * gridDim.y * gridDim.z;
      int* flag = reinterpret_cast<int*>(smem + WM * BN * 3 * sizeof(float));
      if (last_block_arrive(ticket, total, flag, tid < BN)) {
        if (fbwd) bn_bwd_finalize(bb);
        else bn_finalize(a.bn);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-DMA pipelined implicit GEMM (the production fwd / dgrad kernel).
//
// Both operand tiles are filled by buffer_load_dwordx4 ... lds (no VGPR
// staging): lane l of a wave instruction writes 16 B at base + 16*l, i.e. one
// instruction fills 1 KiB = 1024/(2*BK) consecutive tile rows.  The XOR
// swizzle of frag_off is applied on the SOURCE side (lane -> logical chunk)
// so the LDS image is exactly the one the fragment reads expect
// (cdna_hip_programming.md §5.4 rule 21).  Conv padding / tile tails use a
// buffer offset beyond num_records, which the hardware range check turns into
// zeros in LDS.  NS stages are kept in flight with a counted vmcnt and raw
// s_barrier (never __syncthreads inside the loop: its vmcnt(0) would drain
// the pipeline).
// ---------------------------------------------------------------------------
// kOOB, wait_vmcnt, make_rsrc, glds16: common.h

template <int BK>
__device__ __forceinline__ int swz_chunk(int row, int p) {  // physical slot p -> logical chunk (involution)
  if constexpr (BK == 64) return p ^ ((row >> 1) & 7);
  else return p ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3);
}

// DS (MODE_FWD): the block's 1x1 / stride-2 downsample (ConvFwdArgs::wds) rides
// along: its weight tile [BN][C] is staged once (cchunks sub-tiles behind the
// pipeline stages) and multiplied with the centre tap's A stages, whose pixels
// (2 oh, 2 ow) are exactly the downsample's input; a second accumulator set and
// a second epilogue (yds, its BN sums).  The separate downsample launch and its
// re-read of the input disappear.
template <int MODE, int BM, int BN, int BK, int NS, int WM, int WN, bool DS = false>
__global__ void __launch_bounds__(WM * WN * 64)
conv_glds_kernel(ConvFwdArgs a) {
  constexpr int NW = WM * WN;          // 4 or 8 waves
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert((NW == 4 || NW == 8) && FM >= 1 && FN >= 1, "tiling");
  constexpr int CPR = BK / 8;          // 16-B chunks per row
  constexpr int ROWB = BK * 2;
  constexpr int RPI = 1024 / ROWB;     // rows per wave instruction
  constexpr int A_INS = BM / RPI / NW; // per wave per stage
  constexpr int B_INS = (BN / RPI + NW - 1) / NW;
  static_assert(BM % (RPI * NW) == 0, "A rows per wave");
  constexpr int LPS = A_INS + B_INS;   // vm ops per wave per stage
  constexpr int A_BYTES = BM * ROWB;
  constexpr int B_BYTES = ((BN + RPI * NW - 1) / (RPI * NW)) * RPI * NW * ROWB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int nblk = bid % a.nblocks, mblk = bid / a.nblocks;
  const int cls = blockIdx.z, st = a.stride;
  const int py = (MODE == MODE_TRANS) ? cls / st : 0;
  const int px_ = (MODE == MODE_TRANS) ? cls % st : 0;
  const int Pc = a.Pc, Qc = a.Qc;
  const int Mtot = a.N * Pc * Qc;
  const int m0 = mblk * BM, n0 = nblk * BN;
  TapIter ti;
  if constexpr (MODE == MODE_TRANS) {
    ti.st = st;
    ti.r0 = (py + a.pad) % st;
    ti.s0 = (px_ + a.pad) % st;
    ti.nr = (a.R - ti.r0 + st - 1) / st;
    ti.ns = (a.S - ti.s0 + st - 1) / st;
  } else {
    ti.st = 1; ti.r0 = 0; ti.s0 = 0; ti.nr = a.R; ti.ns = a.S;
  }
  const int cchunks = a.C / BK;
  const int KT1 = ti.nr * ti.ns * cchunks;
  // folded downsample dgrad: class 0 continues its K loop over x2 / w2
  const bool ext = MODE == MODE_TRANS && a.x2 != nullptr && cls == 0;
  const int KT = KT1 + (ext ? a.C2 / BK : 0);
  const int Ktot = a.R * a.S * a.C;
  static_assert(!DS || MODE == MODE_FWD, "the downsample fold is a forward");
  const int ctap = DS ? (a.R / 2) * a.S + a.S / 2 : -1;  // centre tap (stride-2, pad-1 3x3: pixel (2 oh, 2 ow))
  char* const W2 = smem + NS * STAGE;                        // DS: [cchunks][B tile]
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (unsigned)((size_t)a.Cout * Ktot * 2));
  const __amdgpu_buffer_rsrc_t x2r = make_rsrc(ext ? a.x2 : a.x, ext ? (unsigned)((size_t)a.N * a.H * a.W * a.ldx2 * 2) : 0u);
  const __amdgpu_buffer_rsrc_t w2r = make_rsrc(ext ? a.w2 : a.w, ext ? (unsigned)((size_t)a.Cout * a.C2 * 2) : 0u);

  // lane geometry inside one wave instruction
  const int lrow = lane / CPR, lslot = lane % CPR;
  int an[A_INS], aa[A_INS], ab[A_INS], ach[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wave * A_INS + j) * RPI + lrow;
    ach[j] = swz_chunk<BK>(row, lslot);
    const int m = m0 + row;
    if (m < Mtot) {
      const int n = m / (Pc * Qc);
      const int rem = m - n * (Pc * Qc);
      an[j] = n;
      aa[j] = rem / Qc;
      ab[j] = rem - aa[j] * Qc;
    } else {
      an[j] = -1; aa[j] = 0; ab[j] = 0;
    }
  }
  int bch[B_INS];
  unsigned bbase[B_INS], bbase2[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wave * B_INS + j) * RPI + lrow;
    bch[j] = swz_chunk<BK>(row, lslot);
    const bool ok = row < BN && n0 + row < a.Cout;
    int wrow = n0 + row;  // packed weight row of GEMM column n0 + row
    if constexpr (MODE == MODE_SHUF) {  // column t*Co + co -> convT pack row co*4 + t
      const int Co = a.Cout >> 2, t = wrow / Co;
      wrow = (wrow - t * Co) * 4 + t;
    }
    bbase[j] = ok ? (unsigned)(wrow * Ktot) * 2u : kOOB;
    bbase2[j] = ok ? (unsigned)((n0 + row) * a.C2) * 2u : kOOB;
  }

  auto issue = [&](int kt, int buf) {
    if (ext && kt >= KT1) {  // downsample range: x2 at the class-0 pixel (aa, ab) itself
      const int c0 = (kt - KT1) * BK;
      char* As = smem + buf * STAGE;
      char* Bs = As + A_BYTES;
#pragma unroll
      for (int j = 0; j < A_INS; ++j) {
        unsigned off = kOOB;
        if (an[j] >= 0) off = (unsigned)(((an[j] * a.H + aa[j]) * a.W + ab[j]) * a.ldx2 + c0 + ach[j] * 8) * 2u;
        glds16(x2r, As + (wave * A_INS + j) * 1024, off);
      }
#pragma unroll
      for (int j = 0; j < B_INS; ++j) {
        const unsigned off = bbase2[j] == kOOB ? kOOB : bbase2[j] + (unsigned)(c0 + bch[j] * 8) * 2u;
        glds16(w2r, Bs + (wave * B_INS + j) * 1024, off);
      }
      return;
    }
    const int cc = kt % cchunks;
    const int tap = kt / cchunks;
    const int jr = tap / ti.ns, js = tap - jr * ti.ns;
    const int r = ti.r0 + ti.st * jr, s = ti.s0 + ti.st * js;
    const int c0 = cc * BK;
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      int ih, iw;
      if constexpr (MODE != MODE_TRANS) {  // MODE_FWD, MODE_SHUF (1x1 over the input grid)
        ih = aa[j] * st - a.pad + r;
        iw = ab[j] * (a.stride_w ? a.stride_w : st) - a.pad + s;
      } else {
        ih = aa[j] + (py + a.pad - r) / st;
        iw = ab[j] + (px_ + a.pad - s) / st;
      }
      unsigned off = kOOB;
      if (an[j] >= 0 && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
        off = (unsigned)(((an[j] * a.H + ih) * a.W + iw) * a.ldx + c0 + ach[j] * 8) * 2u;
      glds16(xr, As + (wave * A_INS + j) * 1024, off);
    }
    const int kb = (r * a.S + s) * a.C + c0;
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const unsigned off = bbase[j] == kOOB ? kOOB : bbase[j] + (unsigned)(kb + bch[j] * 8) * 2u;
      glds16(wr, Bs + (wave * B_INS + j) * 1024, off);
    }
  };

  f32x4 acc[FN][FM];
  f32x4 acc2[DS ? FN : 1][DS ? FM : 1];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (DS) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the downsample weight tile, every K sub-tile, before the first stage
    // (older than it: the first stage's counted wait covers these loads)
    const __amdgpu_buffer_rsrc_t wdr = make_rsrc(a.wds, (unsigned)((size_t)a.Cout * a.C * 2));
    for (int cc = 0; cc < cchunks; ++cc) {
#pragma unroll
      for (int j = 0; j < B_INS; ++j) {
        const int row = (wave * B_INS + j) * RPI + lrow;  // downsample pack row n0 + row: [Cout][C]
        const bool ok = row < BN && n0 + row < a.Cout;
        const unsigned off = ok ? (unsigned)((n0 + row) * a.C + cc * BK + bch[j] * 8) * 2u : kOOB;
        glds16(wdr, W2 + cc * B_BYTES + (wave * B_INS + j) * 1024, off);
      }
    }
  }

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT) issue(s, s);

  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = KT - 1 - kt;  // stages issued after kt (capped at NS-2)
    if (ahead >= NS - 2) wait_vmcnt<(NS - 2) * LPS>();
    else if (NS > 3 && ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < KT) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const char* As = smem + (kt % NS) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 wf[FN], xf[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        wf[i] = *reinterpret_cast<const bf16x8*>(Bs + frag_off<BK>(wn * WTN + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < FM; ++j)
        xf[j] = *reinterpret_cast<const bf16x8*>(As + frag_off<BK>(wm * WTM + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
      if constexpr (DS) {
        if (kt / cchunks == ctap) {  // the centre tap's A tile x the downsample weights
          const char* Ws = W2 + (kt % cchunks) * B_BYTES;
#pragma unroll
          for (int i = 0; i < FN; ++i) {
            const bf16x8 w2 = *reinterpret_cast<const bf16x8*>(Ws + frag_off<BK>(wn * WTN + i * 16 + (lane & 15), ch));
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2, xf[j], acc2[i][j], 0, 0, 0);
          }
        }
      }
    }
  }
  wait_vmcnt<0>();
  __syncthreads();
  conv_epilogue<MODE, BN, WM, WN, FM, FN>(a, acc, smem, m0, n0, Mtot, py, px_);
  if constexpr (DS) {
    ConvFwdArgs d = a;  // the downsample's epilogue: its output and BN sums, no bias
    d.y = a.yds; d.ldy = a.ldyds;
    d.stats = a.stats_ds; d.bn = a.bnds;
    d.bias = nullptr; d.add = nullptr; d.fold_on = 0;
    __syncthreads();  // the first epilogue's LDS reduction is read
    conv_epilogue<MODE, BN, WM, WN, FM, FN>(d, acc2, smem, m0, n0, Mtot, py, px_);
  }
}

// ---------------------------------------------------------------------------
// fp8 (OCP e4m3) implicit-GEMM forward conv (BASELINE configs[4]).  The
// MODE_FWD LDS-DMA pipeline with 128-channel fp8 K tiles: a tile row is 128 B,
// the same byte image and swizzle as a 64-channel bf16 tile, so staging,
// padding (kOOB zero-fill, also for the channel tail of C % 128) and the
// epilogue are unchanged.  v_mfma_scale_f32_16x16x128_f8f6f4 (format 0 = e4m3
// for both operands): each lane feeds 32 consecutive K bytes of its row (two
// 16-B chunks, 2g and 2g+1 for lane group g) — the same k assignment for A
// and B, so the dot product covers the K tile whatever the hardware's internal
// k order — at 2x the bf16 MFMA rate; the per-tensor power-of-two scales are
// its e8m0 block scales (fp8.hip), so the accumulators hold the fp32 conv.
// ---------------------------------------------------------------------------
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int BM, int BN, int NS, int WM, int WN>
__global__ void __launch_bounds__(WM * WN * 64)
conv_f8_kernel(ConvFwdArgs a) {
  constexpr int BK = 128;              // e4m3 elements (= bytes) per K tile row
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int FM = WTM / 16, FN = WTN / 16;
  static_assert((NW == 4 || NW == 8) && FM >= 1 && FN >= 1, "tiling");
  constexpr int CPR = 8;               // 16-B chunks per row
  constexpr int RPI = 8;               // rows per wave instruction
  constexpr int A_INS = BM / RPI / NW;
  constexpr int B_INS = (BN / RPI + NW - 1) / NW;
  static_assert(BM % (RPI * NW) == 0, "A rows per wave");
  constexpr int LPS = A_INS + B_INS;
  constexpr int A_BYTES = BM * BK;
  constexpr int B_BYTES = ((BN + RPI * NW - 1) / (RPI * NW)) * RPI * NW * BK;
  constexpr int STAGE = A_BYTES + B_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int nblk = bid % a.nblocks, mblk = bid / a.nblocks;
  const int Mtot = a.N * a.P * a.Q;
  const int m0 = mblk * BM, n0 = nblk * BN;
  const int cchunks = (a.C + BK - 1) / BK;
  const int KT = a.R * a.S * cchunks;
  const int Ktot = a.R * a.S * a.C;
  const int sx = a.f8x->code, sw = a.f8w->code;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (unsigned)((size_t)a.Cout * Ktot));

  const int lrow = lane / CPR, lslot = lane % CPR;
  int an[A_INS], aa[A_INS], ab[A_INS], ach[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wave * A_INS + j) * RPI + lrow;
    ach[j] = swz_chunk<64>(row, lslot);
    const int m = m0 + row;
    if (m < Mtot) {
      const int n = m / (a.P * a.Q);
      const int rem = m - n * (a.P * a.Q);
      an[j] = n;
      aa[j] = rem / a.Q;
      ab[j] = rem - aa[j] * a.Q;
    } else {
      an[j] = -1; aa[j] = 0; ab[j] = 0;
    }
  }
  int bch[B_INS];
  unsigned bbase[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = (wave * B_INS + j) * RPI + lrow;
    bch[j] = swz_chunk<64>(row, lslot);
    const bool ok = row < BN && n0 + row < a.Cout;
    bbase[j] = ok ? (unsigned)((n0 + row) * Ktot) : kOOB;
  }

  auto issue = [&](int kt, int buf) {
    const int cc = kt % cchunks;
    const int tap = kt / cchunks;
    const int r = tap / a.S, s = tap - r * a.S;
    const int c0 = cc * BK;
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const int ih = aa[j] * a.stride - a.pad + r;
      const int iw = ab[j] * a.stride - a.pad + s;
      const int c = c0 + ach[j] * 16;
      unsigned off = kOOB;
      if (an[j] >= 0 && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W && c < a.C)
        off = (unsigned)(((an[j] * a.H + ih) * a.W + iw) * a.ldx + c);
      glds16(xr, As + (wave * A_INS + j) * 1024, off);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int c = c0 + bch[j] * 16;
      const unsigned off = (bbase[j] == kOOB || c >= a.C) ? kOOB : bbase[j] + (unsigned)((r * a.S + s) * a.C + c);
      glds16(wr, Bs + (wave * B_INS + j) * 1024, off);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int j = 0; j < FM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < KT) issue(st, st);

  const int g = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = KT - 1 - kt;
    if (ahead >= NS - 2) wait_vmcnt<(NS - 2) * LPS>();
    else if (NS > 3 && ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt + NS - 1 < KT) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const char* As = smem + (kt % NS) * STAGE;
    const char* Bs = As + A_BYTES;
    // all FM pixel fragments, then one weight fragment at a time (register budget)
    i32x8 xf[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int row = wm * WTM + j * 16 + (lane & 15);
      const uint4 lo = *reinterpret_cast<const uint4*>(As + frag_off<64>(row, 2 * g));
      const uint4 hi = *reinterpret_cast<const uint4*>(As + frag_off<64>(row, 2 * g + 1));
      xf[j] = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int row = wn * WTN + i * 16 + (lane & 15);
      const uint4 lo = *reinterpret_cast<const uint4*>(Bs + frag_off<64>(row, 2 * g));
      const uint4 hi = *reinterpret_cast<const uint4*>(Bs + frag_off<64>(row, 2 * g + 1));
      const i32x8 wf = i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
#pragma unroll
      for (int j = 0; j < FM; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf, xf[j], acc[i][j], 0, 0, 0, sw, 0, sx);
    }
  }
  wait_vmcnt<0>();
  __syncthreads();
  ConvFwdArgs e = a;
  e.Pc = a.P; e.Qc = a.Q;
  conv_epilogue<MODE_FWD, BN, WM, WN, FM, FN>(e, acc, smem, m0, n0, Mtot, 0, 0);
}

// ---------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------
// [pixel][channel] tile, 32-B units XOR-swizzled per row so that every
// ds_read_b64_tr_b16 half-wave (rows {8g..8g+3} x 2 groups) and every
// ds_write_b128 row sweep is bank-conflict free.
template <int TC>  // channels per tile row: 32 or 64 per panel
__device__ __forceinline__ int tr_off(int row, int col) {
  if constexpr (TC == 32) {
    const int unit = col >> 4;
    return row * 64 + (((unit ^ ((row >> 3) & 1))) << 5) + ((col & 15) << 1);
  } else {
    const int panel = col >> 6;
    const int c = col & 63;
    const int unit = c >> 4;
    const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    (void)panel;
    return row * 128 + ((unit ^ f) << 5) + ((c & 15) << 1);
  }
}

template <int TC, int NCOL, int ROWS>
struct TrTile {
  // byte offset of (row, col) inside a tile of ROWS rows x NCOL channels,
  // made of NCOL/TC panels of TC channels each.
  static __device__ __forceinline__ int off(int row, int col) {
    const int panel = col / TC;
    return panel * (ROWS * TC * 2) + tr_off<TC>(row, col % TC);
  }
};

__device__ __forceinline__ bf16x8 tr_read8(const char* base_lo, const char* base_hi) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base_lo));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, base_hi));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <int XLOAD, int BMO, int BNC, int BKP, int WM, int WN>
__global__ void __launch_bounds__(256)
conv_wgrad_kernel(ConvWgradArgs a) {
  constexpr int TCA = BMO >= 64 ? 64 : 32;
  constexpr int TCB = BNC >= 64 ? 64 : 32;
  constexpr int WTM = BMO / WM;
  constexpr int WTN = BNC / WN;
  constexpr int FM = WTM / 16;
  constexpr int FN = WTN / 16;
  static_assert(WM * WN == 4, "4 waves");
  constexpr int A_BYTES = BKP * BMO * 2;
  constexpr int B_BYTES = BKP * BNC * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int ACPR = BMO / 8;  // 16-B chunks per dY pixel row
  constexpr int BCPR = BNC / 8;
  constexpr int A_LOADS = (BKP * ACPR + 255) / 256;
  constexpr int B_LOADS = (BKP * BCPR + 255) / 256;
  typedef TrTile<TCA, BMO, BKP> TA;
  typedef TrTile<TCB, BNC, BKP> TB;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave % WM, wn = wave / WM;
  const int cob = blockIdx.x % a.co_blocks;
  const int rest = blockIdx.x / a.co_blocks;
  const int cblk = rest % a.c_blocks;
  const int tap = rest / a.c_blocks;
  const int co0 = cob * BMO;
  const int c0 = cblk * BNC;
  const int r = (XLOAD == XLOAD_STEM) ? 0 : tap / a.S;
  const int s = (XLOAD == XLOAD_STEM) ? 0 : tap - r * a.S;
  const int PQ = a.P * a.Q;
  const int Mtot = a.N * PQ;
  const int mbeg = blockIdx.z * a.px_per_split;
  const int mend = min(Mtot, mbeg + a.px_per_split);
  const int KT = (mend - mbeg + BKP - 1) / BKP;

  uint4 ra[A_LOADS], rb[B_LOADS];

  auto load_tiles = [&](int kt) {
    const int kb = mbeg + kt * BKP;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / ACPR, ch = idx % ACPR;
      uint4 v = make_uint4(0, 0, 0, 0);
      const int m = kb + row;
      if (row < BKP && m < mend && co0 + ch * 8 < a.Cout)
        v = *reinterpret_cast<const uint4*>(a.dy + (size_t)m * a.lddy + co0 + ch * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / BCPR, ch = idx % BCPR;
      uint4 v = make_uint4(0, 0, 0, 0);
      const int m = kb + row;
      if (row < BKP && m < mend) {
        const int n = m / PQ;
        const int rem = m - n * PQ;
        const int p = rem / a.Q, q = rem - p * a.Q;
        if constexpr (XLOAD == XLOAD_STEM) {
          const float* img = reinterpret_cast<const float*>(a.x);
          float f[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const int k = c0 + ch * 8 + e;
            const int kr = k >> 3, ks = k & 7;  // stem K layout: k = kr*8 + ks, ks < 7
            const int ih = p * a.stride - a.pad + kr, iw = q * a.stride - a.pad + ks;
            f[e] = (kr < 7 && ks < 7 && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
                       ? img[((size_t)n * a.H + ih) * a.W + iw] : 0.f;
          }
          v = pack8(f);
        } else if constexpr (XLOAD == XLOAD_SHUF) {
          const int c = c0 + ch * 8, Co = a.C >> 2;
          if (c < a.C) {
            const int t = c / Co, co = c - t * Co;
            const int ih = 2 * p + (t >> 1), iw = 2 * q + (t & 1);
            v = *reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + ih) * a.W + iw) * a.ldx + co);
          }
        } else {
          const int ih = p * a.stride - a.pad + r, iw = q * a.stride - a.pad + s;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W && c0 + ch * 8 < a.C)
            v = *reinterpret_cast<const uint4*>(a.x + ((size_t)(n * a.H + ih) * a.W + iw) * a.ldx + c0 + ch * 8);
        }
      }
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / ACPR, ch = idx % ACPR;
      if (row < BKP) *reinterpret_cast<uint4*>(As + TA::off(row, ch * 8)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const int idx = tid + i * 256;
      const int row = idx / BCPR, ch = idx % BCPR;
      if (row < BKP) *reinterpret_cast<uint4*>(Bs + TB::off(row, ch * 8)) = rb[i];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (KT > 0) {
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();
  const int g = lane >> 4, li = lane & 15;
  const int trq = li >> 2, trp = li & 3;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load_tiles(kt + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < BKP / 32; ++kk) {
      const int row_lo = kk * 32 + 8 * g + trq;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * WTM + i * 16 + 4 * trp;
        af[i] = tr_read8(As + TA::off(row_lo, col), As + TA::off(row_lo + 4, col));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * WTN + j * 16 + 4 * trp;
        bfr[j] = tr_read8(Bs + TB::off(row_lo, col), Bs + TB::off(row_lo + 4, col));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store_tiles(buf ^ 1);
    __syncthreads();
  }
  if (a.slab && gridDim.z > 1) {  // this split's partial, register-native (SlabLayout SLAB_GEMM)
    const size_t units = (size_t)gridDim.x * 4 * FM * FN * 64;
    f32x4* dst = reinterpret_cast<f32x4*>(a.slab) + (size_t)blockIdx.z * units +
                 ((size_t)blockIdx.x * 4 + wave) * (FM * FN * 64) + lane;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) dst[(i * FN + j) * 64] = acc[i][j];
    return;
  }
  if (KT == 0 && !a.slab) return;

  // D[co][c]: lane holds column c = .. + li, rows co = .. + 4g + e.  One split
  // with a slab: this block owns its dW tile (plain stores); else fp32 atomics
  const int Krow = (XLOAD == XLOAD_STEM) ? 64 : a.R * a.S * a.C;
  const int kcol0 = (XLOAD == XLOAD_STEM) ? 0 : tap * a.C;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = c0 + wn * WTN + j * 16 + li;
      const int cmax = (XLOAD == XLOAD_STEM) ? 64 : a.C;
      if (c < cmax) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int co = co0 + wm * WTM + i * 16 + 4 * g + e;
          if (co < a.Cout) {
            float* d = a.dw + (size_t)co * Krow + kcol0 + c;
            if (a.slab) *d = acc[i][j][e];
            else atomicAdd(d, acc[i][j][e]);
          }
        }
      }
    }
}

// ---------------------------------------------------------------------------
// 3x3 stride-1 weight gradient with an LDS input halo (all 9 taps per block).
//
// Block = 64 output channels x CI input channels x 9 taps (CI = 32: 4 waves,
// CI = 64: 8 waves; each wave owns 32 co x 16 ci x 9 taps = 72 fp32 acc/lane)
// and a split-K range of TH x TW pixel tiles.  Per tile one LDS-DMA stage
// holds dY [TH*TW px][64 co] and the input halo [(TH+2)(TW+2) px][CI ci];
// every tap reads the halo at a row offset, so the input is fetched once per
// tile instead of 9 times.  Operands are pixel-major, fed to the MFMA through
// ds_read_b64_tr_b16.  The grid is sized to ~one block per CU; each block
// stores its fp32 partial dW with plain stores into its split's slab and
// wgrad_slab_reduce_kernel sums the splits (fp32 atomics into dW when no slab:
// they run at ~1.3 TB/s chip-wide, MI355X_MICROARCH.md "Global float atomics").
// ---------------------------------------------------------------------------
// CO32 (Cout = 32 layers, decoder1): a block owns 32 output channels; the
// two waves of a (wm) pair split each stage's 128 pixels instead of the 64
// channels (no MFMA on the absent channels 32..63), and their partial dW are
// summed through LDS before the store.  The dY DMA still moves 128-B rows
// (pixel p's 32 channels + pixel p+1's, unused).
//
// SD = 2 (3x3 / stride 2 / pad 1, the first conv of encoder stages 2-4): the
// output tile TH x TW reads a (2TH+1) x (2TW+1) input halo (CI = 32 only: 561
// rows of 64 B), tap (r, s) of output pixel (y, x) is halo row (2y + r, 2x + s);
// the same 9-tap reuse of each staged input pixel as the stride-1 kernel
// (the implicit-GEMM wgrad stages an im2col tile per tap).
template <int TW, int CI, int SD>
constexpr int wgrad_halo_rows() {  // LDS halo capacity (rows), a multiple of one DMA round
  constexpr int TH = 128 / TW;
  constexpr int rows = (SD * TH + (SD == 1 ? 2 : 1)) * (SD * TW + (SD == 1 ? 2 : 1));
  constexpr int round = (1024 / (CI * 2)) * (CI / 8);
  return SD == 1 ? 256 : (rows + round - 1) / round * round;
}

// DSF (SD = 2): the block's downsample weight gradient rides in the same
// stages: a dY2 tile beside dY, one more A fragment pair at the centre tap,
// two more accumulator fragments (slab frags 18, 19).
template <int TW, int NS, int CI, bool CO32 = false, int SD = 1, bool DSF = false>
__global__ void __launch_bounds__(CI * 8)
wgrad3x3_halo_kernel(ConvWgradArgs a, int tiles_total, int tiles_per_split) {
  constexpr int NW = CI / 8;            // waves
  constexpr int TH = 128 / TW;
  constexpr int HW2 = SD * TW + (SD == 1 ? 2 : 1);
  constexpr int HROWS = (SD * TH + (SD == 1 ? 2 : 1)) * HW2;
  constexpr int HCAP = wgrad_halo_rows<TW, CI, SD>();
  constexpr int HROWB = CI * 2;         // halo row bytes
  constexpr int HCPR = HROWB / 16;      // 16-B chunks per halo row
  constexpr int HRPI = 1024 / HROWB;    // halo rows per wave instruction
  constexpr int H_INS = HCAP / HRPI / NW;
  constexpr int A_INS = 16 / NW;        // dY: 128 rows of 128 B = 16 instructions
  constexpr int A_BYTES = 128 * 128;
  constexpr int B_BYTES = HCAP * HROWB;
  static_assert(HROWS <= HCAP && HCAP % (HRPI * NW) == 0, "halo rows");
  static_assert(SD == 1 || (CI == 32 && !CO32 && TW % 8 == 0), "stride-2 variant");
  static_assert(!DSF || SD == 2, "downsample fold: stride-2 kernel only");
  constexpr int D_BYTES = DSF ? A_BYTES : 0;  // dY2 tile
  constexpr int STAGE = A_BYTES + B_BYTES + D_BYTES;
  constexpr int NF = DSF ? 20 : 18;           // accumulator fragments per wave
  constexpr int LPS = A_INS * (DSF ? 2 : 1) + H_INS;  // glds per wave per stage
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef TrTile<64, 64, 128> TA;
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;  // wave tile 32 co x 16 ci
  // 1-D grid of combos x splits, XCD-aware: the combos of one split (which
  // share its dY rows and input halos) get consecutive logical ids, i.e. are
  // dealt to one XCD and its L2
  const int combos = a.co_blocks * a.c_blocks;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int combo = bid % combos, split = bid / combos;
  const int cob = combo % a.co_blocks;
  const int cib = combo / a.co_blocks;
  const int co0 = cob * (CO32 ? 32 : 64), c0 = cib * CI;
  const int t0 = split * tiles_per_split;
  const int t1 = min(tiles_total, t0 + tiles_per_split);
  const int KT = t1 - t0;
  const int nsplit = gridDim.x / combos;
  if (KT <= 0 && !(a.slab && nsplit > 1)) return;
  const int tq = a.Q / TW, tp = a.P / TH;
  // asm LDS-DMA (glds16_asm): hipcc would otherwise drain every stage in flight
  // before the first transposed read of each stage
  const i32x4 dyr = make_rsrc_sgpr(a.dy, (unsigned)((size_t)a.N * a.P * a.Q * a.lddy * 2));
  const i32x4 xr = make_rsrc_sgpr(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const i32x4 dy2r = make_rsrc_sgpr(DSF ? a.dy2 : a.dy, DSF ? (unsigned)((size_t)a.N * a.P * a.Q * a.lddy2 * 2) : 0u);

  // per-lane constant parts of the loads
  const int arow = lane >> 3, aslot = lane & 7;                // dY: 8 rows of 128 B per instruction
  const int hrow = lane / HCPR, hslot = lane % HCPR;           // halo: HRPI rows per instruction

  // Per-lane constant parts of the loads, computed once: the dY tile is
  // contiguous rows of one image, so its offset is a per-lane part plus the
  // tile's (wave-uniform, non-negative) origin passed as the scalar offset;
  // the halo keeps a per-stage bounds test on precomputed (row, col).
  unsigned arel[A_INS], arel2[DSF ? A_INS : 1];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = (wave * A_INS + j) * 8 + arow;  // pixel in tile
    const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    const int lchunk = ((((aslot >> 1) ^ f)) << 1) | (aslot & 1);
    arel[j] = (unsigned)((((row / TW) * a.Q + row % TW) * a.lddy) + co0 + lchunk * 8) * 2u;
    if constexpr (DSF) arel2[j] = (unsigned)((((row / TW) * a.Q + row % TW) * a.lddy2) + co0 + lchunk * 8) * 2u;
  }
  int hrr[H_INS], hcc[H_INS], hch[H_INS];
#pragma unroll
  for (int j = 0; j < H_INS; ++j) {
    const int row = (wave * H_INS + j) * HRPI + hrow;  // halo row
    int lchunk;
    if constexpr (CI == 32) {
      lchunk = ((((hslot >> 1) ^ ((row >> 3) & 1))) << 1) | (hslot & 1);
    } else {
      const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
      lchunk = ((((hslot >> 1) ^ f)) << 1) | (hslot & 1);
    }
    hrr[j] = row < HROWS ? row / HW2 - 1 : -(1 << 20);  // rows past the halo fail the bounds test
    hcc[j] = row % HW2 - 1;
    hch[j] = c0 + lchunk * 8;
  }
  auto issue = [&](int kt, int buf) {
    const int t = t0 + kt;
    const int n = t / (tp * tq);
    const int rem = t - n * (tp * tq);
    const int oh0 = (rem / tq) * TH, ow0 = (rem % tq) * TW;
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
    const unsigned abase = (unsigned)(((n * a.P + oh0) * a.Q + ow0) * a.lddy) * 2u;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) glds16_asm(dyr, As + (wave * A_INS + j) * 1024, arel[j], abase);
    if constexpr (DSF) {
      const unsigned abase2 = (unsigned)(((n * a.P + oh0) * a.Q + ow0) * a.lddy2) * 2u;
#pragma unroll
      for (int j = 0; j < A_INS; ++j)
        glds16_asm(dy2r, As + A_BYTES + B_BYTES + (wave * A_INS + j) * 1024, arel2[j], abase2);
    }
#pragma unroll
    for (int j = 0; j < H_INS; ++j) {
      const int ih = SD * oh0 + hrr[j], iw = SD * ow0 + hcc[j];
      unsigned off = kOOB;
      if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        off = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx) + hch[j]) * 2u;
      glds16_asm(xr, Bs + (wave * H_INS + j) * 1024, off, 0u);
    }
  };

  f32x4 acc[9][2], acc2[DSF ? 2 : 1];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < (DSF ? 2 : 1); ++i) acc2[i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KT) issue(s, s);
  const int g = lane >> 4, li = lane & 15, trq = li >> 2, trp = li & 3;
  TSTAMP(a.tim, 1);
  for (int kt = 0; kt < KT; ++kt) {
    const int ahead = KT - 1 - kt;
    if (ahead >= NS - 2) wait_vmcnt<(NS - 2) * LPS>();
    else if (NS > 3 && ahead == 1) wait_vmcnt<LPS>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (kt < 16) TSTAMP(a.tim, 2 + kt);
    if (kt + NS - 1 < KT && UNET_ABL != 2) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const char* As = smem + (kt % NS) * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int k2 = 0; k2 < (UNET_ABL == 1 ? 0 : CO32 ? 2 : 4); ++k2) {
      const int kk = CO32 ? wm * 2 + k2 : k2;    // CO32: the wm pair splits the pixels
      const int p_lo = kk * 32 + 8 * g + trq;  // this lane's pixel (first tr read)
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = (CO32 ? 0 : wm * 32) + i * 16 + 4 * trp;
        af[i] = tr_read8(As + TA::off(p_lo, col), As + TA::off(p_lo + 4, col));
      }
      const int ty = p_lo / TW, tx = p_lo % TW;  // p_lo and p_lo+4 share the tile row
      const int col = wn * 16 + 4 * trp;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int hr = (SD * ty + r) * HW2 + SD * tx + s;
          const bf16x8 bfr = tr_read8(Bs + tr_off<CI>(hr, col), Bs + tr_off<CI>(hr + 4 * SD, col));
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[r * 3 + s][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr, acc[r * 3 + s][i], 0, 0, 0);
          if constexpr (DSF) {
            if (r == 1 && s == 1) {  // centre tap = the downsample's input pixel (2y, 2x)
              const char* Ds = Bs + B_BYTES;
#pragma unroll
              for (int i = 0; i < 2; ++i) {
                const int cl = wm * 32 + i * 16 + 4 * trp;
                const bf16x8 a2 = tr_read8(Ds + TA::off(p_lo, cl), Ds + TA::off(p_lo + 4, cl));
                acc2[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, bfr, acc2[i], 0, 0, 0);
              }
            }
          }
        }
    }
  }
  wait_vmcnt<0>();
  TSTAMP(a.tim, 20);
  if constexpr (CO32) {  // fold the wm = 1 partials into wm = 0 through LDS
    __syncthreads();     // every stage consumed: the staging LDS is free
    f32x4* red = reinterpret_cast<f32x4*>(smem) + (size_t)(wn * 18) * 64 + lane;
    if (wm == 1) {
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < 2; ++i) red[(t * 2 + i) * 64] = acc[t][i];
    }
    __syncthreads();
    if (wm == 1) return;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) acc[t][i] += red[(t * 2 + i) * 64];
  }
  // epilogue: this split's partial in the register-native slab layout
  // (SLAB_HALO: 18 fragments per wave, 16 B per lane per store), or -- one
  // split -- the block's dW tile with plain stores, or fp32 atomics (no slab)
  if (a.slab && nsplit > 1) {
    // CO32: only the wm = 0 waves hold a partial (the slab has NW / 2 wave slots)
    constexpr int SW = CO32 ? NW / 2 : NW;
    const int sw = CO32 ? wn : wave;
    const size_t units = (size_t)combos * SW * NF * 64;  // per split (grid = combos x splits)
    f32x4* dst = reinterpret_cast<f32x4*>(a.slab) + (size_t)split * units +
                 ((size_t)combo * SW + sw) * (NF * 64) + lane;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) dst[(t * 2 + i) * 64] = acc[t][i];
    if constexpr (DSF) {
#pragma unroll
      for (int i = 0; i < 2; ++i) dst[(18 + i) * 64] = acc2[i];
    }
    TSTAMP(a.tim, 21);
    TSTAMP_RT(a.tim, 31);
    return;
  }
  const int Krow = 9 * a.C;
  const int c = c0 + wn * 16 + li;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + (CO32 ? 0 : wm * 32) + i * 16 + 4 * g + e;
        if (co < a.Cout) {
          float* d = a.dw + (size_t)co * Krow + t * a.C + c;
          if (a.slab) *d = acc[t][i][e];
          else atomicAdd(d, acc[t][i][e]);
        }
      }
  if constexpr (DSF) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * 32 + i * 16 + 4 * g + e;
        if (co < a.Cout) {
          float* d = a.dw2 + (size_t)co * a.C + c;
          if (a.slab) *d = acc2[i][e];
          else atomicAdd(d, acc2[i][e]);
        }
      }
  }
}

// ---------------------------------------------------------------------------
// 3x3 / stride-1 weight gradient with dedicated LOADER waves (the C, Cout % 64
// layers at Q % 32 == 0: enc1-3 and decoder2-4).  Same block geometry, split-K
// slab and MFMA work as wgrad3x3_halo_kernel<32, 3, 64> (64 co x 64 ci x 9 taps
// per block, 32 x 4 output-pixel tiles, 3 stages), restructured after the phase
// ablation of that kernel (profiles/r04/s1): one stage took 4340 cycles with
// every wave issuing its share of the LDS-DMA, 1800 for the DMA alone and 3250
// for the MFMA work alone.  Here
//  * 4 loader waves (one per SIMD) issue all of the LDS-DMA and wait for it;
//    the 8 compute waves only read LDS and issue MFMAs (one barrier per stage);
//  * the halo image rows sit at a pitch of 48 LDS rows (a multiple of 16, so the
//    row swizzle of tr_off<64> does not change from one halo row to the next):
//    every fragment read is a per-lane base register plus an immediate offset,
//    no per-read address arithmetic;
//  * fragments are read in halo-row order: the stage's 8 dY fragments first,
//    then each of the 18 halo fragments once, feeding every tap it serves.
// ---------------------------------------------------------------------------
constexpr int kWlNW = 8;                  // compute waves: wave tile 32 co x 16 ci x 9 taps
constexpr int kWlNL = 4;                  // loader waves
constexpr int kWlNS = 3;                  // stages
constexpr int kWlHP = 48;                 // LDS rows per halo image row (34 used)
constexpr int kWlA = 128 * 128;           // dY tile: 128 px x 64 co, bf16
constexpr int kWlB = 6 * kWlHP * 128;     // halo: 6 image rows x 48 x 64 ci, bf16
constexpr int kWlStage = kWlA + kWlB;     // 53,248 B; 3 stages = 159,744 B of LDS
constexpr int kWlHIns = 32;               // halo DMA instructions per stage (30 used + 2 zero-fill)
constexpr int kWlLps = 16 / kWlNL + kWlHIns / kWlNL;  // LDS-DMA per loader wave per stage

// Output-pixel tile geometry of the batched weight gradient (TW x TH = 128
// pixels = one 128-row dY image per item).  TW = 32: 32 x 4 tiles, a 6 x 34
// halo at a pitch of 48 LDS rows (the layout of wgrad3x3_ld_kernel).  TW = 16
// (Q = 16 layers, enc4 at 512^2): 16 x 8 tiles, a 10 x 18 halo stored densely
// (pitch 18; 180 rows + 12 zero rows = 24 DMA instructions).  Both swizzle a
// halo pixel's 32-B units by its COLUMN (tr_off<64> of the column), so an image
// row is a constant byte offset and every fragment read is base + immediate;
// an even pitch keeps a half-wave's 8 rows on distinct banks (tr_off<64>).
template <int TW>
struct WbGeo;
template <>
struct WbGeo<32> {
  static constexpr int TH = 4, HIR = 6, PITCH = kWlHP, HINS = kWlHIns, B = kWlB;
};
template <>
struct WbGeo<16> {
  static constexpr int TH = 8, HIR = 10, PITCH = 18, HINS = 24, B = 24 * 1024;
};
template <int TW>
constexpr int wb_stage() { return kWlA + WbGeo<TW>::B; }
template <int TW>
constexpr int wb_lps() { return 16 / kWlNL + WbGeo<TW>::HINS / kWlNL; }

__global__ void __launch_bounds__((kWlNW + kWlNL) * 64)
wgrad3x3_ld_kernel(ConvWgradArgs a, int tiles_total, int tiles_per_split) {
  constexpr int TW = 32, TH = 4;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef TrTile<64, 64, 128> TA;
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int combos = a.co_blocks * a.c_blocks;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int combo = bid % combos, split = bid / combos;
  const int cob = combo % a.co_blocks, cib = combo / a.co_blocks;
  const int co0 = cob * 64, c0 = cib * 64;
  const int t0 = split * tiles_per_split;
  const int t1 = min(tiles_total, t0 + tiles_per_split);
  const int KT = t1 - t0;
  const int nsplit = gridDim.x / combos;
  if (KT <= 0 && !(a.slab && nsplit > 1)) return;
  const int tq = a.Q / TW, tp = a.P / TH;

  if (wave >= kWlNW) {
    // ---- loader wave lw: dY instructions 4 lw .. 4 lw + 3 of 16, halo
    // instructions 8 lw .. 8 lw + 7 of 32 (image row idx / 5, 8-column block
    // idx % 5; 30 and 31 zero-fill the never-read padding rows 40-47 of image
    // rows 0 and 1, so every loader issues the same count) ----
    constexpr int AI = 16 / kWlNL, HI = kWlHIns / kWlNL;
    const int lw = wave - kWlNW;
    const i32x4 dyr = make_rsrc_sgpr(a.dy, (unsigned)((size_t)a.N * a.P * a.Q * a.lddy * 2));
    const i32x4 xr = make_rsrc_sgpr(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
    const int lrow = lane >> 3, lslot = lane & 7;  // 8 rows of 128 B per instruction
    unsigned arel[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int row = (lw * AI + j) * 8 + lrow;  // pixel of the tile
      const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
      const int lchunk = (((lslot >> 1) ^ f) << 1) | (lslot & 1);
      arel[j] = (unsigned)((((row / TW) * a.Q + row % TW) * a.lddy) + co0 + lchunk * 8) * 2u;
    }
    int hrr[HI], hcc[HI], hdst[HI];
    unsigned hch[HI];
#pragma unroll
    for (int j = 0; j < HI; ++j) {
      const int idx = lw * HI + j;
      const bool pad = idx >= 30;
      const int ir = pad ? idx - 30 : idx / 5;
      const int col = (pad ? 40 : (idx % 5) * 8) + lrow;  // column in the halo image row
      const int f = ((col >> 1) & 1) | (((col >> 3) & 1) << 1);  // = the swizzle of LDS row ir * 48 + col
      const int lchunk = (((lslot >> 1) ^ f) << 1) | (lslot & 1);
      hrr[j] = (!pad && col < TW + 2) ? ir - 1 : -(1 << 20);  // rows past the halo fail the bounds test
      hcc[j] = col - 1;
      hch[j] = (unsigned)(c0 + lchunk * 8);
      hdst[j] = (ir * kWlHP + (pad ? 40 : (idx % 5) * 8)) * 128;
    }
    auto issue = [&](int kt, int buf) {
      const int t = t0 + kt;
      const int n = t / (tp * tq);
      const int rem = t - n * (tp * tq);
      const int oh0 = (rem / tq) * TH, ow0 = (rem % tq) * TW;
      char* As = smem + buf * kWlStage;
      char* Bs = As + kWlA;
      const unsigned abase = (unsigned)(((n * a.P + oh0) * a.Q + ow0) * a.lddy) * 2u;
#pragma unroll
      for (int j = 0; j < AI; ++j) glds16_asm(dyr, As + (lw * AI + j) * 1024, arel[j], abase);
#pragma unroll
      for (int j = 0; j < HI; ++j) {
        const int ih = oh0 + hrr[j], iw = ow0 + hcc[j];
        const bool ok = (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const unsigned off = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx) + (int)hch[j]) * 2u;
        glds16_asm(xr, Bs + hdst[j], ok ? off : kOOB, 0u);
      }
    };
#pragma unroll
    for (int s = 0; s < kWlNS - 1; ++s)
      if (s < KT) issue(s, s);
    for (int kt = 0; kt < KT; ++kt) {
      // stage kt has landed when at most the younger stages are in flight
      if (KT - 1 - kt >= kWlNS - 2) wait_vmcnt<(kWlNS - 2) * kWlLps>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // ... and every compute wave is done with stage kt - 1
      if (kt + kWlNS - 1 < KT && UNET_ABL != 2) issue(kt + kWlNS - 1, (kt + kWlNS - 1) % kWlNS);
    }
    return;  // an exited wave no longer takes part in the compute waves' barriers
  }

  // ---- compute waves ----
  const int wm = wave & 1, wn = wave >> 1;  // wave tile 32 co x 16 ci
  const int g = lane >> 4, li = lane & 15, trq = li >> 2, trp = li & 3;
  // per-lane fragment bases (LDS bytes): dY pixel 8g + trq (+4) of k-step 0 (a
  // k-step adds 32 pixel rows = 4096 B), halo column 8g + trq + s (+4) of image
  // row 0 (an image row adds 48 LDS rows = 6144 B)
  int aoff[2][2], boff[3][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][h] = TA::off(8 * g + trq + 4 * h, wm * 32 + i * 16 + 4 * trp);
#pragma unroll
    for (int s = 0; s < 3; ++s) boff[s][h] = tr_off<64>(8 * g + trq + s + 4 * h, wn * 16 + 4 * trp);
  }
  f32x4 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  TSTAMP(a.tim, 1);
  for (int kt = 0; kt < KT; ++kt) {
    __builtin_amdgcn_s_barrier();  // the loaders have waited for stage kt
    if (kt < 16) TSTAMP(a.tim, 2 + kt);
    const char* As = smem + (kt % kWlNS) * kWlStage;
    const char* Bs = As + kWlA;
    if (UNET_ABL == 1) continue;
    bf16x8 af[4][2];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < 2; ++i) af[kk][i] = tr_read8(As + aoff[i][0] + kk * 4096, As + aoff[i][1] + kk * 4096);
#pragma unroll
    for (int h = 0; h < 6; ++h) {  // halo image row h serves k-step kk at tap row r = h - kk
      bf16x8 bfr[3];
#pragma unroll
      for (int s = 0; s < 3; ++s) bfr[s] = tr_read8(Bs + boff[s][0] + h * 6144, Bs + boff[s][1] + h * 6144);
#pragma unroll
      for (int kk = (h > 2 ? h - 2 : 0); kk <= (h < 3 ? h : 3); ++kk)
#pragma unroll
        for (int s = 0; s < 3; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i)
            acc[(h - kk) * 3 + s][i] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[s], acc[(h - kk) * 3 + s][i], 0, 0, 0);
    }
  }
  TSTAMP(a.tim, 20);
  if (a.slab && nsplit > 1) {  // this split's partial in the SLAB_HALO layout (18 fragments per wave)
    const size_t units = (size_t)combos * kWlNW * 18 * 64;
    f32x4* dst = reinterpret_cast<f32x4*>(a.slab) + (size_t)split * units + ((size_t)combo * kWlNW + wave) * (18 * 64) + lane;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 2; ++i) dst[(t * 2 + i) * 64] = acc[t][i];
    TSTAMP(a.tim, 21);
    TSTAMP_RT(a.tim, 31);
    return;
  }
  const int Krow = 9 * a.C;
  const int c = c0 + wn * 16 + li;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wm * 32 + i * 16 + 4 * g + e;
        if (co < a.Cout) {
          float* d = a.dw + (size_t)co * Krow + t * a.C + c;
          if (a.slab) *d = acc[t][i][e];
          else atomicAdd(d, acc[t][i][e]);
        }
      }
}

// ---------------------------------------------------------------------------
// Batched 3x3 / stride-1 weight gradients (WgBatchArgs, kernels.h): the
// loader / compute structure of wgrad3x3_ld_kernel over a stream-K range of
// (unit, tile) items spanning several layers.  Every block of the one launch
// has the same number of stages; a unit (layer, 64 co x 64 ci block) that
// ends inside the block's range is written out (dW directly when the whole unit
// ran in this block, else a slab partial) and its accumulators restart for the
// next unit.  Replaces one launch + one 37.7 MB split-K slab round trip per
// layer (every halo wgrad launch wrote 256 blocks x 147 KB whatever the layer).
// ---------------------------------------------------------------------------
struct WbPos {  // (layer, unit of the layer, tile) of an item, advanced item by item
  int l, combo, tile;
  __device__ __forceinline__ void locate(const WgBatchArgs& a, long long it) {
    l = 0;
    while (l + 1 < a.nl && it >= a.L[l + 1].item0) ++l;
    const long long r = it - a.L[l].item0;
    combo = (int)(r / a.L[l].tiles);
    tile = (int)(r - (long long)combo * a.L[l].tiles);
  }
  __device__ __forceinline__ void next(const WgBatchArgs& a) {
    if (++tile == a.L[l].tiles) {
      tile = 0;
      if (++combo == a.L[l].co_blocks * a.L[l].c_blocks) {
        combo = 0;
        ++l;
      }
    }
  }
};
__device__ __forceinline__ long long wb_begin(const WgBatchArgs& a, int b) { return (long long)b * a.items / a.grid; }

// the loaders' position, with the current layer's fields and the tile origin
// kept incrementally (no per-stage divisions or kernel-argument loads)
template <int TW>
struct WbLoad {
  static constexpr int TH = WbGeo<TW>::TH;
  int l, tile, cob, cib, n, oh0, ow0;
  const bf16_t* dy;
  const bf16_t* x;
  int H, W, lddy, ldx, co_blocks, c_blocks, tiles;
  __device__ __forceinline__ void layer(const WgBatchArgs& a) {
    const WgBatchLayer& L = a.L[l];
    dy = L.dy; x = L.x;
    H = L.H; W = L.W; lddy = L.lddy; ldx = L.ldx;
    co_blocks = L.co_blocks; c_blocks = L.c_blocks; tiles = L.tiles;
  }
  __device__ __forceinline__ void locate(const WgBatchArgs& a, long long it) {
    WbPos p;
    p.locate(a, it);
    l = p.l;
    layer(a);
    tile = p.tile;
    cob = p.combo % co_blocks;
    cib = p.combo / co_blocks;
    const int tq = W / TW, tp = H / TH;
    n = tile / (tp * tq);
    const int rem = tile - n * (tp * tq);
    oh0 = (rem / tq) * TH;
    ow0 = (rem % tq) * TW;
  }
  __device__ __forceinline__ void next(const WgBatchArgs& a) {
    ow0 += TW;
    if (ow0 == W) {
      ow0 = 0;
      oh0 += TH;
      if (oh0 == H) {
        oh0 = 0;
        ++n;
      }
    }
    if (++tile == tiles) {
      tile = n = oh0 = ow0 = 0;
      if (++cob == co_blocks) {
        cob = 0;
        if (++cib == c_blocks) {
          cib = 0;
          if (++l < a.nl) layer(a);
        }
      }
    }
  }
};

template <int TW>
__global__ void __launch_bounds__((kWlNW + kWlNL) * 64) wgrad3x3_batch_kernel(WgBatchArgs a) {
  typedef WbGeo<TW> G;
  constexpr int STAGE = wb_stage<TW>(), LPS = wb_lps<TW>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef TrTile<64, 64, 128> TA;
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int b = blockIdx.x;
  const long long i0 = wb_begin(a, b), i1 = wb_begin(a, b + 1);
  const int KT = (int)(i1 - i0);
  if (KT <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  if (wave >= kWlNW) {
    // ---- loader wave lw: dY instructions 4 lw .. 4 lw + 3 of 16, halo
    // instructions HI lw .. HI lw + HI - 1 of G::HINS ----
    constexpr int AI = 16 / kWlNL, HI = G::HINS / kWlNL;
    const int lw = wave - kWlNW;
    const int lrow = lane >> 3, lslot = lane & 7;
    int arow[AI], alch[AI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int row = (lw * AI + j) * 8 + lrow;  // pixel of the tile
      const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
      arow[j] = row;
      alch[j] = (((lslot >> 1) ^ f) << 1) | (lslot & 1);
    }
    int hrr[HI], hcc[HI], hdst[HI], hlch[HI];
#pragma unroll
    for (int j = 0; j < HI; ++j) {
      const int idx = lw * HI + j;
      int hr, hc, dst;
      bool ok;
      if constexpr (TW == 32) {  // image row idx / 5, 8-column block idx % 5; 30, 31 zero-fill
        const bool pad = idx >= 30;  // the never-read padding rows 40-47 of image rows 0 and 1
        hr = pad ? idx - 30 : idx / 5;
        hc = (pad ? 40 : (idx % 5) * 8) + lrow;
        ok = !pad && hc < TW + 2;
        dst = (hr * G::PITCH + (pad ? 40 : (idx % 5) * 8)) * 128;
      } else {  // dense: LDS row 8 idx + lrow = halo pixel (row / 18, row % 18)
        const int row = idx * 8 + lrow;
        hr = row / G::PITCH;
        hc = row - hr * G::PITCH;
        ok = row < G::HIR * G::PITCH;
        dst = idx * 1024;
      }
      const int f = ((hc >> 1) & 1) | (((hc >> 3) & 1) << 1);  // the column's swizzle (tr_off<64>)
      hlch[j] = (((lslot >> 1) ^ f) << 1) | (lslot & 1);
      hrr[j] = ok ? hr - 1 : -(1 << 20);  // rows past the halo fail the bounds test
      hcc[j] = hc - 1;
      hdst[j] = dst;
    }
    WbLoad<TW> pos;
    pos.locate(a, i0);
    auto issue = [&](int buf) {  // the stage of item `pos`, then advance
      const int H = pos.H, W = pos.W, lddy = pos.lddy, ldx = pos.ldx;
      const int n = pos.n, oh0 = pos.oh0, ow0 = pos.ow0;
      const int co0 = pos.cob * 64, c0 = pos.cib * 64;
      const i32x4 dyr = make_rsrc_sgpr(pos.dy, (unsigned)((size_t)a.N * H * W * lddy * 2));
      const i32x4 xr = make_rsrc_sgpr(pos.x, (unsigned)((size_t)a.N * H * W * ldx * 2));
      char* As = smem + buf * STAGE;
      char* Bs = As + kWlA;
      const unsigned abase = (unsigned)(((n * H + oh0) * W + ow0) * lddy) * 2u;
#pragma unroll
      for (int j = 0; j < AI; ++j) {
        const unsigned rel = (unsigned)((((arow[j] / TW) * W + arow[j] % TW) * lddy) + co0 + alch[j] * 8) * 2u;
        glds16_asm(dyr, As + (lw * AI + j) * 1024, rel, abase);
      }
#pragma unroll
      for (int j = 0; j < HI; ++j) {
        const int ih = oh0 + hrr[j], iw = ow0 + hcc[j];
        const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        const unsigned off = (unsigned)((((n * H + ih) * W + iw) * ldx) + c0 + hlch[j] * 8) * 2u;
        glds16_asm(xr, Bs + hdst[j], ok ? off : kOOB, 0u);
      }
      pos.next(a);
    };
#pragma unroll
    for (int s = 0; s < kWlNS - 1; ++s)
      if (s < KT) issue(s);
    for (int kt = 0; kt < KT; ++kt) {
      if (KT - 1 - kt >= kWlNS - 2) wait_vmcnt<(kWlNS - 2) * LPS>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (kt + kWlNS - 1 < KT && UNET_ABL != 2) issue((kt + kWlNS - 1) % kWlNS);
    }
    return;
  }

  // ---- compute waves ----
  const int wm = wave & 1, wn = wave >> 1;
  const int g = lane >> 4, li = lane & 15, trq = li >> 2, trp = li & 3;
  // dY pixel 8g + trq (+4) of k-step 0 (a k-step adds 32 pixel rows = 4096 B).
  // Halo: k-step kk, tap (r, s) reads, for k = pixel 8g + j of the k-step, the
  // halo pixel of tile pixel 32 kk + 8g + j shifted by (r, s).  TW = 32: image
  // row kk + r, column 8g + j + s; TW = 16: image row 2 kk + (g >> 1) + r,
  // column 8 (g & 1) + j + s.  boff holds the column part (+ the g >> 1 row),
  // an image row adds PITCH LDS rows.
  int aoff[2][2], boff[3][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) aoff[i][h] = TA::off(8 * g + trq + 4 * h, wm * 32 + i * 16 + 4 * trp);
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      if constexpr (TW == 32) boff[s][h] = tr_off<64>(8 * g + trq + s + 4 * h, wn * 16 + 4 * trp);
      else
        boff[s][h] = (g >> 1) * G::PITCH * 128 + tr_off<64>(8 * (g & 1) + trq + s + 4 * h, wn * 16 + 4 * trp);
    }
  }
  WbPos pos;
  pos.locate(a, i0);
  const int ufirst = a.L[pos.l].unit0 + pos.combo;  // the block's first unit: its slab slot 0
  // the current layer's unit length and count, reloaded only when the layer changes
  int tiles = a.L[pos.l].tiles, ncombo = a.L[pos.l].co_blocks * a.L[pos.l].c_blocks;
  f32x4 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  TSTAMP(a.tim, 1);
  for (int kt = 0; kt < KT; ++kt) {
    __builtin_amdgcn_s_barrier();  // the loaders have waited for stage kt
    if (kt < 16) TSTAMP(a.tim, 2 + kt);
    const char* As = smem + (kt % kWlNS) * STAGE;
    const char* Bs = As + kWlA;
    if (UNET_ABL != 1) {
      bf16x8 af[4][2];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i) af[kk][i] = tr_read8(As + aoff[i][0] + kk * 4096, As + aoff[i][1] + kk * 4096);
      // halo image row h serves the (k-step kk, tap row r) pairs with h = kk + r
      // (TW = 32) or h = 2 kk + r (TW = 16): each fragment is read once
      constexpr int KS = TW == 32 ? 1 : 2, NH = 3 * KS + 3;
#pragma unroll
      for (int h = 0; h < NH; ++h) {
        bf16x8 bfr[3];
#pragma unroll
        for (int s = 0; s < 3; ++s)
          bfr[s] = tr_read8(Bs + boff[s][0] + h * G::PITCH * 128, Bs + boff[s][1] + h * G::PITCH * 128);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int r = h - KS * kk;
          if (r < 0 || r > 2) continue;
#pragma unroll
          for (int s = 0; s < 3; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
              acc[r * 3 + s][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[kk][i], bfr[s], acc[r * 3 + s][i], 0, 0, 0);
        }
      }
    }
    if (pos.tile == tiles - 1 || kt == KT - 1) {  // the unit's last item in this block
      const int l = __builtin_amdgcn_readfirstlane(pos.l);
      const WgBatchLayer& L = a.L[l];
      const int combo = __builtin_amdgcn_readfirstlane(pos.combo);
      const long long S = L.item0 + (long long)combo * L.tiles;
      if (S >= i0 && S + L.tiles <= i1) {  // the whole unit ran here: dW directly
        const int co0 = (combo % L.co_blocks) * 64, c0 = (combo / L.co_blocks) * 64;
        const int Krow = 9 * L.C;
        const int c = c0 + wn * 16 + li;
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              L.dw[(size_t)(co0 + wm * 32 + i * 16 + 4 * g + e) * Krow + t * L.C + c] = acc[t][i][e];
      } else {  // a partial: slot b * maxseg + the unit's rank in this block
        const int slot = b * a.maxseg + (L.unit0 + combo - ufirst);
        f32x4* dst = reinterpret_cast<f32x4*>(a.slab) + (size_t)slot * (kWlNW * 18 * 64) + wave * (18 * 64) + lane;
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int i = 0; i < 2; ++i) dst[(t * 2 + i) * 64] = acc[t][i];
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    if (++pos.tile == tiles) {  // WbPos::next with the layer fields cached
      pos.tile = 0;
      if (++pos.combo == ncombo) {
        pos.combo = 0;
        if (++pos.l < a.nl) {
          tiles = a.L[pos.l].tiles;
          ncombo = a.L[pos.l].co_blocks * a.L[pos.l].c_blocks;
        }
      }
    }
  }
  TSTAMP(a.tim, 20);
  TSTAMP_RT(a.tim, 31);
}

// the block whose item range holds item it
__device__ __forceinline__ int wb_block_of(const WgBatchArgs& a, long long it) {
  int b = (int)((it * a.grid) / a.items);
  while (b + 1 < a.grid && wb_begin(a, b + 1) <= it) ++b;
  while (b > 0 && wb_begin(a, b) > it) --b;
  return b;
}

// dW of every unit spread over several blocks = the sum of its partials in
// block order; grid (units, 36): 256 threads x one f32x4 element of the unit's
// 9216-element (8 waves x 18 fragments x 64 lanes) SLAB_HALO partial each.
// Block y takes fragment y % 18 of the four compute waves wn of half wm = y / 18:
// one tap's 16 output channels x all 64 input channels, so after a transpose
// through LDS every thread stores 4 consecutive input channels and 16 lanes
// write one 256-B dW row segment (the fragment-order stores wrote 64-B pieces).
// The unit's slab slots (one per block it spans, <= grid <= 256) are located
// once per block, one thread per spanned block, into LDS; every thread then
// streams its element of those partials with 8 loads in flight and adds them
// in block order (the order, hence the bits, of a serial loop)
__global__ void __launch_bounds__(256) wgrad_batch_reduce_kernel(WgBatchArgs a) {
  __shared__ int slots[kWbMaxGrid];
  __shared__ float tile[16][65];
  const int u = blockIdx.x;
  int l = 0;
  while (l + 1 < a.nl && u >= a.L[l + 1].unit0) ++l;
  const WgBatchLayer& L = a.L[l];
  const int combo = u - L.unit0;
  const long long S = L.item0 + (long long)combo * L.tiles;
  const int b0 = wb_block_of(a, S), b1 = wb_block_of(a, S + L.tiles - 1);
  if (b0 == b1) return;  // written directly by its block
  const int nb = b1 - b0 + 1;
  if ((int)threadIdx.x < nb) {
    const int b = b0 + threadIdx.x;
    const long long ib = wb_begin(a, b);
    int slot = -1;  // -1: an empty range (batches of fewer items than blocks)
    if (wb_begin(a, b + 1) != ib) {
      WbPos p;
      p.locate(a, ib);
      slot = b * a.maxseg + (u - (a.L[p.l].unit0 + p.combo));
    }
    slots[threadIdx.x] = slot;
  }
  __syncthreads();
  const int wm = blockIdx.y / 18, frag = blockIdx.y % 18, wn = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = ((wm + 2 * wn) * 18 + frag) * 64 + lane;
  const f32x4* slab = reinterpret_cast<const f32x4*>(a.slab) + q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j0 = 0; j0 < nb; j0 += 8) {
    f32x4 v[8];
    int sl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sl[k] = j0 + k < nb ? slots[j0 + k] : -1;
      if (sl[k] >= 0) v[k] = slab[(size_t)sl[k] * (kWlNW * 18 * 64)];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (sl[k] >= 0) acc += v[k];
  }
  const int t = frag >> 1, i = frag & 1;
  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int e = 0; e < 4; ++e) tile[4 * g + e][wn * 16 + li] = acc[e];
  __syncthreads();
  const int co0 = (combo % L.co_blocks) * 64, c0 = (combo / L.co_blocks) * 64;
  const int Krow = 9 * L.C;
  const int col = threadIdx.x >> 4, c4 = (threadIdx.x & 15) * 4;  // output channel, 4 input channels
  const float4 o = make_float4(tile[col][c4], tile[col][c4 + 1], tile[col][c4 + 2], tile[col][c4 + 3]);
  *reinterpret_cast<float4*>(L.dw + (size_t)(co0 + wm * 32 + i * 16 + col) * Krow + t * L.C + c0 + c4) = o;
}

// dW = sum over the splits of the slab (slab_reduce_block, common.h)
__global__ void __launch_bounds__(256) wgrad_slab_reduce_kernel(const f32x4* __restrict__ slab,
                                                                float* __restrict__ dw, SlabLayout L, int T) {
  __shared__ f32x4 part[256];
  slab_reduce_block(slab, dw, L, T, blockIdx.x, part);
}

// ---------------------------------------------------------------------------
// 7x7/s2/p3 stem, 1 -> 64 channels, fp32 image.
//
// A block walks a contiguous range of output rows (Q pixels each, Q <= 256).
// Per row the 7 input rows it needs are fetched once (coalesced fp32, issued
// into registers one row AHEAD so the loads overlap the current row's work),
// converted to a bf16 LDS patch, and each thread builds its pixel's im2col row
// (49 taps padded to K = 64) in LDS.  Forward: D[co][px] = W[co][k] .
// im2col[px][k]; the BN batch sums are kept in registers over all the block's
// rows and committed once (replica atomics + last-block finalise).  Weight
// gradient: D[co][k] += sum_px dY[px][co] . im2col[px][k], both tiles
// pixel-major and read through ds_read_b64_tr_b16; one fp32-atomic 64x64
// partial per block.
// ---------------------------------------------------------------------------
constexpr int kStemPatchW = 2 * 256 + 8;       // bf16 columns of the 7-row input patch
constexpr int kStemPatchPT = (7 * (2 * 256 + 6) + 255) / 256;  // patch values per thread (<= 15)

struct StemPatch { float v[kStemPatchPT]; };

// The stem walks UNITS of <= 256 output pixels: unit u is output row
// u / nseg, columns q0 = (u % nseg) * 256 .. q0 + Q - 1 (nseg = ceil(Q / 256)),
// so rows wider than one 256-thread block (the 1024^2 HiRes input) are split.
struct StemUnit { int n, oh, q0, Qs; size_t row; };
__device__ __forceinline__ StemUnit stem_unit(int u, int P, int Q) {
  const int nseg = (Q + 255) >> 8;
  StemUnit t;
  const int row = u / nseg;
  t.row = (size_t)row;
  t.n = row / P;
  t.oh = row - t.n * P;
  t.q0 = (u - row * nseg) << 8;
  t.Qs = min(256, Q - t.q0);
  return t;
}

// registers <- img rows 2*oh-3 .. 2*oh+3, cols 2*q0-3 .. 2*(q0+Q)+2 (zero outside)
__device__ __forceinline__ void stem_fetch(const float* img, const StemUnit& t, int H, int W, StemPatch& p) {
  const int cols = 2 * t.Qs + 6;
#pragma unroll
  for (int j = 0; j < kStemPatchPT; ++j) {
    const int i = threadIdx.x + j * 256;
    const int r = i / cols, c = i - r * cols;
    const int n = t.n, ih = 2 * t.oh - 3 + r, iw = 2 * t.q0 + c - 3;
    p.v[j] = (r < 7 && ih >= 0 && ih < H && iw >= 0 && iw < W) ? img[((size_t)n * H + ih) * W + iw] : 0.f;
  }
}
__device__ __forceinline__ void stem_store_patch(const StemPatch& p, int Q, bf16_t* patch) {
  const int cols = 2 * Q + 6;
#pragma unroll
  for (int j = 0; j < kStemPatchPT; ++j) {
    const int i = threadIdx.x + j * 256;
    const int r = i / cols, c = i - r * cols;
    if (r < 7) patch[r * kStemPatchW + c] = f2bf(p.v[j]);
  }
}

// im2col row of pixel px as 8 x 16 B in the stem K layout k = kr*8 + ks
// (ks = 7 and kr = 7 are zero): chunk kr is the 8 patch values of row kr from
// column 2*px on (4-B aligned), read as 4 dwords, with the 8th value masked
__device__ __forceinline__ void stem_im2col_row(const bf16_t* patch, int px, uint4 (&row)[8]) {
#pragma unroll
  for (int kr = 0; kr < 7; ++kr) {
    const unsigned* w = reinterpret_cast<const unsigned*>(patch + kr * kStemPatchW + 2 * px);
    row[kr] = make_uint4(w[0], w[1], w[2], w[3] & 0xffffu);
  }
  row[7] = make_uint4(0, 0, 0, 0);
}

__global__ void __launch_bounds__(256, 2) stem_fwd_kernel(ConvFwdArgs a, int rows_per_block) {
  // LDS: weights [64][64] (8 KB) | im2col [256][64] (32 KB) | patch 7 x 520 bf16
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ws = smem;
  char* Xs = smem + 64 * 128;
  bf16_t* patch = reinterpret_cast<bf16_t*>(smem + 64 * 128 + 256 * 128);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float* img = reinterpret_cast<const float*>(a.x);
  const int total_rows = a.N * a.P * ((a.Q + 255) >> 8);  // units
  const int r0 = xcd_remap(blockIdx.x, gridDim.x) * rows_per_block;
  const int r1 = min(total_rows, r0 + rows_per_block);
  const int cg = blockIdx.y * 64;  // 64-channel output group (Wide stem: 2 groups)
  {  // packed weights [64][64] bf16 of the group -> swizzled LDS rows
    const uint4* wsrc = reinterpret_cast<const uint4*>(a.w + (size_t)cg * 64);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = tid + j * 256, co = i >> 3, ch = i & 7;
      *reinterpret_cast<uint4*>(Ws + frag_off<64>(co, ch)) = wsrc[i];
    }
  }
  float q0[4][4], q1[4][4];  // per-lane BN sums of channels i*16 + 4*(lane>>4) + e
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = 0.f;
  StemPatch pf;
  if (r0 < r1) stem_fetch(img, stem_unit(r0, a.P, a.Q), a.H, a.W, pf);
  for (int u = r0; u < r1; ++u) {
    const StemUnit t = stem_unit(u, a.P, a.Q);
    __syncthreads();  // previous unit's patch / im2col consumed
    stem_store_patch(pf, t.Qs, patch);
    if (u + 1 < r1) stem_fetch(img, stem_unit(u + 1, a.P, a.Q), a.H, a.W, pf);
    __syncthreads();
    {
      uint4 r8[8];
      if (tid < t.Qs) {
        stem_im2col_row(patch, tid, r8);
      } else {
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) r8[c8] = make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) *reinterpret_cast<uint4*>(Xs + frag_off<64>(tid, c8)) = r8[c8];
    }
    __syncthreads();
    // 4 waves x (64 px x 64 co): acc[co frag][px frag]
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = kk * 4 + (lane >> 4);
      bf16x8 wf[4], xf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        wf[i] = *reinterpret_cast<const bf16x8*>(Ws + frag_off<64>(i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        xf[j] = *reinterpret_cast<const bf16x8*>(Xs + frag_off<64>(wave * 64 + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }
    // bf16 NHWC stores (4 consecutive channels of one pixel per lane) + sums
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int px = wave * 64 + j * 16 + (lane & 15);
      if (px < t.Qs) {
        bf16_t* yrow = a.y + (t.row * a.Q + t.q0 + px) * a.ldy + cg;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = i * 16 + ((lane >> 4) << 2);
          uint2 o;
          o.x = pack_bf2(acc[i][j][0], acc[i][j][1]);
          o.y = pack_bf2(acc[i][j][2], acc[i][j][3]);
          *reinterpret_cast<uint2*>(yrow + co) = o;
#pragma unroll
          for (int e = 0; e < 4; ++e) { q0[i][e] += acc[i][j][e]; q1[i][e] += acc[i][j][e] * acc[i][j][e]; }
        }
      }
    }
  }
  if (!a.stats) return;
  // fold over the 16 pixel lanes, then the 4 waves, then one replica atomic per channel
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        q0[i][e] += __shfl_xor(q0[i][e], o, 64);
        q1[i][e] += __shfl_xor(q1[i][e], o, 64);
      }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][64][2]
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = i * 16 + ((lane >> 4) << 2) + e;
        red[(wave * 64 + c) * 2] = q0[i][e];
        red[(wave * 64 + c) * 2 + 1] = q1[i][e];
      }
  }
  __syncthreads();
  if (tid < 64) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) { s0 += red[(w * 64 + tid) * 2]; s1 += red[(w * 64 + tid) * 2 + 1]; }
    double* rep = a.stats + (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout + cg;
    atomicAdd(rep + tid, (double)s0);
    atomicAdd(rep + a.Cout + tid, (double)s1);
  }
  if (a.bn.ticket) {
    int* flag = reinterpret_cast<int*>(smem + 4 * 64 * 2 * sizeof(float));
    if (last_block_arrive(a.bn.ticket, gridDim.x * gridDim.y, flag, tid < 64)) bn_finalize(a.bn);
  }
}

template <bool FUSE>
__global__ void __launch_bounds__(256, 2) stem_wgrad_kernel(ConvWgradArgs a, int rows_per_block) {
  // LDS: dY [256 px][64 co] | im2col [256 px][64 k] (pixel-major tr tiles) | patch
  extern __shared__ __attribute__((aligned(16))) char smem[];
  typedef TrTile<64, 64, 256> TT;
  char* Ds = smem;
  char* Xs = smem + 256 * 128;
  bf16_t* patch = reinterpret_cast<bf16_t*>(smem + 2 * 256 * 128);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;  // 32 co x 32 k per wave
  const int g = lane >> 4, li = lane & 15, trq = li >> 2, trp = li & 3;
  const float* img = reinterpret_cast<const float*>(a.x);
  const int total_rows = a.N * a.P * ((a.Q + 255) >> 8);  // units (stem_unit)
  const int r0 = xcd_remap(blockIdx.x, gridDim.x) * rows_per_block;
  const int r1 = min(total_rows, r0 + rows_per_block);
  const int cg = blockIdx.y * 64;  // 64-channel output group (Wide stem: 2 groups)
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused stem BN-backward apply: this thread's 8 channels (c8 = tid & 7 for
  // every j below) get dY = A dZ + B y + C (bn_bwd_apply_kernel's coefficients)
  float cA[FUSE ? 8 : 1], cB[FUSE ? 8 : 1], cC[FUSE ? 8 : 1];
  if constexpr (FUSE) {
    float* coef = reinterpret_cast<float*>(smem + 2 * 256 * 128 + 7 * kStemPatchW * 2);  // [3][64]
    if (tid < 64) {
      const BnBwdArgs& b = a.bn;
      const int ch = cg + tid;
      double s1 = 0.0, s2 = 0.0;
      for (int r = 0; r < kStatRep; ++r) {
        s1 += b.sums[(size_t)r * 2 * b.C + ch];
        s2 += b.sums[(size_t)r * 2 * b.C + b.C + ch];
      }
      const double inv_n = 1.0 / (double)b.npix;
      const float k1 = __fmul_rn(b.gamma[ch], b.invstd[ch]);
      const float m1 = (float)__dmul_rn(s1, inv_n), m2 = (float)__dmul_rn(s2, inv_n);
      bn_bwd_coef_abc(k1, m1, m2, b.invstd[ch], b.mean[ch], coef[tid], coef[64 + tid], coef[128 + tid]);
      if (blockIdx.x == 0) {
        b.dgamma[ch] = (float)s2;
        b.dbeta[ch] = (float)s1;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int c = ((tid & 7) << 3) + k;
      cA[k] = coef[c]; cB[k] = coef[64 + c]; cC[k] = coef[128 + c];
    }
  }
  // register prefetch of the next row: dY (8 x 16 B per thread) + input patch
  // (fused: dZ and y, combined at the LDS store)
  uint4 dyv[8], yv[FUSE ? 8 : 1];
  StemPatch pf;
  auto fetch = [&](int u) {
    const StemUnit t = stem_unit(u, a.P, a.Q);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + j * 256, px = i >> 3, c8 = i & 7;
      const size_t pix = t.row * a.Q + t.q0 + px;
      if constexpr (FUSE) {
        dyv[j] = px < t.Qs ? *reinterpret_cast<const uint4*>(a.bn.da + pix * a.bn.ldda + cg + c8 * 8)
                           : make_uint4(0, 0, 0, 0);
        yv[j] = px < t.Qs ? *reinterpret_cast<const uint4*>(a.bn.y + pix * a.bn.ldy + cg + c8 * 8)
                          : make_uint4(0, 0, 0, 0);
      } else {
        dyv[j] = px < t.Qs ? *reinterpret_cast<const uint4*>(a.dy + pix * a.lddy + cg + c8 * 8)
                           : make_uint4(0, 0, 0, 0);
      }
    }
    stem_fetch(img, t, a.H, a.W, pf);
  };
  if (r0 < r1) fetch(r0);
  for (int row = r0; row < r1; ++row) {
    const StemUnit t = stem_unit(row, a.P, a.Q);
    __syncthreads();  // previous unit's tiles consumed
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = tid + j * 256, px = i >> 3, c8 = i & 7;
      uint4 v = dyv[j];
      if constexpr (FUSE) {
        if (px < t.Qs) {
          float dz[8], y[8], o[8];
          unpack8(dyv[j], dz);
          unpack8(yv[j], y);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = fmaf(cA[k], dz[k], fmaf(cB[k], y[k], cC[k]));
          v = pack8(o);
        } else {
          v = make_uint4(0, 0, 0, 0);
        }
      }
      *reinterpret_cast<uint4*>(Ds + TT::off(px, c8 * 8)) = v;
    }
    stem_store_patch(pf, t.Qs, patch);
    if (row + 1 < r1) fetch(row + 1);
    __syncthreads();
    {
      uint4 r8[8];
      if (tid < t.Qs) {
        stem_im2col_row(patch, tid, r8);
      } else {
#pragma unroll
        for (int c8 = 0; c8 < 8; ++c8) r8[c8] = make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int c8 = 0; c8 < 8; ++c8) *reinterpret_cast<uint4*>(Xs + TT::off(tid, c8 * 8)) = r8[c8];
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {  // 32 px per MFMA k-step
      const int p_lo = kk * 32 + 8 * g + trq;
      bf16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = wm * 32 + i * 16 + 4 * trp;
        af[i] = tr_read8(Ds + TT::off(p_lo, col), Ds + TT::off(p_lo + 4, col));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int col = wn * 32 + j * 16 + 4 * trp;
        bf[j] = tr_read8(Xs + TT::off(p_lo, col), Xs + TT::off(p_lo + 4, col));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  if (a.slab && gridDim.x > 1) {  // one split per block row (SLAB_STEM), summed by the reduce
    f32x4* dst = reinterpret_cast<f32x4*>(a.slab) + ((size_t)blockIdx.x * gridDim.y + blockIdx.y) * 1024 +
                 (size_t)wave * 256 + lane;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) dst[(i * 2 + j) * 64] = acc[i][j];
    return;
  }
  // D[co][k]: lane holds k = .. + li, co = .. + 4g + e;  dW row length 64
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int k = wn * 32 + j * 16 + li;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = cg + wm * 32 + i * 16 + 4 * g + e;
        if (a.slab) a.dw[co * 64 + k] = acc[i][j][e];
        else atomicAdd(a.dw + co * 64 + k, acc[i][j][e]);
      }
    }
}

// split-K partials of the last wgrad launch, summed by launch_wgrad_finish
struct PendingReduce { const float* slab; float* dw; SlabLayout L; };
static thread_local PendingReduce g_pending{};

// largest split count whose register-native partials (bytes_per_split each)
// fit the slab; 1 = no split-K reduction (each block owns its dW tile)
static long long slab_split_cap(const ConvWgradArgs& a, long long bytes_per_split) {
  if (!a.slab || bytes_per_split <= 0) return 1LL << 30;  // atomic path: no cap
  const long long cap = (long long)(a.slab_bytes / (size_t)bytes_per_split);
  return cap < 1 ? 1 : cap;
}

hipError_t launch_stem_fwd(const ConvFwdArgs& a, hipStream_t st) {
  if (a.Cout % 64 || a.R != 7 || a.stride != 2 || a.pad != 3 || a.ldy % 4) return hipErrorInvalidValue;
  const int rows = a.N * a.P * ((a.Q + 255) / 256);  // 256-pixel units
  const int per = std::max(1, (rows + 511) / 512);  // ~2 blocks per CU
  const size_t lds = 64 * 128 + 256 * 128 + 7 * kStemPatchW * 2;
  set_kernel_tag("stem_fwd_kernel");
  hipLaunchKernelGGL(stem_fwd_kernel, dim3((rows + per - 1) / per, a.Cout / 64), dim3(256), lds, st, a, per);
  return hipGetLastError();
}

hipError_t launch_stem_wgrad(const ConvWgradArgs& a, hipStream_t st) {
  if (a.Cout % 64 || a.R != 7 || a.stride != 2 || a.pad != 3 || a.lddy % 8) return hipErrorInvalidValue;
  const int groups = a.Cout / 64;
  const int rows = a.N * a.P * ((a.Q + 255) / 256);  // 256-pixel units
  int per = std::max(1, (rows * groups + 511) / 512);  // ~2 blocks per CU
  // one register-native 64x64 partial (16 KiB) per block
  const long long cap = slab_split_cap(a, 1024 * 16 * groups);
  while ((rows + per - 1) / per > cap) ++per;
  const int blocks = (rows + per - 1) / per;
  const size_t lds = 2 * 256 * 128 + 7 * kStemPatchW * 2 + (a.bn_fuse ? 3 * 64 * sizeof(float) : 0);
  if (a.bn_fuse && (a.bn.C != a.Cout || a.bn.ldda % 8 || a.bn.ldy % 8 || !a.bn.sums)) return hipErrorInvalidValue;
  set_kernel_tag("stem_wgrad_kernel");
  if (a.bn_fuse) hipLaunchKernelGGL(stem_wgrad_kernel<true>, dim3(blocks, groups), dim3(256), lds, st, a, per);
  else hipLaunchKernelGGL(stem_wgrad_kernel<false>, dim3(blocks, groups), dim3(256), lds, st, a, per);
  if (a.slab && blocks > 1) {
    SlabLayout L = {};
    L.kind = SLAB_STEM; L.splits = blocks; L.blocks = groups; L.nw = 4; L.nf = 4; L.units = 1024LL * groups;
    L.Cout = a.Cout; L.C = 64; L.Krow = 64; L.cmax = 64;
    g_pending = PendingReduce{a.slab, a.dw, L};
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// host-side launch selection
// ---------------------------------------------------------------------------

template <int MODE, int ALOAD, int BM, int BN, int BK, int WM, int WN>
static hipError_t launch_fwd_cfg(const ConvFwdArgs& a0, int classes, hipStream_t st) {
  ConvFwdArgs a = a0;
  a.nblocks = (a.Cout + BN - 1) / BN;
  const int M = a.N * a.Pc * a.Qc;
  a.mblocks = (M + BM - 1) / BM;
  const size_t lds = 2 * (size_t)(BM + BN) * BK * 2;
  size_t need = lds;
  const size_t red = (size_t)WM * BN * 3 * sizeof(float) + 16;
  if (red > need) need = red;
  dim3 grid(a.mblocks * a.nblocks, 1, classes);
  set_kernel_tag("conv_fwd_kernel<%d, %d, %d, %d, %d, %d, %d>", MODE, ALOAD, BM, BN, BK, WM, WN);
  hipLaunchKernelGGL((conv_fwd_kernel<MODE, ALOAD, BM, BN, BK, WM, WN>), grid, dim3(256), need, st, a);
  return hipGetLastError();
}

template <int MODE, int BM, int BN, int BK, int NS, int WM, int WN, bool DS = false>
static hipError_t launch_glds_cfg(const ConvFwdArgs& a0, int classes, hipStream_t st) {
  ConvFwdArgs a = a0;
  a.nblocks = (a.Cout + BN - 1) / BN;
  const int M = a.N * a.Pc * a.Qc;
  a.mblocks = (M + BM - 1) / BM;
  constexpr int NW = WM * WN, ROWB = BK * 2, RPI = 1024 / ROWB;
  constexpr size_t B_ROWS = ((BN + RPI * NW - 1) / (RPI * NW)) * RPI * NW;
  // a K loop shorter than the pipeline (1x1 convs, the convT forward as one
  // GEMM) only ever touches its first KT stage buffers: allocate just those,
  // so more blocks fit per CU
  int stages = NS;
  if ((MODE == MODE_FWD || MODE == MODE_SHUF) && a.C % BK == 0) {
    const int kt = a.R * a.S * (a.C / BK);
    if (kt >= 1 && kt < stages) stages = kt;
  }
  if (DS) stages = NS;  // the downsample tile sits behind all NS stages
  size_t lds = (size_t)stages * (BM + B_ROWS) * ROWB;
  if (DS) lds += (size_t)(a.C / BK) * B_ROWS * ROWB;
  const size_t red = (size_t)WM * BN * 3 * sizeof(float) + 16;
  if (red > lds) lds = red;
  dim3 grid(a.mblocks * a.nblocks, 1, classes);
  set_kernel_tag(DS ? "conv_glds_kernel<%d, %d, %d, %d, %d, %d, %d> +ds" : "conv_glds_kernel<%d, %d, %d, %d, %d, %d, %d>",
                 MODE, BM, BN, BK, NS, WM, WN);
  hipLaunchKernelGGL((conv_glds_kernel<MODE, BM, BN, BK, NS, WM, WN, DS>), grid, dim3(NW * 64), lds, st, a);
  return hipGetLastError();
}

static int env_int(const char* name) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : 0;
}
static int g_cfg_override = env_int("UNET_CONV_CFG");  // tuning runs only
void set_conv_config(int cfg) { g_cfg_override = cfg; }

// Explicit tile configurations (tuning / override).  Returns hipErrorNotSupported
// when the configuration does not apply to the shape.
template <int MODE>
static hipError_t launch_glds_fixed(const ConvFwdArgs& a, int classes, int cfg, hipStream_t st) {
  const bool bk64 = (a.C % 64) == 0;
  switch (cfg) {
    case 1: return bk64 ? launch_glds_cfg<MODE, 128, 64, 64, 3, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 2: return bk64 ? launch_glds_cfg<MODE, 128, 64, 64, 2, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 3: return launch_glds_cfg<MODE, 128, 64, 32, 3, 2, 2>(a, classes, st);
    case 4: return bk64 ? launch_glds_cfg<MODE, 128, 128, 64, 2, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 5: return launch_glds_cfg<MODE, 128, 128, 32, 3, 2, 2>(a, classes, st);
    case 6: return bk64 ? launch_glds_cfg<MODE, 128, 128, 64, 3, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 7: return bk64 ? launch_glds_cfg<MODE, 64, 64, 64, 3, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 8: return bk64 ? launch_glds_cfg<MODE, 256, 64, 64, 2, 4, 1>(a, classes, st) : hipErrorNotSupported;
    case 9: return bk64 ? launch_glds_cfg<MODE, 128, 32, 64, 3, 4, 1>(a, classes, st) : hipErrorNotSupported;
    case 10: return launch_glds_cfg<MODE, 256, 32, 32, 3, 4, 1>(a, classes, st);
    case 11: return launch_glds_cfg<MODE, 128, 32, 32, 4, 4, 1>(a, classes, st);
    case 12: return launch_glds_cfg<MODE, 256, 64, 32, 3, 4, 1>(a, classes, st);
    case 13: return bk64 ? launch_glds_cfg<MODE, 128, 64, 64, 4, 2, 2>(a, classes, st) : hipErrorNotSupported;
    case 14: return launch_glds_cfg<MODE, 128, 128, 32, 4, 2, 2>(a, classes, st);
    // 8-wave (512-thread) variants
    case 15: return bk64 ? launch_glds_cfg<MODE, 128, 128, 64, 2, 2, 4>(a, classes, st) : hipErrorNotSupported;
    case 16: return bk64 ? launch_glds_cfg<MODE, 128, 128, 64, 3, 2, 4>(a, classes, st) : hipErrorNotSupported;
    case 17: return bk64 ? launch_glds_cfg<MODE, 256, 128, 64, 2, 4, 2>(a, classes, st) : hipErrorNotSupported;
    case 18: return bk64 ? launch_glds_cfg<MODE, 128, 64, 64, 2, 4, 2>(a, classes, st) : hipErrorNotSupported;
    case 19: return bk64 ? launch_glds_cfg<MODE, 256, 64, 64, 2, 4, 2>(a, classes, st) : hipErrorNotSupported;
    case 20: return bk64 ? launch_glds_cfg<MODE, 256, 256, 64, 2, 2, 4>(a, classes, st) : hipErrorNotSupported;
    case 21: return launch_glds_cfg<MODE, 128, 128, 32, 4, 2, 4>(a, classes, st);
    case 22: return launch_glds_cfg<MODE, 256, 32, 32, 3, 8, 1>(a, classes, st);
    case 23: return bk64 ? launch_glds_cfg<MODE, 256, 128, 64, 3, 4, 2>(a, classes, st) : hipErrorNotSupported;
    case 24: return launch_glds_cfg<MODE, 256, 64, 32, 3, 4, 2>(a, classes, st);
    case 25: return bk64 ? launch_glds_cfg<MODE, 64, 64, 64, 3, 2, 4>(a, classes, st) : hipErrorNotSupported;
    default: return hipErrorNotSupported;
  }
}

// forward with the folded downsample (MODE_FWD, a.wds): the stride-2 conv1
// tiles launch_glds picks for these shapes (enc3.0 / enc4.0 conv1).  0: not
// folded; 1: 128 x 128 3-stage tiles; 2: 64 x 64 3-stage tiles.  enc2.0 (2-stage
// 128 x 128 tiles, 512 blocks) is not: the second accumulator set (169 VGPRs)
// halves its blocks per CU and the fused launch measured slower than the two
// separate ones (61.9 vs 38.0 + 21.8 us)
static int glds_ds_cfg(const ConvFwdArgs& a) {
  if (a.C % 64 || a.R != 3 || a.S != 3 || a.stride != 2 || a.pad != 1 || a.stride_w || a.ldyds % 4 || a.add ||
      a.fold_on || a.bb.sums || a.x2 || a.ysplit || a.xform || a.P * 2 != a.H + (a.H & 1) || a.Q * 2 != a.W + (a.W & 1))
    return 0;
  const long long M = (long long)a.N * a.P * a.Q;
  auto nblk = [&](long long bm, long long bn) { return ((M + bm - 1) / bm) * ((a.Cout + bn - 1) / bn); };
  if (a.Cout == 256 && nblk(128, 128) >= 240) return 1;
  if (a.Cout > 64 && nblk(128, 128) >= 240) return 0;
  return 2;
}
bool conv_fwd_ds_ok(const ConvFwdArgs& a) { return glds_ds_cfg(a) != 0; }
static hipError_t launch_glds_ds(const ConvFwdArgs& a, hipStream_t st) {
  if (!a.yds) return hipErrorInvalidValue;
  switch (glds_ds_cfg(a)) {
    case 1: return launch_glds_cfg<MODE_FWD, 128, 128, 64, 3, 2, 4, true>(a, 1, st);
    case 2: return launch_glds_cfg<MODE_FWD, 64, 64, 64, 3, 2, 2, true>(a, 1, st);
    default: return hipErrorNotSupported;
  }
}

template <int MODE>
static hipError_t launch_glds(const ConvFwdArgs& a, int classes, hipStream_t st) {
  if constexpr (MODE != MODE_SHUF) {  // tuning overrides: conv / dgrad shapes only
    if (g_cfg_override > 0) {
      const hipError_t e = launch_glds_fixed<MODE>(a, classes, g_cfg_override, st);
      if (e != hipErrorNotSupported) return e;
    }
  }
  // Selection measured by scripts/tune_conv.py on MI355X (Base config shapes,
  // profiles/r01/tune_conv*.txt): 8-wave 256x256 / 128x128 2-stage tiles
  // wherever they still give >= ~1 block per CU, 64x64 for the 16x16 encoder
  // stage, 8-wave 256x64 for the 64-channel full-resolution layers.
  const bool bk64 = (a.C % 64) == 0;
  const long long M = (long long)a.N * a.Pc * a.Qc * classes;
  auto nblk = [&](long long bm, long long bn) { return ((M + bm - 1) / bm) * ((a.Cout + bn - 1) / bn); };
  // attention-gate 1x1 convs (scripts/sweep_glds_cfg.sh --attention): the
  // narrow full-resolution ones prefer 8-wave 256-pixel tiles (-25..-30 %)
  const bool pw = a.R == 1 && a.S == 1 && a.stride == 1;
  if (pw && a.Cout <= 32) return launch_glds_cfg<MODE, 256, 32, 32, 3, 8, 1>(a, classes, st);
  if (pw && a.Cout == 64 && !bk64) return launch_glds_cfg<MODE, 256, 64, 32, 3, 4, 2>(a, classes, st);
  if (a.Cout <= 32) {
    return bk64 ? launch_glds_cfg<MODE, 128, 32, 64, 3, 4, 1>(a, classes, st)
                : launch_glds_cfg<MODE, 128, 32, 32, 3, 4, 1>(a, classes, st);
  }
  if (bk64 && a.Cout >= 256 && nblk(256, 256) >= 256)
    return launch_glds_cfg<MODE, 256, 256, 64, 2, 2, 4>(a, classes, st);
  // per-layer sweep (scripts/sweep_glds_cfg.sh): the 256-channel stride-2
  // layers (enc3.0 conv1 forward, enc4.0 conv1+downsample dgrad) keep a third
  // stage in flight (-18 %); upconv1's dgrad (k2s2, 32 -> 64 channels, K = 128)
  // prefers 256-pixel tiles (-14 %)
  if (bk64 && a.stride == 2 && a.Cout == 256 && nblk(128, 128) >= 240)
    return launch_glds_cfg<MODE, 128, 128, 64, 3, 2, 4>(a, classes, st);
  if (!bk64 && a.R == 2 && a.stride == 2 && a.Cout == 64)
    return launch_glds_cfg<MODE, 256, 64, 32, 3, 4, 2>(a, classes, st);
  if (a.Cout > 64 && nblk(128, 128) >= 240) {
    return bk64 ? launch_glds_cfg<MODE, 128, 128, 64, 2, 2, 4>(a, classes, st)
                : launch_glds_cfg<MODE, 128, 128, 32, 3, 2, 2>(a, classes, st);
  }
  if (bk64 && nblk(128, 64) <= 256) return launch_glds_cfg<MODE, 64, 64, 64, 3, 2, 2>(a, classes, st);
  if (bk64 && nblk(256, 64) >= 512) return launch_glds_cfg<MODE, 256, 64, 64, 2, 4, 2>(a, classes, st);
  return bk64 ? launch_glds_cfg<MODE, 128, 64, 64, 2, 2, 2>(a, classes, st)
              : launch_glds_cfg<MODE, 128, 64, 32, 3, 2, 2>(a, classes, st);
}

template <int BM, int BN, int NS, int WM, int WN>
static hipError_t launch_f8_cfg(const ConvFwdArgs& a0, hipStream_t st) {
  ConvFwdArgs a = a0;
  a.nblocks = (a.Cout + BN - 1) / BN;
  const int M = a.N * a.P * a.Q;
  a.mblocks = (M + BM - 1) / BM;
  a.Pc = a.P; a.Qc = a.Q;
  constexpr int NW = WM * WN, RPI = 8;
  constexpr size_t B_ROWS = ((BN + RPI * NW - 1) / (RPI * NW)) * RPI * NW;
  size_t lds = (size_t)NS * (BM + B_ROWS) * 128;
  const size_t red = (size_t)WM * BN * 3 * sizeof(float) + 16;
  if (red > lds) lds = red;
  set_kernel_tag("conv_f8_kernel<%d, %d, %d, %d, %d>", BM, BN, NS, WM, WN);
  hipLaunchKernelGGL((conv_f8_kernel<BM, BN, NS, WM, WN>), dim3(a.mblocks * a.nblocks), dim3(NW * 64), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_conv_fwd_f8(const ConvFwdArgs& a, hipStream_t st) {
  if (!a.f8x || !a.f8w || a.C % 16 || a.ldx % 16 || a.ysplit || a.bb.sums || a.x2) return hipErrorInvalidValue;
  if ((size_t)a.N * a.H * a.W * a.ldx >= 0x80000000ull) return hipErrorInvalidValue;
  if ((size_t)a.Cout * a.R * a.S * a.C >= 0x80000000ull) return hipErrorInvalidValue;
  const long long M = (long long)a.N * a.P * a.Q;
  auto nblk = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((a.Cout + bn - 1) / bn); };
  static const int forced = std::getenv("UNET_F8CFG") ? std::atoi(std::getenv("UNET_F8CFG")) : 0;  // tuning
  switch (forced) {
    case 1: return launch_f8_cfg<256, 64, 3, 4, 2>(a, st);
    case 2: return launch_f8_cfg<256, 128, 2, 4, 2>(a, st);
    case 3: return launch_f8_cfg<128, 128, 3, 2, 2>(a, st);
    case 4: return launch_f8_cfg<256, 256, 2, 2, 4>(a, st);
    case 5: return launch_f8_cfg<128, 256, 2, 2, 4>(a, st);
    default: break;
  }
  if (a.Cout <= 64) return launch_f8_cfg<256, 64, 3, 4, 2>(a, st);
  if (a.Cout >= 256 && nblk(256, 256) >= 256) return launch_f8_cfg<256, 256, 2, 2, 4>(a, st);
  if (a.Cout >= 256 && nblk(128, 256) >= 256) return launch_f8_cfg<128, 256, 2, 2, 4>(a, st);
  if (nblk(256, 128) >= 512) return launch_f8_cfg<256, 128, 2, 4, 2>(a, st);
  if (nblk(128, 128) >= 256) return launch_f8_cfg<128, 128, 3, 2, 2>(a, st);
  return launch_f8_cfg<64, 128, 3, 2, 2>(a, st);
}


hipError_t launch_conv_fwd(const ConvFwdArgs& a0, int mode, hipStream_t st) {
  // a separate column stride exists in the LDS-DMA implicit GEMM's forward only
  if (a0.stride_w && (mode != MODE_FWD || a0.C % 64 || a0.x2 || a0.ysplit || a0.xform)) return hipErrorInvalidValue;
  // the folded downsample range exists only in the LDS-DMA transposed kernel
  if (a0.x2 && (mode != MODE_TRANS || a0.C2 != a0.C || a0.stride != 2 || a0.pad != 1))
    return hipErrorInvalidValue;
  if (a0.ysplit && (mode == MODE_STEM || mode == MODE_SHUF || a0.csplit % 4 || a0.ldysplit % 4 ||
                    a0.bb.sums || a0.add))
    return hipErrorInvalidValue;
  if (a0.fold_on && (mode != MODE_FWD || a0.stats || a0.bb.sums)) return hipErrorInvalidValue;
  // dedicated stem kernel: 64 output channels (Base); the Wide stem (128) takes
  // the generic implicit-GEMM path below
  if (mode == MODE_STEM && a0.Cout % 64 == 0) return launch_stem_fwd(a0, st);
  if (mode == MODE_SHUF) {  // convT k2s2 forward: a0 holds the transposed-conv geometry
    if (a0.R != 2 || a0.S != 2 || a0.stride != 2 || a0.pad != 0 || a0.Cout % 4 || a0.C % 32 ||
        a0.P != 2 * a0.H || a0.Q != 2 * a0.W || a0.stats || a0.add || a0.bb.sums)
      return hipErrorInvalidValue;
    if ((size_t)a0.N * a0.H * a0.W * a0.ldx * 2 >= 0x80000000ull) return hipErrorInvalidValue;
    ConvFwdArgs a = a0;
    a.Cout = 4 * a0.Cout;
    a.R = a.S = 1; a.stride = 1; a.pad = 0;
    a.Pc = a.H; a.Qc = a.W;
    return launch_glds<MODE_SHUF>(a, 1, st);
  }
  if (a0.wds && (mode != MODE_FWD || a0.C % 64)) return hipErrorInvalidValue;
  if (mode != MODE_STEM && a0.C % 32 == 0) {
    ConvFwdArgs a = a0;
    if ((size_t)a.N * a.H * a.W * a.ldx * 2 >= 0x80000000ull) return hipErrorInvalidValue;
    if (a.wds) {  // the folded downsample exists in the implicit-GEMM forward only
      if ((size_t)a.N * a.P * a.Q * a.ldyds * 2 >= 0x80000000ull) return hipErrorInvalidValue;
      a.Pc = a.P;
      a.Qc = a.Q;
      return launch_glds_ds(a, st);
    }
    if (g_cfg_override <= 0) {
      const hipError_t e = launch_conv3x3_ws(a, mode == MODE_TRANS ? 1 : 0, st);
      if (e != hipErrorNotSupported) return e;
    }
    if (a.xform) return hipErrorInvalidValue;  // the BN-apply prologue exists in the weight-stationary kernel only
    if (mode == MODE_TRANS) {
      if (a.P % a.stride || a.Q % a.stride) return hipErrorInvalidValue;
      if (g_cfg_override <= 0) {
        const hipError_t e = launch_conv3x3s2_dgrad(a, st);
        if (e != hipErrorNotSupported) return e;
      }
      a.Pc = a.P / a.stride;
      a.Qc = a.Q / a.stride;
      return launch_glds<MODE_TRANS>(a, a.stride * a.stride, st);
    }
    a.Pc = a.P;
    a.Qc = a.Q;
    return launch_glds<MODE_FWD>(a, 1, st);
  }
  return launch_conv_fwd_v1(a0, mode, st);
}

hipError_t launch_conv_fwd_v1(const ConvFwdArgs& a0, int mode, hipStream_t st) {
  ConvFwdArgs a = a0;
  int classes = 1;
  if (mode == MODE_TRANS) {
    if (a.P % a.stride || a.Q % a.stride) return hipErrorInvalidValue;
    a.Pc = a.P / a.stride;
    a.Qc = a.Q / a.stride;
    classes = a.stride * a.stride;
  } else {
    a.Pc = a.P;
    a.Qc = a.Q;
  }
  if (mode == MODE_STEM) {
    return launch_fwd_cfg<MODE_FWD, ALOAD_STEM, 128, 64, 64, 2, 2>(a, 1, st);
  }
  if (a.C % 32) return hipErrorInvalidValue;
  const bool bk64 = (a.C % 64) == 0;
  const int M = a.N * a.Pc * a.Qc * classes;
#define SEL(MD)                                                                              \
  if (a.Cout <= 32) {                                                                        \
    return bk64 ? launch_fwd_cfg<MD, ALOAD_NHWC, 128, 32, 64, 4, 1>(a, classes, st)          \
                : launch_fwd_cfg<MD, ALOAD_NHWC, 128, 32, 32, 4, 1>(a, classes, st);         \
  } else if (a.Cout <= 64 || M < 32768) {                                                    \
    return bk64 ? launch_fwd_cfg<MD, ALOAD_NHWC, 128, 64, 64, 2, 2>(a, classes, st)          \
                : launch_fwd_cfg<MD, ALOAD_NHWC, 128, 64, 32, 2, 2>(a, classes, st);         \
  } else {                                                                                   \
    return bk64 ? launch_fwd_cfg<MD, ALOAD_NHWC, 128, 128, 64, 2, 2>(a, classes, st)         \
                : launch_fwd_cfg<MD, ALOAD_NHWC, 128, 128, 32, 2, 2>(a, classes, st);        \
  }
  if (mode == MODE_FWD) { SEL(MODE_FWD) } else { SEL(MODE_TRANS) }
#undef SEL
}

template <int XLOAD, int BMO, int BNC, int BKP, int WM, int WN>
static hipError_t launch_wgrad_cfg(const ConvWgradArgs& a0, hipStream_t st) {
  ConvWgradArgs a = a0;
  a.co_blocks = (a.Cout + BMO - 1) / BMO;
  const int ccount = (XLOAD == XLOAD_STEM) ? 64 : a.C;
  a.c_blocks = (ccount + BNC - 1) / BNC;
  const int taps = (XLOAD == XLOAD_STEM) ? 1 : a.R * a.S;
  const int tiles = a.co_blocks * a.c_blocks * taps;
  const long long M = (long long)a.N * a.P * a.Q;
  // split-K over pixels: enough blocks to fill 256 CUs, but keep >= 1024 flop per
  // fp32 atomic byte (chip atomic rate ~1.3 TB/s, MI355X_MICROARCH.md).
  long long splits = (2048 + tiles - 1) / tiles;
  const long long max_by_atomic = M / 512 > 0 ? M / 512 : 1;  // >= 512 px per block
  if (splits > max_by_atomic) splits = max_by_atomic;
  if (splits < 1) splits = 1;
  constexpr int FM = BMO / WM / 16, FN = BNC / WN / 16;
  const long long units = (long long)tiles * 4 * FM * FN * 64;
  ConvWgradArgs capped = a;  // keep the partial slab (and its reduction) <= 16 MiB
  if (capped.slab_bytes > ((size_t)16 << 20)) capped.slab_bytes = (size_t)16 << 20;
  const long long cap = slab_split_cap(capped, units * 16);
  if (splits > cap) splits = cap;
  long long per = (M + splits - 1) / splits;
  per = (per + BKP - 1) / BKP * BKP;
  splits = (M + per - 1) / per;
  a.px_per_split = (int)per;
  dim3 grid(tiles, 1, (unsigned)splits);
  const size_t lds = 2 * (size_t)BKP * (BMO + BNC) * 2;
  set_kernel_tag("conv_wgrad_kernel<%d, %d, %d, %d, %d, %d>", XLOAD, BMO, BNC, BKP, WM, WN);
  hipLaunchKernelGGL((conv_wgrad_kernel<XLOAD, BMO, BNC, BKP, WM, WN>), grid, dim3(256), lds, st, a);
  if (a.slab && splits > 1) {
    SlabLayout L = {};
    L.kind = SLAB_GEMM; L.splits = (int)splits; L.blocks = tiles; L.nw = 4; L.nf = FM * FN; L.units = units;
    L.Cout = a.Cout; L.C = (XLOAD == XLOAD_STEM) ? 0 : a.C; L.Krow = (XLOAD == XLOAD_STEM) ? 64 : a.R * a.S * a.C;
    L.cmax = ccount; L.co_blocks = a.co_blocks; L.c_blocks = a.c_blocks;
    L.bmo = BMO; L.bnc = BNC; L.wm = WM; L.wn = WN; L.fn = FN;
    g_pending = PendingReduce{a.slab, a.dw, L};
  }
  return hipGetLastError();
}


// splits so that the grid is ~one block per CU (the halo kernels hold 96-144 KB
// of LDS), at least one tile per split
template <int TW, int CI, bool CO32>
static void halo_geometry(const ConvWgradArgs& a, int& blocks_xy, int& tiles, int& per, int& splits) {
  constexpr int TH = 128 / TW;
  blocks_xy = (CO32 ? a.Cout / 32 : (a.Cout + 63) / 64) * (a.C / CI);
  tiles = a.N * (a.P / TH) * (a.Q / TW);
  constexpr int target = 256;  // split-K blocks aimed for
  splits = std::max(1, std::min(tiles, target / blocks_xy));
  per = (tiles + splits - 1) / splits;
  splits = (tiles + per - 1) / per;
}

template <int TW, int CI, bool CO32 = false, int NSO = 0, int SD = 1, bool DSF = false>
static hipError_t launch_wgrad_halo(const ConvWgradArgs& a0, hipStream_t st) {
  ConvWgradArgs a = a0;
  a.co_blocks = CO32 ? a.Cout / 32 : (a.Cout + 63) / 64;
  a.c_blocks = a.C / CI;
  int blocks_xy, tiles, per, splits;
  halo_geometry<TW, CI, CO32>(a, blocks_xy, tiles, per, splits);
  constexpr int NW = CI / 8;
  constexpr int SW = CO32 ? NW / 2 : NW;  // wave slots per block in the slab
  constexpr int NF = DSF ? 20 : 18;
  const long long units = (long long)blocks_xy * SW * NF * 64;
  const long long cap = slab_split_cap(a, units * 16);
  if (splits > cap) {
    splits = (int)cap;
    per = (tiles + splits - 1) / splits;
    splits = (tiles + per - 1) / per;
  }
  constexpr int NS = NSO ? NSO : (CI == 64 ? 3 : 4);
  constexpr size_t lds = (size_t)NS * (128 * 128 * (DSF ? 2 : 1) + wgrad_halo_rows<TW, CI, SD>() * CI * 2);
  static_assert(lds <= 163840, "LDS");
  // the full template argument list, as rocprofv3 spells the kernel
  set_kernel_tag("wgrad3x3_halo_kernel<%d, %d, %d, %s, %d, %s>", TW, NS, CI, CO32 ? "true" : "false", SD,
                 DSF ? "true" : "false");
  hipLaunchKernelGGL((wgrad3x3_halo_kernel<TW, NS, CI, CO32, SD, DSF>), dim3(blocks_xy * splits), dim3(CI * 8),
                     lds, st, a, tiles, per);
  if (a.slab && splits > 1) {
    SlabLayout L = {};
    L.kind = SLAB_HALO; L.splits = splits; L.blocks = blocks_xy; L.nw = SW; L.nf = NF; L.units = units;
    L.Cout = a.Cout; L.C = a.C; L.Krow = 9 * a.C; L.cmax = a.C;
    L.co_blocks = a.co_blocks; L.c_blocks = a.c_blocks; L.ci = CI; L.co32 = CO32 ? 1 : 0;
    L.dw2_off = DSF ? (long long)(a.dw2 - a.dw) : 0;
    g_pending = PendingReduce{a.slab, a.dw, L};
  }
  return hipGetLastError();
}

// wgrad3x3_ld_kernel: C % 64 == 0, Cout % 64 == 0, Q % 32 == 0, P % 4 == 0
static hipError_t launch_wgrad_ld(const ConvWgradArgs& a0, hipStream_t st) {
  ConvWgradArgs a = a0;
  a.co_blocks = a.Cout / 64;
  a.c_blocks = a.C / 64;
  int blocks_xy, tiles, per, splits;
  halo_geometry<32, 64, false>(a, blocks_xy, tiles, per, splits);
  const long long units = (long long)blocks_xy * kWlNW * 18 * 64;
  const long long cap = slab_split_cap(a, units * 16);
  if (splits > cap) {
    splits = (int)cap;
    per = (tiles + splits - 1) / splits;
    splits = (tiles + per - 1) / per;
  }
  constexpr size_t lds = (size_t)kWlNS * kWlStage;
  static_assert(lds <= 163840, "LDS");
  set_kernel_tag("wgrad3x3_ld_kernel");
  hipLaunchKernelGGL(wgrad3x3_ld_kernel, dim3(blocks_xy * splits), dim3((kWlNW + kWlNL) * 64), lds, st, a, tiles, per);
  if (a.slab && splits > 1) {
    SlabLayout L = {};
    L.kind = SLAB_HALO; L.splits = splits; L.blocks = blocks_xy; L.nw = kWlNW; L.nf = 18; L.units = units;
    L.Cout = a.Cout; L.C = a.C; L.Krow = 9 * a.C; L.cmax = a.C;
    L.co_blocks = a.co_blocks; L.c_blocks = a.c_blocks; L.ci = 64; L.co32 = 0;
    g_pending = PendingReduce{a.slab, a.dw, L};
  }
  return hipGetLastError();
}

int wgrad_batch_tw(const ConvWgradArgs& a) {
  if (a.Q % 32 == 0 && a.P % 4 == 0) return 32;
  if (a.Q % 16 == 0 && a.P % 8 == 0) return 16;
  return 0;
}

bool wgrad_batch_ok(const ConvWgradArgs& a) {
  return a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.C % 64 == 0 && a.Cout % 64 == 0 && a.P == a.H &&
         a.Q == a.W && wgrad_batch_tw(a) != 0 && !a.dy2 && !a.bn_fuse && a.lddy % 8 == 0 &&
         a.ldx % 8 == 0 && (size_t)a.N * a.H * a.W * a.ldx * 2 < 0x80000000ull &&
         (size_t)a.N * a.P * a.Q * a.lddy * 2 < 0x80000000ull;
}

// CU count of the CURRENT device, cached per device id (the persistent grids
// are sized from it; a plan is bound to the device current at its creation)
int device_cu_count() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (!cus[dev]) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev] = c;
  }
  return cus[dev];
}

// one block per CU, at most kWbMaxGrid: the reduce collects a split unit's
// slot list in a kWbMaxGrid-entry LDS table
int wgrad_batch_grid() {
  const int c = device_cu_count();
  return c < kWbMaxGrid ? c : kWbMaxGrid;
}

// largest number of units any block of the batch touches (its slab slots)
int wgrad_batch_maxseg(const WgBatchArgs& a) {
  auto unit_of = [&](long long it) {
    int l = 0;
    while (l + 1 < a.nl && it >= a.L[l + 1].item0) ++l;
    return a.L[l].unit0 + (int)((it - a.L[l].item0) / a.L[l].tiles);
  };
  int m = 1;
  for (int b = 0; b < a.grid; ++b) {
    const long long i0 = (long long)b * a.items / a.grid, i1 = (long long)(b + 1) * a.items / a.grid;
    if (i1 > i0) m = std::max(m, unit_of(i1 - 1) - unit_of(i0) + 1);
  }
  return m;
}

template <int TW>
static void launch_wgrad_batch_tw(const WgBatchArgs& a, hipStream_t st) {
  constexpr size_t lds = (size_t)kWlNS * wb_stage<TW>();
  static_assert(lds <= 163840, "LDS");
  set_kernel_tag("wgrad3x3_batch_kernel<%d>", TW);
  hipLaunchKernelGGL(wgrad3x3_batch_kernel<TW>, dim3(a.grid), dim3((kWlNW + kWlNL) * 64), lds, st, a);
}

hipError_t launch_wgrad_batch(const WgBatchArgs& a, hipStream_t st) {
  if (a.grid <= 0 || a.grid > kWbMaxGrid) return hipErrorInvalidValue;  // slots[] of the reduce
  if (a.tw == 32) launch_wgrad_batch_tw<32>(a, st);
  else if (a.tw == 16) launch_wgrad_batch_tw<16>(a, st);
  else return hipErrorInvalidValue;
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(wgrad_batch_reduce_kernel, dim3(a.units, (unsigned)(kWbPartBytes / 16 / 256)), dim3(256), 0, st,
                     a);
  // the profiler column names the batch by its MFMA kernel (the fixed-order
  // reduce of the split units is part of the same bracketed launch pair)
  return hipGetLastError();
}

bool wgrad_pending() { return g_pending.slab != nullptr; }

// split lanes per unit (each thread's loads, <= 8, all in flight at once; up to
// 16 lanes) and the block count of the reduction of r
static void reduce_geometry(const PendingReduce& r, int& T, long long& blocks) {
  T = 1;
  while (T < 16 && (long long)T * 8 < r.L.splits) T <<= 1;
  const long long per = 256 / T;
  blocks = (r.L.units + per - 1) / per;
}

static hipError_t launch_reduce(const PendingReduce& r, hipStream_t st) {
  int T;
  long long bx;
  reduce_geometry(r, T, bx);
  set_kernel_tag("wgrad_slab_reduce_kernel");
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((unsigned)bx), dim3(256), 0, st,
                     reinterpret_cast<const f32x4*>(r.slab), r.dw, r.L, T);
  return hipGetLastError();
}

hipError_t launch_wgrad_finish(hipStream_t st) {
  if (!g_pending.slab) return hipSuccess;
  const PendingReduce r = g_pending;
  g_pending = PendingReduce{};
  return launch_reduce(r, st);
}

static thread_local PendingReduce g_deferred{};

bool wgrad_defer() {
  if (!g_pending.slab || g_deferred.slab) return false;
  g_deferred = g_pending;
  g_pending = PendingReduce{};
  return true;
}
bool wgrad_deferred() { return g_deferred.slab != nullptr; }
bool wgrad_deferred_reads(const void* slab) { return g_deferred.slab && g_deferred.slab == slab; }

bool wgrad_take_deferred(ReduceTail* t) {
  if (!g_deferred.slab) return false;
  long long bx;
  reduce_geometry(g_deferred, t->T, bx);
  t->slab = g_deferred.slab;
  t->dw = g_deferred.dw;
  t->L = g_deferred.L;
  t->blocks = (int)bx;
  g_deferred = PendingReduce{};
  return true;
}

hipError_t launch_slab_reduce(const ReduceTail& r, hipStream_t st) {
  set_kernel_tag("wgrad_slab_reduce_kernel");
  hipLaunchKernelGGL(wgrad_slab_reduce_kernel, dim3((unsigned)r.blocks), dim3(256), 0, st,
                     reinterpret_cast<const f32x4*>(r.slab), r.dw, r.L, r.T);
  return hipGetLastError();
}

// drop any split-K reduction left queued by an earlier backward that ended
// on an error (its slab / dW pointers belong to that plan's workspace)
void wgrad_reset() {
  g_pending = PendingReduce{};
  g_deferred = PendingReduce{};
}

hipError_t launch_wgrad_flush(hipStream_t st) {
  if (!g_deferred.slab) return hipSuccess;
  const PendingReduce r = g_deferred;
  g_deferred = PendingReduce{};
  return launch_reduce(r, st);
}

hipError_t launch_convt_wgrad(const ConvWgradArgs& a0, hipStream_t st) {
  ConvWgradArgs a = a0;
  if (a.C % 32 || (a.C / 4) % 8 || a.Cout % 32 || a.H != 2 * a.P || a.W != 2 * a.Q) return hipErrorInvalidValue;
  a.R = a.S = 1; a.stride = 1; a.pad = 0;
  if (a.Cout >= 128 && a.C >= 128) return launch_wgrad_cfg<XLOAD_SHUF, 128, 128, 32, 2, 2>(a, st);
  if (a.Cout % 64 == 0 && a.C % 64 == 0) return launch_wgrad_cfg<XLOAD_SHUF, 64, 64, 64, 2, 2>(a, st);
  return launch_wgrad_cfg<XLOAD_SHUF, 32, 32, 64, 2, 2>(a, st);
}

// UNET_NO_S2WG=1: stride-2 weight gradients on the implicit GEMM (A/B)
bool wgrad_s2_fold_ok(const ConvWgradArgs& a) {
  static const bool s2wg = std::getenv("UNET_NO_S2WG") == nullptr;
  return s2wg && a.R == 3 && a.S == 3 && a.stride == 2 && a.pad == 1 && a.C % 32 == 0 &&
         a.Cout % 64 == 0 && a.H == 2 * a.P && a.W == 2 * a.Q && a.Q % 16 == 0 && a.P % 8 == 0 &&
         (!a.dy2 || a.lddy2 % 8 == 0) && a.lddy % 8 == 0 && a.ldx % 8 == 0 &&
         (size_t)a.N * a.H * a.W * a.ldx * 2 < 0x80000000ull &&
         (size_t)a.N * a.P * a.Q * (a.lddy > a.lddy2 ? a.lddy : a.lddy2) * 2 < 0x80000000ull;
}

hipError_t launch_conv_wgrad(const ConvWgradArgs& a0, int stem, hipStream_t st) {
  const ConvWgradArgs& a = a0;
  if (stem)
    return a.Cout % 64 == 0 ? launch_stem_wgrad(a, st) : launch_wgrad_cfg<XLOAD_STEM, 64, 64, 64, 2, 2>(a, st);
  if (a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.C % 32 == 0 && a.P == a.H &&
      a.Q == a.W && (size_t)a.N * a.H * a.W * a.ldx * 2 < 0x80000000ull &&
      (size_t)a.N * a.P * a.Q * a.lddy * 2 < 0x80000000ull) {
    if (a.C % 64 == 0) {
      // loader-wave kernel where blocks share their tiles (C or Cout >= 128:
      // enc2-3, decoder2-4 first convs), the all-waves-issue kernel for the
      // 64 x 64-channel layers (enc1, decoder2.3), where the loader form
      // measured slower (profiles/r04/s1)
      if ((a.C >= 128 || a.Cout >= 128) && a.Cout % 64 == 0 && a.Q % 32 == 0 && a.P % 4 == 0)
        return launch_wgrad_ld(a, st);
      if (a.Q % 32 == 0 && a.P % 4 == 0) return launch_wgrad_halo<32, 64>(a, st);
      if (a.Q % 16 == 0 && a.P % 8 == 0) return launch_wgrad_halo<16, 64>(a, st);
    }
    if (a.Cout == 32 && a.Q % 32 == 0 && a.P % 4 == 0) return launch_wgrad_halo<32, 32, true>(a, st);
    if (a.Q % 32 == 0 && a.P % 4 == 0) return launch_wgrad_halo<32, 32>(a, st);
    if (a.Q % 16 == 0 && a.P % 8 == 0) return launch_wgrad_halo<16, 32>(a, st);
  }
  // 3x3 / stride 2 / pad 1 (encoder stages 2-4, first conv): the halo kernel
  // with a (2TH+1) x (2TW+1) input halo, the downsample folded in when a.dy2
  if (wgrad_s2_fold_ok(a)) {
    if (a.dy2) return launch_wgrad_halo<16, 32, false, 2, 2, true>(a, st);
    return launch_wgrad_halo<16, 32, false, 3, 2>(a, st);
  }
  if (a.dy2) return hipErrorInvalidValue;
  if (a.C % 32 || a.Cout % 32) return hipErrorInvalidValue;
  const bool co64 = a.Cout % 64 == 0, c64 = a.C % 64 == 0;
  if (a.Cout >= 128 && a.C >= 128)
    return launch_wgrad_cfg<XLOAD_NHWC, 128, 128, 32, 2, 2>(a, st);
  if (co64 && c64) return launch_wgrad_cfg<XLOAD_NHWC, 64, 64, 64, 2, 2>(a, st);
  if (co64) return launch_wgrad_cfg<XLOAD_NHWC, 64, 32, 64, 4, 1>(a, st);
  if (c64) return launch_wgrad_cfg<XLOAD_NHWC, 32, 64, 64, 1, 4>(a, st);
  return launch_wgrad_cfg<XLOAD_NHWC, 32, 32, 64, 2, 2>(a, st);
}

}  // namespace unet

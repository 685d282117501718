// The stem (input_conv 7x7/s2/p3 1 -> C0, bn1, ReLU, MaxPool2d(3,2,1);
// advanced_models.py:76-83 via the resnet34 stem) by RECOMPUTE: the raw conv
// output y (N x H/2 x W/2 x C0 bf16, 134 MB at 16 x 512^2) is never stored.
// Its input is a 1-channel fp32 image (16 MB) and the conv is 49 MACs per
// output value, so recomputing it wherever y is needed costs a few MFMAs per
// pixel against ~0.3 GB of HBM traffic saved per step.
//
//   stats pass   conv -> BN batch sums (fp64 replica atomics, last block
//                finalises scale/shift/save/running stats as stem_fwd did)
//   apply pass   conv -> fp32 y -> relu(y * scale + shift) = act (the
//                decoder1 skip, stored once) -> MaxPool(3,2,1) of act in LDS
//                -> pooled + argmax index.  A block walks pooled rows, keeping
//                the last three act rows in an LDS ring; its first pooled row
//                recomputes the act row above it (owned by the previous block).
//   backward     conv -> fp32 y -> ReLU mask bit and xhat; dZ = [act > 0]
//                (maxpool scatter of dpool + the skip gradient) --
//                maxpool_bwd's expression -- and, in the same pass, the stem
//                weight gradient through
//                the BN-backward identity
//                  dY = k1 dZ - k1 m1 - k1 m2 xhat       (k1 = gamma invstd,
//                  m1 = mean dZ, m2 = mean dZ xhat), so
//                  dW[co][k] = k1 (sum dZ im - m1 sum im - m2 sum xhat im)
//                with im centred by a per-block column mean (sum dY = 0 makes
//                dW independent of it; it keeps the m1 term from cancelling)
//                three GEMMs over the pixels whose coefficients are only known
//                at the end: each block leaves its partial sums (dZ^T im,
//                xhat^T im, sum im, sum dZ, sum dZ xhat), a fixed-order reduce
//                sums them and a finalise forms dW, dgamma, dbeta.
// Nothing here depends on timing: every sum has a fixed order (bit-
// reproducible backward).
//
// im2col K layout (as the packed stem weights [Cout][64]): k = kr * 8 + ks,
// kr, ks < 7 the 7x7 taps, the rest zero.  MFMA 16x16x32 bf16, A = weights
// (rows = channels), B = im2col (cols = pixels): lane holds 4 consecutive
// channels of one pixel.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace unet {

void conv_kernel_tag(const char* tag);  // conv_kernels.hip (profiler column)

namespace {

// [pixel][64 bf16] tile with 16-B chunks XOR-swizzled by (pixel & 7)
__device__ __forceinline__ int ring_off(int px, int co) {
  return px * 128 + ((((co >> 3) ^ px) & 7) << 4) + ((co & 7) << 1);
}

// [pixel][64] tile read through ds_read_b64_tr_b16 (conv_kernels.hip tr_off<64>)
__device__ __forceinline__ int tt_off(int row, int col) {
  const int unit = col >> 4;
  const int f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return row * 128 + ((unit ^ f) << 5) + ((col & 15) << 1);
}

__device__ __forceinline__ bf16x8 tr8(const char* lo, const char* hi) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lo));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, hi));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// Input patch: rows ih0 .. ih0 + nrows - 1 of image n, columns iw0 .. iw0 +
// COLS - 1 (zero outside the image), COLS = 2 * NPX + 6 for NPX output pixels;
// fetched into registers (PT per thread, NT threads), stored as bf16 rows of
// pitch PITCH (4-B aligned: the im2col reads 4 dwords from column 2 px).
template <int NPX, int NT, int PT>
struct Patch {
  static constexpr int COLS = 2 * NPX + 6;
  static constexpr int PITCH = 2 * NPX + 8;
  float v[PT];
  // raw buffer loads with 32-bit offsets: exactly PT loads per thread whatever
  // the borders (an element outside the image or past nrows reads the kOOB
  // zero), so a caller can count them in vmcnt
  __device__ __forceinline__ void fetch_counted(__amdgpu_buffer_rsrc_t r, int H, int W, int n, int ih0, int nrows,
                                                int iw0) {
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = threadIdx.x + j * NT;
      const int rr = i / COLS, c = i - rr * COLS;
      const int ih = ih0 + rr, iw = iw0 + c;
      const bool ok = rr < nrows && ih >= 0 && ih < H && iw >= 0 && iw < W;
      // 32-bit: the launchers check N * H * W * 4 < 2^31
      const unsigned off = ok ? (unsigned)(((n * H + ih) * W + iw) * 4) : kOOB;
      v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
    }
  }
  __device__ __forceinline__ void store(bf16_t* patch, int nrows) const {
#pragma unroll
    for (int j = 0; j < PT; ++j) {
      const int i = threadIdx.x + j * NT;
      const int r = i / COLS, c = i - r * COLS;
      if (r < nrows) patch[r * PITCH + c] = f2bf(v[j]);
    }
  }
};

// im2col chunk kr (8 taps ks = 0..7 of patch row prow0 + kr, 8th masked) of
// output pixel px: 4 dwords from column 2 px
template <int PITCH>
__device__ __forceinline__ uint4 im2col_chunk(const bf16_t* patch, int prow0, int px, int kr) {
  if (kr >= 7) return make_uint4(0, 0, 0, 0);
  const unsigned* w = reinterpret_cast<const unsigned*>(patch + (prow0 + kr) * PITCH + 2 * px);
  return make_uint4(w[0], w[1], w[2], w[3] & 0xffffu);
}

// packed weights of channel group cg as MFMA A fragments: wf[kk][i] = W[cg +
// i*16 + (lane&15)][(kk*4 + (lane>>4)) * 8 ..]
__device__ __forceinline__ void load_wfrag(const bf16_t* w, int cg, bf16x8 (&wf)[2][4]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      wf[kk][i] = *reinterpret_cast<const bf16x8*>(w + (size_t)(cg + i * 16 + (lane & 15)) * 64 +
                                                   (kk * 4 + (lane >> 4)) * 8);
}

// one wave's 32 output pixels (x0 .. x0+31 of the Xs tile) x 64 channels:
// the MFMA sequence of stem_fwd_kernel (same K split), so y is bit-identical
__device__ __forceinline__ void conv32(const char* Xs, int x0, const bf16x8 (&wf)[2][4], f32x4 (&acc)[4][2]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = kk * 4 + (lane >> 4);
    bf16x8 xf[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) xf[j] = *reinterpret_cast<const bf16x8*>(Xs + tt_off(x0 + j * 16 + (lane & 15), ch * 8));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kk][i], xf[j], acc[i][j], 0, 0, 0);
  }
}

// workgroup barrier ordering LDS only (conv_halo.hip lds_barrier): the
// global loads prefetched into registers and the HBM stores stay in flight
// (__syncthreads' fence would wait for every one of them)
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// act = bf16(relu(y * sc + sh)) of the fp32 conv output y (round 6: the
// stored-y0 path, bn_relu_maxpool_fwd, necessarily normalises a bf16 y; the
// recompute passes hold y in fp32 and normalise it as the reference's fp32
// BatchNorm does, advanced_models.py:81-83)
__device__ __forceinline__ float stem_act(float y, float sc, float sh) {
  const float z = y * sc + sh;
  return bf2f(f2bf(z > 0.f ? z : 0.f));
}

}  // namespace

// ---------------------------------------------------------------------------
// forward: MODE 0 = BN statistics (and, for tests, the raw y), MODE 1 = act +
// pool.  512 threads (8 waves x 32 pixels = one 256-pixel output row per conv
// round).  A block owns pooled rows [j0, j1) of the flattened N x Pp grid (one
// pooled row = stem rows 2jp, 2jp+1), channel group blockIdx.y.
// ---------------------------------------------------------------------------
constexpr int kRcNT = 512;
constexpr int kRcNPX = 256;
typedef Patch<kRcNPX, kRcNT, 12> FwdPatch;  // up to 11 input rows x 518 columns
constexpr int kRcRing = 3 * kRcNPX * 128;
constexpr int kRcXs = kRcNPX * 128;
constexpr int kRcPatchB = 11 * FwdPatch::PITCH * 2;

template <int MODE>
__global__ void __launch_bounds__(kRcNT) stem_rc_fwd_kernel(StemRcArgs a, int per) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  char* ring = smem;                                            // MODE 1: act rows r % 3
  char* Xs = smem + (MODE == 1 ? kRcRing : 0);                  // im2col of one output row
  bf16_t* patch = reinterpret_cast<bf16_t*>(Xs + kRcXs);
  float* coef = reinterpret_cast<float*>(Xs + kRcXs + kRcPatchB);  // [2][64] scale | shift
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int cg = blockIdx.y * 64;
  const int total = a.N * a.Pp;
  const int j0 = xcd_remap(blockIdx.x, gridDim.x) * per;
  const int j1 = min(total, j0 + per);
  bf16x8 wf[2][4];
  load_wfrag(a.w, cg, wf);
  if (MODE == 1 && tid < 64) {
    const int c = cg + tid;
    if (a.bn.training && a.bn.ss) {
      coef[tid] = a.bn.ss[c];
      coef[64 + tid] = a.bn.ss[a.Cout + c];
    } else {  // from the batch sums (or running statistics): every block alike
      float m, inv, var;
      bn_scale_shift(a.bn, c, coef[tid], coef[64 + tid], m, inv, var);
      if (blockIdx.x == 0 && a.bn.training) {  // block 0 of the group: saved / running statistics
        a.bn.save_mean[c] = m;
        a.bn.save_invstd[c] = inv;
        const double cnt = a.bn.count;
        const float unb = (float)((double)var * (cnt / (cnt > 1.0 ? cnt - 1.0 : 1.0)));
        a.bn.run_mean[c] = (1.f - a.bn.momentum) * a.bn.run_mean[c] + a.bn.momentum * m;
        a.bn.run_var[c] = (1.f - a.bn.momentum) * a.bn.run_var[c] + a.bn.momentum * unb;
        if (c == 0 && a.bn.nbt) *a.bn.nbt += 1;
      }
    }
  }
  float q0[4][4], q1[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = 0.f;

  // pooled row j: stem rows 2jp - extra .. 2jp + 1, input rows from 4jp - 3 - 2 extra
  auto extra_of = [&](int j) { return (MODE == 1 && j == j0 && (j % a.Pp) > 0) ? 1 : 0; };
  FwdPatch pf;
  // 32-bit buffer offsets, kOOB zero-fill at the borders (no 64-bit address
  // arithmetic or branch per element)
  const __amdgpu_buffer_rsrc_t rimg = make_rsrc(a.img, (unsigned)((size_t)a.N * a.H * a.W * 4));
  auto fetch = [&](FwdPatch& p, int j) {
    const int n = j / a.Pp, jp = j - n * a.Pp, ex = extra_of(j);
    p.fetch_counted(rimg, a.H, a.W, n, 4 * jp - 3 - 2 * ex, 9 + 2 * ex, -3);
  };
  // pooled row j from patch p, which is then refilled with row j + AHEAD
  auto row = [&](int j, FwdPatch& p, int ahead) {
    const int n = j / a.Pp, jp = j - n * a.Pp, ex = extra_of(j);
    lds_sync();  // previous pooled row: patch, Xs and ring slots consumed
    p.store(patch, 9 + 2 * ex);
    if (j + ahead < j1) fetch(p, j + ahead);
    for (int t = -ex; t < 2; ++t) {
      const int h = 2 * jp + t;  // stem row
      lds_sync();           // patch stored / previous round's Xs consumed
      {  // im2col of row h: thread -> (pixel, half of the 8 chunks)
        const int px = tid & (kRcNPX - 1), half = tid >> 8;
        const int prow0 = 2 * (t + ex);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int kr = half * 4 + c;
          const uint4 v = px < a.Q ? im2col_chunk<FwdPatch::PITCH>(patch, prow0, px, kr) : make_uint4(0, 0, 0, 0);
          *reinterpret_cast<uint4*>(Xs + tt_off(px, kr * 8)) = v;
        }
      }
      lds_sync();
      f32x4 acc[4][2];
      conv32(Xs, wave * 32, wf, acc);
      const size_t rowpix = ((size_t)n * a.P + h) * a.Q;
#pragma unroll
      for (int j2 = 0; j2 < 2; ++j2) {
        const int px = wave * 32 + j2 * 16 + li;
        if (px >= a.Q) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = i * 16 + 4 * g;
          if constexpr (MODE == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { q0[i][e] += acc[i][j2][e]; q1[i][e] += acc[i][j2][e] * acc[i][j2][e]; }
            if (a.y) {
              uint2 o;
              o.x = pack_bf2(acc[i][j2][0], acc[i][j2][1]);
              o.y = pack_bf2(acc[i][j2][2], acc[i][j2][3]);
              *reinterpret_cast<uint2*>(a.y + (rowpix + px) * a.ldy + cg + co) = o;
            }
          } else {
            float v[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = stem_act(acc[i][j2][e], coef[co + e], coef[64 + co + e]);
            uint2 o;
            o.x = pack_bf2(v[0], v[1]);
            o.y = pack_bf2(v[2], v[3]);
            *reinterpret_cast<uint2*>(ring + (h % 3) * (kRcNPX * 128) + ring_off(px, co)) = o;
          }
        }
      }
    }
    if (j - j0 < 8) TSTAMP(a.tim, 2 + 2 * (j - j0));
    if constexpr (MODE == 1) {
      lds_sync();  // act rows 2jp-1 .. 2jp+1 in the ring
      // act rows 2jp, 2jp+1 to HBM (whole 128-B pixel lines)
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int h = 2 * jp + t;
        const size_t rowpix = ((size_t)n * a.P + h) * a.Q;
#pragma unroll
        for (int it = 0; it < kRcNPX * 8 / kRcNT; ++it) {
          const int i = tid + it * kRcNT, px = i >> 3, ch = i & 7;
          if (px < a.Q)
            *reinterpret_cast<uint4*>(a.act + (rowpix + px) * a.ldact + cg + ch * 8) =
                *reinterpret_cast<const uint4*>(ring + (h % 3) * (kRcNPX * 128) + ring_off(px, ch * 8));
        }
      }
      // MaxPool2d(3, 2, 1) of pooled row jp: first maximum in (kh, kw) scan
      // order wins (strict >).  act = bf16(relu(.)) is never NaN and never
      // negative (stem_act maps NaN to 0), so its bf16 bits order like its
      // values and one unsigned max over key = bits << 4 | (15 - tap) finds
      // the maximum and, among equal maxima, the first tap
#pragma unroll
      for (int it = 0; it < (kRcNPX / 2) * 8 / kRcNT; ++it) {
        const int i = tid + it * kRcNT, q = i >> 3, ch = i & 7;
        if (q >= a.Qp) continue;
        unsigned key[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) key[k] = 0u;  // the (1, 1) tap is always inside
#pragma unroll
        for (int t9 = 0; t9 < 9; ++t9) {
          const int kh = t9 / 3, kw = t9 % 3;
          const int h = 2 * jp - 1 + kh, w = 2 * q - 1 + kw;
          if (h < 0) continue;  // uniform (first pooled row)
          const bool inw = w >= 0 && w < a.Q;
          const uint4 r = *reinterpret_cast<const uint4*>(ring + (h % 3) * (kRcNPX * 128) + ring_off(inw ? w : 0, ch * 8));
          const unsigned wd[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const unsigned bits = (k & 1) ? (wd[k >> 1] >> 16) : (wd[k >> 1] & 0xffffu);
            const unsigned cand = inw ? ((bits << 4) | (unsigned)(15 - t9)) : 0u;
            key[k] = max(key[k], cand);
          }
        }
        uint4 best;
        best.x = (key[0] >> 4) | ((key[1] >> 4) << 16);
        best.y = (key[2] >> 4) | ((key[3] >> 4) << 16);
        best.z = (key[4] >> 4) | ((key[5] >> 4) << 16);
        best.w = (key[6] >> 4) | ((key[7] >> 4) << 16);
        int bi[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) bi[k] = 15 - (int)(key[k] & 15u);
        const size_t opix = ((size_t)n * a.Pp + jp) * a.Qp + q;
        *reinterpret_cast<uint4*>(a.pool + opix * a.ldpool + cg + ch * 8) = best;
        uint2 ix;
        ix.x = (unsigned)bi[0] | ((unsigned)bi[1] << 8) | ((unsigned)bi[2] << 16) | ((unsigned)bi[3] << 24);
        ix.y = (unsigned)bi[4] | ((unsigned)bi[5] << 8) | ((unsigned)bi[6] << 16) | ((unsigned)bi[7] << 24);
        *reinterpret_cast<uint2*>(a.idx + opix * a.Cout + cg + ch * 8) = ix;
      }
    }
    if (j - j0 < 8) TSTAMP(a.tim, 3 + 2 * (j - j0));
  };
  if constexpr (MODE == 0) {
    // statistics pass: no stores in the loop, so two rows' patches in flight
    // (the fetch of row j lands under rows j - 2 and j - 1; with one row ahead
    // every row waited ~8 k cycles for its patch, conv_timing.py)
    FwdPatch pf2;
    if (j0 < j1) fetch(pf, j0);
    if (j0 + 1 < j1) fetch(pf2, j0 + 1);
    TSTAMP(a.tim, 1);
    for (int j = j0; j < j1; j += 2) {
      row(j, pf, 2);
      if (j + 1 < j1) row(j + 1, pf2, 2);
    }
  } else {
    if (j0 < j1) fetch(pf, j0);
    TSTAMP(a.tim, 1);
    for (int j = j0; j < j1; ++j) row(j, pf, 1);
  }
  TSTAMP(a.tim, 20);
  if constexpr (MODE == 0) {
    // fold over the 16 pixel lanes, then the 8 waves, then one replica atomic per channel
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          q0[i][e] += __shfl_xor(q0[i][e], o, 64);
          q1[i][e] += __shfl_xor(q1[i][e], o, 64);
        }
    lds_sync();
    float* red = reinterpret_cast<float*>(smem);  // [8 waves][64][2]
    if (li == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = i * 16 + 4 * g + e;
          red[(wave * 64 + c) * 2] = q0[i][e];
          red[(wave * 64 + c) * 2 + 1] = q1[i][e];
        }
    }
    lds_sync();
    if (tid < 64) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int w = 0; w < kRcNT / 64; ++w) { s0 += red[(w * 64 + tid) * 2]; s1 += red[(w * 64 + tid) * 2 + 1]; }
      double* rep = a.stats + (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout + cg;
      atomicAdd(rep + tid, (double)s0);
      atomicAdd(rep + a.Cout + tid, (double)s1);
    }
    if (a.bn.ticket) {
      int* flag = reinterpret_cast<int*>(smem + (kRcNT / 64) * 64 * 2 * sizeof(float));
      if (last_block_arrive(a.bn.ticket, gridDim.x * gridDim.y, flag, tid < 64)) bn_finalize(a.bn);
    }
  }
  TSTAMP(a.tim, 21);
  TSTAMP_RT(a.tim, 31);
}

// Block sums of the input image in a fixed order (the backward's im2col
// centring value): block b sums elements b, b + G, b + 2G, ... per thread in
// order, then a fixed tree.
constexpr int kRcImBlocks = 256;
constexpr int kRcImNT = 1024;
__global__ void __launch_bounds__(kRcImNT) stem_rc_imsum_kernel(StemRcArgs a) {
  // 1024 threads x float4 x 4 in flight per block (the one-load-at-a-time
  // scalar loop took 27 us for 16.8 MB); fixed order: per thread, then a tree
  __shared__ float red[kRcImNT];
  const size_t n = (size_t)a.N * a.H * a.W;  // a multiple of 4 (W even, H even)
  const size_t n4 = n >> 2;
  const float4* img4 = reinterpret_cast<const float4*>(a.img);
  const size_t stride = (size_t)kRcImBlocks * kRcImNT;
  float s = 0.f;
  if ((reinterpret_cast<uintptr_t>(a.img) & 15) == 0) {
    for (size_t i = (size_t)blockIdx.x * kRcImNT + threadIdx.x; i < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = i + k * stride < n4 ? img4[i + k * stride] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 4; ++k) s += (v[k].x + v[k].y) + (v[k].z + v[k].w);
    }
  } else {  // a misaligned image view: scalar loads
    for (size_t i = (size_t)blockIdx.x * kRcImNT + threadIdx.x; i < n; i += stride) s += a.img[i];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = kRcImNT / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.imsum[blockIdx.x] = red[0];
}

// ---------------------------------------------------------------------------
// backward.  256 threads, 2 blocks per CU; a unit is one half row (128
// pixels) of the stem output; a block owns units [u0, u1) of channel group
// blockIdx.y.  Per unit: the input patch (prefetched by counted buffer loads
// while the previous unit ran) is stored to LDS and expanded to im2col; the
// skip gradient is loaded into registers; the conv is recomputed; the dZ phase
// gathers the maxpool backward from the pooled rows (LDS-DMA issued one unit
// ahead, after the previous unit's dZ phase), adds the skip gradient, applies
// the ReLU mask and forms the BN-backward sums, xhat and the centred im2col;
// then the two weight-gradient GEMMs.
// LDS: patch (7 x 264 bf16) | Xs im2col [128][64] | Ys y/xhat [128][64] |
//      Ds dZ [128][64] | coefficients [5][64] f32 | Pd dpool [2 slots][65][64] | Pi idx [2 slots][65][64] u8
// Units run down the rows of one 128-column segment (u = s * N * P + n * P + h),
// so consecutive units share pooled rows: pooled row p lives in slot p & 1 and
// a unit loads only the rows the previous one did not have (one row every
// other unit).
// Waves: w>>1 = GEMM (0: dZ^T im, 1: xhat^T im), w&1 = 32-channel half; each
// wave also sums im over pixels for k in [16w, 16w+16) (MFMA against ones).
// ---------------------------------------------------------------------------
constexpr int kRbNT = 256;
constexpr int kRbNPX = 128;
constexpr int kRbPT = 8;
typedef Patch<kRbNPX, kRbNT, kRbPT> BwdPatch;  // 7 x 262
constexpr int kRbTile = kRbNPX * 128;
constexpr int kRbPatchB = 7 * BwdPatch::PITCH * 2;
constexpr int kRbPQ = kRbNPX / 2 + 1;                 // pooled columns a unit's pixels reach
// LDS-DMA of one pooled row, one 16-B piece per lane: dpool [qi][8 pieces],
// idx [qi][4 pieces]; the last wave instruction of a row is moved back so that
// it ends at the row end (rewriting some pieces with the same data) instead of
// spilling into the other slot
constexpr int kRbPdRow = kRbPQ * 8, kRbPiRow = kRbPQ * 4;  // 16-B pieces per row
constexpr int kRbPdIns = (kRbPdRow + 63) / 64, kRbPiIns = (kRbPiRow + 63) / 64;
constexpr int kRbPd = 2 * kRbPdRow * 16, kRbPi = 2 * kRbPiRow * 16;
constexpr int kRbLds = kRbPatchB + 3 * kRbTile + 5 * 64 * 4 + kRbPd + kRbPi;
static_assert(kRbPatchB >= kRbNPX * 8, "the ReLU mask bits ([128 px][64 bits]) reuse the patch area");
// per-block partial: [4 waves][9 tiles][64 lanes] f32x4 | [2][64] sum dZ, sum dZ xhat
constexpr int kRbPartF4 = 4 * 9 * 64 + 32;

__global__ void __launch_bounds__(kRbNT, 2) stem_rc_bwd_kernel(StemRcArgs a, int per) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* patch = reinterpret_cast<bf16_t*>(smem);
  char* Xs = smem + kRbPatchB;
  char* Ys = Xs + kRbTile;
  char* Ds = Ys + kRbTile;
  // [5][64] scale, shift, mean, invstd | mu: the block's im2col column means
  float* cf = reinterpret_cast<float*>(Ds + kRbTile);
  char* Pd = reinterpret_cast<char*>(cf + 5 * 64);
  char* Pi = Pd + kRbPd;
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15, trq = li >> 2, trp = li & 3;
  const int cg = blockIdx.y * 64;
  const int segs = (a.Q + kRbNPX - 1) / kRbNPX;
  const int total = a.N * a.P * segs;
  const int u0 = xcd_remap(blockIdx.x, gridDim.x) * per;
  const int u1 = min(total, u0 + per);
  const int c8 = (tid & 7) * 8;  // this thread's 8 channels in the dZ phase (every item)
  {
    // image mean: the block sums of stem_rc_imsum_kernel added by a fixed fp64
    // tree (the same value in every block), in the Ds region before first use
    static_assert(kRcImBlocks == kRbNT, "one image-sum partial per thread");
    double* red = reinterpret_cast<double*>(Ds);
    red[tid] = (double)a.imsum[tid];
#pragma unroll
    for (int st = kRbNT / 2; st > 0; st >>= 1) {
      lds_sync();
      if (tid < st) red[tid] += red[tid + st];
    }
    lds_sync();
  }
  if (tid < 64) {
    if (a.bn.ss) {
      cf[tid] = a.bn.ss[cg + tid];
      cf[64 + tid] = a.bn.ss[a.Cout + cg + tid];
    } else {  // the forward's scale / shift, recomputed from the same batch sums
      float m, inv, var;
      bn_scale_shift(a.bn, cg + tid, cf[tid], cf[64 + tid], m, inv, var);
    }
    cf[128 + tid] = a.mean[cg + tid];
    cf[192 + tid] = a.invstd[cg + tid];
    // mu[k]: the image mean for the 49 real taps, 0 for the padding.  The
    // weight-gradient GEMMs run on im - mu: sum_px dY = 0 makes dW independent
    // of mu, and centring removes the common mode that m1 * sum(im) would
    // otherwise cancel against dZ^T im (fp32 accumulation).
    const double sum = reinterpret_cast<const double*>(Ds)[0];
    const float mu = bf2f(f2bf((float)(sum / ((double)a.N * a.H * a.W))));
    cf[256 + tid] = ((tid & 7) < 7 && (tid >> 3) < 7) ? mu : 0.f;
  }
  float s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
  f32x4 gacc[2][4], bacc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) gacc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bacc = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int k = 0; k < 8; ++k) ones[k] = (__bf16)1.0f;

  BwdPatch pf;
  const __amdgpu_buffer_rsrc_t rimg = make_rsrc(a.img, (unsigned)((size_t)a.N * a.H * a.W * 4));
  const int rows_total = a.N * a.P;
  auto decode = [&](int u, int& s, int& n, int& h) {
    s = u / rows_total;
    const int row = u - s * rows_total;
    n = row / a.P;
    h = row - n * a.P;
  };
  auto fetch = [&](int u) {
    int s, n, h;
    decode(u, s, n, h);
    pf.fetch_counted(rimg, a.H, a.W, n, 2 * h - 3, 7, 2 * s * kRbNPX - 3);
  };
  // the pooled rows of unit u straight into LDS (DMA, no registers): issued
  // one unit ahead, right after the previous unit's dZ phase (the last reader
  // of Pd / Pi), waited for at this unit's dZ phase.  Rows the previous unit
  // of this block already loaded (same segment, previous stem row) stay.
  auto pool_dma = [&](int u, bool first) {
    int s, n, h;
    decode(u, s, n, h);
    const int q0 = s * kRbNPX, Qs = min(kRbNPX, a.Q - q0);
    const int p_lo = h >= 1 ? h / 2 : 0;
    const int p_hi = min((h + 1) / 2, a.Pp - 1);
    const int qlo = q0 / 2, qhi = min((q0 + Qs) / 2, a.Qp - 1);
    const int nq = qhi - qlo + 1;
    int have = -1;  // highest pooled row already resident
    if (!first) {
      int sp, np, hp;
      decode(u - 1, sp, np, hp);
      if (sp == s && np == n && hp + 1 == h) have = min(h / 2, a.Pp - 1);  // p_hi of row h - 1
    }
    const i32x4 rd = make_rsrc_sgpr(a.dpool, (unsigned)((size_t)a.N * a.Pp * a.Qp * a.lddpool * 2));
    const i32x4 ri = make_rsrc_sgpr(a.idx, (unsigned)((size_t)a.N * a.Pp * a.Qp * a.Cout));
    for (int p = p_lo; p <= p_hi; ++p) {
      if (p <= have) continue;  // uniform
      const size_t rowbase = ((size_t)n * a.Pp + p) * a.Qp + qlo;
      char* pd = Pd + (p & 1) * (kRbPdRow * 16);
      char* pi = Pi + (p & 1) * (kRbPiRow * 16);
      for (int ins = wave; ins < kRbPdIns; ins += kRbNT / 64) {
        const int e0 = min(ins * 64, kRbPdRow - 64), e = e0 + lane, qi = e >> 3, pc = e & 7;
        const unsigned off = qi < nq ? (unsigned)(((rowbase + qi) * a.lddpool + cg + pc * 8) * 2) : kOOB;
        glds16_asm(rd, pd + e0 * 16, off, 0);
      }
      for (int ins = wave; ins < kRbPiIns; ins += kRbNT / 64) {
        const int e0 = min(ins * 64, kRbPiRow - 64), e = e0 + lane, qi = e >> 2, pc = e & 3;
        const unsigned off = qi < nq ? (unsigned)((rowbase + qi) * a.Cout + cg + pc * 16) : kOOB;
        glds16_asm(ri, pi + e0 * 16, off, 0);
      }
    }
  };
  if (u0 < u1) {
    fetch(u0);
    pool_dma(u0, true);
  }
  TSTAMP(a.tim, 1);
  int kt = 0;
  for (int u = u0; u < u1; ++u, ++kt) {
    int s, n, h;
    decode(u, s, n, h);
    const int q0 = s * kRbNPX, Qs = min(kRbNPX, a.Q - q0);
    const size_t rowpix = ((size_t)n * a.P + h) * a.Q;
    // pooled rows p_lo .. p_hi, columns from qlo reach this unit's pixels
    const int p_lo = h >= 1 ? h / 2 : 0;
    const int p_hi = min((h + 1) / 2, a.Pp - 1);
    const int qlo = q0 / 2;
    lds_sync();  // previous unit's GEMM reads done
    if (kt < 2) TSTAMP(a.tim, 2 + 9 * kt);
    pf.store(patch, 7);  // fetched earlier
    if (kt < 2) TSTAMP(a.tim, 3 + 9 * kt);
    // conv weights (L1/L2-resident 8 KiB) re-read per unit, issued before the
    // skip-gradient loads so that the conv's wait for them leaves those in flight
    bf16x8 wf[2][4];
    load_wfrag(a.w, cg, wf);
    // the skip gradient of this thread's dZ items (plain loads, consumed in the
    // dZ phase; the tdv mapping below)
    uint4 addv[kRbNPX * 8 / kRbNT];
    {
      const __amdgpu_buffer_rsrc_t radd = make_rsrc(a.add, (unsigned)((size_t)a.N * a.P * a.Q * a.ldadd * 2));
      int tdl = tid;
      asm volatile("" : "+v"(tdl));
#pragma unroll
      for (int it = 0; it < kRbNPX * 8 / kRbNT; ++it) {
        const int px = 2 * (tdl >> 3) + (it & 1) + (it >> 1) * (kRbNT / 4);
        // raw buffer load (kOOB zero past the row end): always issued, so the
        // compiler's vmcnt bookkeeping stays exact
        const unsigned off = px < Qs ? (unsigned)(((rowpix + q0 + px) * a.ldadd + cg + (tdl & 7) * 8) * 2) : kOOB;
        addv[it] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(radd, (int)off, 0, 0));
      }
    }
    if (kt < 2) TSTAMP(a.tim, 5 + 9 * kt);
    lds_sync();
    {
      const int px = tid & (kRbNPX - 1), half = tid >> 7;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int kr = half * 4 + c;
        const uint4 v = px < Qs ? im2col_chunk<BwdPatch::PITCH>(patch, 0, px, kr) : make_uint4(0, 0, 0, 0);
        *reinterpret_cast<uint4*>(Xs + tt_off(px, kr * 8)) = v;
      }
    }
    lds_sync();
    if (kt < 2) TSTAMP(a.tim, 6 + 9 * kt);
    {  // recompute y in fp32 -> xhat = (y - mean) invstd (bf16: the third GEMM's
      // operand) -> Ys, and the forward's ReLU mask [y sc + sh > 0] of the same
      // fp32 y -> one bit per (pixel, channel) in the patch area (free until the
      // next unit's patch store): pixel px's 64-bit word holds channel
      // c = 16 i + 4 g + e at bit 16 g + 4 i + e, so lane group g writes one
      // 16-bit half word per pixel
      f32x4 acc[4][2];
      conv32(Xs, wave * 32, wf, acc);
      unsigned short* mbits = reinterpret_cast<unsigned short*>(patch);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int px = wave * 32 + j * 16 + li;
        unsigned mk = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int co = i * 16 + 4 * g;
          float xh[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float yv = acc[i][j][e];
            xh[e] = (yv - cf[128 + co + e]) * cf[192 + co + e];
            mk |= (stem_act(yv, cf[co + e], cf[64 + co + e]) > 0.f ? 1u : 0u) << (4 * i + e);
          }
          uint2 o;
          o.x = pack_bf2(xh[0], xh[1]);
          o.y = pack_bf2(xh[2], xh[3]);
          *reinterpret_cast<uint2*>(Ys + tt_off(px, co)) = o;
        }
        mbits[px * 4 + g] = (unsigned short)mk;
      }
    }
    if (kt < 2) TSTAMP(a.tim, 7 + 9 * kt);
    // the next unit's input patch: issued after this unit's DMA, so the wait
    // below can leave exactly these kRbPT loads in flight (the last unit
    // fetches itself again: an unconditional fetch keeps the compiler's own
    // vmcnt bookkeeping exact)
    fetch(min(u + 1, u1 - 1));
    wait_vmcnt<kRbPT>();  // the pooled rows and the skip gradient have landed ...
    lds_sync();           // ... for every wave
    if (kt < 2) TSTAMP(a.tim, 8 + 9 * kt);
    // dZ = [act > 0] (sum of the pooled gradients whose argmax is this pixel +
    // the skip gradient): maxpool_bwd_kernel's expression and order.  The
    // thread's 8 channels are the same in every item: coefficients read once.
    // thread index made opaque here: the item addresses below are recomputed
    // per unit instead of being hoisted out of the unit loop as live registers
    int tdv = tid;
    asm volatile("" : "+v"(tdv));
    const int c8 = (tdv & 7) * 8;
#pragma unroll
    for (int it = 0; it < kRbNPX * 8 / kRbNT; ++it) {
      // items one after the other (no cross-item interleaving that would
      // hold four items' temporaries at once)
      __builtin_amdgcn_sched_barrier(0);
      // pixel parity uniform per item (it & 1), so an even column has one
      // candidate pooled column and an odd one two; the row parity is uniform
      // per unit (h)
      const int px = 2 * (tdv >> 3) + (it & 1) + (it >> 1) * (kRbNT / 4);
      const int w = q0 + px;
      const bool valid = px < Qs;
      const bool hodd = h & 1, wodd = it & 1;
      const uint4 xhv = *reinterpret_cast<const uint4*>(Ys + tt_off(px, c8));
      const unsigned long long mword = reinterpret_cast<const unsigned long long*>(patch)[px];
      const uint4 av = addv[it];
      const uint4 xv = *reinterpret_cast<const uint4*>(Xs + tt_off(px, c8));
      // the pooled cells that may have this pixel as their argmax, in
      // maxpool_bwd_kernel's order (rows p_lo, p_lo + 1; columns qa, qa + 1):
      // even h: row p_lo only (kh = 1); odd h: kh = 2 then kh = 0; even w:
      // column w / 2 only (kw = 1); odd w: kw = 2 then kw = 0
      const int qa = wodd ? (w - 1) / 2 : w / 2;
      uint2 ix[4];
      uint4 pd[4];
      int want[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int rr = jj >> 1, cc = jj & 1;
        want[jj] = -1;
        if ((rr && !hodd) || (cc && !wodd)) continue;  // uniform: never a candidate
        const int p = p_lo + rr, q = qa + cc;
        const int kh = hodd ? (rr ? 0 : 2) : 1, kw = wodd ? (cc ? 0 : 2) : 1;
        const bool ok = valid && p <= p_hi && q < a.Qp;
        const int slot = ok ? (p & 1) * kRbPQ + (q - qlo) : 0;
        want[jj] = ok ? kh * 3 + kw : -1;
        ix[jj] = *reinterpret_cast<const uint2*>(Pi + slot * 64 + c8);
        pd[jj] = *reinterpret_cast<const uint4*>(Pd + slot * 128 + c8 * 2);
      }
      float acc[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int rr = jj >> 1, cc = jj & 1;
        if ((rr && !hodd) || (cc && !wodd)) continue;
        float gv[8];
        unpack8(pd[jj], gv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const unsigned word = k < 4 ? ix[jj].x : ix[jj].y;
          const int bsel = (word >> ((k & 3) * 8)) & 0xff;
          acc[k] = bsel == want[jj] ? acc[k] + gv[k] : acc[k];
        }
      }
      {
        float r[8];
        unpack8(av, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += r[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = c8 + k;  // bit 16 g + 4 i + e of c = 16 i + 4 g + e
        const int bit = ((c >> 2) & 3) * 16 + (c >> 4) * 4 + (c & 3);
        acc[k] = (valid & (((mword >> bit) & 1ull) != 0ull)) ? acc[k] : 0.f;
      }
      const uint4 o = pack8(acc);
      *reinterpret_cast<uint4*>(Ds + tt_off(px, c8)) = o;
      if (a.dz && valid) *reinterpret_cast<uint4*>(a.dz + (rowpix + w) * a.lddz + cg + c8) = o;
      float dz[8], xh[8];
      unpack8(o, dz);
      unpack8(xhv, xh);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1[k] += dz[k];
        s2[k] += dz[k] * xh[k];
      }
      // the xhat operand of the third GEMM: zero rows past the row end (their
      // im2col rows are zero too)
      if (!valid) *reinterpret_cast<uint4*>(Ys + tt_off(px, c8)) = make_uint4(0, 0, 0, 0);
      if (valid) {  // im2col row chunk of this pixel, centred (the conv has read it)
        float im[8];
        unpack8(xv, im);
#pragma unroll
        for (int k = 0; k < 8; ++k) im[k] -= cf[256 + c8 + k];
        *reinterpret_cast<uint4*>(Xs + tt_off(px, c8)) = pack8(im);
      }
    }
    lds_sync();  // Pd / Pi read for the last time
    if (kt < 2) TSTAMP(a.tim, 9 + 9 * kt);
    if (u + 1 < u1) pool_dma(u + 1, false);
    // GEMMs over the unit's pixels: D[co][k] += sum_px S[px][co] im[px][k]
    {
      const char* S = (wave >> 1) ? Ys : Ds;
      const int cb = (wave & 1) * 32;
#pragma unroll 1
      for (int kk = 0; kk < kRbNPX / 32; ++kk) {
        const int pl = kk * 32 + 8 * g + trq;
        bf16x8 af[2], bf[4];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = cb + i * 16 + 4 * trp;
          af[i] = tr8(S + tt_off(pl, col), S + tt_off(pl + 4, col));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = j * 16 + 4 * trp;
          bf[j] = tr8(Xs + tt_off(pl, col), Xs + tt_off(pl + 4, col));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) gacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], gacc[i][j], 0, 0, 0);
        // sum over pixels of im[.][k], k in [16 wave, 16 wave + 16)
        const bf16x8 bw = wave == 0 ? bf[0] : wave == 1 ? bf[1] : wave == 2 ? bf[2] : bf[3];
        bacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bw, bacc, 0, 0, 0);
      }
    }
    if (kt < 2) TSTAMP(a.tim, 10 + 9 * kt);
  }
  TSTAMP(a.tim, 20);
  // partials of this block: fragments lane-contiguous, then the channel sums
  f32x4* part = reinterpret_cast<f32x4*>(a.part) + ((size_t)blockIdx.y * gridDim.x + blockIdx.x) * kRbPartF4;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) part[(wave * 9 + i * 4 + j) * 64 + lane] = gacc[i][j];
  part[(wave * 9 + 8) * 64 + lane] = bacc;
  lds_sync();  // LDS reuse
  float* red = reinterpret_cast<float*>(smem);  // [32 rows][2][64]
  const int r = tid >> 3;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[(r * 2 + 0) * 64 + c8 + k] = s1[k];
    red[(r * 2 + 1) * 64 + c8 + k] = s2[k];
  }
  lds_sync();
  if (tid < 128) {
    const int q = tid >> 6, c = tid & 63;
    float v = 0.f;
    for (int rr = 0; rr < kRbNT / 8; ++rr) v += red[(rr * 2 + q) * 64 + c];
    reinterpret_cast<float*>(part + 4 * 9 * 64)[q * 64 + c] = v;
  }
  TSTAMP(a.tim, 21);
  TSTAMP_RT(a.tim, 31);
}

// fixed-order sums of the blocks' partials, in fp64: level 1 block (chunk,
// seg, group) sums partials [16 seg, 16 seg + 16) of f32x4 units [64 chunk,
// 64 chunk + 64) (4 split lanes of 4 partials, added in lane order); level 2
// sums the segments the same way, and the last of a group's level-2 blocks to
// arrive (ticket) forms dW from the totals (formerly a third launch; same
// orders, bit-identical).  Level 1 takes no ticket: its ~1.2 k blocks would
// each need an agent-scope release (an L2 write-back) and a returning atomic on
// one word — that single-launch form measured 39.5 us against 14 us for the
// three launches.
constexpr int kRbSeg = 16;
constexpr int kRbChunks = (kRbPartF4 + 63) / 64;

// every wave drains its stores, one lane releases them at agent scope (L2
// write-back: the reader may sit on another XCD) and takes a ticket
__device__ __forceinline__ bool rb_arrive(unsigned* ticket, unsigned total, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == total - 1 ? 1 : 0;
    if (*flag) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
  return *flag != 0;
}

// dW[co][k] = k1 (A - m1 B - m2 X), dgamma = sum dZ xhat, dbeta = sum dZ
// (one block per 64-channel group; totals [unit][4] fp64)
__device__ void stem_rc_finalize(const StemRcArgs& a, int grp) {
  __shared__ double cA[64], cM1[64], cM2[64], bsum[64];
  const int tid = threadIdx.x, cg = grp * 64;
  const double* tot = a.tot + (size_t)grp * kRbPartF4 * 4;
  if (tid < 64) {
    // channel sums: floats [0, 64) sum dZ, [64, 128) sum dZ xhat after the 2304 fragment units
    const double s1 = tot[4 * 9 * 64 * 4 + tid], s2 = tot[4 * 9 * 64 * 4 + 64 + tid];
    const double inv_n = 1.0 / (double)a.npix;
    const int ch = cg + tid;
    cA[tid] = (double)__fmul_rn(a.bn.gamma[ch], a.invstd[ch]);
    cM1[tid] = s1 * inv_n;
    cM2[tid] = s2 * inv_n;
    a.dgamma[ch] = (float)s2;
    a.dbeta[ch] = (float)s1;
  } else if (tid < 128) {
    // sum over pixels of im[.][k]: wave w's ones-tile holds k = 16 w + li in every row
    const int k = tid - 64, w = k >> 4, li = k & 15;
    bsum[k] = tot[((w * 9 + 8) * 64 + li) * 4];
  }
  __syncthreads();
  // fragment units (wave, tile = i*4 + j, lane): co = (wave&1)*32 + i*16 + 4g + e, k = j*16 + li;
  // waves 0/1 hold dZ^T im, waves 2/3 the matching xhat^T im
  for (int u = tid; u < 2 * 8 * 64; u += 256) {
    const int lane = u & 63, t = (u >> 6) & 7, w = u >> 9;
    const int i = t >> 2, j = t & 3, g = lane >> 4, li = lane & 15;
    const double* A = tot + ((w * 9 + t) * 64 + lane) * 4;
    const double* X = tot + (((w + 2) * 9 + t) * 64 + lane) * 4;
    const int k = j * 16 + li;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int co = (w & 1) * 32 + i * 16 + 4 * g + e;
      a.dw[(size_t)(cg + co) * 64 + k] = (float)(cA[co] * (A[e] - cM1[co] * bsum[k] - cM2[co] * X[e]));
    }
  }
}

__global__ void __launch_bounds__(256) stem_rc_sum1_kernel(StemRcArgs a, int nblk, int nseg) {
  __shared__ double sp[4][64][4];
  const int tid = threadIdx.x, lane = tid & 63, sl = tid >> 6;
  const int seg = blockIdx.y, grp = blockIdx.z;
  const f32x4* part = reinterpret_cast<const f32x4*>(a.part) + (size_t)grp * nblk * kRbPartF4;
  const int u = blockIdx.x * 64 + lane;
  double d[4] = {0.0, 0.0, 0.0, 0.0};
  if (u < kRbPartF4) {
    const int b0 = seg * kRbSeg + sl * (kRbSeg / 4);
    f32x4 v[kRbSeg / 4];
#pragma unroll
    for (int q = 0; q < kRbSeg / 4; ++q)
      v[q] = b0 + q < nblk ? part[(size_t)(b0 + q) * kRbPartF4 + u] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < kRbSeg / 4; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] += (double)v[q][e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) sp[sl][lane][e] = d[e];
  __syncthreads();
  if (sl == 0 && u < kRbPartF4) {
    double* o = a.l2 + (((size_t)grp * nseg + seg) * kRbPartF4 + u) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = ((sp[0][lane][e] + sp[1][lane][e]) + sp[2][lane][e]) + sp[3][lane][e];
  }
}

__global__ void __launch_bounds__(256) stem_rc_sum2_kernel(StemRcArgs a, int nseg) {
  __shared__ double sp[4][64][4];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, sl = tid >> 6;
  const int grp = blockIdx.y;
  const int u = blockIdx.x * 64 + lane;
  double d[4] = {0.0, 0.0, 0.0, 0.0};
  if (u < kRbPartF4) {
    for (int s = sl; s < nseg; s += 4) {
      const double* o = a.l2 + (((size_t)grp * nseg + s) * kRbPartF4 + u) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] += o[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) sp[sl][lane][e] = d[e];
  __syncthreads();
  if (sl == 0 && u < kRbPartF4) {
    double* o = a.tot + ((size_t)grp * kRbPartF4 + u) * 4;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = ((sp[0][lane][e] + sp[1][lane][e]) + sp[2][lane][e]) + sp[3][lane][e];
  }
  if (!rb_arrive(a.tkt + grp, gridDim.x, &flag)) return;
  stem_rc_finalize(a, grp);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static int rc_cus() { return device_cu_count(); }

bool stem_rc_ok(int Cout, int P, int Q) {
  return Cout % 64 == 0 && Q <= kRcNPX && Q % 2 == 0 && P % 2 == 0 && Q >= 2;
}

hipError_t launch_stem_rc_fwd(const StemRcArgs& a, int mode, hipStream_t st) {
  if (!stem_rc_ok(a.Cout, a.P, a.Q) || a.Pp * 2 != a.P || a.Qp * 2 != a.Q || a.H != 2 * a.P || a.W != 2 * a.Q ||
      (size_t)a.N * a.H * a.W * 4 >= kOOB)
    return hipErrorInvalidValue;
  const int groups = a.Cout / 64;
  const int total = a.N * a.Pp;
  if (mode == 0) {
    if (!a.stats) return hipErrorInvalidValue;
    // one block per CU (183 VGPRs: one 512-thread block is resident per CU;
    // twice as many blocks ran as two rounds, each paying the prologue and the
    // statistics epilogue)
    const int want = std::max(1, rc_cus() / groups);
    const int per = std::max(1, (total + want - 1) / want);
    const size_t lds = kRcXs + kRcPatchB + 2 * 64 * sizeof(float);
    conv_kernel_tag("stem_rc_fwd_kernel<0>");
    hipLaunchKernelGGL(stem_rc_fwd_kernel<0>, dim3((total + per - 1) / per, groups), dim3(kRcNT), lds, st, a, per);
  } else {
    if (!a.act || !a.pool || !a.idx || (a.bn.training && !a.bn.stats)) return hipErrorInvalidValue;
    const int want = rc_cus() / groups;
    const int per = std::max(1, (total + want - 1) / want);
    const size_t lds = kRcRing + kRcXs + kRcPatchB + 2 * 64 * sizeof(float);
    conv_kernel_tag("stem_rc_fwd_kernel<1>");
    hipLaunchKernelGGL(stem_rc_fwd_kernel<1>, dim3((total + per - 1) / per, groups), dim3(kRcNT), lds, st, a, per);
  }
  return hipGetLastError();
}

int stem_rc_bwd_blocks(int N, int P, int Q, int Cout) {
  const int segs = (Q + kRbNPX - 1) / kRbNPX;
  const int total = N * P * segs;
  const int groups = Cout / 64;
  const int want = std::max(1, 2 * rc_cus() / groups);
  const int per = std::max(1, (total + want - 1) / want);
  return (total + per - 1) / per;
}
int stem_rc_tickets(int Cout) { return Cout / 64; }
static int rc_nseg(int nblk) { return (nblk + kRbSeg - 1) / kRbSeg; }
size_t stem_rc_part_bytes(int N, int P, int Q, int Cout) {
  const int nblk = stem_rc_bwd_blocks(N, P, Q, Cout), groups = Cout / 64;
  return (size_t)nblk * groups * kRbPartF4 * 16 + (size_t)rc_nseg(nblk) * groups * kRbPartF4 * 32;
}
size_t stem_rc_imsum_offset(int Cout) { return (size_t)(Cout / 64) * kRbPartF4 * 32; }
size_t stem_rc_tot_bytes(int Cout) { return stem_rc_imsum_offset(Cout) + kRcImBlocks * sizeof(float); }
size_t stem_rc_l2_offset(int N, int P, int Q, int Cout) {
  return (size_t)stem_rc_bwd_blocks(N, P, Q, Cout) * (Cout / 64) * kRbPartF4 * 16;
}

hipError_t launch_stem_rc_bwd(const StemRcArgs& a, int stage, hipStream_t st) {
  if (!stem_rc_ok(a.Cout, a.P, a.Q) || a.Pp * 2 != a.P || a.Qp * 2 != a.Q || a.H != 2 * a.P || a.W != 2 * a.Q ||
      !a.part || !a.l2 || !a.tot || !a.imsum || !a.dw || !a.bn.training || !a.bn.stats || a.lddpool % 8 || a.ldadd % 8 ||
      !a.add || !a.dpool || !a.idx || !a.tkt || stem_rc_tickets(a.Cout) > kStemTickets)
    return hipErrorInvalidValue;
  // 32-bit buffer offsets of the LDS-DMA (kOOB = 2^31 must lie past every range)
  if ((size_t)a.N * a.P * a.Q * a.ldadd * 2 >= kOOB || (size_t)a.N * a.Pp * a.Qp * a.lddpool * 2 >= kOOB ||
      (size_t)a.N * a.Pp * a.Qp * a.Cout >= kOOB || (size_t)a.N * a.H * a.W * 4 >= kOOB)
    return hipErrorInvalidValue;
  const int groups = a.Cout / 64;
  const int segs = (a.Q + kRbNPX - 1) / kRbNPX;
  const int total = a.N * a.P * segs;
  const int blocks = stem_rc_bwd_blocks(a.N, a.P, a.Q, a.Cout);
  const int per = (total + blocks - 1) / blocks;
  const int nseg = rc_nseg(blocks);
  const int chunks = kRbChunks;
  if (stage == 0) {
    conv_kernel_tag("stem_rc_bwd_kernel");
    hipLaunchKernelGGL(stem_rc_imsum_kernel, dim3(kRcImBlocks), dim3(kRcImNT), 0, st, a);
    hipLaunchKernelGGL(stem_rc_bwd_kernel, dim3(blocks, groups), dim3(kRbNT), kRbLds, st, a, per);
  } else {
    conv_kernel_tag("stem_rc_sum1/sum2");
    hipLaunchKernelGGL(stem_rc_sum1_kernel, dim3(chunks, nseg, groups), dim3(256), 0, st, a, blocks, nseg);
    hipLaunchKernelGGL(stem_rc_sum2_kernel, dim3(chunks, groups), dim3(256), 0, st, a, nseg);
  }
  return hipGetLastError();
}

}  // namespace unet

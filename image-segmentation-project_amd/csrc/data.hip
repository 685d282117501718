// On-GPU image preprocessing of the reference's data path (SURVEY.md §8(f)
// row 3): CellSegmentationDataset.__getitem__ / normalize_microscopy_image
// (/root/reference/dataset.py:30-66) and the index-exact transforms of
// CellAugmenter (dataset.py:147-151), for a batch of decoded uint8 frames
// resident in HBM.  The reference runs this per image on the host with cv2 and
// num_workers=0 (dataset.py:138), which cannot feed even one MI355X.
//
//   resize_area_kernel      cv2.resize INTER_AREA (downscale): integer factors
//                           as resizeAreaFast_ (block sum * 1/area), otherwise
//                           the computeResizeAreaTab coverage weights, float
//                           accumulation, cvRound                        (:51)
//   resize_area_up_kernel   the same call enlarging an axis: OpenCV's
//                           fixed-point area-mode linear resize          (:51)
//   mask_kernel             cv2.resize INTER_NEAREST, then mask > 0 -> 1.f (:52,61)
//   normalize_kernel        np.percentile(2, 98) + clip + astype(uint8) (:33-34),
//                           CLAHE(2.0, 8x8) (:37-38), min-max to [0, 1] (:41);
//                           one 1024-thread block per image: 256-bin and
//                           64 x 256 tile histograms in LDS (integer atomics:
//                           order-independent), tile LUTs, bilinear LUT blend
//   rot90_vflip_kernel      A.RandomRotate90 (np.rot90 by k) + A.VerticalFlip
//
// Everything is byte / integer work except the float blends, which follow the
// restated OpenCV expressions with explicit roundings (no FMA contraction) so
// the numpy oracle (oracle/dataset_ref.py) reproduces them bit for bit.
#include <math.h>

#include "common.h"
#include "kernels.h"

// The float blends restate OpenCV's expressions operation by operation: no
// fused multiply-adds in this file (hipcc contracts a*b+c by default, and the
// __fmul_rn / __fadd_rn spellings alone do not stop it).
#pragma clang fp contract(off)

namespace unet {

__device__ __forceinline__ int cv_round(float v) { return (int)rintf(v); }
__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// computeResizeAreaTab entries of destination index d: up to 3 kinds (partial
// head, full cells, partial tail); returns the count and fills (si, alpha)
__device__ __forceinline__ int area_entries(int d, int ssize, double scale, int* si, float* al, int cap) {
  const double fs1 = d * scale, fs2 = fs1 + scale;
  const double cell = fmin(scale, (double)ssize - fs1);
  int s1 = (int)ceil(fs1), s2 = (int)floor(fs2);
  s2 = min(s2, ssize - 1);
  s1 = min(s1, s2);
  int k = 0;
  if (s1 - fs1 > 1e-3 && k < cap) { si[k] = s1 - 1; al[k++] = (float)((s1 - fs1) / cell); }
  for (int s = s1; s < s2 && k < cap; ++s) { si[k] = s; al[k++] = (float)(1.0 / cell); }
  if (fs2 - s2 > 1e-3 && k < cap) { si[k] = s2; al[k++] = (float)(fmin(fmin(fs2 - s2, 1.0), cell) / cell); }
  return k;
}

constexpr int kAreaCap = 64;  // scale factors up to 62 per axis

__global__ void __launch_bounds__(256) resize_area_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          int N, int H, int W, int oh, int ow, int fx, int fy) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * oh * ow) return;
  const int dx = (int)(i % ow), dy = (int)((i / ow) % oh), n = (int)(i / ((int64_t)oh * ow));
  const uint8_t* img = src + (int64_t)n * H * W;
  if (fx > 0) {  // integer factors: resizeAreaFast_
    int s = 0;
    for (int y = 0; y < fy; ++y)
      for (int x = 0; x < fx; ++x) s += img[(int64_t)(dy * fy + y) * W + dx * fx + x];
    if (fx == 2 && fy == 2) {  // ResizeAreaFastVec_SIMD_8u: (a + b + c + d + 2) >> 2
      dst[i] = (uint8_t)((s + 2) >> 2);
      return;
    }
    const float scale = __fdiv_rn(1.f, (float)(fx * fy));
    dst[i] = sat_u8(cv_round(__fmul_rn((float)s, scale)));
    return;
  }
  int xs[kAreaCap], ys[kAreaCap];
  float xa[kAreaCap], ya[kAreaCap];
  const int nx = area_entries(dx, W, 1.0 / ((double)ow / W), xs, xa, kAreaCap);
  const int ny = area_entries(dy, H, 1.0 / ((double)oh / H), ys, ya, kAreaCap);
  float acc = 0.f;
  for (int j = 0; j < ny; ++j) {
    const uint8_t* row = img + (int64_t)ys[j] * W;
    float b = 0.f;
    for (int k = 0; k < nx; ++k) b = __fadd_rn(b, __fmul_rn((float)row[xs[k]], xa[k]));
    const float t = __fmul_rn(b, ya[j]);
    acc = j == 0 ? t : __fadd_rn(acc, t);
  }
  dst[i] = sat_u8(cv_round(acc));
}

// cv2.resize INTER_AREA when an axis is ENLARGED (OpenCV resize.cpp: not
// is-area: resizeGeneric_ with area_mode linear coefficients, fixed point for
// 8U): per axis sx = floor(d * scale), f = (float)((d+1) - (sx+1) * inv_scale),
// f = f <= 0 ? 0 : f - floor(f), coefficients saturate_cast<short>({1-f, f} *
// 2048); horizontal D = S[sx] a0 + S[sx+1] a1 (S[sx] * 2048 once sx + 1 >= W),
// vertical ((b0 (D0 >> 4)) >> 16) + ((b1 (D1 >> 4)) >> 16) + 2) >> 2 over rows
// clip(sy, sy+1 to H-1).  Integer arithmetic after the coefficients.
__device__ __forceinline__ void area_linear_coef(int d, int ssize, int dsize, int& s, int& c0, int& c1) {
  const double inv = (double)dsize / ssize, scale = 1.0 / inv;
  s = (int)floor(d * scale);
  float f = (float)((d + 1) - (s + 1) * inv);
  f = f <= 0.f ? 0.f : __fsub_rn(f, floorf(f));
  if (s >= ssize - 1) s = ssize - 1;
  c0 = (int)rintf(__fmul_rn(__fsub_rn(1.f, f), 2048.f));
  c1 = (int)rintf(__fmul_rn(f, 2048.f));
}

__global__ void __launch_bounds__(256) resize_area_up_kernel(const uint8_t* __restrict__ src,
                                                             uint8_t* __restrict__ dst, int N, int H, int W, int oh,
                                                             int ow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * oh * ow) return;
  const int dx = (int)(i % ow), dy = (int)((i / ow) % oh), n = (int)(i / ((int64_t)oh * ow));
  const uint8_t* img = src + (int64_t)n * H * W;
  int sx, a0, a1, sy, b0, b1;
  area_linear_coef(dx, W, ow, sx, a0, a1);
  area_linear_coef(dy, H, oh, sy, b0, b1);
  int D[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint8_t* row = img + (int64_t)min(sy + k, H - 1) * W;
    D[k] = sx + 1 >= W ? (int)row[sx] * 2048 : (int)row[sx] * a0 + (int)row[sx + 1] * a1;
  }
  dst[i] = (uint8_t)((((b0 * (D[0] >> 4)) >> 16) + ((b1 * (D[1] >> 4)) >> 16) + 2) >> 2);
}

__global__ void __launch_bounds__(256) mask_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst, int N,
                                                   int H, int W, int oh, int ow) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * oh * ow) return;
  const int dx = (int)(i % ow), dy = (int)((i / ow) % oh), n = (int)(i / ((int64_t)oh * ow));
  const int sx = min((int)floor(dx * (1.0 / ((double)ow / W))), W - 1);  // cv::resize ifx = 1 / inv_scale
  const int sy = min((int)floor(dy * (1.0 / ((double)oh / H))), H - 1);
  dst[i] = src[((int64_t)n * H + sy) * W + sx] > 0 ? 1.f : 0.f;
}

// k-th smallest value (0-based) of an image from its 256-bin histogram
__device__ __forceinline__ int kth_from_hist(const int* hist, int64_t k) {
  int64_t c = 0;
  for (int v = 0; v < 256; ++v) {
    c += hist[v];
    if (c > k) return v;
  }
  return 255;
}

// np.percentile(img, q), method 'linear' (numpy's _lerp form), float64
__device__ double percentile_from_hist(const int* hist, int64_t n, double q) {
  const double h = (double)(n - 1) * (q / 100.0);
  const int64_t lo = (int64_t)floor(h);
  const int64_t hi = lo + 1 < n ? lo + 1 : n - 1;
  const double t = h - (double)lo;
  const double a = kth_from_hist(hist, lo), b = kth_from_hist(hist, hi);
  const double d = b - a;
  return t >= 0.5 ? b - d * (1.0 - t) : a + d * t;
}

// clip to [plo, phi] in float64, then astype(uint8) (truncation)
__device__ __forceinline__ int clip_trunc(int v, double plo, double phi) {
  const double c = v < plo ? plo : (v > phi ? phi : (double)v);
  return (int)c;
}

// BORDER_REFLECT_101 index into [0, n)
__device__ __forceinline__ int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

constexpr int kGrid = 8;

struct NormSmem {
  int hist[256];
  int thist[kGrid * kGrid][256];
  uint8_t lut[kGrid * kGrid][256];
  double plo, phi;
  int mn, mx;
};

// CLAHE value of pixel (y, x) of the clipped image (LUT blend, clahe.cpp
// CLAHE_Interpolation_Body)
__device__ __forceinline__ int clahe_px(const NormSmem& s, int v, int y, int x, int tw, int th) {
  const float inv_tw = __fdiv_rn(1.f, (float)tw), inv_th = __fdiv_rn(1.f, (float)th);
  const float txf = __fadd_rn(__fmul_rn((float)x, inv_tw), -0.5f);
  const float tyf = __fadd_rn(__fmul_rn((float)y, inv_th), -0.5f);
  int tx1 = (int)floorf(txf), ty1 = (int)floorf(tyf);
  const float xa = __fadd_rn(txf, -(float)tx1), ya = __fadd_rn(tyf, -(float)ty1);
  const float xa1 = __fadd_rn(1.f, -xa), ya1 = __fadd_rn(1.f, -ya);
  const int tx2 = min(tx1 + 1, kGrid - 1), ty2 = min(ty1 + 1, kGrid - 1);
  tx1 = max(tx1, 0);
  ty1 = max(ty1, 0);
  const float l11 = s.lut[ty1 * kGrid + tx1][v], l12 = s.lut[ty1 * kGrid + tx2][v];
  const float l21 = s.lut[ty2 * kGrid + tx1][v], l22 = s.lut[ty2 * kGrid + tx2][v];
  const float top = __fadd_rn(__fmul_rn(l11, xa1), __fmul_rn(l12, xa));
  const float bot = __fadd_rn(__fmul_rn(l21, xa1), __fmul_rn(l22, xa));
  const float r = __fadd_rn(__fmul_rn(top, ya1), __fmul_rn(bot, ya));
  return sat_u8(cv_round(r));
}

__global__ void __launch_bounds__(1024) normalize_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                         int H, int W, int normalize) {
  __shared__ NormSmem s;
  const int n = blockIdx.x, tid = threadIdx.x;
  const uint8_t* img = src + (int64_t)n * H * W;
  float* out = dst + (int64_t)n * H * W;
  const int64_t npx = (int64_t)H * W;
  if (!normalize) {  // image.astype(np.float32) / 255.0  (dataset.py:56)
    for (int64_t i = tid; i < npx; i += blockDim.x) out[i] = __fdiv_rn((float)img[i], 255.f);
    return;
  }
  for (int i = tid; i < 256; i += blockDim.x) s.hist[i] = 0;
  for (int i = tid; i < kGrid * kGrid * 256; i += blockDim.x) (&s.thist[0][0])[i] = 0;
  if (tid == 0) { s.mn = 255; s.mx = 0; }
  __syncthreads();
  for (int64_t i = tid; i < npx; i += blockDim.x) atomicAdd(&s.hist[img[i]], 1);
  __syncthreads();
  if (tid == 0) {
    s.plo = percentile_from_hist(s.hist, npx, 2.0);
    s.phi = percentile_from_hist(s.hist, npx, 98.0);
  }
  __syncthreads();
  const double plo = s.plo, phi = s.phi;
  // tile histograms of the clipped image, padded to a multiple of the grid by reflection
  // clahe.cpp pads BOTH sides by kGrid - size % kGrid when EITHER is not a
  // multiple of the grid (a side that is a multiple gains a whole tile)
  const bool pad = (H % kGrid) != 0 || (W % kGrid) != 0;
  const int He = pad ? H + kGrid - H % kGrid : H, We = pad ? W + kGrid - W % kGrid : W;
  const int th = He / kGrid, tw = We / kGrid;
  for (int64_t i = tid; i < (int64_t)He * We; i += blockDim.x) {
    const int y = (int)(i / We), x = (int)(i % We);
    const int v = clip_trunc(img[(int64_t)reflect101(y, H) * W + reflect101(x, W)], plo, phi);
    atomicAdd(&s.thist[(y / th) * kGrid + x / tw][v], 1);
  }
  __syncthreads();
  // per tile: clip at the limit, redistribute the excess, cumulative LUT
  const int area = th * tw;
  const int limit = max((int)(2.0 * area / 256.0), 1);
  const float lut_scale = __fdiv_rn(255.f, (float)area);
  if (tid < kGrid * kGrid) {
    int* hst = s.thist[tid];
    int clipped = 0;
    for (int v = 0; v < 256; ++v)
      if (hst[v] > limit) { clipped += hst[v] - limit; hst[v] = limit; }
    const int batch = clipped / 256;
    int residual = clipped - batch * 256;
    for (int v = 0; v < 256; ++v) hst[v] += batch;
    if (residual) {
      const int step = max(256 / residual, 1);
      for (int v = 0; v < 256 && residual > 0; v += step, --residual) hst[v] += 1;
    }
    int sum = 0;
    for (int v = 0; v < 256; ++v) {
      sum += hst[v];
      s.lut[tid][v] = sat_u8(cv_round(__fmul_rn((float)sum, lut_scale)));
    }
  }
  __syncthreads();
  int mn = 255, mx = 0;
  for (int64_t i = tid; i < npx; i += blockDim.x) {
    const int y = (int)(i / W), x = (int)(i % W);
    const int c = clahe_px(s, clip_trunc(img[i], plo, phi), y, x, tw, th);
    mn = min(mn, c);
    mx = max(mx, c);
  }
  atomicMin(&s.mn, mn);
  atomicMax(&s.mx, mx);
  __syncthreads();
  const int cmin = s.mn;
  const double den = (double)(s.mx - cmin) + 1e-8;  // uint8 range + 1e-8 -> float64
  for (int64_t i = tid; i < npx; i += blockDim.x) {
    const int y = (int)(i / W), x = (int)(i % W);
    const int c = clahe_px(s, clip_trunc(img[i], plo, phi), y, x, tw, th);
    out[i] = (float)((double)(c - cmin) / den);
  }
}

// out = vflip(rot90(in, k)) per image (square frames when k is odd)
__global__ void __launch_bounds__(256) rot90_vflip_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          int N, int H, int W, const int* __restrict__ ks,
                                                          const int* __restrict__ flips) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * H * W) return;
  const int n = (int)(i / ((int64_t)H * W));
  const int k = ((ks[n] % 4) + 4) % 4;
  const int Ho = (k & 1) ? W : H, Wo = (k & 1) ? H : W;  // output dims
  const int64_t r = i - (int64_t)n * H * W;
  int y = (int)(r / Wo), x = (int)(r % Wo);
  if (flips[n]) y = Ho - 1 - y;
  // np.rot90(a, k) (counter-clockwise): out[y][x] = a[...]
  int sy, sx;
  switch (k) {
    case 0: sy = y; sx = x; break;
    case 1: sy = x; sx = W - 1 - y; break;
    case 2: sy = H - 1 - y; sx = W - 1 - x; break;
    default: sy = H - 1 - x; sx = y; break;
  }
  dst[i] = src[(int64_t)n * H * W + (int64_t)sy * W + sx];
}


// A.Affine (dataset.py:150-151) = cv2.warpAffine, OpenCV's fixed-point path
// (imgwarp.cpp WarpAffineInvoker + remapBilinear / remapNearest, BORDER_CONSTANT
// 0), restated in oracle/dataset_ref.py warp_affine_u8.  m: per frame the
// dst -> src map [6] (cv::invertAffineTransform of the forward matrix, made on
// the host); the source coordinate of output column x, row y is
// X = cvRound((m1*y + m2)*1024) + rd + cvRound(m0*x*1024) (Y likewise), double
// products rounded separately (no fma: this file is built -ffp-contract=off).
// active[n] == 0: the frame is copied; vflip[n]: A.VerticalFlip, which follows
// the affine step in the reference pipeline, folded into the output row.
__device__ __forceinline__ long long cv_round_d(double v) {
  double r = rint(v);
  r = fmin(fmax(r, -2147483648.0), 2147483647.0);  // saturate_cast<int>
  return (long long)r;
}

__global__ void __launch_bounds__(256) warp_affine_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                          int N, int H, int W, const double* __restrict__ m,
                                                          const int* __restrict__ active,
                                                          const int* __restrict__ vflip, int nearest) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * H * W) return;
  const int n = (int)(i / ((int64_t)H * W));
  const int64_t r = i - (int64_t)n * H * W;
  const int y = (int)(r / W), x = (int)(r - (int64_t)(r / W) * W);
  const int yy = vflip[n] ? H - 1 - y : y;  // the warp's output row stored at row y
  const uint8_t* S = src + (int64_t)n * H * W;
  if (!active[n]) {
    dst[i] = S[(int64_t)yy * W + x];
    return;
  }
  const double* M = m + (size_t)n * 6;
  const double xd = (double)x, yd = (double)yy;
  const long long adelta = cv_round_d(__dmul_rn(__dmul_rn(M[0], xd), 1024.0));
  const long long bdelta = cv_round_d(__dmul_rn(__dmul_rn(M[3], xd), 1024.0));
  const int rd = nearest ? 512 : 16;
  const long long X0 = cv_round_d(__dmul_rn(__dadd_rn(__dmul_rn(M[1], yd), M[2]), 1024.0)) + rd;
  const long long Y0 = cv_round_d(__dmul_rn(__dadd_rn(__dmul_rn(M[4], yd), M[5]), 1024.0)) + rd;
  const long long X = X0 + adelta, Y = Y0 + bdelta;
  if (nearest) {
    const long long sx = X >> 10, sy = Y >> 10;
    dst[i] = (sx >= 0 && sx < W && sy >= 0 && sy < H) ? S[sy * W + sx] : (uint8_t)0;
    return;
  }
  const long long Xs = X >> 5, Ys = Y >> 5;
  const long long sx = Xs >> 5, sy = Ys >> 5;
  const int fx = (int)(Xs & 31), fy = (int)(Ys & 31);
  if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
    dst[i] = 0;
    return;
  }
  auto tap = [&](long long yv, long long xv) -> int {
    return (xv >= 0 && xv < W && yv >= 0 && yv < H) ? (int)S[yv * W + xv] : 0;
  };
  const int w0 = (32 - fy) * (32 - fx) * 32, w1 = (32 - fy) * fx * 32;
  const int w2 = fy * (32 - fx) * 32, w3 = fy * fx * 32;
  const int v = tap(sy, sx) * w0 + tap(sy, sx + 1) * w1 + tap(sy + 1, sx) * w2 + tap(sy + 1, sx + 1) * w3;
  dst[i] = sat_u8((v + (1 << 14)) >> 15);
}

// A.AdvancedBlur (dataset.py:153) = cv2.filter2D(img, -1, kernel), anchor at
// the centre, BORDER_REFLECT_101: fp32 s = s + k * v over the non-zero
// coefficients in row-major order, cvRound, saturate (oracle filter2d_u8).
// kern: [N][7][7] (top-left ksz[n] x ksz[n] used); ksz[n] == 0: copy.
__global__ void __launch_bounds__(256) filter2d_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                       int N, int H, int W, const float* __restrict__ kern,
                                                       const int* __restrict__ ksz) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * H * W) return;
  const int n = (int)(i / ((int64_t)H * W));
  const int64_t r = i - (int64_t)n * H * W;
  const int y = (int)(r / W), x = (int)(r - (int64_t)(r / W) * W);
  const uint8_t* S = src + (int64_t)n * H * W;
  const int k = ksz[n];
  if (k == 0) {
    dst[i] = S[r];
    return;
  }
  const float* K = kern + (size_t)n * 49;
  const int rad = k >> 1;
  float acc = 0.f;
  for (int a = 0; a < k; ++a) {
    const int sy = reflect101(y + a - rad, H);
    for (int b = 0; b < k; ++b) {
      const float f = K[a * 7 + b];
      if (f == 0.f) continue;
      acc = __fadd_rn(acc, __fmul_rn(f, (float)S[(int64_t)sy * W + reflect101(x + b - rad, W)]));
    }
  }
  dst[i] = sat_u8(cv_round(acc));
}

static inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

hipError_t launch_resize_area(const uint8_t* src, uint8_t* dst, int N, int H, int W, int oh, int ow, hipStream_t st) {
  if (N <= 0 || oh <= 0 || ow <= 0 || H <= 0 || W <= 0) return hipErrorInvalidValue;
  if (oh > H || ow > W) {  // an axis is enlarged: cv::resize leaves the area path
    hipLaunchKernelGGL(resize_area_up_kernel, dim3(blocks_for((int64_t)N * oh * ow)), dim3(256), 0, st, src, dst, N, H,
                       W, oh, ow);
    return hipGetLastError();
  }
  if ((double)W / ow > kAreaCap - 2 || (double)H / oh > kAreaCap - 2) return hipErrorInvalidValue;
  // cv::resize is_area_fast: both scales 1 / (dsize / ssize) within DBL_EPSILON of an integer
  const double sx = 1.0 / ((double)ow / W), sy = 1.0 / ((double)oh / H);
  const bool fast = fabs(sx - rint(sx)) < 2.220446049250313e-16 && fabs(sy - rint(sy)) < 2.220446049250313e-16;
  const int fx = fast ? (int)rint(sx) : 0;
  const int fy = fast ? (int)rint(sy) : 0;
  hipLaunchKernelGGL(resize_area_kernel, dim3(blocks_for((int64_t)N * oh * ow)), dim3(256), 0, st, src, dst, N, H, W,
                     oh, ow, fx, fy);
  return hipGetLastError();
}

hipError_t launch_mask_prep(const uint8_t* src, float* dst, int N, int H, int W, int oh, int ow, hipStream_t st) {
  if (N <= 0 || oh <= 0 || ow <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mask_kernel, dim3(blocks_for((int64_t)N * oh * ow)), dim3(256), 0, st, src, dst, N, H, W, oh, ow);
  return hipGetLastError();
}

hipError_t launch_normalize(const uint8_t* src, float* dst, int N, int H, int W, int normalize, hipStream_t st) {
  if (N <= 0 || H < kGrid || W < kGrid) return hipErrorInvalidValue;
  hipLaunchKernelGGL(normalize_kernel, dim3(N), dim3(1024), 0, st, src, dst, H, W, normalize);
  return hipGetLastError();
}

hipError_t launch_rot90_vflip(const uint8_t* src, uint8_t* dst, int N, int H, int W, const int* k, const int* flip,
                              hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rot90_vflip_kernel, dim3(blocks_for((int64_t)N * H * W)), dim3(256), 0, st, src, dst, N, H, W, k,
                     flip);
  return hipGetLastError();
}

hipError_t launch_warp_affine(const uint8_t* src, uint8_t* dst, int N, int H, int W, const double* m, const int* active,
                              const int* vflip, int nearest, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0 || (int64_t)H * W >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(warp_affine_kernel, dim3(blocks_for((int64_t)N * H * W)), dim3(256), 0, st, src, dst, N, H, W, m,
                     active, vflip, nearest);
  return hipGetLastError();
}

hipError_t launch_filter2d(const uint8_t* src, uint8_t* dst, int N, int H, int W, const float* kern, const int* ksz,
                           hipStream_t st) {
  if (N <= 0 || H < 4 || W < 4) return hipErrorInvalidValue;  // reflect-101 of a 7x7 footprint
  hipLaunchKernelGGL(filter2d_kernel, dim3(blocks_for((int64_t)N * H * W)), dim3(256), 0, st, src, dst, N, H, W, kern,
                     ksz);
  return hipGetLastError();
}

}  // namespace unet

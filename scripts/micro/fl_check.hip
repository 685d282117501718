// Standalone check of conv3x3_fl_kernel (conv_fl.hip; -DWS2: conv3x3_ws2_kernel,
// C = 64, standard weight pack) against a CPU reference: every buffer sits inside a guard region filled with a sentinel,
// so an out-of-range access lands in mapped memory and shows up as a changed
// guard instead of a GPU fault.  Forward (bias + BN sums) and data gradient
// (addend + fused BN-backward epilogue), C = Cout = 128, 16 x 32 x 64 pixels
// (256 work items: the smallest shape the launcher takes on 256 CUs).
// build: hipcc -O3 --offload-arch=gfx950 -I../../image-segmentation-project_amd/csrc \
//          -o fl_check fl_check.hip ../../image-segmentation-project_amd/csrc/conv_fl.hip
//        (the same with -DWS2 -o ws2_check)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "kernels.h"

namespace unet {
void conv_kernel_tag(const char*) {}
}
using namespace unet;

static const size_t kGuard = 8 << 20;
static const unsigned char kSent = 0x5a;

struct Buf {
  char* base = nullptr;
  size_t n = 0;
  void* p() const { return base + kGuard; }
};
static Buf alloc(size_t bytes) {
  Buf b;
  b.n = bytes;
  if (hipMalloc(&b.base, bytes + 2 * kGuard) != hipSuccess) { printf("alloc failed\n"); exit(1); }
  hipMemset(b.base, kSent, bytes + 2 * kGuard);
  return b;
}
static bool guards_ok(const Buf& b, const char* name) {
  std::vector<unsigned char> h(b.n + 2 * kGuard);
  hipMemcpy(h.data(), b.base, h.size(), hipMemcpyDeviceToHost);
  size_t bad = 0, first = 0;
  for (size_t i = 0; i < kGuard; ++i)
    if (h[i] != kSent && !bad++) first = i;
  for (size_t i = kGuard + b.n; i < h.size(); ++i)
    if (h[i] != kSent && !bad++) first = i;
  if (bad) printf("GUARD %s: %zu bytes changed (first at %zd rel)\n", name, bad, (ssize_t)first - (ssize_t)kGuard);
  return bad == 0;
}
static uint16_t f2b(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float b2f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}
static uint64_t rng = 88172645463325252ull;
static float frand() {
  rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
  return (float)((rng >> 11) * (1.0 / 9007199254740992.0)) * 2.f - 1.f;
}

int main(int argc, char** argv) {
#ifdef WS2
  const int N = 4, H = 32, W = 64, C = 64, Co = 64;
#else
  const int N = 16, H = 32, W = 64, C = 128, Co = 128;
#endif
  const int npix = N * H * W;
  // weights W[co][ci][3][3] (fp32 reference), input x[n][h][w][ci]
  std::vector<float> w((size_t)Co * C * 9), x((size_t)npix * C), bias(Co);
  for (auto& v : w) v = b2f(f2b(frand() * 0.05f));
  for (auto& v : x) v = b2f(f2b(frand()));
  for (auto& v : bias) v = frand();
  bool all_ok = true;
  for (int mode = 0; mode < 2; ++mode) {
    // mode 0: y = conv(x) + bias, BN sums of y; mode 1: dgrad of conv(., w)
    // applied to x as dY (Ci <-> Co swap is symmetric here), + addend, fused BN bwd
    const int K = C, M = Co;  // reduction / output channels
    std::vector<uint16_t> wch((size_t)K * 9 * M);
    for (int co = 0; co < Co; ++co)
      for (int ci = 0; ci < C; ++ci)
        for (int t = 0; t < 9; ++t) {
          const float v = w[((size_t)co * C + ci) * 9 + t];
#ifdef WS2  // standard pack [out][9][K]
          if (mode == 0) wch[((size_t)co * 9 + t) * C + ci] = f2b(v);
          else wch[((size_t)ci * 9 + t) * Co + co] = f2b(v);
#else
          if (mode == 0) wch[((size_t)((ci >> 5) * 9 + t) * M + co) * 32 + (ci & 31)] = f2b(v);
          else wch[((size_t)((co >> 5) * 9 + t) * C + ci) * 32 + (co & 31)] = f2b(v);  // K = Co
#endif
        }
    std::vector<uint16_t> xb((size_t)npix * K), addb((size_t)npix * M), actb((size_t)npix * M), yb((size_t)npix * M);
    for (size_t i = 0; i < xb.size(); ++i) xb[i] = f2b(x[i]);
    for (size_t i = 0; i < addb.size(); ++i) {
      addb[i] = f2b(frand());
      actb[i] = f2b(frand());  // mask: act > 0
      yb[i] = f2b(frand());
    }
    std::vector<float> mean(M), invstd(M);
    for (int c = 0; c < M; ++c) { mean[c] = frand() * 0.1f; invstd[c] = 1.f + 0.5f * frand(); }
    // reference
    std::vector<float> ref((size_t)npix * M);
    std::vector<double> r0(M, 0.0), r1(M, 0.0);
    for (int n = 0; n < N; ++n)
      for (int oh = 0; oh < H; ++oh)
        for (int ow = 0; ow < W; ++ow)
          for (int co = 0; co < M; ++co) {
            double s = 0;
            for (int r = 0; r < 3; ++r)
              for (int q = 0; q < 3; ++q) {
                int ih, iw;
                if (mode == 0) { ih = oh - 1 + r; iw = ow - 1 + q; }
                else { ih = oh + 1 - r; iw = ow + 1 - q; }
                if (ih < 0 || ih >= H || iw < 0 || iw >= W) continue;
                const float* xp = &x[((size_t)(n * H + ih) * W + iw) * K];
                for (int k = 0; k < K; ++k) {
                  // mode 0: w[co][k]; mode 1 (dgrad, out = ci = co here): w[k][co] tap (r, q)
                  const float wv = mode == 0 ? w[((size_t)co * C + k) * 9 + r * 3 + q] : w[((size_t)k * C + co) * 9 + r * 3 + q];
                  s += (double)b2f(f2b(xp[k])) * wv;
                }
              }
            const size_t o = ((size_t)(n * H + oh) * W + ow) * M + co;
            float v = (float)s;
            if (mode == 0) {
              v += bias[co];
              r0[co] += v; r1[co] += (double)v * v;
            } else {
              v += b2f(addb[o]);
              if (!(b2f(actb[o]) > 0.f)) v = 0.f;
              const float dz = b2f(f2b(v));
              r0[co] += dz;
              r1[co] += (double)dz * (b2f(yb[o]) - mean[co]) * invstd[co];
            }
            ref[o] = v;
          }
    Buf dx = alloc(xb.size() * 2), dw = alloc(wch.size() * 2), dy = alloc((size_t)npix * M * 2);
    Buf dadd = alloc(addb.size() * 2), dact = alloc(actb.size() * 2), dyy = alloc(yb.size() * 2);
    Buf dbias = alloc(M * 4), dmean = alloc(M * 4), dinv = alloc(M * 4);
    Buf dsums = alloc((size_t)kStatRep * 2 * M * 8);
    hipMemcpy(dx.p(), xb.data(), xb.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dw.p(), wch.data(), wch.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dadd.p(), addb.data(), addb.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dact.p(), actb.data(), actb.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dyy.p(), yb.data(), yb.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(dbias.p(), bias.data(), M * 4, hipMemcpyHostToDevice);
    hipMemcpy(dmean.p(), mean.data(), M * 4, hipMemcpyHostToDevice);
    hipMemcpy(dinv.p(), invstd.data(), M * 4, hipMemcpyHostToDevice);
    hipMemset(dsums.p(), 0, (size_t)kStatRep * 2 * M * 8);
    ConvFwdArgs a = {};
    a.x = (const bf16_t*)dx.p(); a.ldx = K;
#ifdef WS2
    a.w = (const bf16_t*)dw.p();
#else
    a.wch = (const bf16_t*)dw.p();
#endif
    a.y = (bf16_t*)dy.p(); a.ldy = M;
    a.N = N; a.H = H; a.W = W; a.C = K; a.P = H; a.Q = W; a.Cout = M;
    a.R = 3; a.S = 3; a.stride = 1; a.pad = 1;
    if (mode == 0) {
      a.bias = (const float*)dbias.p();
      a.stats = (double*)dsums.p();
    } else {
      a.add = (const bf16_t*)dadd.p(); a.ldadd = M;
      a.bb.sums = (double*)dsums.p();
      a.bb.act = (const bf16_t*)dact.p(); a.bb.ldact = M;
      a.bb.y = (const bf16_t*)dyy.p(); a.bb.ldy = M;
      a.bb.mean = (const float*)dmean.p(); a.bb.invstd = (const float*)dinv.p();
      a.bb.C = M;
    }
#ifdef WS2
    hipError_t e = launch_conv3x3_ws2(a, mode, 0);
#else
    hipError_t e = launch_conv3x3_fl(a, mode, 0);
#endif
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { printf("mode %d: launch/sync error %s\n", mode, hipGetErrorString(e)); return 1; }
    std::vector<uint16_t> out((size_t)npix * M);
    hipMemcpy(out.data(), dy.p(), out.size() * 2, hipMemcpyDeviceToHost);
    std::vector<double> sums((size_t)kStatRep * 2 * M);
    hipMemcpy(sums.data(), dsums.p(), sums.size() * 8, hipMemcpyDeviceToHost);
    double num = 0, den = 0;
    for (size_t i = 0; i < out.size(); ++i) {
      const double d = b2f(out[i]) - ref[i];
      num += d * d; den += (double)ref[i] * ref[i];
    }
    double s0e = 0, s1e = 0, s0n = 0, s1n = 0;
    for (int c = 0; c < M; ++c) {
      double t0 = 0, t1 = 0;
      for (int r = 0; r < kStatRep; ++r) { t0 += sums[(size_t)r * 2 * M + c]; t1 += sums[(size_t)r * 2 * M + M + c]; }
      s0e += (t0 - r0[c]) * (t0 - r0[c]); s0n += r0[c] * r0[c];
      s1e += (t1 - r1[c]) * (t1 - r1[c]); s1n += r1[c] * r1[c];
    }
    const double rel = sqrt(num / den), rs0 = sqrt(s0e / s0n), rs1 = sqrt(s1e / s1n);
    bool ok = rel < 1e-2 && rs0 < 1e-2 && rs1 < 1e-2;
    for (auto* b : {&dx, &dw, &dy, &dadd, &dact, &dyy, &dbias, &dmean, &dinv, &dsums}) ok &= guards_ok(*b, "buf");
    printf("mode %d: out rel L2 %.3e  sum0 rel %.3e  sum1 rel %.3e  %s\n", mode, rel, rs0, rs1, ok ? "OK" : "FAIL");
    all_ok &= ok;
  }
  return all_ok ? 0 : 1;
}

// Full-line halo convolution: the 3x3 / stride-1 / pad-1 forward conv and its
// data gradient for C % 128 == 0 and Cout % 64 == 0 (SURVEY.md §8(a) rows a3 /
// a6: enc2-4 BasicBlocks, decoder4 / decoder3; reference
// advanced_models.py:84-87,197-205).
//
// Why a separate kernel: the per-CU L2 -> LDS rate of LDS-DMA is set by cache
// LINES, not bytes (scripts/micro/dma_rate.hip, profiles/r05/s1/dma_rate.txt:
// 64-B pieces of 128-B lines 32 B/clk/CU, whole lines 54 B/clk/CU).  The
// halo-streamed kernel (conv_halo.hip) stages 32 channels = 64 B per pixel and
// per weight row, so its stages ran at the DMA rate of half lines (~2.9k cycles
// per stage for ~2.0k cycles of MFMA, profiles/r04/s1 conv_timing*), and its
// epilogue read its operands in 32-B pieces.  Here every global access moves
// whole lines:
//  * halo: 64-channel super-chunks, one 128-B LDS row per halo pixel holding
//    both 32-channel panels (fl_off swizzle, conv_halo.hip);
//  * weights: a chunk-major pack [C/32][9][Cout][32] (PK_CONV_*_CH, pack_kernel):
//    one 32-channel sub-stage of a 64-output-channel block is 9 contiguous
//    4 KB runs;
//  * epilogue: the accumulators are transposed through LDS so that a lane owns
//    (pixel, 8 channels): operand loads and stores are 16 B per lane, 8 lanes per
//    128-B line.
// One 512-thread block per CU (158 KB LDS): a 16 x 16 pixel x 64 channel output
// tile per work item; 4 compute waves (4 rows x 4 channel fragments each: per
// 32-channel sub-stage 144 v_mfma_f32_16x16x32_bf16 per wave, 2304 MFMA cycles)
// and 4 loader waves that issue all LDS-DMA (~58 KB of whole lines per
// sub-stage, ~1.1k cycles at 54 B/clk/CU) and own the epilogue.  The grid is
// persistent (one block per CU, a multiple of the output-channel blocks): the
// next item's first super-chunk and weights stage under this item's last
// sub-stage, its epilogue runs beside the next item's first sub-stage; BN sums
// are kept per thread across items and committed once.  Epilogue flags
// (bias / fold / addend / fused BN backward / statistics) are a template
// argument for the training-step combinations (EP_*), so the epilogue has no
// per-item branches and reads its per-channel constants once.
//
// LDS: H0 | W0 | W1 | H1 | constants.  Sub-stage t of a tile reads panel t & 1
// of halo H[(t >> 1) & 1] and weights W[t & 1]; C / 64 is even, so every tile
// starts on H0 / W0 and ends on W1 / H1, which the epilogue then uses as its
// 64 KB transpose buffer while the next tile's first stage lands in H0 / W0.
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace unet {

void conv_kernel_tag(const char* tag);  // conv_kernels.hip: per-launch profiler column

namespace {

// 4 compute waves (MFMA + epilogue) and 4 loader waves (all LDS-DMA): a wave
// that issues LDS-DMA pays ~100-200 cycles per instruction beside its MFMAs
// (MI355X_MICROARCH.md, LDS-DMA piece issue cost; the all-waves-issue form of
// this kernel measured 3.7-5.3k cycles per sub-stage against 2.3k of MFMA,
// profiles/r05/s1), and a compute wave that issues none keeps every load it
// makes visible to the compiler's waitcnt pass.  One compute and one loader
// wave per SIMD.
constexpr int kNC = 4, kNL = 4, kNW = kNC + kNL, kCOT = 64, kRW = 4, kFN = 4, kTH = 16;
constexpr int kHW = 18;                       // halo width
constexpr int kHPix = (kTH + 2) * kHW;        // 324 halo pixels
constexpr int kHIns = (kHPix + 7) / 8;        // 41 DMA instructions of 8 x 128 B
constexpr int kHBytes = kHIns * 1024;         // 41,984
constexpr int kWIns = 9 * kCOT / 16;          // 36 DMA instructions of 16 x 64 B
constexpr int kWBytes = kWIns * 1024;         // 36,864
constexpr int kOffH0 = 0, kOffW0 = kHBytes, kOffW1 = kOffW0 + kWBytes, kOffH1 = kOffW1 + kWBytes;
constexpr int kOffCst = kOffH1 + kHBytes;     // 157,696
constexpr int kNCst = 5;                      // bias|shift', scale|mean, invstd, mean2, invstd2
constexpr int kLds = kOffCst + kNCst * kCOT * 4;
static_assert(kLds <= 163840, "LDS");
static_assert(256 * 256 <= kWBytes + kHBytes, "transpose buffer fits W1 | H1");
static_assert(kTH == kNC * kRW, "rows");
constexpr int kItems = 4;  // epilogue items (pixel, 8 channels): 2 x 4 per loader thread
constexpr int kWPer = kWIns / kNL;                         // 9 weight DMA per loader wave
constexpr int kHPer = (kHIns + kNL - 1) / kNL;             // <= 11 halo DMA per loader wave
static_assert(kWIns % kNL == 0, "weight DMA per loader");

__device__ __forceinline__ int fl_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 6)) << 4); }
__device__ __forceinline__ int ws_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 1) & 2)) << 4); }
// transpose buffer [256 px][64 f32]: 16-B chunk c of pixel px at c ^ (px & 15)
// (conflict-free for the accumulator writes and the (pixel, 8-channel) reads)
__device__ __forceinline__ int tp_off(int px, int c16) { return px * 256 + ((c16 ^ (px & 15)) << 4); }

__device__ __forceinline__ void wait_vm_h(int n) {  // loader: all but its n halo DMA of the sub-stage
  if (n == 11) wait_vmcnt<11>();
  else wait_vmcnt<10>();
}
__device__ __forceinline__ void barrier_lds() {  // this wave's LDS reads/writes done, then the barrier
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

}  // namespace

// Epilogue flags (a template argument, so the epilogue of the hot variants has
// no per-item branches): EP_RT = read them from the arguments instead
constexpr int EP_FOLD = 1, EP_ADD = 2, EP_FBWD = 4, EP_STATS = 8, EP_RELU = 16, EP_RT = 32;

__device__ __forceinline__ void fl_ld8(const float* p, float (&d)[8]) {
  const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
  d[0] = x0[0]; d[1] = x0[1]; d[2] = x0[2]; d[3] = x0[3]; d[4] = x1[0]; d[5] = x1[1]; d[6] = x1[2]; d[7] = x1[3];
}

// One epilogue item: 8 channels q8 .. q8 + 7 of pixel slot px (transpose
// buffer T) / global pixel pix -- bias or eval fold, addend, ReLU mask of the
// fused BN backward, bf16 store, BN sums (register accumulators s0 / s1 / s2)
template <bool FLIP, bool TWO>
__device__ __forceinline__ void fl_item(const ConvFwdArgs& a, const char* T, const float* cst, const float (&kb)[8],
                                        const float (&km)[8], const float (&mu)[8], const float (&is)[8], int q8, int px,
                                        int pix, int cob, bool fold, bool want_add, bool fbwd, bool stats,
                                        bool relu, const uint4& uadd, const uint4& uact, const uint4& uy,
                                        const uint4& uy2, float (&s0)[8], float (&s1)[8], float (&s2)[8]) {
  const f32x4 lo = *reinterpret_cast<const f32x4*>(T + tp_off(px, 2 * (q8 >> 3)));
  const f32x4 hi = *reinterpret_cast<const f32x4*>(T + tp_off(px, 2 * (q8 >> 3) + 1));
  float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  float kb_[8];  // TWO: per item from LDS (registers)
  if (TWO) fl_ld8(cst + q8, kb_);
  if (fold) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] * km[e] + kb[e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += TWO ? kb_[e] : kb[e];
  }
  if (want_add) {
    float ad[8];
    unpack8(uadd, ad);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += ad[e];
  }
  if (!FLIP && relu) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  if (fbwd) {
    float m[8];
    unpack8(uact, m);
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (!(m[e] > 0.f)) v[e] = 0.f;
  }
  const uint4 ob = pack8(v);
  if (UNET_ABL != 4) *reinterpret_cast<uint4*>(a.y + (size_t)pix * a.ldy + cob * kCOT + q8) = ob;
  if (fbwd) {  // sums of the stored bf16 dZ, as bn_bwd_reduce_kernel would read them
    float dz[8], yv[8];
    unpack8(ob, dz);
    unpack8(uy, yv);
    float mu_[8], is_[8];  // TWO: per item from LDS (registers)
    if (TWO) {
      fl_ld8(cst + kCOT + q8, mu_);
      fl_ld8(cst + 2 * kCOT + q8, is_);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      s0[e] += dz[e];
      s1[e] += dz[e] * (yv[e] - (TWO ? mu_[e] : mu[e])) * (TWO ? is_[e] : is[e]);
    }
    if constexpr (TWO) {
      float y2[8];
      unpack8(uy2, y2);
      const f32x4 n0 = *reinterpret_cast<const f32x4*>(cst + 3 * kCOT + q8);
      const f32x4 n1 = *reinterpret_cast<const f32x4*>(cst + 3 * kCOT + q8 + 4);
      const f32x4 j0 = *reinterpret_cast<const f32x4*>(cst + 4 * kCOT + q8);
      const f32x4 j1 = *reinterpret_cast<const f32x4*>(cst + 4 * kCOT + q8 + 4);
      const float mu2[8] = {n0[0], n0[1], n0[2], n0[3], n1[0], n1[1], n1[2], n1[3]};
      const float is2[8] = {j0[0], j0[1], j0[2], j0[3], j1[0], j1[1], j1[2], j1[3]};
#pragma unroll
      for (int e = 0; e < 8; ++e) s2[e] += dz[e] * (y2[e] - mu2[e]) * is2[e];
    }
  } else if (stats) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { s0[e] += v[e]; s1[e] += v[e] * v[e]; }
  }
}

// FLIP: data gradient (dgrad pack, taps mirrored); TWO: two-BN fused backward
// epilogue (downsample blocks); grid = persistent slots, work item = spatial
// tile * ncb + output-channel block.
//
// Roles and barriers.  Per item both roles pass B_0 .. B_{NSUB-1} (sub-stage s
// may start) and F (every compute wave is done reading W1 / H1); after the
// last item one more barrier Z.  Compute waves: MFMAs of sub-stage s after
// B_s; after F they write their accumulators to the transpose buffer T (W1 |
// H1) and go on to the next item's B_0.  Loader waves: before B_s they wait
// for sub-stage s's DMA and after it issue the next one; they own the whole
// epilogue: its operands are fetched at B_{NSUB-1} (after the next item's
// DMA, which B_0 then waits for alone), and the epilogue of item i runs right
// after the next item's B_0 -- beside that item's first sub-stage, which reads
// only W0 / H0 -- or after Z; only then do they refill W1 / H1 (= T).
template <bool FLIP, bool TWO, int EP>
__global__ void __launch_bounds__(kNW * 64) conv3x3_fl_kernel(ConvFwdArgs a, int ncb, int nitems) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cst = reinterpret_cast<float*>(smem + kOffCst);
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slot = xcd_remap(blockIdx.x, gridDim.x);
  int item = slot;
  if (item >= nitems) return;
  const int tq = a.Q >> 4, tp = a.P / kTH;
  const int NSUB = a.C >> 5;  // 32-channel sub-stages per item (even)
  constexpr bool RT = EP & EP_RT;
  const bool fbwd = RT ? FLIP && a.bb.sums != nullptr : (EP & EP_FBWD) != 0;
  const bool stats = RT ? a.stats != nullptr || fbwd : (EP & EP_STATS) != 0;
  const bool fold = RT ? !FLIP && a.fold_on : (EP & EP_FOLD) != 0;
  const bool want_add = RT ? a.add != nullptr : (EP & EP_ADD) != 0;
  const bool relu = RT ? a.fold_relu != 0 : (EP & EP_RELU) != 0;
  const int cob = item % ncb;  // fixed per block: gridDim % ncb == 0 (launcher)

  if (wave < kNC) {
    // ================= compute waves: MFMAs, accumulators to T =================
    const int aoff = ws_off(lane & 15, lane >> 4);
    int boff[kRW + 2][3];
#pragma unroll
    for (int h = 0; h < kRW + 2; ++h)
#pragma unroll
      for (int d = 0; d < 3; ++d) boff[h][d] = fl_off((wave * kRW + h) * kHW + d + (lane & 15), lane >> 4);
    TSTAMP(a.tim, 1);
    int stg = 0;
    for (;;) {
      f32x4 acc[kRW][kFN];
#pragma unroll
      for (int j = 0; j < kRW; ++j)
#pragma unroll
        for (int i = 0; i < kFN; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s = 0; s < NSUB; ++s, ++stg) {
        barrier_lds();  // B_s: the loaders have waited for sub-stage s
        if (stg < 16) TSTAMP(a.tim, 2 + stg);
        const char* W = smem + ((s & 1) ? kOffW1 : kOffW0);
        const char* H = smem + (((s >> 1) & 1) ? kOffH1 : kOffH0);
        const int pb = (s & 1) << 6;  // panel: byte offset ^ 64
        if (UNET_ABL == 1) continue;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            bf16x8 A[kFN];
#pragma unroll
            for (int i = 0; i < kFN; ++i)
              A[i] = *reinterpret_cast<const bf16x8*>(W + ((r * 3 + c) * kCOT + i * 16) * 64 + aoff);
            const int dr = FLIP ? 2 - r : r, dc = FLIP ? 2 - c : c;
#pragma unroll
            for (int j = 0; j < kRW; ++j) {
              const bf16x8 B = *reinterpret_cast<const bf16x8*>(H + (boff[j + dr][dc] ^ pb));
#pragma unroll
              for (int i = 0; i < kFN; ++i)
                acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B, acc[j][i], 0, 0, 0);
            }
          }
      }
      TSTAMP(a.tim, 20);
      barrier_lds();  // F: every compute wave is done reading W1 / H1
      char* T = smem + kOffW1;
#pragma unroll
      for (int j = 0; j < kRW; ++j)
#pragma unroll
        for (int i = 0; i < kFN; ++i) {
          const int px = (wave * kRW + j) * 16 + (lane & 15);
          *reinterpret_cast<f32x4*>(T + tp_off(px, i * 4 + (lane >> 4))) = acc[j][i];
        }
      item += gridDim.x;
      if (item >= nitems) break;
    }
    barrier_lds();  // Z: T holds the last item
    if (stats) {  // the loaders' reduction barriers
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_s_barrier();
      const unsigned* tk = fbwd ? a.bb.ticket : a.bn.ticket;
      if (tk) {
        int* flag = reinterpret_cast<int*>(smem + kOffH0 + 32 * kCOT * 3 * sizeof(float));
        if (last_block_arrive(const_cast<unsigned*>(tk), gridDim.x, flag, false)) {
          if (fbwd) bn_bwd_finalize(a.bb);
          else bn_finalize(a.bn);
        }
      }
    }
    return;
  }

  // ================= loader waves: all LDS-DMA (inline asm, glds16_asm: hipcc's
  // waitcnt pass would otherwise drain the halo still in flight) + epilogue =====
  const int lw = wave - kNC, lt = tid - kNC * 64;
  const int nh = (kHIns - lw + kNL - 1) / kNL;  // 11 or 10
  const i32x4 xr = make_rsrc_sgpr(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const i32x4 wr = make_rsrc_sgpr(a.wch, (unsigned)((size_t)a.C * 9 * a.Cout * 2));
  unsigned woff[kWPer], hoff[kHPer];
#pragma unroll
  for (int k = 0; k < kWPer; ++k) {
    const int ins = lw + k * kNL;
    const int tap = ins >> 2, co = (ins & 3) * 16 + (lane >> 2);
    const int lch = (lane & 3) ^ ((co >> 1) & 2);
    woff[k] = (unsigned)(((tap * a.Cout + cob * kCOT + co) * 32 + lch * 8) * 2);
  }
  auto set_hoff = [&](int it) {
    const int t = it / ncb;
    const int n = t / (tp * tq), rem = t - n * (tp * tq);
    const int oh0 = (rem / tq) * kTH, ow0 = (rem % tq) << 4;
#pragma unroll
    for (int k = 0; k < kHPer; ++k) {
      const int hp = (lw + k * kNL) * 8 + (lane >> 3);
      const int hr = hp / kHW, hc = hp - hr * kHW;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      const int q = (lane & 7) ^ (hp & 6);
      hoff[k] = kOOB;
      if (hp < kHPix && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        hoff[k] = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + q * 8) * 2);
    }
  };
  auto issue_w = [&](int t, int b) {  // sub-stage t's weights (32 channels, 9 taps) into W[b]
    char* dst = smem + (b ? kOffW1 : kOffW0);
    const unsigned so = (unsigned)t * 9u * (unsigned)a.Cout * 64u;
#pragma unroll
    for (int k = 0; k < kWPer; ++k) glds16_asm(wr, dst + (lw + k * kNL) * 1024, woff[k], so);
  };
  auto issue_h = [&](int sc, int b) {  // super-chunk sc's halo (64 channels) into H[b]
    char* dst = smem + (b ? kOffH1 : kOffH0);
    const unsigned so = (unsigned)sc * 128u;
#pragma unroll
    for (int k = 0; k < kHPer; ++k)
      if (k < nh) glds16_asm(xr, dst + (lw + k * kNL) * 1024, hoff[k], so);
  };
  [[maybe_unused]] constexpr int LT = kNC * 64;  // the loader thread that stamps (timing build)
  set_hoff(item);
  TSTAMP_TH(a.tim, 23, LT);
  issue_w(0, 0);
  issue_h(0, 0);
  TSTAMP_TH(a.tim, 24, LT);
  if (lt < kCOT) {  // per-channel epilogue constants of the block's output channels
    const int c = lt, co = cob * kCOT + c;
    float b = a.bias ? a.bias[co] : 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f, c4 = 0.f;
    if (fold) {
      float sc, sh, m, is, var;
      bn_scale_shift(a.fold, co, sc, sh, m, is, var);
      b = b * sc + sh;
      c1 = sc;
    } else if (fbwd) {
      c1 = a.bb.mean[co];
      c2 = a.bb.invstd[co];
      if (TWO) { c3 = a.bb.mean2[co]; c4 = a.bb.invstd2[co]; }
    }
    cst[c] = b; cst[kCOT + c] = c1; cst[2 * kCOT + c] = c2; cst[3 * kCOT + c] = c3; cst[4 * kCOT + c] = c4;
  }
  // epilogue: loader wave lw owns the pixels px with (px >> 2) & 3 == lw -- the
  // T rows in the 1-KB stripes that its own DMA refills (stripe = px >> 2,
  // DMA instructions lw + 4 k of W1 and H1, T = W1 | H1), so no other wave's
  // DMA can overwrite a row it has not read yet; lane l owns channels
  // 8 (l & 7) .. + 7 of pixel slot j = (l >> 3) + 8 k (k < 8), 4 consecutive
  // pixels per 512 B
  const int q8 = (lane & 7) * 8;
  auto px_of = [&](int k) {
    const int j = (lane >> 3) + 8 * k;
    return 16 * (j >> 2) + 4 * lw + (j & 3);
  };
  float s0[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = s2[e] = 0.f;
  constexpr int NI = 2 * kItems;  // 8 items per loader thread
  // items whose operands are prefetched at B_{NSUB-1}: all but for the
  // dgrad without addend, where half (the rest issued by the epilogue itself)
  // keeps the loader in registers (measured, profiles/r05/s2 conv_timing*)
  // (round 6: the half prefetch of the FBWD-without-addend instance produced
  // wrong BN-backward sums -- sum dZ * xhat came out 0 -- caught by
  // tests/test_conv_fl_gpu.py; every instance now prefetches all NI items)
  // two-BN epilogue (TWO): no prefetch -- its four operands per item (addend,
  // mask, y, y2) for 8 items held across the sub-stage loop pushed the loader
  // waves into scratch, and that instance produced wrong BN-backward sums; it
  // now loads each group of 4 items' operands inside the epilogue
  constexpr int NP = TWO ? 0 : NI;
  int ep_pix0 = 0;                 // the pending epilogue's tile origin pixel (N * P * Q < 2^31: launcher)
  auto pix_of = [&](int k) {
    const int px = px_of(k);
    return ep_pix0 + (px >> 4) * a.Q + (px & 15);
  };
  // operands of item k (k >= NP: issued by the epilogue itself, where nothing
  // else is in flight, so the compiler's own waits are exact)
  auto load_ops = [&](int k, uint4& oa, uint4& om, uint4& oy, uint4& oy2) {
    const size_t pp = (size_t)pix_of(k);
    const int co = cob * kCOT + q8;
    oa = want_add ? *reinterpret_cast<const uint4*>(a.add + pp * a.ldadd + co) : make_uint4(0, 0, 0, 0);
    om = fbwd ? *reinterpret_cast<const uint4*>(a.bb.act + pp * a.bb.ldact + co) : make_uint4(0, 0, 0, 0);
    oy = fbwd ? *reinterpret_cast<const uint4*>(a.bb.y + pp * a.bb.ldy + co) : make_uint4(0, 0, 0, 0);
    if constexpr (TWO) oy2 = fbwd ? *reinterpret_cast<const uint4*>(a.bb.y2 + pp * a.bb.ldy2 + co) : make_uint4(0, 0, 0, 0);
    else oy2 = make_uint4(0, 0, 0, 0);
  };
  constexpr int NPA = NP > 0 ? NP : 1;
  uint4 opa[NPA], opm[NPA], opy[NPA], opy2[TWO ? NPA : 1];
  // the epilogue of the item whose accumulators are in T (items < NP: operands
  // prefetched)
  auto epilogue = [&]() {
    // the thread's channel constants, once per epilogue (mu / is unused by TWO,
    // zeroed so that no path reads an uninitialised register)
    float kb[8], km[8], mu[8], is[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) kb[e] = km[e] = mu[e] = is[e] = 0.f;
    if (!TWO) fl_ld8(cst + q8, kb);
    if (fold) fl_ld8(cst + kCOT + q8, km);
    if (fbwd && !TWO) {
      fl_ld8(cst + kCOT + q8, mu);
      fl_ld8(cst + 2 * kCOT + q8, is);
    }
    if constexpr (NP > 0) {
#pragma unroll
      for (int k = 0; k < NI; ++k) {
        fl_item<FLIP, TWO>(a, smem + kOffW1, cst, kb, km, mu, is, q8, px_of(k), pix_of(k), cob, fold, want_add, fbwd,
                           stats, relu, opa[k], opm[k], opy[k], opy2[TWO ? k : 0], s0, s1, s2);
        asm volatile("" ::: "memory");  // one item at a time: bounded registers
      }
    } else {
      // groups of G items: their operand loads all in flight, then the items
      constexpr int G = 4;
#pragma unroll
      for (int k0 = 0; k0 < NI; k0 += G) {
        uint4 la[G], lm[G], ly[G], ly2[G];
#pragma unroll
        for (int k = 0; k < G; ++k) load_ops(k0 + k, la[k], lm[k], ly[k], ly2[k]);
#pragma unroll
        for (int k = 0; k < G; ++k) {
          fl_item<FLIP, TWO>(a, smem + kOffW1, cst, kb, km, mu, is, q8, px_of(k0 + k), pix_of(k0 + k), cob, fold,
                             want_add, fbwd, stats, relu, la[k], lm[k], ly[k], ly2[k], s0, s1, s2);
          asm volatile("" ::: "memory");
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's T rows are read before its DMA refills them
  };
  // prefetched epilogue operand loads per thread: with the half prefetch they
  // are issued AFTER the next item's first-stage DMA, so that B_0 waits for
  // that DMA alone (vmcnt <= NOPS); with the full prefetch (more registers,
  // spills whose reloads wait for vmcnt(0) anyway) before it, and B_0 waits for
  // everything (measured both ways per variant, profiles/r05/s2 conv_timing*)
  constexpr int NOPS = (RT || NP == NI) ? -1 : NP * (((EP & EP_ADD) ? 1 : 0) + ((EP & EP_FBWD) ? (TWO ? 3 : 2) : 0));
  auto fetch_operands = [&]() {
#pragma unroll
    for (int k = 0; k < NP; ++k) load_ops(k, opa[k], opm[k], opy[k], opy2[TWO ? k : 0]);
  };
  (void)opa; (void)opm; (void)opy; (void)opy2;
  bool pending = false;  // an epilogue waits for the next B_0 / Z
  int nit = 0;             // items done (timing stamps of the first two)
  for (;;) {
    const int next = item + gridDim.x;
    // s = 0 (peeled): this sub-stage's DMA landed (the previous item's
    // epilogue operands may still be in flight); then that epilogue, beside
    // this item's first sub-stage; then the refill of W1 / H1 (= T)
    if constexpr (NOPS > 0) {
      if (pending) wait_vmcnt<(NOPS > 0 ? NOPS : 0)>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    if (nit == 0) TSTAMP_TH(a.tim, 25, LT);
    if (nit == 1) TSTAMP_TH(a.tim, 27, LT);
    __builtin_amdgcn_s_barrier();  // B_0
    if (pending) epilogue();
    if (UNET_ABL != 2) {
      issue_w(1, 1);
      if (2 < NSUB) issue_h(1, 1);
    }
    // s = 1 .. NSUB - 2: at odd s all but the next super-chunk's halo (issued
    // after this sub-stage's weights) has landed; at even s everything
    for (int s = 1; s < NSUB - 1; ++s) {
      if (s & 1) wait_vm_h(nh);
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // B_s: sub-stage s - 1 is no longer read
      if (UNET_ABL != 2) {
        issue_w(s + 1, (s + 1) & 1);
        if (!(s & 1) && s + 2 < NSUB) issue_h((s >> 1) + 1, ((s >> 1) + 1) & 1);
      }
    }
    // s = NSUB - 1 (peeled): everything landed; this item's epilogue operands
    // (whole lines), then the next item's first stage (H0 / W0 are free)
    wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();  // B_{NSUB-1}
    {
      const int t = item / ncb;
      const int n = t / (tp * tq), rem = t - n * (tp * tq);
      const int oh0 = (rem / tq) * kTH, ow0 = (rem % tq) << 4;
      ep_pix0 = (n * a.P + oh0) * a.Q + ow0;
    }
    if constexpr (NOPS < 0) fetch_operands();
    if (nit == 0) TSTAMP_TH(a.tim, 26, LT);
    ++nit;
    if (next < nitems) {
      set_hoff(next);
      issue_w(0, 0);
      issue_h(0, 0);
    }
    if constexpr (NOPS >= 0) fetch_operands();
    __builtin_amdgcn_s_barrier();  // F
    pending = true;
    item = next;
    if (item >= nitems) break;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // Z: T holds the last item
  TSTAMP_TH(a.tim, 28, LT);
  epilogue();
  TSTAMP_TH(a.tim, 21, LT);
  if (!stats) {
    TSTAMP_RT_TH(a.tim, 31, LT);
    return;
  }
  // ---- BN sums: [32 pixel slots][64 channels][3] in H0 (no DMA in flight any
  // more), summed over the slots in a fixed order (4 independent partial sums),
  // fp64 atomics into replica blockIdx % kStatRep ----
  float* red = reinterpret_cast<float*>(smem + kOffH0);
  {
    const int sl = lt >> 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(sl * kCOT + q8 + e) * 3 + 0] = s0[e];
      red[(sl * kCOT + q8 + e) * 3 + 1] = s1[e];
      red[(sl * kCOT + q8 + e) * 3 + 2] = s2[e];
    }
  }
  barrier_lds();  // R1
  if (lt < (TWO ? 3 : 2) * kCOT) {
    const int c = lt % kCOT, which = lt / kCOT;
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int sl = 0; sl < 32; ++sl) p[sl & 3] += red[(sl * kCOT + c) * 3 + which];
    const float tsum = (p[0] + p[1]) + (p[2] + p[3]);
    const int co = cob * kCOT + c;
    const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout;
    if (which == 2) atomicAdd(a.bb.sums2 + rep + a.Cout + co, (double)tsum);
    else atomicAdd((fbwd ? a.bb.sums : a.stats) + rep + which * a.Cout + co, (double)tsum);
  }
  __builtin_amdgcn_s_barrier();  // R2
  const unsigned* tk = fbwd ? a.bb.ticket : a.bn.ticket;
  if (tk) {
    int* flag = reinterpret_cast<int*>(smem + kOffH0 + 32 * kCOT * 3 * sizeof(float));
    if (last_block_arrive(const_cast<unsigned*>(tk), gridDim.x, flag, lt < 3 * kCOT)) {
      if (fbwd) bn_bwd_finalize(a.bb);
      else bn_finalize(a.bn);
    }
  }
  TSTAMP_TH(a.tim, 22, LT);
  TSTAMP_RT_TH(a.tim, 31, LT);
}

static int cu_count() { return device_cu_count(); }

// shapes the kernel covers AND fills: at least one 16 x 16 x 64 work item per
// CU (enc4 at 512^2 has 128: it stays on the 32-channel halo-streamed kernel)
bool conv3x3_fl_geom(int C, int Cout, int P, int Q) {
  return C > 0 && Cout > 0 && P > 0 && Q > 0 && C % 128 == 0 && Cout % kCOT == 0 && P % kTH == 0 && Q % 16 == 0;
}

bool conv3x3_fl_shape(int N, int C, int Cout, int P, int Q) {
  static const bool off = std::getenv("UNET_NO_FL") != nullptr;  // A/B: the halo-streamed kernel
  if (off || !conv3x3_fl_geom(C, Cout, P, Q)) return false;
  return (long long)N * (P / kTH) * (Q / 16) * (Cout / kCOT) >= cu_count();
}

// a.wch: the chunk-major weight pack (PK_CONV_FWD_CH / PK_CONV_DGRAD_CH)
hipError_t launch_conv3x3_fl(const ConvFwdArgs& a, int mode, hipStream_t st) {
  const bool flip = mode == 1;
  if (!a.wch || a.R != 3 || a.S != 3 || a.stride != 1 || a.pad != 1 || a.x2 || a.ysplit || a.xform)
    return hipErrorInvalidValue;
  if (a.N <= 0 || a.H != a.P || a.W != a.Q || !conv3x3_fl_geom(a.C, a.Cout, a.P, a.Q)) return hipErrorInvalidValue;
  if (a.ldx % 8 || a.ldy % 8 || (a.add && a.ldadd % 8)) return hipErrorInvalidValue;
  if (flip && (a.fold_on || a.stats || (a.bb.sums && (a.bb.ldact % 8 || a.bb.ldy % 8 ||
                                                     (a.bb.y2 && a.bb.ldy2 % 8)))))
    return hipErrorInvalidValue;
  if (!flip && a.bb.sums) return hipErrorInvalidValue;
  if ((size_t)a.N * a.H * a.W * a.ldx * 2 >= 0x80000000ull || (size_t)a.C * 9 * a.Cout * 2 >= 0x80000000ull ||
      (size_t)a.N * a.P * a.Q >= 0x80000000ull)
    return hipErrorInvalidValue;
  const int ncb = a.Cout / kCOT;
  const int nitems = a.N * (a.P / kTH) * (a.Q / 16) * ncb;
  // persistent grid: one block per CU, a multiple of ncb so that every block
  // keeps one output-channel block
  int grid = cu_count() / ncb * ncb;
  if (a.grid_cap > 0 && a.grid_cap < grid) grid = a.grid_cap / ncb * ncb;
  if (grid < ncb) grid = ncb;
  if (grid > nitems) grid = nitems;
  const bool two = flip && a.bb.sums && a.bb.y2;
  const bool fbwd = flip && a.bb.sums;
  const int ep = (!flip && a.fold_on ? EP_FOLD : 0) | (a.add ? EP_ADD : 0) | (fbwd ? EP_FBWD : 0) |
                 (a.stats || fbwd ? EP_STATS : 0) | (!flip && a.fold_relu ? EP_RELU : 0);
  // the training-step epilogues as their own instances, anything else reads
  // its flags at run time
  int sel = EP_RT;
  if (!flip && (ep == EP_STATS || ep == 0)) sel = ep;
  if (flip && !two && (ep == 0 || ep == EP_ADD || ep == (EP_FBWD | EP_STATS) || ep == (EP_FBWD | EP_STATS | EP_ADD)))
    sel = ep;
  // (two: the run-time instance -- the specialised ones spill heavily)
  char tag[96];
  std::snprintf(tag, sizeof(tag), "conv3x3_fl_kernel<%s, %s, %d>", flip ? "true" : "false", two ? "true" : "false",
                sel);
  conv_kernel_tag(tag);
  const dim3 g(grid), b(kNW * 64);
#define FL_LAUNCH(F, T, E) hipLaunchKernelGGL((conv3x3_fl_kernel<F, T, E>), g, b, kLds, st, a, ncb, nitems)
  if (!flip) {
    if (sel == EP_STATS) FL_LAUNCH(false, false, EP_STATS);
    else if (sel == 0) FL_LAUNCH(false, false, 0);
    else FL_LAUNCH(false, false, EP_RT);
  } else if (two) {
    FL_LAUNCH(true, true, EP_RT);
  } else {
    if (sel == (EP_FBWD | EP_STATS)) FL_LAUNCH(true, false, EP_FBWD | EP_STATS);
    else if (sel == (EP_FBWD | EP_STATS | EP_ADD)) FL_LAUNCH(true, false, EP_FBWD | EP_STATS | EP_ADD);
    else if (sel == EP_ADD) FL_LAUNCH(true, false, EP_ADD);
    else if (sel == 0) FL_LAUNCH(true, false, 0);
    else FL_LAUNCH(true, false, EP_RT);
  }
#undef FL_LAUNCH
  return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Weight-stationary full-line conv for C == 64 (enc1 and decoder2.3 at Base,
// SURVEY.md §8(a) rows a3 / a6): the same roles as conv3x3_fl_kernel, with the
// block's 9 x 64 x 64 weights loaded ONCE (the conv3x3_ws_kernel layout: one
// 128-B fl_off row per (tap, output channel), from the standard pack) and only
// the 16 x 16 tiles' halos streamed, double-buffered.  The weight-stationary
// kernel before it ran MFMA, epilogue, halo issue and barrier one after the
// other in every wave (profiles/r05/s2 conv_timing_abl3: 4.2k MFMA cycles of a
// 10.9k-cycle tile); here the loader waves stage the next halo and write the
// previous tile's outputs while the compute waves run the current tile's MFMAs.
//
// Per tile: compute waves (4 rows x 4 channel fragments each, 288 MFMAs) add
// the bias (forward: BN sums from the fp32 values, in registers) or the
// addend (data gradient, loaded by the compute wave itself), round to bf16
// and write the 256 x 64 bf16 tile T into the halo buffer they just consumed;
// the loader waves then store T as whole lines (data gradient with fused BN
// backward: ReLU mask and the BN-backward sums there) and refill that buffer
// with the halo of the tile after next.  Loader wave lw reads only the T rows
// of the 1-KB stripes its own DMA refills (stripe = px >> 3, (px >> 3) & 3 ==
// lw), so no cross-wave hazard exists on the refill.
// LDS: W (73,728) | H0 | H1 (41,984 each) | constants.
constexpr int kW2Bytes = 9 * kCOT * 128;
constexpr int k2OffH0 = kW2Bytes, k2OffH1 = k2OffH0 + kHBytes, k2OffCst = k2OffH1 + kHBytes;
constexpr int k2OffXss = k2OffCst + 3 * kCOT * 4;  // xform: scale | shift of the 64 input channels
constexpr int k2Lds = k2OffXss + 2 * 64 * 4;
constexpr int EP_XF = 64;  // ws2 only: the previous BN + ReLU applied to the staged halo (ConvFwdArgs::xform)
static_assert(k2Lds <= 163840, "LDS");
static_assert(256 * 128 <= kHBytes, "bf16 tile fits a halo buffer");
__device__ __forceinline__ int t2_off(int px, int c16) { return px * 128 + ((c16 ^ (px & 7)) << 4); }

// items q0 .. q1 - 1 of one wave's share of a bf16 tile T: item q = stripe
// sw + 4 q (8 pixels x 128 B), lane = (pixel (lane >> 3), 8 channels
// c8 = 8 (lane & 7)); stores whole lines; FBWD: ReLU mask of the BN whose
// backward is fused and its sums (s0, s1) from the stored bf16 dZ
// (TV: the T values were read before -- tv[q - Q0] -- so that the buffer could
// be refilled in between)
template <bool FBWD, int Q0, int Q1, bool TV = false>
__device__ __forceinline__ void ws2_items(const ConvFwdArgs& a, const char* T, int cob, int pix0, int sw, int lane,
                                          const float (&mu)[8], const float (&is)[8], float (&s0)[8],
                                          float (&s1)[8], const uint4* tv = nullptr) {
  const int c8 = (lane & 7) * 8;
  uint4 om[Q1 - Q0], oy[Q1 - Q0];
  if constexpr (FBWD) {
#pragma unroll
    for (int q = Q0; q < Q1; ++q) {
      const int px = (sw + 4 * q) * 8 + (lane >> 3);
      const size_t gp = (size_t)(pix0 + (px >> 4) * a.Q + (px & 15));
      om[q - Q0] = *reinterpret_cast<const uint4*>(a.bb.act + gp * a.bb.ldact + cob * kCOT + c8);
      oy[q - Q0] = *reinterpret_cast<const uint4*>(a.bb.y + gp * a.bb.ldy + cob * kCOT + c8);
    }
  }
#pragma unroll
  for (int q = Q0; q < Q1; ++q) {
    const int px = (sw + 4 * q) * 8 + (lane >> 3);
    const size_t gp = (size_t)(pix0 + (px >> 4) * a.Q + (px & 15));
    uint4 o = TV ? tv[q - Q0] : *reinterpret_cast<const uint4*>(T + t2_off(px, lane & 7));
    if constexpr (FBWD) {
      float v[8], m[8], yv[8];
      unpack8(o, v);
      unpack8(om[q - Q0], m);
      unpack8(oy[q - Q0], yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (!(m[e] > 0.f)) v[e] = 0.f;
        s0[e] += v[e];
        s1[e] += v[e] * (yv[e] - mu[e]) * is[e];
      }
      o = pack8(v);
    }
    if (UNET_ABL != 4) *reinterpret_cast<uint4*>(a.y + gp * a.ldy + cob * kCOT + c8) = o;
  }
}

template <bool FLIP, int EP>
__global__ void __launch_bounds__(kNW * 64) conv3x3_ws2_kernel(ConvFwdArgs a, int ncb, int nitems) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cst = reinterpret_cast<float*>(smem + k2OffCst);  // bias | mean | invstd
  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slot = xcd_remap(blockIdx.x, gridDim.x);
  if (slot >= nitems) return;
  const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout;  // BN-sum replica of the block
  const int cob = slot % ncb;  // fixed per block: gridDim % ncb == 0 (launcher)
  const int tq = a.Q >> 4, tp = a.P / kTH;
  constexpr bool FBWD = FLIP && (EP & EP_FBWD), ADD = (EP & EP_ADD) != 0, STATS = (EP & EP_STATS) != 0;
  constexpr bool XF = !FLIP && (EP & EP_XF);
  float* xss = reinterpret_cast<float*>(smem + k2OffXss);
  auto tile_pix0 = [&](int it) {  // global pixel of the item's tile origin
    const int t = it / ncb;
    const int n = t / (tp * tq), rem = t - n * (tp * tq);
    return (n * a.P + (rem / tq) * kTH) * a.Q + ((rem % tq) << 4);
  };
  const char* Wl = smem;

  if (wave < kNC) {
    // ================= compute waves =================
    const int aoff = fl_off(lane & 15, lane >> 4), g = lane >> 4;
    int boff[kRW + 2][3];
#pragma unroll
    for (int h = 0; h < kRW + 2; ++h)
#pragma unroll
      for (int d = 0; d < 3; ++d) boff[h][d] = fl_off((wave * kRW + h) * kHW + d + (lane & 15), lane >> 4);
    float q0[kFN][4], q1[kFN][4];
#pragma unroll
    for (int i = 0; i < kFN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = 0.f;
    if constexpr (XF) {
      if (blockIdx.x == 0) bn_finalize(a.xbn);  // saved mean / invstd, running statistics (wave 0)
      __builtin_amdgcn_s_barrier();             // X: the loaders' scale / shift table is in LDS
    }
    TSTAMP(a.tim, 1);
    int b = 0, k = 0;
    for (int it = slot; it < nitems; it += gridDim.x, b ^= 1, ++k) {
      const int pix0 = tile_pix0(it);
      __builtin_amdgcn_s_barrier();  // B: this tile's halo landed (the loaders waited)
      asm volatile("" ::: "memory");
      if (k < 8) TSTAMP(a.tim, 2 + 2 * k);
      uint2 uadd[kRW][kFN];
      if constexpr (ADD) {  // lands under the MFMAs
#pragma unroll
        for (int j = 0; j < kRW; ++j) {
          const int px = (wave * kRW + j) * 16 + (lane & 15);
          const size_t gp = (size_t)(pix0 + (px >> 4) * a.Q + (px & 15));
#pragma unroll
          for (int i = 0; i < kFN; ++i)
            uadd[j][i] = *reinterpret_cast<const uint2*>(a.add + gp * a.ldadd + cob * kCOT + i * 16 + 4 * g);
        }
        asm volatile("" ::: "memory");  // issued here, not sunk next to their use after the MFMAs
      }
      const char* H = smem + k2OffH0 + b * kHBytes;
      f32x4 acc[kRW][kFN];
#pragma unroll
      for (int j = 0; j < kRW; ++j)
#pragma unroll
        for (int i = 0; i < kFN; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (UNET_ABL != 1) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              bf16x8 A[kFN];
#pragma unroll
              for (int i = 0; i < kFN; ++i)
                A[i] = *reinterpret_cast<const bf16x8*>(Wl + (r * 3 + c) * kCOT * 128 + i * 2048 + (aoff ^ (p << 6)));
              const int dr = FLIP ? 2 - r : r, dc = FLIP ? 2 - c : c;
#pragma unroll
              for (int j = 0; j < kRW; ++j) {
                const bf16x8 B = *reinterpret_cast<const bf16x8*>(H + (boff[j + dr][dc] ^ (p << 6)));
#pragma unroll
                for (int i = 0; i < kFN; ++i)
                  acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B, acc[j][i], 0, 0, 0);
              }
            }
      }
      if (k < 8) TSTAMP(a.tim, 3 + 2 * k);
      barrier_lds();  // F: every compute wave is done reading H (it becomes T)
      char* T = smem + k2OffH0 + b * kHBytes;
#pragma unroll
      for (int i = 0; i < kFN; ++i) {
        float kb[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) kb[e] = cst[i * 16 + 4 * g + e];
#pragma unroll
        for (int j = 0; j < kRW; ++j) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[j][i][e] + kb[e];
          if constexpr (ADD) {
            const float ad[4] = {__uint_as_float(uadd[j][i].x << 16), __uint_as_float(uadd[j][i].x & 0xffff0000u),
                                 __uint_as_float(uadd[j][i].y << 16), __uint_as_float(uadd[j][i].y & 0xffff0000u)};
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += ad[e];
          }
          if constexpr (!FLIP && STATS) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { q0[i][e] += v[e]; q1[i][e] += v[e] * v[e]; }
          }
          const int px = (wave * kRW + j) * 16 + (lane & 15);
          *reinterpret_cast<uint2*>(T + t2_off(px, 2 * i + (g >> 1)) + (g & 1) * 8) =
              make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        }
      }
      barrier_lds();  // E: T written
    }
    TSTAMP(a.tim, 20);
    float es0[8], es1[8], emu[8], eis[8];  // the compute waves' share of the last tile's epilogue
#pragma unroll
    for (int e = 0; e < 8; ++e) es0[e] = es1[e] = 0.f;
    {
      const int ce8 = (lane & 7) * 8;
      if constexpr (FBWD) {
        fl_ld8(cst + kCOT + ce8, emu);
        fl_ld8(cst + 2 * kCOT + ce8, eis);
      }
      int lit = slot;  // the block's last item
      while (lit + (int)gridDim.x < nitems) lit += gridDim.x;
      ws2_items<FBWD, 4, 8>(a, smem + k2OffH0 + (b ^ 1) * kHBytes, cob, tile_pix0(lit), wave, lane, emu, eis, es0,
                            es1);
    }
    if constexpr (FBWD) {  // partials into slots 32 .. 63 of the loaders' sum table
      float* red = reinterpret_cast<float*>(smem + k2OffH0 + b * kHBytes);
      const int sl = 32 + (tid >> 3), ce8 = (lane & 7) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(sl * kCOT + ce8 + e) * 2 + 0] = es0[e];
        red[(sl * kCOT + ce8 + e) * 2 + 1] = es1[e];
      }
    }
    if constexpr (!FLIP && STATS) {
      // BN sums: per-lane partials to LDS (the halo buffer the last tile did NOT
      // use: free), summed in a fixed order by 128 threads
      float* red = reinterpret_cast<float*>(smem + k2OffH0 + b * kHBytes);  // b: the buffer after the last
#pragma unroll
      for (int i = 0; i < kFN; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[(wave * 64 + lane) * 32 + i * 4 + e] = q0[i][e];
          red[(wave * 64 + lane) * 32 + 16 + i * 4 + e] = q1[i][e];
        }
    }
    __builtin_amdgcn_s_barrier();  // R1
    __builtin_amdgcn_s_barrier();  // R2
    return;
  }

  // ================= loader waves: LDS-DMA, the tile stores, BN-backward sums =====
  const int lw = wave - kNC, lt = tid - kNC * 64;
  const int nh = (kHIns - lw + kNL - 1) / kNL;  // 11 or 10
  const i32x4 xr = make_rsrc_sgpr(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const i32x4 wr = make_rsrc_sgpr(a.w, (unsigned)((size_t)a.Cout * 9 * a.C * 2));
  [[maybe_unused]] constexpr int LT = kNC * 64;
  unsigned hoff[kHPer];
  auto set_hoff = [&](int it) {
    const int t = it / ncb;
    const int n = t / (tp * tq), rem = t - n * (tp * tq);
    const int oh0 = (rem / tq) * kTH, ow0 = (rem % tq) << 4;
#pragma unroll
    for (int k = 0; k < kHPer; ++k) {
      const int hp = (lw + k * kNL) * 8 + (lane >> 3);
      const int hr = hp / kHW, hc = hp - hr * kHW;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      const int q = (lane & 7) ^ (hp & 6);
      hoff[k] = kOOB;
      if (hp < kHPix && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        hoff[k] = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + q * 8) * 2);
    }
  };
  const unsigned l0 = lds_addr(smem);
  auto issue_h = [&](int bb) {
    const unsigned dst = l0 + k2OffH0 + bb * kHBytes;
#pragma unroll
    for (int k = 0; k < kHPer; ++k)
      if (k < nh) glds16_asm_at(xr, dst + (lw + k * kNL) * 1024, hoff[k], 0u);
  };
  if constexpr (XF) {  // the previous BN's scale / shift, before any DMA is in flight
    if (lt < 64) {
      float m, iv, var;
      bn_scale_shift(a.xbn, lt, xss[lt], xss[64 + lt], m, iv, var);
    }
  }
  // the weights, once: 72 instructions of 8 (tap, channel) rows x 128 B
  TSTAMP_TH(a.tim, 23, LT);
  for (int ins = lw; ins < 9 * kCOT / 8; ins += kNL) {
    const int row = ins * 8 + (lane >> 3);
    const int co = row % kCOT, tap = row / kCOT;
    const int q = (lane & 7) ^ (row & 6);
    const unsigned off = (unsigned)((((cob * kCOT + co) * 9 + tap) * a.C + q * 8) * 2);
    glds16_asm_at(wr, l0 + ins * 1024, off, 0u);
  }
  int item = slot;
  set_hoff(item);
  issue_h(0);
  TSTAMP_TH(a.tim, 24, LT);
  if (lt < kCOT) {
    const int co = cob * kCOT + lt;
    cst[lt] = a.bias ? a.bias[co] : 0.f;
    cst[kCOT + lt] = FBWD ? a.bb.mean[co] : 0.f;
    cst[2 * kCOT + lt] = FBWD ? a.bb.invstd[co] : 0.f;
  }
  if constexpr (XF) __builtin_amdgcn_s_barrier();  // X: xss (computed first thing) visible
  // xform: relu(x * scale + shift) of the halo chunks this lane's own DMA
  // staged (its wait covers exactly those), in place; conv padding (kOOB, zero
  // filled) stays 0; the tile interior is the activation h, stored by the
  // blocks of output-channel block 0 (bn_apply's expression: bit-identical)
  auto xform_halo = [&](int bb, int it) {
    char* Hb = smem + k2OffH0 + bb * kHBytes;
    const int t = it / ncb;
    const int n = t / (tp * tq), rem = t - n * (tp * tq);
    const int oh0 = (rem / tq) * kTH, ow0 = (rem % tq) << 4;
#pragma unroll
    for (int k = 0; k < kHPer; ++k) {
      if (k >= nh || hoff[k] == kOOB) continue;
      const int hp = (lw + k * kNL) * 8 + (lane >> 3);
      const int c0 = ((lane & 7) ^ (hp & 6)) * 8;
      uint4* q = reinterpret_cast<uint4*>(Hb + (lw + k * kNL) * 1024 + lane * 16);
      float v[8];
      unpack8(*q, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] * xss[c0 + e] + xss[64 + c0 + e];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
      const uint4 o = pack8(v);
      *q = o;
      const int hr = hp / kHW, hc = hp - hr * kHW;
      if (cob == 0 && hr >= 1 && hr <= kTH && hc >= 1 && hc <= 16 && UNET_ABL != 4)
        *reinterpret_cast<uint4*>(a.xh + ((size_t)(n * a.H + oh0 - 1 + hr) * a.W + ow0 - 1 + hc) * a.ldxh + c0) = o;
    }
  };
  const int c8 = (lane & 7) * 8;  // this lane's 8 channels of every epilogue item
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s0[e] = s1[e] = 0.f;
  bool have_cst = false;
  // the epilogue of the tile whose bf16 outputs are in T (buffer tb): item q =
  // stripe lw + 4 q, pixel 8 stripe + (lane >> 3)
  // (the fused-backward operands are loaded by the epilogue itself: a
  // prefetch a tile ahead made hipcc wait for vmcnt(0) -- the next halo's DMA
  // -- before reusing the store-data registers; measured slower)
  // the previous tile's epilogue in two halves around the refill of its
  // buffer: this wave's T rows into registers, then (the caller) the next
  // halo's DMA, then the operand loads, mask / sums and stores -- the DMA is
  // older than the operand loads, so hipcc's waits for those cover it exactly
  uint4 tv[8];
  auto epi_read = [&](int tb) {
    const char* T = smem + k2OffH0 + tb * kHBytes;
#pragma unroll
    for (int q = 0; q < 8; ++q) tv[q] = *reinterpret_cast<const uint4*>(T + t2_off((lw + 4 * q) * 8 + (lane >> 3), lane & 7));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own T rows read before the refill
  };
  auto epilogue = [&](int tb, int pix0) {
    if (FBWD && !have_cst) {
      fl_ld8(cst + kCOT + c8, mu);
      fl_ld8(cst + 2 * kCOT + c8, is);
      have_cst = true;
    }
    ws2_items<FBWD, 0, 8, true>(a, nullptr, cob, pix0, lw, lane, mu, is, s0, s1, tv);
  };
  int k = 0, b = 0, prev_pix0 = 0;
  for (; item < nitems; item += gridDim.x, b ^= 1, ++k) {
    const int next = item + gridDim.x;
    // this tile's halo (first time also the weights and constants); XF: after
    // the first tile it was waited for and transformed in the previous
    // iteration, under the MFMAs
    if (!XF || k == 0) wait_vmcnt<0>();
    if (XF && k == 0) xform_halo(b, item);
    if (k == 0) TSTAMP_TH(a.tim, 25, LT);
    if (k == 1) TSTAMP_TH(a.tim, 27, LT);
    __builtin_amdgcn_s_barrier();  // B
    if (k > 0) epi_read(b ^ 1);  // the previous tile's T, in the other buffer
    if (k == 0) TSTAMP_TH(a.tim, 26, LT);
    if (next < nitems) {  // its halo into the buffer just emptied
      set_hoff(next);
      issue_h(b ^ 1);
    }
    if (k > 0) epilogue(b ^ 1, prev_pix0);
    prev_pix0 = tile_pix0(item);
    if (XF && next < nitems) {  // the next halo: landed and transformed before F
      wait_vmcnt<0>();
      xform_halo(b ^ 1, next);
    }
    __builtin_amdgcn_s_barrier();  // F
    __builtin_amdgcn_s_barrier();  // E
  }
  // the last tile (buffer b ^ 1 after the loop's final flip): items 0 .. 3 of
  // every stripe set here, 4 .. 7 by the compute waves (nothing else to do)
  {
    if (FBWD && !have_cst) {
      fl_ld8(cst + kCOT + c8, mu);
      fl_ld8(cst + 2 * kCOT + c8, is);
    }
    ws2_items<FBWD, 0, 4>(a, smem + k2OffH0 + (b ^ 1) * kHBytes, cob, prev_pix0, lw, lane, mu, is, s0, s1);
  }
  TSTAMP_TH(a.tim, 21, LT);
  // BN-backward sums: [64 slots (32 loader, 32 compute)][64 channels][2] in the other buffer (free),
  // then 128 threads sum the slots in a fixed order
  float* red = reinterpret_cast<float*>(smem + k2OffH0 + b * kHBytes);
  if constexpr (FBWD) {
    const int sl = lt >> 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(sl * kCOT + c8 + e) * 2 + 0] = s0[e];
      red[(sl * kCOT + c8 + e) * 2 + 1] = s1[e];
    }
  }
  __builtin_amdgcn_s_barrier();  // R1
  if constexpr (!FLIP && STATS) {  // the compute waves' forward BN partials: [wave][lane][2][16]
    if (lt < 2 * kCOT) {
      const int co = lt % kCOT, which = lt / kCOT;
      const int i = co >> 4, gg = (co >> 2) & 3, e = co & 3;
      float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < kNC; ++w)
#pragma unroll
        for (int l = 0; l < 16; ++l) p[l & 3] += red[(w * 64 + gg * 16 + l) * 32 + which * 16 + i * 4 + e];
      const float tsum = (p[0] + p[1]) + (p[2] + p[3]);
      atomicAdd(a.stats + rep + which * a.Cout + cob * kCOT + co, (double)tsum);
    }
  }
  if constexpr (FBWD) {
    if (lt < 2 * kCOT) {
      const int c = lt % kCOT, which = lt / kCOT;
      float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int sl = 0; sl < 64; ++sl) p[sl & 3] += red[(sl * kCOT + c) * 2 + which];
      const float tsum = (p[0] + p[1]) + (p[2] + p[3]);
      atomicAdd(a.bb.sums + rep + which * a.Cout + cob * kCOT + c, (double)tsum);
    }
  }
  __builtin_amdgcn_s_barrier();  // R2
  TSTAMP_TH(a.tim, 22, LT);
  TSTAMP_RT_TH(a.tim, 31, LT);
}

// the shapes and epilogues conv3x3_ws2_kernel covers (training step: forward
// with bias and / or BN sums, data gradient with or without addend and fused
// BN backward); everything else stays on conv3x3_ws_kernel
bool conv3x3_ws2_ok(const ConvFwdArgs& a, bool flip) {
  // A/B: the previous kernel (read per launch: tests set it); "f" / "b" / "x":
  // only the forward / the data gradient / the xform forward
  const char* ev = std::getenv("UNET_NO_WS2");
  const bool off = ev && (ev[0] == '1' || (ev[0] == 'f' && !flip) || (ev[0] == 'b' && flip) ||
                          (ev[0] == 'x' && !flip && a.xform));
  // (the last-block BN finalisation, UNET_BN_TICKET, is not built in)
  if (a.bn.ticket || a.bb.ticket) return false;
  if (off || a.C != 64 || a.Cout % kCOT || a.P % kTH || a.Q % 16 || a.H != a.P || a.W != a.Q) return false;
  if (a.R != 3 || a.S != 3 || a.stride != 1 || a.pad != 1 || a.x2 || a.ysplit || a.fold_on) return false;
  if (a.xform && (flip || !a.xh || a.ldxh % 8)) return false;
  if (a.ldx % 8 || a.ldy % 8 || (a.add && a.ldadd % 4)) return false;
  if (!flip && (a.add || a.bb.sums)) return false;
  if (flip && (a.stats || (a.bb.sums && (a.bb.y2 || a.bb.ldact % 8 || a.bb.ldy % 8)))) return false;
  if ((size_t)a.N * a.H * a.W * a.ldx * 2 >= 0x80000000ull || (size_t)a.N * a.P * a.Q >= 0x80000000ull) return false;
  return true;
}

hipError_t launch_conv3x3_ws2(const ConvFwdArgs& a, int mode, hipStream_t st) {
  const bool flip = mode == 1;
  if (!conv3x3_ws2_ok(a, flip)) return hipErrorInvalidValue;
  const int ncb = a.Cout / kCOT;
  const int nitems = a.N * (a.P / kTH) * (a.Q / 16) * ncb;
  int grid = cu_count() / ncb * ncb;
  if (a.grid_cap > 0 && a.grid_cap < grid) grid = a.grid_cap / ncb * ncb;
  if (grid < ncb) grid = ncb;
  if (grid > nitems) grid = nitems;
  const bool fbwd = flip && a.bb.sums;
  const int ep = (a.add ? EP_ADD : 0) | (fbwd ? EP_FBWD : 0) | (a.stats || fbwd ? EP_STATS : 0) |
                 (!flip && a.xform ? EP_XF : 0);
  char tag[96];
  std::snprintf(tag, sizeof(tag), "conv3x3_ws2_kernel<%s, %d>", flip ? "true" : "false", ep);
  conv_kernel_tag(tag);
  const dim3 g(grid), bl(kNW * 64);
#define WS2_LAUNCH(F, E) hipLaunchKernelGGL((conv3x3_ws2_kernel<F, E>), g, bl, k2Lds, st, a, ncb, nitems)
  if (!flip) {
    if (ep == (EP_STATS | EP_XF)) WS2_LAUNCH(false, EP_STATS | EP_XF);
    else if (ep == EP_XF) WS2_LAUNCH(false, EP_XF);
    else if (ep == EP_STATS) WS2_LAUNCH(false, EP_STATS);
    else WS2_LAUNCH(false, 0);
  } else {
    switch (ep) {
      case EP_FBWD | EP_STATS: WS2_LAUNCH(true, EP_FBWD | EP_STATS); break;
      case EP_FBWD | EP_STATS | EP_ADD: WS2_LAUNCH(true, EP_FBWD | EP_STATS | EP_ADD); break;
      case EP_ADD: WS2_LAUNCH(true, EP_ADD); break;
      default: WS2_LAUNCH(true, 0); break;
    }
  }
#undef WS2_LAUNCH
  return hipGetLastError();
}

}  // namespace unet

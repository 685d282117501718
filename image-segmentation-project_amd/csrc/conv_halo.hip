// Halo convolutions for the 3x3 / stride-1 / pad-1 layers (SURVEY.md §8(a)
// rows a3 BasicBlocks and a6 decoder blocks): forward conv and its data
// gradient (FLIP: the transposed gather of s1 p1 is the same stencil with the
// taps mirrored, on the dgrad weight pack [Cin][R][S][Cout]).
//
// The implicit-GEMM kernel (conv_kernels.hip) stages an im2col tile per
// (tap, channel chunk), so every input pixel crosses L2 -> LDS once per tap
// (9x) and per output tile.  Here an output tile of TH x 16 pixels reads one
// (TH+2) x 18 input halo per 32-channel chunk and all 9 taps are MFMA'd from
// it at a row shift:
//
//  * conv3x3_ws_kernel (weight-stationary, C <= 96): a persistent block keeps
//    ALL 9 taps of its COT output channels in LDS (<= 74 KB, loaded once) and
//    streams output tiles through a double-buffered halo; the BN-statistics
//    epilogue is reduced once per block.
//  * conv3x3_hs_kernel (halo-streamed, C >= 128): one output tile per block;
//    the K loop walks 32-channel chunks, each stage = that chunk's halo plus
//    its 9 weight taps, double-buffered by LDS-DMA.  Per stage it moves
//    ((TH+2)*18 + 9*COT) * 64 B for 2*TH*16*COT*288 flop — 2.5x the flop per
//    staged byte of a 128x128 im2col tile.
//
// LDS images are panels of 32 channels = 64-B rows (a halo pixel or a weight
// row).  An MFMA operand fragment reads 16 CONSECUTIVE rows starting at an
// arbitrary row (tap shift); with the 16-B chunk XOR-swizzled by bit 2 of the
// row (chunk ^ ((row >> 1) & 2)) every ds_read_b128 lane group hits 16
// distinct bank slots for every start row (exhaustively checked for the
// gfx950 lane grouping {0-3,12-15,20-27}, ...; SQ_LDS_BANK_CONFLICT = 0
// measured).  The swizzle is applied on the DMA source side
// (cdna_hip_programming.md §5.4 rule 21).
//
// GEMM view: D[co][px] += W[co][(tap, c)] . X[px + shift(tap)][c],
// v_mfma_f32_16x16x32_bf16 with A = weight fragment (16 co x 32 c), B = halo
// fragment (16 px of one output row x 32 c); each wave owns RW output rows x
// COT channels (acc[RW][FN]).
#include <cstdio>
#include "common.h"
#include "kernels.h"

namespace unet {

void conv_kernel_tag(const char* tag);  // conv_kernels.hip: per-launch profiler column

// 8-B global load the compiler does not track (its waitcnt pass would
// otherwise drain the in-flight halo DMA at the first such load,
// cdna_hip_programming.md §5 item 4(b)); the consumer waits by hand.
__device__ __forceinline__ uint2 ld_u2_asm(const void* p) {
  uint2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

__device__ __forceinline__ int ws_off(int row, int chunk) {  // byte offset of (row, logical 16-B chunk)
  return row * 64 + ((chunk ^ ((row >> 1) & 2)) << 4);
}

constexpr int kHW = 18;  // halo width: 16 output columns + 2

// sum over the 16 lanes of a lane row, complete in lane 15 of the row
// (DPP row_shr adds; bound_ctrl reads 0 past the row start)
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x112, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x114, 0xf, 0xf, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x118, 0xf, 0xf, true));
  return v;
}

// workgroup barrier ordering LDS only: outstanding global stores stay in
// flight (__syncthreads' fence would wait for them)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Halo of one output tile (TH x 16 at (n, oh0, ow0)): np 32-channel panels of
// input channels c0 .. c0 + 32*np into LDS, HPR rows per panel.  DMA
// instructions are dealt round-robin over the NW waves.
// 9 taps x COT output rows x np panels of 32 reduction channels from kc0,
// LDS layout [tap][panel][co][32]; weights packed [Cout][9][K = a.C].
template <int COT, int NW>
__device__ __forceinline__ void issue_weight_dma(const ConvFwdArgs& a, __amdgpu_buffer_rsrc_t wr, char* dst,
                                                 int co0, int kc0, int np, int wave, int lane) {
  const int K = a.C;
  const int nins = 9 * np * COT / 16;
  for (int ins = wave; ins < nins; ins += NW) {
    const int rowg = ins * 16 + (lane >> 2);
    const int co = rowg % COT, tpn = rowg / COT;
    const int p = tpn % np, tap = tpn / np;
    const int lchunk = (lane & 3) ^ ((co >> 1) & 2);
    unsigned off = kOOB;
    if (co0 + co < a.Cout) off = (unsigned)(((co0 + co) * 9 * K + tap * K + kc0 + p * 32 + lchunk * 8) * 2);
    glds16(wr, dst + ins * 1024, off);
  }
}

// One 32-channel panel of a tile: 9 taps x RW rows x FN channel fragments.
// W: the panel's weight image (tap stride WTS bytes, 16-co fragment stride
// 1 KiB); H: the panel's halo image.
// Per column shift s the RW + 2 halo rows the wave's RW output rows reach are
// read once and serve all three tap rows r (output row j reads halo row j +
// dr): 3 (RW + 2) B-fragment reads per panel instead of 9 RW (RW = 2: 12
// instead of 18 -- the LDS port, not the MFMA, bounds these narrow convs).
template <int FN, int RW, int WTS, bool FLIP>
__device__ __forceinline__ void mfma_panel(f32x4 (&acc)[RW][FN], const char* W, const char* H, int aoff,
                                           const int (&boff)[RW + 2][3]) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    const int ds = FLIP ? 2 - s : s;
    bf16x8 B[RW + 2];
#pragma unroll
    for (int h = 0; h < RW + 2; ++h) B[h] = *reinterpret_cast<const bf16x8*>(H + boff[h][ds]);
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      bf16x8 A[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) A[i] = *reinterpret_cast<const bf16x8*>(W + (r * 3 + s) * WTS + i * 1024 + aoff);
      const int dr = FLIP ? 2 - r : r;
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B[j + dr], acc[j][i], 0, 0, 0);
    }
  }
}

// ---- full-line staging (64 reduction channels = one 128-B line per pixel /
// weight row): an LDS-DMA piece of 64 B fetches half a line, and the per-CU
// L2 -> LDS rate is set by lines, not bytes (scripts/micro/dma_rate.hip,
// profiles/r05: 32 B/clk/CU for 64-B pieces, 54 for whole lines from L2; 3.5
// vs 6.7 TB/s chip-wide from HBM).  A 128-B LDS row holds both 32-channel
// panels; 16-B chunk q = 4 p + c of row r sits at physical chunk q ^ (r & 6),
// which keeps every ds_read_b128 lane group of a 16-row fragment on 16
// distinct bank slots for any start row and either panel (exhaustive search
// over the gfx950 lane groups).  Panel 1 of a row = panel 0's offset ^ 64.
__device__ __forceinline__ int fl_off(int row, int chunk) {  // byte offset of panel-0 chunk `chunk` of `row`
  return row * 128 + ((chunk ^ (row & 6)) << 4);
}

// all 9 taps x COT output rows x 64 reduction channels (weights [Cout][9][64],
// full lines), LDS layout [tap][co][128 B]
template <int COT, int NW>
__device__ __forceinline__ void issue_weight_dma_fl(const ConvFwdArgs& a, __amdgpu_buffer_rsrc_t wr, char* dst, int co0,
                                                    int wave, int lane) {
  const int K = a.C;
  constexpr int nins = 9 * COT / 8;
  for (int ins = wave; ins < nins; ins += NW) {
    const int rowg = ins * 8 + (lane >> 3);
    const int co = rowg % COT, tap = rowg / COT;
    const int q = (lane & 7) ^ (co & 6);  // logical 16-B chunk = 8 channels
    unsigned off = kOOB;
    if (co0 + co < a.Cout) off = (unsigned)(((co0 + co) * 9 * K + tap * K + q * 8) * 2);
    glds16(wr, dst + ins * 1024, off);
  }
}

// both panels of a full-line stage: 9 taps x RW rows x FN channel fragments
// per panel; aoff / boff are panel-0 offsets (fl_off)
template <int FN, int RW, int COT, bool FLIP>
__device__ __forceinline__ void mfma_fl(f32x4 (&acc)[RW][FN], const char* W, const char* H, int aoff,
                                        const int (&boff)[RW + 2][3]) {
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        bf16x8 A[FN];
#pragma unroll
        for (int i = 0; i < FN; ++i)
          A[i] = *reinterpret_cast<const bf16x8*>(W + (r * 3 + s) * COT * 128 + i * 2048 + (aoff ^ (p << 6)));
        const int dr = FLIP ? 2 - r : r, ds = FLIP ? 2 - s : s;
#pragma unroll
        for (int j = 0; j < RW; ++j) {
          const bf16x8 B = *reinterpret_cast<const bf16x8*>(H + (boff[j + dr][ds] ^ (p << 6)));
#pragma unroll
          for (int i = 0; i < FN; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B, acc[j][i], 0, 0, 0);
        }
      }
}

// Epilogue of one tile: bias, addend, ReLU mask (fused BN backward), bf16
// store, BN sums accumulated in registers (q0, q1).  cst = LDS [3][COT]
// bias | mean | invstd.  The per-pixel operands of a dgrad (addend, forward
// activation, raw conv output of the BN) are fetched by fetch(): early with
// untracked loads (PREF) so their latency hides behind MFMA work, else right
// before use; landed() is the matching wait.
template <int FN, int RW, bool FLIP, bool PREF, bool TWO>
struct TileEpi {
  uint2 uadd[RW][FN], uact[RW][FN], uy[RW][FN];
  uint2 uy2[TWO ? RW : 1][TWO ? FN : 1];  // raw conv output of the second BN (downsample pair)

  __device__ __forceinline__ void fetch(const ConvFwdArgs& a, const size_t (&pix)[RW], int co0, int lane) {
    if (!FLIP && !a.add) return;
    const BnBwdArgs& bb = a.bb;
    if (a.add) {  // conditions hoisted out of the loads (no per-load branch + wait)
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int co = min(co0 + i * 16 + ((lane >> 4) << 2), a.Cout - 4);
          const void* src = a.add + pix[j] * a.ldadd + co;
          uadd[j][i] = PREF ? ld_u2_asm(src) : *reinterpret_cast<const uint2*>(src);
        }
    } else {
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) uadd[j][i] = make_uint2(0, 0);
    }
    if (FLIP && bb.sums) {
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) {
          const int co = min(co0 + i * 16 + ((lane >> 4) << 2), a.Cout - 4);
          const void* s1 = bb.act + pix[j] * bb.ldact + co;
          const void* s2 = bb.y + pix[j] * bb.ldy + co;
          uact[j][i] = PREF ? ld_u2_asm(s1) : *reinterpret_cast<const uint2*>(s1);
          uy[j][i] = PREF ? ld_u2_asm(s2) : *reinterpret_cast<const uint2*>(s2);
          if constexpr (TWO) {
            const void* s3 = bb.y2 + pix[j] * bb.ldy2 + co;
            uy2[j][i] = PREF ? ld_u2_asm(s3) : *reinterpret_cast<const uint2*>(s3);
          }
        }
    } else {
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) uact[j][i] = uy[j][i] = make_uint2(0, 0);
    }
  }

  __device__ __forceinline__ void landed() {
    if (!PREF) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int i = 0; i < FN; ++i)  // order every use after the wait
        asm volatile("" : "+v"(uadd[j][i].x), "+v"(uadd[j][i].y), "+v"(uact[j][i].x), "+v"(uact[j][i].y),
                     "+v"(uy[j][i].x), "+v"(uy[j][i].y));
    if constexpr (TWO) {
#pragma unroll
      for (int j = 0; j < RW; ++j)
#pragma unroll
        for (int i = 0; i < FN; ++i) asm volatile("" : "+v"(uy2[j][i].x), "+v"(uy2[j][i].y));
    }
  }

  // bias, addend, ReLU mask, BN sums as before; the bf16 quads of a row pair
  // (channel fragments i, i+1) are exchanged between lane rows 0<->1 and
  // 2<->3 (v_permlane16_swap) so every lane stores 16 contiguous bytes and a
  // wave instruction writes 64 B per pixel instead of 8-B pieces.  vec16:
  // ld / channel split multiples of 8 (else the 8-B stores).
  __device__ __forceinline__ void store(const ConvFwdArgs& a, const f32x4 (&acc)[RW][FN], const size_t (&pix)[RW],
                                        int co0, int lane, const float* cst, float (&q0)[FN][4],
                                        float (&q1)[FN][4], float (&q2)[FN][4]) {
    constexpr int COT = FN * 16;
    static_assert(FN % 2 == 0, "fragment pairs");
    const bool fbwd = a.bb.sums != nullptr;
    const bool stats = a.stats != nullptr || fbwd;
    const bool vec16 = (a.ldy % 8 == 0) && (!a.ysplit || (a.ldysplit % 8 == 0 && a.csplit % 8 == 0));
    const bool fold = !FLIP && a.fold_on;
    const int g = lane >> 4;
    // fragment pairs (2 ip, 2 ip + 1) outermost: the lane's channel constants
    // of the pair (4 consecutive channels per fragment: bias or shift' | scale
    // or mean | invstd | mean2 | invstd2) are read from LDS once, together,
    // and serve every row of the tile
#pragma unroll
    for (int ip = 0; ip < FN / 2; ++ip) {
      f32x4 kb[2], km[2], ki[2], km2[2], ki2[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int cl = (2 * ip + h) * 16 + (g << 2);
        kb[h] = *reinterpret_cast<const f32x4*>(cst + cl);
        if (fold || (FLIP && fbwd)) km[h] = *reinterpret_cast<const f32x4*>(cst + COT + cl);
        if (FLIP && fbwd) ki[h] = *reinterpret_cast<const f32x4*>(cst + 2 * COT + cl);
        if (TWO && FLIP && fbwd) {
          km2[h] = *reinterpret_cast<const f32x4*>(cst + 3 * COT + cl);
          ki2[h] = *reinterpret_cast<const f32x4*>(cst + 4 * COT + cl);
        }
      }
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        uint2 oq[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int i = 2 * ip + h;
          const int cl = i * 16 + (g << 2);
          const int co = co0 + cl;
          const bool live = co < a.Cout;
          float v[4];
          if (fold) {  // eval BN folded: (conv + bias) * scale + shift' (cst: shift' | scale)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[j][i][e] * km[h][e] + kb[h][e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = acc[j][i][e] + kb[h][e];
          }
          if (!FLIP && a.add) {  // forward residual, then the folded BN's ReLU
            const uint2 u = uadd[j][i];
            v[0] += __uint_as_float(u.x << 16); v[1] += __uint_as_float(u.x & 0xffff0000u);
            v[2] += __uint_as_float(u.y << 16); v[3] += __uint_as_float(u.y & 0xffff0000u);
          }
          if (!FLIP && a.fold_relu) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
          }
          if (FLIP) {
            const uint2 u = uadd[j][i], m = uact[j][i];
            v[0] += __uint_as_float(u.x << 16); v[1] += __uint_as_float(u.x & 0xffff0000u);
            v[2] += __uint_as_float(u.y << 16); v[3] += __uint_as_float(u.y & 0xffff0000u);
            if (fbwd) {
              if (!(__uint_as_float(m.x << 16) > 0.f)) v[0] = 0.f;
              if (!(__uint_as_float(m.x & 0xffff0000u) > 0.f)) v[1] = 0.f;
              if (!(__uint_as_float(m.y << 16) > 0.f)) v[2] = 0.f;
              if (!(__uint_as_float(m.y & 0xffff0000u) > 0.f)) v[3] = 0.f;
            }
          }
          uint2 o;
          o.x = pack_bf2(v[0], v[1]);
          o.y = pack_bf2(v[2], v[3]);
          oq[h] = o;
          if (!live) continue;
          if (!vec16) {
            if (a.ysplit && co >= a.csplit) *reinterpret_cast<uint2*>(a.ysplit + pix[j] * a.ldysplit + co - a.csplit) = o;
            else *reinterpret_cast<uint2*>(a.y + pix[j] * a.ldy + co) = o;
          }
          if (FLIP && fbwd) {  // sums of the stored bf16 dZ, as bn_bwd_reduce_kernel would read them
            const float dz[4] = {__uint_as_float(o.x << 16), __uint_as_float(o.x & 0xffff0000u),
                                 __uint_as_float(o.y << 16), __uint_as_float(o.y & 0xffff0000u)};
            const uint2 u = uy[j][i];
            const float yv[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                 __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              q0[i][e] += dz[e];
              q1[i][e] += dz[e] * (yv[e] - km[h][e]) * ki[h][e];
            }
            if constexpr (TWO) {
              const uint2 w = uy2[j][i];
              const float y2[4] = {__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                                   __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u)};
#pragma unroll
              for (int e = 0; e < 4; ++e) q2[i][e] += dz[e] * (y2[e] - km2[h][e]) * ki2[h][e];
            }
          } else if (stats) {
#pragma unroll
            for (int e = 0; e < 4; ++e) { q0[i][e] += v[e]; q1[i][e] += v[e] * v[e]; }
          }
        }
        if (vec16) {
          // rows (0,1,2,3) end up holding channels (0-7, 16-23, 8-15, 24-31) of the pair
          const auto sx = __builtin_amdgcn_permlane16_swap(oq[0].x, oq[1].x, false, false);
          const auto sy = __builtin_amdgcn_permlane16_swap(oq[0].y, oq[1].y, false, false);
          const uint4 chunk = make_uint4(sx[0], sy[0], sx[1], sy[1]);
          const int co = co0 + ip * 32 + ((g & 1) << 4) + ((g >> 1) << 3);
          if (co < a.Cout && UNET_ABL != 4) {  // (ABL 4: timing build without the tile stores)
            if (a.ysplit && co >= a.csplit)
              *reinterpret_cast<uint4*>(a.ysplit + pix[j] * a.ldysplit + co - a.csplit) = chunk;
            else *reinterpret_cast<uint4*>(a.y + pix[j] * a.ldy + co) = chunk;
          }
        }
      }
    }
  }
};

// bias | mean | invstd | mean2 | invstd2 of the block's COT channels into LDS
constexpr int kEpiConsts = 5;
template <int COT>
__device__ __forceinline__ void load_epi_constants(const ConvFwdArgs& a, float* cst, int co0, int tid, int nthr) {
  const bool fbwd = a.bb.sums != nullptr;
  const bool two = fbwd && a.bb.y2 != nullptr;
  for (int c = tid; c < COT; c += nthr) {
    const int co = co0 + c;
    const bool ok = co < a.Cout;
    cst[c] = (a.bias && ok) ? a.bias[co] : 0.f;
    if (a.fold_on) {  // eval BN: shift' = bias * scale + shift, scale (running statistics)
      float sc = 1.f, sh = 0.f, m, is, var;
      if (ok) bn_scale_shift(a.fold, co, sc, sh, m, is, var);
      cst[c] = cst[c] * sc + sh;
      cst[COT + c] = sc;
      continue;
    }
    cst[COT + c] = (fbwd && ok) ? a.bb.mean[co] : 0.f;
    cst[2 * COT + c] = (fbwd && ok) ? a.bb.invstd[co] : 0.f;
    cst[3 * COT + c] = (two && ok) ? a.bb.mean2[co] : 0.f;
    cst[4 * COT + c] = (two && ok) ? a.bb.invstd2[co] : 0.f;
  }
}

// Block reduction of the BN sums (16 pixel lanes, then the NW waves through
// LDS at `scratch`), fp64 atomics into replica blockIdx.x % kStatRep, and the
// optional last-block finalisation.
template <int FN, int NW, bool TWO>
__device__ __forceinline__ void stats_atomics(const ConvFwdArgs& a, float (&q0)[FN][4], float (&q1)[FN][4],
                                              float (&q2)[FN][4], int co0, char* scratch) {
  constexpr int COT = FN * 16;
  const BnBwdArgs& bb = a.bb;
  const bool fbwd = bb.sums != nullptr;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q0[i][e] = row16_sum(q0[i][e]);
      q1[i][e] = row16_sum(q1[i][e]);
      if (TWO) q2[i][e] = row16_sum(q2[i][e]);
    }
  float* red = reinterpret_cast<float*>(scratch);  // [NW][COT][3]
  lds_barrier();  // every wave is done reading the staging LDS (no wait for the tile stores)
  if ((lane & 15) == 15) {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int cl = i * 16 + ((lane >> 4) << 2) + e;
        red[(wave * COT + cl) * 3 + 0] = q0[i][e];
        red[(wave * COT + cl) * 3 + 1] = q1[i][e];
        red[(wave * COT + cl) * 3 + 2] = TWO ? q2[i][e] : 0.f;
      }
  }
  lds_barrier();
  for (int cl = tid; cl < COT; cl += NW * 64) {
    const int co = co0 + cl;
    if (co < a.Cout) {
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        s0 += red[(w * COT + cl) * 3];
        s1 += red[(w * COT + cl) * 3 + 1];
        s2 += red[(w * COT + cl) * 3 + 2];
      }
      const size_t rep = (size_t)(blockIdx.x % kStatRep) * 2 * a.Cout;
      double* dst = fbwd ? bb.sums + rep : a.stats + rep;
      atomicAdd(dst + co, (double)s0);
      atomicAdd(dst + a.Cout + co, (double)s1);
      if (TWO) atomicAdd(bb.sums2 + rep + a.Cout + co, (double)s2);
    }
  }
}

// the launch's last block (ticket) finalises the BN (forward or backward) whose
// sums the blocks added (stats_atomics)
template <int COT, int NW>
__device__ __forceinline__ void stats_ticket(const ConvFwdArgs& a, char* scratch) {
  const BnBwdArgs& bb = a.bb;
  const bool fbwd = bb.sums != nullptr;
  const int tid = threadIdx.x;
  unsigned* ticket = fbwd ? bb.ticket : a.bn.ticket;
  if (ticket) {
    int* flag = reinterpret_cast<int*>(scratch + NW * COT * 3 * sizeof(float));
    if (last_block_arrive(ticket, gridDim.x * gridDim.y * gridDim.z, flag, tid < COT)) {
      if (fbwd) bn_bwd_finalize(bb);
      else bn_finalize(a.bn);
    }
  }
}

template <int FN, int NW, bool TWO>
__device__ __forceinline__ void commit_stats(const ConvFwdArgs& a, float (&q0)[FN][4], float (&q1)[FN][4],
                                             float (&q2)[FN][4], int co0, char* scratch) {
  stats_atomics<FN, NW, TWO>(a, q0, q1, q2, co0, scratch);
  stats_ticket<FN * 16, NW>(a, scratch);
}

// ---------------------------------------------------------------------------
// weight-stationary (C = 32 * NP <= 96)
// ---------------------------------------------------------------------------
template <int NP, int FN, int TH, int NW, bool FLIP>
__global__ void __launch_bounds__(NW * 64) conv3x3_ws_kernel(ConvFwdArgs a, int ntiles, int ncg) {
  constexpr int COT = FN * 16;               // output channels per block
  constexpr int RW = TH / NW;                // output rows per wave
  constexpr int HPR = ((TH + 2) * kHW + 15) / 16 * 16;
  constexpr int PANEL = HPR * 64;
  constexpr int HBUF = NP * PANEL;
  constexpr int WBYTES = 9 * NP * COT * 64;
  constexpr bool PREF = FLIP && RW * FN <= 8;
  static_assert(TH % NW == 0 && RW >= 1, "rows per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* wl = smem;
  char* hl = smem + WBYTES;
  float* cst = reinterpret_cast<float*>(hl + 2 * HBUF);  // [kEpiConsts][COT]
  float* xss = cst + kEpiConsts * COT;                   // xform: [2][NP*32] scale | shift

  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = blockIdx.x % ncg;
  const int nslot = gridDim.x / ncg;
  const int co0 = cg * COT;
  const int tq = a.Q >> 4, tp = a.P / TH;
  // halo DMA as inline asm (untracked by the compiler): with the builtin,
  // hipcc puts an s_waitcnt vmcnt(0) in front of every LDS store that follows
  // it (the BN transform of the staged halo) -- each one draining the next
  // tile's halo AND every activation store still in flight.  The kernel
  // waits for its DMA itself (wait_vmcnt before the tile barrier).
  const i32x4 xr = make_rsrc_sgpr(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (unsigned)((size_t)a.Cout * 9 * a.C * 2));

  // NP == 2 (64 channels): full-line staging of the weights and the halo (fl_off)
  constexpr bool FL = NP == 2;
  if constexpr (FL) issue_weight_dma_fl<COT, NW>(a, wr, wl, co0, wave, lane);  // all 9 taps, once
  else issue_weight_dma<COT, NW>(a, wr, wl, co0, 0, NP, wave, lane);
  load_epi_constants<COT>(a, cst, co0, tid, NW * 64);
  if (!FLIP && a.xform) {  // the previous BN's affine map (bn_apply's coefficients)
    for (int c = tid; c < NP * 32; c += NW * 64) {
      float m, is, var;
      bn_scale_shift(a.xbn, c, xss[c], xss[NP * 32 + c], m, is, var);
    }
    if (blockIdx.x == 0) bn_finalize(a.xbn);  // saved mean / invstd, running statistics
  }
  float q0[FN][4], q1[FN][4], q2[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = q2[i][e] = 0.f;

  // loop-invariant fragment offsets: weights (16 co rows from co = 0) and the
  // halo rows this wave's output rows need for every tap shift
  const int aoff = FL ? fl_off(lane & 15, lane >> 4) : ws_off(lane & 15, lane >> 4);
  int boff[RW + 2][3];
#pragma unroll
  for (int h = 0; h < RW + 2; ++h)
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const int row = (wave * RW + h) * kHW + d + (lane & 15);
      boff[h][d] = FL ? fl_off(row, lane >> 4) : ws_off(row, lane >> 4);
    }

  // per-lane constant part of the halo DMA (pixel of the halo, channel
  // offset); per tile only the image bounds test and the address remain.
  // FL: 8 pixels x 128 B per instruction, else 16 pixels x 64 B of one panel
  constexpr int H_NINS = FL ? HPR / 8 : NP * HPR / 16, H_PER = (H_NINS + NW - 1) / NW;
  int hrow[H_PER], hcol[H_PER], hch[H_PER];
#pragma unroll
  for (int k = 0; k < H_PER; ++k) {
    int hp, ch;
    if constexpr (FL) {
      hp = (wave + k * NW) * 8 + (lane >> 3);
      ch = ((lane & 7) ^ (hp & 6)) * 8;
    } else {
      const int rowg = (wave + k * NW) * 16 + (lane >> 2);
      const int p = rowg / HPR;
      hp = rowg - p * HPR;
      ch = p * 32 + ((lane & 3) ^ ((hp >> 1) & 2)) * 8;
    }
    hrow[k] = hp < (TH + 2) * kHW ? hp / kHW - 1 : -(1 << 20);  // invalid rows fail the bounds test
    hcol[k] = hp - (hp / kHW) * kHW - 1;
    hch[k] = ch;
  }
  auto issue_halo = [&](char* dst, int n, int oh0, int ow0) {
#pragma unroll
    for (int k = 0; k < H_PER; ++k) {
      if (wave + k * NW >= H_NINS) break;
      const int ih = oh0 + hrow[k], iw = ow0 + hcol[k];
      unsigned off = kOOB;
      if ((unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
        off = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + hch[k]) * 2);
      glds16_asm(xr, dst + (wave + k * NW) * 1024, off, 0u);
    }
  };

  auto tile_origin = [&](int t, int& n, int& oh0, int& ow0) {
    n = t / (tp * tq);
    const int rem = t - n * (tp * tq);
    oh0 = (rem / tq) * TH;
    ow0 = (rem % tq) << 4;
  };

  int t = blockIdx.x / ncg;
  if (t < ntiles) {
    int n, oh0, ow0;
    tile_origin(t, n, oh0, ow0);
    issue_halo(hl, n, oh0, ow0);
  }
  wait_vmcnt<0>();
  __syncthreads();
  TSTAMP(a.tim, 1);

  for (int k = 0; t < ntiles; ++k, t += nslot) {
    const int b = k & 1;
    if (t + nslot < ntiles && UNET_ABL != 2) {  // lands while this tile computes
      int n, oh0, ow0;
      tile_origin(t + nslot, n, oh0, ow0);
      issue_halo(hl + (b ^ 1) * HBUF, n, oh0, ow0);
    }
    int n, oh0, ow0;
    tile_origin(t, n, oh0, ow0);
    size_t pix[RW];
#pragma unroll
    for (int j = 0; j < RW; ++j) pix[j] = ((size_t)n * a.P + oh0 + wave * RW + j) * a.Q + ow0 + (lane & 15);
    TileEpi<FN, RW, FLIP, PREF, false> epi;
    if (PREF) epi.fetch(a, pix, co0, lane);
    if (!FLIP && a.xform) {
      // relu(y * scale + shift) of every in-image halo pixel, in place (the
      // zero-filled conv padding stays 0); the interior is the stored activation
      char* Hb = hl + b * HBUF;
      constexpr int XI = (NP * HPR * 4 + NW * 64 - 1) / (NW * 64);  // fixed trip count: unrolled,
#pragma unroll                                                       // every LDS read issued up front
      for (int it = 0; it < XI; ++it) {
        const int idx = tid + it * NW * 64;
        if (idx >= NP * HPR * 4) break;
        int row, c0;
        uint4* q;
        if constexpr (FL) {  // physical chunk idx & 7 of row idx >> 3 holds channels 8 (phys ^ (row & 6))
          row = idx >> 3;
          q = reinterpret_cast<uint4*>(Hb + idx * 16);
          c0 = ((idx & 7) ^ (row & 6)) * 8;
        } else {
          const int p = idx / (HPR * 4), rem = idx - p * (HPR * 4);
          const int ch = rem & 3;
          row = rem >> 2;
          q = reinterpret_cast<uint4*>(Hb + p * PANEL + ws_off(row, ch));
          c0 = p * 32 + ch * 8;
        }
        if (row >= (TH + 2) * kHW) continue;
        const int hr = row / kHW, hc = row - hr * kHW;
        const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
        if ((unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) continue;
        float v[8];
        unpack8(*q, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] * xss[c0 + k] + xss[NP * 32 + c0 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = v[k] > 0.f ? v[k] : 0.f;
        const uint4 o = pack8(v);
        *q = o;
        if (cg == 0 && hr >= 1 && hr <= TH && hc >= 1 && hc <= 16 && UNET_ABL != 4)
          *reinterpret_cast<uint4*>(a.xh + (((size_t)n * a.H + ih) * a.W + iw) * a.ldxh + c0) = o;
      }
      lds_barrier();  // transformed halo visible to every wave (DMA / h stores stay in flight)
    }
    if (UNET_ABL >= 3 && k < 3) TSTAMP(a.tim, 2 + 5 * k);
    const char* H = hl + b * HBUF;
    f32x4 acc[RW][FN];
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int i = 0; i < FN; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (FL) {
      if (UNET_ABL != 1) mfma_fl<FN, RW, COT, FLIP>(acc, wl, H, aoff, boff);
    } else {
#pragma unroll
      for (int p = 0; p < (UNET_ABL == 1 ? 0 : NP); ++p)
        mfma_panel<FN, RW, NP * COT * 64, FLIP>(acc, wl + p * COT * 64, H + p * PANEL, aoff, boff);
    }
    // stamps: 2 per tile (after the MFMAs, after the epilogue); UNET_ABL == 3
    // (fine build): 4 per tile for the first 4 tiles (+ after the wait, after the barrier)
    if (UNET_ABL >= 3 ? k < 3 : k < 9) TSTAMP(a.tim, UNET_ABL >= 3 ? 3 + 5 * k : 2 + 2 * k);
    if (!PREF) epi.fetch(a, pix, co0, lane);
    epi.landed();
    wait_vmcnt<0>();               // the next tile's halo (issued before this tile's MFMAs) has landed ...
    if (UNET_ABL >= 3 && k < 3) TSTAMP(a.tim, 4 + 5 * k);
    __builtin_amdgcn_s_barrier();  // ... everyone's part; buffer b is free for reuse
    if (UNET_ABL >= 3 && k < 3) TSTAMP(a.tim, 5 + 5 * k);
    // the stores go out AFTER the wait: they drain under the next tile's MFMAs
    // instead of being waited for here (vmcnt counts stores too)
    epi.store(a, acc, pix, co0, lane, cst, q0, q1, q2);
    if (UNET_ABL >= 3 ? k < 3 : k < 9) TSTAMP(a.tim, UNET_ABL >= 3 ? 6 + 5 * k : 3 + 2 * k);
  }
  TSTAMP(a.tim, 20);
  if (a.stats || a.bb.sums) commit_stats<FN, NW, false>(a, q0, q1, q2, co0, smem);
  TSTAMP(a.tim, 21);
  TSTAMP_RT(a.tim, 31);
}

// ---------------------------------------------------------------------------
// halo-streamed (C >= 128, multiple of 32): TH x 16 x COT output tiles, K
// loop over 32-channel chunks, stage = halo panel + 9 weight taps.  A block
// owns output-channel block cob and the tiles slot, slot + nslot, ... (grid =
// ncb x nslot): when the grid is larger than the resident slots the blocks are
// persistent, the first stage of the next tile is staged under the last
// chunk's MFMAs and the BN sums of all its tiles are committed once (enc2 /
// decoder3: 1024 tiles x co-blocks on 512 slots, formerly two rounds of
// blocks, each paying its own prologue; profiles/r04/s1 conv_timing.txt)
// ---------------------------------------------------------------------------
template <int FN, int TH, int NW, bool FLIP, bool TWO, bool MT>
__global__ void __launch_bounds__(NW * 64) conv3x3_hs_kernel(ConvFwdArgs a, int ncb, int ntiles) {
  constexpr int COT = FN * 16;
  constexpr int RW = TH / NW;
  constexpr int HPR = ((TH + 2) * kHW + 15) / 16 * 16;
  constexpr int HBYTES = HPR * 64;
  constexpr int WBYTES = 9 * COT * 64;
  constexpr int STAGE = HBYTES + WBYTES;
  constexpr bool PREF = FLIP && RW * FN <= 8;
  static_assert(TH % NW == 0 && RW >= 1, "rows per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cst = reinterpret_cast<float*>(smem + 2 * STAGE);  // [kEpiConsts][COT]

  TSTAMP_RT(a.tim, 30);
  TSTAMP(a.tim, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cob = bid % ncb, nslot = gridDim.x / ncb;
  const int co0 = cob * COT;
  const int tq = a.Q >> 4, tp = a.P / TH;
  const int KC = a.C >> 5;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (unsigned)((size_t)a.Cout * 9 * a.C * 2));
  int tile = bid / ncb;

  // Per-lane DMA offsets of channel chunk 0 (per tile for the halo): chunk kc
  // only adds kc * 64 B, passed as the instruction's scalar offset (the address
  // arithmetic would otherwise sit between the barrier and the MFMAs of every
  // stage, on both waves of a SIMD at once).
  constexpr int H_NINS = HPR / 16, H_PER = (H_NINS + NW - 1) / NW;
  constexpr int W_NINS = 9 * COT / 16, W_PER = (W_NINS + NW - 1) / NW;
  unsigned hoff[H_PER], woff[W_PER];
  auto tile_origin = [&](int t, int& n, int& oh0, int& ow0) {
    n = t / (tp * tq);
    const int rem = t - n * (tp * tq);
    oh0 = (rem / tq) * TH;
    ow0 = (rem % tq) << 4;
  };
  auto set_hoff = [&](int t) {
    int n, oh0, ow0;
    tile_origin(t, n, oh0, ow0);
#pragma unroll
    for (int k = 0; k < H_PER; ++k) {
      const int hp = (wave + k * NW) * 16 + (lane >> 2);  // one panel per stage
      const int lchunk = (lane & 3) ^ ((hp >> 1) & 2);
      const int hr = hp / kHW, hc = hp - hr * kHW;
      const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
      hoff[k] = kOOB;
      if (hp < (TH + 2) * kHW && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
        hoff[k] = (unsigned)((((n * a.H + ih) * a.W + iw) * a.ldx + lchunk * 8) * 2);
    }
  };
#pragma unroll
  for (int k = 0; k < W_PER; ++k) {
    const int rowg = (wave + k * NW) * 16 + (lane >> 2);
    const int co = rowg % COT, tap = rowg / COT;
    const int lchunk = (lane & 3) ^ ((co >> 1) & 2);
    woff[k] = (unsigned)(((co0 + co) * 9 * a.C + tap * a.C + lchunk * 8) * 2);
  }
  auto issue = [&](int kc, int b) {
    char* S = smem + b * STAGE;
    const unsigned so = (unsigned)kc * 64u;
#pragma unroll
    for (int k = 0; k < H_PER; ++k)
      if (wave + k * NW < H_NINS) glds16s(xr, S + (wave + k * NW) * 1024, hoff[k], so);
#pragma unroll
    for (int k = 0; k < W_PER; ++k)
      if (wave + k * NW < W_NINS) glds16s(wr, S + HBYTES + (wave + k * NW) * 1024, woff[k], so);
  };
  set_hoff(tile);
  issue(0, 0);
  load_epi_constants<COT>(a, cst, co0, tid, NW * 64);

  const int aoff = ws_off(lane & 15, lane >> 4);
  int boff[RW + 2][3];
#pragma unroll
  for (int h = 0; h < RW + 2; ++h)
#pragma unroll
    for (int d = 0; d < 3; ++d) boff[h][d] = ws_off((wave * RW + h) * kHW + d + (lane & 15), lane >> 4);
  TSTAMP(a.tim, 1);
  const bool stats = a.stats || a.bb.sums;
  int stg = 0;  // stages so far: LDS buffer parity across tiles
  for (;;) {
    int n, oh0, ow0;
    tile_origin(tile, n, oh0, ow0);
    size_t pix[RW];
#pragma unroll
    for (int j = 0; j < RW; ++j) pix[j] = ((size_t)n * a.P + oh0 + wave * RW + j) * a.Q + ow0 + (lane & 15);
    const int next = tile + nslot;
    f32x4 acc[RW][FN];
#pragma unroll
    for (int j = 0; j < RW; ++j)
#pragma unroll
      for (int i = 0; i < FN; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    TileEpi<FN, RW, FLIP, PREF, TWO> epi;
    for (int kc = 0; kc < KC; ++kc, ++stg) {
      // stage kc landed (this wave's part) ...; at the first chunk of a later
      // tile the previous tile's epilogue stores (at least RW * FN / 2 per wave,
      // issued after this chunk's DMA) may stay in flight
      if (MT && kc == 0 && stg > 0) wait_vmcnt<RW * FN / 2>();
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();  // ... everyone's; and stage kc-1 is no longer read
      if (stg < 16) TSTAMP(a.tim, 2 + stg);
      if (kc + 1 < KC) {
        if (UNET_ABL != 2) issue(kc + 1, (stg + 1) & 1);
      } else {
        if (MT && next < ntiles) {  // the next tile's first chunk stages under this one's MFMAs
          set_hoff(next);
          issue(0, (stg + 1) & 1);
        }
        if (PREF) epi.fetch(a, pix, co0, lane);  // epilogue operands ride beside the last chunk
      }
      const char* S = smem + (stg & 1) * STAGE;
      if (UNET_ABL != 1) mfma_panel<FN, RW, COT * 64, FLIP>(acc, S + HBYTES, S, aoff, boff);
    }
    TSTAMP(a.tim, 20);
    if (!PREF) epi.fetch(a, pix, co0, lane);
    epi.landed();
    float q0[FN][4], q1[FN][4], q2[FN][4];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = q2[i][e] = 0.f;
    epi.store(a, acc, pix, co0, lane, cst, q0, q1, q2);
    TSTAMP(a.tim, 21);
    // per tile: the buffer of the last chunk is free once every wave is past
    // the barrier inside (the next tile's first chunk lands in the other one)
    if (stats) stats_atomics<FN, NW, TWO>(a, q0, q1, q2, co0, smem + ((stg - 1) & 1) * STAGE);
    tile = next;
    if (!MT || tile >= ntiles) break;
  }
  if (stats) stats_ticket<COT, NW>(a, smem);
  TSTAMP(a.tim, 22);
  TSTAMP_RT(a.tim, 31);
}

// ---------------------------------------------------------------------------
// stride-2 3x3 / pad-1 data gradient by output parity class (a, b):
//   dX[2i+a][2j+b] = sum of W[r][s] . dY[i + dr][j + ds] over the taps of the class,
//   a = 0: r = 1 (dr 0);  a = 1: r = 0 (dr 1), r = 2 (dr 0);  the same for b / s.
// A block owns class rows i0 .. i0+TI and class columns j0 .. j0+16 of all
// four classes (a 2TI x 32 tile of dX) and COT dX channels.  Per 32-channel
// chunk of dY it stages one (TI+1) x 18 dY halo and the chunk's 9 weight taps;
// each class is an MFMA over that halo at a (dr, ds) shift, so the dY tile
// crosses L2 -> LDS once for all 9 taps and 4 classes (the implicit-GEMM
// MODE_TRANS kernel stages it once per class and tap).  Every wave owns RW
// class rows of all four classes, i.e. the same 9 tap-MFMA sets per row as the
// stride-1 kernel.  EXT: the block's folded 1x1 / stride-2 downsample dgrad
// (x2 = dY_ds, w2) rides in the SAME stages (a TI x 16 dY_ds tile + its 1x1
// weights per chunk, C2 == C) and feeds class (0, 0) only: pixel (2i, 2j) reads
// dY_ds (i, j).  Epilogue: TileEpi per class.
// ---------------------------------------------------------------------------
template <int FN, int RW, int NW, bool EXT>
__global__ void __launch_bounds__(NW * 64) conv3x3s2_dgrad_kernel(ConvFwdArgs a, int ncb) {
  constexpr int COT = FN * 16;
  constexpr int TI = RW * NW;
  constexpr int HR = TI + 1;
  constexpr int HPR = (HR * kHW + 15) / 16 * 16;
  constexpr int HBYTES = HPR * 64;
  constexpr int WBYTES = 9 * COT * 64;
  constexpr int DBYTES = EXT ? TI * 16 * 64 : 0;  // dY_ds tile
  constexpr int D2BYTES = EXT ? COT * 64 : 0;     // 1x1 weights
  constexpr int STAGE = HBYTES + WBYTES + DBYTES + D2BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* cst = reinterpret_cast<float*>(smem + 2 * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cob = bid % ncb, tile = bid / ncb;
  const int co0 = cob * COT;
  const int tq = a.W >> 4, tp = a.H / TI;  // class grid = the dY grid
  const int n = tile / (tp * tq);
  const int rem = tile - n * (tp * tq);
  const int i0 = (rem / tq) * TI, j0 = (rem % tq) << 4;
  const int KC = a.C >> 5;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, (unsigned)((size_t)a.N * a.H * a.W * a.ldx * 2));
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (unsigned)((size_t)a.Cout * 9 * a.C * 2));
  const __amdgpu_buffer_rsrc_t x2r =
      make_rsrc(EXT ? a.x2 : a.x, EXT ? (unsigned)((size_t)a.N * a.H * a.W * a.ldx2 * 2) : 0u);
  const __amdgpu_buffer_rsrc_t w2r = make_rsrc(EXT ? a.w2 : a.w, EXT ? (unsigned)((size_t)a.Cout * a.C2 * 2) : 0u);

  constexpr int H_NINS = HPR / 16, H_PER = (H_NINS + NW - 1) / NW;
  constexpr int W_NINS = 9 * COT / 16, W_PER = (W_NINS + NW - 1) / NW;
  constexpr int D_NINS = EXT ? TI : 0, D_PER = EXT ? (D_NINS + NW - 1) / NW : 1;
  constexpr int W2_NINS = EXT ? COT / 16 : 0, W2_PER = EXT ? (W2_NINS + NW - 1) / NW : 1;
  unsigned hoff[H_PER], woff[W_PER], doff[D_PER], woff2[W2_PER];
#pragma unroll
  for (int k = 0; k < H_PER; ++k) {
    const int hp = (wave + k * NW) * 16 + (lane >> 2);
    const int lchunk = (lane & 3) ^ ((hp >> 1) & 2);
    const int hr = hp / kHW, hc = hp - hr * kHW;
    const int ih = i0 + hr, iw = j0 + hc;
    const bool ok = hp < HR * kHW && ih < a.H && iw < a.W;
    hoff[k] = ok ? (unsigned)(((((size_t)n * a.H + ih) * a.W + iw) * a.ldx + lchunk * 8) * 2) : kOOB;
  }
#pragma unroll
  for (int k = 0; k < W_PER; ++k) {
    const int rowg = (wave + k * NW) * 16 + (lane >> 2);
    const int co = rowg % COT, tap = rowg / COT;
    const int lchunk = (lane & 3) ^ ((co >> 1) & 2);
    woff[k] = (unsigned)(((co0 + co) * 9 * a.C + tap * a.C + lchunk * 8) * 2);
  }
#pragma unroll
  for (int k = 0; k < D_PER; ++k) {  // dY_ds tile row (class row) = instruction index
    const int dp = (wave + k * NW) * 16 + (lane >> 2);
    const int lchunk = (lane & 3) ^ ((dp >> 1) & 2);
    const int ih = i0 + (dp >> 4), iw = j0 + (dp & 15);
    doff[k] = EXT ? (unsigned)(((((size_t)n * a.H + ih) * a.W + iw) * a.ldx2 + lchunk * 8) * 2) : kOOB;
  }
#pragma unroll
  for (int k = 0; k < W2_PER; ++k) {
    const int co = (wave + k * NW) * 16 + (lane >> 2);
    const int lchunk = (lane & 3) ^ ((co >> 1) & 2);
    woff2[k] = EXT ? (unsigned)(((co0 + co) * a.C2 + lchunk * 8) * 2) : kOOB;
  }
  auto issue = [&](int kt, int b) {
    char* S = smem + b * STAGE;
    const unsigned so = (unsigned)kt * 64u;
#pragma unroll
    for (int k = 0; k < H_PER; ++k)
      if (wave + k * NW < H_NINS) glds16s(xr, S + (wave + k * NW) * 1024, hoff[k], so);
#pragma unroll
    for (int k = 0; k < W_PER; ++k)
      if (wave + k * NW < W_NINS) glds16s(wr, S + HBYTES + (wave + k * NW) * 1024, woff[k], so);
    if constexpr (EXT) {
#pragma unroll
      for (int k = 0; k < D_PER; ++k)
        if (wave + k * NW < D_NINS) glds16s(x2r, S + HBYTES + WBYTES + (wave + k * NW) * 1024, doff[k], so);
#pragma unroll
      for (int k = 0; k < W2_PER; ++k)
        if (wave + k * NW < W2_NINS)
          glds16s(w2r, S + HBYTES + WBYTES + DBYTES + (wave + k * NW) * 1024, woff2[k], so);
    }
  };
  issue(0, 0);
  load_epi_constants<COT>(a, cst, co0, tid, NW * 64);

  const int aoff = ws_off(lane & 15, lane >> 4);
  int boff[RW + 1][2], doffl[RW];
#pragma unroll
  for (int h = 0; h < RW + 1; ++h)
#pragma unroll
    for (int d = 0; d < 2; ++d) boff[h][d] = ws_off((wave * RW + h) * kHW + d + (lane & 15), lane >> 4);
#pragma unroll
  for (int j = 0; j < RW; ++j) doffl[j] = ws_off((wave * RW + j) * 16 + (lane & 15), lane >> 4);

  f32x4 acc[4 * RW][FN];
#pragma unroll
  for (int q = 0; q < 4 * RW; ++q)
#pragma unroll
    for (int i = 0; i < FN; ++i) acc[q][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one tap of class c: weight tap (r, s), halo shift (dr, ds)
  auto tap_mfma = [&](const char* W, const char* Hh, int c, int r, int dr, int s, int ds) {
    bf16x8 A[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) A[i] = *reinterpret_cast<const bf16x8*>(W + (r * 3 + s) * COT * 64 + i * 1024 + aoff);
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const bf16x8 B = *reinterpret_cast<const bf16x8*>(Hh + boff[j + dr][ds]);
#pragma unroll
      for (int i = 0; i < FN; ++i)
        acc[c * RW + j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B, acc[c * RW + j][i], 0, 0, 0);
    }
  };
  for (int kt = 0; kt < KC; ++kt) {
    wait_vmcnt<0>();               // stage kt landed (this wave's part) ...
    __builtin_amdgcn_s_barrier();  // ... everyone's; and stage kt-1 is no longer read
    if (kt + 1 < KC) issue(kt + 1, (kt + 1) & 1);
    const char* S = smem + (kt & 1) * STAGE;
    const char* W = S + HBYTES;
    tap_mfma(W, S, 0, 1, 0, 1, 0);                                 // (0, 0)
    tap_mfma(W, S, 1, 1, 0, 0, 1); tap_mfma(W, S, 1, 1, 0, 2, 0);  // (0, 1)
    tap_mfma(W, S, 2, 0, 1, 1, 0); tap_mfma(W, S, 2, 2, 0, 1, 0);  // (1, 0)
    tap_mfma(W, S, 3, 0, 1, 0, 1); tap_mfma(W, S, 3, 0, 1, 2, 0);  // (1, 1)
    tap_mfma(W, S, 3, 2, 0, 0, 1); tap_mfma(W, S, 3, 2, 0, 2, 0);
    if constexpr (EXT) {  // downsample: class (0, 0), 1x1 weights, no shift
      const char* D = S + HBYTES + WBYTES;
      bf16x8 A[FN];
#pragma unroll
      for (int i = 0; i < FN; ++i) A[i] = *reinterpret_cast<const bf16x8*>(D + DBYTES + i * 1024 + aoff);
#pragma unroll
      for (int j = 0; j < RW; ++j) {
        const bf16x8 B = *reinterpret_cast<const bf16x8*>(D + doffl[j]);
#pragma unroll
        for (int i = 0; i < FN; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[i], B, acc[j][i], 0, 0, 0);
      }
    }
  }
  float q0[FN][4], q1[FN][4], q2[FN][4];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) q0[i][e] = q1[i][e] = q2[i][e] = 0.f;
  // one class at a time: its epilogue operands are the only ones live
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    size_t pix[RW];
    f32x4 ac[RW][FN];
#pragma unroll
    for (int j = 0; j < RW; ++j) {
      const int oh = 2 * (i0 + wave * RW + j) + (c >> 1), ow = 2 * (j0 + (lane & 15)) + (c & 1);
      pix[j] = ((size_t)n * a.P + oh) * a.Q + ow;
#pragma unroll
      for (int i = 0; i < FN; ++i) ac[j][i] = acc[c * RW + j][i];
    }
    TileEpi<FN, RW, true, false, false> epi;
    epi.fetch(a, pix, co0, lane);
    epi.store(a, ac, pix, co0, lane, cst, q0, q1, q2);
  }
  if (a.bb.sums) commit_stats<FN, NW, false>(a, q0, q1, q2, co0, smem);
}

template <int FN, int RW, int NW, bool EXT>
static hipError_t launch_s2d(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int COT = FN * 16, TI = RW * NW;
  constexpr int HPR = ((TI + 1) * kHW + 15) / 16 * 16;
  constexpr size_t stage = (size_t)HPR * 64 + 9 * COT * 64 + (EXT ? (size_t)TI * 16 * 64 + COT * 64 : 0);
  constexpr size_t lds = 2 * stage + kEpiConsts * COT * sizeof(float);
  static_assert(lds <= 163840, "LDS");
  static_assert((size_t)NW * COT * 3 * sizeof(float) + sizeof(int) <= 2 * stage, "stats scratch");
  const int ncb = a.Cout / COT;
  const int ntiles = a.N * (a.H / TI) * (a.W / 16);
  char tag[96];
  std::snprintf(tag, sizeof(tag), "conv3x3s2_dgrad_kernel<%d, %d, %d, %s>", FN, RW, NW, EXT ? "true" : "false");
  conv_kernel_tag(tag);
  hipLaunchKernelGGL((conv3x3s2_dgrad_kernel<FN, RW, NW, EXT>), dim3(ntiles * ncb), dim3(NW * 64), lds, st, a, ncb);
  return hipGetLastError();
}

template <int FN, int RW, int NW>
static hipError_t launch_s2d_ext(const ConvFwdArgs& a, hipStream_t st) {
  return a.x2 ? launch_s2d<FN, RW, NW, true>(a, st) : launch_s2d<FN, RW, NW, false>(a, st);
}

static int g_s2_disabled = std::getenv("UNET_NO_S2HALO") != nullptr;  // A/B switch for measurements

// 3x3 / stride-2 / pad-1 data gradient (+ the folded 1x1 / s2 downsample
// dgrad) when the shape is covered; hipErrorNotSupported otherwise (the caller
// falls back to the implicit-GEMM MODE_TRANS kernel).  a: x = dY [N,H,W,C],
// y = dX [N,P=2H,Q=2W,Cout], w = dgrad pack [Cout][9][C].
hipError_t launch_conv3x3s2_dgrad(const ConvFwdArgs& a, hipStream_t st) {
  if (g_s2_disabled || a.ysplit || a.fold_on || a.stats || a.bias) return hipErrorNotSupported;
  if (a.R != 3 || a.S != 3 || a.stride != 2 || a.pad != 1) return hipErrorNotSupported;
  if (a.P != 2 * a.H || a.Q != 2 * a.W || a.W % 16 || a.C % 32 || a.Cout % 64) return hipErrorNotSupported;
  if (a.ldx % 8 || a.ldy % 4 || (a.x2 && (a.C2 != a.C || a.ldx2 % 8))) return hipErrorNotSupported;
  if ((a.add && a.ldadd % 4) || (a.bb.sums && (a.bb.y2 || a.bb.ldact % 4 || a.bb.ldy % 4)))
    return hipErrorNotSupported;
  if ((size_t)a.N * a.H * a.W * a.ldx * 2 >= 0x80000000ull) return hipErrorNotSupported;
  if (a.x2 && (size_t)a.N * a.H * a.W * a.ldx2 * 2 >= 0x80000000ull) return hipErrorNotSupported;
  if ((size_t)a.Cout * 9 * a.C * 2 >= 0x80000000ull) return hipErrorNotSupported;
  const long long ncb = a.Cout / 64;
  auto fits = [&](int ti) { return a.H % ti == 0; };
  auto blocks = [&](int ti) { return (long long)a.N * (a.H / ti) * (a.W / 16) * ncb; };
  // measured (16 x 512^2 Base, round-2 tile sweep): 16-row tiles while they fill
  // the chip (enc2.0: 51 us, was 79 on the implicit-GEMM kernel), else 32-channel
  // blocks of 8 rows (enc3.0 36 us, was 49; enc4.0 33 us, was 52)
  if (fits(16) && blocks(16) >= 256) return launch_s2d_ext<4, 2, 8>(a, st);
  if (fits(8)) return launch_s2d_ext<2, 1, 8>(a, st);
  if (fits(4)) return launch_s2d_ext<2, 1, 4>(a, st);
  return hipErrorNotSupported;
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
template <int NP, int FN, int TH, int NW, bool FLIP>
static hipError_t launch_ws(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int COT = FN * 16;
  constexpr int HPR = ((TH + 2) * kHW + 15) / 16 * 16;
  constexpr size_t lds = (size_t)9 * NP * COT * 64 + 2 * (size_t)NP * HPR * 64 + kEpiConsts * COT * sizeof(float) +
                         (FLIP ? 0 : 2 * NP * 32 * sizeof(float));
  static_assert(lds <= 163840, "LDS");
  const int ncg = (a.Cout + COT - 1) / COT;
  const int ntiles = a.N * (a.P / TH) * (a.Q / 16);
  const int per_cu = 163840 / (int)lds >= 2 ? 2 : 1;  // resident blocks per CU (LDS-limited)
  int slots = 256 * per_cu / ncg;
  if (slots > ntiles) slots = ntiles;
  if (slots < 1) slots = 1;
  char tag[96];
  std::snprintf(tag, sizeof(tag), "conv3x3_ws_kernel<%d, %d, %d, %d, %s>", NP, FN, TH, NW, FLIP ? "true" : "false");
  conv_kernel_tag(tag);
  hipLaunchKernelGGL((conv3x3_ws_kernel<NP, FN, TH, NW, FLIP>), dim3(slots * ncg), dim3(NW * 64), lds, st, a,
                     ntiles, ncg);
  return hipGetLastError();
}

template <int FN, int TH, int NW, bool FLIP, bool TWO>
static hipError_t launch_hs(const ConvFwdArgs& a, hipStream_t st) {
  constexpr int COT = FN * 16;
  constexpr int HPR = ((TH + 2) * kHW + 15) / 16 * 16;
  constexpr size_t lds = 2 * ((size_t)HPR * 64 + 9 * COT * 64) + kEpiConsts * COT * sizeof(float);
  static_assert(lds <= 163840, "LDS");
  if (a.Cout % COT || a.P % TH) return hipErrorNotSupported;
  const int ncb = a.Cout / COT;
  const int ntiles = a.N * (a.P / TH) * (a.Q / 16);
  // two 80 KB blocks per CU: past 512 blocks the grid stays at 512 and each
  // block walks several tiles
  constexpr int slots_env = 512;
  // (forward only: the multi-tile data gradient holds its fused BN-backward
  // epilogue operands across tiles, 324 VGPRs, one block per CU)
  long long grid = (long long)ntiles * ncb;
  if (!FLIP && slots_env > 0 && grid > slots_env && slots_env % ncb == 0) grid = slots_env;
  const bool mt = grid < (long long)ntiles * ncb;
  char tag[96];
  std::snprintf(tag, sizeof(tag), "conv3x3_hs_kernel<%d, %d, %d, %s, %s, %s>", FN, TH, NW, FLIP ? "true" : "false",
                TWO ? "true" : "false", mt ? "true" : "false");
  conv_kernel_tag(tag);
  if constexpr (!FLIP) {
    if (mt) {
      hipLaunchKernelGGL((conv3x3_hs_kernel<FN, TH, NW, FLIP, TWO, true>), dim3((unsigned)grid), dim3(NW * 64), lds,
                         st, a, ncb, ntiles);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL((conv3x3_hs_kernel<FN, TH, NW, FLIP, TWO, false>), dim3((unsigned)grid), dim3(NW * 64), lds, st,
                     a, ncb, ntiles);
  return hipGetLastError();
}

template <bool FLIP>
static hipError_t launch_halo_shape(const ConvFwdArgs& a, hipStream_t st) {
  const int C = a.C, Co = a.Cout;
  // dgrad producing dA of a downsample block's BN pair (bn2 + downsample BN):
  // the halo-streamed kernel with the two-BN epilogue
  if (FLIP && a.bb.sums && a.bb.y2) {
    if (!(C % 32 == 0 && C >= 128 && Co % 64 == 0)) return hipErrorNotSupported;
    // 32-channel blocks, 8 waves (two blocks per CU): enc2-4 downsample-block
    // dgrads 63 / 49 / 42 -> 56 / 40 / 35 us (Base, measured)
    if (a.P % 16 == 0 && Co % 32 == 0) return launch_hs<2, 16, 8, true, true>(a, st);
    const long long t16 = (long long)a.N * (a.P / 16) * (a.Q / 16) * (Co / 64);
    if (a.P % 16 == 0 && t16 >= 256) return launch_hs<4, 16, 8, true, true>(a, st);
    if (a.P % 8 == 0) return launch_hs<4, 8, 4, true, true>(a, st);
    return hipErrorNotSupported;
  }
  // weight-stationary: every tap of the block's channels fits in LDS
  if (C == 64 && conv3x3_ws2_ok(a, FLIP)) return launch_conv3x3_ws2(a, FLIP ? 1 : 0, st);
  if (C == 64 && Co % 64 == 0 && a.P % 16 == 0) return launch_ws<2, 4, 16, 8, FLIP>(a, st);
  // decoder1 shapes (256^2, 96 / 32 channels), round-3 sweep on the Base
  // config: 8-row tiles on 8 waves (one row each, two waves per SIMD hide each
  // other's LDS latency) beat the 4-wave and 16-row tiles except for the 32->32
  // forward (decoder1.0 dgrad 140 -> 111 us: the FN = 6 block spilled 36
  // VGPRs; decoder1.0 fwd 121 -> 104, decoder1.3 dgrad 60 -> 55)
  if (C == 32 && Co == 32 && a.P % 16 == 0) {
    if (FLIP) return launch_ws<1, 2, 8, 8, FLIP>(a, st);
    return launch_ws<1, 2, 16, 4, FLIP>(a, st);
  }
  // decoder1.0's data gradient (32 -> 96): 16-row tiles on 4 waves, 4 rows
  // each, with the per-shift halo-row reuse of mfma_panel (round 6 sweep:
  // 118 -> 104 us; the same tiles for the forwards and decoder1.3 were slower)
  if (C == 32 && Co == 96 && a.P % 16 == 0) {
    if (FLIP) return launch_ws<1, 2, 16, 4, FLIP>(a, st);
    return launch_ws<1, 2, 8, 8, FLIP>(a, st);
  }
  if (C == 32 && Co % 64 == 0 && a.P % 16 == 0) return launch_ws<1, 4, 16, 8, FLIP>(a, st);
  if (C == 96 && Co == 32 && a.P % 8 == 0) return launch_ws<3, 2, 8, 8, FLIP>(a, st);
  // halo-streamed: 256-pixel tiles while they still give >= ~1 block per CU
  if (C % 32 == 0 && C >= 128 && Co % 64 == 0) {
    const long long t16 = (long long)a.N * (a.P / 16) * (a.Q / 16) * (Co / 64);
    // round 1 ran the C = 128 forwards (enc2, decoder3.3) as a 128x128 im2col
    // tile (faster than the 64-channel halo blocks then); the 32-channel
    // halo blocks below beat it (37-43 -> 31 us)
    // 32-channel output blocks (80 KB of LDS: two blocks per CU, so one
    // block's epilogue overlaps the other's MFMAs; measured on the Base
    // config: enc3/decoder4 dgrads -5..-7 %, enc4 -11..-19 %): 8 waves when
    // the grid is one round, else 4 waves with 4 rows each
    if (a.P % 16 == 0 && Co % 32 == 0) {
      const long long b32 = (long long)a.N * (a.P / 16) * (a.Q / 16) * (Co / 32);
      if (b32 <= 256) return launch_hs<2, 16, 8, FLIP, false>(a, st);
      return launch_hs<2, 16, 4, FLIP, false>(a, st);
    }
    if (a.P % 16 == 0 && t16 >= 256) return launch_hs<4, 16, 8, FLIP, false>(a, st);
    if (a.P % 8 == 0) return launch_hs<4, 8, 4, FLIP, false>(a, st);
  }
  return hipErrorNotSupported;
}


// the default weight-stationary selections of launch_halo_shape<false> (the
// launcher checks the same; xform is only supported there)
static bool ws_fwd_shape(const ConvFwdArgs& a) {
  const int C = a.C, Co = a.Cout;
  return (C == 64 && Co % 64 == 0 && a.P % 16 == 0) || (C == 32 && Co == 32 && a.P % 16 == 0) ||
         (C == 32 && Co == 96 && a.P % 16 == 0) || (C == 32 && Co % 64 == 0 && a.P % 16 == 0) ||
         (C == 96 && Co == 32 && a.P % 8 == 0);
}

bool conv3x3_ws_xform_ok(const ConvFwdArgs& a) {
  return a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 && a.H == a.P &&
         a.W == a.Q && a.Q % 16 == 0 && a.ldx % 8 == 0 && a.ldy % 4 == 0 && !a.x2 && !a.fold_on && !a.add &&
         !a.bb.sums && a.ldxh % 8 == 0 && ws_fwd_shape(a) && (size_t)a.N * a.H * a.W * a.ldx * 2 < 0x80000000ull;
}

// 3x3 / s1 / p1 conv (mode 0) or its data gradient (mode 1, dgrad weight pack)
// when the shape is covered; hipErrorNotSupported otherwise (the caller falls
// back to the implicit-GEMM kernel).
hipError_t launch_conv3x3_ws(const ConvFwdArgs& a, int mode, hipStream_t st) {
  if (a.x2) return hipErrorNotSupported;
  if (a.R != 3 || a.S != 3 || a.stride != 1 || a.pad != 1) return hipErrorNotSupported;
  if (a.H != a.P || a.W != a.Q || a.Q % 16 || a.ldx % 8 || a.ldy % 4) return hipErrorNotSupported;
  // fused BN-backward epilogue operands are read 4 channels (8 B) at a time
  if ((a.add && a.ldadd % 4) ||
      (a.bb.sums && (a.bb.ldact % 4 || a.bb.ldy % 4 || (a.bb.y2 && a.bb.ldy2 % 4))))
    return hipErrorNotSupported;
  if ((size_t)a.N * a.H * a.W * a.ldx * 2 >= 0x80000000ull) return hipErrorNotSupported;
  if ((size_t)a.Cout * 9 * a.C * 2 >= 0x80000000ull) return hipErrorNotSupported;
  // forward epilogue: bias, BN sums, or the eval-folded BN (+ residual addend, ReLU)
  if (mode == 0 && (a.bb.sums || (a.add && !a.fold_on))) return hipErrorNotSupported;
  if (mode == 1 && a.fold_on) return hipErrorNotSupported;
  if (a.xform && (mode != 0 || !conv3x3_ws_xform_ok(a))) return hipErrorInvalidValue;
  return mode == 0 ? launch_halo_shape<false>(a, st) : launch_halo_shape<true>(a, st);
}

}  // namespace unet

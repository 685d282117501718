// Kernel argument blocks and launchers (internal to libunet_hip.so).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace unet {

typedef unsigned short bf16_t;

// CU count of the current device (cached per device id; queried on first use,
// which initialises the HIP runtime: unet_plan_create calls it)
int device_cu_count();

// in-kernel phase timing buffer geometry (common.h TSTAMP, debug build only)
constexpr int kTimBlocks = 1024, kTimSlots = 32, kTimLaunches = 320;

// MODE_SHUF: ConvTranspose2d(k2, s2) forward as ONE 1x1 GEMM over the input
// pixels with 4*Cout columns (j = (a*2+b)*Cout + co) and a pixel-shuffle store
// y[2i+a, 2j+b, co]; every input pixel is staged once instead of once per
// output parity class.
enum { MODE_FWD = 0, MODE_TRANS = 1, MODE_STEM = 2, MODE_SHUF = 3 };

// Per-channel fp64 reductions (BN sums) are spread over kStatRep replicas of
// [2][C] (replica = blockIdx.x % kStatRep) so thousands of blocks do not all
// hit the same addresses (MI355X_MICROARCH.md, float atomics "contention");
// readers sum the replicas.  Layout everywhere: [kStatRep][2][C].
constexpr int kStatRep = 16;
enum { ALOAD_NHWC = 0, ALOAD_STEM = 1 };
// XLOAD_SHUF: ConvTranspose2d(k2,s2) weight gradient as one GEMM over the
// INPUT pixels: dW[ci][t][co] = sum_px X[px][ci] * dY[2i + t/2, 2j + t%2][co]
// (x = dY gathered 4 output pixels per input pixel, C = 4*Co, R = S = 1)
enum { XLOAD_NHWC = 0, XLOAD_STEM = 1, XLOAD_SHUF = 2 };

// BatchNorm parameters of one layer.  Training: the producer of the batch sums
// (conv epilogue) finalises them in its LAST block (ticket counter) into
// ss = {scale[C], shift[C]}, save_mean/save_invstd and the running stats;
// consumers then only read ss.  Eval: scale/shift from the running stats.
struct BnLaunch {
  const double* stats; const float* gamma; const float* beta;
  float* run_mean; float* run_var; float* save_mean; float* save_invstd;
  double count; int C; float eps, momentum; int training;
  float* ss;          // [2][C] scale | shift (written by the finaliser)
  unsigned* ticket;   // zeroed per step; last arriving block finalises
  long long* nbt;     // num_batches_tracked (int64), += 1 with channel 0's running stats; null: untouched
};

// backward: dZ = dA * (A > 0); sums over pixels of dZ and dZ*xhat (and for bn2)
struct BnBwdArgs {
  const bf16_t* da; int ldda;
  const bf16_t* act; int ldact;      // forward output (relu mask source)
  const bf16_t* y; int ldy;          // raw conv output of bn
  const bf16_t* y2; int ldy2;        // raw conv output of bn2 (downsample) or null
  const float* mean; const float* invstd; const float* gamma;
  const float* mean2; const float* invstd2; const float* gamma2;
  double* sums;                      // [2][C]: sum dZ, sum dZ*xhat
  double* sums2;                     // [2][C] for bn2
  bf16_t* dy; int lddy;              // apply: dY out
  bf16_t* dy2; int lddy2;            // apply: dY2 out (bn2)
  bf16_t* dres; int lddres;          // apply: dZ out (identity residual) or null
  float* dgamma; float* dbeta;       // param grads (written by the reduce's last block)
  float* dgamma2; float* dbeta2;
  unsigned* ticket;                  // zeroed per step; reduce's last block finalises
  float* coef;                       // [5][C]: k1, mean dZ, mean dZ*xhat, k1b, mean dZ*xhat2
  int64_t npix; int C; int relu;
};
// fp8 per-tensor scale state (fp8.hip): amax of the previous step (the scale
// in use), amax accumulating this step (float bits), e8m0 dequant code 127 - e
struct F8State { unsigned prev_bits; unsigned cur_bits; int code; int pad; };

struct ConvFwdArgs {
  const bf16_t* x; int ldx;      // input NHWC bf16, channel stride ldx (stem: fp32 [N,H,W])
  const bf16_t* w;               // packed weights [Cout][R*S*C] (stem: [64][64])
  const bf16_t* wch;             // chunk-major 3x3 pack [C/32][9][Cout][32] (conv3x3_fl_kernel)
  bf16_t* y; int ldy;            // output NHWC bf16
  const float* bias;             // [Cout] or null
  const bf16_t* add; int ldadd;  // optional addend (same pixel grid as y)
  double* stats;                 // optional BN sums [kStatRep][2][Cout] (fp64 atomics)
  BnLaunch bn;                   // finalised by the last block when bn.ticket != null
  // fused BN(+ReLU) backward reduction (conv dgrad producing dA of a BN):
  // when bb.sums != null the epilogue writes dZ = dA * (act > 0) instead of dA
  // and adds sum dZ, sum dZ*xhat (and dZ*xhat2) into bb.sums / bb.sums2; the
  // last block runs bn_bwd_finalize (common.h).
  BnBwdArgs bb;
  // optional second reduction range of parity class 0 (MODE_TRANS only): the
  // 1x1 / stride-2 downsample dgrad folded into its block's conv1 dgrad.
  // Output pixels (2p, 2q) also get sum_k x2[n,p,q,k] * w2[co][k], k < C2.
  const bf16_t* x2; int ldx2; const bf16_t* w2; int C2;
  // optional split output: channels co >= csplit go to ysplit[pix*ldysplit +
  // co - csplit] instead of y (a concat gradient whose narrow up-conv part is
  // kept in its own dense buffer so its consumers read whole cache lines)
  bf16_t* ysplit; int ldysplit; int csplit;
  // eval-mode BatchNorm folded into the forward epilogue (fold_on != 0):
  // y = act( (conv + bias) * scale + shift [+ add] ), scale/shift per output
  // channel from the running statistics of `fold` (BnLaunch, training = 0);
  // act = ReLU when fold_relu.  `add` (forward) is the block's residual.
  BnLaunch fold; int fold_on; int fold_relu;
  // fp8 forward (launch_conv_fwd_f8): x / w are e4m3 bytes (x dense, ldx = C;
  // w packed [Cout][R*S*C]) whose dequant codes the kernel reads from f8x / f8w
  const F8State* f8x; const F8State* f8w;
  // BN(+ReLU) of the PREVIOUS conv applied while staging (xform != 0;
  // weight-stationary 3x3 forward, training): x holds that conv's raw output y,
  // every staged halo pixel becomes relu(y * scale + shift) of BN `xbn` (batch
  // statistics, bn_apply's expression, so bit-identical), padding stays 0, the
  // tile interior is stored to xh (= the BN+ReLU activation the backward
  // needs) and block 0 finalises that BN (saved / running statistics): the
  // standalone bn_apply pass disappears.
  BnLaunch xbn; bf16_t* xh; int ldxh; int xform;
  int N, H, W, C;                // input geometry (C = GEMM reduction channels)
  int P, Q, Cout;                // output geometry
  int R, S, stride, pad;
  // forward 3x3 / stride-2 conv1 of a downsample block with its 1x1 / stride-2
  // downsample folded in (MODE_FWD, launch_conv_fwd): wds = the downsample's
  // packed weights [Cout][C]; its output yds (+ BN sums stats_ds / bnds as
  // `stats` / `bn`) comes from the same staged input (the centre tap's K range)
  const bf16_t* wds; bf16_t* yds; int ldyds; double* stats_ds; BnLaunch bnds;
  // MODE_FWD implicit GEMM only: a column stride other than `stride` (0 = the
  // same).  The ConvTranspose data gradient runs as R = 2, S = 1, stride (2, 1)
  // over a view of dY that merges each pair of adjacent pixels into one of 2C
  // channels, so every K step stages whole 128-B lines (conv_dgrad)
  int stride_w;
  int mblocks, nblocks, Pc, Qc;  // filled by the launcher
  // persistent kernels (conv3x3_fl_kernel, convt2x2_kernel): 0 = one block per
  // CU (two for the up-conv); > 0 caps the grid (single-op tests: several
  // work items per block)
  int grid_cap;
  // ConvTranspose data gradient (launch_convt2x2 mode 1): the up-conv's bias
  // gradient, sum of dY, added into replicas [kStatRep][Co] (fp64), or null
  double* bias_acc;
  // in-kernel phase stamps (debug build -DUNET_TIMING only, null otherwise):
  // [block < kTimBlocks][kTimSlots] s_memtime values (scripts/conv_timing.py)
  unsigned long long* tim;
};

// Split-K partials of the weight-gradient kernels ("register-native" slab):
// every block stores its f32x4 accumulator fragments lane-contiguously (16 B
// per lane, 1 KiB per wave instruction) at unit
//   u = ((blk * nw + wave) * nf + frag) * 64 + lane     of split s: slab[s * units + u];
// wgrad_slab_reduce_kernel sums the splits in a FIXED order (s = 0, 1, ...) and
// scatters each unit's 4 values to dW [Cout][Krow]: deterministic, no atomics.
enum { SLAB_HALO = 0, SLAB_GEMM = 1, SLAB_STEM = 2 };
struct SlabLayout {
  int kind, splits, blocks, nw, nf;
  long long units;                 // f32x4 units per split
  int Cout, C, Krow, cmax;         // dW geometry (cmax: valid reduction columns per tap)
  int co_blocks, c_blocks;         // blk -> (co block, c block[, tap])
  int bmo, bnc, wm, wn, fn;        // GEMM tile (BMO x BNC, WM x WN waves, FN column frags)
  int ci, co32;                    // HALO: channels per block, 32-output-channel variant
  long long dw2_off;               // HALO + folded downsample: its dW [Cout][C] at dw + dw2_off (frags 18, 19)
};

struct ConvWgradArgs {
  const bf16_t* dy; int lddy;    // gradient wrt conv output [N,P,Q,Cout]
  const bf16_t* x; int ldx;      // conv input [N,H,W,C] (stem: fp32 image)
  float* dw;                     // fp32 dW [Cout][R*S*C] (stem: [64][64])
  // split-K partial scratch (16-B aligned).  With a slab every element of dW is
  // WRITTEN (plain stores, deterministic split order; dW need not be zeroed);
  // without one (single-op C ABI) the kernels add into a zeroed dW with fp32
  // atomics.
  float* slab; size_t slab_bytes;
  // bn_fuse != 0 (stem only): the stem does not store dY; it forms it while
  // loading, dY = A dZ + B y + C per channel, from the stem BN's backward sums
  // (bn.sums, reduced by the fused maxpool backward), bn.da = dZ, bn.y = the raw
  // stem conv output — the expression of bn_bwd_apply_kernel, so dY is bit-
  // identical — and writes the BN's dgamma / dbeta (block (0, group))
  BnBwdArgs bn; int bn_fuse;
  int N, H, W, C, P, Q, Cout, R, S, stride, pad;
  int px_per_split, co_blocks, c_blocks;  // filled by the launcher
  // stride-2 halo kernel only: the block's 1x1 / stride-2 downsample weight
  // gradient folded in (its input pixels are the centre tap's): dW2[co][c] =
  // sum dY2[px][co] x[2p][2q][c], dY2 with the same Cout (wgrad_s2_fold_ok)
  const bf16_t* dy2; int lddy2; float* dw2;
  unsigned long long* tim;  // phase stamps (debug build only), as ConvFwdArgs::tim
};
// the stride-2 halo weight gradient covers this shape (and then folds a.dy2)
bool wgrad_s2_fold_ok(const ConvWgradArgs& a);

hipError_t launch_conv_fwd(const ConvFwdArgs& a, int mode, hipStream_t st);
hipError_t launch_conv_fwd_v1(const ConvFwdArgs& a, int mode, hipStream_t st);  // register-staged
// weight-stationary halo kernel for 3x3/s1/p1 layers with few channels
// (conv_halo.hip); mode 0 conv, 1 dgrad.  hipErrorNotSupported if not covered.
hipError_t launch_conv3x3_ws(const ConvFwdArgs& a, int mode, hipStream_t st);
// the forward of this shape runs on the weight-stationary halo kernel, which
// supports ConvFwdArgs::xform (the BN-apply prologue)
bool conv3x3_ws_xform_ok(const ConvFwdArgs& a);
// full-line halo kernel (conv_fl.hip) for 3x3/s1/p1 layers with C % 128 == 0,
// Cout % 64 == 0 (P, Q multiples of 16): a.wch holds the chunk-major pack
// (PK_CONV_FWD_CH / PK_CONV_DGRAD_CH); mode 0 conv, 1 dgrad.  The plan packs
// those convs chunk-major exactly when conv3x3_fl_shape holds (UNET_NO_FL=1: never)
bool conv3x3_fl_shape(int N, int C, int Cout, int P, int Q);
// the geometry alone (what launch_conv3x3_fl accepts; the single-op C ABI may
// launch shapes that do not fill the chip)
bool conv3x3_fl_geom(int C, int Cout, int P, int Q);
hipError_t launch_conv3x3_fl(const ConvFwdArgs& a, int mode, hipStream_t st);
// ConvTranspose2d(k2, s2) (convt.hip): N, H, W = the INPUT-resolution grid, C =
// Ci, Cout = Co.  mode 0 forward: x = X [.., Ci], w = PK_CONVT_FWD pack, y = Y
// [N, 2H, 2W] (+ bias); mode 1 data gradient: x = dY [N, 2H, 2W, Co], w =
// PK_CONVT_DGRAD pack, y = dX (+ the fused BN backward bb, + bias_acc).
// hipErrorNotSupported for shapes it does not cover (the caller falls back to
// the implicit-GEMM path).
hipError_t launch_convt2x2(const ConvFwdArgs& a, int mode, hipStream_t st);
// forward with xform (the previous BN + ReLU applied to the pixel operand,
// the activation stored to xh, block 0 finalising that BN; training, no
// ticket): shape / stride test; the launch itself fails (no fallback) when an
// xform launch is not taken
bool convt2x2_xform_ok(const ConvFwdArgs& a);
// 1 x 1 / stride-1 conv as a weight-stationary per-pixel GEMM (convt.hip): mode
// 0 forward (w = forward pack [Cout][C], bias, BN sums `stats` / `bn`), mode 1
// data gradient (w = dgrad pack [C_out_of_op][C], a.C = dY channels, a.Cout =
// dX channels, optional `add`).  hipErrorNotSupported outside its (Cout, C)
// table {32, 64}^2 or for other epilogues (the caller falls back).
hipError_t launch_conv1x1(const ConvFwdArgs& a, int mode, hipStream_t st);
// does launch_conv_fwd fold the downsample (a.wds) into this 3x3 / stride-2
// forward's launch (geometry, tile choice)?  false: launch them separately
bool conv_fwd_ds_ok(const ConvFwdArgs& a);
// weight-stationary full-line conv for C == 64 (conv_fl.hip), standard weight
// pack; launch_conv3x3_ws uses it where conv3x3_ws2_ok holds (UNET_NO_WS2=1: never)
bool conv3x3_ws2_ok(const ConvFwdArgs& a, bool flip);
hipError_t launch_conv3x3_ws2(const ConvFwdArgs& a, int mode, hipStream_t st);
// 3x3 / stride-2 / pad-1 data gradient by parity class on a shared dY halo
// (conv_halo.hip), with the optional folded downsample (x2 / w2) range
hipError_t launch_conv3x3s2_dgrad(const ConvFwdArgs& a, hipStream_t st);
void set_conv_config(int cfg);  // 0: automatic tile selection, >0: fixed tile config (tuning)
hipError_t launch_conv_wgrad(const ConvWgradArgs& a, int stem, hipStream_t st);
// fp8 e4m3 implicit-GEMM forward conv (MODE_FWD geometry, any R/S/stride/pad,
// C % 16 == 0), block-scaled MFMA dequantizing with the F8State codes
hipError_t launch_conv_fwd_f8(const ConvFwdArgs& a, hipStream_t st);
// fp8.hip: delayed-amax quantization of activations / conv weights.  `calibrate`
// flags: F8_CALIBRATE = amax pass into prev first (a plan's first forward);
// F8_FROZEN = quantize with the scale in use and do NOT accumulate this call's
// amax (eval forwards: validation must not steer the next training step's scale)
enum { F8_CALIBRATE = 1, F8_FROZEN = 2 };
hipError_t launch_f8_roll(F8State* s, int n, hipStream_t st);
hipError_t launch_f8_quant_act(const bf16_t* x, int ld, int C, int64_t npix, uint8_t* q, F8State* s, int calibrate,
                               hipStream_t st);
hipError_t launch_f8_pack_w(const float* w, int Co, int Ci, int R, int S, uint8_t* dst, F8State* s, int calibrate,
                            hipStream_t st);
// ConvTranspose2d(k2,s2) weight gradient (XLOAD_SHUF): dy = X [N,P,Q,Ci] (Cout = Ci),
// x = dY [N,H=2P,W=2Q,Co] with C = 4*Co; dw [Ci][4][Co]
hipError_t launch_convt_wgrad(const ConvWgradArgs& a, hipStream_t st);
// sums the split-K slab of the preceding launch_conv_wgrad into dW (no-op when
// that launch needed no reduction: one split, or the atomic path)
hipError_t launch_wgrad_finish(hipStream_t st);
bool wgrad_pending();
// A split-K reduction riding as extra blocks [apply_blocks, apply_blocks +
// blocks) of the next BN-backward apply launch (same stream): the apply and the
// reduction are independent streaming passes, one launch boundary instead of
// two.  wgrad_defer() moves the pending reduction into the deferred slot (false
// if that slot is taken); wgrad_take_deferred() hands it to an apply launch;
// launch_wgrad_flush() runs a deferred one on its own.
struct ReduceTail {
  const void* slab; float* dw; SlabLayout L; int T; int blocks;
};
bool wgrad_defer();
bool wgrad_deferred();
// the deferred reduction reads this slab (it must run before the slab is refilled)
bool wgrad_deferred_reads(const void* slab);
bool wgrad_take_deferred(ReduceTail* t);
hipError_t launch_wgrad_flush(hipStream_t st);
void wgrad_reset();  // clears the pending and deferred slots (start of every backward)
hipError_t launch_slab_reduce(const ReduceTail& r, hipStream_t st);  // r on its own

// Batched 3x3 / stride-1 weight gradients (wgrad3x3_batch_kernel): the weight
// gradients of several layers (wgrad_batch_ok) in ONE stream-K launch.  Layer l
// has co_blocks x c_blocks units of 64 x 64 channels, each a K loop over `tiles`
// 128-pixel output tiles (32 x 4, or 16 x 8 for Q = 16: one geometry per launch); the units' items (unit, tile) are numbered layer by
// layer, unit by unit, and block b of the grid runs items [b I / G, (b+1) I / G).
// A unit inside one block is written to dW directly; a unit spread over blocks
// b0..b1 leaves one partial per block in the slab (slot b * maxseg + the unit's
// rank among block b's units), summed in block order by the reduce (fixed order:
// bit-reproducible).
constexpr int kWbMaxLayers = 16;
struct WgBatchLayer {
  const bf16_t* dy; const bf16_t* x; float* dw;
  int H, W, C, Cout, lddy, ldx, tq, tp, co_blocks, c_blocks, tiles, unit0;
  long long item0;
};
struct WgBatchArgs {
  WgBatchLayer L[kWbMaxLayers];
  int nl, grid, maxseg, units, N;
  int tw;                    // tile width of every layer: 32 (32 x 4 tiles) or 16 (16 x 8, Q = 16 layers)
  long long items;
  float* slab;               // grid * maxseg partials of 147,456 B
  unsigned long long* tim;   // phase stamps (debug build only)
};
bool wgrad_batch_ok(const ConvWgradArgs& a);
int wgrad_batch_tw(const ConvWgradArgs& a);  // the batch tile width of a layer (0: not batchable)
constexpr size_t kWbPartBytes = 8 * 18 * 64 * 16;  // one block's 64 x 64 x 9 fp32 partial (SLAB_HALO layout)
// the grid of a batch (one block per CU, at most kWbMaxGrid) and the largest slab slot count it needs
constexpr int kWbMaxGrid = 256;
int wgrad_batch_grid();
int wgrad_batch_maxseg(const WgBatchArgs& a);
hipError_t launch_wgrad_batch(const WgBatchArgs& a, hipStream_t st);
const char* last_kernel_tag();  // template instance of the last conv launch (profiler)

// ---- elementwise / reduction kernels (elementwise.hip) ----

// A = act( bn(Y) + residual ), residual: 0 none, 1 identity tensor R, 2 bn2(R)
struct BnApplyArgs {
  const bf16_t* y; int ldy;
  bf16_t* out; int ldo;
  const bf16_t* res; int ldr;
  BnLaunch bn, bn2;
  int64_t npix; int C; int res_mode; int relu;
};
hipError_t launch_bn_apply(const BnApplyArgs& a, hipStream_t st);

hipError_t launch_bn_bwd_reduce(const BnBwdArgs& a, hipStream_t st);
hipError_t launch_bn_bwd_apply(const BnBwdArgs& a, hipStream_t st);
// the same with a deferred split-K reduction as trailing blocks (256-thread
// apply blocks only, i.e. C % 64 == 0); hipErrorNotSupported otherwise
hipError_t launch_bn_bwd_apply_reduce(const BnBwdArgs& a, const ReduceTail& r, hipStream_t st);

struct MaxPoolArgs {
  const bf16_t* x; int ldx; bf16_t* y; int ldy; uint8_t* idx;
  const bf16_t* dy; int lddy; const bf16_t* add; int ldadd; bf16_t* dx; int lddx;
  int N, H, W, C, P, Q;
  // backward only, optional: dx is dA of a BN(+ReLU) (the stem BN); as in the
  // conv-dgrad epilogue, store dZ = dA * (act > 0) and run its BN-backward
  // reduction (bb.sums != null)
  BnBwdArgs bb;
  // forward, fused (launch_bn_relu_maxpool_fwd): x is the RAW conv output of
  // BN `bn`; act = relu(bn(x)) is written to act (every pixel once) and pooled
  BnLaunch bn; bf16_t* act; int ldact;
};
hipError_t launch_maxpool_fwd(const MaxPoolArgs& a, hipStream_t st);
// stem: BN apply + ReLU + MaxPool2d(3,2,1) in one pass over the raw conv output
hipError_t launch_bn_relu_maxpool_fwd(const MaxPoolArgs& a, hipStream_t st);
hipError_t launch_maxpool_bwd(const MaxPoolArgs& a, hipStream_t st);

// The stem by recompute (stem_rc.hip): conv 7x7/s2 (1 -> Cout) + BN + ReLU +
// MaxPool(3,2,1) without storing the raw conv output.  Forward: a statistics
// pass (mode 0: BN sums, last block finalises bn; y stored only when y != null,
// tests) and an apply pass (mode 1: act, pooled, idx).  Backward: dZ of the
// stem BN from dpool / idx / add (the maxpool backward, stored to dz only when
// dz != null) and, in the same pass, partial sums of dZ^T im2col, xhat^T
// im2col, im2col, dZ, dZ xhat per block (part); a fixed-order reduce (tot,
// tot64) and a finalise write dw [Cout][64], dgamma, dbeta.
struct StemRcArgs {
  const float* img; int H, W;        // fp32 [N][H][W]
  const bf16_t* w;                   // packed [Cout][64] bf16
  int N, P, Q, Cout, Pp, Qp;         // conv output P x Q, pooled Pp x Qp
  double* stats; BnLaunch bn;        // BN of the stem (bn.ss: scale | shift)
  bf16_t* y; int ldy;
  bf16_t* act; int ldact;
  bf16_t* pool; int ldpool; uint8_t* idx;   // idx [pixel][Cout]
  const bf16_t* dpool; int lddpool;
  const bf16_t* add; int ldadd;
  const float* mean; const float* invstd;   // saved batch statistics
  bf16_t* dz; int lddz;
  float* part; double* l2; double* tot;   // partials, fp64 level-1 sums, fp64 totals
  unsigned* tkt;                     // reduce tickets (stem_rc_tickets(Cout) words, zeroed)
  float* imsum;                      // [256] fixed-order block sums of img (backward centring)
  float* dw; float* dgamma; float* dbeta;
  int64_t npix;
  unsigned long long* tim;           // phase stamps (debug build only)
};
bool stem_rc_ok(int Cout, int P, int Q);
hipError_t launch_stem_rc_fwd(const StemRcArgs& a, int mode, hipStream_t st);
// stage 0: the fused backward pass; stage 1: the fixed-order reduce + finalise (one launch)
hipError_t launch_stem_rc_bwd(const StemRcArgs& a, int stage, hipStream_t st);
int stem_rc_tickets(int Cout);
constexpr int kStemTickets = 1024;  // ticket words the executor reserves
size_t stem_rc_part_bytes(int N, int P, int Q, int Cout);  // a.part followed by a.l2
size_t stem_rc_tot_bytes(int Cout);                        // a.tot followed by a.imsum
size_t stem_rc_imsum_offset(int Cout);                     // bytes from a.tot to a.imsum
size_t stem_rc_l2_offset(int N, int P, int Q, int Cout);   // bytes from a.part to a.l2

// fused ConvTranspose2d(k2,s2, Cin->16) + Conv1x1(16->1): logits[2i+a,2j+b] =
// c0 + sum_c X[i,j,c] V[c][a][b],  V[c][ab] = sum_o Wf[o] W0[c][o][ab].
struct HeadArgs {
  const bf16_t* x; int ldx;          // decoder1 output [N,H,W,Cin]
  const float* w0; const float* b0;  // upconv0 weight [Cin][Co][2][2], bias [Co]
  const float* wf; const float* bf;  // conv_final weight [1][Co][1][1], bias [1]
  float* logits;                     // [N,2H,2W]
  const float* dl;                   // backward: dL/dlogits
  bf16_t* dx; int lddx;              // backward: dL/dX
  double* usum;                      // backward: [kStatRep][Cin*4 + 1] sums U[c][ab], S (zeroed replicas)
  float* gw0; float* gb0; float* gwf; float* gbf;  // param grads
  // backward, optional (bb.sums != null): dX is dA of decoder1's last
  // BN+ReLU; as in the conv-dgrad epilogue, dZ = dA * (act > 0) is stored and
  // the BN-backward sums (dZ, dZ*xhat) are reduced here (bn_bwd apply follows)
  BnBwdArgs bb;
  // optional (bn_fold != 0): x is decoder1's raw conv output y and the head
  // forms its input act = bf16(relu(bn(y))) itself, in both passes; decoder1's
  // last BN apply pass and its activation buffer drop out.  The forward's
  // block 0 finalises the batch statistics as bn_apply_kernel would; the
  // backward needs bb (its fused sums) with bb.y == x.
  BnLaunch bn;
  int bn_fold;
  int N, H, W, Cin, Co;
};
hipError_t launch_head_fwd(const HeadArgs& a, hipStream_t st);
hipError_t launch_head_bwd(const HeadArgs& a, hipStream_t st);
hipError_t launch_head_grads(const HeadArgs& a, hipStream_t st);

// per-channel sum over pixels (ConvTranspose bias grads): acc[r][c] += partial
// sums of x[px][c] (acc: fp64 [kStatRep][C], zeroed); an UP_D2F unpack entry
// (or launch_d2f) then writes dst[c] = sum_r acc[r][c]
hipError_t launch_channel_sum(const bf16_t* x, int ldx, int64_t npix, int C, double* acc,
                              hipStream_t st);
hipError_t launch_d2f(const double* src, float* dst, int n, hipStream_t st);
// the same over replicas `stride` elements apart (src[r * stride + i], r < kStatRep)
hipError_t launch_d2f_strided(const double* src, float* dst, int n, int stride, hipStream_t st);

// weight (un)packing between torch fp32 layouts and kernel bf16 layouts
// PK_CONV_*_CH: 3x3 convs of conv3x3_fl_kernel, chunk-major [K/32][9][Cout'][32]
// (forward: K = Ci, Cout' = Co; data gradient: K = Co, Cout' = Ci)
// PK_ZERO: 16-B units dst[0 .. Co) = 0 (the step's zeroed workspace region, no fill launch)
enum { PK_CONV_FWD = 0, PK_CONV_DGRAD = 1, PK_CONVT_FWD = 2, PK_CONVT_DGRAD = 3, PK_STEM = 4, PK_CONV_FWD_CH = 5,
       PK_CONV_DGRAD_CH = 6, PK_ZERO = 7 };
// dst2 / kind2 (optional, conv data-gradient kinds only): the same tile pass also
// writes the forward layout kind2 (PK_CONV_FWD / PK_CONV_FWD_CH) to dst2, so a
// training step reads each fp32 weight once for both packs
struct PackEntry { const float* src; bf16_t* dst; int kind, Co, Ci, R, S; bf16_t* dst2; int kind2; };
// UP_ZERO: dst[0 .. Co) = 0; UP_D2F: dst[i] = sum_r acc[r][i], acc fp64 [kStatRep][Co]
enum { UP_CONV = 0, UP_CONVT = 1, UP_STEM = 2, UP_ZERO = 3, UP_D2F = 4 };
struct UnpackEntry { const float* acc; float* dst; int kind, Co, Ci, R, S; };
constexpr int kMaxPack = 56;  // PackTable 3.1 KB of kernel arguments (< 4 KB)
struct PackTable { int n; PackEntry e[kMaxPack]; };
struct UnpackTable { int n; UnpackEntry e[kMaxPack]; };
static_assert(sizeof(PackTable) <= 4096 && sizeof(UnpackTable) <= 4096, "tables travel as kernel arguments");
hipError_t launch_pack(const PackTable& t, hipStream_t st);
hipError_t launch_unpack(const UnpackTable& t, hipStream_t st);

// loss + metrics
enum { LOSS_BCE = 0, LOSS_DICE = 1, LOSS_COMBO = 2 };
// sums[0..8): sum bce, sum sig*y, sum sig, sum y, tp, fp, fn, tn; part[0..8*kLossBlocks):
// per-block partials (UNET_LOSS_SCRATCH_LEN doubles).  out != nullptr: also the loss value.
constexpr int kLossBlocks = 256;
hipError_t launch_loss_sums(const float* logits, const float* target, int64_t n, double* sums, double* part,
                            int from_prob, int kind, float alpha, float smooth, float* out, hipStream_t st);
hipError_t launch_loss_grad(const float* logits, const float* target, int64_t n, const double* sums,
                            int kind, float alpha, float smooth, const float* gscale, float* dl,
                            hipStream_t st);

// fused Adam over flat fp32 buffers (optim.hip); coef = {step, step_size, sqrt(bc2)} on device
hipError_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float* coef, float lr,
                       float beta1, float beta2, float eps, float wd, int advance_step, hipStream_t st);
hipError_t launch_grad_to_bf16(const float* src, bf16_t* dst, int64_t n, hipStream_t st);
hipError_t launch_grad_from_bf16(const bf16_t* src, float* dst, int64_t n, float scale, hipStream_t st);

// on-GPU preprocessing of uint8 frames (data.hip; dataset.py:30-66,147-151)
hipError_t launch_resize_area(const uint8_t* src, uint8_t* dst, int N, int H, int W, int oh, int ow, hipStream_t st);
hipError_t launch_mask_prep(const uint8_t* src, float* dst, int N, int H, int W, int oh, int ow, hipStream_t st);
hipError_t launch_normalize(const uint8_t* src, float* dst, int N, int H, int W, int normalize, hipStream_t st);
// A.Affine (+ the following A.VerticalFlip folded in) as cv2.warpAffine's
// fixed-point path; A.AdvancedBlur as cv2.filter2D (data.hip)
hipError_t launch_warp_affine(const uint8_t* src, uint8_t* dst, int N, int H, int W, const double* m, const int* active,
                              const int* vflip, int nearest, hipStream_t st);
hipError_t launch_filter2d(const uint8_t* src, uint8_t* dst, int N, int H, int W, const float* kern, const int* ksz,
                           hipStream_t st);
hipError_t launch_rot90_vflip(const uint8_t* src, uint8_t* dst, int N, int H, int W, const int* k, const int* flip,
                              hipStream_t st);

// attention decoder (attention.hip; advanced_models.py:7-61)
struct AttGateArgs {
  const bf16_t* s; int lds;            // relu(BN_g + BN_x), F_int channels
  const float* psi_w; const float* psi_b;
  float* p; float* psi; float* dbnp;   // fp32 [npix]
  double* pst; double* pbs;            // BN(1) fwd sums (sum, sumsq) / bwd sums (sum dZ, sum dZ phat)
  float* save;                         // mean, invstd
  const float* gamma; const float* beta; float* run_mean; float* run_var;
  long long* nbt;     // num_batches_tracked of the psi BN (+= 1 with the running stats), or null
  double count; float eps, momentum; int training;
  const bf16_t* x; int ldx;            // skip activation (F_l channels)
  bf16_t* xatt; int ldxatt;            // x * psi (concat slice)
  const bf16_t* dxatt; int lddxatt;    // its gradient
  bf16_t* dxpsi; int lddxpsi;          // gate-path skip gradient
  bf16_t* dS; int lddS;                // dA of relu(BN_g + BN_x)
  float* gpsi_w; float* ggamma; float* gbeta;
  double* gpsi_acc;                    // fp64 [kStatRep][Fi] psi-weight gradient partials (zeroed; -> gpsi_w)
  BnBwdArgs bb;                        // backward: relu(BN_g + BN_x) reduction fused into pass 3 (bb.sums != null)
  int64_t npix; int Fi, Fl;
};
struct ChAttArgs {
  const bf16_t* y; int ldy;            // decoder output
  bf16_t* out; int ldo;                // y * gate
  double* psum; unsigned long long* pkey;   // fp64 pooled sums (zeroed): order-independent to far below fp32
  const float* w1; const float* w2;    // fc.0 [Cr][C], fc.2 [C][Cr]
  float* am; float* h; float* gate;    // avg|max [N][2][C], hidden [N][2][Cr], gate [N][C]
  const bf16_t* dout2; int lddo2;
  double* dgate; float* dam;           // fp64 [N][C] (zeroed), [N][2][C]
  float* gw1; float* gw2;
  double* gw_acc;                      // fp64 [kStatRep][2][C*Cr] fc.2 | fc.0 gradient partials (zeroed)
  bf16_t* dout; int lddo;
  BnBwdArgs bb;                        // backward: the decoder BN's reduction fused into pass 5 (bb.sums != null)
  float inv_hw;
  int64_t HW; int N, C, Cr;
};
// pass 0 psi fwd, 1 gate fwd, 2 bwd reduce, 3 bwd apply
hipError_t launch_att_gate(const AttGateArgs& a, int pass, hipStream_t st);
// pass 0 pool, 1 MLP fwd, 2 scale, 3 bwd reduce, 4 MLP bwd, 5 bwd apply
hipError_t launch_ch_att(const ChAttArgs& a, int pass, hipStream_t st);

}  // namespace unet

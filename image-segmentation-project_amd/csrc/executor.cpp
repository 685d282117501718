// Native executor for the resnet34 U-Net training step (forward + backward).
//
// The plan mirrors UNetWithBackbone(backbone='resnet34', use_attention=False)
// (/root/reference/advanced_models.py:64-100,157-160,197-205,264-357) with the
// torchvision ResNet34 encoder.  It owns: the parameter table in reference
// state_dict order, the workspace layout (bf16 NHWC activations, skip-concat
// buffers that the up-convs write into directly, BN sums, packed weights and
// fp32 weight-gradient accumulators), and the launch sequence.  Python passes
// raw device pointers; nothing here allocates device memory.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the functions are resolved at run time (unet_allreduce_init)

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/unet_hip.h"
#include "kernels.h"

namespace unet {

thread_local std::string g_err;
void set_err(const std::string& s) { g_err = s; }

#define CK(expr)                                                                      \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) {                                                           \
      set_err(std::string(#expr) + " -> " + hipGetErrorString(e_) + " @" + __FILE__ + \
              ":" + std::to_string(__LINE__));                                        \
      return (int)e_;                                                                 \
    }                                                                                 \
  } while (0)

#define RUN(expr)              \
  do {                         \
    int r_ = (expr);           \
    if (r_) return r_;         \
  } while (0)

struct Act {  // bf16 NHWC view: ws + off, channel stride ld
  size_t off = 0;
  int ld = 0, C = 0, H = 0, W = 0;
};

struct Param {
  std::string name;
  std::vector<int64_t> shape;
  int64_t numel = 0, flat = 0;
};

struct Bn {
  int gamma, beta;        // param indices
  int idx;                // BN ordinal (buffers 3*idx + 0/1)
  int C;
  size_t stats, bsums, save;  // ws offsets: fp64 [R][2C] fwd, fp64 [R][2C] bwd, fp32 mean|invstd
  size_t ss, coef;            // fp32 scale|shift [2C], backward coefficients [5C]
  size_t tfwd, tbwd;          // last-block tickets (zeroed with the fwd / bwd sums)
};

enum { L_CONV = 0, L_CONVT = 1, L_STEM = 2 };
struct Conv {
  int w, b = -1;  // param indices
  int kind, Ci, Co, R, S, stride, pad;
  size_t pk_fwd = 0, pk_dgrad = 0, wacc = 0;  // ws offsets
  size_t bias_acc = 0;                        // fp64 [kStatRep][Co] (convT bias grads)
  bool f8 = false;                            // forward in fp8 e4m3 (cfg.fp8, C >= 128)
  // forward / data gradient on conv3x3_fl_kernel: pk_fwd / pk_dgrad hold the
  // chunk-major packs (PK_CONV_FWD_CH / PK_CONV_DGRAD_CH) instead
  bool fl_fwd = false, fl_dgrad = false;
  size_t f8w = 0;                             // ws offset: e4m3 [Co][R*S*Ci]
  int f8st = -1;                              // F8State index of the weight
};

// fp8 forward: the e4m3 copy of one conv input activation (quantized once per
// forward, before its first fp8 consumer)
struct F8Act {
  size_t src = 0; int C = 0;  // the bf16 activation (ws offset, channels)
  size_t q = 0;               // ws offset: dense e4m3 [npix][C]
  int st = -1;                // F8State index
};

// BasicBlock (resnet34): conv1 3x3/s - bn1 - relu - conv2 3x3 - bn2 (+ skip) - relu.
// Bottleneck (resnet50, torchvision v1.5): conv1 1x1 - bn1 - relu - conv2 3x3/s -
// bn2 - relu - conv3 1x1 (x4 channels) - bn3 (+ skip) - relu; the block's LAST
// conv / BN are (conv3, bn3), its middle pair (conv2, bn2, y2 -> h2).
struct Block {
  int conv1, bn1, conv2, bn2, ds = -1, dsbn = -1;
  int conv3 = -1, bn3 = -1;             // bottleneck only
  Act in, y1, h, y2, yds, out;
  Act h2, y3;                           // bottleneck: relu(bn2(y2)), conv3 output
  Act d_out, dy1, dh, dy2, dyds, dres;  // grads
  Act dh2, dy3, dds;                    // bottleneck: grads of h2 / y3, downsample dgrad (then added)
  Act d_in;                             // == previous block's d_out (or dP0)
  Act skip_add;                         // skip-concat gradient slice for the input (or empty)
  bool bottleneck() const { return conv3 >= 0; }
  int last_conv() const { return conv3 >= 0 ? conv3 : conv2; }
  int last_bn() const { return conv3 >= 0 ? bn3 : bn2; }
  const Act& last_y() const { return conv3 >= 0 ? y3 : y2; }
  const Act& last_dy() const { return conv3 >= 0 ? dy3 : dy2; }
};

struct Dec {
  int up, conv1, bn1, conv2, bn2;
  Act up_in, up_out;  // up_out = cat slice
  Act cat, y1, h, y2, out;
  Act d_out, dy2, dh, dy1, dcat, d_up_in;
  // gradient of the up-conv part of the concat: a slice of dcat, or (split,
  // when that part is narrower than a 128-B line) its own dense buffer while
  // dcat then holds only the skip channels
  Act dcat_up;
  bool split = false;
};

// use_attention=True: AttentionGate on the skip (advanced_models.py:7-40,286-331)
// and ChannelAttention on the decoder output (:43-61,294,...) of one level
struct Att {
  int wg, bng, wx, bnx, psi_w, psi_b, psibn, fc1, fc2;  // conv / BN / param indices
  int Fg, Fl, Fi, C, Cr;
  Act x;               // the skip activation (own buffer; the concat slice holds x * psi)
  Act g1, xa, s;       // W_g g, W_x x, relu(BN_g + BN_x)
  size_t p = 0, psi = 0, dbnp = 0;     // fp32 [npix]: psi logits, sigmoid(BN(p)), dL/dBN(p)
  size_t pst = 0, pbs = 0, psave = 0;  // fp64 [2] fwd sums, fp64 [2] bwd sums, fp32 mean|invstd
  Act dS, dg1, dxa, dxpsi, dskip, du;  // gradients (du = up-conv output grad incl. the W_g path)
  Act out2, d_out2;                    // decoder output * channel gate, and its gradient
  size_t psum = 0, pkey = 0;           // fp64 [N][C] pooled sums, u64 [N][C] (max, first index) keys
  size_t ca = 0, ch = 0, cam = 0;      // fp32 gate [N][C], hidden [N][2][Cr], avg|max [N][2][C]
  size_t cda = 0, cdam = 0;            // fp64 dL/dgate [N][C], fp32 dL/d(avg|max) [N][2][C]
  size_t gpsi = 0, gfc = 0;            // fp64 replica partials of the psi / fc.2|fc.0 weight gradients
};

}  // namespace unet

using namespace unet;

struct unet_plan {
  unet_config cfg;
  std::vector<Param> params;
  std::vector<Bn> bns;
  std::vector<Conv> convs;
  std::vector<Block> blocks;  // 16 encoder blocks
  std::vector<Dec> decs;      // decoder4..decoder1 (index 0 = level 4)
  std::vector<Att> atts;      // attention of decoder level (same index), when cfg.attention
  int stem_conv, stem_bn, up0_w, up0_b, fin_w, fin_b;
  Act x1, y0, p0, d_x1, d_y0, d_p0;
  size_t pidx = 0;
  size_t ws_bytes = 0;
  size_t zero_fwd_off = 0, zero_fwd_bytes = 0;
  size_t zero_bwd_off = 0, zero_bwd_bytes = 0;
  // a training forward zeroes the backward's region too (it follows the
  // forward's, one fill instead of two); the next backward then skips its fill
  bool bwd_zeroed = false;          // the last training forward zeroed the backward accumulators ...
  const char* bwd_zeroed_ws = nullptr;  // ... of this workspace
  size_t head_usum = 0;
  size_t wslab = 0, wslab_bytes = 0;  // split-K partials of the halo weight-gradient kernel
  int64_t grad_numel = 0;
  std::vector<std::pair<int64_t, int64_t>> buckets;  // flat element ranges
  std::vector<std::vector<int>> bucket_convs;        // convs to unpack per bucket
  hipEvent_t events[8] = {};
  int nevents = 0;
  // without bucket events (no DDP overlap) the buckets' unpack entries are
  // collected here and launched together at the end of the backward
  UnpackTable pend{};
  // The whole backward runs on the caller's stream.  Weight gradients on a
  // second stream and split-K reduces on a third were both measured slower on
  // MI355X (8.39 vs 7.86 ms/step; 2019 vs 2201 img/s: the LDS-heavy wgrad and
  // reduce blocks contend for CUs with the critical dgrad chain) and were
  // removed.  Two split-K slabs alternate so a deferred
  // reduction never reads partials the next weight gradient overwrites.
  int slab_next = 0;
  std::vector<hipEvent_t> syncpool;
  int syncused = 0;
  bool want_events = false;  // DDP overlap: record one hipEvent per gradient bucket
  // in-kernel phase timing (debug build only, unet_timing_enable): one slot of
  // kTimBlocks x kTimSlots stamps per conv launch, in launch order
  unsigned long long* tim_buf = nullptr;
  int tim_n = 0;
  bool tim_on = false;
  std::vector<std::string> tim_names;
  // BN-backward reductions fused into the producing conv dgrad (UNET_NO_BWD_FUSE=1: off, A/B only)
  bool fuse_bwd = std::getenv("UNET_NO_BWD_FUSE") == nullptr;
  // BN coefficients recomputed by every consumer block from the replica sums
  // (default; measured 0.28 ms/step faster) vs finalised by the producing
  // kernel's last block, whose blocks must then drain their atomics and take a
  // ticket before exiting (UNET_BN_TICKET=1)
  bool bn_ticket = std::getenv("UNET_BN_TICKET") && std::getenv("UNET_BN_TICKET")[0] == '1';
  // eval forward: BN folded into the conv epilogues (UNET_NO_EVAL_FOLD=1: separate BN passes, A/B only)
  bool eval_fold = std::getenv("UNET_NO_EVAL_FOLD") == nullptr;
  // stem BN-backward apply fused into the stem weight gradient's dY load
  // (UNET_NO_STEM_FUSE=1: separate apply pass writing dY, A/B only)
  bool stem_bn_fuse = std::getenv("UNET_NO_STEM_FUSE") == nullptr;
  // BN1 + ReLU of a block / decoder level applied in the staging of the next
  // (weight-stationary) conv, which also stores the activation: no bn_apply
  // pass (UNET_NO_BN_XFORM=1: separate pass, A/B only)
  bool bn_xform = std::getenv("UNET_NO_BN_XFORM") == nullptr;
  // BasicBlock downsample (1x1 / s2) weight gradient folded into the conv1
  // (3x3 / s2) halo weight gradient (UNET_NO_DS_FOLD=1: separate launch, A/B)
  bool ds_wgrad_fold = std::getenv("UNET_NO_DS_FOLD") == nullptr;
  // training: decoder1's last BN + ReLU formed inside the head's two passes
  // from the raw conv output (no bn_apply pass, decoder1's activation never
  // stored; plain U-Net with the fused BN backward only).  UNET_NO_HEAD_BN_FOLD=1:
  // separate pass (A/B only)
  bool head_bn_fold = std::getenv("UNET_NO_HEAD_BN_FOLD") == nullptr;
  // single-stream backward: a weight gradient's split-K reduction rides in the
  // next BN-backward apply launch (UNET_NO_MERGE_REDUCE=1: separate launches)
  bool merge_reduce = std::getenv("UNET_NO_MERGE_REDUCE") == nullptr;
  // 3x3 / s1 weight gradients of a gradient bucket collected and run as ONE
  // batched stream-K launch at the bucket boundary (wgrad3x3_batch_kernel):
  // no per-layer split-K slab round trip.  UNET_WG_BATCH=0: one launch per layer (A/B)
  bool wg_batch = !(std::getenv("UNET_WG_BATCH") && std::atoi(std::getenv("UNET_WG_BATCH")) == 0);
  // the stem by recompute (stem_rc.hip): the raw 7x7 conv output y0 is never
  // stored; statistics pass + act/pool pass forward, one pass for the maxpool
  // backward, the stem BN backward and the stem weight gradient.  Shapes with
  // stem rows over 256 pixels (HiRes) keep the stored-y0 path.  UNET_STEM_RC=0:
  // stored-y0 path everywhere (A/B); UNET_STEM_KEEP=1: y0 and dZ are stored
  // too (tests of the intermediates)
  bool stem_rc = !(std::getenv("UNET_STEM_RC") && std::atoi(std::getenv("UNET_STEM_RC")) == 0);
  bool stem_keep = std::getenv("UNET_STEM_KEEP") && std::atoi(std::getenv("UNET_STEM_KEEP")) != 0;
  size_t stem_part = 0, stem_tot = 0, stem_tkt = 0;
  std::vector<ConvWgradArgs> wgb;  // collected weight gradients of the current bucket
  std::vector<std::string> wgb_names;
  double wgb_flops = 0;
  double flops_fwd = 0, flops_train = 0;
  // fp8 forward (cfg.fp8): per-tensor delayed-amax states (fp8.hip) for the
  // conv weights and activations; the first forward calibrates
  std::vector<F8Act> f8acts;
  std::vector<char> f8_done;  // per F8Act: quantized in the current forward
  size_t f8st = 0;            // ws offset of the F8State array
  int f8n = 0;
  bool f8_calibrated = false;
  std::vector<std::pair<std::string, Act>> named;  // debug / test introspection
  // per-launch HIP-event profiler (unet_profile_*): one record per kernel
  struct ProfRec { std::string name; double flops; int e0, e1; std::string kernel; };
  bool prof = false;
  std::vector<hipEvent_t> evpool;
  int evused = 0;
  std::vector<ProfRec> recs;
};

namespace {
int prof_event(unet_plan* p, hipStream_t st) {
  if (p->evused == (int)p->evpool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return -1;
    p->evpool.push_back(e);
  }
  const int i = p->evused++;
  if (hipEventRecord(p->evpool[i], st) != hipSuccess) return -1;
  return i;
}
// RAII: brackets one launch with two events when profiling is on
// the next conv launch's phase-stamp slot (null unless timing is on)
unsigned long long* tim_slot(unet_plan* p, const std::string& name) {
  if (!p->tim_on || !p->tim_buf || p->tim_n >= kTimLaunches) return nullptr;
  p->tim_names.push_back(name);
  return p->tim_buf + (size_t)(p->tim_n++) * kTimBlocks * kTimSlots;
}

struct ProfScope {
  unet_plan* p; hipStream_t st; std::string name; double flops; int e0 = -1;
  ProfScope(unet_plan* p_, hipStream_t s, std::string n, double f) : p(p_), st(s), name(std::move(n)), flops(f) {
    if (p->prof) e0 = prof_event(p, st);
  }
  void close() {
    if (p->prof && e0 >= 0) {
      const int e1 = prof_event(p, st);
      if (e1 >= 0) p->recs.push_back({name, flops, e0, e1, flops > 0 ? unet::last_kernel_tag() : ""});
    }
    e0 = -1;
  }
  ~ProfScope() { close(); }
};
}  // namespace

namespace {

struct Alloc {
  size_t top = 0;
  size_t take(size_t bytes) {
    const size_t off = top;
    top += (bytes + 255) & ~size_t(255);
    return off;
  }
};

int add_param(unet_plan* p, const std::string& name, std::vector<int64_t> shape) {
  Param q;
  q.name = name;
  q.shape = shape;
  q.numel = 1;
  for (auto s : shape) q.numel *= s;
  q.flat = p->grad_numel;
  p->grad_numel += q.numel;
  p->params.push_back(q);
  return (int)p->params.size() - 1;
}

int add_bn(unet_plan* p, const std::string& prefix, int C) {
  Bn b;
  b.gamma = add_param(p, prefix + ".weight", {C});
  b.beta = add_param(p, prefix + ".bias", {C});
  b.idx = (int)p->bns.size();
  b.C = C;
  p->bns.push_back(b);
  return b.idx;
}

int add_conv(unet_plan* p, const std::string& prefix, int kind, int Ci, int Co, int R, int stride, int pad,
             bool bias) {
  Conv c;
  c.kind = kind;
  c.Ci = Ci; c.Co = Co; c.R = R; c.S = R; c.stride = stride; c.pad = pad;
  if (kind == L_CONVT) c.w = add_param(p, prefix + ".weight", {Ci, Co, R, R});
  else c.w = add_param(p, prefix + ".weight", {Co, Ci, R, R});
  if (bias) c.b = add_param(p, prefix + ".bias", {Co});
  p->convs.push_back(c);
  return (int)p->convs.size() - 1;
}

Act act(Alloc& A, int N, int H, int W, int C) {
  Act a;
  a.off = A.take((size_t)N * H * W * C * 2);
  a.ld = C; a.C = C; a.H = H; a.W = W;
  return a;
}
Act slice(const Act& base, int c0, int C) {
  Act a = base;
  a.off = base.off + (size_t)c0 * 2;
  a.C = C;
  return a;
}

}  // namespace

// ---------------------------------------------------------------------------
// plan construction
// ---------------------------------------------------------------------------
static int build_plan(unet_plan* p) {
  const unet_config& c = p->cfg;
  const int N = c.N, H = c.H, W = c.W, w = c.width;
  if (H % 32 || W % 32 || N <= 0 || w <= 0) {
    set_err("unet_plan_create: H and W must be multiples of 32 (advanced_models.py:317-347 crops "
            "only fix the last two levels)");
    return 1;
  }
  if (c.n_classes != 1) { set_err("unet_plan_create: only n_classes == 1 is supported"); return 1; }
  const bool r50 = c.backbone == 50;
  if (c.backbone != 0 && c.backbone != 34 && c.backbone != 50) {
    set_err("unet_plan_create: backbone must be 34 (resnet34) or 50 (resnet50)");
    return 1;
  }
  if (r50 && w != 1) { set_err("unet_plan_create: resnet50 is built at width 1 only"); return 1; }
  if (c.fp8 && (r50 || c.attention)) {
    set_err("unet_plan_create: the fp8 forward is built for the resnet34 U-Net without attention (Wide / Base)");
    return 1;
  }
  // stage output channels (x2..x5): resnet34 64..512, resnet50 (expansion 4) 256..2048
  const int c0 = 64 * w, c1 = 128 * w, c2 = 256 * w, c3 = 512 * w;
  const int chan[4] = {r50 ? 256 : c0, r50 ? 512 : c1, r50 ? 1024 : c2, r50 ? 2048 : c3};
  const int planes[4] = {64, 128, 256, 512};
  const int nblk[4] = {3, 4, 6, 3};

  // ---- parameters, in reference registration order ----
  p->stem_conv = add_conv(p, "input_conv", L_STEM, 1, c0, 7, 2, 3, false);
  p->stem_bn = add_bn(p, "bn1", c0);
  struct BlkSpec { int conv1, bn1, conv2, bn2, conv3, bn3, ds, dsbn, cin, cout, mid, stride, stage; };
  std::vector<BlkSpec> specs;
  int cin = c0;
  for (int s = 0; s < 4; ++s) {
    for (int b = 0; b < nblk[s]; ++b) {
      const std::string pre = "enc" + std::to_string(s + 1) + "." + std::to_string(b);
      const int stride = (b == 0 && s > 0) ? 2 : 1;
      const int cout = chan[s];
      BlkSpec bs;
      bs.conv3 = bs.bn3 = -1;
      if (r50) {  // torchvision Bottleneck: 1x1 -> 3x3/stride -> 1x1 (x4)
        const int mid = planes[s];
        bs.conv1 = add_conv(p, pre + ".conv1", L_CONV, cin, mid, 1, 1, 0, false);
        bs.bn1 = add_bn(p, pre + ".bn1", mid);
        bs.conv2 = add_conv(p, pre + ".conv2", L_CONV, mid, mid, 3, stride, 1, false);
        bs.bn2 = add_bn(p, pre + ".bn2", mid);
        bs.conv3 = add_conv(p, pre + ".conv3", L_CONV, mid, cout, 1, 1, 0, false);
        bs.bn3 = add_bn(p, pre + ".bn3", cout);
        bs.mid = mid;
      } else {
        bs.conv1 = add_conv(p, pre + ".conv1", L_CONV, cin, cout, 3, stride, 1, false);
        bs.bn1 = add_bn(p, pre + ".bn1", cout);
        bs.conv2 = add_conv(p, pre + ".conv2", L_CONV, cout, cout, 3, 1, 1, false);
        bs.bn2 = add_bn(p, pre + ".bn2", cout);
        bs.mid = cout;
      }
      bs.ds = bs.dsbn = -1;
      if (stride != 1 || cin != cout) {
        bs.ds = add_conv(p, pre + ".downsample.0", L_CONV, cin, cout, 1, stride, 0, false);
        bs.dsbn = add_bn(p, pre + ".downsample.1", cout);
      }
      bs.cin = cin; bs.cout = cout; bs.stride = stride; bs.stage = s;
      specs.push_back(bs);
      cin = cout;
    }
  }
  const int enc_end_param = (int)p->params.size();
  // decoder: level 4 (deepest) .. 1
  struct DecSpec { int up, conv1, bn1, conv2, bn2, upin, upout, skipc, outc; };
  std::vector<DecSpec> dspecs;
  {
    // advanced_models.py:89-100 (resnet34) / :119-130 (resnet50)
    const int upin[4] = {chan[3], chan[2], chan[1], chan[0]};
    const int upout[4] = {chan[2], chan[1], chan[0], r50 ? c0 : c0 / 2};
    const int skipc[4] = {chan[2], chan[1], chan[0], c0};
    const int outc[4] = {chan[2], chan[1], chan[0], r50 ? c0 : c0 / 2};
    for (int l = 0; l < 4; ++l) {
      const int lvl = 4 - l;
      DecSpec d;
      d.up = add_conv(p, "upconv" + std::to_string(lvl), L_CONVT, upin[l], upout[l], 2, 2, 0, true);
      const std::string pre = "decoder" + std::to_string(lvl);
      const int catc = skipc[l] + upout[l];
      d.conv1 = add_conv(p, pre + ".0", L_CONV, catc, outc[l], 3, 1, 1, true);
      d.bn1 = add_bn(p, pre + ".1", outc[l]);
      d.conv2 = add_conv(p, pre + ".3", L_CONV, outc[l], outc[l], 3, 1, 1, true);
      d.bn2 = add_bn(p, pre + ".4", outc[l]);
      d.upin = upin[l]; d.upout = upout[l]; d.skipc = skipc[l]; d.outc = outc[l];
      dspecs.push_back(d);
    }
  }
  const int up0_in = dspecs[3].outc;  // 32 (resnet34) / 64 (resnet50), advanced_models.py:158-159
  p->up0_w = add_param(p, "upconv0.weight", {up0_in, c0 / 4, 2, 2});
  p->up0_b = add_param(p, "upconv0.bias", {c0 / 4});
  p->fin_w = add_param(p, "conv_final.weight", {c.n_classes, c0 / 4, 1, 1});
  p->fin_b = add_param(p, "conv_final.bias", {c.n_classes});
  if (c.attention) {  // advanced_models.py:163-172 / :175-183, registered after conv_final
    const int fi34[4] = {c1, c0, c0 / 2, c0 / 2}, fi50[4] = {512, 256, 128, 32};
    const int* fi = r50 ? fi50 : fi34;
    for (int l = 0; l < 4; ++l) {
      const std::string pre = "attention" + std::to_string(4 - l);
      Att t;
      t.Fg = dspecs[l].upout; t.Fl = dspecs[l].skipc; t.Fi = fi[l];
      t.wg = add_conv(p, pre + ".W_g.0", L_CONV, t.Fg, t.Fi, 1, 1, 0, true);
      t.bng = add_bn(p, pre + ".W_g.1", t.Fi);
      t.wx = add_conv(p, pre + ".W_x.0", L_CONV, t.Fl, t.Fi, 1, 1, 0, true);
      t.bnx = add_bn(p, pre + ".W_x.1", t.Fi);
      t.psi_w = add_param(p, pre + ".psi.0.weight", {1, t.Fi, 1, 1});
      t.psi_b = add_param(p, pre + ".psi.0.bias", {1});
      t.psibn = add_bn(p, pre + ".psi.1", 1);
      p->atts.push_back(t);
    }
    for (int l = 0; l < 4; ++l) {
      const std::string pre = "ch_attention" + std::to_string(4 - l);
      Att& t = p->atts[l];
      t.C = dspecs[l].outc; t.Cr = t.C / 16;
      t.fc1 = add_param(p, pre + ".fc.0.weight", {t.Cr, t.C, 1, 1});
      t.fc2 = add_param(p, pre + ".fc.2.weight", {t.C, t.Cr, 1, 1});
    }
  }

  // ---- DDP buckets in backward completion order ----
  auto stage_range = [&](int s) {
    int lo = -1, hi = -1;
    const std::string pre = "enc" + std::to_string(s + 1) + ".";
    for (int i = 0; i < (int)p->params.size(); ++i)
      if (p->params[i].name.rfind(pre, 0) == 0) { if (lo < 0) lo = i; hi = i; }
    return std::make_pair(lo, hi);
  };
  {
    const int64_t dec_begin = p->params[enc_end_param].flat;
    p->buckets.push_back({dec_begin, p->grad_numel});
    auto r4 = stage_range(3), r3 = stage_range(2), r1 = stage_range(0);
    p->buckets.push_back({p->params[r4.first].flat, p->params[r4.second].flat + p->params[r4.second].numel});
    p->buckets.push_back({p->params[r3.first].flat, p->params[r3.second].flat + p->params[r3.second].numel});
    // enc2 + enc1 final before the stem's backward, so only the stem's 3.3 k
    // parameters (bucket 4) trail the backward
    p->buckets.push_back({p->params[r1.first].flat, p->params[r3.first].flat});
    p->buckets.push_back({0, p->params[r1.first].flat});
  }
  static_assert(sizeof(((unet_plan*)nullptr)->events) / sizeof(hipEvent_t) >= 5, "one event per bucket");

  // ---- workspace ----
  Alloc A;
  // zeroed at forward start: BN fwd sums
  p->zero_fwd_off = A.take(0);
  for (auto& b : p->bns) {
    b.stats = A.take((size_t)kStatRep * 2 * b.C * sizeof(double));
    b.tfwd = A.take(sizeof(unsigned));
  }
  for (int l = 0; l < (int)p->atts.size(); ++l) {
    Att& t = p->atts[l];
    t.pst = A.take(2 * sizeof(double));
    t.psum = A.take((size_t)N * t.C * sizeof(double));
    t.pkey = A.take((size_t)N * t.C * sizeof(unsigned long long));
  }
  p->zero_fwd_bytes = A.top - p->zero_fwd_off;
  // zeroed at backward start: BN bwd sums, convT bias sums, head sums, wgrad accumulators
  p->zero_bwd_off = A.take(0);
  for (auto& b : p->bns) {
    b.bsums = A.take((size_t)kStatRep * 2 * b.C * sizeof(double));
    b.tbwd = A.take(sizeof(unsigned));
  }
  for (auto& cv : p->convs)
    if (cv.kind == L_CONVT) cv.bias_acc = A.take((size_t)kStatRep * cv.Co * sizeof(double));
  p->head_usum = A.take((size_t)kStatRep * (up0_in * 4 + 1) * sizeof(double));  // [kStatRep][Cin*4 + 1]
  p->stem_tkt = A.take(kStemTickets * sizeof(unsigned));
  for (auto& t : p->atts) {
    t.pbs = A.take(2 * sizeof(double));
    t.cda = A.take((size_t)N * t.C * sizeof(double));
    t.gpsi = A.take((size_t)kStatRep * t.Fi * sizeof(double));
    t.gfc = A.take((size_t)kStatRep * 2 * t.C * t.Cr * sizeof(double));
  }
  p->zero_bwd_bytes = A.top - p->zero_bwd_off;  // starts where the forward's region ends: one fill spans both
  // weight-gradient accumulators: every element is WRITTEN by its wgrad launch
  // (deterministic split-K slab reduction, kernels.h SlabLayout), so they are
  // not zeroed
  for (auto& cv : p->convs) {
    size_t n;
    if (cv.kind == L_STEM) n = (size_t)cv.Co * 64;
    else n = (size_t)cv.Co * cv.Ci * cv.R * cv.S;
    cv.wacc = A.take(n * sizeof(float));
  }
  for (auto& b : p->bns) {
    b.save = A.take((size_t)2 * b.C * sizeof(float));
    b.ss = A.take((size_t)2 * b.C * sizeof(float));
    b.coef = A.take((size_t)5 * b.C * sizeof(float));
  }
  for (auto& cv : p->convs) {
    if (cv.kind == L_STEM) {
      cv.pk_fwd = A.take((size_t)cv.Co * 64 * 2);
    } else {
      const size_t n = (size_t)cv.Co * cv.Ci * cv.R * cv.S * 2;
      cv.pk_fwd = A.take(n);
      cv.pk_dgrad = A.take(n);
    }
  }

  // forward activations
  const int H2 = H / 2, W2 = W / 2, H4 = H / 4, W4 = W / 4;
  Act cat1 = act(A, N, H2, W2, c0 + dspecs[3].upout);
  p->x1 = c.attention ? act(A, N, H2, W2, c0) : slice(cat1, 0, c0);
  p->y0 = act(A, N, H2, W2, c0);
  p->p0 = act(A, N, H4, W4, c0);
  p->pidx = A.take((size_t)N * H4 * W4 * c0);
  p->stem_rc = p->stem_rc && p->fuse_bwd && p->stem_bn_fuse && stem_rc_ok(c0, H2, W2) && H2 == 2 * H4 &&
               W2 == 2 * W4 && H == 2 * H2 && W == 2 * W2;
  if (p->stem_rc) {
    p->stem_part = A.take(stem_rc_part_bytes(N, H2, W2, c0));
    p->stem_tot = A.take(stem_rc_tot_bytes(c0));
  }
  // split-K partials of one weight-gradient launch (register-native layout);
  // launchers cap their split count to what fits
  p->wslab_bytes = (size_t)(64 * w * w) << 20;
  p->wslab = A.take(2 * p->wslab_bytes);  // two slabs, alternating
  Act cats[4];  // cats[l] for decoder level index l (0 = level 4)
  cats[3] = cat1;
  cats[2] = act(A, N, H4, W4, 2 * chan[0]);
  cats[1] = act(A, N, H / 8, W / 8, 2 * chan[1]);
  cats[0] = act(A, N, H / 16, W / 16, 2 * chan[2]);
  Act x5 = act(A, N, H / 32, W / 32, chan[3]);

  Act prev = p->p0;
  for (size_t i = 0; i < specs.size(); ++i) {
    const BlkSpec& s = specs[i];
    Block b;
    b.conv1 = s.conv1; b.bn1 = s.bn1; b.conv2 = s.conv2; b.bn2 = s.bn2; b.ds = s.ds; b.dsbn = s.dsbn;
    b.conv3 = s.conv3; b.bn3 = s.bn3;
    const int Hs = H4 >> s.stage, Ws = W4 >> s.stage;
    b.in = prev;
    if (b.bottleneck()) {  // conv1 (1x1) at the input resolution, the stride sits on conv2
      b.y1 = act(A, N, prev.H, prev.W, s.mid);
      b.h = act(A, N, prev.H, prev.W, s.mid);
      b.y2 = act(A, N, Hs, Ws, s.mid);
      b.h2 = act(A, N, Hs, Ws, s.mid);
      b.y3 = act(A, N, Hs, Ws, s.cout);
    } else {
      b.y1 = act(A, N, Hs, Ws, s.cout);
      b.h = act(A, N, Hs, Ws, s.cout);
      b.y2 = act(A, N, Hs, Ws, s.cout);
    }
    if (s.ds >= 0) b.yds = act(A, N, Hs, Ws, s.cout);
    const bool last = (i + 1 == specs.size()) || specs[i + 1].stage != s.stage;
    if (last) {
      if (s.stage == 3) b.out = x5;
      else if (c.attention) b.out = act(A, N, Hs, Ws, s.cout);  // gated copy goes into the concat
      else b.out = slice(cats[2 - s.stage], 0, s.cout);  // x2->cat2, x3->cat3, x4->cat4
    } else {
      b.out = act(A, N, Hs, Ws, s.cout);
    }
    p->blocks.push_back(b);
    prev = b.out;
  }
  Act dec_in = x5;
  for (int l = 0; l < 4; ++l) {
    const DecSpec& s = dspecs[l];
    Dec d;
    d.up = s.up; d.conv1 = s.conv1; d.bn1 = s.bn1; d.conv2 = s.conv2; d.bn2 = s.bn2;
    d.cat = cats[l];
    d.up_in = dec_in;
    d.up_out = slice(cats[l], s.skipc, s.upout);
    const int Hl = d.cat.H, Wl = d.cat.W;
    d.y1 = act(A, N, Hl, Wl, s.outc);
    d.h = act(A, N, Hl, Wl, s.outc);
    d.y2 = act(A, N, Hl, Wl, s.outc);
    d.out = act(A, N, Hl, Wl, s.outc);
    p->decs.push_back(d);
    dec_in = d.out;
    if (c.attention) {
      Att& t = p->atts[l];
      const int64_t np = (int64_t)N * Hl * Wl;
      t.g1 = act(A, N, Hl, Wl, t.Fi);
      t.xa = act(A, N, Hl, Wl, t.Fi);
      t.s = act(A, N, Hl, Wl, t.Fi);
      t.p = A.take(np * sizeof(float));
      t.psi = A.take(np * sizeof(float));
      t.dbnp = A.take(np * sizeof(float));
      t.psave = A.take(2 * sizeof(float));
      t.ca = A.take((size_t)N * t.C * sizeof(float));
      t.ch = A.take((size_t)N * 2 * t.Cr * sizeof(float));
      t.cam = A.take((size_t)N * 2 * t.C * sizeof(float));
      t.cdam = A.take((size_t)N * 2 * t.C * sizeof(float));
      t.out2 = act(A, N, Hl, Wl, t.C);
      t.d_out2 = act(A, N, Hl, Wl, t.C);
      t.dS = act(A, N, Hl, Wl, t.Fi);
      t.dg1 = act(A, N, Hl, Wl, t.Fi);
      t.dxa = act(A, N, Hl, Wl, t.Fi);
      t.dxpsi = act(A, N, Hl, Wl, t.Fl);
      t.dskip = act(A, N, Hl, Wl, t.Fl);
      t.du = act(A, N, Hl, Wl, t.Fg);
      dec_in = t.out2;
    }
  }
  if (c.attention) {  // skips: x4 = enc3 out, x3 = enc2 out, x2 = enc1 out, x1 = stem
    int last[3] = {-1, -1, -1};
    for (size_t i = 0; i < specs.size(); ++i)
      if (specs[i].stage < 3) last[specs[i].stage] = (int)i;
    p->atts[0].x = p->blocks[last[2]].out;
    p->atts[1].x = p->blocks[last[1]].out;
    p->atts[2].x = p->blocks[last[0]].out;
    p->atts[3].x = p->x1;
  }

  // fp8 forward: e4m3 weight packs and input copies of every conv with C >= 128
  if (c.fp8) {
    auto f8_input = [&](int ci, const Act& in) {
      Conv& cv = p->convs[ci];
      if (cv.kind != L_CONV || cv.Ci < 128 || cv.Ci % 16 || in.ld % 8) return;
      cv.f8 = true;
      cv.f8w = A.take((size_t)cv.Co * cv.Ci * cv.R * cv.S);
      cv.f8st = p->f8n++;
      for (auto& f : p->f8acts)
        if (f.src == in.off && f.C == in.C) return;
      F8Act f;
      f.src = in.off; f.C = in.C;
      f.q = A.take((size_t)N * in.H * in.W * in.C);
      f.st = p->f8n++;
      p->f8acts.push_back(f);
    };
    for (auto& b : p->blocks) {
      f8_input(b.conv1, b.in);
      f8_input(b.conv2, b.h);
      if (b.ds >= 0) f8_input(b.ds, b.in);
    }
    for (auto& d : p->decs) {
      f8_input(d.conv1, d.cat);
      f8_input(d.conv2, d.h);
    }
    p->f8st = A.take((size_t)p->f8n * sizeof(F8State));
    p->f8_done.assign(p->f8acts.size(), 0);
  }

  // 3x3 / s1 convs on the full-line halo kernel (conv_fl.hip): their packs
  // are chunk-major, every launch of them goes to that kernel
  {
    auto fl_mark = [&](int ci, const Act& in) {
      Conv& cv = p->convs[ci];
      if (cv.kind != L_CONV || cv.R != 3 || cv.S != 3 || cv.stride != 1 || cv.pad != 1) return;
      cv.fl_fwd = !cv.f8 && conv3x3_fl_shape(N, cv.Ci, cv.Co, in.H, in.W);
      cv.fl_dgrad = conv3x3_fl_shape(N, cv.Co, cv.Ci, in.H, in.W);
    };
    for (auto& b : p->blocks) {
      fl_mark(b.conv1, b.in);
      fl_mark(b.conv2, b.h);
    }
    for (auto& d : p->decs) {
      fl_mark(d.conv1, d.cat);
      fl_mark(d.conv2, d.h);
    }
  }

  // backward gradient tensors
  for (int l = 3; l >= 0; --l) {
    Dec& d = p->decs[l];
    const int Hl = d.cat.H, Wl = d.cat.W, oc = d.out.C;
    d.d_out = act(A, N, Hl, Wl, oc);
    d.dy2 = act(A, N, Hl, Wl, oc);
    d.dh = act(A, N, Hl, Wl, oc);
    d.dy1 = act(A, N, Hl, Wl, oc);
    const int upc = d.up_out.C, skc = d.cat.C - upc;
    d.split = upc * 2 < 128;
    if (d.split) {
      d.dcat = act(A, N, Hl, Wl, skc);
      d.dcat_up = act(A, N, Hl, Wl, upc);
    } else {
      d.dcat = act(A, N, Hl, Wl, d.cat.C);
      d.dcat_up = slice(d.dcat, skc, upc);
    }
  }
  for (int l = 0; l < 4; ++l) {
    Dec& d = p->decs[l];
    d.d_up_in = (l == 0) ? act(A, N, H / 32, W / 32, chan[3])
                         : (c.attention ? p->atts[l - 1].d_out2 : p->decs[l - 1].d_out);
  }
  for (auto& b : p->blocks) {
    b.dy1 = act(A, N, b.y1.H, b.y1.W, b.y1.C);
    b.dh = act(A, N, b.h.H, b.h.W, b.h.C);
    b.dy2 = act(A, N, b.y2.H, b.y2.W, b.y2.C);
    if (b.bottleneck()) {
      b.dh2 = act(A, N, b.h2.H, b.h2.W, b.h2.C);
      b.dy3 = act(A, N, b.y3.H, b.y3.W, b.y3.C);
      if (b.ds >= 0) b.dds = act(A, N, b.in.H, b.in.W, b.in.C);
    }
    const Act& o = b.out;
    if (b.ds >= 0) b.dyds = act(A, N, o.H, o.W, o.C);
    else b.dres = act(A, N, o.H, o.W, o.C);
  }
  // block output grads: last encoder block's d_out = decoder-4's d_up_in
  const int nb = (int)p->blocks.size();
  p->blocks[nb - 1].d_out = p->decs[0].d_up_in;
  for (int i = nb - 2; i >= 0; --i) {
    Block& b = p->blocks[i];
    b.d_out = act(A, N, b.out.H, b.out.W, b.out.C);
  }
  p->d_p0 = act(A, N, H4, W4, c0);
  for (int i = 0; i < nb; ++i) {
    Block& b = p->blocks[i];
    b.d_in = i == 0 ? p->d_p0 : p->blocks[i - 1].d_out;
    b.skip_add = Act();
    if (i > 0 && specs[i].stage != specs[i - 1].stage) {
      // input x_{s+1} also fed cat_{s+1} slice 0: add that slice's gradient
      const int s = specs[i].stage;            // 1..3
      const int l = 3 - s;                     // x2 (s=1) -> cats[2], x3 -> cats[1], x4 -> cats[0]
      b.skip_add = c.attention ? p->atts[l].dskip : slice(p->decs[l].dcat, 0, specs[i].cin);
    }
  }
  p->d_x1 = act(A, N, H2, W2, c0);
  p->d_y0 = act(A, N, H2, W2, c0);
  p->ws_bytes = A.top;

  {
    const int hc = p->decs[3].out.C;
    p->head_bn_fold = p->head_bn_fold && p->fuse_bwd && p->atts.empty() && (hc == 32 || hc == 64) &&
                      p->decs[3].y2.C == hc;
  }

  // named views for tests: forward activations and their gradients
  auto& nm = p->named;
  const bool y0_stored = !p->stem_rc || p->stem_keep;  // recompute: y0 / dZ only kept for tests
  if (y0_stored) nm.push_back({"y0", p->y0});
  nm.push_back({"x1", p->x1}); nm.push_back({"p0", p->p0});
  if (y0_stored) nm.push_back({"d.x1", p->d_x1});
  nm.push_back({"d.p0", p->d_p0});
  if (!(p->fuse_bwd && p->stem_bn_fuse) && !p->stem_rc) nm.push_back({"d.y0", p->d_y0});  // else never stored
  {
    int bi = 0;
    for (int s = 0; s < 4; ++s)
      for (int k = 0; k < nblk[s]; ++k, ++bi) {
        const Block& b = p->blocks[bi];
        const std::string pre = "enc" + std::to_string(s + 1) + "." + std::to_string(k) + ".";
        nm.push_back({pre + "y1", b.y1}); nm.push_back({pre + "h", b.h}); nm.push_back({pre + "y2", b.y2});
        if (b.bottleneck()) {
          nm.push_back({pre + "h2", b.h2}); nm.push_back({pre + "y3", b.y3});
          nm.push_back({pre + "d.h2", b.dh2}); nm.push_back({pre + "d.y3", b.dy3});
        }
        if (b.ds >= 0) { nm.push_back({pre + "yds", b.yds}); nm.push_back({pre + "d.yds", b.dyds}); }
        nm.push_back({pre + "out", b.out});
        nm.push_back({pre + "d.out", b.d_out}); nm.push_back({pre + "d.y2", b.dy2});
        nm.push_back({pre + "d.h", b.dh}); nm.push_back({pre + "d.y1", b.dy1});
      }
  }
  for (int l = 0; l < 4; ++l) {
    const Dec& d = p->decs[l];
    const std::string pre = "dec" + std::to_string(4 - l) + ".";
    nm.push_back({pre + "up", d.up_out}); nm.push_back({pre + "cat", d.cat});
    nm.push_back({pre + "y1", d.y1}); nm.push_back({pre + "h", d.h}); nm.push_back({pre + "y2", d.y2});
    // (dec1.out: written by eval forwards; a training forward with head_bn_fold leaves it untouched)
    nm.push_back({pre + "out", d.out});
    nm.push_back({pre + "d.out", d.d_out}); nm.push_back({pre + "d.y2", d.dy2}); nm.push_back({pre + "d.h", d.dh});
    nm.push_back({pre + "d.y1", d.dy1});
    if (!p->atts.empty()) {
      const Att& t = p->atts[l];
      const std::string ap = "att" + std::to_string(4 - l) + ".";
      nm.push_back({ap + "x", t.x}); nm.push_back({ap + "g1", t.g1}); nm.push_back({ap + "xa", t.xa});
      nm.push_back({ap + "s", t.s}); nm.push_back({ap + "out2", t.out2}); nm.push_back({ap + "d.out2", t.d_out2});
      nm.push_back({ap + "d.S", t.dS}); nm.push_back({ap + "d.g1", t.dg1}); nm.push_back({ap + "d.xa", t.dxa});
      nm.push_back({ap + "d.skip", t.dskip}); nm.push_back({ap + "d.u", t.du});
    }
    if (d.split) { nm.push_back({pre + "d.cat.skip", d.dcat}); nm.push_back({pre + "d.cat.up", d.dcat_up}); }
    else nm.push_back({pre + "d.cat", d.dcat});
  }

  // unpack groups per bucket
  p->bucket_convs.assign(p->buckets.size(), {});
  for (int i = 0; i < (int)p->convs.size(); ++i) {
    const int64_t f = p->params[p->convs[i].w].flat;
    for (int bk = 0; bk < (int)p->buckets.size(); ++bk)
      if (f >= p->buckets[bk].first && f < p->buckets[bk].second) p->bucket_convs[bk].push_back(i);
  }

  // algorithmic FLOPs: 2*MACs; training = 3x fwd - stem dgrad
  double fw = 0, stem = 0;
  for (auto& cv : p->convs) {
    double macs;
    if (cv.kind == L_STEM) { macs = (double)N * H2 * W2 * cv.Co * 49; stem = 2 * macs; }
    else if (cv.kind == L_CONVT) {
      // input pixels x Ci x Co x 4
      int hin = 0;
      for (auto& d : p->decs) if (d.up >= 0 && &p->convs[d.up] == &cv) hin = d.up_in.H * d.up_in.W;
      macs = (double)N * hin * cv.Ci * cv.Co * 4;
    } else {
      macs = 0;
    }
    fw += 2 * macs;
  }
  for (auto& b : p->blocks) {
    const double px = (double)N * b.y1.H * b.y1.W;
    auto cf = [&](int ci, const Act& o) {
      const Conv& cv = p->convs[ci];
      return 2.0 * N * o.H * o.W * cv.Ci * cv.Co * cv.R * cv.S;
    };
    (void)px;
    fw += cf(b.conv1, b.y1) + cf(b.conv2, b.y2);
    if (b.bottleneck()) fw += cf(b.conv3, b.y3);
    if (b.ds >= 0) fw += cf(b.ds, b.yds);
  }
  for (auto& d : p->decs) {
    const double px = (double)N * d.y1.H * d.y1.W;
    fw += 2 * px * p->convs[d.conv1].Ci * p->convs[d.conv1].Co * 9;
    fw += 2 * px * p->convs[d.conv2].Ci * p->convs[d.conv2].Co * 9;
  }
  for (int l = 0; l < (int)p->atts.size(); ++l) {  // attention 1x1 convs + psi + channel MLP
    const Att& t = p->atts[l];
    const double px = (double)N * p->decs[l].y1.H * p->decs[l].y1.W;
    fw += 2 * px * t.Fi * (t.Fg + t.Fl + 1) + 2.0 * N * 2 * 2 * t.C * t.Cr;
  }
  fw += 2.0 * N * H2 * W2 * up0_in * (c0 / 4) * 4;  // upconv0
  fw += 2.0 * N * H * W * (c0 / 4);                    // conv_final
  p->flops_fwd = fw;
  p->flops_train = 3 * fw - stem;

  // bucket events are created lazily; plan creation does query the current
  // device's CU count (device_cu_count: the full-line conv routing and the
  // chunk-major packs depend on it), so it initialises the HIP runtime and the
  // plan is bound to the device current at creation
  return 0;
}

static int ensure_events(unet_plan* p) {
  if (p->nevents) return 0;
  const int nb = (int)p->buckets.size();
  for (int i = 0; i < nb; ++i) CK(hipEventCreateWithFlags(&p->events[i], hipEventDisableTiming));
  p->nevents = nb;
  return 0;
}

// ---------------------------------------------------------------------------
// execution helpers
// ---------------------------------------------------------------------------
int stream_edge(unet_plan* p, hipStream_t from, hipStream_t to);
int pooled_event(unet_plan* p, hipEvent_t* out);

namespace {

struct Ctx {
  unet_plan* p;
  char* ws;
  const float* const* prm;
  float* const* buf;
  hipStream_t st;
  int training;
  // weight-gradient and split-K reduction streams: both are st (the backward
  // is single-stream since the two-stream variants were removed);
  // kept as names so the launch sites say which role a launch plays
  hipStream_t wst = nullptr;
  hipStream_t rst = nullptr;
  bf16_t* A(const Act& a) const { return reinterpret_cast<bf16_t*>(ws + a.off); }
  template <class T> T* W(size_t off) const { return reinterpret_cast<T*>(ws + off); }
};

BnLaunch bn_launch(const Ctx& x, int bi, int64_t npix) {
  const Bn& b = x.p->bns[bi];
  BnLaunch l;
  l.stats = x.W<double>(b.stats);
  l.gamma = x.prm[b.gamma];
  l.beta = x.prm[b.beta];
  l.run_mean = x.buf ? x.buf[3 * b.idx + 0] : nullptr;  // (backward contexts carry no buffers)
  l.run_var = x.buf ? x.buf[3 * b.idx + 1] : nullptr;
  l.save_mean = x.W<float>(b.save);
  l.save_invstd = x.W<float>(b.save) + b.C;
  l.count = (double)npix;
  l.C = b.C;
  l.eps = x.p->cfg.bn_eps;
  l.momentum = x.p->cfg.bn_momentum;
  l.training = x.training;
  l.ss = x.p->bn_ticket ? x.W<float>(b.ss) : nullptr;
  l.ticket = x.p->bn_ticket ? x.W<unsigned>(b.tfwd) : nullptr;
  // buffers are (running_mean, running_var, num_batches_tracked) per BN
  l.nbt = x.buf && x.training ? reinterpret_cast<long long*>(x.buf[3 * b.idx + 2]) : nullptr;
  return l;
}

double conv_flops(const unet_plan* p, const Conv& cv, const Act& fwd_out) {
  const double N = p->cfg.N;
  if (cv.kind == L_CONVT) return 2.0 * N * (fwd_out.H / 2) * (fwd_out.W / 2) * cv.Ci * cv.Co * 4;
  return 2.0 * N * fwd_out.H * fwd_out.W * cv.Co * cv.Ci * cv.R * cv.S;
}
const std::string& pname(const Ctx& x, int param) { return x.p->params[param].name; }

// fold_bn >= 0 (eval only): that BN (running statistics) is applied in the
// conv epilogue, then `res` is added and ReLU applied (relu), so the BN pass
// after the conv disappears (§8(f) row 4)
// xbn >= 0 (training): `in` is the RAW output of the previous conv; BN xbn +
// ReLU is applied while staging and the activation is stored to *xh by the
// conv itself (ConvFwdArgs::xform), replacing that BN's bn_apply pass
// ds >= 0 (training, the 3x3 / stride-2 conv1 of a downsample block): that
// 1x1 / stride-2 downsample (output *yds, BN dsbn's sums) rides in the same
// launch when the implicit-GEMM forward takes it; *ds_done says whether it did
bool ds_fold_fwd_ok(const Ctx& x, int ci, int ds) {
  const Conv& cv = x.p->convs[ci];
  if (ds < 0 || !x.training || cv.f8 || cv.fl_fwd || cv.kind != L_CONV) return false;
  const Conv& dv = x.p->convs[ds];
  return cv.R == 3 && cv.S == 3 && cv.stride == 2 && cv.pad == 1 && cv.Ci % 64 == 0 && !dv.f8 &&
         dv.kind == L_CONV && dv.R == 1 && dv.S == 1 && dv.stride == 2 && dv.pad == 0 && dv.Co == cv.Co &&
         dv.Ci == cv.Ci && dv.b < 0;
}
int conv_forward(const Ctx& x, int ci, const Act& in, const Act& out, int bn_for_stats, int fold_bn = -1,
                 bool relu = false, const Act* res = nullptr, int xbn = -1, const Act* xh = nullptr, int ds = -1,
                 const Act* yds = nullptr, int dsbn = -1, bool* ds_done = nullptr) {
  const Conv& cv = x.p->convs[ci];
  if (ds_done) *ds_done = false;
  bool dsf = yds && ds_fold_fwd_ok(x, ci, ds) && fold_bn < 0 && xbn < 0;
  if (dsf) {  // the kernel's own geometry / tile test
    ConvFwdArgs g = {};
    g.N = x.p->cfg.N; g.H = in.H; g.W = in.W; g.C = cv.Ci; g.P = out.H; g.Q = out.W; g.Cout = cv.Co;
    g.R = cv.R; g.S = cv.S; g.stride = cv.stride; g.pad = cv.pad; g.ldyds = yds->ld;
    dsf = conv_fwd_ds_ok(g);
  }
  ProfScope ps(x.p, x.st, "fwd " + pname(x, cv.w) + (xbn >= 0 ? " +bn" : "") + (dsf ? " +ds" : ""),
               conv_flops(x.p, cv, out) + (dsf ? conv_flops(x.p, x.p->convs[ds], *yds) : 0.0));
  ConvFwdArgs a = {};
  a.x = x.A(in); a.ldx = in.ld;
  a.w = x.W<bf16_t>(cv.pk_fwd);
  a.y = x.A(out); a.ldy = out.ld;
  a.bias = cv.b >= 0 ? x.prm[cv.b] : nullptr;
  a.stats = (bn_for_stats >= 0 && x.training) ? x.W<double>(x.p->bns[bn_for_stats].stats) : nullptr;
  if (a.stats) a.bn = bn_launch(x, bn_for_stats, (int64_t)x.p->cfg.N * out.H * out.W);
  if (fold_bn >= 0) {
    a.fold = bn_launch(x, fold_bn, (int64_t)x.p->cfg.N * out.H * out.W);
    a.fold.training = 0;
    a.fold_on = 1;
    a.fold_relu = relu ? 1 : 0;
    if (res) { a.add = x.A(*res); a.ldadd = res->ld; }
  }
  a.N = x.p->cfg.N; a.H = in.H; a.W = in.W; a.C = cv.Ci;
  a.P = out.H; a.Q = out.W; a.Cout = cv.Co;
  a.R = cv.R; a.S = cv.S; a.stride = cv.stride; a.pad = cv.pad;
  if (xbn >= 0) {
    a.xbn = bn_launch(x, xbn, (int64_t)x.p->cfg.N * in.H * in.W);
    a.xh = x.A(*xh); a.ldxh = xh->ld;
    a.xform = 1;
  }
  if (cv.f8) {  // e4m3 operands: quantize the input once per forward, block-scaled MFMA
    unet_plan* p = x.p;
    int fi = -1;
    for (int i = 0; i < (int)p->f8acts.size(); ++i)
      if (p->f8acts[i].src == in.off && p->f8acts[i].C == in.C) fi = i;
    if (fi < 0) { set_err("fp8 conv without a registered input"); return 1; }
    const F8Act& f = p->f8acts[fi];
    F8State* sts = x.W<F8State>(p->f8st);
    if (!p->f8_done[fi]) {
      ProfScope pq(p, x.st, "f8_quant " + pname(x, cv.w), 0);
      CK(launch_f8_quant_act(x.A(in), in.ld, in.C, (int64_t)a.N * in.H * in.W, x.W<uint8_t>(f.q), sts + f.st,
                             (p->f8_calibrated ? 0 : F8_CALIBRATE) | (x.training ? 0 : F8_FROZEN), x.st));
      p->f8_done[fi] = 1;
    }
    a.x = reinterpret_cast<const bf16_t*>(x.W<uint8_t>(f.q)); a.ldx = in.C;
    a.w = reinterpret_cast<const bf16_t*>(x.W<uint8_t>(cv.f8w));
    a.f8x = sts + f.st; a.f8w = sts + cv.f8st;
    CK(launch_conv_fwd_f8(a, x.st));
    return 0;
  }
  a.tim = tim_slot(x.p, "fwd " + pname(x, cv.w));
  if (cv.fl_fwd) {  // chunk-major pack: only conv3x3_fl_kernel reads it
    a.wch = a.w;
    a.w = nullptr;
    CK(launch_conv3x3_fl(a, 0, x.st));
    return 0;
  }
  if (dsf) {
    ConvFwdArgs b = a;
    b.wds = x.W<bf16_t>(x.p->convs[ds].pk_fwd);
    b.yds = x.A(*yds); b.ldyds = yds->ld;
    b.stats_ds = dsbn >= 0 ? x.W<double>(x.p->bns[dsbn].stats) : nullptr;
    if (b.stats_ds) b.bnds = bn_launch(x, dsbn, (int64_t)x.p->cfg.N * yds->H * yds->W);
    const hipError_t e = launch_conv_fwd(b, MODE_FWD, x.st);
    if (e != hipErrorNotSupported) {
      CK(e);
      if (ds_done) *ds_done = true;
      return 0;
    }
  }
  if (cv.kind == L_CONV && cv.R == 1 && cv.S == 1 && cv.stride == 1) {  // weight-stationary 1x1 where covered
    const hipError_t e = launch_conv1x1(a, 0, x.st);
    if (e != hipErrorNotSupported) {
      CK(e);
      return 0;
    }
  }
  if (cv.kind == L_CONVT) {  // weight-stationary up-conv (convt.hip) where it covers the shape
    const hipError_t e = launch_convt2x2(a, 0, x.st);
    if (e != hipErrorNotSupported || a.xform) {  // (an xform launch has no fallback)
      CK(e);
      return 0;
    }
  }
  CK(launch_conv_fwd(a, cv.kind == L_CONVT ? MODE_SHUF : MODE_FWD, x.st));
  return 0;
}

// can conv `ci` (input: raw y of BN bi's conv, output `out`) apply that BN +
// ReLU in its staging and store the activation `h` itself?
bool xform_ok(const Ctx& x, int ci, const Act& yraw, const Act& h, const Act& out) {
  const unet_plan* p = x.p;
  if (!x.training || !p->bn_xform || p->bn_ticket) return false;
  const Conv& cv = p->convs[ci];
  if (cv.f8 || cv.kind != L_CONV || h.H != yraw.H || h.W != yraw.W || h.C != yraw.C) return false;
  ConvFwdArgs a = {};
  a.ldx = yraw.ld; a.ldy = out.ld; a.ldxh = h.ld;
  a.N = p->cfg.N; a.H = yraw.H; a.W = yraw.W; a.C = cv.Ci;
  a.P = out.H; a.Q = out.W; a.Cout = cv.Co;
  a.R = cv.R; a.S = cv.S; a.stride = cv.stride; a.pad = cv.pad;
  return conv3x3_ws_xform_ok(a);
}

// the same for the next decoder level's up-conv (convt2x2_kernel forward):
// decoder level l's last BN + ReLU applied to the up-conv's pixel operand and
// the activation d.out stored by it (the plain U-Net: with attention the
// channel-attention forward reads d.out first)
bool up_xform_ok(const Ctx& x, int l) {
  const unet_plan* p = x.p;
  if (!x.training || !p->bn_xform || p->bn_ticket || !p->atts.empty() || l + 1 >= (int)p->decs.size()) return false;
  const Dec& d = p->decs[l];
  const Dec& n = p->decs[l + 1];
  const Conv& cv = p->convs[n.up];
  if (cv.f8 || cv.kind != L_CONVT || n.up_in.off != d.out.off || d.y2.C != d.out.C || d.y2.H != d.out.H ||
      d.y2.W != d.out.W)
    return false;
  ConvFwdArgs a = {};
  a.ldx = d.y2.ld; a.ldy = n.up_out.ld; a.ldxh = d.out.ld;
  a.N = p->cfg.N; a.H = d.y2.H; a.W = d.y2.W; a.C = cv.Ci; a.Cout = cv.Co;
  return cv.Ci == d.y2.C && convt2x2_xform_ok(a);
}

// conv dgrad: dx = dgrad(dy) (+ addend).  fuse: dx is dA of that BN(+ReLU);
// the epilogue stores dZ and runs the BN-backward reduction (ConvFwdArgs::bb).
// ds >= 0: the block's 1x1/s2 downsample dgrad (dY = dyds) is folded into this
// 3x3/s2 conv1 dgrad as a second reduction range of parity class 0.
// convT only: bias_acc = the up-conv's bias-gradient replicas; *bias_done tells
// whether the launch summed them (the weight-stationary kernel does, in the
// same pass over dY)
int conv_dgrad(const Ctx& x, int ci, const Act& dy, const Act& dx, const Act* add,
               const BnBwdArgs* fuse = nullptr, int ds = -1, const Act* dyds = nullptr,
               const Act* dx_split = nullptr, double* bias_acc = nullptr, bool* bias_done = nullptr) {
  const Conv& cv = x.p->convs[ci];
  const double fl = conv_flops(x.p, cv, dy) + (ds >= 0 ? conv_flops(x.p, x.p->convs[ds], *dyds) : 0.0);
  ProfScope ps(x.p, x.st, "dgrad " + pname(x, cv.w) + (ds >= 0 ? " +ds" : ""), fl);
  ConvFwdArgs a = {};
  a.x = x.A(dy); a.ldx = dy.ld;
  a.w = x.W<bf16_t>(cv.pk_dgrad);
  a.y = x.A(dx); a.ldy = dx.ld;
  if (add && add->ld) { a.add = x.A(*add); a.ldadd = add->ld; }
  if (fuse) a.bb = *fuse;
  if (dx_split) {  // channels >= dx.C go to their own buffer
    a.ysplit = x.A(*dx_split); a.ldysplit = dx_split->ld; a.csplit = dx.C;
  }
  if (ds >= 0) {
    const Conv& dv = x.p->convs[ds];
    a.x2 = x.A(*dyds); a.ldx2 = dyds->ld;
    a.w2 = x.W<bf16_t>(dv.pk_dgrad); a.C2 = dv.Co;
  }
  a.N = x.p->cfg.N;
  a.H = dy.H; a.W = dy.W;
  a.P = dx.H; a.Q = dx.W;
  a.R = cv.R; a.S = cv.S; a.stride = cv.stride; a.pad = cv.pad;
  a.C = cv.Co; a.Cout = cv.Ci;
  // convT: an ordinary k2s2 conv of dY; conv: the transposed gather
  a.tim = tim_slot(x.p, "dgrad " + pname(x, cv.w));
  if (cv.fl_dgrad) {  // chunk-major pack: only conv3x3_fl_kernel reads it
    a.wch = a.w;
    a.w = nullptr;
    CK(launch_conv3x3_fl(a, 1, x.st));
    return 0;
  }
  if (bias_done) *bias_done = false;
  if (cv.kind == L_CONV && cv.R == 1 && cv.S == 1 && cv.stride == 1 && !fuse) {  // weight-stationary 1x1
    const hipError_t e = launch_conv1x1(a, 1, x.st);
    if (e != hipErrorNotSupported) {
      CK(e);
      return 0;
    }
  }
  if (cv.kind == L_CONVT) {  // weight-stationary up-conv (convt.hip): its own geometry, the input grid
    ConvFwdArgs b = a;
    b.H = dx.H; b.W = dx.W; b.C = cv.Ci; b.Cout = cv.Co;
    b.P = dy.H; b.Q = dy.W;
    b.bias_acc = bias_acc;
    const hipError_t e = launch_convt2x2(b, 1, x.st);
    if (e != hipErrorNotSupported) {
      CK(e);
      if (bias_done) *bias_done = bias_acc != nullptr;
      return 0;
    }
  }
  if (cv.kind == L_CONVT && dy.ld == cv.Co && (2 * cv.Co) % 64 == 0 && dy.W % 2 == 0 && !a.x2 && !a.ysplit) {
    // ConvTranspose2d(k2, s2) data gradient = the k2s2 conv of dY.  Output
    // pixel (i, j) reads dY rows 2i, 2i+1 at columns 2j, 2j+1: in a dense dY
    // those column pairs are one contiguous 2*Co-channel "pixel", so the conv
    // runs as R = 2, S = 1, stride (2, 1) over W/2 merged pixels with K steps of
    // whole 128-B lines (the round-5 form staged 64-B half lines per tap).  The
    // PK_CONVT_DGRAD pack [Ci][a][b][Co] is already the [Ci][a][b*Co + c]
    // layout this view reads.
    a.W = dy.W / 2; a.C = 2 * cv.Co; a.ldx = 2 * dy.ld;
    a.R = 2; a.S = 1; a.stride = 2; a.stride_w = 1; a.pad = 0;
  }
  CK(launch_conv_fwd(a, cv.kind == L_CONVT ? MODE_FWD : MODE_TRANS, x.st));
  return 0;
}

// launch one weight gradient (args a, slab filled in here) and its split-K
// reduction, deferred into the next BN-backward apply launch when possible
int wgrad_and_reduce(const Ctx& x, ConvWgradArgs& a, int mode, const std::string& name, double flops) {
  unet_plan* p = x.p;
  const int si = p->slab_next;
  p->slab_next ^= 1;
  a.slab = x.W<float>(p->wslab + (size_t)si * p->wslab_bytes);
  a.slab_bytes = p->wslab_bytes;
  // a reduction deferred two wgrads ago (the one between had no split-K, and
  // no apply launch took it) still reads this slab: it runs first
  if (wgrad_deferred_reads(a.slab)) {
    ProfScope pr(p, x.rst, "wgrad_reduce (deferred)", 0);
    CK(launch_wgrad_flush(x.rst));
  }
  a.tim = tim_slot(p, "wgrad " + name);
  {
    ProfScope ps(p, x.wst, "wgrad " + name, flops);
    if (mode == 2) CK(launch_convt_wgrad(a, x.wst));
    else CK(launch_conv_wgrad(a, mode, x.wst));
  }
  if (!wgrad_pending()) return 0;
  if (p->merge_reduce && x.rst == x.wst && x.wst == x.st) {
    // one reduction at most waits for an apply launch; an older one runs now
    // (it reads the other slab, so the order against this wgrad is free)
    if (wgrad_deferred()) {
      ProfScope pr(p, x.rst, "wgrad_reduce (deferred)", 0);
      CK(launch_wgrad_flush(x.rst));
    }
    if (wgrad_defer()) return 0;
  }
  {
    ProfScope pr(p, x.rst, "wgrad_reduce " + name, 0);
    CK(launch_wgrad_finish(x.rst));
  }
  return 0;
}

// ds >= 0: the block's 1x1 / stride-2 downsample weight gradient (dY = *dyds,
// same input) folded into this 3x3 / stride-2 conv's launch (ds_fold_ok).
int conv_wgrad(const Ctx& x, int ci, const Act& dy, const Act& in, int ds = -1, const Act* dyds = nullptr) {
  const Conv& cv = x.p->convs[ci];
  ConvWgradArgs a = {};
  a.N = x.p->cfg.N;
  a.dw = x.W<float>(cv.wacc);
  a.R = cv.R; a.S = cv.S; a.stride = cv.stride; a.pad = cv.pad;
  if (cv.kind == L_CONVT) {
    // one GEMM over the input pixels: "dy" := X [Ci], "x" := dY gathered as
    // 4 output pixels x Co per input pixel (XLOAD_SHUF), dW [Ci][2][2][Co]
    a.dy = x.A(in); a.lddy = in.ld;
    a.x = x.A(dy); a.ldx = dy.ld;
    a.H = dy.H; a.W = dy.W; a.C = 4 * cv.Co;
    a.P = in.H; a.Q = in.W; a.Cout = cv.Ci;
    return wgrad_and_reduce(x, a, 2, pname(x, cv.w), conv_flops(x.p, cv, dy));
  }
  a.dy = x.A(dy); a.lddy = dy.ld;
  a.x = x.A(in); a.ldx = in.ld;
  a.H = in.H; a.W = in.W; a.C = cv.Ci;
  a.P = dy.H; a.Q = dy.W; a.Cout = cv.Co;
  double fl = conv_flops(x.p, cv, dy);
  std::string name = pname(x, cv.w);
  if (ds >= 0) {
    const Conv& dv = x.p->convs[ds];
    a.dy2 = x.A(*dyds); a.lddy2 = dyds->ld;
    a.dw2 = x.W<float>(dv.wacc);
    fl += conv_flops(x.p, dv, *dyds);
    name += " +ds";
  }
  if (x.p->wg_batch && wgrad_batch_ok(a)) {  // runs in the bucket's batch (flush_wgrad_batch)
    x.p->wgb.push_back(a);
    x.p->wgb_names.push_back(name);
    x.p->wgb_flops += fl;
    return 0;
  }
  return wgrad_and_reduce(x, a, 0, name, fl);
}

int flush_reduce(const Ctx& x);

// the collected weight gradients (conv_wgrad) as batched launches of at most
// kWbMaxLayers layers whose partials fit the halo slab (the per-layer
// reductions that read it have run: flush_reduce first)
int flush_wgrad_batch(const Ctx& x) {
  unet_plan* p = x.p;
  if (p->wgb.empty()) return 0;
  RUN(flush_reduce(x));
  const int grid = wgrad_batch_grid();
  const size_t cap = 2 * p->wslab_bytes / kWbPartBytes;  // slab slots
  size_t first = 0;
  while (first < p->wgb.size()) {
    // as many layers of one tile geometry as the table and the slab hold
    const int tw = wgrad_batch_tw(p->wgb[first]);
    size_t n = 0;
    while (first + n < p->wgb.size() && n < (size_t)kWbMaxLayers && wgrad_batch_tw(p->wgb[first + n]) == tw) ++n;
    WgBatchArgs b;
    for (;;) {
      b = WgBatchArgs{};
      b.grid = grid;
      b.N = p->cfg.N;
      b.tw = tw;
      long long items = 0;
      int units = 0;
      for (size_t j = 0; j < n; ++j) {
        const ConvWgradArgs& a = p->wgb[first + j];
        WgBatchLayer& L = b.L[j];
        L.dy = a.dy; L.x = a.x; L.dw = a.dw;
        L.H = a.H; L.W = a.W; L.C = a.C; L.Cout = a.Cout; L.lddy = a.lddy; L.ldx = a.ldx;
        L.tq = a.Q / tw; L.tp = a.P / (128 / tw);
        L.co_blocks = a.Cout / 64; L.c_blocks = a.C / 64;
        L.tiles = a.N * L.tp * L.tq;
        L.unit0 = units; L.item0 = items;
        units += L.co_blocks * L.c_blocks;
        items += (long long)L.co_blocks * L.c_blocks * L.tiles;
      }
      b.nl = (int)n; b.units = units; b.items = items;
      b.maxseg = wgrad_batch_maxseg(b);
      if ((size_t)grid * b.maxseg <= cap || n == 1) break;
      n = (n + 1) / 2;
    }
    if ((size_t)grid * b.maxseg > cap) {
      set_err("weight-gradient batch: slab too small");
      return -1;
    }
    b.slab = x.W<float>(p->wslab);
    std::string nm = "wgrad batch";
    for (size_t j = 0; j < n; ++j) nm += (j ? "," : " ") + p->wgb_names[first + j];
    b.tim = tim_slot(p, "wgrad batch x" + std::to_string(n));
    double fl = 0;
    for (size_t j = 0; j < n; ++j) {
      const ConvWgradArgs& a = p->wgb[first + j];
      fl += 2.0 * a.N * a.P * a.Q * a.Cout * a.C * 9;
    }
    {
      ProfScope ps(p, x.wst, nm, fl);
      CK(launch_wgrad_batch(b, x.wst));
    }
    first += n;
  }
  p->wgb.clear();
  p->wgb_names.clear();
  p->wgb_flops = 0;
  return 0;
}

// the downsample's weight gradient can ride in conv1's stride-2 halo wgrad
bool ds_fold_ok(const Ctx& x, const Block& b) {
  if (b.ds < 0 || b.bottleneck()) return false;
  const Conv& c1 = x.p->convs[b.conv1];
  const Conv& dv = x.p->convs[b.ds];
  if (dv.R != 1 || dv.stride != 2 || dv.pad != 0 || dv.Co != c1.Co || dv.Ci != c1.Ci) return false;
  ConvWgradArgs a = {};
  a.N = x.p->cfg.N;
  a.R = c1.R; a.S = c1.S; a.stride = c1.stride; a.pad = c1.pad;
  a.lddy = b.dy1.ld; a.ldx = b.in.ld; a.lddy2 = b.dyds.ld;
  a.dy2 = x.A(b.dyds);
  a.H = b.in.H; a.W = b.in.W; a.C = c1.Ci;
  a.P = b.dy1.H; a.Q = b.dy1.W; a.Cout = c1.Co;
  return b.dyds.H == b.dy1.H && b.dyds.W == b.dy1.W && wgrad_s2_fold_ok(a);
}

int bn_apply(const Ctx& x, int bi, const Act& y, const Act& out, int res_mode, const Act* res, int bi2,
             bool relu) {
  BnApplyArgs a = {};
  const int64_t npix = (int64_t)x.p->cfg.N * y.H * y.W;
  ProfScope ps(x.p, x.st, "bn_fwd " + pname(x, x.p->bns[bi].gamma), 0);
  a.y = x.A(y); a.ldy = y.ld;
  a.out = x.A(out); a.ldo = out.ld;
  a.bn = bn_launch(x, bi, npix);
  if (res_mode) { a.res = x.A(*res); a.ldr = res->ld; }
  if (res_mode == 2) a.bn2 = bn_launch(x, bi2, npix);
  a.npix = npix; a.C = y.C; a.res_mode = res_mode; a.relu = relu ? 1 : 0;
  CK(launch_bn_apply(a, x.st));
  return 0;
}

// BN(+ReLU) backward argument block for out = relu(bn(y) [+ bn2(y2) | + res]).
BnBwdArgs bwd_args(const Ctx& x, int bi, const Act& dout, const Act& out, const Act& y, const Act& dy,
                   int bi2, const Act* y2, const Act* dy2, const Act* dres, float* grads) {
  BnBwdArgs a = {};
  const Bn& b = x.p->bns[bi];
  a.da = x.A(dout); a.ldda = dout.ld;
  a.act = x.A(out); a.ldact = out.ld;
  a.y = x.A(y); a.ldy = y.ld;
  a.mean = x.W<float>(b.save); a.invstd = x.W<float>(b.save) + b.C; a.gamma = x.prm[b.gamma];
  a.sums = x.W<double>(b.bsums);
  a.dy = x.A(dy); a.lddy = dy.ld;
  a.dgamma = grads + x.p->params[b.gamma].flat;
  a.dbeta = grads + x.p->params[b.beta].flat;
  if (bi2 >= 0) {
    const Bn& b2 = x.p->bns[bi2];
    a.y2 = x.A(*y2); a.ldy2 = y2->ld;
    a.mean2 = x.W<float>(b2.save); a.invstd2 = x.W<float>(b2.save) + b2.C; a.gamma2 = x.prm[b2.gamma];
    a.sums2 = x.W<double>(b2.bsums);
    a.dy2 = x.A(*dy2); a.lddy2 = dy2->ld;
    a.dgamma2 = grads + x.p->params[b2.gamma].flat;
    a.dbeta2 = grads + x.p->params[b2.beta].flat;
  }
  if (dres) { a.dres = x.A(*dres); a.lddres = dres->ld; }
  a.ticket = x.p->bn_ticket ? x.W<unsigned>(b.tbwd) : nullptr;
  a.coef = x.p->bn_ticket ? x.W<float>(b.coef) : nullptr;
  a.npix = (int64_t)x.p->cfg.N * y.H * y.W; a.C = y.C; a.relu = 1;
  return a;
}

// fused: the producer of dA already stored dZ (in dA's buffer, which then also
// serves as the identity-residual gradient) and reduced it; only apply runs.
int bn_backward(const Ctx& x, int bi, BnBwdArgs a, bool fused) {
  ProfScope ps(x.p, x.st, "bn_bwd " + pname(x, x.p->bns[bi].gamma), 0);
  if (fused) {
    a.relu = 0;
    a.dres = nullptr;
  } else {
    CK(launch_bn_bwd_reduce(a, x.st));
  }
  ReduceTail r;
  if (wgrad_deferred() && x.wst == x.st && wgrad_take_deferred(&r)) {
    const hipError_t e = launch_bn_bwd_apply_reduce(a, r, x.st);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotSupported) CK(e);
    // this apply's shape cannot carry it: the reduction on its own, then the apply
    CK(launch_bn_bwd_apply(a, x.st));
    CK(launch_slab_reduce(r, x.st));
    return 0;
  }
  CK(launch_bn_bwd_apply(a, x.st));
  return 0;
}

// a deferred reduction that no apply launch took (bucket boundaries, end of
// the backward)
int flush_reduce(const Ctx& x) {
  if (!wgrad_deferred()) return 0;
  ProfScope pr(x.p, x.wst, "wgrad_reduce (deferred)", 0);
  CK(launch_wgrad_flush(x.wst));
  return 0;
}

int unpack_bucket(const Ctx& x, int bk, float* grads) {
  RUN(flush_wgrad_batch(x));
  RUN(flush_reduce(x));
  if (x.rst != x.wst) RUN(stream_edge(x.p, x.rst, x.wst));  // every reduction so far is in dW
  ProfScope ps(x.p, x.wst, "unpack", 0);
  UnpackTable local;
  local.n = 0;
  // no bucket events: nothing waits for this bucket before the backward ends,
  // so its entries join the pending table (fewer, fuller launches)
  const bool defer = x.p->nevents == 0;
  UnpackTable& t = defer ? x.p->pend : local;
  if (bk == 0) {
    // decoder (and attention W_g / W_x / psi) conv biases feed a training-mode
    // BN: their exact gradient is sum(dY) = 0 (BN removes the mean); written
    // here instead of one memset launch each
    auto zero = [&](int param) -> int {
      t.e[t.n++] = UnpackEntry{nullptr, grads + x.p->params[param].flat, UP_ZERO,
                               (int)x.p->params[param].numel, 1, 1, 1};
      if (t.n == kMaxPack) { CK(launch_unpack(t, x.wst)); t.n = 0; }
      return 0;
    };
    for (const Dec& d : x.p->decs) {
      RUN(zero(x.p->convs[d.conv1].b));
      RUN(zero(x.p->convs[d.conv2].b));
    }
    for (const Att& a : x.p->atts) {
      RUN(zero(x.p->convs[a.wg].b));
      RUN(zero(x.p->convs[a.wx].b));
      RUN(zero(a.psi_b));
    }
    // up-conv (ConvTranspose) bias gradients: the channel sums' fp64 replicas
    for (const Dec& d : x.p->decs) {
      if (d.up < 0) continue;
      const Conv& up = x.p->convs[d.up];
      t.e[t.n++] = UnpackEntry{reinterpret_cast<const float*>(x.W<double>(up.bias_acc)),
                               grads + x.p->params[up.b].flat, UP_D2F, up.Co, 1, 1, 1};
      if (t.n == kMaxPack) { CK(launch_unpack(t, x.wst)); t.n = 0; }
    }
  }
  for (int ci : x.p->bucket_convs[bk]) {
    const Conv& cv = x.p->convs[ci];
    UnpackEntry& e = t.e[t.n++];
    e.acc = x.W<float>(cv.wacc);
    e.dst = grads + x.p->params[cv.w].flat;
    e.R = cv.R; e.S = cv.S;
    if (cv.kind == L_CONV) { e.kind = UP_CONV; e.Co = cv.Co; e.Ci = cv.Ci; }
    else if (cv.kind == L_CONVT) { e.kind = UP_CONVT; e.Co = cv.Co; e.Ci = cv.Ci; }
    else { e.kind = UP_STEM; e.Co = cv.Co; e.Ci = 1; e.R = 7; e.S = 7; }
    if (t.n == kMaxPack) { CK(launch_unpack(t, x.wst)); t.n = 0; }
  }
  if (!defer || bk == (int)x.p->buckets.size() - 1) {  // the last bucket (the stem's) ends the backward
    CK(launch_unpack(t, x.wst));
    t.n = 0;
  }
  return 0;
}

}  // namespace


// attention-gate / channel-attention argument blocks of decoder level l
AttGateArgs gate_args(const Ctx& x, int l, float* grads) {
  const unet_plan* p = x.p;
  const Att& t = p->atts[l];
  const Dec& d = p->decs[l];
  const Bn& b = p->bns[t.psibn];
  AttGateArgs a = {};
  a.s = x.A(t.s); a.lds = t.s.ld;
  a.psi_w = x.prm[t.psi_w]; a.psi_b = x.prm[t.psi_b];
  a.p = x.W<float>(t.p); a.psi = x.W<float>(t.psi); a.dbnp = x.W<float>(t.dbnp);
  a.pst = x.W<double>(t.pst); a.pbs = x.W<double>(t.pbs); a.save = x.W<float>(t.psave);
  a.gamma = x.prm[b.gamma]; a.beta = x.prm[b.beta];
  a.run_mean = x.buf ? x.buf[3 * b.idx + 0] : nullptr;
  a.run_var = x.buf ? x.buf[3 * b.idx + 1] : nullptr;
  a.nbt = x.buf && x.training ? reinterpret_cast<long long*>(x.buf[3 * b.idx + 2]) : nullptr;
  a.npix = (int64_t)p->cfg.N * d.cat.H * d.cat.W;
  a.count = (double)a.npix; a.eps = p->cfg.bn_eps; a.momentum = p->cfg.bn_momentum; a.training = x.training;
  a.x = x.A(t.x); a.ldx = t.x.ld;
  const Act xs = slice(d.cat, 0, t.Fl);
  a.xatt = x.A(xs); a.ldxatt = xs.ld;
  a.dxatt = x.A(d.dcat); a.lddxatt = d.dcat.ld;  // skip channels come first (split or not)
  a.dxpsi = x.A(t.dxpsi); a.lddxpsi = t.dxpsi.ld;
  a.dS = x.A(t.dS); a.lddS = t.dS.ld;
  if (grads) {
    a.gpsi_w = grads + p->params[t.psi_w].flat;
    a.gpsi_acc = x.W<double>(t.gpsi);
    a.ggamma = grads + p->params[b.gamma].flat;
    a.gbeta = grads + p->params[b.beta].flat;
  }
  a.Fi = t.Fi; a.Fl = t.Fl;
  return a;
}

ChAttArgs ch_args(const Ctx& x, int l, float* grads) {
  const unet_plan* p = x.p;
  const Att& t = p->atts[l];
  const Dec& d = p->decs[l];
  ChAttArgs c = {};
  c.y = x.A(d.out); c.ldy = d.out.ld;
  c.out = x.A(t.out2); c.ldo = t.out2.ld;
  c.psum = x.W<double>(t.psum); c.pkey = x.W<unsigned long long>(t.pkey);
  c.gw_acc = x.W<double>(t.gfc);
  c.w1 = x.prm[t.fc1]; c.w2 = x.prm[t.fc2];
  c.am = x.W<float>(t.cam); c.h = x.W<float>(t.ch); c.gate = x.W<float>(t.ca);
  c.dout2 = x.A(t.d_out2); c.lddo2 = t.d_out2.ld;
  c.dgate = x.W<double>(t.cda); c.dam = x.W<float>(t.cdam);
  if (grads) {
    c.gw1 = grads + p->params[t.fc1].flat;
    c.gw2 = grads + p->params[t.fc2].flat;
  }
  c.dout = x.A(d.d_out); c.lddo = d.d_out.ld;
  c.HW = (int64_t)d.out.H * d.out.W;
  c.inv_hw = 1.0f / (float)c.HW;
  c.N = p->cfg.N; c.C = t.C; c.Cr = t.Cr;
  return c;
}

// AttentionGate forward (advanced_models.py:28-40): x_att = x * sigmoid(BN(psi(relu(BN(W_g g) + BN(W_x x)))))
int att_gate_forward(const Ctx& x, int l) {
  const Att& t = x.p->atts[l];
  const Dec& d = x.p->decs[l];
  RUN(conv_forward(x, t.wg, d.up_out, t.g1, t.bng));
  RUN(conv_forward(x, t.wx, t.x, t.xa, t.bnx));
  RUN(bn_apply(x, t.bng, t.g1, t.s, 2, &t.xa, t.bnx, true));
  const AttGateArgs a = gate_args(x, l, nullptr);
  ProfScope ps(x.p, x.st, "att_gate_fwd", 0);
  CK(launch_att_gate(a, 0, x.st));
  CK(launch_att_gate(a, 1, x.st));
  return 0;
}

// ChannelAttention forward (advanced_models.py:56-61)
int ch_att_forward(const Ctx& x, int l) {
  const ChAttArgs c = ch_args(x, l, nullptr);
  ProfScope ps(x.p, x.st, "ch_att_fwd", 0);
  for (int pass = 0; pass < 3; ++pass) CK(launch_ch_att(c, pass, x.st));
  return 0;
}

// the stem-by-recompute arguments shared by its forward and backward passes
StemRcArgs stem_rc_args(const Ctx& x, const float* image) {
  const unet_plan* p = x.p;
  const Conv& cv = p->convs[p->stem_conv];
  StemRcArgs s = {};
  s.img = image; s.H = p->cfg.H; s.W = p->cfg.W;
  s.w = x.W<bf16_t>(cv.pk_fwd);
  s.N = p->cfg.N; s.P = p->y0.H; s.Q = p->y0.W; s.Cout = cv.Co; s.Pp = p->p0.H; s.Qp = p->p0.W;
  s.bn = bn_launch(x, p->stem_bn, (int64_t)s.N * s.P * s.Q);
  s.stats = x.training ? x.W<double>(p->bns[p->stem_bn].stats) : nullptr;
  if (p->stem_keep) { s.y = x.A(p->y0); s.ldy = p->y0.ld; }
  s.act = x.A(p->x1); s.ldact = p->x1.ld;
  s.pool = x.A(p->p0); s.ldpool = p->p0.ld; s.idx = x.W<uint8_t>(p->pidx);
  return s;
}

static int run_forward(unet_plan* p, const float* image, const float* const* prm, float* const* buf, char* ws,
                       float* logits, int training, hipStream_t st) {
  Ctx x{p, ws, prm, buf, st, training};
  const int N = p->cfg.N;
  // the zeroed region: one PK_ZERO entry of the weight-pack launch below (the
  // first kernel of the step) unless the fp8 kernels run before that launch
  const size_t zbytes = p->zero_fwd_bytes + (training ? p->zero_bwd_bytes : 0);
  const bool zero_in_pack = !p->f8n && zbytes % 16 == 0 && zbytes / 16 < (size_t)INT32_MAX;
  if (!zero_in_pack) CK(hipMemsetAsync(ws + p->zero_fwd_off, 0, zbytes, st));
  // the backward accumulators were zeroed for THIS workspace (an eval forward or
  // another workspace makes the next unet_backward zero them itself)
  p->bwd_zeroed = training != 0;
  p->bwd_zeroed_ws = training ? ws : nullptr;
  if (p->f8n) {  // fp8 scale states: calibrate on the plan's first forward, else roll
    // (training only: an eval forward quantizes with the scales in use and
    // commits no amax, so validation never moves the training scales)
    if (!p->f8_calibrated) CK(hipMemsetAsync(ws + p->f8st, 0, (size_t)p->f8n * sizeof(F8State), st));
    else if (training) CK(launch_f8_roll(x.W<F8State>(p->f8st), p->f8n, st));
    std::fill(p->f8_done.begin(), p->f8_done.end(), 0);
    for (auto& cv : p->convs)
      if (cv.f8) {
        ProfScope ps(p, st, "f8_pack " + pname(x, cv.w), 0);
        CK(launch_f8_pack_w(prm[cv.w], cv.Co, cv.Ci, cv.R, cv.S, x.W<uint8_t>(cv.f8w), x.W<F8State>(p->f8st) + cv.f8st,
                            (p->f8_calibrated ? 0 : F8_CALIBRATE) | (training ? 0 : F8_FROZEN), st));
      }
  }
  // pack weights (fp32 torch layout -> bf16 kernel layouts)
  {
    PackTable t;
    t.n = 0;
    if (zero_in_pack)
      t.e[t.n++] = PackEntry{nullptr, reinterpret_cast<bf16_t*>(ws + p->zero_fwd_off), PK_ZERO, (int)(zbytes / 16), 0, 0, 0};
    auto flush = [&]() -> int {
      ProfScope ps(p, st, "pack", 0);
      CK(launch_pack(t, st));
      t.n = 0;
      return 0;
    };
    for (auto& cv : p->convs) {
      if (cv.kind == L_STEM) {
        t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_fwd), PK_STEM, cv.Co, 1, 7, 7};
      } else if (cv.kind == L_CONV) {
        const int fk = cv.fl_fwd ? PK_CONV_FWD_CH : PK_CONV_FWD;
        const int dk = cv.fl_dgrad ? PK_CONV_DGRAD_CH : PK_CONV_DGRAD;
        if (training && !cv.f8) {  // both layouts from one read of the fp32 weight
          t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_dgrad), dk, cv.Co, cv.Ci, cv.R, cv.S,
                                 x.W<bf16_t>(cv.pk_fwd), fk};
        } else {
          if (!cv.f8) t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_fwd), fk, cv.Co, cv.Ci, cv.R, cv.S};
          if (t.n == kMaxPack) RUN(flush());
          if (training) t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_dgrad), dk, cv.Co, cv.Ci, cv.R, cv.S};
        }
      } else {
        t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_fwd), PK_CONVT_FWD, cv.Co, cv.Ci, cv.R, cv.S};
        if (t.n == kMaxPack) RUN(flush());
        if (training) t.e[t.n++] = PackEntry{prm[cv.w], x.W<bf16_t>(cv.pk_dgrad), PK_CONVT_DGRAD, cv.Co, cv.Ci, cv.R, cv.S};
      }
      if (t.n >= kMaxPack - 1) RUN(flush());
    }
    RUN(flush());
  }
  // stem: conv7x7/s2 -> bn1 -> relu into cat1[:, :c0]; maxpool
  if (p->stem_rc) {
    StemRcArgs s = stem_rc_args(x, image);
    const double fl = 2.0 * N * p->y0.H * p->y0.W * p->convs[p->stem_conv].Co * 49;
    if (training) {
      ProfScope ps(p, st, "fwd input_conv.weight (stats)", fl);
      s.tim = tim_slot(p, "fwd input_conv.weight (stats)");
      CK(launch_stem_rc_fwd(s, 0, st));
    }
    ProfScope ps(p, st, "fwd input_conv.weight +bn+pool", fl);
    s.tim = tim_slot(p, "fwd input_conv.weight +bn+pool");
    CK(launch_stem_rc_fwd(s, 1, st));
  } else {
    const Conv& cv = p->convs[p->stem_conv];
    ConvFwdArgs a = {};
    a.x = reinterpret_cast<const bf16_t*>(image); a.ldx = 1;
    a.w = x.W<bf16_t>(cv.pk_fwd);
    a.y = x.A(p->y0); a.ldy = p->y0.ld;
    a.stats = training ? x.W<double>(p->bns[p->stem_bn].stats) : nullptr;
    if (a.stats) a.bn = bn_launch(x, p->stem_bn, (int64_t)N * p->y0.H * p->y0.W);
    a.N = N; a.H = p->cfg.H; a.W = p->cfg.W; a.C = 1;
    a.P = p->y0.H; a.Q = p->y0.W; a.Cout = cv.Co;
    a.R = 7; a.S = 7; a.stride = 2; a.pad = 3;
    {
      ProfScope ps(p, st, "fwd input_conv.weight", 2.0 * N * p->y0.H * p->y0.W * cv.Co * 49);
      CK(launch_conv_fwd(a, MODE_STEM, st));
    }
    // bn1 + relu + maxpool in one pass: x1 (the decoder1 skip, inside the
    // concat buffer) and the pooled p0 + argmax index
    MaxPoolArgs m = {};
    m.x = x.A(p->y0); m.ldx = p->y0.ld; m.y = x.A(p->p0); m.ldy = p->p0.ld; m.idx = x.W<uint8_t>(p->pidx);
    m.act = x.A(p->x1); m.ldact = p->x1.ld;
    m.bn = bn_launch(x, p->stem_bn, (int64_t)N * p->y0.H * p->y0.W);
    m.N = N; m.H = p->x1.H; m.W = p->x1.W; m.C = p->x1.C; m.P = p->p0.H; m.Q = p->p0.W;
    {
      ProfScope ps(p, st, "bn_relu_maxpool_fwd", 0);
      CK(launch_bn_relu_maxpool_fwd(m, st));
    }
  }
  // eval: every BN of the encoder / decoder blocks folded into its conv's
  // epilogue (running statistics; residual added there), no BN passes
  const bool fold = !training && p->eval_fold;
  for (auto& b : p->blocks) {
    if (b.bottleneck()) {  // torchvision Bottleneck (resnet50)
      if (fold) {
        RUN(conv_forward(x, b.conv1, b.in, b.h, -1, b.bn1, true));
        RUN(conv_forward(x, b.conv2, b.h, b.h2, -1, b.bn2, true));
        if (b.ds >= 0) RUN(conv_forward(x, b.ds, b.in, b.yds, -1, b.dsbn, false));
        RUN(conv_forward(x, b.conv3, b.h2, b.out, -1, b.bn3, true, b.ds >= 0 ? &b.yds : &b.in));
        continue;
      }
      RUN(conv_forward(x, b.conv1, b.in, b.y1, b.bn1));
      RUN(bn_apply(x, b.bn1, b.y1, b.h, 0, nullptr, -1, true));
      RUN(conv_forward(x, b.conv2, b.h, b.y2, b.bn2));
      RUN(bn_apply(x, b.bn2, b.y2, b.h2, 0, nullptr, -1, true));
      RUN(conv_forward(x, b.conv3, b.h2, b.y3, b.bn3));
      if (b.ds >= 0) {
        RUN(conv_forward(x, b.ds, b.in, b.yds, b.dsbn));
        RUN(bn_apply(x, b.bn3, b.y3, b.out, 2, &b.yds, b.dsbn, true));
      } else {
        RUN(bn_apply(x, b.bn3, b.y3, b.out, 1, &b.in, -1, true));
      }
      continue;
    }
    if (fold) {
      RUN(conv_forward(x, b.conv1, b.in, b.h, -1, b.bn1, true));
      if (b.ds >= 0) RUN(conv_forward(x, b.ds, b.in, b.yds, -1, b.dsbn, false));
      RUN(conv_forward(x, b.conv2, b.h, b.out, -1, b.bn2, true, b.ds >= 0 ? &b.yds : &b.in));
      continue;
    }
    // (a downsample block's 1x1 / stride-2 conv folded into conv1's launch)
    bool ds_done = false;
    RUN(conv_forward(x, b.conv1, b.in, b.y1, b.bn1, -1, false, nullptr, -1, nullptr, b.ds,
                     b.ds >= 0 ? &b.yds : nullptr, b.dsbn, &ds_done));
    if (xform_ok(x, b.conv2, b.y1, b.h, b.y2)) {  // bn1 + ReLU inside conv2's staging
      RUN(conv_forward(x, b.conv2, b.y1, b.y2, b.bn2, -1, false, nullptr, b.bn1, &b.h));
    } else {
      RUN(bn_apply(x, b.bn1, b.y1, b.h, 0, nullptr, -1, true));
      RUN(conv_forward(x, b.conv2, b.h, b.y2, b.bn2));
    }
    if (b.ds >= 0) {
      if (!ds_done) RUN(conv_forward(x, b.ds, b.in, b.yds, b.dsbn));
      RUN(bn_apply(x, b.bn2, b.y2, b.out, 2, &b.yds, b.dsbn, true));
    } else {
      RUN(bn_apply(x, b.bn2, b.y2, b.out, 1, &b.in, -1, true));
    }
  }
  const bool att = !p->atts.empty();
  const bool hfold = training && p->head_bn_fold;
  bool up_xf = false;  // the previous level's last BN + ReLU rides in this level's up-conv
  for (int l = 0; l < (int)p->decs.size(); ++l) {
    Dec& d = p->decs[l];
    if (up_xf) {
      const Dec& pd = p->decs[l - 1];
      RUN(conv_forward(x, d.up, pd.y2, d.up_out, -1, -1, false, nullptr, pd.bn2, &pd.out));
    } else {
      RUN(conv_forward(x, d.up, d.up_in, d.up_out, -1));
    }
    up_xf = !fold && up_xform_ok(x, l);
    if (att) RUN(att_gate_forward(x, l));
    if (fold) {
      RUN(conv_forward(x, d.conv1, d.cat, d.h, -1, d.bn1, true));
      RUN(conv_forward(x, d.conv2, d.h, d.out, -1, d.bn2, true));
    } else {
      RUN(conv_forward(x, d.conv1, d.cat, d.y1, d.bn1));
      if (xform_ok(x, d.conv2, d.y1, d.h, d.y2)) {
        RUN(conv_forward(x, d.conv2, d.y1, d.y2, d.bn2, -1, false, nullptr, d.bn1, &d.h));
      } else {
        RUN(bn_apply(x, d.bn1, d.y1, d.h, 0, nullptr, -1, true));
        RUN(conv_forward(x, d.conv2, d.h, d.y2, d.bn2));
      }
      if (!(hfold && l == 3) && !up_xf) RUN(bn_apply(x, d.bn2, d.y2, d.out, 0, nullptr, -1, true));
    }
    if (att) RUN(ch_att_forward(x, l));
  }
  {
    const Act& o = att ? p->atts[3].out2 : p->decs[3].out;
    HeadArgs h = {};
    h.x = x.A(o); h.ldx = o.ld;
    if (hfold) {  // the head reads decoder1's raw conv output and applies its last BN + ReLU
      const Dec& d = p->decs[3];
      h.x = x.A(d.y2); h.ldx = d.y2.ld;
      h.bn = bn_launch(x, d.bn2, (int64_t)N * d.y2.H * d.y2.W);
      h.bn_fold = 1;
    }
    h.w0 = prm[p->up0_w]; h.b0 = prm[p->up0_b]; h.wf = prm[p->fin_w]; h.bf = prm[p->fin_b];
    h.logits = logits;
    h.N = N; h.H = o.H; h.W = o.W; h.Cin = o.C; h.Co = (int)p->params[p->up0_b].numel;
    ProfScope ps(p, st, hfold ? "head_fwd +bn" : "head_fwd", 0);
    CK(launch_head_fwd(h, st));
  }
  return 0;
}

// a fresh event of the per-pass pool (reset at every backward)
int pooled_event(unet_plan* p, hipEvent_t* out) {
  if (p->syncused == (int)p->syncpool.size()) {
    hipEvent_t e;
    CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p->syncpool.push_back(e);
  }
  *out = p->syncpool[p->syncused++];
  return 0;
}

// `to` waits for everything issued so far on `from` (fresh pool event per
// edge, so the order is also right under stream capture)
int stream_edge(unet_plan* p, hipStream_t from, hipStream_t to) {
  if (from == to) return 0;
  hipEvent_t e;
  RUN(pooled_event(p, &e));
  CK(hipEventRecord(e, from));
  CK(hipStreamWaitEvent(to, e, 0));
  return 0;
}

static int run_backward(unet_plan* p, const float* image, const float* dlogits, const float* const* prm, char* ws,
                        float* grads, hipStream_t st) {
  Ctx x{p, ws, prm, nullptr, st, 1};
  const int N = p->cfg.N;
  wgrad_reset();  // nothing queued by an earlier backward that failed midway
  p->pend.n = 0;
  p->wgb.clear();
  p->wgb_names.clear();
  p->wgb_flops = 0;
  if (p->want_events) RUN(ensure_events(p));
  x.wst = st;
  x.rst = st;
  p->syncused = 0;
  // fork: the weight stream starts after the zeroing of the accumulators
  auto fork = [&]() { return stream_edge(p, st, x.wst); };
  if (!p->bwd_zeroed || p->bwd_zeroed_ws != ws) CK(hipMemsetAsync(ws + p->zero_bwd_off, 0, p->zero_bwd_bytes, st));
  p->bwd_zeroed = false;
  p->bwd_zeroed_ws = nullptr;
  const bool att = !p->atts.empty();
  // head (upconv0 + conv_final)
  {
    const Act& o = att ? p->atts[3].out2 : p->decs[3].out;
    HeadArgs h = {};
    h.x = x.A(o); h.ldx = o.ld;
    h.w0 = prm[p->up0_w]; h.b0 = prm[p->up0_b]; h.wf = prm[p->fin_w]; h.bf = prm[p->fin_b];
    h.dl = dlogits;
    const Act& hdx = att ? p->atts[3].d_out2 : p->decs[3].d_out;
    h.dx = x.A(hdx); h.lddx = hdx.ld;
    h.usum = x.W<double>(p->head_usum);
    h.gw0 = grads + p->params[p->up0_w].flat; h.gb0 = grads + p->params[p->up0_b].flat;
    h.gwf = grads + p->params[p->fin_w].flat; h.gbf = grads + p->params[p->fin_b].flat;
    h.N = N; h.H = o.H; h.W = o.W; h.Cin = o.C; h.Co = (int)p->params[p->up0_b].numel;
    if (p->fuse_bwd && !att) {  // the head produces dA of decoder1's last BN: reduce it here
      const Dec& d = p->decs[3];
      h.bb = bwd_args(x, d.bn2, d.d_out, d.out, d.y2, d.dy2, -1, nullptr, nullptr, nullptr, grads);
      if (p->head_bn_fold) {  // the forward never stored act: recomputed from y2 (same bits)
        h.x = x.A(d.y2); h.ldx = d.y2.ld;
        h.bb.act = nullptr;
        h.bn = bn_launch(x, d.bn2, (int64_t)N * d.y2.H * d.y2.W);
        h.bn_fold = 1;
      }
    }
    ProfScope ps(p, st, h.bn_fold ? "head_bwd +bn" : "head_bwd", 0);
    CK(launch_head_bwd(h, st));
    CK(launch_head_grads(h, st));
  }
  // BN-backward reductions are fused into the conv dgrad that produces each
  // BN's dA (all but decoder1's second BN, fed by the head, and the stem BN).
  const bool fz = p->fuse_bwd;
  const int nb = (int)p->blocks.size();
  auto dec_bn1 = [&](int l) {
    Dec& d = p->decs[l];
    return bwd_args(x, d.bn1, d.dh, d.h, d.y1, d.dy1, -1, nullptr, nullptr, nullptr, grads);
  };
  auto dec_bn2 = [&](int l) {
    Dec& d = p->decs[l];
    return bwd_args(x, d.bn2, d.d_out, d.out, d.y2, d.dy2, -1, nullptr, nullptr, nullptr, grads);
  };
  auto blk_bn1 = [&](int i) {
    Block& b = p->blocks[i];
    return bwd_args(x, b.bn1, b.dh, b.h, b.y1, b.dy1, -1, nullptr, nullptr, nullptr, grads);
  };
  // the block's last BN (bn2 of a BasicBlock, bn3 of a Bottleneck), paired
  // with the downsample BN when the block has one
  auto blk_bn2 = [&](int i) {
    Block& b = p->blocks[i];
    const int bl = b.last_bn();
    const Act& yl = b.last_y();
    const Act& dyl = b.last_dy();
    if (b.ds >= 0) return bwd_args(x, bl, b.d_out, b.out, yl, dyl, b.dsbn, &b.yds, &b.dyds, nullptr, grads);
    return bwd_args(x, bl, b.d_out, b.out, yl, dyl, -1, nullptr, nullptr, &b.dres, grads);
  };
  // decoder1 .. decoder4 (+ their up-convs)
  for (int l = 3; l >= 0; --l) {
    Dec& d = p->decs[l];
    if (att) {  // ChannelAttention backward: dOut2 -> dZ of the decoder's last BN (its reduction fused)
      ChAttArgs c = ch_args(x, l, grads);
      c.bb = dec_bn2(l);
      c.bb.ticket = nullptr;  // the apply recomputes its coefficients from the sums
      c.bb.coef = nullptr;
      {
        ProfScope ps(p, st, "ch_att_bwd", 0);
        for (int pass = 3; pass < 6; ++pass) CK(launch_ch_att(c, pass, st));
      }
      RUN(bn_backward(x, d.bn2, c.bb, true));
    }
    if (!att) RUN(bn_backward(x, d.bn2, dec_bn2(l), fz));
    RUN(fork());
    RUN(conv_wgrad(x, d.conv2, d.dy2, d.h));
    const BnBwdArgs f1 = dec_bn1(l);
    RUN(conv_dgrad(x, d.conv2, d.dy2, d.dh, nullptr, fz ? &f1 : nullptr));
    RUN(bn_backward(x, d.bn1, f1, fz));
    RUN(fork());
    RUN(conv_wgrad(x, d.conv1, d.dy1, d.cat));
    RUN(conv_dgrad(x, d.conv1, d.dy1, d.dcat, nullptr, nullptr, -1, nullptr, d.split ? &d.dcat_up : nullptr));
    // (decoder conv bias gradients: exactly 0, written by bucket 0's unpack)
    // up-conv: dU = dcat[:, skip:]; its dgrad is dA of the previous decoder's
    // (or enc4's) last BN
    if (att) {  // AttentionGate backward (skip gradient -> dskip, g-path gradient added into du)
      Att& t = p->atts[l];
      AttGateArgs a = gate_args(x, l, grads);
      // relu(BN_g + BN_x) backward: its reduction runs inside the gate's apply
      // pass (which produces dA and already reads the relu output)
      a.bb = bwd_args(x, t.bng, t.dS, t.s, t.g1, t.dg1, t.bnx, &t.xa, &t.dxa, nullptr, grads);
      a.bb.ticket = nullptr;  // the apply recomputes its coefficients from the sums
      a.bb.coef = nullptr;
      {
        ProfScope ps(p, st, "att_gate_bwd", 0);
        CK(launch_att_gate(a, 2, st));
        CK(launch_att_gate(a, 3, st));
      }
      RUN(bn_backward(x, t.bng, a.bb, true));
      RUN(fork());
      RUN(conv_wgrad(x, t.wg, t.dg1, d.up_out));
      RUN(conv_wgrad(x, t.wx, t.dxa, t.x));
      RUN(conv_dgrad(x, t.wg, t.dg1, t.du, &d.dcat_up));
      RUN(conv_dgrad(x, t.wx, t.dxa, t.dskip, &t.dxpsi));
      // (W_g / W_x / psi conv bias gradients: exactly 0, written by bucket 0's unpack)
    }
    const Conv& up = p->convs[d.up];
    const Act du = att ? p->atts[l].du : d.dcat_up;
    RUN(fork());
    RUN(conv_wgrad(x, d.up, du, d.up_in));
    const BnBwdArgs fu = l > 0 ? dec_bn2(l - 1) : blk_bn2(nb - 1);
    // with attention the up-conv input of levels 3..1 is the channel-gated
    // output: its gradient is not dA of a BN
    const bool fuse_up = fz && (l == 0 || !att);
    // the bias gradient (replicas -> fp32 in bucket 0's unpack launch, UP_D2F)
    // rides in the data-gradient pass when its kernel covers the shape
    bool bias_fused = false;
    RUN(conv_dgrad(x, d.up, du, d.d_up_in, nullptr, fuse_up ? &fu : nullptr, -1, nullptr, nullptr,
                   x.W<double>(up.bias_acc), &bias_fused));
    if (!bias_fused) {
      ProfScope ps(p, x.wst, "bias_sum", 0);
      CK(launch_channel_sum(x.A(du), du.ld, (int64_t)N * du.H * du.W, up.Co, x.W<double>(up.bias_acc), x.wst));
    }
  }
  // bucket 0 also holds the head's and the decoder biases' gradients (main stream)
  RUN(stream_edge(p, st, x.wst));
  RUN(unpack_bucket(x, 0, grads));
  if (p->nevents) CK(hipEventRecord(p->events[0], x.wst));
  // encoder blocks, deepest first
  for (int i = nb - 1; i >= 0; --i) {
    Block& b = p->blocks[i];
    if (b.bottleneck()) {
      RUN(bn_backward(x, b.bn3, blk_bn2(i), fz));  // dY3 (+ dY of the downsample BN)
      RUN(fork());
      RUN(conv_wgrad(x, b.conv3, b.dy3, b.h2));
      if (b.ds >= 0) RUN(conv_wgrad(x, b.ds, b.dyds, b.in));
      const BnBwdArgs f2 = bwd_args(x, b.bn2, b.dh2, b.h2, b.y2, b.dy2, -1, nullptr, nullptr, nullptr, grads);
      RUN(conv_dgrad(x, b.conv3, b.dy3, b.dh2, nullptr, fz ? &f2 : nullptr));
      RUN(bn_backward(x, b.bn2, f2, fz));
      RUN(fork());
      RUN(conv_wgrad(x, b.conv2, b.dy2, b.h));
      const BnBwdArgs f1 = blk_bn1(i);
      RUN(conv_dgrad(x, b.conv2, b.dy2, b.dh, nullptr, fz ? &f1 : nullptr));
      RUN(bn_backward(x, b.bn1, f1, fz));
      RUN(fork());
      RUN(conv_wgrad(x, b.conv1, b.dy1, b.in));
      BnBwdArgs fp = {};
      const BnBwdArgs* fprev = nullptr;
      if (fz && i > 0) { fp = blk_bn2(i - 1); fprev = &fp; }
      if (b.ds >= 0) {
        // downsample (1x1 / stride) data gradient (+ the skip-concat gradient
        // of the input), then conv1's (1x1) added to it with the previous
        // block's BN-backward reduction in the epilogue
        RUN(conv_dgrad(x, b.ds, b.dyds, b.dds, b.skip_add.ld ? &b.skip_add : nullptr));
        RUN(conv_dgrad(x, b.conv1, b.dy1, b.d_in, &b.dds, fprev));
      } else {
        RUN(conv_dgrad(x, b.conv1, b.dy1, b.d_in, fz ? &b.d_out : &b.dres, fprev));
      }
      if (i == 13 || i == 7) {
        const int bk = i == 13 ? 1 : 2;
        RUN(stream_edge(p, st, x.wst));
        RUN(unpack_bucket(x, bk, grads));
        if (p->nevents) CK(hipEventRecord(p->events[bk], x.wst));
      }
      continue;
    }
    RUN(bn_backward(x, b.bn2, blk_bn2(i), fz));
    RUN(fork());
    RUN(conv_wgrad(x, b.conv2, b.dy2, b.h));
    const bool dsfold = p->ds_wgrad_fold && ds_fold_ok(x, b);
    if (b.ds >= 0 && !dsfold) RUN(conv_wgrad(x, b.ds, b.dyds, b.in));
    const BnBwdArgs f1 = blk_bn1(i);
    RUN(conv_dgrad(x, b.conv2, b.dy2, b.dh, nullptr, fz ? &f1 : nullptr));
    RUN(bn_backward(x, b.bn1, f1, fz));
    RUN(fork());
    RUN(conv_wgrad(x, b.conv1, b.dy1, b.in, dsfold ? b.ds : -1, &b.dyds));
    // the last writer of d_in produces dA of the previous block's bn2
    BnBwdArgs fp = {};
    const BnBwdArgs* fprev = nullptr;
    if (fz && i > 0) { fp = blk_bn2(i - 1); fprev = &fp; }
    if (b.ds >= 0) {
      // conv1 (3x3/s2) and downsample (1x1/s2) data gradients in one launch
      RUN(conv_dgrad(x, b.conv1, b.dy1, b.d_in, b.skip_add.ld ? &b.skip_add : nullptr, fprev, b.ds, &b.dyds));
    } else {
      // identity path: dZ of bn2 (held in d_out when fused)
      RUN(conv_dgrad(x, b.conv1, b.dy1, b.d_in, fz ? &b.d_out : &b.dres, fprev));
    }
    // bucket boundaries (weight stream; BN parameter grads come from the main
    // stream's reductions): enc4 done at i == 13, enc3 at i == 7
    if (i == 13 || i == 7) {
      const int bk = i == 13 ? 1 : 2;
      RUN(stream_edge(p, st, x.wst));
      RUN(unpack_bucket(x, bk, grads));
      if (p->nevents) CK(hipEventRecord(p->events[bk], x.wst));
    }
  }
  // bucket 3 (enc2 + enc1) is final: its all-reduce overlaps the stem's backward
  {
    const int bk = (int)p->buckets.size() - 2;
    RUN(stream_edge(p, st, x.wst));
    RUN(unpack_bucket(x, bk, grads));
    if (p->nevents) CK(hipEventRecord(p->events[bk], x.wst));
  }
  // maxpool + stem
  if (p->stem_rc && fz) {
    // one pass: maxpool backward, stem BN backward, stem weight gradient
    StemRcArgs s = stem_rc_args(x, image);
    const Act skip = att ? p->atts[3].dskip : slice(p->decs[3].dcat, 0, p->x1.C);
    const BnBwdArgs sb = bwd_args(x, p->stem_bn, p->d_x1, p->x1, p->y0, p->d_y0, -1, nullptr, nullptr, nullptr,
                                  grads);
    s.dpool = x.A(p->d_p0); s.lddpool = p->d_p0.ld;
    s.add = x.A(skip); s.ldadd = skip.ld;
    s.mean = sb.mean; s.invstd = sb.invstd;
    if (p->stem_keep) { s.dz = x.A(p->d_x1); s.lddz = p->d_x1.ld; }
    s.part = x.W<float>(p->stem_part);
    s.l2 = reinterpret_cast<double*>(s.part + stem_rc_l2_offset(N, p->y0.H, p->y0.W, p->x1.C) / sizeof(float));
    s.tot = x.W<double>(p->stem_tot);
    s.tkt = x.W<unsigned>(p->stem_tkt);
    s.imsum = reinterpret_cast<float*>(reinterpret_cast<char*>(s.tot) + stem_rc_imsum_offset(p->x1.C));
    s.dw = x.W<float>(p->convs[p->stem_conv].wacc);
    s.dgamma = sb.dgamma; s.dbeta = sb.dbeta;
    s.npix = (int64_t)N * p->y0.H * p->y0.W;
    {
      ProfScope ps(p, st, "wgrad input_conv.weight +maxpool+bn", 3.0 * 2.0 * N * p->y0.H * p->y0.W * p->x1.C * 49);
      s.tim = tim_slot(p, "wgrad input_conv.weight +maxpool+bn");
      CK(launch_stem_rc_bwd(s, 0, st));
    }
    {
      ProfScope ps(p, st, "wgrad_reduce input_conv.weight", 0);
      CK(launch_stem_rc_bwd(s, 1, st));
    }
    RUN(fork());
  } else {
    MaxPoolArgs m = {};
    m.dy = x.A(p->d_p0); m.lddy = p->d_p0.ld; m.idx = x.W<uint8_t>(p->pidx);
    const Act skip = att ? p->atts[3].dskip : slice(p->decs[3].dcat, 0, p->x1.C);
    m.add = x.A(skip); m.ldadd = skip.ld;
    m.dx = x.A(p->d_x1); m.lddx = p->d_x1.ld;
    m.N = N; m.H = p->x1.H; m.W = p->x1.W; m.C = p->x1.C; m.P = p->p0.H; m.Q = p->p0.W;
    // the maxpool backward produces dA of the stem BN: fuse its reduction
    const BnBwdArgs sb = bwd_args(x, p->stem_bn, p->d_x1, p->x1, p->y0, p->d_y0, -1, nullptr, nullptr, nullptr,
                                  grads);
    if (fz) m.bb = sb;
    {
      ProfScope ps(p, st, "maxpool_bwd", 0);
      CK(launch_maxpool_bwd(m, st));
    }
    const Conv& cv = p->convs[p->stem_conv];
    // fused: the stem wgrad forms dY from dZ and y itself (no apply pass, dY never stored)
    const bool stem_fuse = fz && p->stem_bn_fuse && cv.Co % 64 == 0;
    if (!stem_fuse) RUN(bn_backward(x, p->stem_bn, sb, fz));
    RUN(fork());
    ConvWgradArgs a = {};
    a.dy = x.A(p->d_y0); a.lddy = p->d_y0.ld;
    if (stem_fuse) { a.bn = sb; a.bn_fuse = 1; }
    a.dw = x.W<float>(cv.wacc);
    a.N = N; a.H = p->cfg.H; a.W = p->cfg.W; a.C = 1;
    a.P = p->y0.H; a.Q = p->y0.W; a.Cout = cv.Co;
    a.R = 7; a.S = 7; a.stride = 2; a.pad = 3;
    a.x = reinterpret_cast<const bf16_t*>(image);
    RUN(wgrad_and_reduce(x, a, 1, "input_conv.weight", 2.0 * N * p->y0.H * p->y0.W * cv.Co * 49));
  }
  {
    const int bk = (int)p->buckets.size() - 1;
    RUN(unpack_bucket(x, bk, grads));
    if (p->nevents) CK(hipEventRecord(p->events[bk], x.wst));
  }
  // join: the caller's stream (optimizer, next forward) sees every gradient
  RUN(stream_edge(p, x.wst, st));
  return 0;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
#define API_GUARD(body)                                    \
  try {                                                    \
    body                                                   \
  } catch (const std::exception& e) {                      \
    set_err(std::string("exception: ") + e.what());        \
    return 1;                                              \
  } catch (...) {                                          \
    set_err("unknown exception");                          \
    return 1;                                              \
  }

extern "C" {

const char* unet_last_error(void) { return g_err.c_str(); }
const char* unet_version(void) { return "unet_hip 0.1 gfx950"; }

int unet_plan_create(const unet_config* cfg, unet_plan** out) {
  API_GUARD({
    if (!cfg || !out) { set_err("null argument"); return 1; }
    unet_plan* p = new unet_plan();
    p->cfg = *cfg;
    const int r = build_plan(p);
    if (r) { delete p; return r; }
    *out = p;
    return 0;
  })
}

void unet_plan_destroy(unet_plan* p) {
  if (!p) return;
  if (p->tim_buf) (void)hipFree(p->tim_buf);
  for (int i = 0; i < p->nevents; ++i) (void)hipEventDestroy(p->events[i]);
  for (hipEvent_t e : p->syncpool) (void)hipEventDestroy(e);
  delete p;
}

int64_t unet_plan_workspace_bytes(const unet_plan* p) { return p ? (int64_t)p->ws_bytes : -1; }
int unet_plan_num_params(const unet_plan* p) { return p ? (int)p->params.size() : -1; }
int unet_plan_param_name(const unet_plan* p, int i, char* buf, int buflen) {
  if (!p || i < 0 || i >= (int)p->params.size() || !buf || buflen <= 0) { set_err("bad index"); return 1; }
  std::snprintf(buf, (size_t)buflen, "%s", p->params[i].name.c_str());
  return 0;
}
int unet_plan_param_shape(const unet_plan* p, int i, int64_t shape[4]) {
  if (!p || i < 0 || i >= (int)p->params.size()) { set_err("bad index"); return -1; }
  const auto& s = p->params[i].shape;
  for (size_t k = 0; k < s.size() && k < 4; ++k) shape[k] = s[k];
  return (int)s.size();
}
int64_t unet_plan_param_offset(const unet_plan* p, int i) {
  if (!p || i < 0 || i >= (int)p->params.size()) return -1;
  return p->params[i].flat;
}
int64_t unet_plan_grad_numel(const unet_plan* p) { return p ? p->grad_numel : -1; }
int unet_plan_num_bn(const unet_plan* p) { return p ? (int)p->bns.size() : -1; }
int unet_plan_num_buckets(const unet_plan* p) { return p ? (int)p->buckets.size() : -1; }
int unet_plan_bucket_range(const unet_plan* p, int b, int64_t* begin, int64_t* end) {
  if (!p || b < 0 || b >= (int)p->buckets.size()) { set_err("bad bucket"); return 1; }
  *begin = p->buckets[b].first;
  *end = p->buckets[b].second;
  return 0;
}
double unet_plan_flops(const unet_plan* p, int training) {
  return p ? (training ? p->flops_train : p->flops_fwd) : -1.0;
}

int unet_plan_num_tensors(const unet_plan* p) { return p ? (int)p->named.size() : -1; }
int unet_plan_tensor_info(const unet_plan* p, int i, char* name, int namelen, int64_t info[5]) {
  if (!p || i < 0 || i >= (int)p->named.size() || !name || namelen <= 0) { set_err("bad tensor index"); return 1; }
  const auto& t = p->named[i];
  std::snprintf(name, (size_t)namelen, "%s", t.first.c_str());
  info[0] = (int64_t)t.second.off; info[1] = t.second.ld; info[2] = t.second.C;
  info[3] = t.second.H; info[4] = t.second.W;
  return 0;
}

int unet_forward(unet_plan* p, const float* image, const float* const* params, float* const* buffers,
                 void* workspace, float* logits, int training, hipStream_t stream) {
  API_GUARD({
    if (!p || !image || !params || !buffers || !workspace || !logits) { set_err("null argument"); return 1; }
    const int r = run_forward(p, image, params, buffers, reinterpret_cast<char*>(workspace), logits, training, stream);
    if (r == 0 && p->f8n) p->f8_calibrated = true;
    return r;
  })
}

int unet_backward(unet_plan* p, const float* image, const float* dlogits, const float* const* params,
                  void* workspace, float* grads, hipStream_t stream) {
  API_GUARD({
    if (!p || !image || !dlogits || !params || !workspace || !grads) { set_err("null argument"); return 1; }
    return run_backward(p, image, dlogits, params, reinterpret_cast<char*>(workspace), grads, stream);
  })
}

int unet_set_conv_config(int cfg) {
  set_conv_config(cfg);
  return 0;
}

int unet_plan_use_bucket_events(unet_plan* p, int on) {
  if (!p) { set_err("null plan"); return 1; }
  p->want_events = on != 0;
  return 0;
}

int unet_timing_enable(unet_plan* p, int on) {
  if (!p) { set_err("null plan"); return 1; }
  const size_t bytes = (size_t)kTimLaunches * kTimBlocks * kTimSlots * sizeof(unsigned long long);
  if (on && !p->tim_buf) CK(hipMalloc(&p->tim_buf, bytes));
  if (on) CK(hipMemset(p->tim_buf, 0, bytes));
  p->tim_on = on != 0;
  p->tim_n = 0;
  p->tim_names.clear();
  return 0;
}

int64_t unet_timing_read(unet_plan* p, unsigned long long* host, int64_t max_launches, char* names, int64_t nlen) {
  if (!p || !p->tim_buf) { set_err("timing not enabled"); return -1; }
  CK(hipDeviceSynchronize());
  const int64_t n = p->tim_n < max_launches ? p->tim_n : max_launches;
  if (host && n > 0)
    CK(hipMemcpy(host, p->tim_buf, (size_t)n * kTimBlocks * kTimSlots * sizeof(unsigned long long),
                 hipMemcpyDeviceToHost));
  std::string all;
  for (int64_t i = 0; i < n; ++i) all += p->tim_names[(size_t)i] + "\n";
  if (names && nlen > 0) std::snprintf(names, (size_t)nlen, "%s", all.c_str());
  return n;
}

int unet_profile_enable(unet_plan* p, int on) {
  if (!p) { set_err("null plan"); return 1; }
  p->prof = on != 0;
  p->recs.clear();
  p->evused = 0;
  return 0;
}

int unet_profile_report(unet_plan* p, char* buf, int64_t buflen) {
  if (!p) { set_err("null plan"); return -1; }
  std::string out;
  if (!p->recs.empty()) {
    if (hipEventSynchronize(p->evpool[p->recs.back().e1]) != hipSuccess) { set_err("event sync failed"); return -1; }
  }
  char num[64];
  for (const auto& r : p->recs) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p->evpool[r.e0], p->evpool[r.e1]) != hipSuccess) ms = -1.f;
    // names of batched launches list every layer: no fixed-size line buffer
    std::snprintf(num, sizeof(num), "\t%.6f\t%.6e\t", ms, r.flops);
    out += r.name;
    out += num;
    out += r.kernel;
    out += '\n';
  }
  if (buf && buflen > 0) std::snprintf(buf, (size_t)buflen, "%s", out.c_str());
  return (int)out.size() + 1;
}

int unet_bucket_wait(unet_plan* p, int bucket, hipStream_t waiter) {
  if (!p || bucket < 0 || bucket >= p->nevents) { set_err("bad bucket"); return 1; }
  CK(hipStreamWaitEvent(waiter, p->events[bucket], 0));
  return 0;
}

static_assert(UNET_LOSS_SCRATCH_LEN == 8 * kLossBlocks, "loss partial slots");

static bool loss_bufs_ok(const char* fn, const double* sums8, const double* scratch, int64_t scratch_len) {
  if (!sums8 || !scratch || scratch_len < UNET_LOSS_SCRATCH_LEN) {
    char m[160];
    std::snprintf(m, sizeof(m), "%s: sums8 / scratch null or scratch_len %lld < UNET_LOSS_SCRATCH_LEN (%d)", fn,
                  (long long)scratch_len, UNET_LOSS_SCRATCH_LEN);
    set_err(m);
    return false;
  }
  return true;
}

int unet_loss_forward(const float* logits, const float* target, int64_t n, int kind, float alpha, float smooth,
                      double* sums8, double* scratch, int64_t scratch_len, float* loss_out, hipStream_t stream) {
  if (!loss_bufs_ok("unet_loss_forward", sums8, scratch, scratch_len)) return 1;
  CK(launch_loss_sums(logits, target, n, sums8, scratch, 0, kind, alpha, smooth, loss_out, stream));
  return 0;
}

int unet_loss_backward(const float* logits, const float* target, int64_t n, int kind, float alpha, float smooth,
                       const double* sums8, const float* grad_scale, float* dlogits, hipStream_t stream) {
  CK(launch_loss_grad(logits, target, n, sums8, kind, alpha, smooth, grad_scale, dlogits, stream));
  return 0;
}

int unet_mask_metrics(const float* values, const float* target, int64_t n, int values_are_prob, double* sums8,
                      double* scratch, int64_t scratch_len, hipStream_t stream) {
  if (!loss_bufs_ok("unet_mask_metrics", sums8, scratch, scratch_len)) return 1;
  CK(launch_loss_sums(values, target, n, sums8, scratch, values_are_prob, 0, 0.f, 0.f, nullptr, stream));
  return 0;
}

int unet_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* step_coef,
                   int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
                   int advance_step, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!params || !grads || !exp_avg || !exp_avg_sq)) || !step_coef) {
    set_err("unet_adam_step: null buffer or negative size");
    return 1;
  }
  CK(launch_adam(params, grads, exp_avg, exp_avg_sq, n, step_coef, lr, beta1, beta2, eps, weight_decay, advance_step, stream));
  return 0;
}

int unet_grad_to_bf16(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!src || !dst))) {
    set_err("unet_grad_to_bf16: null buffer or negative size");
    return 1;
  }
  CK(launch_grad_to_bf16(src, (bf16_t*)dst, n, stream));
  return 0;
}

int unet_grad_from_bf16(const void* src, float* dst, int64_t n, float scale, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!src || !dst))) {
    set_err("unet_grad_from_bf16: null buffer or negative size");
    return 1;
  }
  CK(launch_grad_from_bf16((const bf16_t*)src, dst, n, scale, stream));
  return 0;
}

int unet_conv_fwd(const void* x, int ldx, const void* w, void* y, int ldy, const float* bias, const void* addend,
                  int ldadd, double* stats, int N, int H, int W, int C, int P, int Q, int Cout, int R, int S,
                  int stride, int pad, int mode, hipStream_t stream) {
  ConvFwdArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.w = (const bf16_t*)w; a.y = (bf16_t*)y; a.ldy = ldy;
  a.bias = bias; a.add = (const bf16_t*)addend; a.ldadd = ldadd; a.stats = stats;
  a.N = N; a.H = H; a.W = W; a.C = C; a.P = P; a.Q = Q; a.Cout = Cout;
  a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  if (mode < 0 || mode > 2) { set_err("bad mode"); return 1; }
  CK(launch_conv_fwd(a, mode, stream));
  return 0;
}

int unet_convt2x2(const void* x, int ldx, const void* w, void* y, int ldy, const float* bias, const void* act,
                  int ldact, const void* yraw, int ldyraw, const float* mean, const float* invstd, double* bsums,
                  double* bias_acc, int N, int H, int W, int Ci, int Co, int mode, int grid, hipStream_t stream) {
  if (mode != 0 && mode != 1) { set_err("unet_convt2x2: mode must be 0 (forward) or 1 (data gradient)"); return 1; }
  if (mode == 0 && (bsums || bias_acc)) { set_err("unet_convt2x2: bsums / bias_acc belong to the data gradient"); return 1; }
  if (bsums && (!act || !yraw || !mean || !invstd)) {
    set_err("unet_convt2x2: fused BN backward needs act, yraw, mean, invstd");
    return 1;
  }
  ConvFwdArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.w = (const bf16_t*)w; a.y = (bf16_t*)y; a.ldy = ldy;
  a.bias = mode == 0 ? bias : nullptr;
  a.N = N; a.H = H; a.W = W; a.C = Ci; a.Cout = Co; a.P = 2 * H; a.Q = 2 * W;
  a.R = 2; a.S = 2; a.stride = 2; a.pad = 0;
  a.grid_cap = grid;
  a.bias_acc = bias_acc;
  if (bsums) {
    a.bb.act = (const bf16_t*)act; a.bb.ldact = ldact; a.bb.y = (const bf16_t*)yraw; a.bb.ldy = ldyraw;
    a.bb.mean = mean; a.bb.invstd = invstd; a.bb.sums = bsums;
    a.bb.npix = (int64_t)N * H * W; a.bb.C = Ci; a.bb.relu = 1;
  }
  const hipError_t e = launch_convt2x2(a, mode, stream);
  if (e == hipErrorNotSupported) {
    set_err("unet_convt2x2: shape / alignment not covered ((Ci, Co) in {(64,32),(64,64),(128,64)}, N*H*W % 32)");
    return 1;
  }
  CK(e);
  return 0;
}

int unet_conv3x3_fl(const void* x, int ldx, const void* wch, void* y, int ldy, const float* bias, const void* addend,
                    int ldadd, double* stats, const void* act, int ldact, const void* yraw, int ldyraw,
                    const float* mean, const float* invstd, const void* yraw2, int ldyraw2, const float* mean2,
                    const float* invstd2, double* bsums, double* bsums2, int N, int H, int W, int C, int Cout,
                    int mode, int grid, hipStream_t stream) {
  if (mode != 0 && mode != 1) { set_err("unet_conv3x3_fl: mode must be 0 (conv) or 1 (data gradient)"); return 1; }
  if (!conv3x3_fl_geom(C, Cout, H, W) || N <= 0) {
    set_err("unet_conv3x3_fl: needs C % 128 == 0, Cout % 64 == 0, H % 16 == 0, W % 16 == 0, N > 0");
    return 1;
  }
  if (mode == 0 && bsums) { set_err("unet_conv3x3_fl: the fused BN backward is a data-gradient epilogue"); return 1; }
  if (bsums && (!act || !yraw || !mean || !invstd || (yraw2 && (!mean2 || !invstd2 || !bsums2)))) {
    set_err("unet_conv3x3_fl: fused BN backward needs act, yraw, mean, invstd (and mean2, invstd2, bsums2 with yraw2)");
    return 1;
  }
  ConvFwdArgs a = {};
  a.x = (const bf16_t*)x; a.ldx = ldx; a.wch = (const bf16_t*)wch; a.y = (bf16_t*)y; a.ldy = ldy;
  a.bias = bias; a.add = (const bf16_t*)addend; a.ldadd = ldadd; a.stats = mode == 0 ? stats : nullptr;
  a.N = N; a.H = H; a.W = W; a.C = C; a.P = H; a.Q = W; a.Cout = Cout;
  a.R = 3; a.S = 3; a.stride = 1; a.pad = 1;
  a.grid_cap = grid;
  if (bsums) {
    a.bb.act = (const bf16_t*)act; a.bb.ldact = ldact; a.bb.y = (const bf16_t*)yraw; a.bb.ldy = ldyraw;
    a.bb.mean = mean; a.bb.invstd = invstd; a.bb.sums = bsums;
    a.bb.npix = (int64_t)N * H * W; a.bb.C = Cout; a.bb.relu = 1;
    if (yraw2) {
      a.bb.y2 = (const bf16_t*)yraw2; a.bb.ldy2 = ldyraw2; a.bb.mean2 = mean2; a.bb.invstd2 = invstd2;
      a.bb.sums2 = bsums2;
    }
  }
  CK(launch_conv3x3_fl(a, mode, stream));
  return 0;
}

int unet_f8_quantize(const void* x, int ld, int C, int64_t npix, void* q, void* state, int calibrate,
                     hipStream_t stream) {
  CK(launch_f8_quant_act((const bf16_t*)x, ld, C, npix, (uint8_t*)q, (F8State*)state, calibrate, stream));
  return 0;
}

int unet_f8_pack_weight(const float* w, int Co, int Ci, int R, int S, void* dst, void* state, int calibrate,
                        hipStream_t stream) {
  CK(launch_f8_pack_w(w, Co, Ci, R, S, (uint8_t*)dst, (F8State*)state, calibrate, stream));
  return 0;
}

int unet_f8_roll(void* states, int n, hipStream_t stream) {
  CK(launch_f8_roll((F8State*)states, n, stream));
  return 0;
}

int unet_conv_fwd_f8(const void* xq, int ldx, const void* wq, const void* state_x, const void* state_w, void* y,
                     int ldy, const float* bias, const void* addend, int ldadd, double* stats, int N, int H, int W,
                     int C, int P, int Q, int Cout, int R, int S, int stride, int pad, hipStream_t stream) {
  ConvFwdArgs a = {};
  a.x = (const bf16_t*)xq; a.ldx = ldx; a.w = (const bf16_t*)wq; a.y = (bf16_t*)y; a.ldy = ldy;
  a.f8x = (const F8State*)state_x; a.f8w = (const F8State*)state_w;
  a.bias = bias; a.add = (const bf16_t*)addend; a.ldadd = ldadd; a.stats = stats;
  a.N = N; a.H = H; a.W = W; a.C = C; a.P = P; a.Q = Q; a.Cout = Cout;
  a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  CK(launch_conv_fwd_f8(a, stream));
  return 0;
}

int unet_conv_wgrad(const void* dy, int lddy, const void* x, int ldx, float* dw_acc, int N, int H, int W, int C,
                    int P, int Q, int Cout, int R, int S, int stride, int pad, int stem, hipStream_t stream) {
  ConvWgradArgs a = {};
  a.dy = (const bf16_t*)dy; a.lddy = lddy; a.x = (const bf16_t*)x; a.ldx = ldx; a.dw = dw_acc;
  a.N = N; a.H = H; a.W = W; a.C = C; a.P = P; a.Q = Q; a.Cout = Cout;
  a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  CK(launch_conv_wgrad(a, stem, stream));
  return 0;
}

int unet_conv_wgrad_slab(const void* dy, int lddy, const void* x, int ldx, float* dw, void* slab,
                         int64_t slab_bytes, int N, int H, int W, int C, int P, int Q, int Cout, int R, int S,
                         int stride, int pad, int stem, hipStream_t stream) {
  if (!slab || slab_bytes <= 0 || ((uintptr_t)slab & 15)) { set_err("unet_conv_wgrad_slab: bad slab"); return 1; }
  ConvWgradArgs a = {};
  a.dy = (const bf16_t*)dy; a.lddy = lddy; a.x = (const bf16_t*)x; a.ldx = ldx; a.dw = dw;
  a.slab = (float*)slab; a.slab_bytes = (size_t)slab_bytes;
  a.N = N; a.H = H; a.W = W; a.C = C; a.P = P; a.Q = Q; a.Cout = Cout;
  a.R = R; a.S = S; a.stride = stride; a.pad = pad;
  CK(launch_conv_wgrad(a, stem, stream));
  CK(launch_wgrad_finish(stream));
  return 0;
}

int unet_convt_wgrad_slab(const void* dy, int lddy, const void* x, int ldx, float* dw, void* slab,
                          int64_t slab_bytes, int N, int H, int W, int Ci, int Co, hipStream_t stream) {
  if (!slab || slab_bytes <= 0 || ((uintptr_t)slab & 15)) { set_err("unet_convt_wgrad_slab: bad slab"); return 1; }
  ConvWgradArgs a = {};  // as the executor: "dy" := X [N,H,W,Ci], "x" := dY [N,2H,2W,Co]
  a.dy = (const bf16_t*)x; a.lddy = ldx; a.x = (const bf16_t*)dy; a.ldx = lddy; a.dw = dw;
  a.slab = (float*)slab; a.slab_bytes = (size_t)slab_bytes;
  a.N = N; a.H = 2 * H; a.W = 2 * W; a.C = 4 * Co; a.P = H; a.Q = W; a.Cout = Ci;
  a.R = 2; a.S = 2; a.stride = 2; a.pad = 0;
  CK(launch_convt_wgrad(a, stream));
  CK(launch_wgrad_finish(stream));
  return 0;
}

int unet_pack_weight(const float* src, void* dst, int kind, int Co, int Ci, int R, int S, hipStream_t stream) {
  if (kind < PK_CONV_FWD || kind > PK_CONV_DGRAD_CH) { set_err("unet_pack_weight: kind must be 0..6"); return 1; }
  if ((kind == PK_CONV_FWD_CH || kind == PK_CONV_DGRAD_CH) &&
      (R != 3 || S != 3 || Co % 32 || Ci % 32)) {
    set_err("unet_pack_weight: chunk-major packs are 3x3 with Co, Ci multiples of 32");
    return 1;
  }
  PackTable t;
  t.n = 1;
  t.e[0] = PackEntry{src, (bf16_t*)dst, kind, Co, Ci, R, S};
  CK(launch_pack(t, stream));
  return 0;
}

int unet_unpack_grad(const float* acc, float* dst, int kind, int Co, int Ci, int R, int S, hipStream_t stream) {
  UnpackTable t;
  t.n = 1;
  t.e[0] = UnpackEntry{acc, dst, kind, Co, Ci, R, S};
  CK(launch_unpack(t, stream));
  return 0;
}

int unet_bn_forward(const void* y, int ldy, void* out, int ldo, const void* res, int ldr, int res_mode,
                    const double* stats, const float* gamma, const float* beta, float* run_mean, float* run_var,
                    float* save, int64_t npix, int C, int relu, int training, hipStream_t stream) {
  if (res_mode < 0 || res_mode > 1) { set_err("res_mode must be 0 or 1"); return 1; }
  BnApplyArgs a = {};
  a.y = (const bf16_t*)y; a.ldy = ldy; a.out = (bf16_t*)out; a.ldo = ldo;
  a.res = (const bf16_t*)res; a.ldr = ldr; a.res_mode = res_mode; a.relu = relu;
  a.bn.stats = stats; a.bn.gamma = gamma; a.bn.beta = beta; a.bn.run_mean = run_mean; a.bn.run_var = run_var;
  a.bn.save_mean = save; a.bn.save_invstd = save + C; a.bn.count = (double)npix; a.bn.C = C;
  a.bn.eps = 1e-5f; a.bn.momentum = 0.1f; a.bn.training = training;
  a.npix = npix; a.C = C;
  CK(launch_bn_apply(a, stream));
  return 0;
}

int unet_bn_backward(const void* dout, int ldd, const void* out, int ldo, const void* y, int ldy, const float* save,
                     const float* gamma, double* sums, void* dy, int lddy, void* dres, float* dgamma, float* dbeta,
                     int64_t npix, int C, hipStream_t stream) {
  BnBwdArgs a = {};
  a.da = (const bf16_t*)dout; a.ldda = ldd; a.act = (const bf16_t*)out; a.ldact = ldo;
  a.y = (const bf16_t*)y; a.ldy = ldy; a.mean = save; a.invstd = save + C; a.gamma = gamma;
  a.sums = sums; a.dy = (bf16_t*)dy; a.lddy = lddy; a.dres = (bf16_t*)dres; a.lddres = C;
  a.dgamma = dgamma; a.dbeta = dbeta; a.npix = npix; a.C = C; a.relu = 1;
  CK(launch_bn_bwd_reduce(a, stream));
  CK(launch_bn_bwd_apply(a, stream));
  return 0;
}

int unet_resize_area_u8(const uint8_t* src, int N, int H, int W, uint8_t* dst, int oh, int ow, hipStream_t stream) {
  if (!src || !dst) { set_err("unet_resize_area_u8: null buffer"); return 1; }
  CK(launch_resize_area(src, dst, N, H, W, oh, ow, stream));
  return 0;
}

int unet_mask_prep(const uint8_t* src, int N, int H, int W, float* dst, int oh, int ow, hipStream_t stream) {
  if (!src || !dst) { set_err("unet_mask_prep: null buffer"); return 1; }
  CK(launch_mask_prep(src, dst, N, H, W, oh, ow, stream));
  return 0;
}

int unet_normalize_microscopy(const uint8_t* src, int N, int H, int W, float* dst, int normalize,
                              hipStream_t stream) {
  if (!src || !dst) { set_err("unet_normalize_microscopy: null buffer"); return 1; }
  CK(launch_normalize(src, dst, N, H, W, normalize, stream));
  return 0;
}

int unet_rot90_vflip_u8(const uint8_t* src, int N, int H, int W, const int* k, const int* vflip, uint8_t* dst,
                        hipStream_t stream) {
  if (!src || !dst || !k || !vflip) { set_err("unet_rot90_vflip_u8: null buffer"); return 1; }
  CK(launch_rot90_vflip(src, dst, N, H, W, k, vflip, stream));
  return 0;
}

int unet_warp_affine_u8(const uint8_t* src, int N, int H, int W, const double* minv, const int* active,
                        const int* vflip, int nearest, uint8_t* dst, hipStream_t stream) {
  if (!src || !dst || !minv || !active || !vflip) { set_err("unet_warp_affine_u8: null buffer"); return 1; }
  CK(launch_warp_affine(src, dst, N, H, W, minv, active, vflip, nearest, stream));
  return 0;
}

int unet_filter2d_u8(const uint8_t* src, int N, int H, int W, const float* kernels, const int* ksize, uint8_t* dst,
                     hipStream_t stream) {
  if (!src || !dst || !kernels || !ksize) { set_err("unet_filter2d_u8: null buffer"); return 1; }
  CK(launch_filter2d(src, dst, N, H, W, kernels, ksize, stream));
  return 0;
}

// ---------------------------------------------------------------------------
// DDP gradient reduction over RCCL for non-Python hosts (SURVEY.md §8(b):
// "unet_allreduce_* ... communicator init from a ncclUniqueId byte blob";
// insertion point /root/reference/train.py:48-49).  RCCL is resolved at run
// time: the process's already-loaded RCCL (torch's, when a Python host loaded
// it globally) or /opt/rocm's librccl.so.1, so the library itself has no
// link-time RCCL dependency and plan-only / CPU users never load it.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllReduce) allreduce = nullptr;
  decltype(&ncclGetErrorString) errstr = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = nullptr;
    if (!dlsym(RTLD_DEFAULT, "ncclCommInitRank")) {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
      if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    }
    auto sym = [&](const char* n) { return h ? dlsym(h, n) : dlsym(RTLD_DEFAULT, n); };
    x.get_id = reinterpret_cast<decltype(x.get_id)>(sym("ncclGetUniqueId"));
    x.init = reinterpret_cast<decltype(x.init)>(sym("ncclCommInitRank"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(sym("ncclCommDestroy"));
    x.allreduce = reinterpret_cast<decltype(x.allreduce)>(sym("ncclAllReduce"));
    x.errstr = reinterpret_cast<decltype(x.errstr)>(sym("ncclGetErrorString"));
    x.ok = x.get_id && x.init && x.destroy && x.allreduce && x.errstr;
    return x;
  }();
  return r;
}
int rccl_check(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return 0;
  set_err(std::string(what) + ": " + rccl().errstr(r));
  return 1;
}
}  // namespace

struct unet_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, world = 1;
};

extern "C" {

static_assert(UNET_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "ncclUniqueId blob size");

int unet_allreduce_unique_id(void* id) {
  if (!id) { set_err("unet_allreduce_unique_id: null buffer"); return 1; }
  if (!rccl().ok) { set_err("unet_allreduce_unique_id: RCCL (librccl.so.1) not found"); return 1; }
  ncclUniqueId u;
  if (rccl_check(rccl().get_id(&u), "ncclGetUniqueId")) return 1;
  std::memcpy(id, &u, sizeof(u));
  return 0;
}

int unet_allreduce_init(const void* id, int rank, int world, unet_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) {
    set_err("unet_allreduce_init: null argument or rank outside [0, world)");
    return 1;
  }
  if (!rccl().ok) { set_err("unet_allreduce_init: RCCL (librccl.so.1) not found"); return 1; }
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  unet_comm* c = new unet_comm();
  c->rank = rank;
  c->world = world;
  if (rccl_check(rccl().init(&c->comm, world, u, rank), "ncclCommInitRank")) {
    delete c;
    return 1;
  }
  *out = c;
  return 0;
}

void unet_allreduce_destroy(unet_comm* c) {
  if (!c) return;
  if (c->comm && rccl().ok) (void)rccl().destroy(c->comm);
  delete c;
}

int unet_allreduce_mean(unet_comm* c, float* buf, int64_t n, hipStream_t stream) {
  if (!c || n < 0 || (n > 0 && !buf)) { set_err("unet_allreduce_mean: null communicator / buffer"); return 1; }
  if (n == 0) return 0;
  return rccl_check(rccl().allreduce(buf, buf, (size_t)n, ncclFloat32, ncclAvg, c->comm, stream), "ncclAllReduce");
}

int unet_allreduce_bucket(unet_comm* c, unet_plan* p, float* grads, int bucket, hipStream_t comm_stream) {
  if (!c || !p || !grads || bucket < 0 || bucket >= (int)p->buckets.size()) {
    set_err("unet_allreduce_bucket: null argument or bad bucket");
    return 1;
  }
  // after the bucket's event when the last backward recorded one (DDP overlap);
  // otherwise the caller has ordered comm_stream after the whole backward
  if (bucket < p->nevents) CK(hipStreamWaitEvent(comm_stream, p->events[bucket], 0));
  const auto& r = p->buckets[(size_t)bucket];
  return unet_allreduce_mean(c, grads + r.first, r.second - r.first, comm_stream);
}

int unet_maxpool_fwd(const void* x, int ldx, void* y, uint8_t* idx, int N, int H, int W, int C,
                     hipStream_t stream) {
  MaxPoolArgs m = {};
  m.x = (const bf16_t*)x; m.ldx = ldx; m.y = (bf16_t*)y; m.ldy = C; m.idx = idx;
  m.N = N; m.H = H; m.W = W; m.C = C; m.P = (H + 1) / 2; m.Q = (W + 1) / 2;
  CK(launch_maxpool_fwd(m, stream));
  return 0;
}

int unet_maxpool_bwd(const void* dy, const uint8_t* idx, const void* addend, int ldadd, void* dx, int N, int H,
                     int W, int C, hipStream_t stream) {
  MaxPoolArgs m = {};
  m.dy = (const bf16_t*)dy; m.lddy = C; m.idx = (uint8_t*)idx; m.add = (const bf16_t*)addend; m.ldadd = ldadd;
  m.dx = (bf16_t*)dx; m.lddx = C;
  m.N = N; m.H = H; m.W = W; m.C = C; m.P = (H + 1) / 2; m.Q = (W + 1) / 2;
  CK(launch_maxpool_bwd(m, stream));
  return 0;
}

}  // extern "C"

/* unet_hip.h — C ABI of libunet_hip.so, the MI355X (gfx950) U-Net training path.
 *
 * Drop-in boundary for the reference's hot path (SwagMag1213/image-segmentation-
 * project, /root/reference).  The reference is pure Python over PyTorch, so its
 * "FFI" is the Python API; each entry point below replaces the compute under one
 * reference call (file:line in /root/reference):
 *
 *   unet_forward         UNetWithBackbone.forward (advanced_models.py:264-357),
 *                        resnet34 encoder (:72-100), use_attention=False
 *   unet_backward        loss.backward() through that graph (train.py:48)
 *   unet_bucket_wait     DDP gradient reduction insertion point between
 *                        loss.backward() and optimizer.step() (train.py:48-49)
 *   unet_loss_forward    BCELoss / DiceLoss / ComboLoss forward (losses.py:13-37,161-171)
 *   unet_loss_backward   their gradient wrt the logits
 *   unet_mask_metrics    calculate_metrics tp/fp/fn/tn counts (utils.py:120-151)
 *   unet_adam_step       optimizer.step() of torch.optim.Adam(model.parameters(),
 *                        lr, weight_decay) (train.py:49,331-335)
 *   unet_conv_* / unet_maxpool_* / unet_bn_*   single ops of the graph above
 *                        (torchvision BasicBlock, advanced_models.py:197-205) for tests
 *
 * Conventions: every pointer is a DEVICE pointer owned by the caller (PyTorch's
 * caching allocator); the library never allocates or frees on the hot path.
 * Activations are bf16 NHWC; parameters / grads fp32 in torch layouts.  All work
 * is enqueued asynchronously on the given hipStream_t.  Every function returns
 * 0 on success or a non-zero hipError_t-style code; unet_last_error() gives a
 * thread-local message.  No C++ exception crosses the ABI.
 */
#ifndef UNET_HIP_H
#define UNET_HIP_H
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct unet_plan unet_plan;

typedef struct unet_config {
  int N, H, W;       /* batch and input size (H, W multiples of 32)            */
  int width;         /* channel multiplier: 1 = resnet34 U-Net (64..512)       */
  int n_classes;     /* must be 1 (binary segmentation, advanced_models.py:160) */
  float bn_eps;      /* 1e-5  (torch.nn.BatchNorm2d default)                   */
  float bn_momentum; /* 0.1                                                    */
  int attention;     /* 1: AttentionGate + ChannelAttention decoder            */
                     /*    (use_attention=True, advanced_models.py:7-61,163-172) */
  int backbone;      /* 34: resnet34 (BasicBlock encoder, advanced_models.py:72-100);     */
                     /* 50: resnet50 (Bottleneck encoder 256..2048, :102-130,158-159)     */
  int fp8;           /* 1: forward convs with >= 128 input channels in fp8 e4m3 (per-tensor */
                     /*    delayed scaling, block-scaled MFMA); backward stays bf16.        */
                     /*    Build extension for BASELINE configs[4] (Wide fp8); resnet34,   */
                     /*    no attention.  The reference trains in fp32 only.               */
} unet_config;

const char* unet_last_error(void);
const char* unet_version(void);

/* ---- plan: layer graph, parameter table, workspace layout ---- */
int unet_plan_create(const unet_config* cfg, unet_plan** out);
void unet_plan_destroy(unet_plan* p);
int64_t unet_plan_workspace_bytes(const unet_plan* p);
int unet_plan_num_params(const unet_plan* p);
int unet_plan_param_name(const unet_plan* p, int i, char* buf, int buflen);
int unet_plan_param_shape(const unet_plan* p, int i, int64_t shape[4]); /* returns ndim */
int64_t unet_plan_param_offset(const unet_plan* p, int i);             /* in flat grads */
int64_t unet_plan_grad_numel(const unet_plan* p);
int unet_plan_num_bn(const unet_plan* p);
int unet_plan_num_buckets(const unet_plan* p);
int unet_plan_bucket_range(const unet_plan* p, int b, int64_t* begin, int64_t* end);
double unet_plan_flops(const unet_plan* p, int training); /* algorithmic FLOPs per step */
/* named workspace views (tests): info = {byte offset, ld, C, H, W} of a bf16 NHWC tensor */
int unet_plan_num_tensors(const unet_plan* p);
int unet_plan_tensor_info(const unet_plan* p, int i, char* name, int namelen, int64_t info[5]);

/* params[i]: fp32 tensors in unet_plan_param_name order (== reference
 * state_dict parameter order); buffers[3*k+0/1/2]: running_mean/var (fp32) and
 * num_batches_tracked (int64) of BN k in named_buffers order.  A training
 * forward updates the running statistics and adds 1 to num_batches_tracked,
 * as torch.nn.BatchNorm2d.train() does. */
int unet_forward(unet_plan* p, const float* image, const float* const* params, float* const* buffers,
                 void* workspace, float* logits, int training, hipStream_t stream);
/* grads: flat fp32 [unet_plan_grad_numel], param i at unet_plan_param_offset(i).
 * Ordering contract: unet_backward differentiates the LAST training
 * unet_forward of the same plan and workspace (its saved activations and BN
 * statistics).  A training forward also zeroes the backward's accumulators
 * inside its first launch; if the workspace differs, or an eval forward came in
 * between, unet_backward zeroes them itself (one memset), so a mismatched call
 * order is never silently wrong about the accumulators -- but the gradients
 * are only meaningful for the pairing above.
 * unet_plan_create queries the current device's CU count (HIP runtime init);
 * use the plan on that device. */
int unet_backward(unet_plan* p, const float* image, const float* dlogits, const float* const* params,
                  void* workspace, float* grads, hipStream_t stream);
/* record one hipEvent per gradient bucket in every unet_backward (DDP overlap) */
int unet_plan_use_bucket_events(unet_plan* p, int on);
/* make `waiter` wait until bucket b of the last unet_backward is final */
int unet_bucket_wait(unet_plan* p, int bucket, hipStream_t waiter);
/* per-launch hipEvent profiler: enable (clears records), then report lines
 * "name\tms\tflops\n" for every launch since; returns bytes needed (incl. NUL). */
/* In-kernel phase timing of the conv launches (a debug aid; the stamps are
 * written only by a library built with -DUNET_TIMING, `make timing`): enable
 * zeroes a device buffer of kTimLaunches x 1024 blocks x 32 u64 stamps and gives
 * every following conv launch of the plan the next slot; read copies the slots
 * used so far to `host` (max_launches slots) and the launch names (one per
 * line) to `names`, and returns the number of slots used. */
int unet_timing_enable(unet_plan* p, int on);
int64_t unet_timing_read(unet_plan* p, unsigned long long* host, int64_t max_launches, char* names, int64_t nlen);
int unet_profile_enable(unet_plan* p, int on);
int unet_profile_report(unet_plan* p, char* buf, int64_t buflen);

/* ---- loss + metrics (kind: 0 bce, 1 dice, 2 combo) ---- */
/* sums8: exactly 8 doubles out, the sums (bce, sigma*y, sigma, y, tp, fp, fn, tn).
 * scratch: caller-owned device scratch of scratch_len >= UNET_LOSS_SCRATCH_LEN
 * doubles for the per-block partials, which the library reduces in a fixed
 * order (no atomics: the sums are bit-reproducible); a shorter or null scratch
 * is rejected with an error before anything is launched.  Nothing needs to be
 * zeroed beforehand.  (Round 5 wrote the partials behind sums8; the separate,
 * length-checked scratch makes an 8-double sums8 buffer safe again.) */
#define UNET_LOSS_SCRATCH_LEN (8 * 256)
int unet_loss_forward(const float* logits, const float* target, int64_t n, int kind, float alpha,
                      float smooth, double* sums8, double* scratch, int64_t scratch_len, float* loss_out,
                      hipStream_t stream);
int unet_loss_backward(const float* logits, const float* target, int64_t n, int kind, float alpha,
                       float smooth, const double* sums8, const float* grad_scale, float* dlogits,
                       hipStream_t stream);
/* sums8[4..8) = tp, fp, fn, tn.  values_are_prob=0: logits (mask = sigmoid>0.5
 * evaluated bit-exactly as logit >= 0x33C00001); 1: probabilities (p > 0.5).
 * scratch / scratch_len as for unet_loss_forward. */
int unet_mask_metrics(const float* values, const float* target, int64_t n, int values_are_prob,
                      double* sums8, double* scratch, int64_t scratch_len, hipStream_t stream);

/* ---- optimizer ---- */
/* One Adam step (coupled L2 weight decay, torch.optim.Adam semantics) over n
 * fp32 elements of four flat buffers.  step_coef[3] is device memory:
 * step_coef[0] is the step count (incremented on device, so the call is
 * graph-capturable) when advance_step != 0, and [1], [2] then receive
 * step_size = lr/(1-b1^t) and sqrt(1-b2^t); advance_step = 0 reuses them
 * (several slices updated in one optimizer step).  exp_avg / exp_avg_sq must
 * be zero before the first step. */
int unet_adam_step(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* step_coef,
                   int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
                   int advance_step, hipStream_t stream);

/* ---- DDP gradient reduction over RCCL (non-Python hosts) ----
 * The reference trains in one process; these sit at its DDP insertion point,
 * between loss.backward() and optimizer.step() (train.py:48-49), and replace
 * torch.distributed for a C / C++ / FFI host.  RCCL (the
 * process's own, else /opt/rocm's librccl.so.1) is resolved at run time.
 * Rank 0 calls unet_allreduce_unique_id and ships the UNET_UNIQUE_ID_BYTES blob
 * to every rank out of band; each rank (one process per GPU, its device
 * current) calls unet_allreduce_init -- collective over the world.
 * unet_allreduce_bucket: mean all-reduce, in place in the flat fp32 gradient
 * buffer, of bucket `bucket` (unet_plan_bucket_range) of the last
 * unet_backward, enqueued on comm_stream after that bucket's hipEvent when
 * unet_plan_use_bucket_events(p, 1) was on during that backward (the
 * all-reduce then overlaps the rest of the backward); otherwise the caller
 * orders comm_stream after the backward.  The caller orders its compute
 * stream after comm_stream before optimizer.step().  Graph-capturable. */
#define UNET_UNIQUE_ID_BYTES 128
typedef struct unet_comm unet_comm;
int unet_allreduce_unique_id(void* id);
int unet_allreduce_init(const void* id, int rank, int world, unet_comm** out);
void unet_allreduce_destroy(unet_comm* c);
int unet_allreduce_bucket(unet_comm* c, unet_plan* p, float* grads, int bucket, hipStream_t comm_stream);
/* mean all-reduce of n floats in place (any flat buffer) */
int unet_allreduce_mean(unet_comm* c, float* buf, int64_t n, hipStream_t stream);

/* ---- bf16 gradient exchange (opt-in DDP compression) ----
 * Replace nothing in the reference (it trains in one process); they sit at
 * the DDP insertion point train.py:48-49, around each bucket's all-reduce:
 * dst[i] = bf16_rne(src[i]) before it, dst[i] = float(src[i]) * scale after
 * it (scale = 1/world for a SUM collective).  n elements; any alignment (16-B
 * aligned buffers take the 8-wide path). */
int unet_grad_to_bf16(const float* src, void* dst, int64_t n, hipStream_t stream);
int unet_grad_from_bf16(const void* src, float* dst, int64_t n, float scale, hipStream_t stream);

/* ---- single ops (tests / custom graphs) ---- */
/* mode 0: conv  y = conv(x, w) [stride, pad]           (w packed [Cout][R][S][C])
 * mode 1: transposed gather (conv dgrad / ConvTranspose2d forward)
 * mode 2: 7x7 stem on an fp32 single-channel image     (w packed [64][64]) */
int unet_conv_fwd(const void* x, int ldx, const void* w, void* y, int ldy, const float* bias,
                  const void* addend, int ldadd, double* stats, int N, int H, int W, int C, int P,
                  int Q, int Cout, int R, int S, int stride, int pad, int mode, hipStream_t stream);
int unet_conv_wgrad(const void* dy, int lddy, const void* x, int ldx, float* dw_acc, int N, int H,
                    int W, int C, int P, int Q, int Cout, int R, int S, int stride, int pad, int stem,
                    hipStream_t stream);
/* the same with the executor's deterministic split-K: partials in the caller's
 * 16-B aligned `slab` scratch, summed in a fixed split order; every element of
 * dw is WRITTEN (no zeroing needed, bit-reproducible).  The convT form computes
 * ConvTranspose2d(k2, s2) dW [Ci][Co][2][2]-packed as [Ci][4*Co] from
 * x [N,H,W,Ci] and dy [N,2H,2W,Co]. */
int unet_conv_wgrad_slab(const void* dy, int lddy, const void* x, int ldx, float* dw, void* slab,
                         int64_t slab_bytes, int N, int H, int W, int C, int P, int Q, int Cout, int R,
                         int S, int stride, int pad, int stem, hipStream_t stream);
int unet_convt_wgrad_slab(const void* dy, int lddy, const void* x, int ldx, float* dw, void* slab,
                          int64_t slab_bytes, int N, int H, int W, int Ci, int Co, hipStream_t stream);
/* The full-line halo conv (conv3x3_fl_kernel: every 3x3 / stride-1 conv with
 * C >= 128 that fills the chip, i.e. the enc2 / enc3 BasicBlocks and decoder4 /
 * decoder3 of the reference, advanced_models.py:84-87,197-205) as a single op.
 * C % 128 == 0, Cout % 64 == 0, H % 16 == 0, W % 16 == 0 (here C = the op's
 * input channels, Cout its output channels).  wch: the chunk-major pack of
 * unet_pack_weight kind 5 (mode 0, forward weight [Cout][C][3][3]) or kind 6
 * (mode 1, data gradient of a forward conv whose weight is [C][Cout][3][3]).
 * mode 0: y = conv3x3(x) (+bias)(+addend); stats != null: BN sums of y into
 *   stats[16][2][Cout] (fp64 atomics, caller zeroes).
 * mode 1: y = conv3x3_transpose(x) (+addend); bsums != null: the fused BN(+ReLU)
 *   backward epilogue: y := dZ = dA * (act > 0) and bsums[16][2][Cout] +=
 *   (sum dZ, sum dZ * (yraw - mean) * invstd); yraw2 != null (downsample blocks,
 *   two BNs): bsums2[16][1][Cout] (the second half of each replica) +=
 *   sum dZ * (yraw2 - mean2) * invstd2.
 * grid: 0 = the production persistent grid (one block per CU); > 0 caps it
 * (rounded down to a multiple of Cout / 64) so blocks run several work items. */
int unet_conv3x3_fl(const void* x, int ldx, const void* wch, void* y, int ldy, const float* bias,
                    const void* addend, int ldadd, double* stats, const void* act, int ldact, const void* yraw,
                    int ldyraw, const float* mean, const float* invstd, const void* yraw2, int ldyraw2,
                    const float* mean2, const float* invstd2, double* bsums, double* bsums2, int N, int H,
                    int W, int C, int Cout, int mode, int grid, hipStream_t stream);
/* The weight-stationary ConvTranspose2d(k2, s2) (convt2x2_kernel: the narrow
 * decoder up-convs, advanced_models.py:96-99 upconv2 / upconv1, applied at
 * :305,315) as a single op.  N, H, W = the INPUT-resolution grid; (Ci, Co) in
 * {(64, 32), (64, 64), (128, 64)}; N*H*W % 32 == 0; 16-B aligned x / w, 8-B
 * aligned y, ldx % 8 == 0, ldy % 4 == 0.
 * mode 0 (forward): x = X [N,H,W] (ld ldx >= Ci), w = unet_pack_weight kind 2
 *   of the [Ci][Co][2][2] weight, y = Y [N,2H,2W] (ld ldy) = convT(X) + bias.
 * mode 1 (data gradient): x = dY [N,2H,2W] (ld ldx >= Co), w = kind 3 pack,
 *   y = dX [N,H,W] (ld ldy); bsums != null: the fused BN(+ReLU) backward as
 *   unet_conv3x3_fl mode 1 (act, yraw, mean, invstd over Ci channels,
 *   bsums[16][2][Ci]); bias_acc != null: bias_acc[16][Co] += the bias
 *   gradient sum of dY (fp64, caller zeroes).
 * grid: 0 = the production persistent grid; > 0 caps it. */
int unet_convt2x2(const void* x, int ldx, const void* w, void* y, int ldy, const float* bias, const void* act,
                  int ldact, const void* yraw, int ldyraw, const float* mean, const float* invstd, double* bsums,
                  double* bias_acc, int N, int H, int W, int Ci, int Co, int mode, int grid, hipStream_t stream);
/* ---- fp8 e4m3 forward conv (BASELINE.json configs[4]; no reference counterpart:
 * the reference's convs are fp32 torch.nn.Conv2d, advanced_models.py:72-100) ----
 * state: 16-B scale state {amax prev (float bits), amax this step, e8m0 code,
 * pad}, zeroed before first use; calibrate flags: 1 measures amax before
 * quantizing, 2 ("frozen", eval forwards) quantizes with the scale in use and
 * does not accumulate this call's amax into the state.
 * q = sat448(v * 2^e) with 2 * amax_prev * 2^e <= 448, code = 127 - e.
 * unet_f8_quantize: bf16 [npix][C] (stride ld) -> dense e4m3 [npix][C].
 * unet_f8_pack_weight: fp32 [Co][Ci][R][S] -> e4m3 [Co][R][S][Ci].
 * unet_f8_roll: prev <- this step's amax (if any), this step's amax <- 0.
 * unet_conv_fwd_f8: y = conv(dequant(xq), dequant(wq)) (+bias, +addend, BN
 * sums) as unet_conv_fwd mode 0, K = R*S*C in e4m3 on the block-scaled MFMA. */
int unet_f8_quantize(const void* x, int ld, int C, int64_t npix, void* q, void* state, int calibrate,
                     hipStream_t stream);
int unet_f8_pack_weight(const float* w, int Co, int Ci, int R, int S, void* dst, void* state, int calibrate,
                        hipStream_t stream);
int unet_f8_roll(void* states, int n, hipStream_t stream);
int unet_conv_fwd_f8(const void* xq, int ldx, const void* wq, const void* state_x, const void* state_w, void* y,
                     int ldy, const float* bias, const void* addend, int ldadd, double* stats, int N, int H,
                     int W, int C, int P, int Q, int Cout, int R, int S, int stride, int pad,
                     hipStream_t stream);
/* tile configuration of the implicit-GEMM conv kernels: 0 automatic (default),
 * >0 a fixed configuration from the tuning table (scripts/tune_conv.py) */
int unet_set_conv_config(int cfg);
/* kind: 0 conv fwd, 1 conv dgrad, 2 convT fwd, 3 convT dgrad, 4 stem,
 * 5 conv fwd chunk-major [Ci/32][3*3][Co][32], 6 conv dgrad chunk-major
 * [Co/32][3*3][Ci][32] (3x3 only; unet_conv3x3_fl) */
int unet_pack_weight(const float* src, void* dst, int kind, int Co, int Ci, int R, int S,
                     hipStream_t stream);
/* kind: 0 conv [Co][R][S][Ci] -> [Co][Ci][R][S], 1 convT, 2 stem */
int unet_unpack_grad(const float* acc, float* dst, int kind, int Co, int Ci, int R, int S,
                     hipStream_t stream);
/* BatchNorm2d (+identity residual)(+ReLU) forward from fp64 sums
 * stats[16][2][C] (16 atomic-spreading replicas of (sum, sumsq) over npix
 * pixels, summed by the kernel; training) or running stats (eval); save[2C] =
 * batch mean | invstd.  res_mode: 0 none, 1 out = act(bn(y) + res).
 * unet_conv_fwd's `stats` output has the same [16][2][Cout] layout. */
int unet_bn_forward(const void* y, int ldy, void* out, int ldo, const void* res, int ldr, int res_mode,
                    const double* stats, const float* gamma, const float* beta, float* run_mean,
                    float* run_var, float* save, int64_t npix, int C, int relu, int training,
                    hipStream_t stream);
/* backward of out = relu(bn(y)[+res]): dY, optional dres (= dZ), dgamma/dbeta;
 * sums[16][2][C] must be zero on entry. */
int unet_bn_backward(const void* dout, int ldd, const void* out, int ldo, const void* y, int ldy,
                     const float* save, const float* gamma, double* sums, void* dy, int lddy, void* dres,
                     float* dgamma, float* dbeta, int64_t npix, int C, hipStream_t stream);
int unet_maxpool_fwd(const void* x, int ldx, void* y, uint8_t* idx, int N, int H, int W, int C,
                     hipStream_t stream);
int unet_maxpool_bwd(const void* dy, const uint8_t* idx, const void* addend, int ldadd, void* dx,
                     int N, int H, int W, int C, hipStream_t stream);

/* ---- on-GPU data pipeline (CellSegmentationDataset / CellAugmenter,
 * dataset.py:30-66,147-151) over N decoded uint8 frames [N][H][W] ---- */
/* cv2.resize(..., INTER_AREA) downscale to [N][oh][ow] uint8 (dataset.py:51) */
int unet_resize_area_u8(const uint8_t* src, int N, int H, int W, uint8_t* dst, int oh, int ow, hipStream_t stream);
/* cv2.resize(..., INTER_NEAREST) then (mask > 0) -> float32 [N][oh][ow] (dataset.py:52,61) */
int unet_mask_prep(const uint8_t* src, int N, int H, int W, float* dst, int oh, int ow, hipStream_t stream);
/* normalize_microscopy_image (dataset.py:30-42: 2/98 percentile clip, CLAHE(2.0, 8x8),
 * min-max) -> float32 [N][H][W]; normalize = 0: x / 255 (dataset.py:56) */
int unet_normalize_microscopy(const uint8_t* src, int N, int H, int W, float* dst, int normalize,
                              hipStream_t stream);
/* A.RandomRotate90 + A.VerticalFlip (dataset.py:147,150): dst[n] = vflip?(rot90(src[n], k[n]));
 * k, vflip: device int32 [N]; frames square when any k is odd */
int unet_rot90_vflip_u8(const uint8_t* src, int N, int H, int W, const int* k, const int* vflip, uint8_t* dst,
                        hipStream_t stream);

/* A.Affine (dataset.py:150-151; albumentations 2.0 -> cv2.warpAffine, fixed-point
 * INTER_LINEAR for images / INTER_NEAREST for masks, BORDER_CONSTANT 0) with the
 * pipeline's following A.VerticalFlip folded in.  minv: device double [N][6],
 * the dst -> src map (cv::invertAffineTransform of the forward matrix);
 * active[n] == 0 copies frame n (still flipped when vflip[n]). */
int unet_warp_affine_u8(const uint8_t* src, int N, int H, int W, const double* minv, const int* active,
                        const int* vflip, int nearest, uint8_t* dst, hipStream_t stream);
/* A.AdvancedBlur (dataset.py:153) = cv2.filter2D(img, -1, kernel), BORDER_REFLECT_101.
 * kernels: device float32 [N][7][7] (top-left ksize[n]^2 used, odd ksize <= 7);
 * ksize[n] == 0 copies frame n. */
int unet_filter2d_u8(const uint8_t* src, int N, int H, int W, const float* kernels, const int* ksize, uint8_t* dst,
                     hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* UNET_HIP_H */

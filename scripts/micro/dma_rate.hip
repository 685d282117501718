// Per-CU LDS-DMA (buffer_load ... lds) throughput microbenchmark: what one CU
// moves from L2 into LDS per clock as a function of the piece shape (bytes of
// one cache line a 4/8-lane group reads), bytes in flight (stages, blocks per
// CU) and footprint.  Mimics the halo-streamed conv's staging: every stage is
// STAGE bytes of 1-KiB DMA instructions dealt round-robin over the block's
// waves, counted vmcnt + s_barrier per stage, no compute.
// build: hipcc -O3 --offload-arch=gfx950 -o dma_rate dma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ i32x4 rsrc(const void* base, unsigned bytes) {
  const unsigned long long p = (unsigned long long)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)p);
  r.y = __builtin_amdgcn_readfirstlane((int)((unsigned)(p >> 32) & 0xffffu));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ void glds(const i32x4& r, char* lds, unsigned voff) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(char, lds));
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(l) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// PIECE: contiguous bytes per group of PIECE/16 lanes; STRIDE: distance between
// consecutive pieces (512 = a 32-channel chunk of a 256-channel NHWC pixel)
template <int PIECE, int STRIDE, int NW, int STAGE, int NBUF>
__global__ void __launch_bounds__(NW * 64) dma_kernel(const char* src, unsigned foot, int iters,
                                                      unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NINS = STAGE / 1024, PER = NINS / NW, LPP = PIECE / 16, PPI = 64 / LPP;
  static_assert(NINS % NW == 0, "instructions per wave");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const i32x4 r = rsrc(src, foot);
  const unsigned pieces = foot / STRIDE;
  auto issue = [&](int s, int b) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int ins = wave + k * NW;
      const unsigned p = ((unsigned)blockIdx.x * 977u + (unsigned)s * (NINS * PPI) + ins * PPI + lane / LPP) % pieces;
      glds(r, smem + b * STAGE + ins * 1024, p * STRIDE + (lane % LPP) * 16);
    }
  };
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) issue(s, s);
  for (int s = 0; s < iters; ++s) {
    wait_vm<(NBUF - 2) * PER>();
    __builtin_amdgcn_s_barrier();
    issue(s + NBUF - 1, (s + NBUF - 1) % NBUF);
  }
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int PIECE, int STRIDE, int NW, int STAGE, int NBUF>
void run(const char* name, const char* src, unsigned foot, int bpc, unsigned long long* dcyc) {
  const int blocks = 256 * bpc, iters = 200;
  const size_t lds = (size_t)STAGE * NBUF;
  auto k = dma_kernel<PIECE, STRIDE, NW, STAGE, NBUF>;
  hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(NW * 64), lds, 0, src, foot, iters, dcyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  std::vector<unsigned long long> c(blocks);
  hipMemcpy(c.data(), dcyc, blocks * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : c) avg += (double)v;
  avg /= blocks;
  const double bytes_cu = (double)bpc * STAGE * iters;  // per CU
  printf("%-44s foot %7.1f MB  %6.1f us  %6.2f TB/s  per-CU %5.1f B/clk (block cycles %.0f, %.1f k/stage)\n", name,
         foot / 1e6, best * 1e3, bytes_cu * 256 / (best * 1e-3) / 1e12, bytes_cu / (avg), avg,
         avg / iters / 1e3);
}

int main() {
  const unsigned big = 512u << 20;
  char* src;
  unsigned long long* dcyc;
  hipMalloc(&src, big);
  hipMemset(src, 1, big);
  hipMalloc(&dcyc, 4096 * 8);
  for (unsigned foot : {2u << 20, 16u << 20, big}) {
    run<64, 512, 4, 40960, 2>("hs-like: 64B pieces s512, 4w x2blk, 40K x2", src, foot, 2, dcyc);
    run<128, 512, 4, 40960, 2>("128B pieces s512, 4w x2blk, 40K x2", src, foot, 2, dcyc);
    run<64, 64, 4, 40960, 2>("contiguous, 4w x2blk, 40K x2", src, foot, 2, dcyc);
    run<32, 512, 4, 40960, 2>("32B pieces s512, 4w x2blk, 40K x2", src, foot, 2, dcyc);
    run<64, 512, 8, 40960, 2>("64B s512, 8w x1blk, 40K x2", src, foot, 1, dcyc);
    run<64, 512, 8, 40960, 3>("64B s512, 8w x1blk, 40K x3", src, foot, 1, dcyc);
    run<128, 512, 8, 40960, 3>("128B s512, 8w x1blk, 40K x3", src, foot, 1, dcyc);
    run<64, 512, 8, 24576, 4>("64B s512, 8w x1blk, 24K x4", src, foot, 1, dcyc);
    run<64, 512, 4, 16384, 4>("64B s512, 4w x2blk, 16K x4", src, foot, 2, dcyc);
    run<128, 512, 4, 53248, 3>("wgrad-like 128B, 4w x1blk, 52K x3", src, foot, 1, dcyc);
    run<64, 512, 8, 57344, 2>("64B s512, 8w x1blk, 56K x2", src, foot, 1, dcyc);
  }
  return 0;
}

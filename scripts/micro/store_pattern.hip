// Microbenchmark: HBM write rate of two store patterns of a [npix][64 ch] bf16
// tensor (128 B per pixel): (A) the halo epilogue's: one wave instruction = 16
// pixels x 64 B (half lines, the other half by the next instruction);
// (B) one wave instruction = 8 pixels x 128 B (full lines).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void store_a(uint4* y, long long npix) {
  // wave w handles 16-pixel groups; lane: pixel = lane & 15, 16-B chunk = (lane >> 4) + 4 * half
  const long long wave = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long g = wave; g * 16 < npix; g += nw) {
    const long long px = g * 16 + (lane & 15);
    uint4 v = make_uint4(lane, px, 1, 2);
    y[px * 8 + (lane >> 4)] = v;      // chunks 0-3 (64 B)
    y[px * 8 + 4 + (lane >> 4)] = v;  // chunks 4-7 (64 B)
  }
}
__global__ void store_b(uint4* y, long long npix) {
  const long long wave = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long long nw = ((long long)gridDim.x * blockDim.x) >> 6;
  for (long long g = wave; g * 16 < npix; g += nw) {
    // same 16 pixels, two instructions, each 8 pixels x 8 chunks
    const long long px0 = g * 16 + (lane >> 3);
    uint4 v = make_uint4(lane, px0, 1, 2);
    y[px0 * 8 + (lane & 7)] = v;
    y[(px0 + 8) * 8 + (lane & 7)] = v;
  }
}
int main() {
  const long long npix = 16LL * 256 * 256;  // decoder1-sized: 16 x 256^2 pixels x 64 ch bf16 = 134 MB
  uint4* y;
  hipMalloc(&y, npix * 128);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(store_a, dim3(2048), dim3(256), 0, 0, y, npix);
      else hipLaunchKernelGGL(store_b, dim3(2048), dim3(256), 0, 0, y, npix);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s: %.1f us  %.2f TB/s\n", k == 0 ? "A half-line" : "B full-line", ms * 1e3, npix * 128 / (ms * 1e-3) / 1e12);
    }
  }
  hipFree(y);
  return 0;
}

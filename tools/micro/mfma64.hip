// f64 MFMA (v_mfma_f64_16x16x4_f64) vs VALU fp64 FMA throughput on one MI355X.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/mfma64.hip -o tools/micro/mfma64 && ./tools/micro/mfma64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a0) {
  d4 acc[4];
  for (int i = 0; i < 4; ++i) acc[i] = d4{0.0, 0.0, 0.0, 0.0};
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a0, long long* clk) {
  const long long c0 = clock64(), w0 = wall_clock64();
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = i;
  double a = a0 + threadIdx.x * 1e-9, b = a0 - threadIdx.x * 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = fma(a, acc[i], b);
  }
  double s = 0;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    clk[0] = clock64() - c0;
    clk[1] = wall_clock64() - w0;
  }
}

int main() {
  double* out;
  long long* clk;
  hipMalloc(&out, 256 * 4096 * sizeof(double));
  hipMalloc(&clk, 2 * sizeof(long long));
  int wall_khz = 0;
  hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 20000;
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    hipEventRecord(e0);
    k_mfma<<<blocks, 256>>>(out, iters, 1.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    double flops = 2.0 * 16 * 16 * 4 * 4 * (double)iters * (blocks * 4);
    printf("mfma f64 16x16x4: %.3f ms  %.1f TFLOP/s\n", ms, flops / ms / 1e9);
    hipEventRecord(e0);
    k_valu<<<blocks, 256>>>(out, iters, 1.0, clk);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    flops = 2.0 * 16 * (double)iters * blocks * 256;
    long long c[2];
    hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    printf("valu f64 fma:     %.3f ms  %.1f TFLOP/s  (block 0: %lld shader cycles in %lld wall ticks at %d kHz -> %.2f GHz)\n",
           ms, flops / ms / 1e9, c[0], c[1], wall_khz, wall_khz > 0 ? (double)c[0] / ((double)c[1] / (wall_khz * 1e3)) / 1e9 : 0.0);
  }
  return 0;
}

// HBM read/write bandwidth vs contiguous chunk size (frequency-minor layout question):
// every wave-instruction moves 64 lanes x 16 B = 1 KiB made of (1 KiB / C) chunks of C bytes,
// chunk i of the buffer visited in a scattered order (stride 32 KiB, wrapping), as the
// frequency-minor front storage is visited (one entry = Fc x 16 B; 16 frequencies = 256 B).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void rd(const double2* __restrict__ buf, int64_t nchunks, int cw, int64_t stride_chunks, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int per = 64 / cw;                 // chunks per wave-instruction
  double2 acc = make_double2(0, 0);
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = wave * per; base < nchunks; base += nwaves * per) {
    const int64_t c = base + lane / cw;
    const int64_t pos = (c * stride_chunks) % nchunks;        // scattered chunk order
    const double2 v = buf[pos * cw + lane % cw];
    acc.x += v.x; acc.y += v.y;
  }
  if (acc.x == 12345.678) out[0] = acc.y;
}

__global__ void wr(double2* __restrict__ buf, int64_t nchunks, int cw, int64_t stride_chunks) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int per = 64 / cw;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t base = wave * per; base < nchunks; base += nwaves * per) {
    const int64_t c = base + lane / cw;
    const int64_t pos = (c * stride_chunks) % nchunks;
    buf[pos * cw + lane % cw] = make_double2((double)c, 1.0);
  }
}

int main() {
  const int64_t bytes = 8ll << 30;
  double2* buf;
  double* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
  hipMemset(buf, 0, bytes);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int cws[] = {4, 8, 16, 32, 64};   // chunk = cw x 16 B: 64 B .. 1 KiB
  for (int cw : cws) {
    const int64_t nchunks = bytes / (cw * 16);
    for (int64_t stride_b : {(int64_t)0, (int64_t)32768, (int64_t)1 << 20}) {
      int64_t sc = stride_b / (cw * 16);
      if (stride_b == 0) sc = 1;
      else sc += 1;   // odd stride in chunks: a permutation of the chunks (coprime with 2^k)
      float msr = 0, msw = 0;
      for (int it = 0; it < 3; ++it) {
        hipEventRecord(a);
        rd<<<8192, 256>>>(buf, nchunks, cw, sc, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&msr, a, b);
        hipEventRecord(a);
        wr<<<8192, 256>>>(buf, nchunks, cw, sc);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&msw, a, b);
      }
      printf("chunk %5d B  stride %8lld B : read %7.0f GB/s  write %7.0f GB/s\n", cw * 16, (long long)stride_b,
             bytes / (msr * 1e-3) / 1e9, bytes / (msw * 1e-3) / 1e9);
    }
  }
  return 0;
}

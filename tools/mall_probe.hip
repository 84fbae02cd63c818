// Streaming-read bandwidth by footprint (GPU box): is a 64-256 MB working set re-read from the
// Infinity Cache faster than from HBM? Each pass reads the whole buffer once (16 B per lane,
// grid-stride, 2048 workgroups x 256 threads) and sums it (so the loads are not dead); the
// buffer is read twice back to back and the second pass is timed, for footprints 32 MB .. 2 GB.
//   hipcc -O3 --offload-arch=gfx950 tools/mall_probe.hip -o /tmp/mall_probe && /tmp/mall_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void read_kernel(const uint4* __restrict__ p, long n, float* out) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    s += __uint_as_float(v.x) + __uint_as_float(v.y) + __uint_as_float(v.z) + __uint_as_float(v.w);
  }
  if (s == 12345.f) out[0] = s;   // never true for the zero-filled buffer
}

__global__ __launch_bounds__(256) void copy_kernel(const uint4* __restrict__ p, uint4* __restrict__ q, long n) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    q[i] = p[i];
}

int main() {
  const long maxb = 2L << 30;
  uint4 *buf, *dst;
  float* out;
  if (hipMalloc(&buf, maxb) != hipSuccess || hipMalloc(&dst, maxb / 2) != hipSuccess ||
      hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, maxb);
  (void)hipMemset(dst, 0, maxb / 2);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const long sizes_mb[] = {32, 64, 128, 192, 256, 384, 512, 1024, 2048};
  printf("footprint_MB  read_TBps(2nd pass)  read+write_half(TB/s of bytes moved)\n");
  for (long mb : sizes_mb) {
    const long bytes = mb << 20;
    const long n = bytes / 16;
    float best = 1e9f, bestc = 1e9f;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, 0, buf, n, out);   // warm
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, 0, buf, n, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
      // read the first 2/3 of the footprint, write the last 1/3 (a BN-backward apply's shape)
      const long nr = n * 2 / 3, nw = n - nr;
      hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, 0, buf, nr, out);   // warm reads
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(copy_kernel, dim3(2048), dim3(256), 0, 0, buf, dst, nw);
      hipLaunchKernelGGL(read_kernel, dim3(2048), dim3(256), 0, 0, buf + nw, nr - nw, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < bestc) bestc = ms;
    }
    printf("%6ld  %8.2f  %8.2f\n", mb, bytes / (best * 1e-3) / 1e12, (bytes) / (bestc * 1e-3) / 1e12);
  }
  return 0;
}

// LDS atomic throughput on one MI355X: no-return add vs returning compare-and-swap vs plain read,
// 64 KB table per 512-thread workgroup, 2 workgroups per CU (k_sp_main's shape), random slots.
// Prints lane-operations per CU-cycle for each.  Build: hipcc -O3 --offload-arch=gfx950 -o lds_atomics lds_atomics.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kThreads = 512, kSlots = 8192, kIters = 4096;

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_lds(unsigned *out, unsigned seed) {
  __shared__ unsigned keys[kSlots], cnts[kSlots];
  for (int i = threadIdx.x; i < kSlots; i += kThreads) keys[i] = cnts[i] = 0;
  __syncthreads();
  unsigned x = seed ^ (blockIdx.x * kThreads + threadIdx.x) * 0x9E3779B1u, acc = 0;
  for (int it = 0; it < kIters; it++) {
    unsigned h[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      h[k] = x & (kSlots - 1);
    }
    if (MODE == 0) {  // no-return add
#pragma unroll
      for (int k = 0; k < 4; k++) atomicAdd(&cnts[h[k]], 1u);
    } else if (MODE == 1) {  // returning CAS, 4 in flight, then a no-return add
      unsigned c[4];
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = atomicCAS(&keys[h[k]], 0u, h[k] + 1u);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        acc += c[k];
        atomicAdd(&cnts[h[k]], 1u);
      }
    } else {  // plain reads, 4 in flight
      unsigned c[4];
#pragma unroll
      for (int k = 0; k < 4; k++) c[k] = __hip_atomic_load(&keys[h[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
      for (int k = 0; k < 4; k++) acc += c[k];
    }
  }
  __syncthreads();
  if (acc == 0xFFFFFFFFu) out[0] = acc + cnts[threadIdx.x];
}

int main() {
  unsigned *out;
  hipMalloc(&out, 4);
  int dev = 0, n_cu = 0, clk = 0;
  hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  const int grid = 2 * n_cu;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char *names[3] = {"ds_add (no return)", "ds_cmpst_rtn + ds_add", "ds_read"};
  for (int mode = 0; mode < 3; mode++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(a);
      if (mode == 0) k_lds<0><<<grid, kThreads>>>(out, 7u + rep);
      if (mode == 1) k_lds<1><<<grid, kThreads>>>(out, 7u + rep);
      if (mode == 2) k_lds<2><<<grid, kThreads>>>(out, 7u + rep);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 1) {
        const double ops = double(grid) * kThreads * kIters * 4;  // lane-operations (CAS+add counted once)
        const double cycles = double(ms) * 1e-3 * double(clk) * 1e3;
        printf("%-24s %8.3f ms  %.2f lane-ops per CU-cycle (%d CUs, %d MHz)\n", names[mode], ms, ops / cycles / n_cu, n_cu,
               clk / 1000);
      }
    }
  }
  return hipGetLastError() != hipSuccess;
}

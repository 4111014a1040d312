// Random-line read ceiling on MI355X: every lane reads 16 B from a random
// 64 B line of a table (uniform, or Zipf-like through a hot subset), N
// independent reads in flight per lane, optionally beside a streaming read of
// a large buffer (the record stream's share of the memory system).
//   randread <table_MB> <hot_frac_permille> <stream_MB>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

template <int N>
__global__ __launch_bounds__(256) void rand_kernel(const uint4* __restrict__ t, uint64_t lines, uint64_t hot_lines,
                                                   uint32_t hot_pm, const uint4* __restrict__ s, uint64_t s_vec,
                                                   uint32_t iters, uint4* out) {
  uint32_t seed = hash32(blockIdx.x * 256 + threadIdx.x + 1);
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint64_t sp = (uint64_t(blockIdx.x) * 256 + threadIdx.x);
  const uint64_t sstride = uint64_t(gridDim.x) * 256;
  for (uint32_t it = 0; it < iters; it++) {
    uint4 v[N];
#pragma unroll
    for (int k = 0; k < N; k++) {
      seed = hash32(seed + k);
      const bool hot = (seed % 1000) < hot_pm;
      const uint32_t r = hash32(seed ^ 0x9e3779b9u);
      const uint64_t line = hot ? (r % hot_lines) : (uint64_t(r) * 2654435761ull + seed) % lines;
      v[k] = t[line * 4 + (seed & 3)];
    }
    uint4 sv = make_uint4(0, 0, 0, 0);
    if (s_vec) {
      sv = s[sp % s_vec];
      sp += sstride;
    }
#pragma unroll
    for (int k = 0; k < N; k++) {
      acc.x ^= v[k].x; acc.y += v[k].y; acc.z ^= v[k].z; acc.w += v[k].w;
    }
    acc.x ^= sv.x; acc.y += sv.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const double table_mb = argc > 1 ? atof(argv[1]) : 80;
  const uint32_t hot_pm = argc > 2 ? atoi(argv[2]) : 0;
  const double stream_mb = argc > 3 ? atof(argv[3]) : 0;
  const uint64_t lines = uint64_t(table_mb * 1e6 / 64);
  const uint64_t hot_lines = 16384;  // 1 MiB hot set
  uint4 *t, *s = nullptr, *out;
  CHECK(hipMalloc(&t, lines * 64));
  CHECK(hipMemset(t, 1, lines * 64));
  const uint64_t s_vec = uint64_t(stream_mb * 1e6 / 16);
  if (s_vec) { CHECK(hipMalloc(&s, s_vec * 16)); CHECK(hipMemset(s, 2, s_vec * 16)); }
  CHECK(hipMalloc(&out, 16));
  const int grid = 256 * 8;
  const uint32_t iters = 64;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int n : {1, 2, 4, 8}) {
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipEventRecord(a));
      switch (n) {
        case 1: hipLaunchKernelGGL(rand_kernel<1>, dim3(grid), dim3(256), 0, 0, t, lines, hot_lines, hot_pm, s, s_vec, iters, out); break;
        case 2: hipLaunchKernelGGL(rand_kernel<2>, dim3(grid), dim3(256), 0, 0, t, lines, hot_lines, hot_pm, s, s_vec, iters, out); break;
        case 4: hipLaunchKernelGGL(rand_kernel<4>, dim3(grid), dim3(256), 0, 0, t, lines, hot_lines, hot_pm, s, s_vec, iters, out); break;
        case 8: hipLaunchKernelGGL(rand_kernel<8>, dim3(grid), dim3(256), 0, 0, t, lines, hot_lines, hot_pm, s, s_vec, iters, out); break;
      }
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      const double reads = double(grid) * 256 * iters * n;
      if (rep == 2)
        printf("{\"table_MB\": %.0f, \"hot_permille\": %u, \"stream_MB\": %.0f, \"inflight_per_lane\": %d, \"ms\": %.3f, "
               "\"Greads_s\": %.2f, \"stream_GBs\": %.0f}\n",
               table_mb, hot_pm, stream_mb, n, ms, reads / ms / 1e6, s_vec ? double(grid) * 256 * iters * 16 / ms / 1e6 : 0.0);
    }
  }
  return 0;
}

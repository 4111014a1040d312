// Vector-memory shape costs on gfx950 (not the product path): what a wave
// instruction of 16 B per lane costs the CU when its lanes' addresses are
// contiguous, grouped in 64 B / 32 B runs, or scattered -- the store shapes a
// route pass can produce -- and the 40 B-stride record loads against
// contiguous ones.
//   vmem <footprint_MB> <iters>
// One 1024-thread workgroup per CU (grid 256), every wave issuing `iters`
// wave-instructions; prints GB/s of useful bytes and wave-instructions per
// CU per microsecond for each shape.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

// store shapes: 0 contiguous 1 KiB per wave, 1 runs of 4 lanes (64 B),
// 2 runs of 2 lanes (32 B), 3 every lane its own 16 B
template <int SHAPE>
__global__ __launch_bounds__(1024) void store_kernel(uint4* dst, uint64_t n16, int iters) {
  const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * 1024 + threadIdx.x) >> 6;
  const uint4 v = make_uint4(lane, wave, 1, 2);
  const uint64_t mask = n16 - 1;  // n16: power of two
  for (int it = 0; it < iters; it++) {
    const uint32_t h = hash32(wave * 0x9E3779B1u + it * 0x85ebca6bu + 1);
    uint64_t i;
    if (SHAPE == 0) i = (uint64_t(h) * 64 + lane) & mask;
    else if (SHAPE == 1) i = (uint64_t(hash32(h ^ (lane >> 2))) * 4 + (lane & 3)) & mask;
    else if (SHAPE == 2) i = (uint64_t(hash32(h ^ (lane >> 1))) * 2 + (lane & 1)) & mask;
    else i = uint64_t(hash32(h ^ lane)) & mask;
    dst[i] = v;
  }
}

// load shapes: 0 a 2560 B window of 40 B records, three loads per lane at
// 40 B stride (16 + 16 + 8 B, the route pass's); 1 the same window as
// contiguous 16 B per lane (2.5 loads)
template <int SHAPE>
__global__ __launch_bounds__(1024) void load_kernel(const uint8_t* src, uint64_t nbytes, int iters, uint32_t* out) {
  const uint32_t lane = threadIdx.x & 63, wave = (blockIdx.x * 1024 + threadIdx.x) >> 6;
  const uint64_t nwin = nbytes / 2560;
  uint32_t acc = 0;
  for (int it = 0; it < iters; it++) {
    const uint64_t w = (uint64_t(wave) * 7919 + uint64_t(it) * 104729) % nwin;
    const uint8_t* base = src + w * 2560;
    if (SHAPE == 0) {
      const uint32_t pos = lane * 40, odd = (pos >> 3) & 1;
      const uint4 x = *reinterpret_cast<const uint4*>(base + pos + (odd ? 8 : 0));
      const uint4 y = *reinterpret_cast<const uint4*>(base + pos + (odd ? 24 : 16));
      const uint2 z = *reinterpret_cast<const uint2*>(base + pos + (odd ? 0 : 32));
      acc ^= x.x ^ x.w ^ y.y ^ y.z ^ z.x ^ z.y;
    } else {
      const uint4 x = reinterpret_cast<const uint4*>(base)[lane];
      const uint4 y = reinterpret_cast<const uint4*>(base + 1024)[lane];
      const uint4 z = lane < 32 ? reinterpret_cast<const uint4*>(base + 2048)[lane] : make_uint4(0, 0, 0, 0);
      acc ^= x.x ^ x.w ^ y.y ^ y.z ^ z.x ^ z.y;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t mb = argc > 1 ? strtoull(argv[1], 0, 10) : 2048;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  uint64_t bytes = 1;
  while (bytes < mb * (1ull << 20)) bytes <<= 1;
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 4));
  CHECK(hipMemset(buf, 1, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int grid = 256;
  const double waves = grid * 16.0;
  auto run = [&](const char* name, auto launch, double useful_per_inst, double insts_per_iter) {
    launch();  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 5; r++) launch();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    ms /= 5;
    const double inst = waves * iters * insts_per_iter;
    printf("{\"footprint_MB\": %llu, \"shape\": \"%s\", \"ms\": %.4f, \"useful_GBps\": %.0f, \"wave_insts_per_CU_per_us\": %.2f}\n",
           (unsigned long long)(bytes >> 20), name, ms, waves * iters * useful_per_inst / (ms * 1e6),
           inst / 256.0 / (ms * 1e3));
  };
  const uint64_t n16 = bytes / 16;
  run("store_contig_1KiB", [&] { hipLaunchKernelGGL(store_kernel<0>, dim3(grid), dim3(1024), 0, 0, (uint4*)buf, n16, iters); }, 1024, 1);
  run("store_runs_64B", [&] { hipLaunchKernelGGL(store_kernel<1>, dim3(grid), dim3(1024), 0, 0, (uint4*)buf, n16, iters); }, 1024, 1);
  run("store_runs_32B", [&] { hipLaunchKernelGGL(store_kernel<2>, dim3(grid), dim3(1024), 0, 0, (uint4*)buf, n16, iters); }, 1024, 1);
  run("store_scatter_16B", [&] { hipLaunchKernelGGL(store_kernel<3>, dim3(grid), dim3(1024), 0, 0, (uint4*)buf, n16, iters); }, 1024, 1);
  run("load_stride40_3x", [&] { hipLaunchKernelGGL(load_kernel<0>, dim3(grid), dim3(1024), 0, 0, buf, bytes, iters, out); }, 2560, 3);
  run("load_contig_2.5x", [&] { hipLaunchKernelGGL(load_kernel<1>, dim3(grid), dim3(1024), 0, 0, buf, bytes, iters, out); }, 2560, 3);
  return 0;
}

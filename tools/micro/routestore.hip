// The store side of a route pass at the configs[3] shard's shape (not the
// product path): 125M 40 B records streamed by 12-wave workgroups, each
// record sent to one of P partitions (skewed like the c4 workload: 10 % to
// one partition, 40 % to 64, the rest uniform), and written as a 16 B record
// into its partition's 64-record chunk of the workgroup's pool.  Variants
// isolate what the claim, the scattered stores and an LDS line stage cost:
//   0 stream only (records loaded and reduced, no claim, no store)
//   1 + claim (LDS atomic with return on the partition's counter)
//   2 + claim + scattered 16 B store to the chunk slot
//   3 + claim + LDS line stage (4 records per partition line, 64 B) and a
//       wave-cooperative flush of completed lines: 4 lanes per line, one
//       store instruction per 16 lines (a cost model: lines overrun by
//       hot partitions are not guarded, so the bytes are not exact)
//   4 + claim + store to a fixed coalesced slot (the lane's own)
//   routestore <records_M> <parts>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                    \
  do {                                                              \
    hipError_t e = (x);                                             \
    if (e != hipSuccess) {                                          \
      printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      exit(1);                                                      \
    }                                                               \
  } while (0)

constexpr int kWG = 768, kWaves = kWG / 64;
constexpr uint32_t kMaxP = 2048;
constexpr uint32_t kPoolChunks = 16384;  // per workgroup: 16 MB of 1 KiB chunks

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ void gen_kernel(uint64_t* rec, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const uint32_t h = hash32((uint32_t)i * 2654435761u + 17);
    uint64_t* q = rec + 5 * i;
    q[0] = (40ull << 48) | 9;
    q[1] = i;
    q[2] = (uint64_t(hash32(h)) << 20) | h;
    q[3] = 1 + (h >> 22);
    q[4] = 0x42;
  }
}

struct P {
  const uint8_t* rec;
  uint64_t n;
  uint32_t parts;
  uint4* out;
  unsigned long long* sink;
};

__device__ __forceinline__ uint32_t pick(uint32_t h, uint32_t parts) {
  const uint32_t r = h & 1023;
  if (r < 102) return 0;
  if (r < 512) return 1 + (h >> 10) % 64;
  return (h >> 10) % parts;
}

template <int V>
__global__ __launch_bounds__(kWG, 1) void route_kernel(P p) {
  __shared__ uint32_t s_cnt[kMaxP];
  __shared__ uint4 s_line[V == 3 ? kMaxP * 4 : 1];
  __shared__ uint32_t s_fill[V == 3 ? kMaxP : 1];
  __shared__ uint2 s_tab[kWaves][64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (uint32_t i = tid; i < kMaxP; i += kWG) {
    s_cnt[i] = 0;
    if (V == 3) s_fill[i] = 0;
  }
  __syncthreads();
  const uint64_t nwin = p.n / 64;
  const uint64_t per = (nwin + gridDim.x - 1) / gridDim.x;
  const uint64_t w0 = blockIdx.x * per, w1 = min(nwin, w0 + per);
  uint4* pool = p.out + uint64_t(blockIdx.x) * kPoolChunks * 64;
  unsigned long long acc = 0;
  uint64_t fixed = 0;
  for (uint64_t w = w0 + wave; w < w1; w += kWaves) {
    const uint8_t* base = p.rec + w * 2560;
    const uint32_t pos = lane * 40, odd = (pos >> 3) & 1;
    const uint4 x = *reinterpret_cast<const uint4*>(base + pos + (odd ? 8 : 0));
    const uint4 y = *reinterpret_cast<const uint4*>(base + pos + (odd ? 24 : 16));
    const uint2 z = *reinterpret_cast<const uint2*>(base + pos + (odd ? 0 : 32));
    const uint32_t h = hash32(x.x ^ y.y ^ z.x ^ (uint32_t)w);
    const uint4 r = make_uint4(x.y ^ h, y.x, y.w, z.y);
    if (V == 0) {
      acc += r.x ^ r.y ^ r.z ^ r.w;
      continue;
    }
    const uint32_t q = pick(h, p.parts);
    if (V == 4) {
      pool[(fixed * kWG + tid) % (uint64_t(kPoolChunks) * 64)] = r;
      fixed++;
      continue;
    }
    const uint32_t n = atomicAdd(&s_cnt[q], 1u);
    const uint64_t dst = uint64_t((q * 64 + (n >> 6)) % kPoolChunks) * 64 + (n & 63);
    if (V == 1) {
      acc += n ^ r.x;
      continue;
    }
    if (V == 2) {
      pool[dst] = r;
      continue;
    }
    // V == 3: the line stage
    s_line[q * 4 + (n & 3)] = r;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    const uint32_t f = atomicAdd(&s_fill[q], 1u);
    const bool done = (f & 3) == 3;  // this write completed a line
    const uint64_t m = __ballot(done);
    if (done) {
      const uint32_t k = __popcll(m & ((1ull << lane) - 1));
      s_tab[wave][k] = make_uint2(q, (uint32_t)(dst & ~3ull));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    const uint32_t nd = __popcll(m);
    for (uint32_t j0 = 0; j0 < nd; j0 += 16) {
      const uint32_t j = j0 + (lane >> 2);
      if (j < nd) {
        const uint2 t = s_tab[wave][j];
        const uint4 v = s_line[t.x * 4 + (lane & 3)];
        pool[uint64_t(t.y) + (lane & 3)] = v;
      }
    }
  }
  if (acc == 0x1234567ull) p.sink[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t n = (argc > 1 ? strtoull(argv[1], 0, 10) : 125) * 1000000ull / 64 * 64;
  const uint32_t parts = argc > 2 ? atoi(argv[2]) : 1250;
  uint8_t* rec;
  uint4* out;
  unsigned long long* sink;
  const int grid = 256;
  CHECK(hipMalloc(&rec, n * 40));
  CHECK(hipMalloc(&out, uint64_t(grid) * kPoolChunks * 64 * 16));
  CHECK(hipMalloc(&sink, 8));
  hipLaunchKernelGGL(gen_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t*)rec, n);
  CHECK(hipDeviceSynchronize());
  P p{rec, n, parts, out, sink};
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  auto run = [&](int v, auto k) {
    hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), 0, 0, p);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int r = 0; r < 10; r++) hipLaunchKernelGGL(k, dim3(grid), dim3(kWG), 0, 0, p);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    printf("{\"variant\": %d, \"records\": %llu, \"parts\": %u, \"ms\": %.4f, \"Gsamples_s\": %.2f}\n", v,
           (unsigned long long)n, parts, ms / 10, n / (ms / 10 * 1e6));
  };
  run(0, route_kernel<0>);
  run(1, route_kernel<1>);
  run(2, route_kernel<2>);
  run(3, route_kernel<3>);
  run(4, route_kernel<4>);
  return 0;
}

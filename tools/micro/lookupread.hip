// Lookup-shaped random reads on MI355X (the 1M-interval attribution lookup):
// per lane and iteration, an 8 B "directory" read from a D-MB table and a
// dependent read of a "node" in an N-MB table, in several shapes.  1024-thread
// workgroups, one per CU, like attribute_kernel; optional Zipf-like hot set.
//   lookupread <dir_MB> <node_MB> <hot_permille>
// modes: 0 node 1x16B (no dir)    1 node 3x16B same 64 B line (no dir)
//        2 node 2x16B (no dir)    3 dir 8B only
//        4 dir -> node 3x16B      5 dir -> node 2x16B      6 dir -> node 1x16B
//        7 dir(prefetched one iteration ahead) -> node 3x16B
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__device__ __forceinline__ uint64_t pick(uint32_t& seed, uint64_t n, uint32_t hot_pm) {
  seed = hash32(seed + 0x632be5abu);
  const bool hot = (seed % 1000) < hot_pm;
  const uint32_t r = hash32(seed ^ 0x9e3779b9u);
  return hot ? (r % min(n, (uint64_t)8192)) * 97 % n : (uint64_t(r) * 2654435761ull + seed) % n;
}

template <int MODE>
__global__ __launch_bounds__(1024, 1) void look_kernel(const uint2* __restrict__ dir, uint64_t ndir,
                                                       const uint4* __restrict__ node, uint64_t nnode,
                                                       uint32_t hot_pm, uint32_t iters, uint4* out) {
  uint32_t seed = hash32(blockIdx.x * 1024 + threadIdx.x + 1);
  uint4 acc = make_uint4(0, 0, 0, 0);
  uint2 pre = make_uint2(0, 0);
  if (MODE == 7) pre = dir[pick(seed, ndir, hot_pm)];
  for (uint32_t it = 0; it < iters; it++) {
    uint64_t k;
    if (MODE >= 3 && MODE <= 6) {
      const uint2 d = dir[pick(seed, ndir, hot_pm)];
      k = (uint64_t(d.x) * 0x9E3779B1u + d.y) % nnode;  // dependent on the loaded value
      k = (k + pick(seed, nnode, hot_pm)) % nnode;
    } else if (MODE == 7) {
      k = (uint64_t(pre.x) * 0x9E3779B1u + pre.y) % nnode;
      k = (k + pick(seed, nnode, hot_pm)) % nnode;
      pre = dir[pick(seed, ndir, hot_pm)];  // next iteration's
    } else {
      k = pick(seed, nnode, hot_pm);
    }
    if (MODE == 3) {
      acc.x += (uint32_t)k;
      continue;
    }
    const uint4* q = node + k * 4;
    uint4 a = q[0], b = make_uint4(0, 0, 0, 0), c = make_uint4(0, 0, 0, 0);
    if (MODE == 1 || MODE == 2 || MODE == 4 || MODE == 5 || MODE == 7) b = q[1];
    if (MODE == 1 || MODE == 4 || MODE == 7) c = q[2];
    acc.x ^= a.x ^ b.y ^ c.z; acc.y += a.y + b.z + c.w; acc.z ^= a.z; acc.w += a.w ^ b.x ^ c.x;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

typedef void (*K)(const uint2*, uint64_t, const uint4*, uint64_t, uint32_t, uint32_t, uint4*);

int main(int argc, char** argv) {
  const double dir_mb = argc > 1 ? atof(argv[1]) : 16;
  const double node_mb = argc > 2 ? atof(argv[2]) : 64;
  const uint32_t hot_pm = argc > 3 ? atoi(argv[3]) : 0;
  const uint64_t ndir = uint64_t(dir_mb * 1e6 / 8), nnode = uint64_t(node_mb * 1e6 / 64);
  uint2* dir; uint4* node; uint4* out;
  CHECK(hipMalloc(&dir, ndir * 8));
  CHECK(hipMemset(dir, 1, ndir * 8));
  CHECK(hipMalloc(&node, nnode * 64));
  CHECK(hipMemset(node, 2, nnode * 64));
  CHECK(hipMalloc(&out, 16));
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t iters = 256;
  const K ks[8] = {look_kernel<0>, look_kernel<1>, look_kernel<2>, look_kernel<3>,
                   look_kernel<4>, look_kernel<5>, look_kernel<6>, look_kernel<7>};
  const char* names[8] = {"node1x16", "node3x16", "node2x16", "dir8", "dir>node3x16", "dir>node2x16",
                          "dir>node1x16", "dirpre>node3x16"};
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
  for (int m = 0; m < 8; m++) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CHECK(hipEventRecord(a));
      hipLaunchKernelGGL(ks[m], dim3(ncu), dim3(1024), 98304, 0, dir, ndir, node, nnode, hot_pm, iters, out);
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (rep && ms < best) best = ms;
    }
    const double lookups = double(ncu) * 1024 * iters;
    printf("{\"mode\": \"%s\", \"dir_MB\": %.0f, \"node_MB\": %.0f, \"hot_permille\": %u, \"ms\": %.3f, "
           "\"Glookups_s\": %.2f}\n", names[m], dir_mb, node_mb, hot_pm, best, lookups / best / 1e6);
  }
  return 0;
}

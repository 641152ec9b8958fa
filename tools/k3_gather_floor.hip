// k3_gather_floor — timing probe for VERDICT r5 #3 (the priced K3 mode-1 restructure).
//
// The restructure ("K3 mode 1") would have K1 write each tile's
// claim words bucket-sorted beside the record-order word, and K3 become
//   (a) a RECORD-ORDER claim -> id gather: out_id[r] = omap[claim[r]], plus
//   (b) a bucket pass over per-tile segments (pkts / bytes per claim).
// Part (a) alone is measured here, at the two config-4 table sizes, against the
// product's whole K3 mode 1 (k_count_chunk2 + k_count_bucket: 564 us per 124.9M
// records at the N=8 share, 847 us at 1M flows; profiles/r05_summary.md). If (a)
// alone is not well below those, the restructure cannot reach VERDICT r5's
// <= 0.45 / 0.70 ms targets.
//
// Build: hipcc -O3 --offload-arch=gfx950 -o ab/k3_gather_floor tools/k3_gather_floor.hip
// Run:   ab/k3_gather_floor [records=125000000]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// claims: splitmix64 of the record index mod F (uniform flows, as the synthetic
// config-4 trace), generated on the device
__global__ void k_fill(uint32_t* claim, uint64_t n, uint32_t F) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t z = i + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    claim[i] = (uint32_t)(z % F);
  }
}

__global__ void k_map(uint32_t* omap, uint32_t F) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < F; i += gridDim.x * blockDim.x)
    omap[i] = F - 1 - i;
}

// (a): 8 records per lane in flight, non-temporal word loads and id stores (as K3)
template <bool GATHER>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ claim,
                                                const uint32_t* __restrict__ omap,
                                                uint32_t* __restrict__ out, uint64_t n) {
  constexpr int U = 8;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * U;
  for (uint64_t b = (blockIdx.x * (uint64_t)blockDim.x) * U + threadIdx.x; b < n; b += stride) {
    uint32_t w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * blockDim.x;
      w[u] = i < n ? __builtin_nontemporal_load(&claim[i]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = GATHER ? omap[w[u]] : w[u] ^ 0x5A5A5A5Au;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * blockDim.x;
      if (i < n) __builtin_nontemporal_store(w[u], &out[i]);
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 124'900'000ull;
  uint32_t *claim, *omap, *out;
  CK(hipMalloc(&claim, n * 4));
  CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&omap, (1u << 20) * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) == hipSuccess) ncu = prop.multiProcessorCount;
  const uint32_t grid = (uint32_t)ncu * 16;
  std::printf("{\"records\": %llu, \"grid\": %u, \"results\": [", (unsigned long long)n, grid);
  const uint32_t flows[] = {10'000, 125'000, 1'000'000};
  bool first = true;
  for (uint32_t F : flows) {
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, claim, n, F);
    hipLaunchKernelGGL(k_map, dim3(1024), dim3(256), 0, 0, omap, F);
    CK(hipDeviceSynchronize());
    for (int g = 0; g < 2; ++g) {
      float best = 1e30f, sum = 0;
      const int reps = 20;
      for (int r = 0; r < reps + 3; ++r) {
        CK(hipEventRecord(e0, 0));
        if (g) hipLaunchKernelGGL(k_gather<true>, dim3(grid), dim3(256), 0, 0, claim, omap, out, n);
        else hipLaunchKernelGGL(k_gather<false>, dim3(grid), dim3(256), 0, 0, claim, omap, out, n);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
          sum += ms;
          best = ms < best ? ms : best;
        }
      }
      // check a few gathered ids
      if (g) {
        std::vector<uint32_t> hc(64), ho(64);
        CK(hipMemcpy(hc.data(), claim + n / 2, 256, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ho.data(), out + n / 2, 256, hipMemcpyDeviceToHost));
        for (int i = 0; i < 64; ++i)
          if (ho[i] != F - 1 - hc[i]) {
            std::fprintf(stderr, "wrong id at %d\n", i);
            return 1;
          }
      }
      std::printf("%s{\"flows\": %u, \"kernel\": \"%s\", \"mean_us\": %.1f, \"best_us\": %.1f, "
                  "\"GBs_8B_per_record\": %.0f}",
                  first ? "" : ", ", F, g ? "record-order gather omap[claim]" : "stream copy (no gather)",
                  1e3f * sum / reps, 1e3f * best, n * 8.0 / (sum / reps * 1e-3) / 1e9);
      first = false;
    }
  }
  std::printf("]}\n");
  return 0;
}

// tcbee_synth.hip — synthetic traces on the device (tcbee_gen.h): frame headers,
// the flow-hash shard of a global trace (config 4: the NIC-RSS view of N GPUs)
// and RSS bucket loads. Bench and test infrastructure: frames the path parses.
#include "tcbee_table.h"

namespace tcbee {

// ---------------------------------------------------------------------------
// synthetic trace headers (payload stays as the caller zeroed it)
// ---------------------------------------------------------------------------
__global__ void k_gen(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                      uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed,
                      const uint64_t* gidx, const uint64_t* zcdf) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint8_t h[kGenHdrMax];
    gen_header(h, gidx ? gidx[i] : first_index + i, len[i], kind, n_flows, seed, zcdf);
    const uint32_t hl = gen_header_len(kind);
    const uint32_t m = len[i] < hl ? len[i] : hl;
    uint8_t* dst = arena + off[i];
    for (uint32_t b = 0; b < m; ++b) dst[b] = h[b];
  }
}

// ---------------------------------------------------------------------------
// flow-hash shard of the synthetic trace (config 4: the NIC-RSS view of 8 GPUs)
// ---------------------------------------------------------------------------
// caplen of global frame i (== tcbee_amd.trace.synth_index)
__device__ __forceinline__ uint32_t gen_caplen(uint64_t i, int imix, uint64_t seed) {
  if (!imix) return 64u;
  const uint64_t r = splitmix64((seed ^ 0x1A1Eull) + i) % 12u;
  return r < 7 ? 64u : (r < 11 ? 576u : 1500u);
}
// the flow hash of global frame i (the IpTuple K1 builds for this IPv4/TCP frame,
// xdp.rs:116-127) folded to 32 bits
__device__ __forceinline__ uint32_t gen_fold(const ShardArgs& a, uint64_t i) {
  const GenFields g = gen_fields(i, a.kind, a.n_flows, a.seed);
  const uint64_t k1 = (uint64_t)bswap32(g.saddr) << 32, k3 = (uint64_t)bswap32(g.daddr) << 32;
  const uint64_t k4 = (uint64_t)g.sport | ((uint64_t)g.dport << 16) | ((uint64_t)kTcpProtocol << 32);
  return fold32(flow_hash64(0, k1, 0, k3, k4));
}
// owner GPU of global frame i: the folded hash mod world, or through the RSS
// indirection table (a NIC's receive-side scaling: hash bucket -> queue)
__device__ __forceinline__ uint32_t gen_owner(const ShardArgs& a, uint64_t i) {
  const uint32_t h = gen_fold(a, i);
  return a.rss ? (uint32_t)a.rss[h % a.rss_len] : h % a.world;
}

__device__ __forceinline__ uint32_t shard_mine(const ShardArgs& a, uint64_t i0, uint32_t& bits) {
  bits = 0;
#pragma unroll 4
  for (int k = 0; k < kShardPer; ++k) {
    const uint64_t i = i0 + k;
    if (i < a.n_global && gen_owner(a, i) == a.rank) bits |= 1u << k;
  }
  return (uint32_t)__popc(bits);
}

__global__ __launch_bounds__(kBlock) void k_shard_count(ShardArgs a) {
  __shared__ uint32_t s_tmp[4];
  uint32_t bits;
  const uint32_t c = shard_mine(a, blockIdx.x * kShardChunk + threadIdx.x * (uint64_t)kShardPer, bits);
  uint32_t total;
  (void)block_excl_scan(c, s_tmp, total);
  if (threadIdx.x == 0) a.scratch[blockIdx.x] = total;
}

// one block: exclusive prefix over the chunk counts (each thread a contiguous run)
__global__ __launch_bounds__(kBlock) void k_shard_scan(ShardArgs a, uint64_t nchunks) {
  __shared__ uint64_t s_sum[kBlock];
  __shared__ uint32_t s_bad;
  const uint64_t per = (nchunks + kBlock - 1) / kBlock;
  const uint64_t lo = threadIdx.x * per, hi = lo + per < nchunks ? lo + per : nchunks;
  uint64_t sum = 0;
  for (uint64_t b = lo; b < hi; ++b) sum += a.scratch[b];
  s_sum[threadIdx.x] = sum;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  // an RSS entry >= world would drop its bucket's frames on every rank: such a
  // table yields the count ~0 (TCBEE_RSS_INVALID), which no shard can have
  if (a.rss)
    for (uint32_t b = threadIdx.x; b < a.rss_len; b += kBlock)
      if ((uint32_t)a.rss[b] >= (uint32_t)a.world) s_bad = 1;
  __syncthreads();
  uint64_t base = 0;
  for (uint32_t t = 0; t < threadIdx.x; ++t) base += s_sum[t];
  for (uint64_t b = lo; b < hi; ++b) {
    const uint64_t c = a.scratch[b];
    a.scratch[b] = base;
    base += c;
  }
  if (threadIdx.x == kBlock - 1) *a.n_out = s_bad ? ~0ull : base;
}

__global__ __launch_bounds__(kBlock) void k_shard_write(ShardArgs a) {
  __shared__ uint32_t s_tmp[4];
  const uint64_t i0 = blockIdx.x * kShardChunk + threadIdx.x * (uint64_t)kShardPer;
  uint32_t bits;
  const uint32_t c = shard_mine(a, i0, bits);
  uint32_t total;
  uint64_t pos = a.scratch[blockIdx.x] + block_excl_scan(c, s_tmp, total);
  while (bits) {
    const int k = __ffs(bits) - 1;
    bits &= bits - 1;
    if (pos < a.cap) {
      a.gidx[pos] = i0 + k;
      a.caplen[pos] = gen_caplen(i0 + k, a.imix, a.seed);
    }
    ++pos;
  }
}

// frames per RSS bucket: an LDS histogram per block, one device add per bucket
__global__ __launch_bounds__(kBlock) void k_rss_load(ShardArgs a) {
  __shared__ uint32_t s_h[kRssMaxLen];
  for (uint32_t b = threadIdx.x; b < a.rss_len; b += kBlock) s_h[b] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)kBlock + threadIdx.x; i < a.n_global;
       i += (uint64_t)gridDim.x * kBlock)
    atomicAdd(&s_h[gen_fold(a, a.first + i) % a.rss_len], 1u);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < a.rss_len; b += kBlock)
    if (s_h[b]) atomicAdd((unsigned long long*)&a.scratch[b], (unsigned long long)s_h[b]);
}

hipError_t launch_rss_load(const ShardArgs& a, hipStream_t s) {
  const hipError_t e = hipMemsetAsync(a.scratch, 0, sizeof(uint64_t) * a.rss_len, s);
  if (e != hipSuccess) return e;
  if (a.n_global == 0) return hipSuccess;
  // a block covers >= 64k frames (its histogram flush costs rss_len adds)
  uint64_t g = (a.n_global + 65535) / 65536;
  if (g > 2048) g = 2048;
  hipLaunchKernelGGL(k_rss_load, dim3((unsigned)g), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_shard_index(const ShardArgs& a, hipStream_t s) {
  const uint64_t nchunks = (a.n_global + kShardChunk - 1) / kShardChunk;
  if (nchunks == 0) return hipMemsetAsync(a.n_out, 0, sizeof(uint64_t), s);
  hipLaunchKernelGGL(k_shard_count, dim3((unsigned)nchunks), dim3(kBlock), 0, s, a);
  hipLaunchKernelGGL(k_shard_scan, dim3(1), dim3(kBlock), 0, s, a, nchunks);
  hipLaunchKernelGGL(k_shard_write, dim3((unsigned)nchunks), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static unsigned grid_for(uint64_t n, unsigned cap = 4096) {
  const uint64_t g = (n + kBlock - 1) / kBlock;
  return (unsigned)(g == 0 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_gen(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                      uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed,
                      hipStream_t s, const uint64_t* gidx, const uint64_t* zcdf) {
  hipLaunchKernelGGL(k_gen, dim3(grid_for(n, 8192)), dim3(kBlock), 0, s, arena, off, len, n,
                     first_index, kind, n_flows, seed, gidx, zcdf);
  return hipGetLastError();
}

}  // namespace tcbee

// tcbee_exchange.hip — kernels of the multi-GPU rows: flow-table
// export, the all-gather merge, the owner exchange of contiguous shards, the
// flow-hash exchange's first frames and global ids, and the local -> global id
// remap. None of them runs in a one-GPU step.
#include "tcbee_table.h"

namespace tcbee {

// ---------------------------------------------------------------------------
// flow-table export / multi-table merge / id remap (multi-GPU row of DESIGN.md §7)
// An entry is tcbee_flow_entry viewed as u64[8]: key k0..k4, pkts, bytes, first_seen.
// ---------------------------------------------------------------------------
__global__ void k_export(FlowTable t, uint64_t* out, uint64_t cap, const PersistState* p,
                         uint64_t* n_out) {
  const uint64_t nflows = p->flow_count;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nflows;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* m = t.ent + 8 * c;  // key m[0..4]
    const uint64_t id = t.cmap[c];
    if (id >= cap) continue;
    uint64_t* e = out + 8 * id;
#pragma unroll
    for (int j = 0; j < 5; ++j) e[j] = m[j];
    e[5] = t.cnt[2 * id];
    e[6] = t.cnt[2 * id + 1];
    e[7] = t.cfs[c];
  }
  if (n_out && blockIdx.x == 0 && threadIdx.x == 0) {
    n_out[0] = nflows < cap ? nflows : cap;
    n_out[1] = p->rec_base;  // accepted frames so far = records of this segment
  }
}

// Global-order export (flow-hash shards). The table holds the flows of ONE batch
// (records [rec_base - n_acc, rec_base) of the context); a flow's first record r
// is mapped to its frame (rec_frame[r], or r itself when every frame of the batch
// was accepted) and that frame to its position in the global trace. A first
// record that cannot be placed flags kStShard and exports first_seen ~0.
__device__ __forceinline__ uint64_t place_first(const GlobalExportArgs& g, uint64_t fs, uint64_t lo,
                                                uint64_t hi, bool bad_batch) {
  if (fs >= lo && fs < hi && fs - lo < g.out_cap && !bad_batch) {
    const uint64_t r = fs - lo;
    const uint64_t fr = g.rec_frame == nullptr ? r : g.rec_frame[r];
    if (fr < g.n_frames) return g.frame_gidx[fr];
  }
  return ~0ull;
}

__global__ void k_export_global(GlobalExportArgs g) {
  const uint64_t nacc = g.batch->n_acc;
  const uint64_t lo = g.persist->rec_base - nacc;  // advanced by K2
  const uint64_t hi = lo + nacc;
  const uint64_t nflows = g.persist->flow_count;
  const bool bad_batch = g.rec_frame == nullptr && nacc != g.n_frames;
  bool bad = false;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nflows;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t* m = g.tab.ent + 8 * c;
    const uint64_t id = g.tab.cmap[c];
    if (id >= g.cap) continue;
    uint64_t* e = g.out + 8 * id;
#pragma unroll
    for (int j = 0; j < 5; ++j) e[j] = m[j];
    e[5] = g.tab.cnt[2 * id];
    e[6] = g.tab.cnt[2 * id + 1];
    const uint64_t gfs = place_first(g, g.tab.cfs[c], lo, hi, bad_batch);
    bad = bad || gfs == ~0ull;
    e[7] = gfs;
  }
  if (__any(bad) && __lane_id() == 0) atomicOr(&g.persist->status, kStShard);
  if (g.n_out && blockIdx.x == 0 && threadIdx.x == 0) {
    g.n_out[0] = nflows < g.cap ? nflows : g.cap;
    g.n_out[1] = 0;  // first_seen is already global: the merge rebases nothing
    if (bad_batch) atomicOr(&g.persist->status, kStShard);
  }
}

// Records of this rank below each merged flow's first frame: a binary search
// over the rank's record stream, whose global frame indices ascend.
__global__ void k_records_before(FlowTable t, const PersistState* p, const uint32_t* rec_frame,
                                 const uint64_t* frame_gidx, const uint64_t* n_rec_dev,
                                 uint64_t n_rec_max, uint64_t* out, uint64_t cap) {
  const uint64_t nflows = p->flow_count;
  const uint64_t n = n_rec_dev && *n_rec_dev < n_rec_max ? *n_rec_dev : n_rec_max;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nflows;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t id = t.cmap[c];
    if (id >= cap) continue;
    const uint64_t G = t.cfs[c];
    uint64_t lo = 0, len = n;  // first record whose global frame >= G
    while (len > 0) {
      const uint64_t half = len >> 1, mid = lo + half;
      const uint64_t gm = frame_gidx[rec_frame ? rec_frame[mid] : mid];
      if (gm < G) {
        lo = mid + 1;
        len -= half + 1;
      } else {
        len = half;
      }
    }
    out[id] = lo;
  }
}

__global__ void k_set_first_seen(FlowTable t, const PersistState* p, const uint64_t* fs_by_id,
                                 uint64_t cap) {
  const uint64_t nflows = p->flow_count;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nflows;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t id = t.cmap[c];
    if (id < cap) t.cfs[c] = fs_by_id[id];
  }
}

// Flow-hash exchange (disjoint per-rank tables): for the flows FIRST
// SEEN IN THIS BATCH (local ids [fbase, fbase + n_new)), the global frame index of
// each one's first record (placed as k_export_global places it) at out[id - fbase];
// n_out = {n_new, fbase}. Batches are windows of one global trace (the same global
// frame range on every rank), so the flows new in a window are exactly the union
// of every rank's new flows, and older flows keep the ids they already have. The
// batch's new flows are its claims [fbase, fbase + n_new) (ids a permutation of them).
__global__ void k_first_frames(GlobalExportArgs g) {
  const uint64_t nacc = g.batch->n_acc;
  const uint64_t lo = g.persist->rec_base - nacc;  // advanced by K2
  const uint64_t hi = lo + nacc;
  const uint64_t nnew = g.batch->n_new;
  const uint64_t fbase = g.persist->flow_count - nnew;
  const bool bad_batch = g.rec_frame == nullptr && nacc != g.n_frames;
  bool bad = false;
  for (uint64_t c = fbase + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < fbase + nnew;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t id = g.tab.cmap[c];
    if (id < fbase || id - fbase >= g.cap) continue;
    const uint64_t gfs = place_first(g, g.tab.cfs[c], lo, hi, bad_batch);
    bad = bad || gfs == ~0ull;
    g.out[id - fbase] = gfs;
  }
  if (__any(bad) && __lane_id() == 0) atomicOr(&g.persist->status, kStShard);
  if (g.n_out && blockIdx.x == 0 && threadIdx.x == 0) {
    g.n_out[0] = nnew < g.cap ? nnew : g.cap;
    g.n_out[1] = fbase;
    if (bad_batch || nnew > g.cap) atomicOr(&g.persist->status, kStShard);
  }
}

// gid[fbase_r + l] = gbase + l + (this window's new flows of the other ranks whose
// first frame comes earlier): each rank's array is ascending (its new flows are in
// local first-seen order, a subsequence of the global order; frames are distinct
// across ranks), so one binary search per other rank counts them. gbase = global
// flows of earlier windows; gbase_out = gbase + every rank's new flows.
__global__ void k_global_ids(const uint64_t* allG, const uint64_t* alln, uint64_t nstride,
                             uint32_t world, uint32_t rank, uint64_t stride, uint32_t* gid,
                             uint64_t cap, const uint64_t* gbase_in, uint64_t* gbase_out) {
  const uint64_t gbase = gbase_in ? *gbase_in : 0;
  const uint64_t mine = alln[nstride * rank] < stride ? alln[nstride * rank] : stride;
  const uint64_t fb = alln[nstride * rank + 1];
  if (gbase_out && blockIdx.x == 0 && threadIdx.x == 0) {
    uint64_t tot = gbase;
    for (uint32_t r = 0; r < world; ++r) tot += alln[nstride * r];
    *gbase_out = tot;
  }
  for (uint64_t l = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; l < mine;
       l += (uint64_t)gridDim.x * blockDim.x) {
    if (fb + l >= cap) break;
    const uint64_t G = allG[(uint64_t)rank * stride + l];
    uint64_t id = gbase + l;
    for (uint32_t r = 0; r < world; ++r) {
      if (r == rank) continue;
      const uint64_t* A = allG + (uint64_t)r * stride;
      uint64_t lo = 0, len = alln[nstride * r] < stride ? alln[nstride * r] : stride;
      while (len > 0) {
        const uint64_t half = len >> 1;
        if (A[lo + half] < G) {
          lo += half + 1;
          len -= half + 1;
        } else {
          len = half;
        }
      }
      id += lo;
    }
    gid[fb + l] = (uint32_t)id;
  }
}

// ---------------------------------------------------------------------------
// Owner exchange (contiguous shards): every rank may hold every
// flow, so each flow is merged at ONE owner rank, owner = fold32(flow_hash64(key))
// % world (the NIC-RSS function of tcbee_flowhash_owner), instead of every rank
// merging every table.
// ---------------------------------------------------------------------------
// The local table's flows bucketed by owner: per block, LDS counts per owner, one
// device-scope reservation per (block, owner), then the entries at their places.
__global__ __launch_bounds__(kBlock) void k_owner_bucket(OwnerArgs a) {
  __shared__ uint32_t s_cnt[kMaxOwners];
  __shared__ uint64_t s_base[kMaxOwners];
  const uint32_t tid = threadIdx.x;
  const uint64_t nflows = a.persist->flow_count;
  if (tid < a.world) s_cnt[tid] = 0;
  if (blockIdx.x == 0 && tid == 0) a.meta[a.world] = a.persist->rec_base;
  __syncthreads();
  uint32_t own[kOwnerItems], rank[kOwnerItems];
  const uint64_t s0 = (uint64_t)blockIdx.x * kBlock * kOwnerItems + tid;
  uint32_t dropped = 0;
#pragma unroll
  for (int k = 0; k < kOwnerItems; ++k) {
    own[k] = 0xFFFFFFFFu;
    const uint64_t c = s0 + (uint64_t)k * kBlock;  // claim
    if (c >= nflows) continue;
    const uint64_t* m = a.tab.ent + 8 * c;
    // a flow whose local id has no place in the id map takes NO segment slot (a
    // counted but unwritten slot would reach its owner as a phantom flow)
    if (a.tab.cmap[c] >= a.map_cap) {
      ++dropped;
      continue;
    }
    own[k] = fold32(flow_hash64(m[0], m[1], m[2], m[3], m[4])) % a.world;
    rank[k] = atomicAdd(&s_cnt[own[k]], 1u);
  }
  __syncthreads();
  if (tid < a.world) {
    const uint32_t c = s_cnt[tid];
    s_base[tid] = c ? atomicAdd((unsigned long long*)&a.meta[tid], (unsigned long long)c) : 0ull;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kOwnerItems; ++k) {
    if (own[k] == 0xFFFFFFFFu) continue;
    const uint64_t pos = s_base[own[k]] + rank[k];
    const uint64_t c = s0 + (uint64_t)k * kBlock;
    const uint64_t* m = a.tab.ent + 8 * c;
    if (pos >= a.seg_cap) {  // positions [0, seg_cap) of every segment stay dense
      ++dropped;
      continue;
    }
    const uint64_t e = (uint64_t)own[k] * a.seg_cap + pos;
    uint64_t* out = a.ent + 8 * e;
#pragma unroll
    for (int j = 0; j < 5; ++j) out[j] = m[j];
    out[5] = 0;  // pkts / bytes: K3 has not run (the ids come first)
    out[6] = 0;
    out[7] = a.tab.cfs[c];  // first_seen, local to this rank's record stream
    a.lid[e] = a.tab.cmap[c];
  }
  // meta[world + 1]: entries this rank dropped. Every rank sees it after the meta
  // all-gather, so the PEERS of an overflowing rank can flag their ids as wrong too
  // (tcbee_status_raise_device), not only the rank that dropped them
  for (int o = 32; o > 0; o >>= 1) dropped += __shfl_xor(dropped, o);
  if (dropped && __lane_id() == 0) {
    atomicOr(a.status, kStShard);
    atomicAdd((unsigned long long*)&a.meta[a.world + 1], (unsigned long long)dropped);
  }
}

// status |= kStShard when any v[i * stride] (i < n) is non-zero: a peer's dropped
// owner entries (OwnerExchange) make this rank's global ids unreliable as well
__global__ void k_status_raise(const uint64_t* v, uint64_t n, uint64_t stride, uint32_t* status) {
  bool any = false;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) any |= v[i * stride] != 0;
  if (__any(any) && __lane_id() == 0) atomicOr(status, kStShard);
}

__global__ void k_first_seen(FlowTable t, const PersistState* p, uint64_t* out, uint64_t cap,
                             uint64_t* n_out) {
  const uint64_t nflows = p->flow_count;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nflows;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t id = t.cmap[c];
    if (id < cap) out[id] = t.cfs[c];
  }
  if (n_out && blockIdx.x == 0 && threadIdx.x == 0) {
    n_out[0] = p->flow_count < cap ? p->flow_count : cap;
    n_out[1] = 0;
  }
}

__global__ void k_owner_return(const uint32_t* ids, const uint64_t* seg_meta, uint32_t world,
                               uint64_t seg_cap, const uint32_t* gmap, uint64_t gmap_len,
                               uint32_t* ret) {
  const uint64_t total = (uint64_t)world * seg_cap;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t r = e / seg_cap, j = e - r * seg_cap;
    if (j >= seg_meta[2 * r]) continue;
    const uint32_t id = ids[e];
    ret[e] = id < gmap_len ? gmap[id] : 0xFFFFFFFFu;
  }
}

__global__ void k_owner_apply(const uint32_t* back, const uint32_t* lid, const uint64_t* meta,
                              uint32_t world, uint64_t seg_cap, uint32_t* map, uint64_t map_cap) {
  const uint64_t total = (uint64_t)world * seg_cap;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = e / seg_cap, j = e - o * seg_cap;
    if (j >= meta[o]) continue;
    const uint32_t l = lid[e];
    if (l < map_cap) map[l] = back[e];
  }
}

// omap[claim] = id_map[cmap[claim]] for this batch's flows (output ids of K3)
__global__ void k_compose(const uint32_t* cmap, const uint32_t* id_map, uint64_t map_len,
                          const BatchState* b, uint32_t* omap) {
  const uint64_t n = b->flow_total;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < n;
       c += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t l = cmap[c];
    omap[c] = l < map_len ? id_map[l] : 0xFFFFFFFFu;
  }
}

// Inserts every valid entry of nseg segments (segment r = rank r's local table,
// first_seen local to that rank) with first_seen rebased to the global record
// index; per-slot counters summed. out_slot[e] = merged slot (or ~0).
__global__ void k_merge_insert(MergeArgs g) {
  const uint64_t total = g.nseg * g.stride;
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < total;
       e += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t seg = e / g.stride, j = e % g.stride;
    if (j >= g.seg_meta[2 * seg]) {
      g.out_slot[e] = 0xFFFFFFFFu;
      continue;
    }
    const uint64_t* E = g.ent + 8 * e;
    const uint64_t K[5] = {E[0], E[1], E[2], E[3], E[4]};
    uint32_t fs = 0xFFFFFFFFu, claim = 0xFFFFFFFFu;
    // (a fresh table: every claim is new, fbase 0)
    const uint32_t s = flow_upsert(g.tab, K, flow_hash64(K[0], K[1], K[2], K[3], K[4]), g.batch,
                                   g.new_list, g.persist, 0, fs, claim);
    g.out_slot[e] = s == 0xFFFFFFFFu ? 0xFFFFFFFFu : claim;
    if (s == 0xFFFFFFFFu) continue;
    atomicAdd((unsigned long long*)&g.mcnt[2ull * claim], (unsigned long long)E[5]);
    atomicAdd((unsigned long long*)&g.mcnt[2ull * claim + 1], (unsigned long long)E[6]);
    uint64_t base = 0;  // records of the segments before this one
    for (uint64_t q = 0; q < seg; ++q) base += g.seg_meta[2 * q + 1];
    // the slot's fs32 (max_total_records < 2^31, checked by the ABI); an unplaceable
    // first_seen (~0 from a flagged exporter) stays past every record of the merge
    const uint64_t gfs = base + E[7];
    atomicMin(slot_fs_any(g.tab, s), gfs < (uint64_t)kFs32Flag ? (uint32_t)gfs : kFs32Flag - 1u);
  }
}

// entry slot -> merged dense id; per-slot counters -> by-id counters; flow count
__global__ void k_merge_finish(MergeArgs g) {
  const uint64_t total = g.nseg * g.stride;
  const uint64_t nflows = g.batch->n_new;  // a fresh table: claims [0, n_new)
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  for (uint64_t e = t0; e < total; e += stride) {
    const uint32_t c = g.out_slot[e];
    g.out_slot[e] = c == 0xFFFFFFFFu || c >= nflows ? 0xFFFFFFFFu : g.tab.cmap[c];
  }
  for (uint64_t c = t0; c < nflows; c += stride) {
    const uint64_t id = g.tab.cmap[c];
    g.tab.cnt[2 * id] = g.mcnt[2 * c];
    g.tab.cnt[2 * id + 1] = g.mcnt[2 * c + 1];
  }
  for (uint64_t w = t0; w <= g.batch->fs_max_word; w += stride) g.bitmap[w] = 0;
  if (t0 == 0) {
    uint64_t recs = 0;
    for (uint64_t q = 0; q < g.nseg; ++q) recs += g.seg_meta[2 * q + 1];
    g.persist->flow_count += g.batch->n_new;
    g.persist->rec_base += recs;
  }
}

// ids[p] = map[ids[p]] (N>1 local -> global flow ids). The first kRemapLds map
// entries are staged in LDS as u16 (a rank's local ids are dense from 0; a global
// id >= 0xFFFF is looked up in HBM instead), 32 KiB per workgroup, so the remap
// that overlaps the next step's K1 takes few of K1's LDS slots; the ids stream
// through as 16-B non-temporal vectors, 4 per thread in flight.
constexpr uint32_t kRemapLds = 16384;
constexpr int kRemapBlock = 512;
__global__ __launch_bounds__(kRemapBlock) void k_remap(uint32_t* ids, uint64_t n_max,
                                                       const uint64_t* n_dev, const uint32_t* map,
                                                       uint64_t map_len) {
  __shared__ uint16_t s_map[kRemapLds];
  const uint64_t n = n_dev && *n_dev < n_max ? *n_dev : n_max;
  const uint32_t m = map_len < kRemapLds ? (uint32_t)map_len : kRemapLds;
  for (uint32_t j = threadIdx.x; j < m; j += kRemapBlock) {
    const uint32_t g = map[j];
    s_map[j] = g < 0xFFFFu ? (uint16_t)g : (uint16_t)0xFFFFu;
  }
  __syncthreads();
  auto tr = [&](uint32_t v) -> uint32_t {
    if (v < m) {
      const uint32_t g = s_map[v];
      return g != 0xFFFFu ? g : map[v];
    }
    return v < map_len ? map[v] : 0xFFFFFFFFu;
  };
  const uint64_t t0 = blockIdx.x * (uint64_t)kRemapBlock + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * kRemapBlock;
  uint64_t head = ((16u - ((uintptr_t)ids & 15u)) & 15u) >> 2;  // scalar up to 16-B alignment
  if (head > n) head = n;
  for (uint64_t p = t0; p < head; p += stride) ids[p] = tr(ids[p]);
  u32x4* v4 = reinterpret_cast<u32x4*>(ids + head);
  const uint64_t n4 = (n - head) >> 2;
  constexpr int R = 4;
  for (uint64_t q0 = t0; q0 < n4; q0 += stride * R) {
    u32x4 v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint64_t q = q0 + (uint64_t)u * stride;
      v[u] = __builtin_nontemporal_load(v4 + (q < n4 ? q : n4 - 1));  // unconditional loads
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const uint64_t q = q0 + (uint64_t)u * stride;
      if (q < n4) {
        u32x4 o;
        o[0] = tr(v[u][0]);
        o[1] = tr(v[u][1]);
        o[2] = tr(v[u][2]);
        o[3] = tr(v[u][3]);
        __builtin_nontemporal_store(o, v4 + q);
      }
    }
  }
  for (uint64_t p = head + (n4 << 2) + t0; p < n; p += stride) ids[p] = tr(ids[p]);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static unsigned grid_for(uint64_t n, unsigned cap = 4096) {
  const uint64_t g = (n + kBlock - 1) / kBlock;
  return (unsigned)(g == 0 ? 1 : (g > cap ? cap : g));
}

hipError_t launch_export(FlowTable t, uint64_t* out, uint64_t cap, const PersistState* p,
                         uint64_t* n_out, hipStream_t s) {
  hipLaunchKernelGGL(k_export, dim3(grid_for(t.max_claims)), dim3(kBlock), 0, s, t, out, cap, p, n_out);
  return hipGetLastError();
}

hipError_t launch_export_global(const GlobalExportArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_export_global, dim3(grid_for(g.tab.max_claims)), dim3(kBlock), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_records_before(FlowTable t, const PersistState* p, const uint32_t* rec_frame,
                                 const uint64_t* frame_gidx, const uint64_t* n_rec,
                                 uint64_t n_rec_max, uint64_t* out, uint64_t cap, hipStream_t s) {
  hipLaunchKernelGGL(k_records_before, dim3(grid_for(t.max_claims)), dim3(kBlock), 0, s, t, p,
                     rec_frame, frame_gidx, n_rec, n_rec_max, out, cap);
  return hipGetLastError();
}

hipError_t launch_set_first_seen(FlowTable t, const PersistState* p, const uint64_t* fs_by_id,
                                 uint64_t cap, hipStream_t s) {
  hipLaunchKernelGGL(k_set_first_seen, dim3(grid_for(t.max_claims)), dim3(kBlock), 0, s, t, p,
                     fs_by_id, cap);
  return hipGetLastError();
}

hipError_t launch_owner_bucket(const OwnerArgs& a, hipStream_t s) {
  const uint64_t per = (uint64_t)kBlock * kOwnerItems;
  const uint64_t nb = (a.tab.max_claims + per - 1) / per;
  hipLaunchKernelGGL(k_owner_bucket, dim3((unsigned)nb), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_status_raise(const uint64_t* v, uint64_t n, uint64_t stride, uint32_t* status,
                               hipStream_t s) {
  hipLaunchKernelGGL(k_status_raise, dim3(1), dim3(kBlock), 0, s, v, n, stride, status);
  return hipGetLastError();
}

hipError_t launch_first_seen(FlowTable t, const PersistState* p, uint64_t* out, uint64_t cap,
                             uint64_t* n_out, hipStream_t s) {
  hipLaunchKernelGGL(k_first_seen, dim3(grid_for(t.max_claims)), dim3(kBlock), 0, s, t, p, out, cap,
                     n_out);
  return hipGetLastError();
}

hipError_t launch_owner_return(const uint32_t* ids, const uint64_t* seg_meta, uint32_t world,
                               uint64_t seg_cap, const uint32_t* gmap, uint64_t gmap_len,
                               uint32_t* ret, hipStream_t s) {
  hipLaunchKernelGGL(k_owner_return, dim3(grid_for((uint64_t)world * seg_cap)), dim3(kBlock), 0, s,
                     ids, seg_meta, world, seg_cap, gmap, gmap_len, ret);
  return hipGetLastError();
}

hipError_t launch_owner_apply(const uint32_t* back, const uint32_t* lid, const uint64_t* meta,
                              uint32_t world, uint64_t seg_cap, uint32_t* map, uint64_t map_cap,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_owner_apply, dim3(grid_for((uint64_t)world * seg_cap)), dim3(kBlock), 0, s,
                     back, lid, meta, world, seg_cap, map, map_cap);
  return hipGetLastError();
}

hipError_t launch_first_frames(const GlobalExportArgs& g, hipStream_t s) {
  hipLaunchKernelGGL(k_first_frames, dim3(grid_for(g.tab.max_claims)), dim3(kBlock), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_global_ids(const uint64_t* allG, const uint64_t* alln, uint64_t nstride,
                             uint32_t world, uint32_t rank, uint64_t stride, uint32_t* gid,
                             uint64_t cap, const uint64_t* gbase_in, uint64_t* gbase_out,
                             hipStream_t s) {
  hipLaunchKernelGGL(k_global_ids, dim3(grid_for(stride)), dim3(kBlock), 0, s, allG, alln, nstride,
                     world, rank, stride, gid, cap, gbase_in, gbase_out);
  return hipGetLastError();
}

hipError_t launch_compose(const uint32_t* cmap, const uint32_t* id_map, uint64_t map_len,
                          const BatchState* b, uint32_t* omap, uint64_t max_flows, hipStream_t s) {
  hipLaunchKernelGGL(k_compose, dim3(grid_for(max_flows)), dim3(kBlock), 0, s, cmap, id_map, map_len,
                     b, omap);
  return hipGetLastError();
}

hipError_t launch_merge(const MergeArgs& g, const RankArgs& r, hipStream_t s) {
  const unsigned grid = grid_for(g.nseg * g.stride);
  hipLaunchKernelGGL(k_merge_insert, dim3(grid), dim3(kBlock), 0, s, g);
  hipError_t e = launch_rank(r, s);
  if (e != hipSuccess) return e;
  const uint64_t work = g.nseg * g.stride > g.tab.max_claims ? g.nseg * g.stride : g.tab.max_claims;
  hipLaunchKernelGGL(k_merge_finish, dim3(grid_for(work)), dim3(kBlock), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_remap(uint32_t* ids, uint64_t n_max, const uint64_t* n_dev, const uint32_t* map,
                        uint64_t map_len, hipStream_t s) {
  // up to 512 workgroups (beside the next step's K1, 32..512 workgroups gave the
  // same step time once the LDS map was u16, round 2)
  constexpr uint64_t gmax = 512;
  const uint64_t want = (n_max + 4ull * kRemapBlock - 1) / (4ull * kRemapBlock);
  hipLaunchKernelGGL(k_remap, dim3((unsigned)(want < gmax ? (want ? want : 1) : gmax)),
                     dim3(kRemapBlock), 0, s, ids, n_max, n_dev, map,
                     map_len);
  return hipGetLastError();
}

}  // namespace tcbee

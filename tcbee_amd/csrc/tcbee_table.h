// tcbee_table.h — device-side building blocks shared by the kernel translation
// units: agent-scope loads/stores, byte helpers, and the flow table's slot layout
// and insert protocol (flow_upsert: K1's slow path and the multi-GPU merge).
// Included by tcbee_kernels.hip (K1-K3), tcbee_exchange.hip (N>1 table / id
// exchange) and tcbee_synth.hip (synthetic traces).
#pragma once
#include <hip/hip_runtime.h>

#include "tcbee_gen.h"
#include "tcbee_internal.h"
#include "tcbee_layout.h"

namespace tcbee {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ld_agent(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Read at the coherence point (an RMW is never served from a stale cache).
__device__ __forceinline__ uint64_t ld_coherent(uint64_t* p) {
  return __hip_atomic_fetch_or(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }
__device__ __forceinline__ uint32_t bswap16(uint32_t v) {
  return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}
// bytes [r, r+4) of the 8-byte little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t align_bytes(uint32_t hi, uint32_t lo, uint32_t r) {
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}
__device__ __forceinline__ uint64_t lanemask_lt() {
  const uint32_t lane = __lane_id();
  return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

constexpr uint32_t kSpinLimit = 1u << 24;

// ---------------------------------------------------------------------------
// Flow table (tcbee_internal.h): compact slot lines + per-claim entries.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld_agent32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint64_t kKindBusy = 1ull << 56;
constexpr uint64_t kClaimBits = 0xFFFFFFull << 32;  // w1 bits 55:32
__device__ __forceinline__ uint32_t slot_line(uint32_t s) { return __umulhi(s, 0xAAAAAAABu) >> 1; }  // s / 3
__device__ __forceinline__ uint64_t* slot_ptr(const FlowTable& T, uint32_t s) {
  const uint32_t l = slot_line(s);
  return T.slots + 8ull * l + 2u * (s - l * kSlotsPerLine);
}
__device__ __forceinline__ uint32_t* slot_fs(const FlowTable& T, uint32_t s) {
  const uint32_t l = slot_line(s);
  return reinterpret_cast<uint32_t*>(T.slots + 8ull * l + 6) + (s - l * kSlotsPerLine);
}
// home slot: line from the hash's high word (range reduction), position from its low bits
__device__ __forceinline__ uint32_t home_slot(uint64_t h, uint64_t nlines) {
  const uint32_t line = (uint32_t)(((h >> 32) * nlines) >> 32);
  return line * kSlotsPerLine + (uint32_t)(((h & 0xFFFFFFull) * kSlotsPerLine) >> 24);
}
// the compact slot words that name an IPv4-form key K: w0 and the kind | lo32 bits
// of w1 (all but the claim)
__device__ __forceinline__ void key_slot_words(const uint64_t (&K)[5], uint64_t h, uint64_t& w0,
                                               uint64_t& kl) {
  (void)h;
  w0 = (K[1] >> 32) | (K[3] & 0xFFFFFFFF00000000ull);
  kl = (2ull << 56) | (uint32_t)K[4];  // sport | dport << 16 (protocol is always 6)
}

// first_seen (fs32) while a flow's first record index is not known yet: the
// claimer stores kFs32Flag | its frame index, so later readers of a hot new flow
// can tell locally whether they precede the claimer (and only those contend on the
// atomicMin) instead of all seeing "unset". Batch-local: batches stay < 2^31 frames.
__device__ __forceinline__ bool fs_needs_min(uint32_t fs_seen, uint32_t frame_i, uint32_t p) {
  if (fs_seen & kFs32Flag) return (fs_seen & ~kFs32Flag) >= frame_i;  // the claimer or earlier
  return p < fs_seen;
}

// the fs32 word of slot id s (compact or wide)
__device__ __forceinline__ uint32_t* slot_fs_any(const FlowTable& T, uint32_t s) {
  if (s & kWideSlot) return reinterpret_cast<uint32_t*>(T.wide + 8ull * (s & ~kWideSlot) + 6);
  return slot_fs(T, s);
}
__device__ __forceinline__ bool key_is_v4form(const uint64_t (&K)[5]) {
  return (K[0] | K[2] | (K[1] & 0xFFFFFFFFull) | (K[3] & 0xFFFFFFFFull)) == 0;
}

// Flow-table upsert; identity = the full 40-B key. Returns the slot id (~0 on
// failure; wide slots carry kWideSlot); `claim` = the flow's claim index
// (flow_count before this batch + its position in this batch's new-flow list),
// fixed before the slot is published. A claim at or past max_claims is refused:
// the slot is published dead (this key, no claim) so the flow's later frames find
// it instead of claiming again, and the status reports TCBEE_EFLOWFULL.
//
// Compact slots (IPv4-form keys): CAS w1 empty -> busy, the entry (key) and the
// slot's fs32 mark and w0 by agent-scope stores, drain, then w1 (agent-scope
// store). The slot's line holds w0, w1 and fs32 together, so a snapshot that shows
// a published w1 shows its w0 and mark, and the slot alone decides a match.
__device__ inline uint32_t flow_upsert_compact(const FlowTable& T, const uint64_t (&K)[5], uint64_t h,
                                        BatchState* batch, uint64_t* new_list,
                                        PersistState* persist, uint64_t fbase, uint32_t& fs_seen,
                                        uint32_t& claim, uint32_t claim_mark) {
  uint64_t w0k, kl;
  key_slot_words(K, h, w0k, kl);
  const uint32_t nslots = (uint32_t)T.nlines * kSlotsPerLine;
  uint32_t s = home_slot(h, T.nlines);
  for (uint32_t probe = 0; probe < nslots; ++probe) {
    uint64_t* m = slot_ptr(T, s);
    uint64_t cur = ld_agent(m + 1);
    if (cur == 0) {
      uint64_t expected = 0;
      if (__hip_atomic_compare_exchange_strong(m + 1, &expected, kKindBusy, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        const uint64_t slot_no = atomicAdd((unsigned long long*)&batch->n_new, 1ull);
        const uint64_t cl = fbase + slot_no;
        if (cl >= T.max_claims) {
          st_agent(m, w0k);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_agent(m + 1, kl + (2ull << 56));  // dead
          atomicOr(&persist->status, kStFlowFull);
          return 0xFFFFFFFFu;
        }
        new_list[slot_no] = s;
        claim = (uint32_t)cl;
        uint64_t* e = T.ent + 8 * cl;
#pragma unroll
        for (int j = 0; j < 5; ++j) st_agent(e + j, K[j]);
        st_agent32(slot_fs(T, s), claim_mark);
        st_agent(m, w0k);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(m + 1, kl | (cl << 32));
        fs_seen = claim_mark;
        return s;
      }
      cur = expected;
    }
    for (uint32_t spins = 0; cur == kKindBusy; ++spins) {
      if (spins > kSpinLimit) {
        atomicOr(&persist->status, kStSpin);
        return 0xFFFFFFFFu;
      }
      __builtin_amdgcn_s_sleep(1);
      cur = ld_agent(m + 1);
    }
    const uint64_t ckl = cur & ~kClaimBits;
    if ((ckl == kl || ckl == kl + (2ull << 56)) && ld_agent(m) == w0k) {
      if (ckl != kl) return 0xFFFFFFFFu;  // dead slot of this key: the table was full
      fs_seen = ld_agent32(slot_fs(T, s));
      claim = (uint32_t)((cur & kClaimBits) >> 32);
      return s;
    }
    s = s + 1 == nslots ? 0u : s + 1;
  }
  atomicOr(&persist->status, kStFlowFull);
  return 0xFFFFFFFFu;
}

// Wide slots (other keys): the rounds-1/2 protocol — CAS the tag word empty ->
// busy, key (and entry) and the fs32 mark by agent-scope stores, drain, then the
// tag word. Readers poll the tag relaxed and compare the key by agent-scope loads;
// a mismatch is re-checked at the coherence point before the probe moves on
// (never a duplicate flow).
__device__ inline uint32_t flow_upsert_wide(const FlowTable& T, const uint64_t (&K)[5], uint64_t h,
                                     BatchState* batch, uint64_t* new_list, PersistState* persist,
                                     uint64_t fbase, uint32_t& fs_seen, uint32_t& claim,
                                     uint32_t claim_mark) {
  const uint32_t tag = hash_tag32(h);
  uint64_t s = h & T.wide_mask;
  for (uint64_t probe = 0; probe <= T.wide_mask; ++probe) {
    uint64_t* m = T.wide + s * 8;
    uint64_t cur = ld_agent(m);
    if (cur == kTagEmpty) {
      // the key is not in the table (it would lie before the first empty slot of its
      // probe sequence): once the wide-key budget is spent it is refused here, with a
      // plain load and no slot taken — only keys racing past this check publish dead
      // slots, so unexpected IPv6 traffic cannot fill the table with them
      if (T.max_wide < T.max_claims &&
          ld_agent(reinterpret_cast<const uint64_t*>(&persist->wide_claims)) >= T.max_wide) {
        atomicOr(&persist->status, kStFlowFull);
        return 0xFFFFFFFFu;
      }
      uint64_t expected = kTagEmpty;
      if (__hip_atomic_compare_exchange_strong(m, &expected, kTagBusy, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        if (!ld_agent32(T.wide_used)) st_agent32(T.wide_used, 1u);
#pragma unroll
        for (int j = 0; j < 5; ++j) st_agent(m + 1 + j, K[j]);
        // a context with fewer wide slots than max_flows (tcbee_ctx_create_ex) bounds
        // its wide keys exactly: refused BEFORE a claim number is taken (claims stay
        // dense), the slot published dead
        const bool wide_full =
            T.max_wide < T.max_claims &&
            atomicAdd((unsigned long long*)&persist->wide_claims, 1ull) >= T.max_wide;
        const uint64_t slot_no =
            wide_full ? 0ull : atomicAdd((unsigned long long*)&batch->n_new, 1ull);
        const uint64_t cl = wide_full ? T.max_claims : fbase + slot_no;
        if (cl >= T.max_claims) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_agent(m, (uint64_t)tag | (0xFFFFFFFFull << 32));  // dead
          atomicOr(&persist->status, kStFlowFull);
          return 0xFFFFFFFFu;
        }
        new_list[slot_no] = (uint32_t)s | kWideSlot;
        claim = (uint32_t)cl;
        uint64_t* e = T.ent + 8 * cl;
#pragma unroll
        for (int j = 0; j < 5; ++j) st_agent(e + j, K[j]);
        st_agent(m + 6, (uint64_t)claim_mark);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(m, (uint64_t)tag | (cl << 32));
        fs_seen = claim_mark;
        return (uint32_t)s | kWideSlot;
      }
      cur = expected;
    }
    for (uint32_t spins = 0; cur == kTagBusy; ++spins) {
      if (spins > kSpinLimit) {
        atomicOr(&persist->status, kStSpin);
        return 0xFFFFFFFFu;
      }
      __builtin_amdgcn_s_sleep(1);
      cur = ld_agent(m);
    }
    if ((uint32_t)cur == tag) {
      bool eq = true;
#pragma unroll
      for (int j = 0; j < 5; ++j) eq = eq && (ld_agent(m + 1 + j) == K[j]);
      if (!eq) {
        eq = true;
#pragma unroll
        for (int j = 0; j < 5; ++j) eq = eq && (ld_coherent(m + 1 + j) == K[j]);
      }
      if (eq) {
        if ((cur >> 32) == 0xFFFFFFFFull) return 0xFFFFFFFFu;  // dead: the table was full
        fs_seen = (uint32_t)ld_agent(m + 6);
        claim = (uint32_t)(cur >> 32);
        return (uint32_t)s | kWideSlot;
      }
    }
    s = (s + 1) & T.wide_mask;
  }
  atomicOr(&persist->status, kStFlowFull);
  return 0xFFFFFFFFu;
}

__device__ __forceinline__ uint32_t flow_upsert(const FlowTable& T, const uint64_t (&K)[5], uint64_t h,
                                                BatchState* batch, uint64_t* new_list,
                                                PersistState* persist, uint64_t fbase,
                                                uint32_t& fs_seen, uint32_t& claim,
                                                uint32_t claim_mark = 0xFFFFFFFFu) {
  return key_is_v4form(K)
             ? flow_upsert_compact(T, K, h, batch, new_list, persist, fbase, fs_seen, claim, claim_mark)
             : flow_upsert_wide(T, K, h, batch, new_list, persist, fbase, fs_seen, claim, claim_mark);
}


// exclusive scan over a 256-thread block; s_tmp: 4 words of LDS
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_tmp, uint32_t& total) {
  // 256 threads, 4 waves
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) s_tmp[wave] = x;
  __syncthreads();
  uint32_t wbase = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    if ((uint32_t)w < wave) wbase += s_tmp[w];
    total += s_tmp[w];
  }
  __syncthreads();
  return wbase + x - v;
}

}  // namespace tcbee

// tcbee_kernels.hip — HIP kernels (gfx950) of the packet-record path.
//
//   K1 k_parse     one lane per frame: bounds/ethertype/proto/port checks,
//                  fixed-offset header extraction, the 74-B record, the flow
//                  key + hash + flow-table upsert, and ORDER-PRESERVING
//                  compaction of the records (decoupled look-back over dynamic
//                  tiles), records staged in LDS and stored as 16-B vectors.
//                  Restates xdp_hook / tc_hook (tcbee-ebpf/src/probes/xdp.rs:
//                  27-223, tc.rs:28-183) + FLOWS insert (flow_tracker.rs:17-23)
//                  + the drain task's serializer (tcbee/src/handlers/mod.rs:
//                  104-139).
//   K2 k_mark / k_scan_words / k_scan_blocks / k_assign
//                  dense flow ids in first-seen order (the order in which
//                  tcbee-process creates flows, db_writer.rs:51-65): a bitmap
//                  over this batch's accepted frames marks each new flow's first
//                  frame; id = popcount prefix.
//   K3 k_gather    per record: slot -> dense id.
//   k_finalize     counters (counters.rs) + record count + running bases.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "tcbee_gen.h"
#include "tcbee_internal.h"
#include "tcbee_layout.h"

namespace tcbee {

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
constexpr uint32_t kRecountSpins = 4096;  // ~0.1 ms of polling before recounting
// K1's wave priority while a tile's index and header loads are issued (then 0).
// Build-time knob for A/B libraries only (tools/lib_ab.sh, HIPEXTRA=-D...).
#ifndef TCBEE_K1_LOAD_PRIO
#define TCBEE_K1_LOAD_PRIO 2
#endif
constexpr int kK1LoadPrio = TCBEE_K1_LOAD_PRIO;
// K3 (mode 0 k_count, mode 1 k_count_chunk2): the same load-phase priority around
// each iteration's / chunk's record-word loads (0: off)
#ifndef TCBEE_K3_LOAD_PRIO
#define TCBEE_K3_LOAD_PRIO 0
#endif
constexpr int kK3LoadPrio = TCBEE_K3_LOAD_PRIO;
// K1: a probe that misses its plain-load snapshot (a new flow, a slot still BUSY
// with another lane's insert, a stale line) takes flow_upsert's coherent path
// AFTER the tile's records are stored instead of before (the spin on a BUSY slot
// then overlaps the record work; a cold table's first tiles all wait on a few
// inserts). Build-time A/B knob (tools/lib_ab.sh, HIPEXTRA=-D...).
#ifndef TCBEE_K1_DEFER_UPSERT
#define TCBEE_K1_DEFER_UPSERT 0
#endif
constexpr bool kDeferUpsert = TCBEE_K1_DEFER_UPSERT != 0;
[[maybe_unused]] constexpr int kAuxSc1 = 16;  // buffer cache-policy bits: sc1 (agent coherence, bypass L1)
constexpr int kAuxPlain = 0;  // plain: L1/L2 allocating
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16 bytes at arena[a .. a+16), zero past arena_len (a is 16-B aligned).
__device__ __forceinline__ uint4 load_chunk(const uint8_t* arena, uint64_t arena_len, uint64_t a) {
  if (a + 16 <= arena_len) return *reinterpret_cast<const uint4*>(arena + a);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int b = 0; b < 16; ++b)
    if (a + b < arena_len) w[b >> 2] |= (uint32_t)arena[a + b] << (8 * (b & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------------------
// The per-frame hook, split into window loads (so every load of a lane's frames
// is in flight before the first use) and the parse proper.
// Accept set (identical for xdp_hook and tc_hook):
//   caplen >= 14 && ethertype in {0x0800, 0x86DD} &&
//   (v4: caplen >= 54 && ip[9] == 6  |  v6: caplen >= 74 && ip6[6] == 6) &&
//   (filter_port == 0 || sport == filter_port || dport == filter_port)
// ---------------------------------------------------------------------------
// a frame never extends past arena_len
__device__ __forceinline__ uint32_t clamp_caplen(uint64_t off, uint32_t caplen, uint64_t arena_len) {
  if (off >= arena_len) return 0;
  return caplen > arena_len - off ? (uint32_t)(arena_len - off) : caplen;
}

// streaming (non-temporal) access helpers: NT=true keeps the once-touched frame
// stream and record stream from evicting the flow table's lines out of L2
template <bool NT, class T>
__device__ __forceinline__ T ld_stream(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT, class T>
__device__ __forceinline__ void st_stream(T* p, T v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__device__ __forceinline__ void put_chunk(uint32_t (&w)[24], int c, uint4 v) {
  w[4 * c + 0] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
}

// Header window of FPL frames: 16-B aligned chunks 0..4 from off & ~15 (all an
// IPv4 frame needs: s + 54 <= 69 < 80). When every lane's 80 B lie inside the
// arena (the common case) all FPL x 5 loads are issued unconditionally, back to
// back; otherwise each lane loads only the chunks of [off, off+min(len,54)),
// bounds-checked. Chunk 5 (IPv6 tail) is loaded later, for IPv6 frames only.
// Header-chunk load with an explicit cache policy (A/B of how the L2 fetches a
// frame's header line; HPOL 0 = the compiler's plain load). Inline asm is not
// tracked by the compiler's waitcnt insertion: load_windows waits explicitly.
template <int HPOL>
__device__ __forceinline__ u32x4 ld_hdr(const u32x4* p) {
  u32x4 v;
  if constexpr (HPOL == 1) asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (HPOL == 2) asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (HPOL == 3) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (HPOL == 4) asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1 nt" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (HPOL == 5) asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(v) : "v"(p) : "memory");
  else if constexpr (HPOL == 6) asm volatile("global_load_dwordx4 %0, %1, off sc0" : "=v"(v) : "v"(p) : "memory");
  else v = *p;
  return v;
}

template <int FPL, bool NOLOAD, bool NT = false, int HPOL = 0>
__device__ __forceinline__ void load_windows(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                             const uint64_t (&off)[FPL], const uint32_t (&len)[FPL],
                                             uint32_t (&w)[FPL][24]) {
  if (NOLOAD) {
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      // timing ablation: a synthetic IPv4/TCP header (8192 flows) instead of the frame
      const uint32_t fl = (uint32_t)(off[f] >> 6) & 8191u;
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        uint4 v = make_uint4(0x01010101u * c, 0x02020202u * c + fl, 0x03030303u * c, 0x04040404u * c);
        if (c == 0) v.w = 0x00450008u;  // ethertype 0x0800, ver/ihl 0x45
        if (c == 1) v.y = 0x06400000u;  // ttl 64, proto 6
        put_chunk(w[f], c, v);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    return;
  }
  bool inb = true;
#pragma unroll
  for (int f = 0; f < FPL; ++f) inb = inb && (off[f] & ~15ull) + 80 <= arena_len;
#pragma unroll
  for (int f = 0; f < FPL; ++f) put_chunk(w[f], 5, make_uint4(0u, 0u, 0u, 0u));
  if (__all(inb)) {
    // Only the chunks holding frame bytes [12, 52) — ethertype .. TCP checksum,
    // all an IPv4 record uses (the MACs and the urgent pointer are never read):
    // 3 or 4 chunks instead of 5, so a window touches one 64-B sector more
    // often. Lanes whose chunk is not needed are masked off the load.
    u32x4 q[FPL][5];
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      const u32x4* src = reinterpret_cast<const u32x4*>(arena + (off[f] & ~15ull));
      const uint32_t sh = (uint32_t)(off[f] & 15u);
      const uint32_t c_lo = (sh + kFirstUsedByte) >> 4, c_hi = (sh + kV4LastUsedByte) >> 4;
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if ((uint32_t)c >= c_lo && (uint32_t)c <= c_hi)
          v = HPOL ? ld_hdr<HPOL>(src + c) : ld_stream<NT>(src + c);
        q[f][c] = v;
      }
    }
    if constexpr (HPOL != 0) {
#pragma unroll
      for (int f = 0; f < FPL; ++f)
#pragma unroll
        for (int c = 0; c < 5; ++c) asm volatile("s_waitcnt vmcnt(0)" : "+v"(q[f][c]) :: "memory");
    }
    __builtin_amdgcn_s_setprio(0);  // the tile's loads are issued: back to normal priority
#pragma unroll
    for (int f = 0; f < FPL; ++f)
#pragma unroll
      for (int c = 0; c < 5; ++c) put_chunk(w[f], c, make_uint4(q[f][c][0], q[f][c][1], q[f][c][2], q[f][c][3]));
  } else {
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      const uint64_t abase = off[f] & ~15ull;
      const uint32_t need4 = (uint32_t)(off[f] & 15u) + (len[f] < kV4MinLen ? len[f] : kV4MinLen);
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if ((uint32_t)(16 * c) < need4) v = load_chunk(arena, arena_len, abase + 16u * c);
        put_chunk(w[f], c, v);
      }
    }
    __builtin_amdgcn_s_setprio(0);  // (a window at the arena end: bounded loads, done)
  }
}

template <bool NOLOAD = false>
__device__ __forceinline__ bool parse_window(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                             uint64_t off, uint32_t caplen, uint64_t ts,
                                             uint32_t filter_port, uint32_t (&w)[24],
                                             uint32_t (&R)[19], uint64_t (&K)[5]) {
  if (caplen < kEthHdrLen) return false;  // xdp.rs:37-39
  const uint64_t abase = off & ~15ull;
  const uint32_t s = NOLOAD ? 0u : (uint32_t)(off & 15u);
  if (!NOLOAD) {
    // ethertype straight from the raw window: bytes s+12, s+13 (dwords 3..7)
    const uint32_t e = s + 12, t3 = (e >> 2) - 3, m1 = 0u - (t3 & 1u), m2 = 0u - ((t3 >> 1) & 1u);
    const uint32_t x0 = (w[3] & ~m1) | (w[4] & m1), x1 = (w[4] & ~m1) | (w[5] & m1);
    const uint32_t x2 = (w[5] & ~m1) | (w[6] & m1), x3 = (w[6] & ~m1) | (w[7] & m1);
    const uint32_t lo = (x0 & ~m2) | (x2 & m2), hi = (x1 & ~m2) | (x3 & m2);
    const uint32_t et = bswap16(align_bytes(hi, lo, e & 3u) & 0xFFFFu);
    const uint32_t need6 = s + (caplen < kV6LastUsedByte + 1 ? caplen : kV6LastUsedByte + 1);
    if (et == kEthertypeIPv6) {
      // IPv6 tail: the chunks holding frame bytes [52, 72) (TCP header at 54),
      // which the IPv4 window never loads
#pragma unroll
      for (int c = 3; c < 6; ++c) {
        if ((uint32_t)(16 * c) < need6 && (uint32_t)(16 * c + 16) > s + kV4LastUsedByte + 1)
          put_chunk(w, c, load_chunk(arena, arena_len, abase + 16u * c));
      }
    }
  }
  // Normalise so that u[j] holds frame bytes [4j, 4j+4): shift by s bytes
  // (dword shift by s>>2 via two select stages, then a byte align by s&3).
  // (bit masks, not ?: — hipcc turns a select cascade over an array into a
  //  runtime-indexed scratch copy)
  const uint32_t q = s >> 2, r = s & 3u;
  const uint32_t m1 = 0u - (q & 1u), m2 = 0u - ((q >> 1) & 1u);
  uint32_t t[23];
#pragma unroll
  for (int j = 0; j < 23; ++j) t[j] = (w[j] & ~m1) | (w[j + 1] & m1);
  uint32_t v2[21];
#pragma unroll
  for (int j = 0; j < 21; ++j) v2[j] = (t[j] & ~m2) | (t[j + 2] & m2);
  uint32_t u[19];
#pragma unroll
  for (int j = 0; j < 19; ++j) u[j] = align_bytes(v2[j + 1], v2[j], r);

  const uint32_t ethertype = bswap16(u[3] & 0xFFFFu);  // bytes 12..13, xdp.rs:49
  const bool v4 = ethertype == kEthertypeIPv4;
  const bool v6 = ethertype == kEthertypeIPv6;
  if (!v4 && !v6) return false;                               // xdp.rs:52
  const uint32_t proto = v4 ? (u[5] >> 24) : (u[5] & 0xFFu);  // ip[9] @23 | ip6[6] @20
  if (proto != kTcpProtocol) return false;                    // xdp.rs:73, :147
  if (caplen < (v4 ? kV4MinLen : kV6MinLen)) return false;    // xdp.rs:60,78 / :134,152

  // TCP header at frame byte 34 (v4) or 54 (v6): both are 2 mod 4.
  uint32_t T[5];
#pragma unroll
  for (int j = 0; j < 5; ++j) T[j] = v4 ? u[8 + j] : u[13 + j];
  const uint32_t sport = bswap16(T[0] >> 16);                 // tcp[0..1]
  const uint32_t dport = bswap16(T[1] & 0xFFFFu);             // tcp[2..3]
  if (filter_port != 0 && sport != filter_port && dport != filter_port)
    return false;                                              // xdp.rs:89-92
  const uint32_t seq = bswap32(align_bytes(T[2], T[1], 2));   // tcp[4..7]
  const uint32_t ack = bswap32(align_bytes(T[3], T[2], 2));   // tcp[8..11]
  const uint32_t flagbits = T[3] >> 16;                       // tcp[12..13]
  const uint32_t window = bswap16(T[4] & 0xFFFFu);            // tcp[14..15]
  const uint32_t check = bswap16(T[4] >> 16);                 // tcp[16..17]
  // `tcp_hdr.urg().to_be() == 1` (xdp.rs:105-110): bit -> u16 0/1 -> to_be()
  // (0 or 0x0100 on little endian) == 1  => always false. Kept literal.
  auto flag = [&](int index) -> uint32_t {
    const uint32_t bit = (flagbits >> index) & 1u;  // bindgen bit `index` of bytes 12..13
    return bswap16(bit) == 1u ? 1u : 0u;
  };
  const uint32_t f_urg = flag(13), f_ack = flag(12), f_psh = flag(11), f_rst = flag(10),
                 f_syn = flag(9), f_fin = flag(8);

  // addresses
  const uint32_t sa4 = align_bytes(u[7], u[6], 2);  // wire bytes 26..29 as LE word
  const uint32_t da4 = align_bytes(u[8], u[7], 2);  // 30..33
  uint32_t sa6[4], da6[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sa6[j] = align_bytes(u[6 + j], u[5 + j], 2);    // 22..37
    da6[j] = align_bytes(u[10 + j], u[9 + j], 2);   // 38..53
  }

  // record (tcp_packet_trace bincode + marker), xdp.rs:94-112 / :168-186
  R[0] = (uint32_t)ts;
  R[1] = (uint32_t)(ts >> 32);
  R[2] = v4 ? bswap32(sa4) : 0u;  // saddr.to_be()
  R[3] = v4 ? bswap32(da4) : 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    R[4 + j] = v6 ? sa6[j] : 0u;
    R[8 + j] = v6 ? da6[j] : 0u;
  }
  R[12] = sport | (dport << 16);
  R[13] = seq;
  R[14] = ack;
  R[15] = window | (f_urg << 16) | (f_ack << 24);
  R[16] = f_psh | (f_rst << 8) | (f_syn << 16) | (f_fin << 24);
  R[17] = check | 0xFFFF0000u;  // checksum + first half of FF FF FF FF
  R[18] = 0x0000FFFFu;

  // IpTuple key (xdp.rs:116-127 / :189-195): v4 address = 12 zero bytes + wire bytes
  if (v4) {
    K[0] = 0;
    K[1] = (uint64_t)sa4 << 32;
    K[2] = 0;
    K[3] = (uint64_t)da4 << 32;
  } else {
    K[0] = (uint64_t)sa6[0] | ((uint64_t)sa6[1] << 32);
    K[1] = (uint64_t)sa6[2] | ((uint64_t)sa6[3] << 32);
    K[2] = (uint64_t)da6[0] | ((uint64_t)da6[1] << 32);
    K[3] = (uint64_t)da6[2] | ((uint64_t)da6[3] << 32);
  }
  K[4] = (uint64_t)sport | ((uint64_t)dport << 16) | ((uint64_t)kTcpProtocol << 32);
  return true;
}

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
__device__ uint32_t flow_upsert_compact(const FlowTable& T, const uint64_t (&K)[5], uint64_t h,
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
__device__ uint32_t flow_upsert_wide(const FlowTable& T, const uint64_t (&K)[5], uint64_t h,
                                     BatchState* batch, uint64_t* new_list, PersistState* persist,
                                     uint64_t fbase, uint32_t& fs_seen, uint32_t& claim,
                                     uint32_t claim_mark) {
  const uint32_t tag = hash_tag32(h);
  uint64_t s = h & T.wide_mask;
  for (uint64_t probe = 0; probe <= T.wide_mask; ++probe) {
    uint64_t* m = T.wide + s * 8;
    uint64_t cur = ld_agent(m);
    if (cur == kTagEmpty) {
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

// ---------------------------------------------------------------------------
// Decoupled look-back (one wave). Status word: bits 63:62 = 1 aggregate,
// 2 inclusive prefix; bits 61:0 = value. Words are single 8-B agent-scope
// stores polled by agent-scope loads (the data IS the flag).
// ---------------------------------------------------------------------------
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagInc = 2ull << 62, kValMask = (1ull << 62) - 1;

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ void lookback_publish(uint64_t* status, uint64_t tile, uint64_t count) {
  st_agent(status + tile, (tile == 0 ? kFlagInc : kFlagAgg) | count);
}

template <int TILE>
__device__ uint32_t tile_accept_count(const ParseArgs& a, uint64_t tile);

// Resolves this tile's exclusive prefix (one wave) and publishes its inclusive
// prefix. Tiles are blockIdx.x: no dispatch order is assumed. A predecessor
// whose word stays unpublished for kRecountSpins polls (not yet dispatched, or
// slow) has its aggregate recounted from the input by this wave, so the walk
// always terminates; results never depend on which block publishes first.
template <int TILE>
__device__ uint64_t lookback_resolve(const ParseArgs& a, uint64_t tile, uint64_t count,
                                    bool withhold) {
  const uint32_t lane = __lane_id();
  if (tile == 0) return 0;
  uint64_t* status = a.tile_status;
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  for (;;) {
    const int64_t idx = base - (int64_t)lane;
    uint64_t v = idx >= 0 ? ld_agent(status + idx) : kFlagInc;
    uint32_t spins = 0;
    for (;;) {
      const uint64_t inv = __ballot((v >> 62) == 0);
      if (!inv) break;
      // only the invalid lanes nearer than the nearest inclusive prefix matter
      const uint64_t inc = __ballot((v >> 62) == 2);
      const uint64_t need = inc ? (inv & ((inc & (~inc + 1)) - 1)) : inv;
      if (!need) break;
      if (++spins > kRecountSpins) {
        const uint32_t j = (uint32_t)__ffsll((unsigned long long)need) - 1;
        const uint32_t cnt = tile_accept_count<TILE>(a, (uint64_t)(base - (int64_t)j));
        if (lane == j) v = kFlagAgg | cnt;
        spins = 0;
        continue;
      }
      __builtin_amdgcn_s_sleep(1);
      if ((v >> 62) == 0) v = ld_agent(status + idx);
    }
    const uint64_t inc = __ballot((v >> 62) == 2);
    if (inc) {
      const uint32_t first = (uint32_t)__ffsll((unsigned long long)inc) - 1;
      excl += wave_sum64(lane <= first ? (v & kValMask) : 0ull);
      break;
    }
    excl += wave_sum64(v & kValMask);
    base -= 64;
  }
  if (lane == 0 && !withhold) st_agent(status + tile, kFlagInc | (excl + count));
  return excl;
}

// record -> LDS at byte offset `bo` (even)
__device__ __forceinline__ void lds_put_record(uint32_t* srec, uint32_t bo, const uint32_t (&R)[19]) {
  uint16_t* s16 = reinterpret_cast<uint16_t*>(srec);
  if ((bo & 3u) == 0) {
    const uint32_t d = bo >> 2;
#pragma unroll
    for (int j = 0; j < 18; ++j) srec[d + j] = R[j];
    s16[(bo + 72) >> 1] = (uint16_t)R[18];
  } else {
    s16[bo >> 1] = (uint16_t)R[0];
    const uint32_t d = (bo + 2) >> 2;
#pragma unroll
    for (int j = 0; j < 18; ++j) srec[d + j] = (R[j] >> 16) | (R[j + 1] << 16);
  }
}

__device__ __forceinline__ bool parse_frame(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                            uint64_t off, uint32_t caplen, uint64_t ts,
                                            uint32_t filter_port, uint32_t (&R)[19],
                                            uint64_t (&K)[5]) {
  const uint64_t o[1] = {off};
  const uint32_t l[1] = {clamp_caplen(off, caplen, arena_len)};
  uint32_t w[1][24];
  load_windows<1, false>(arena, arena_len, o, l, w);
  return parse_window(arena, arena_len, off, l[0], ts, filter_port, w[0], R, K);
}

// Accepted frames of one tile, recomputed from the input by one wave (the
// look-back's fallback when a predecessor has not published).
template <int TILE>
__device__ uint32_t tile_accept_count(const ParseArgs& a, uint64_t tile) {
  const uint32_t lane = __lane_id();
  uint32_t cnt = 0;
  for (int k = 0; k < TILE / 64; ++k) {
    const uint64_t i = tile * (uint64_t)TILE + (uint64_t)k * 64 + lane;
    bool ok = false;
    if (i < a.n) {
      uint32_t R[19];
      uint64_t K[5];
      ok = parse_frame(a.arena, a.arena_len, a.offset[i], a.caplen[i], 0, a.filter_port, R, K);
    }
    cnt += (uint32_t)__popcll(__ballot(ok));
  }
  return cnt;
}

// Copies staged records [G0, G1) (global byte range; sbuf byte 0 = global byte G0)
// to out: 16-B stores for whole chunks, 2-B stores for the partial chunks at the
// ends (bytes there belong to neighbouring groups). Threads t0, t0+step, ...
template <bool NT = false>
__device__ __forceinline__ void copy_out(uint8_t* __restrict__ out, uint64_t G0, uint64_t G1,
                                         const uint32_t* sbuf, uint32_t t0, uint32_t step) {
  const uint64_t A = G0 & ~15ull;
  const uint32_t head = (uint32_t)(G0 & 15u);
  const uint32_t nchunks = (uint32_t)((G1 - A + 15) >> 4);
  const uint16_t* s16 = reinterpret_cast<const uint16_t*>(sbuf);
  for (uint32_t c = t0; c < nchunks; c += step) {
    const uint64_t g = A + 16ull * c;
    if (g >= G0 && g + 16 <= G1) {
      const uint32_t sb = 16u * c - head;
      const uint32_t d0 = sb >> 2;
      uint4 o;
      if ((sb & 3u) == 0) {
        o = make_uint4(sbuf[d0], sbuf[d0 + 1], sbuf[d0 + 2], sbuf[d0 + 3]);
      } else {
        const uint32_t x0 = sbuf[d0], x1 = sbuf[d0 + 1], x2 = sbuf[d0 + 2], x3 = sbuf[d0 + 3],
                       x4 = sbuf[d0 + 4];
        o = make_uint4((x0 >> 16) | (x1 << 16), (x1 >> 16) | (x2 << 16), (x2 >> 16) | (x3 << 16),
                       (x3 >> 16) | (x4 << 16));
      }
      u32x4 ov;
      ov[0] = o.x; ov[1] = o.y; ov[2] = o.z; ov[3] = o.w;
      st_stream<NT>(reinterpret_cast<u32x4*>(out + g), ov);
    } else {
      const uint64_t lo = g > G0 ? g : G0;
      const uint64_t hi = (g + 16) < G1 ? (g + 16) : G1;
      for (uint64_t b = lo; b < hi; b += 2)
        *reinterpret_cast<uint16_t*>(out + b) = s16[(b - G0) >> 1];
    }
  }
}

__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// ---------------------------------------------------------------------------
// K1
// ---------------------------------------------------------------------------
// ABL: timing-only ablation bits (0 in every product launch; see tools/ablate.py)
//   1 no look-back, 2 no record stores, 4 no header loads, 8 no index loads,
//   16 no side outputs, 32 no first-seen competition (atomicMin), 64 IPv4-form
//   probes load a line of the table's first 16 MiB instead of their slot and take a
//   hash-derived claim (what a probe served from a table small enough for the
//   Infinity Cache would cost)
// STAGE 0: the whole tile's records staged in LDS, stored by the block after the
// look-back; STAGE 1: each wave stages and stores its own 64-record group per
// round (its records are contiguous in the output), 4.7 KB of LDS per wave.
// OCC: minimum waves per SIMD requested from the register allocator (0: default)
template <int FPL, bool FLOWS, int PROBE_AUX, int ABL = 0, int STAGE = 0, bool NT = false, int OCC = 0,
          int HPOL = 0, int BLK = kBlock>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(OCC ? OCC : 1, OCC ? 8 : 8)))
void k_parse(ParseArgs a) {
  constexpr int TILE = BLK * FPL;
  constexpr int NW = BLK / 64;  // waves per tile
  constexpr int WBUF_DW = (64 * kRecBytes + 32) / 4;
  constexpr int SREC_DW = STAGE ? NW * WBUF_DW : (TILE * kRecBytes + 32) / 4;
  __shared__ __attribute__((aligned(16))) uint32_t s_rec[SREC_DW];
  __shared__ uint32_t s_wcnt[FPL][NW];
  __shared__ uint64_t s_excl;

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t tile = blockIdx.x;
  const uint64_t i0 = tile * (uint64_t)TILE;
  // a starting wave issues its index and header loads ahead of resident waves'
  // parse / record work (priority dropped once they are in flight, load_windows)
  __builtin_amdgcn_s_setprio(kK1LoadPrio);
  // flows claimed before this batch (claims below it have first records in earlier
  // batches: their frames never compete for first_seen)
  const uint64_t fbase = FLOWS ? a.persist->flow_count : 0;

  uint32_t R[FPL][19];
  bool acc[FPL];
  uint32_t rank[FPL], slot[FPL], hsh[FPL], clen[FPL], claim[FPL];
  uint32_t fs_seen[FPL];
  uint64_t K[FPL][5];

  // phase A: index loads of all the lane's frames, then all their header-window
  // loads (in flight together), then the parse
  uint64_t offv[FPL], tsv[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    const uint64_t i = i0 + (uint64_t)f * BLK + tid;
    acc[f] = false;
    slot[f] = 0xFFFFFFFFu;
    claim[f] = 0xFFFFFFFFu;
    hsh[f] = 0;
    fs_seen[f] = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < 5; ++j) K[f][j] = 0;
    const bool in = i < a.n;
    const uint64_t ic = in ? i : a.n - 1;  // loads stay unconditional (no branch per frame)
    const uint64_t o = (ABL & 8) ? ic * 64 : ld_stream<NT>(a.offset + ic);
    const uint32_t l = (ABL & 8) ? 64u : ld_stream<NT>(a.caplen + ic);
    const uint64_t t = (ABL & 8) ? ic : ld_stream<NT>(a.ts + ic);
    offv[f] = in ? o : 0;
    clen[f] = in ? l : 0;
    tsv[f] = t;
  }
  uint32_t lenc[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) lenc[f] = clamp_caplen(offv[f], clen[f], a.arena_len);
  {
    uint32_t W[FPL][24];
    load_windows<FPL, (ABL & 4) != 0, NT, HPOL>(a.arena, a.arena_len, offv, lenc, W);
#pragma unroll
    for (int f = 0; f < FPL; ++f)
      acc[f] = parse_window<(ABL & 4) != 0>(a.arena, a.arena_len, offv[f], lenc[f], tsv[f],
                                            a.filter_port, W[f], R[f], K[f]);
  }
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    const uint64_t b = __ballot(acc[f]);
    if (lane == 0) s_wcnt[f][wave] = (uint32_t)__popcll(b);
    rank[f] = (uint32_t)__popcll(b & lanemask_lt());
  }
  __syncthreads();
  uint32_t running = 0;
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t c = s_wcnt[f][w];
      if ((uint32_t)w == wave) rank[f] += running;
      running += c;
    }
  }
  const uint32_t total = running;
  // publish this tile's aggregate as early as possible (successors look back on it)
  // (a.withhold_every: test hook, tiles t % k == k-1 never publish, forcing their
  //  successors down the recount path)
  const bool withhold = a.withhold_every && (tile % a.withhold_every) == a.withhold_every - 1;
  if (!(ABL & 1) && !withhold && tid == 0) lookback_publish(a.tile_status, tile, total);

  // probe results per frame group (lane-private until publish_probe shares a
  // wave-uniform key's leader result with its wave)
  uint32_t psl[FPL], pcl[FPL], pfs[FPL];
  bool pend[FPL], uni[FPL], want[FPL];
  uint32_t leader[FPL];
  uint64_t h[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) pend[f] = uni[f] = want[f] = false;
  auto publish_probe = [&](int f) {
    if (uni[f]) {
      slot[f] = __shfl(psl[f], leader[f]);
      claim[f] = __shfl(pcl[f], leader[f]);
      fs_seen[f] = __shfl(pfs[f], leader[f]);
    } else if (acc[f]) {
      slot[f] = psl[f];
      claim[f] = psl[f] == 0xFFFFFFFFu ? 0xFFFFFFFFu : pcl[f];
      fs_seen[f] = pfs[f];
    }
  };
  if (FLOWS) {
    // phase B: hash, then issue the first probe's loads of every frame: an IPv4-form
    // key's 16-B compact slot + its fs32 (one line), any other key's 64-B wide slot
    u32x4 Q[FPL][4];
    uint32_t FS[FPL], S0[FPL];
    bool v4k[FPL];
    // num_records = the slot lines' bytes (< 2^32: max_flows <= kMaxTableFlows; the
    // bits are read as unsigned), and the wide slots' (<= 2^31 bytes: see the ABI)
    const __amdgpu_buffer_rsrc_t sl_rs = __builtin_amdgcn_make_buffer_rsrc(
        a.tab.slots, 0, (int)(uint32_t)(a.tab.nlines * 64u), 0x00020000);
    const __amdgpu_buffer_rsrc_t wd_rs = __builtin_amdgcn_make_buffer_rsrc(
        a.tab.wide, 0, (int)(uint32_t)((a.tab.wide_mask + 1) * 64u), 0x00020000);
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      const uint64_t am = __ballot(acc[f]);
      leader[f] = am ? (uint32_t)__ffsll((unsigned long long)am) - 1 : 0u;
      bool same = true;
#pragma unroll
      for (int j = 0; j < 5; ++j) same = same && (!acc[f] || K[f][j] == __shfl(K[f][j], leader[f]));
      // wave-uniform key (one flow in the whole wave): only the leader probes
      uni[f] = am != 0 && __all(same);
      h[f] = flow_hash64(K[f][0], K[f][1], K[f][2], K[f][3], K[f][4]);
      if (acc[f]) hsh[f] = fold32(h[f]);
      want[f] = uni[f] ? lane == leader[f] : acc[f];
      v4k[f] = key_is_v4form(K[f]);
      if (want[f]) {
        // Plain (cacheable) loads are exact here: a claimer stores everything a
        // reader compares (drained) before the word that publishes the slot, in the
        // same line; a stale snapshot shows EMPTY/BUSY or a mismatch, and every such
        // miss falls through to flow_upsert's coherent path.
        if (v4k[f]) {
          S0[f] = home_slot(h[f], a.tab.nlines);
          uint32_t l = slot_line(S0[f]), pos = S0[f] - l * kSlotsPerLine;
          // probe window of the ceiling ablation: 64 = 16 MiB (Infinity-Cache resident),
          // +128 = 2 MiB, +256 = 4 MiB, +384 = 512 KiB (L2-sized first levels)
          constexpr uint32_t kAblWin = (ABL & 384) == 128 ? (2u << 20) : (ABL & 384) == 256 ? (4u << 20)
                                     : (ABL & 384) == 384 ? (512u << 10) : (16u << 20);
          if (ABL & 64) l = (uint32_t)(h[f] >> 40) & (kAblWin / 64u - 1u);
          Q[f][0] = __builtin_amdgcn_raw_buffer_load_b128(sl_rs, l * 64u + 16u * pos, 0, PROBE_AUX);
          // (the slot and its fs32 share one 64-B half-line: the two halves of a
          //  128-B line can be of different ages in L1/L2 — a fresh published slot
          //  beside a stale fs32 lost first_seen values when fs32 sat in the other half)
          FS[f] = __builtin_amdgcn_raw_buffer_load_b32(sl_rs, l * 64u + 48u + 4u * pos, 0, PROBE_AUX);
        } else {
          S0[f] = (uint32_t)(h[f] & a.tab.wide_mask);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            Q[f][j] = __builtin_amdgcn_raw_buffer_load_b128(wd_rs, S0[f] * 64u + 16u * j, 0, PROBE_AUX);
        }
      }
    }
    // phase C: resolve; a miss (new flow, busy slot, a stale snapshot) takes the full
    // upsert. Walk on with plain loads while the slots hold OTHER flows (published,
    // another key): within a batch a slot only goes EMPTY -> BUSY -> published, so a
    // published foreign slot seen in any snapshot is foreign for good; EMPTY/BUSY may
    // be stale and end the walk. A wide slot whose tag equals ours but whose key
    // differs goes to the coherent path (it may be a stale snapshot of our flow).
    const uint32_t nslots = (uint32_t)a.tab.nlines * kSlotsPerLine;
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      uint32_t sl = 0xFFFFFFFFu, cl = 0xFFFFFFFFu, fs = 0xFFFFFFFFu;
      if (want[f]) {
        bool slow = true;
        if (v4k[f]) {
          uint64_t w0k, kl;
          key_slot_words(K[f], h[f], w0k, kl);
          uint32_t s = S0[f];
          uint64_t w0 = (uint64_t)Q[f][0][0] | ((uint64_t)Q[f][0][1] << 32);
          uint64_t w1 = (uint64_t)Q[f][0][2] | ((uint64_t)Q[f][0][3] << 32);
          uint32_t fsv = FS[f];
          if (ABL & 64) {
            asm volatile("" ::"v"(Q[f][0][0]), "v"(fsv));
            sl = s;
            cl = (uint32_t)(h[f] % a.tab.max_claims);
            fs = 0xFFFFFFFFu;
            slow = false;
            w1 = 0;  // skip the walk
          }
          for (uint32_t step = 0; !(ABL & 64); ++step) {
            if (w1 <= kKindBusy) break;
            if ((w1 & ~kClaimBits) == kl && w0 == w0k) {  // the whole key: a hit
              sl = s;
              cl = (uint32_t)((w1 & kClaimBits) >> 32);
              fs = fsv;
              slow = false;
              break;
            }
            if (step >= a.plain_walk) break;
            s = s + 1 == nslots ? 0u : s + 1;
            const uint32_t l = slot_line(s), pos = s - l * kSlotsPerLine;
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(sl_rs, l * 64u + 16u * pos, 0, PROBE_AUX);
            fsv = __builtin_amdgcn_raw_buffer_load_b32(sl_rs, l * 64u + 48u + 4u * pos, 0, PROBE_AUX);
            w0 = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
            w1 = (uint64_t)q[2] | ((uint64_t)q[3] << 32);
          }
        } else {
          const uint32_t mytag = hash_tag32(h[f]);
          uint32_t s = S0[f];
          uint64_t V[7];
#pragma unroll
          for (int j = 0; j < 7; ++j) {
            const u32x4 v = Q[f][j >> 1];
            V[j] = (j & 1) ? ((uint64_t)v[2] | ((uint64_t)v[3] << 32)) : ((uint64_t)v[0] | ((uint64_t)v[1] << 32));
          }
          for (uint32_t step = 0;; ++step) {
            if (V[0] < 2) break;
            if ((uint32_t)V[0] == mytag) {
              if (V[1] == K[f][0] && V[2] == K[f][1] && V[3] == K[f][2] && V[4] == K[f][3] &&
                  V[5] == K[f][4] && (V[0] >> 32) != 0xFFFFFFFFull) {
                sl = s | kWideSlot;
                cl = (uint32_t)(V[0] >> 32);
                fs = (uint32_t)V[6];
                slow = false;
              }
              break;
            }
            if (step >= a.plain_walk) break;
            s = (uint32_t)((s + 1) & a.tab.wide_mask);
            u32x4 q[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = __builtin_amdgcn_raw_buffer_load_b128(wd_rs, s * 64u + 16u * j, 0, PROBE_AUX);
#pragma unroll
            for (int j = 0; j < 7; ++j) {
              const u32x4 v = q[j >> 1];
              V[j] = (j & 1) ? ((uint64_t)v[2] | ((uint64_t)v[3] << 32)) : ((uint64_t)v[0] | ((uint64_t)v[1] << 32));
            }
          }
        }
        if (slow && !kDeferUpsert)
          sl = flow_upsert(a.tab, K[f], h[f], a.batch, a.new_list, a.persist, fbase, fs, cl,
                           kFs32Flag | (uint32_t)(i0 + (uint64_t)f * BLK + tid));
        pend[f] = slow && kDeferUpsert;
      }
      psl[f] = sl;
      pcl[f] = cl;
      pfs[f] = fs;
      if (!kDeferUpsert) publish_probe(f);
    }
  }
  if (!(ABL & 2)) {
    if (STAGE == 0) {
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        if (acc[f]) lds_put_record(s_rec, rank[f] * kRecBytes, R[f]);
    }
  } else {
#pragma unroll
    for (int f = 0; f < FPL; ++f)
      if (acc[f]) asm volatile("" ::"v"(R[f][0]), "v"(R[f][5]), "v"(R[f][13]), "v"(R[f][17]));
  }

  // (wave 0 resolving the look-back before its own probes instead — its inclusive
  //  prefix published a probe phase earlier — was 22 % slower, round 3)
  if (wave == 0) {
    const uint64_t excl =
        (ABL & 1) ? tile * (uint64_t)TILE : lookback_resolve<TILE>(a, tile, total, withhold);
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const uint64_t excl = s_excl;
  if (tid == 0 && tile == a.ntiles - 1) a.batch->n_acc = excl + total;

  // ---- records: LDS -> HBM, 16-B stores, partial chunks as 2-B stores ----
  if (!(ABL & 2)) {
    if (STAGE == 0) {
      const uint64_t wr_lo = excl < a.out_cap ? excl : a.out_cap;
      const uint64_t wr_hi = (excl + total) < a.out_cap ? (excl + total) : a.out_cap;
      if (wr_hi > wr_lo)
        copy_out<NT>(a.out_rec, wr_lo * kRecBytes, wr_hi * kRecBytes, s_rec, tid, BLK);
    } else {
      uint32_t* wbuf = s_rec + wave * WBUF_DW;
#pragma unroll
      for (int f = 0; f < FPL; ++f) {
        const uint64_t b = __ballot(acc[f]);
        const uint32_t lrank = (uint32_t)__popcll(b & lanemask_lt());
        const uint64_t g0 = excl + rank[f] - lrank;  // this wave's group start
        const uint64_t g1 = g0 + (uint64_t)__popcll(b);
        const uint64_t lo = g0 < a.out_cap ? g0 : a.out_cap;
        const uint64_t hi = g1 < a.out_cap ? g1 : a.out_cap;
        if (hi > lo) {
          if (acc[f]) lds_put_record(wbuf, lrank * kRecBytes, R[f]);
          wave_lds_sync();
          copy_out<NT>(a.out_rec, lo * kRecBytes, hi * kRecBytes, wbuf, lane, 64);
          wave_lds_sync();
        }
      }
    }
  }

  if (FLOWS && kDeferUpsert) {
    // the probes whose snapshot missed, after the records are out
#pragma unroll
    for (int f = 0; f < FPL; ++f) {
      if (want[f] && pend[f])
        psl[f] = flow_upsert(a.tab, K[f], h[f], a.batch, a.new_list, a.persist, fbase, pfs[f],
                             pcl[f], kFs32Flag | (uint32_t)(i0 + (uint64_t)f * BLK + tid));
      publish_probe(f);
    }
  }

  // ---- per-record side outputs; first_seen = min accepted index ----
  // (pkts/bytes are NOT counted here: per-record memory-side atomics cost more
  //  than the whole parse; k_count histograms them by dense id in LDS.)
  uint32_t prev_s0 = 0xFFFFFFFFu;  // slot of the wave's last all-one-slot new-flow group
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    const uint64_t p = excl + rank[f];
    if (acc[f] && !(ABL & 16)) {
      if (a.out_hash && p < a.out_cap) st_stream<NT>(a.out_hash + p, hsh[f]);
      // record -> frame map (flow-hash shards of traces with rejected frames)
      if (a.out_frame && p < a.out_cap) st_stream<NT>(a.out_frame + p, (uint32_t)(i0 + (uint64_t)f * BLK + tid));
      if (FLOWS) {
        if (a.pack_bits) {
          // (claim, caplen) in one word; a caplen that does not fit saturates the
          // field and is stored in full beside it (K3 reads it only then)
          const uint32_t lmax = 0xFFFFFFFFu >> a.pack_bits;
          const uint32_t lq = clen[f] < lmax ? clen[f] : lmax;
          st_stream<NT>(a.acc_flow + p, claim[f] == 0xFFFFFFFFu ? 0xFFFFFFFFu
                                                                : claim[f] | (lq << a.pack_bits));
          if (lq == lmax) a.acc_len[p] = clen[f];
        } else {
          st_stream<NT>(a.acc_flow + p, claim[f]);
          st_stream<NT>(a.acc_len + p, clen[f]);
        }
      }
    }
    if (FLOWS && !(ABL & 32)) {
      // first_seen competition: only flows new in this batch (claim >= fbase)
      const bool mine = acc[f] && slot[f] != 0xFFFFFFFFu && claim[f] >= fbase;
      const uint64_t am = __ballot(mine);
      if (am) {
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)am) - 1;
        const uint32_t s0 = __shfl(slot[f], leader);
        const uint32_t p32 = (uint32_t)p;
        const uint32_t frame_i = (uint32_t)(i0 + (uint64_t)f * BLK + tid);
        if (__all(!mine || slot[f] == s0)) {
          // leader = lowest rank of the wave = its smallest accepted index; when the
          // wave's previous frame group was all this slot too, its earlier leader
          // competes for both (a hot new flow: one add per wave, not per group)
          const bool first = s0 != prev_s0;
          prev_s0 = s0;
          if (first && lane == leader && fs_needs_min(fs_seen[f], frame_i, p32))
            atomicMin(slot_fs_any(a.tab, s0), p32);
        } else if (mine && fs_needs_min(fs_seen[f], frame_i, p32)) {
          atomicMin(slot_fs_any(a.tab, slot[f]), p32);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// flow table init: tags/keys/ids 0, first_seen ~0, counters 0
// ---------------------------------------------------------------------------
// An empty slot unit: w0/w1 zero (empty); fs32 all ones, so a frame that reads a
// snapshot of the unit older than its slot's claim mark competes for first_seen
// (safe) instead of skipping (0 would lose the first record). Wide slots: tag word
// 0 and fs word ~0, as rounds 1-2.
__device__ __forceinline__ void empty_units(const FlowTable& t, uint64_t t0, uint64_t stride) {
  uint4* L = reinterpret_cast<uint4*>(t.slots);
  for (uint64_t q = t0; q < 4 * t.nlines; q += stride)
    L[q] = (q & 3) == 3 ? make_uint4(~0u, ~0u, ~0u, 0u) : make_uint4(0u, 0u, 0u, 0u);
  if (*t.wide_used)  // (cleared at context creation; swept only once used)
    for (uint64_t w = t0; w <= t.wide_mask; w += stride) {
      t.wide[8 * w] = 0;
      t.wide[8 * w + 6] = ~0ull;
    }
}

__global__ void k_table_init(FlowTable t) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  empty_units(t, t0, stride);
  for (uint64_t i = t0; i < 2 * t.max_claims; i += stride) t.cnt[i] = 0;
}

// ---------------------------------------------------------------------------
// per-batch preparation in one launch (instead of 3-5 memsets + table init)
// ---------------------------------------------------------------------------
__global__ void k_prep(PrepArgs p) {
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if (t0 < sizeof(BatchState) / 8) reinterpret_cast<uint64_t*>(p.batch)[t0] = 0;
  for (uint64_t i = t0; i < p.ntiles; i += stride) p.tile_status[i] = 0;
  // (the first-seen bitmap is not swept here: it is all zero between batches —
  //  K3 clears the words the rank step set)
  if (p.reset) {
    if (t0 < sizeof(PersistState) / 8) reinterpret_cast<uint64_t*>(p.persist)[t0] = 0;
    // empty slot lines (16 B of slot lines per 16-B store); entries need nothing
    // (claims restart at 0), and the by-id counters are zeroed by K2 as ids are
    // handed out (the previous batch's K3 may still be adding to them on another
    // stream)
    // (wide slots only once a non-IPv4 key was claimed)
    empty_units(p.tab, t0, stride);
  }
  if (p.zero_free_counters) {
    // (ordered after the previous batch's K3 by the caller; <= kFuseRankMax ids)
    const uint64_t fbase = p.reset ? 0 : p.persist->flow_count;
    for (uint64_t i = 2 * fbase + t0; i < 2 * p.tab.max_claims; i += stride) p.tab.cnt[i] = 0;
  }
}

// ---------------------------------------------------------------------------
// K2: ranks of this batch's new flows by first_seen
// ---------------------------------------------------------------------------
// Small batches (nwords <= kRankSmallWords): rank in ONE block.
//  - n_new <= kRankSortMax: rank = number of this batch's new flows seen earlier,
//    counted over the first_seen values staged in LDS (no bitmap pass at all);
//  - otherwise mark + scan + assign: the bitmap is scanned by 16 waves, each over
//    a contiguous word range read 64 consecutive words at a time (coalesced).
constexpr uint32_t kRankSortMax = 2048;

// new flows this batch that got a claim (claims past max_claims were refused:
// their slots are dead, nothing was written to new_list for them)
__device__ __forceinline__ uint64_t rank_new(const RankArgs& r, uint64_t fbase) {
  const uint64_t n = r.batch->n_new;
  const uint64_t room = r.tab.max_claims > fbase ? r.tab.max_claims - fbase : 0;
  return n < room ? n : room;
}
// the batch-local first record index of new flow j (its slot's fs32)
__device__ __forceinline__ uint32_t new_flow_fs(const RankArgs& r, uint64_t j) {
  return *slot_fs_any(r.tab, (uint32_t)r.new_list[j]);
}

// End of a single-block rank: the batch is classified — advance the context's
// record base and flow count (K1 of the next batch reads them; K3 no longer does)
__device__ __forceinline__ void rank_done(const RankArgs& r, uint32_t tid, uint64_t base,
                                          uint64_t fbase, uint64_t n_new) {
  __syncthreads();  // every thread has read the old base / fbase / n_new
  if (tid == 0) {
    r.batch->n_new = n_new;  // the claimed ones (readers after K2 see the clamp)
    if (r.update_persist) {
      r.persist->rec_base = base + r.batch->n_acc;
      r.persist->flow_count = fbase + n_new;
    }
  }
}

__global__ __launch_bounds__(1024) void k_rank_small(RankArgs r) {
  __shared__ uint32_t s_fs[kRankSortMax];
  __shared__ uint32_t s_tmp[16];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const uint64_t base = r.persist->rec_base;
  const uint64_t fbase = r.persist->flow_count;
  const uint64_t n_new = rank_new(r, fbase);
  if (tid == 0) r.batch->flow_total = fbase + n_new;
  if (n_new <= kRankSortMax) {
    for (uint32_t j = tid; j < n_new; j += 1024) s_fs[j] = new_flow_fs(r, j);
    for (uint32_t j = (uint32_t)n_new + tid; j < ((uint32_t)n_new + 3u) / 4u * 4u; j += 1024)
      s_fs[j] = 0xFFFFFFFFu;  // pad to a multiple of 4 (never below a real value)
    __syncthreads();
    const uint32_t n4 = ((uint32_t)n_new + 3u) / 4u;
    const uint4* v4 = reinterpret_cast<const uint4*>(s_fs);
    for (uint32_t j = tid; j < n_new; j += 1024) {
      const uint32_t v = s_fs[j];
      uint32_t rank = 0;
      for (uint32_t i = 0; i < n4; ++i) {  // broadcast reads: every lane reads the same word
        const uint4 q = v4[i];
        rank += (q.x < v) + (q.y < v) + (q.z < v) + (q.w < v);
      }
      r.tab.cfs[fbase + j] = base + v;  // first_seen, global record index
      r.tab.cmap[fbase + j] = (uint32_t)(fbase + rank);
      if (r.update_persist) r.tab.cnt[2 * (fbase + rank)] = r.tab.cnt[2 * (fbase + rank) + 1] = 0;
    }
    rank_done(r, tid, base, fbase, n_new);
    return;
  }
  uint64_t wmax = 0;
  for (uint64_t j = tid; j < n_new; j += 1024) {
    const uint64_t local = new_flow_fs(r, j);
    if ((local >> 5) < r.nwords) {
      atomicOr(&r.bitmap[local >> 5], 1u << (local & 31));
      wmax = (local >> 5) > wmax ? (local >> 5) : wmax;
    }
  }
  // words past the last first-seen position are all zero: scan only [0, lim)
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(wmax, o);
    wmax = y > wmax ? y : wmax;
  }
  __shared__ uint64_t s_wmax[16];
  if (lane == 0) s_wmax[wave] = wmax;
  __syncthreads();
  for (int w = 0; w < 16; ++w) wmax = s_wmax[w] > wmax ? s_wmax[w] : wmax;
  if (tid == 0) r.batch->fs_max_word = wmax;
  const uint64_t lim = wmax + 1 < r.nwords ? wmax + 1 : r.nwords;
  // wave w owns words [w*per, (w+1)*per), per a multiple of 64; lane l holds words
  // w*per + 64k + l in wv[k]. Wave totals first (for the wave's base), then a
  // per-64-word scan writes the exclusive prefixes.
  constexpr int kMaxK = (int)(kRankSmallWords / 1024);
  const uint32_t per = (uint32_t)((lim + 16 * 64 - 1) / (16 * 64)) * 64u;
  const uint64_t w0 = (uint64_t)wave * per;
  const uint32_t kk = per / 64u;
  uint32_t wv[kMaxK];
  uint32_t mine = 0;
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) {
    const uint64_t w = w0 + 64u * k + lane;
    wv[k] = ((uint32_t)k < kk && w < lim)
                ? __hip_atomic_load(&r.bitmap[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                : 0u;
    mine += __popc(wv[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o);
  if (lane == 0) s_tmp[wave] = mine;
  __syncthreads();
  uint32_t carry = 0;
  for (uint32_t w = 0; w < wave; ++w) carry += s_tmp[w];
#pragma unroll
  for (int k = 0; k < kMaxK; ++k) {
    if ((uint32_t)k < kk) {  // wave-uniform
      const uint32_t c = __popc(wv[k]);
      uint32_t x = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
      }
      const uint64_t w = w0 + 64u * k + lane;
      if (w < lim) r.wprefix[w] = carry + x - c;
      carry += __shfl(x, 63);
    }
  }
  __syncthreads();
  for (uint64_t j = tid; j < n_new; j += 1024) {
    const uint64_t local = new_flow_fs(r, j);
    const uint64_t w = local >> 5;
    uint64_t id = fbase + n_new - 1;  // first_seen outside the batch (an invalid merge
                                      // input, flagged by its exporter): no bitmap read
    if (w < lim) {
      const uint32_t below = __hip_atomic_load(&r.bitmap[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &
                             ((1u << (local & 31)) - 1u);
      id = fbase + r.wprefix[w] + __popc(below);
    }
    r.tab.cfs[fbase + j] = base + local;
    r.tab.cmap[fbase + j] = (uint32_t)id;
    if (r.update_persist) r.tab.cnt[2 * id] = r.tab.cnt[2 * id + 1] = 0;
  }
  rank_done(r, tid, base, fbase, n_new);
}

__global__ __launch_bounds__(kBlock) void k_mark(RankArgs r) {
  __shared__ uint64_t s_wmax[kBlock / 64];
  const uint64_t n_new = rank_new(r, r.persist->flow_count);
  uint64_t wmax = 0;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n_new;
       j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t local = new_flow_fs(r, j);
    r.new_fs[j] = (uint32_t)local;  // k_assign reads it densely (not through the slots)
    if ((local >> 5) < r.nwords) {
      atomicOr(&r.bitmap[local >> 5], 1u << (local & 31));
      wmax = (local >> 5) > wmax ? (local >> 5) : wmax;
    }
  }
  // highest word set (one device atomic per block): bounds the scan and the clear
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(wmax, o);
    wmax = y > wmax ? y : wmax;
  }
  if ((threadIdx.x & 63u) == 0) s_wmax[threadIdx.x >> 6] = wmax;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) wmax = s_wmax[w] > wmax ? s_wmax[w] : wmax;
    if (wmax) atomicMax((unsigned long long*)&r.batch->fs_max_word, (unsigned long long)wmax);
  }
}

// words [0, lim) of the bitmap can be non-zero this batch
__device__ __forceinline__ uint64_t rank_words(const RankArgs& r) {
  const uint64_t m = r.batch->fs_max_word + 1;
  return m < r.nwords ? m : r.nwords;
}

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

__global__ __launch_bounds__(kBlock) void k_scan_words(RankArgs r) {
  __shared__ uint32_t s_tmp[4];
  const uint64_t lim = rank_words(r);
  // grid-stride over scan blocks (the launch covers the batch; only [0, lim) is live)
  for (uint64_t b = blockIdx.x; b * kScanWordsPerBlock < lim; b += gridDim.x) {  // block-uniform
    const uint64_t w0 = b * kScanWordsPerBlock + threadIdx.x * 8ull;
    uint32_t c[8], sum = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      c[k] = (w0 + k < lim) ? (uint32_t)__popc(r.bitmap[w0 + k]) : 0u;
      sum += c[k];
    }
    uint32_t total;
    uint32_t pre = block_excl_scan(sum, s_tmp, total);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (w0 + k < lim) r.wprefix[w0 + k] = pre;
      pre += c[k];
    }
    if (threadIdx.x == 0) r.bprefix[b] = total;
  }
}

__global__ __launch_bounds__(kBlock) void k_scan_blocks(RankArgs r) {
  __shared__ uint32_t s_tmp[4];
  if (threadIdx.x == 0) {
    // k_assign (next launch) reads the bases staged here; the batch is classified
    // once it runs, so the context's bases advance now (nothing between this
    // launch and k_assign reads them). Round 2 had k_assign's last block do it:
    // one same-address device atomic per block cost ~10 us
    const uint64_t base = r.persist->rec_base, fbase = r.persist->flow_count;
    const uint64_t n_new = rank_new(r, fbase);
    r.persist->rank_base = base;
    r.persist->rank_fbase = fbase;
    r.batch->n_new = n_new;  // the claimed ones (k_assign and everything after)
    r.batch->flow_total = fbase + n_new;
    if (r.update_persist) {
      r.persist->rec_base = base + r.batch->n_acc;
      r.persist->flow_count = fbase + n_new;
    }
  }
  uint32_t carry = 0;
  const uint64_t nb = (rank_words(r) + kScanWordsPerBlock - 1) / kScanWordsPerBlock;
  for (uint64_t b0 = 0; b0 < nb; b0 += kBlock) {
    const uint64_t b = b0 + threadIdx.x;
    const uint32_t v = b < nb ? r.bprefix[b] : 0u;
    uint32_t total;
    const uint32_t pre = block_excl_scan(v, s_tmp, total);
    if (b < nb) r.bprefix[b] = carry + pre;
    carry += total;
  }
}

__global__ void k_assign(RankArgs r) {
  const uint64_t n_new = r.batch->n_new;
  // surplus blocks (the grid is fixed: the host does not know n_new) leave at once
  if (blockIdx.x * (uint64_t)blockDim.x >= n_new) return;
  const uint64_t lim = rank_words(r);
  const uint64_t base = r.persist->rank_base;    // staged by k_scan_blocks
  const uint64_t fbase = r.persist->rank_fbase;
  for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < n_new;
       j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t local = r.new_fs[j];  // (k_mark's copy of the slot's fs32)
    const uint64_t w = local >> 5;
    uint64_t id = fbase + n_new - 1;  // first_seen outside the batch: see k_rank_small
    if (w < lim) {
      const uint32_t below = r.bitmap[w] & ((1u << (local & 31)) - 1u);
      id = fbase + r.bprefix[w / kScanWordsPerBlock] + r.wprefix[w] + __popc(below);
    }
    r.tab.cfs[fbase + j] = base + local;
    r.tab.cmap[fbase + j] = (uint32_t)id;
    if (r.update_persist) r.tab.cnt[2 * id] = r.tab.cnt[2 * id + 1] = 0;
  }
}


// K3: per accepted frame, claim index -> dense id (written for records p <
// out_cap) and pkts/bytes per flow. Three modes, chosen on the device from the
// batch's flow count F (the host cannot know it without a sync):
//  0  F <= kCountBins: each block histograms a contiguous range of accepted
//     frames in LDS with the claim->id map staged beside the bins — one 64-bit
//     bin per flow (pkts in bits 63:40, bytes in 39:0), one LDS atomic per record,
//     one per wave-iteration when all of a wave's records share a flow — then
//     writes its bins as a dense partial row that k_count_reduce sums. A block
//     covers < 2^24 records and frames of >= kBigLen bytes go to global atomics,
//     so no bin field can overflow (no flushes inside the loop).
//  1  F <= nb_max * kBucket (the large-table path): claims are bucketed by
//     claim >> kBucketBits. Each block counts its range's records per bucket,
//     scans the counts, then scatters (claim, caplen) into its own region of a
//     scratch buffer, bucket by bucket; k_count_bucket then histograms one bucket
//     (from every block's segment of it) in LDS per workgroup; the reduce maps
//     claims to ids. Region entries are one word (claim within the bucket,
//     20-bit caplen). Replaces per-record device atomics (~86 ps per record at
//     1M flows) with ~28 B of streaming traffic per record.
//  2  otherwise (or no scratch): per-record global atomics, wave-uniform flows
//     aggregated first.
constexpr uint64_t kBinByMask = (1ull << kBinPkShift) - 1;

// records [lo, hi) of K3 block `b` (identical in k_count and k_count_bucket)
__device__ __forceinline__ uint64_t count_per(uint64_t n_acc, uint32_t grid) {
  return ((n_acc + grid - 1) / grid + kK3Gran - 1) / kK3Gran * kK3Gran;
}

// mode 3 geometry from the flow count: R ranges, groups per XCD column
__device__ __forceinline__ uint32_t range_count(uint64_t nflows) {
  return (uint32_t)((nflows + kCountBins - 1) / kCountBins);
}
__device__ __forceinline__ uint32_t range_groups_per_x(const CountArgs& c, uint64_t nflows) {
  return (c.g1 / 8u) / range_count(nflows);
}

__device__ __forceinline__ int count_mode(const CountArgs& c, uint64_t nflows) {
  if (nflows <= (uint64_t)kCountBins) return 0;
  // mode 3: every group of R blocks re-reads its segment R times (from the XCD's
  // L2); a group must cover < kK3MaxPer records (bin fields cannot overflow)
  if (c.range_ok && nflows <= kRangeFlows && c.g1 % 8u == 0 && range_groups_per_x(c, nflows) > 0 &&
      count_per(c.batch->n_acc, 8u * range_groups_per_x(c, nflows)) <= kK3MaxPer &&
      8ull * range_groups_per_x(c, nflows) * nflows <= c.part_words)
    return 3;
  if (c.region && nflows <= (uint64_t)c.nb_max * kBucket) return 1;
  return 2;
}


// K1's per-record scratch of U accepted records p0 + k*kCountBlock (p < hi;
// others give claim ~0, len 0): claim (~0: no flow) and caplen, packed in one
// word when the context's table is small enough (pack_bits != 0). All words are
// loaded before any is inspected (a branch between them would serialize them).
template <int U, bool PACK, int STRIDE = kCountBlock>
__device__ __forceinline__ void load_acc(const CountArgs& c, uint64_t p0, uint64_t lo, uint64_t hi,
                                         uint32_t (&claim)[U], uint32_t (&len)[U]) {
  uint32_t v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const uint64_t p = p0 + (uint64_t)k * STRIDE;
    v[k] = __builtin_nontemporal_load(&c.acc_flow[p < hi ? p : lo]);
    if (!PACK) len[k] = __builtin_nontemporal_load(&c.acc_len[p < hi ? p : lo]);
  }
  const uint32_t lmax = 0xFFFFFFFFu >> c.pack_bits;
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const uint64_t p = p0 + (uint64_t)k * STRIDE;
    if (PACK) {
      claim[k] = v[k] == 0xFFFFFFFFu ? v[k] : (v[k] & ((1u << c.pack_bits) - 1u));
      len[k] = v[k] >> c.pack_bits;
    } else {
      claim[k] = v[k];
    }
    if (p >= hi) claim[k] = 0xFFFFFFFFu, len[k] = 0;
  }
  if (PACK) {
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (len[k] == lmax && claim[k] != 0xFFFFFFFFu) len[k] = c.acc_len[p0 + (uint64_t)k * STRIDE];
  }
}

// The same for packed words, four consecutive records per 16-B load: entry 4k + j
// is record p0 + 4 k kCountBlock + j (p0 = base + 4 tid, 16-B aligned: block ranges
// start at multiples of kK3Gran). Four times the bytes in flight per load
// instruction of the scalar form (K3 mode 0 holds one 1024-thread block per CU).
template <int U>
__device__ __forceinline__ void load_acc4(const CountArgs& c, uint64_t p0, uint64_t hi,
                                          uint32_t (&claim)[4 * U], uint32_t (&len)[4 * U]) {
  uint32_t v[4 * U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const uint64_t p = p0 + 4ull * k * kCountBlock;
    if (p + 3 < hi) {
      const u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(c.acc_flow + p));
      v[4 * k] = q[0];
      v[4 * k + 1] = q[1];
      v[4 * k + 2] = q[2];
      v[4 * k + 3] = q[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[4 * k + j] = p + j < hi ? c.acc_flow[p + j] : 0xFFFFFFFFu;
    }
  }
  const uint32_t lmax = 0xFFFFFFFFu >> c.pack_bits;
  bool sat = false;
#pragma unroll
  for (int e = 0; e < 4 * U; ++e) {
    claim[e] = v[e] == 0xFFFFFFFFu ? v[e] : (v[e] & ((1u << c.pack_bits) - 1u));
    len[e] = v[e] == 0xFFFFFFFFu ? 0u : v[e] >> c.pack_bits;
    sat |= len[e] == lmax;
  }
  if (__any(sat)) {  // a caplen past the packed field: the side array (rare)
#pragma unroll
    for (int e = 0; e < 4 * U; ++e)
      if (len[e] == lmax) len[e] = c.acc_len[p0 + 4ull * (e / 4) * kCountBlock + (e % 4)];
  }
}

template <bool PACK>
__device__ __forceinline__ uint32_t load_claim(const CountArgs& c, uint64_t p) {
  const uint32_t v = __builtin_nontemporal_load(&c.acc_flow[p]);
  return (PACK && v != 0xFFFFFFFFu) ? (v & ((1u << c.pack_bits) - 1u)) : v;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// exclusive scan over the 1024 threads of a block; s_w: 16 words of LDS
template <int NT = kCountBlock>
__device__ __forceinline__ uint32_t block1024_excl_scan(uint32_t v, uint32_t* s_w, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) s_w[wave] = x;
  __syncthreads();
  uint32_t base = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) {
    const uint32_t t = s_w[w];
    if ((uint32_t)w < wave) base += t;
    total += t;
  }
  __syncthreads();
  return base + x - v;
}

// Mode 1, phase 1 (inside k_count): ids out, bucket counts, scan, scatter.
// SABL (timing-only ablations, 0 in product launches): 1 no region stores,
// 2 no second pass, 4 no id gather/stores in the first pass
// STAGED (nb <= kSmallNb): pass 2 counting-sorts each chunk of U x 1024 entries
// by bucket in LDS (stage / sb / ch / co) and stores them as per-bucket runs.
struct ScatterStage {
  uint32_t* stage;  // [U * kCountBlock] entries of one chunk, bucket-sorted
  uint16_t* sb;     // their buckets
  uint32_t* ch;     // [kSmallNb + 1] chunk counts per bucket (+ spare)
  uint32_t* co;     // [kSmallNb + 1] chunk offsets per bucket
};

template <int U, bool PACK, int SABL = 0, bool STAGED = false>
__device__ void count_scatter(const CountArgs& c, uint64_t lo, uint64_t hi, uint64_t nflows,
                              uint32_t* hist, uint32_t* cur, uint32_t* s_w,
                              const ScatterStage& st = ScatterStage{}) {
  constexpr uint32_t kMaxBuckets = STAGED ? kSmallNb : tcbee::kMaxBuckets;  // the spare slot
  const uint32_t tid = threadIdx.x;
  const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);
  // Cost at 125M records, 31 buckets (tools/k3_ablate.sh): claim stream 0.09 ms,
  // histogram atomics ~0, id gather + out_id stores ~0.55 ms, scattered region
  // stores ~0.45 ms. The stores' cost is their count and scatter, not their
  // bytes (8 -> 4-B entries saved 0.16 ms); moving the id gather into the second
  // pass did not help (tried)
  for (uint32_t b = tid; b < nb; b += kCountBlock) hist[b] = 0;
  if (tid == 0) hist[kMaxBuckets] = cur[kMaxBuckets] = 0;
  __syncthreads();
  for (uint64_t base = lo; base < hi; base += (uint64_t)U * kCountBlock) {
    uint32_t s[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
      s[k] = load_claim<PACK>(c, p < hi ? p : lo);
      if (p >= hi) s[k] = 0xFFFFFFFFu;
    }
    if (!(SABL & 4)) {
      uint32_t id[U];
#pragma unroll
      for (int k = 0; k < U; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : c.omap[s[k]];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
        if (c.out_id && p < hi && p < c.out_cap) __builtin_nontemporal_store(id[k], &c.out_id[p]);
      }
    }
    // no-flow records bump the spare counter hist[kMaxBuckets]: no branch per record
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (SABL & 8) {
        asm volatile("" ::"v"(s[k]));
        continue;
      }
      atomicAdd(&hist[s[k] != 0xFFFFFFFFu ? (s[k] >> kBucketBits) : kMaxBuckets], 1u);
    }
  }
  __syncthreads();
  // exclusive scan of hist[0, nb): thread t owns buckets [t*q, t*q + q)
  const uint32_t q = (nb + kCountBlock - 1) / kCountBlock;
  uint32_t mine = 0;
  for (uint32_t b = tid * q; b < nb && b < (tid + 1) * q; ++b) mine += hist[b];
  uint32_t total;
  uint32_t run = block1024_excl_scan(mine, s_w, total);
  uint32_t* offs = c.offs + (uint64_t)blockIdx.x * (c.nb_max + 1);
  for (uint32_t b = tid * q; b < nb && b < (tid + 1) * q; ++b) {
    cur[b] = run;
    offs[b] = run;
    run += hist[b];
  }
  if (tid == 0) offs[nb] = total;
  __syncthreads();
  if (SABL & 2) return;
  if constexpr (STAGED) {
    for (uint32_t b = tid; b <= kMaxBuckets; b += kCountBlock) st.ch[b] = 0;
    __syncthreads();
    for (uint64_t base = lo; base < hi; base += (uint64_t)U * kCountBlock) {
      uint32_t sc[U], len[U], lp[U];
      load_acc<U, PACK>(c, base + tid, lo, hi, sc, len);
#pragma unroll
      for (int k = 0; k < U; ++k)
        lp[k] = atomicAdd(&st.ch[sc[k] != 0xFFFFFFFFu ? (sc[k] >> kBucketBits) : kMaxBuckets], 1u);
      __syncthreads();
      // chunk offsets (buckets 0..nb-1; no-flow entries in the spare are dropped)
      // and each bucket's global base for this chunk, from the block's cursors
      {
        const uint32_t v = tid < nb ? st.ch[tid] : 0u;
        uint32_t tot;
        const uint32_t off = block1024_excl_scan(v, s_w, tot);
        if (tid < nb) {
          st.co[tid] = off;
          hist[tid] = cur[tid];  // hist (pass-1 counts, done with) = chunk base
          cur[tid] += v;
        }
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (sc[k] == 0xFFFFFFFFu) continue;
        const uint32_t b = sc[k] >> kBucketBits;
        const uint32_t idx = st.co[b] + lp[k];
        st.stage[idx] = (sc[k] & (kBucket - 1u)) | ((len[k] < kRegLenEsc ? len[k] : 0u) << kBucketBits);
        st.sb[idx] = (uint16_t)b;
        if (len[k] >= kRegLenEsc)
          atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[sc[k]] + 1], (unsigned long long)len[k]);
      }
      __syncthreads();
      const uint32_t nval = nb ? st.co[nb - 1] + st.ch[nb - 1] : 0u;
      for (uint32_t idx = tid; idx < nval; idx += kCountBlock) {
        const uint32_t b = st.sb[idx];
        c.region[lo + hist[b] + (idx - st.co[b])] = st.stage[idx];  // runs: coalesced
      }
      __syncthreads();
      for (uint32_t b = tid; b <= kMaxBuckets; b += kCountBlock) st.ch[b] = 0;
      __syncthreads();
    }
    return;
  }
  for (uint64_t base = lo; base < hi; base += (uint64_t)U * kCountBlock) {
    uint32_t s[U], len[U], pos[U];
    load_acc<U, PACK>(c, base + tid, lo, hi, s, len);
    // every cursor bump issued (unconditionally: no-flow records bump the spare
    // cur[kMaxBuckets]) before the first store, so the LDS round trips overlap
#pragma unroll
    for (int k = 0; k < U; ++k)
      pos[k] = atomicAdd(&cur[s[k] != 0xFFFFFFFFu ? (s[k] >> kBucketBits) : kMaxBuckets], 1u);
    if (SABL & 1) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < U; ++k) x ^= pos[k] ^ len[k];
      asm volatile("" ::"v"(x));
      continue;
    }
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (s[k] != 0xFFFFFFFFu)
        c.region[lo + pos[k]] = (s[k] & (kBucket - 1u)) | ((len[k] < kRegLenEsc ? len[k] : 0u) << kBucketBits);
#pragma unroll
    for (int k = 0; k < U; ++k)
      if (s[k] != 0xFFFFFFFFu && len[k] >= kRegLenEsc)
        atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[s[k]] + 1], (unsigned long long)len[k]);
  }
}

// Mode 3 (kCountBins < F <= kRangeFlows): the claims are split into R ranges of
// at most kCountBins; block b works for range r of group g, where the R blocks of a
// group share b % 8 — one XCD under the observed round-robin placement (speed only)
// — and one contiguous record segment. Each block streams its group's segment
// (after the first of the R readers, from that XCD's L2), keeps only the records
// whose claim lies in its range: output id from the range's map in LDS (written
// where it lands: the R blocks fill each out_id line between them), pkts/bytes
// into the range's LDS bins; one partial row per group, summed by the reduce.
// Replaces the bucket scatter's two passes + region round trip and the per-record
// claim -> id gather from L2 (mode 1) for the sizes one GPU's flow-hash share of
// config 4 has (~125k flows).
template <int U, bool PACK>
__device__ void count_ranges(const CountArgs& c, uint64_t n_acc, uint64_t nflows,
                             uint64_t* s_bin, uint32_t* s_map) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t R = range_count(nflows), px = range_groups_per_x(c, nflows);
  const uint32_t b = blockIdx.x, x = b % 8u, j = b / 8u;
  const uint32_t gx = j / R, r = j % R;
  if (gx >= px) return;
  const uint32_t G = 8u * px, g = gx * 8u + x;
  const uint64_t per = count_per(n_acc, G);
  const uint64_t lo = (uint64_t)g * per < n_acc ? (uint64_t)g * per : n_acc;
  const uint64_t hi = lo + per < n_acc ? lo + per : n_acc;
  const uint64_t width = (nflows + R - 1) / R;  // <= kCountBins
  const uint64_t c0 = (uint64_t)r * width;
  const uint64_t c1 = c0 + width < nflows ? c0 + width : nflows;
  const uint32_t nb = c1 > c0 ? (uint32_t)(c1 - c0) : 0u;
  for (uint32_t i = tid; i < nb; i += kCountBlock) {
    s_bin[i] = 0;
    s_map[i] = c.omap[c0 + i];
  }
  __syncthreads();
  for (uint64_t base = lo; base < hi; base += (uint64_t)U * kCountBlock) {
    uint32_t v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
      v[k] = __builtin_nontemporal_load(&c.acc_flow[p < hi ? p : lo]);
      if (p >= hi) v[k] = 0xFFFFFFFFu;
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t cl = (PACK && v[k] != 0xFFFFFFFFu) ? (v[k] & ((1u << c.pack_bits) - 1u)) : v[k];
      const uint32_t rel = cl - (uint32_t)c0;  // wraps for claims below the range
      const bool hit = cl != 0xFFFFFFFFu && rel < nb;
      if (!__any(hit)) continue;
      const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
      uint32_t len = 0;
      if (hit) {
        len = PACK ? v[k] >> c.pack_bits : c.acc_len[p];
        if (PACK && len == (0xFFFFFFFFu >> c.pack_bits)) len = c.acc_len[p];  // saturated
        if (c.out_id && p < c.out_cap) c.out_id[p] = s_map[rel];
      }
      // a hot flow: every lane of the wave on one claim -> one LDS add
      const uint32_t r0 = __builtin_amdgcn_readfirstlane(rel);
      if (__all(hit && rel == r0 && len < kBigLen)) {
        const uint32_t by = wave_sum32(len);
        if (lane == 0) atomicAdd((unsigned long long*)&s_bin[r0], (64ull << kBinPkShift) | by);
      } else if (hit) {
        if (len < kBigLen) {
          atomicAdd((unsigned long long*)&s_bin[rel], (1ull << kBinPkShift) | len);
        } else {
          const uint32_t lid = c.cmap[cl];  // counters by local id
          atomicAdd((unsigned long long*)&c.cnt[2ull * lid], 1ull);
          atomicAdd((unsigned long long*)&c.cnt[2ull * lid + 1], (unsigned long long)len);
        }
      }
    }
  }
  __syncthreads();
  uint64_t* part = c.part + (uint64_t)g * nflows + c0;
  for (uint32_t i = tid; i < nb; i += kCountBlock) part[i] = s_bin[i];
}

// Fused rank (CountArgs::fused_rank): this batch's new flows' output ids, ranked by
// their first records (as k_rank_small's <= kRankSortMax path), into s_map[fbase + j];
// block 0 also publishes what K2 would have (cmap, cfs, flow_total, the clamped
// n_new). The new ids' counters were zeroed by k_prep (zero_free_counters): every
// block may add a big frame to them, and nothing orders those adds after a zeroing
// here. Returns the flow count after the batch.
__device__ uint64_t fused_rank_block(const CountArgs& c, uint32_t* s_map, uint64_t& fbase_out) {
  __shared__ uint32_t s_nfs[kFuseRankMax];
  const uint32_t tid = threadIdx.x;
  const uint64_t base = c.persist->rec_base, fbase = c.persist->flow_count;
  fbase_out = fbase;
  const uint64_t room = c.tab.max_claims > fbase ? c.tab.max_claims - fbase : 0;
  const uint64_t n_new = c.batch->n_new < room ? c.batch->n_new : room;
  for (uint32_t j = tid; j < n_new; j += kCountBlock)
    s_nfs[j] = *slot_fs_any(c.tab, (uint32_t)c.new_list[j]);
  __syncthreads();
  for (uint32_t j = tid; j < n_new; j += kCountBlock) {
    const uint32_t v = s_nfs[j];
    uint32_t rank = 0;
    for (uint32_t i = 0; i < n_new; ++i) rank += s_nfs[i] < v;  // broadcast reads
    const uint32_t id = (uint32_t)(fbase + rank);
    s_map[fbase + j] = id;
    if (blockIdx.x == 0) {
      c.tab.cfs[fbase + j] = base + v;  // first_seen, global record index
      c.tab.cmap[fbase + j] = id;
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    c.batch_rw->n_new = n_new;
    c.batch_rw->flow_total = fbase + n_new;
  }
  return fbase + n_new;
}

// ABL3 (timing-only ablations, 0 in every product launch): 1 no bin updates,
// 2 no id gather, 4 no id stores; 8 (A/B, variants build) plain id stores instead of
// non-temporal ones.
// Bins are indexed by CLAIM (dense in [0, F)); the record's output id is
// omap[claim] (the local dense id, or — after a flow-hash exchange — the global
// one), staged in LDS; k_count_reduce maps claims to local ids for the counters.
template <int U, int ABL3, bool PACK, bool VEC = false>
__global__ __launch_bounds__(kCountBlock) void k_count(CountArgs c) {
  __shared__ uint64_t s_bin[kCountBins];  // by claim
  __shared__ uint32_t s_map[kCountBins];  // claim index -> output id
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint64_t n_acc = c.batch->n_acc;
  // (fused rank: K2 did not run; the flow count is this block's own)
  uint64_t fbase_f = 0;
  const uint64_t nflows = c.fused_rank ? fused_rank_block(c, s_map, fbase_f) : c.batch->flow_total;
  if (blockIdx.x == 0 && tid == 0) {
    // finalize (nothing here writes what other blocks read: with a fused rank every
    // block reads the old record base / flow count, which the reduce advances)
    const uint64_t written = n_acc < c.out_cap ? n_acc : c.out_cap;
    if (c.out_n) *c.out_n = written;
    if (c.ctr) {
      if (c.direction) c.ctr->egress += n_acc;  // EGRESS_EVENTS, tc.rs:167
      else c.ctr->ingress += n_acc;             // INGRESS_EVENTS, xdp.rs:207
      c.ctr->handled += written;                // EVENTS_HANDLED, xdp.rs:214
      c.ctr->dropped += n_acc - written;        // EVENTS_DROPPED, xdp.rs:217
    }
    // (rec_base / flow_count were advanced by K2: this may run on another stream
    //  beside the next batch's K1, which reads them)
  }
  {
    // the first-seen bitmap back to all-zero (the rank kernels are done with it)
    const uint64_t wlast = c.batch->fs_max_word;
    for (uint64_t w = blockIdx.x * (uint64_t)kCountBlock + tid; w <= wlast;
         w += (uint64_t)gridDim.x * kCountBlock)
      c.bitmap[w] = 0;
  }
  const int mode = count_mode(c, nflows);
  if (blockIdx.x == 0 && tid == 0) c.persist_rw->k3_mode = (uint32_t)mode + 1u;
  const uint64_t per = count_per(n_acc, gridDim.x);
  const uint64_t lo = (uint64_t)blockIdx.x * per < n_acc ? (uint64_t)blockIdx.x * per : n_acc;
  const uint64_t hi = lo + per < n_acc ? lo + per : n_acc;
  if (mode == 1) return;  // k_count_scatter
  if (mode == 3) {
    count_ranges<U, PACK>(c, n_acc, nflows, s_bin, s_map);
    return;
  }
  if (mode == 0) {
    // (fused rank: claims of this batch's new flows were mapped above)
    const uint64_t mapped = c.fused_rank ? fbase_f : nflows;
    for (uint32_t b = tid; b < nflows; b += kCountBlock) {
      s_bin[b] = 0;
      if (b < mapped) s_map[b] = c.omap[b];
    }
    __syncthreads();
  }
  // counters are kept by LOCAL dense id (fused rank: omap is the local map and
  // s_map holds it — block 0's cmap stores for this batch's new flows are not
  // ordered before other blocks' reads)
  auto global_add = [&](uint32_t claim, uint64_t pk, uint64_t by) {
    const uint32_t lid = c.fused_rank ? s_map[claim] : c.cmap[claim];
    atomicAdd((unsigned long long*)&c.cnt[2ull * lid], (unsigned long long)pk);
    atomicAdd((unsigned long long*)&c.cnt[2ull * lid + 1], (unsigned long long)by);
  };
  // VEC: four consecutive records per lane and load (packed words only)
  constexpr int UU = VEC ? 4 * U : U;
  for (uint64_t base = lo; base < hi; base += (uint64_t)UU * kCountBlock) {
    uint32_t s[UU], len[UU], id[UU];
    if (kK3LoadPrio) __builtin_amdgcn_s_setprio(kK3LoadPrio);
    if constexpr (VEC) load_acc4<U>(c, base + 4ull * tid, hi, s, len);  // non-temporal
    else load_acc<U, PACK>(c, base + tid, lo, hi, s, len);  // streamed once: non-temporal
    if (kK3LoadPrio) __builtin_amdgcn_s_setprio(0);
    if (ABL3 & 2) {
#pragma unroll
      for (int k = 0; k < UU; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : (s[k] & 8191u);
    } else if (mode == 0) {
#pragma unroll
      for (int k = 0; k < UU; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : s_map[s[k]];
    } else {
#pragma unroll
      for (int k = 0; k < UU; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : c.omap[s[k]];
    }
    if (c.out_id && !(ABL3 & 4)) {
      if constexpr (VEC) {
        const uint64_t lim = hi < c.out_cap ? hi : c.out_cap;
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const uint64_t p = base + 4ull * ((uint64_t)k * kCountBlock + tid);
          if (p + 3 < lim) {
            u32x4 q;
            q[0] = id[4 * k];
            q[1] = id[4 * k + 1];
            q[2] = id[4 * k + 2];
            q[3] = id[4 * k + 3];
            __builtin_nontemporal_store(q, reinterpret_cast<u32x4*>(c.out_id + p));
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (p + j < lim) c.out_id[p + j] = id[4 * k + j];
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
          if (p < hi && p < c.out_cap) {
            if constexpr ((ABL3 & 8) != 0) c.out_id[p] = id[k];
            else __builtin_nontemporal_store(id[k], &c.out_id[p]);
          }
        }
      }
    }
    if (ABL3 & 1) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < UU; ++k) x ^= id[k] ^ len[k];
      asm volatile("" ::"v"(x));
      continue;
    }
    if (mode == 0) {
      // one flow in all of the wave's records this iteration (a hot flow): one add
      const uint32_t s0 = __builtin_amdgcn_readfirstlane(s[0]);
      bool same = s0 != 0xFFFFFFFFu;
      uint32_t nk = 0, sl = 0;
#pragma unroll
      for (int k = 0; k < UU; ++k) {
        const bool v = s[k] != 0xFFFFFFFFu;
        same = same && (!v || (s[k] == s0 && len[k] < kBigLen));
        nk += v ? 1u : 0u;
        sl += v ? len[k] : 0u;
      }
      if (__all(same)) {
        // pk <= 64*UU, by <= 64*UU*(kBigLen-1) < 2^32 at UU <= 32 (sums in 64 bits)
        const uint64_t pk = wave_sum64(nk), by = wave_sum64(sl);
        if (lane == 0)
          atomicAdd((unsigned long long*)&s_bin[s0], ((unsigned long long)pk << kBinPkShift) | by);
      } else {
#pragma unroll
        for (int k = 0; k < UU; ++k) {
          if (s[k] == 0xFFFFFFFFu) continue;
          if (len[k] < kBigLen)
            atomicAdd((unsigned long long*)&s_bin[s[k]], (1ull << kBinPkShift) | len[k]);
          else
            global_add(s[k], 1, len[k]);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < UU; ++k) {
        const bool mine = s[k] != 0xFFFFFFFFu;
        const uint64_t am = __ballot(mine);
        const uint32_t leader = am ? (uint32_t)__ffsll((unsigned long long)am) - 1 : 0u;
        const uint32_t s0 = __shfl(s[k], leader);
        if (__all(!mine || s[k] == s0)) {
          const uint64_t bs = wave_sum64(mine ? (uint64_t)len[k] : 0ull);
          if (am && lane == leader) global_add(s0, (uint64_t)__popcll(am), bs);
        } else if (mine) {
          global_add(s[k], 1, len[k]);
        }
      }
    }
  }
  if (c.next_batch) {
    // (small contexts) the next batch's preparation, grid-strided: nothing here is
    // read by this launch (this batch's K1 is done with its tile words; the next
    // slot and the inactive generation are untouched by this batch)
    const uint64_t t0 = blockIdx.x * (uint64_t)kCountBlock + tid;
    const uint64_t stride = (uint64_t)gridDim.x * kCountBlock;
    for (uint64_t i = t0; i < c.clean_ntiles; i += stride) c.clean_tiles[i] = 0;
    if (t0 < sizeof(BatchState) / 8) reinterpret_cast<uint64_t*>(c.next_batch)[t0] = 0;
    if (c.clean_alt) {
      if (t0 < sizeof(PersistState) / 8) reinterpret_cast<uint64_t*>(c.alt_persist)[t0] = 0;
      empty_units(c.alt, t0, stride);
      for (uint64_t i = t0; i < 2 * c.alt.max_claims; i += stride) c.alt.cnt[i] = 0;
    }
  }
  if (mode == 0 && c.fused_rank) {
    // (fused rank, <= kFuseRankMax flows: no reduce launch) the block's bins go
    // straight to the counters by local id — at most 2 x 256 device adds per block —
    // and the last block to finish advances the record base / flow count: every
    // block has read (and used) the old ones by now
    __syncthreads();
    for (uint32_t b = tid; b < nflows; b += kCountBlock) {
      const uint64_t v = s_bin[b];
      if (v) {
        const uint32_t id = s_map[b];
        atomicAdd((unsigned long long*)&c.cnt[2ull * id], (unsigned long long)(v >> kBinPkShift));
        atomicAdd((unsigned long long*)&c.cnt[2ull * id + 1], (unsigned long long)(v & kBinByMask));
      }
    }
    if (tid == 0 &&
        atomicAdd((unsigned long long*)&c.batch_rw->k3_done, 1ull) == (unsigned long long)gridDim.x - 1) {
      c.persist_rw->rec_base += n_acc;
      c.persist_rw->flow_count = nflows;
    }
  } else if (mode == 0) {
    // per-block partial histogram, dense and coalesced; k_count_reduce sums them
    // (one writer per flow: no device-scope atomics)
    __syncthreads();
    uint64_t* part = c.part + (uint64_t)blockIdx.x * kCountBins;
    for (uint32_t b = tid; b < nflows; b += kCountBlock) part[b] = s_bin[b];
  }
}

// Mode 1, phase 1 as its own launch: 32 KiB of LDS, so two workgroups share a CU
// (k_count's 144 KiB of bins + map allow one).
// the single-pass chunked scatter (k_count_chunk) takes every mode-1 batch of up to
// kChunkMaxNb - 1 buckets when the context has its chunk offsets
__device__ __forceinline__ bool chunk_scatter(const CountArgs& c, uint64_t nflows) {
  const uint64_t nb = (nflows + kBucket - 1) >> kBucketBits;
  return c.coffs != nullptr && !c.chunk_off && nb < kChunkMaxNb;
}
__device__ __forceinline__ bool staged_scatter(const CountArgs& c, uint64_t nflows) {
  const uint64_t nb = (nflows + kBucket - 1) >> kBucketBits;
  return !c.scatter_unstaged && nb >= kStagedMinNb && nb <= kSmallNb && !chunk_scatter(c, nflows);
}

template <int U, bool PACK, int SABL = 0>
__global__ __launch_bounds__(kCountBlock) void k_count_scatter(CountArgs c) {
  __shared__ uint32_t s_hist[kMaxBuckets + 1], s_cur[kMaxBuckets + 1];  // + spare counter
  __shared__ uint32_t s_w[kCountBlock / 64];
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1) return;
  if (staged_scatter(c, nflows) || chunk_scatter(c, nflows)) return;  // the other two
  const uint64_t n_acc = c.batch->n_acc;
  const uint64_t per = count_per(n_acc, gridDim.x);
  const uint64_t lo = (uint64_t)blockIdx.x * per < n_acc ? (uint64_t)blockIdx.x * per : n_acc;
  const uint64_t hi = lo + per < n_acc ? lo + per : n_acc;
  count_scatter<U, PACK, SABL>(c, lo, hi, nflows, s_hist, s_cur, s_w);
}

// The same for tables of kStagedMinNb..kSmallNb buckets, pass 2 staged through LDS: 4 KiB of
// counters + 48 KiB of chunk staging = 2 workgroups per CU, as the plain kernel.
template <int U, bool PACK>
__global__ __launch_bounds__(kCountBlock) void k_count_scatter_staged(CountArgs c) {
  __shared__ uint32_t s_hist[kSmallNb + 1], s_cur[kSmallNb + 1];
  __shared__ uint32_t s_ch[kSmallNb + 1], s_co[kSmallNb + 1];
  __shared__ uint32_t s_stage[U * kCountBlock];
  __shared__ uint16_t s_sb[U * kCountBlock];
  __shared__ uint32_t s_w[kCountBlock / 64];
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1) return;
  if (!staged_scatter(c, nflows)) return;
  const uint64_t n_acc = c.batch->n_acc;
  const uint64_t per = count_per(n_acc, gridDim.x);
  const uint64_t lo = (uint64_t)blockIdx.x * per < n_acc ? (uint64_t)blockIdx.x * per : n_acc;
  const uint64_t hi = lo + per < n_acc ? lo + per : n_acc;
  ScatterStage st{s_stage, s_sb, s_ch, s_co};
  count_scatter<U, PACK, 0, true>(c, lo, hi, nflows, s_hist, s_cur, s_w, st);
}

// Mode 1, single pass (nb < kChunkMaxNb): each workgroup takes chunks of c.chunk
// accepted records (16 per thread) and
//  1. ranks them by bucket in LDS (counts per bucket, one LDS add per record or one
//     per wave when the wave's records share a bucket; no-flow records go to a
//     spare bucket nb), scans the counts;
//  2. places every record's region entry (claim within the bucket | caplen) and its
//     chunk position + bucket at its bucket-sorted slot in LDS;
//  3. walks the sorted entries with consecutive lanes on consecutive entries: the
//     region entry is stored coalesced at region[chunk + idx] (the chunk's buckets
//     are contiguous runs; coffs[q] = their offsets for k_count_bucket) and the
//     claim -> output id gather reads omap inside one bucket's 16 KiB window per
//     wave (L1-local), where the record-order gather of the two-pass scatter hit 64
//     random lines of a table of every flow;
//  4. writes each id back to its record position in LDS and stores the chunk's ids
//     in record order, coalesced.
// One pass over the K1 -> K3 words, no per-block cursors, no scattered stores.
template <bool PACK, int BS>
__global__ __launch_bounds__(BS) void k_count_chunk(CountArgs c) {
  constexpr int U = 16, CH = U * BS;  // records per chunk (c.chunk)
  __shared__ uint32_t s_ent[CH];   // region entries, bucket-sorted; then ids by position
  __shared__ uint32_t s_pb[CH];    // chunk position | bucket << 14 of each sorted entry
  __shared__ uint32_t s_ch[kChunkMaxNb + 1], s_co[kChunkMaxNb + 1];
  __shared__ uint32_t s_w[BS / 64];
  static_assert(CH <= (1 << 14) && kChunkMaxNb < BS && kChunkMaxNb < (1u << 18), "layout");
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1 || !chunk_scatter(c, nflows) || c.chunk != (uint32_t)CH) return;
  constexpr uint32_t kCountBlock = BS;  // (the loops below are per workgroup thread)
  constexpr uint32_t kChunk = CH;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);  // spare bucket: nb
  const uint64_t n_acc = c.batch->n_acc;
  const uint64_t nchunks = (n_acc + kChunk - 1) / kChunk;
  // Barriers per chunk: rank | scan (2) | offsets | placed | read | ids. The counts
  // are zeroed right after the scan has read them (before three more barriers), so a
  // workgroup's waves may run into the next chunk's loads and ranks while others
  // still store this chunk's ids (nothing those touch is reused before the next
  // rank barrier)
  for (uint32_t b = tid; b <= nb; b += kCountBlock) s_ch[b] = 0;
  __syncthreads();
  // packed K1 -> K3 words: the next chunk's words are loaded while this chunk's
  // sorted entries are read and its ids stored (one workgroup per CU: nothing else
  // hides that load)
  uint32_t nxt[PACK ? U : 1];
  auto prefetch = [&](uint64_t qn) {
    if constexpr (PACK) {
      const uint64_t b0 = qn * kChunk;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t p = b0 + (uint64_t)k * kCountBlock + tid;
        nxt[k] = qn < nchunks && p < n_acc ? __builtin_nontemporal_load(&c.acc_flow[p]) : 0xFFFFFFFFu;
      }
    }
  };
  prefetch(blockIdx.x);
  const uint32_t lmax = 0xFFFFFFFFu >> c.pack_bits;
  for (uint64_t q = blockIdx.x; q < nchunks; q += gridDim.x) {
    const uint64_t base = q * kChunk;
    const uint64_t hi = base + kChunk < n_acc ? base + kChunk : n_acc;
    const uint32_t nval = (uint32_t)(hi - base);
    uint32_t ent[U], bk[U], lp[U];
    if constexpr (PACK) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t v = nxt[k];
        const uint32_t cl = v == 0xFFFFFFFFu ? v : (v & ((1u << c.pack_bits) - 1u));
        uint32_t len = v == 0xFFFFFFFFu ? 0u : v >> c.pack_bits;
        if (len == lmax) len = c.acc_len[base + (uint64_t)k * kCountBlock + tid];  // saturated
        const bool big = len >= kRegLenEsc;
        bk[k] = cl != 0xFFFFFFFFu ? (cl >> kBucketBits) : nb;
        ent[k] = (cl & (kBucket - 1u)) | ((big ? 0u : len) << kBucketBits);
        if (big && cl != 0xFFFFFFFFu)
          atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[cl] + 1], (unsigned long long)len);
      }
    } else
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // two halves of U / 2 loads (register pressure)
      constexpr int H = U / 2;
      uint32_t cl[H], len[H];
      load_acc<H, PACK, BS>(c, base + (uint64_t)h * H * kCountBlock + tid, base, hi, cl, len);
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const bool big = len[k] >= kRegLenEsc;
        bk[h * H + k] = cl[k] != 0xFFFFFFFFu ? (cl[k] >> kBucketBits) : nb;
        ent[h * H + k] = (cl[k] & (kBucket - 1u)) | ((big ? 0u : len[k]) << kBucketBits);
        if (big && cl[k] != 0xFFFFFFFFu)
          atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[cl[k]] + 1], (unsigned long long)len[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool valid = (uint32_t)k * kCountBlock + tid < nval;
      const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk[k]);
      const uint64_t vm = __ballot(valid);
      if (__all(!valid || bk[k] == b0)) {
        // one add for the wave (a hot flow's bucket): ranks in lane order
        uint32_t r0 = 0;
        if (lane == 0 && vm) r0 = atomicAdd(&s_ch[b0], (uint32_t)__popcll(vm));
        r0 = __shfl(r0, 0);
        lp[k] = r0 + (uint32_t)__popcll(vm & lanemask_lt());
      } else {
        lp[k] = valid ? atomicAdd(&s_ch[bk[k]], 1u) : 0u;
      }
    }
    __syncthreads();
    {
      uint32_t tot;
      const uint32_t off = block1024_excl_scan<BS>(tid <= nb ? s_ch[tid] : 0u, s_w, tot);
      if (tid <= nb) s_co[tid] = off;
      if (tid <= nb) c.coffs[q * (kChunkMaxNb + 1) + tid] = off;  // [nb] = end of the real buckets
      if (tid <= nb) s_ch[tid] = 0;  // read by the scan only: zero for the next chunk
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * kCountBlock + tid;
      if (pos >= nval) continue;
      const uint32_t idx = s_co[bk[k]] + lp[k];
      s_ent[idx] = ent[k];
      s_pb[idx] = pos | (bk[k] << 14);
    }
    __syncthreads();
    prefetch(q + gridDim.x);
    uint32_t id[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t idx = (uint32_t)k * kCountBlock + tid;
      id[k] = 0xFFFFFFFFu;
      if (idx >= nval) continue;
      const uint32_t e = s_ent[idx], b = s_pb[idx] >> 14;
      if (b < nb) {
        c.region[base + idx] = e;  // consecutive lanes, consecutive entries
        id[k] = c.omap[(b << kBucketBits) | (e & (kBucket - 1u))];
      }
    }
    __syncthreads();  // every sorted entry read: s_ent becomes the id array
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t idx = (uint32_t)k * kCountBlock + tid;
      if (idx < nval) s_ent[s_pb[idx] & (kChunk - 1u)] = id[k];
    }
    __syncthreads();
    if (c.out_id) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
        if (p < hi && p < c.out_cap) __builtin_nontemporal_store(s_ent[(uint32_t)k * kCountBlock + tid], &c.out_id[p]);
      }
    }
  }
}

// k_count_chunk in 76 KiB of LDS, so TWO workgroups share a CU and one's barrier
// waits hide under the other's loads and gathers (round 3; k_count_chunk needs
// 132 KiB and ran latency-bound at 2.5 TB/s, one workgroup per CU). Per chunk of
// U * BS = 12288 records:
//  s_rw[pos]  = claim | min(caplen, kLenSat) << 21 of the record at chunk position
//               pos (claims < 510 * 4096 < 2^21 wherever the chunked mode runs;
//               ~0 = no flow); after the gather, the record's output id
//  s_pos[idx] = the chunk position of bucket-sorted entry idx (u16)
// 6 B per record instead of 8. The sorted walk reads s_pos[idx] -> s_rw[pos], stores
// the region entry at region[chunk + idx] and the id back into s_rw[pos] — a slot
// only its own reader touches, so no barrier between the gather and the write-back.
constexpr uint32_t kLenSat = 2047;  // caplens >= kLenSat are re-read from the K1 scratch
// CABL (timing-only ablations, variants build; 0 in product launches): 1 no claim -> id
// gather (id = claim), 2 no region stores, 4 no id stores
template <bool PACK, int BS, int U, int WG_PER_CU = 2, int CABL = 0>
// (WG_PER_CU workgroups of BS / 64 waves on a CU's 4 SIMDs)
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WG_PER_CU * BS / 256, 8)))
void k_count_chunk2(CountArgs c) {
  constexpr int CH = U * BS;
  __shared__ uint32_t s_rw[CH];
  __shared__ uint16_t s_pos[CH];
  __shared__ uint32_t s_ch[kChunkMaxNb + 1], s_co[kChunkMaxNb + 1];
  __shared__ uint32_t s_w[BS / 64];
  static_assert(CH <= (1 << 16) && kChunkMaxNb < BS && (uint64_t)kChunkMaxNb * kBucket < (1u << 21),
                "layout");
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1 || !chunk_scatter(c, nflows) || c.chunk != (uint32_t)CH) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);  // spare bucket: nb
  const uint64_t n_acc = c.batch->n_acc;
  const uint64_t nchunks = (n_acc + CH - 1) / CH;
  const uint32_t lmax = 0xFFFFFFFFu >> c.pack_bits;
  for (uint32_t b = tid; b <= nb; b += BS) s_ch[b] = 0;
  __syncthreads();
  for (uint64_t q = blockIdx.x; q < nchunks; q += gridDim.x) {
    const uint64_t base = q * CH;
    const uint64_t hi = base + CH < n_acc ? base + CH : n_acc;
    const uint32_t nval = (uint32_t)(hi - base);
    uint32_t w[U], lp[U];
    // chunk-relative 32-bit offsets from a uniform base: global loads with an SGPR
    // base address (64-bit per-lane addresses cost the registers that let two
    // workgroups share a CU)
    const uint32_t* af = c.acc_flow + base;
    const uint32_t* al = c.acc_len + base;
    if (kK3LoadPrio) __builtin_amdgcn_s_setprio(kK3LoadPrio);
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * BS + tid;
      w[k] = __builtin_nontemporal_load(&af[pos < nval ? pos : 0u]);
      if (!PACK) lp[k] = __builtin_nontemporal_load(&al[pos < nval ? pos : 0u]);  // (lp: len)
    }
    if (kK3LoadPrio) __builtin_amdgcn_s_setprio(0);
    // decode: claim | min(caplen, kLenSat) << 21 (~0: no flow). A caplen of
    // >= kLenSat (2047 B: never on an IMIX trace) is rare: the wave then redoes its
    // words with the full value (the side array when the packed field saturated) and
    // sends a caplen past the region field to the flow's counter by a device atomic;
    // the common path has no per-word branches (their exec masks cost registers)
    bool rare = false;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * BS + tid;
      const uint32_t v = w[k];
      uint32_t cl = PACK ? (v == 0xFFFFFFFFu ? v : (v & ((1u << c.pack_bits) - 1u))) : v;
      const uint32_t len = PACK ? (v >> c.pack_bits) : lp[k];
      if (pos >= nval) cl = 0xFFFFFFFFu;
      rare |= cl != 0xFFFFFFFFu && len >= kLenSat;
      w[k] = cl == 0xFFFFFFFFu ? 0xFFFFFFFFu : (cl | (len < kLenSat ? len : kLenSat) << 21);
    }
    if (__any(rare)) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t pos = (uint32_t)k * BS + tid;
        const uint32_t cl = w[k] == 0xFFFFFFFFu ? w[k] : (w[k] & 0x1FFFFFu);
        if (cl == 0xFFFFFFFFu || (w[k] >> 21) != kLenSat) continue;
        uint32_t len = PACK ? (af[pos] >> c.pack_bits) : al[pos];
        if (PACK && len == lmax) len = al[pos];  // saturated packed field: the side array
        if (len >= kRegLenEsc) {  // past the region entry's field: counted here
          atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[cl] + 1], (unsigned long long)len);
          w[k] = cl;  // caplen 0 in the region entry
        }
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool valid = (uint32_t)k * BS + tid < nval;
      const uint32_t bk = w[k] == 0xFFFFFFFFu ? nb : (w[k] & 0x1FFFFFu) >> kBucketBits;
      const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk);
      const uint64_t vm = __ballot(valid);
      if (__all(!valid || bk == b0)) {
        // one add for the wave (a hot flow's bucket): ranks in lane order
        uint32_t r0 = 0;
        if (lane == 0 && vm) r0 = atomicAdd(&s_ch[b0], (uint32_t)__popcll(vm));
        r0 = __shfl(r0, 0);
        lp[k] = r0 + (uint32_t)__popcll(vm & lanemask_lt());
      } else {
        lp[k] = valid ? atomicAdd(&s_ch[bk], 1u) : 0u;
      }
    }
    __syncthreads();
    {
      uint32_t tot;
      const uint32_t off = block1024_excl_scan<BS>(tid <= nb ? s_ch[tid] : 0u, s_w, tot);
      if (tid <= nb) s_co[tid] = off;
      if (tid <= nb) c.coffs[q * (kChunkMaxNb + 1) + tid] = off;  // [nb] = end of the real buckets
      if (tid <= nb) s_ch[tid] = 0;  // read by the scan only: zero for the next chunk
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * BS + tid;
      if (pos >= nval) continue;
      const uint32_t bk = w[k] == 0xFFFFFFFFu ? nb : (w[k] & 0x1FFFFFu) >> kBucketBits;
      s_pos[s_co[bk] + lp[k]] = (uint16_t)pos;
      s_rw[pos] = w[k];
    }
    __syncthreads();
    uint32_t* rg = c.region + base;
#pragma unroll 6
    for (int k = 0; k < U; ++k) {
      const uint32_t idx = (uint32_t)k * BS + tid;
      if (idx >= nval) continue;
      const uint32_t pos = s_pos[idx];
      const uint32_t x = s_rw[pos];
      uint32_t id = 0xFFFFFFFFu;
      const uint32_t cl = x & 0x1FFFFFu;
      if (x != 0xFFFFFFFFu && (cl >> kBucketBits) < nb) {
        uint32_t l = x >> 21;
        if (l == kLenSat) {  // a caplen of >= 2047 B: the full value from the K1 scratch
          if (PACK) {
            l = af[pos] >> c.pack_bits;
            if (l == lmax) l = al[pos];
          } else {
            l = al[pos];
          }
        }
        if (!(CABL & 2)) rg[idx] = (cl & (kBucket - 1u)) | l << kBucketBits;  // coalesced runs
        else asm volatile("" ::"v"(l));
        id = (CABL & 1) ? cl : c.omap[cl];  // one bucket's 16 KiB window per wave: L1-local
      }
      s_rw[pos] = id;  // only this thread reads or writes slot pos in this phase
    }
    __syncthreads();
    if (c.out_id && base < c.out_cap && !(CABL & 4)) {
      uint32_t* oi = c.out_id + base;
      const uint32_t lim = c.out_cap - base < nval ? (uint32_t)(c.out_cap - base) : nval;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t pos = (uint32_t)k * BS + tid;
        if (pos < lim) __builtin_nontemporal_store(s_rw[pos], &oi[pos]);
      }
    }
  }
}

// Mode 1, phase 2: workgroup (j, s) histograms bucket j over the segments of K3
// blocks s, s+S, ... (S = gridDim / nb) in LDS; each wave walks one block's
// segment at a time, 4 records per lane in flight. Writes a dense partial row.
__global__ __launch_bounds__(kCountBlock) void k_count_bucket(CountArgs c, uint32_t g1) {
  __shared__ uint64_t s_pk[kBucket], s_by[kBucket];
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1) return;
  const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);
  const uint32_t S = gridDim.x / nb;
  const uint32_t j = blockIdx.x % nb, s = blockIdx.x / nb;
  if (s >= S) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  for (uint32_t t = tid; t < kBucket; t += kCountBlock) s_pk[t] = s_by[t] = 0;
  __syncthreads();
  const uint64_t n_acc = c.batch->n_acc;
  // segments: the two-pass scatter's g1 blocks, or k_count_chunk's chunks
  const bool chunked = chunk_scatter(c, nflows);
  const uint64_t per = chunked ? (uint64_t)c.chunk : count_per(n_acc, g1);
  const uint64_t G = chunked ? (n_acc + c.chunk - 1) / c.chunk : g1;
  const uint32_t* obase = chunked ? c.coffs : c.offs;
  const uint64_t ostride = chunked ? kChunkMaxNb + 1 : c.nb_max + 1;
  constexpr uint32_t kWaves = kCountBlock / 64;
  // This workgroup's segments: bucket j of chunks (blocks) q_k = s + S * k. A wave
  // takes 64 segments at a time — lane l loads segment l's offsets (one load for 64
  // segments) — and walks their records as ONE flattened range of T elements, 64
  // consecutive elements per load: the segments a group of 64 elements touches are
  // found by a wave-uniform walk over the segment starts (readlane, no per-lane
  // search), and element e of segment l sits at region[d_l + e], d_l = start - exc_l.
  // Every region load is independent of the others, so short runs (1M flows: 245
  // buckets, ~50 records per chunk and bucket) no longer cost a dependent offset ->
  // data round trip each (round 2: 0.43 ms per 125M records at 1M flows).
  // Runs of >= 256 records on average (few buckets: 125k flows = 31 buckets,
  // ~400 records per chunk and bucket) go one segment per wave, 4 loads per lane in
  // flight: the run hides the offset round trip, and the flattened walk's scalar
  // segment tracking cost more there (125M records: 166 vs 210 us)
  if (per / nb >= 256) {
    // the next segment's offsets are loaded while this one is counted (one round
    // trip less per segment), 8 records per lane in flight
    auto offs_of = [&](uint64_t q, uint32_t& o0, uint32_t& o1) {
      o0 = o1 = 0;
      if (q < G && q * per < n_acc) {
        const uint32_t* o = obase + q * ostride;
        o0 = o[j];
        o1 = o[j + 1];
      }
    };
    uint32_t o0, o1;
    offs_of(s + S * wave, o0, o1);
    for (uint64_t q = s + S * wave; q < G; q += S * kWaves) {
      const uint64_t lo_q = q * per;
      if (lo_q >= n_acc) break;
      uint32_t n0, n1;
      offs_of(q + S * kWaves, n0, n1);
      const uint64_t a0 = lo_q + o0, a1 = lo_q + o1;
      for (uint64_t x = a0 + lane; x < a1; x += 512) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = __builtin_nontemporal_load(&c.region[x + 64u * u < a1 ? x + 64u * u : x]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (x + 64u * u >= a1) continue;
          const uint32_t t = v[u] & (kBucket - 1);
          atomicAdd((unsigned long long*)&s_pk[t], 1ull);
          atomicAdd((unsigned long long*)&s_by[t], (unsigned long long)(v[u] >> kBucketBits));
        }
      }
      o0 = n0;
      o1 = n1;
    }
  }
  const uint64_t K = per / nb >= 256 ? 0 : (G > s ? (G - s + S - 1) / S : 0);
  for (uint64_t kb = (uint64_t)wave * 64; kb < K; kb += 64ull * kWaves) {
    const uint64_t k = kb + lane;
    uint64_t st = 0;
    uint32_t len = 0;
    if (k < K) {
      const uint64_t q = s + S * k;
      const uint64_t lo_q = q * per;
      if (lo_q < n_acc) {
        const uint32_t* o = obase + q * ostride;
        const uint32_t o0 = o[j], o1 = o[j + 1];
        st = lo_q + o0;
        len = o1 - o0;
      }
    }
    uint32_t inc = len;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d);
      if (lane >= (uint32_t)d) inc += y;
    }
    const uint32_t exc = inc - len;
    const uint64_t dl = st - exc;  // element e of this lane's segment: region[dl + e]
    const uint32_t T = __shfl(inc, 63);
    // wave-uniform: the segment holding the current group's first element, its
    // region offset and the start of the segment after it (scalar registers)
    auto dl_of = [&](uint32_t l) {
      return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(dl >> 32), l) << 32) |
             (uint32_t)__builtin_amdgcn_readlane((uint32_t)dl, l);
    };
    auto exc_of = [&](uint32_t l) { return l < 64 ? (uint32_t)__builtin_amdgcn_readlane(exc, l) : 0xFFFFFFFFu; };
    uint32_t seg = 0;
    uint64_t dseg = dl_of(0);
    uint32_t xnext = exc_of(1);
    for (uint32_t e0 = 0; e0 < T; e0 += 256) {
      uint32_t v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t g0 = e0 + 64u * u;  // first element of this group
        while (xnext <= g0) {  // (empty segments are skipped too)
          ++seg;
          dseg = dl_of(seg);
          xnext = exc_of(seg + 1);
        }
        const uint32_t e = g0 + lane;
        uint64_t d = dseg;
        // segment starts inside this group (none while runs are longer than 64)
        for (uint32_t b = seg + 1, xb = xnext; xb < g0 + 64u; xb = exc_of(++b))
          if (e >= xb) d = dl_of(b);
        v[u] = e < T ? __builtin_nontemporal_load(&c.region[d + e]) : 0u;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (e0 + 64u * u + lane >= T) continue;
        const uint32_t t = v[u] & (kBucket - 1);
        atomicAdd((unsigned long long*)&s_pk[t], 1ull);
        atomicAdd((unsigned long long*)&s_by[t], (unsigned long long)(v[u] >> kBucketBits));
      }
    }
  }
  __syncthreads();
  uint64_t* lp = c.lpart + 2ull * ((uint64_t)s * nb * kBucket + (uint64_t)j * kBucket);
  for (uint32_t t = tid; t < kBucket; t += kCountBlock) {
    lp[2 * t] = s_pk[t];
    lp[2 * t + 1] = s_by[t];
  }
}

// K3 reduce: mode 0 sums the g1 packed partial rows per dense id; mode 1 sums
// the S partial rows per claim and maps claims to ids. cnt is by dense id.
constexpr int kReduceWaves = 16;  // k_count_reduce: 1024-thread blocks
__global__ __launch_bounds__(64 * kReduceWaves) void k_count_reduce(CountArgs c, uint32_t g1, uint32_t g2) {
  const uint64_t nflows = c.batch->flow_total;
  if (c.fused_rank && blockIdx.x == 0 && threadIdx.x == 0) {
    // (fused rank) the batch is classified: the bases K2 would have advanced, now
    // that every k_count block has read the old ones
    c.persist_rw->rec_base += c.batch->n_acc;
    c.persist_rw->flow_count = nflows;
  }
  const int mode = count_mode(c, nflows);
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  if (mode == 0 && nflows * 64 <= stride) {
    // few flows (config 2 has one): one wave per flow, its lanes over the rows —
    // a thread per flow would walk all g1 rows in a dependent-latency chain
    const uint64_t f = t0 >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    if (f < nflows) {
      uint64_t pk = 0, by = 0;
      for (uint32_t b = lane; b < g1; b += 64) {
        const uint64_t v = c.part[(uint64_t)b * kCountBins + f];
        pk += v >> kBinPkShift;
        by += v & kBinByMask;
      }
      pk = wave_sum64(pk);
      by = wave_sum64(by);
      if (lane == 0 && pk) {
        const uint32_t id = c.cmap[f];
        c.cnt[2ull * id] += pk;
        c.cnt[2ull * id + 1] += by;
      }
    }
  } else if (mode == 0) {
    // a block takes 64 consecutive claims (lane = claim) and its waves split the
    // g1 rows (each row read as one 512-B run, 8 rows in flight per lane); the
    // waves' sums meet in LDS — a thread per claim walking all g1 rows was a
    // dependent chain of g1 / 8 load rounds (config 3: 15 us)
    __shared__ uint64_t s_red[2][kReduceWaves][64];
    const uint32_t nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (uint64_t fg = blockIdx.x; fg * 64 < nflows; fg += gridDim.x) {
      const uint64_t f = fg * 64 + lane;
      uint64_t pk = 0, by = 0;
      if (f < nflows) {
        uint32_t b = w;
        for (; b + 7 * nw < g1; b += 8 * nw) {
          uint64_t v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = c.part[(uint64_t)(b + k * nw) * kCountBins + f];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            pk += v[k] >> kBinPkShift;
            by += v[k] & kBinByMask;
          }
        }
        for (; b < g1; b += nw) {
          const uint64_t v = c.part[(uint64_t)b * kCountBins + f];
          pk += v >> kBinPkShift;
          by += v & kBinByMask;
        }
      }
      s_red[0][w][lane] = pk;
      s_red[1][w][lane] = by;
      __syncthreads();
      if (w == 0 && f < nflows) {
        for (uint32_t x = 1; x < nw; ++x) {
          pk += s_red[0][x][lane];
          by += s_red[1][x][lane];
        }
        if (pk) {  // rows are by claim; counters by local dense id
          const uint32_t id = c.cmap[f];
          c.cnt[2ull * id] += pk;
          c.cnt[2ull * id + 1] += by;
        }
      }
      __syncthreads();
    }
  } else if (mode == 3) {
    const uint32_t G = 8u * range_groups_per_x(c, nflows);
    for (uint64_t f = t0; f < nflows; f += stride) {
      uint64_t pk = 0, by = 0;
      for (uint32_t g = 0; g < G; ++g) {
        const uint64_t v = c.part[(uint64_t)g * nflows + f];
        pk += v >> kBinPkShift;
        by += v & kBinByMask;
      }
      if (pk) {
        const uint32_t id = c.cmap[f];
        c.cnt[2ull * id] += pk;
        c.cnt[2ull * id + 1] += by;
      }
    }
  } else if (mode == 1) {
    const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);
    const uint32_t S = g2 / nb;
    const uint64_t row = (uint64_t)nb * kBucket;
    for (uint64_t f = t0; f < nflows; f += stride) {
      uint64_t pk = 0, by = 0;
      for (uint32_t s = 0; s < S; ++s) {
        pk += c.lpart[2 * (s * row + f)];
        by += c.lpart[2 * (s * row + f) + 1];
      }
      if (pk) {
        const uint32_t id = c.cmap[f];
        c.cnt[2ull * id] += pk;
        c.cnt[2ull * id + 1] += by;
      }
    }
  }
}


__global__ void k_finalize(BatchState* b, PersistState* p, uint64_t out_cap, uint64_t* out_n,
                           tcbee_counters* ctr, int direction) {
  const uint64_t n_acc = b->n_acc;
  const uint64_t written = n_acc < out_cap ? n_acc : out_cap;
  if (out_n) *out_n = written;
  if (ctr) {
    if (direction) ctr->egress += n_acc;  // EGRESS_EVENTS, tc.rs:167
    else ctr->ingress += n_acc;           // INGRESS_EVENTS, xdp.rs:207
    ctr->handled += written;              // EVENTS_HANDLED, xdp.rs:214
    ctr->dropped += n_acc - written;      // EVENTS_DROPPED, xdp.rs:217
  }
  p->rec_base += n_acc;
  p->flow_count += b->n_new;
}

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

hipError_t launch_table_init(FlowTable t, hipStream_t s) {
  hipLaunchKernelGGL(k_table_init, dim3(grid_for(4 * t.nlines)), dim3(kBlock), 0, s, t);
  return hipGetLastError();
}

#if TCBEE_VARIANTS
// k1v (TCBEE_K1V at context creation) and the TCBEE_PROBE_AUX / TCBEE_ABLATE /
// TCBEE_STAGE / TCBEE_NT environment: staging, occupancy, cache-policy A/B variants
// and timing-only ablations (several write wrong records on purpose), read at every
// launch (a process may switch them between contexts). Returns true when it
// launched a variant.
template <int FPL>
static bool launch_parse_variant(const ParseArgs& a, bool flows, hipStream_t s, int k1v, dim3 grid) {
  if constexpr (FPL == 2) if (flows && k1v) {
    switch (k1v) {
      case 1: hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 1, false, 0>), grid, dim3(kBlock), 0, s, a); return true;
      case 2: hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 1, false, 5>), grid, dim3(kBlock), 0, s, a); return true;
      case 3: hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 1, false, 6>), grid, dim3(kBlock), 0, s, a); return true;
      // 512-thread tiles (1024 frames): half the tiles and look-back hops (the
      // context sizes ntiles for it: k1_tile_blocks)
      case 20: hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 0, false, 0, 0, 512>), grid, dim3(512), 0, s, a); return true;
#define TCBEE_HPOL_CASE(P) \
      case 10 + P: hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 0, false, 0, P>), grid, dim3(kBlock), 0, s, a); return true;
      TCBEE_HPOL_CASE(1) TCBEE_HPOL_CASE(2) TCBEE_HPOL_CASE(3) TCBEE_HPOL_CASE(4) TCBEE_HPOL_CASE(5)
      TCBEE_HPOL_CASE(6)
#undef TCBEE_HPOL_CASE
      default: return false;
    }
  }
  const int aux = [] {
    const char* e = getenv("TCBEE_PROBE_AUX");
    return e ? atoi(e) : kAuxPlain;
  }();
  const int abl = [] {
    const char* e = getenv("TCBEE_ABLATE");
    return e ? atoi(e) : 0;
  }();
  if (FPL == 2 && abl) {
#define TCBEE_ABL_CASE(B)                                                                      \
  case B:                                                                                      \
    if (flows) hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, B>), grid, dim3(kBlock), 0, s, a); \
    else hipLaunchKernelGGL((k_parse<FPL, false, kAuxPlain, B>), grid, dim3(kBlock), 0, s, a);     \
    return true;
    switch (abl) {
      TCBEE_ABL_CASE(1) TCBEE_ABL_CASE(2) TCBEE_ABL_CASE(4) TCBEE_ABL_CASE(8)
      TCBEE_ABL_CASE(16) TCBEE_ABL_CASE(3) TCBEE_ABL_CASE(31) TCBEE_ABL_CASE(32) TCBEE_ABL_CASE(96)
      TCBEE_ABL_CASE(224) TCBEE_ABL_CASE(352) TCBEE_ABL_CASE(480)
      default: break;
    }
#undef TCBEE_ABL_CASE
  }
  const int stage = [] {
    const char* e = getenv("TCBEE_STAGE");
    return e ? atoi(e) : 0;
  }();
  if (stage == 1) {
    if (flows) hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 1>), grid, dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_parse<FPL, false, kAuxPlain, 0, 1>), grid, dim3(kBlock), 0, s, a);
    return true;
  }
  const int nt = [] {
    const char* e = getenv("TCBEE_NT");
    return e ? atoi(e) : 0;
  }();
  if (nt) {
    if (flows) hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain, 0, 0, true>), grid, dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_parse<FPL, false, kAuxPlain, 0, 0, true>), grid, dim3(kBlock), 0, s, a);
    return true;
  }
  if (flows && aux == kAuxSc1) {
    hipLaunchKernelGGL((k_parse<FPL, true, kAuxSc1>), grid, dim3(kBlock), 0, s, a);
    return true;
  }
  return false;
}
#endif

template <int FPL>
static hipError_t launch_parse_fpl(const ParseArgs& a, bool flows, hipStream_t s, int k1v) {
  const dim3 grid((unsigned)a.ntiles);
#if TCBEE_VARIANTS
  // timing-only ablations and A/B variants: the variants build only
  // (libtcbee_amd_variants.so); the product library has no such dispatch
  if (launch_parse_variant<FPL>(a, flows, s, k1v, grid)) return hipGetLastError();
#else
  (void)k1v;
#endif
  if (flows) hipLaunchKernelGGL((k_parse<FPL, true, kAuxPlain>), grid, dim3(kBlock), 0, s, a);
  else hipLaunchKernelGGL((k_parse<FPL, false, kAuxPlain>), grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_parse(const ParseArgs& a, int fpl, bool flows, hipStream_t s, int k1v) {
  switch (fpl) {
    case 1: return launch_parse_fpl<1>(a, flows, s, k1v);
    case 2: return launch_parse_fpl<2>(a, flows, s, k1v);
    case 4: return launch_parse_fpl<4>(a, flows, s, k1v);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_prep(const PrepArgs& p, hipStream_t s) {
  uint64_t work = p.ntiles;
  if (p.reset && 4 * p.tab.nlines > work) work = 4 * p.tab.nlines;
  // (the wide-slot sweep, when it runs, is grid-strided over the same launch)
  hipLaunchKernelGGL(k_prep, dim3(grid_for(work < 4 ? 4 : work)), dim3(kBlock), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_rank(const RankArgs& r, hipStream_t s) {
  if (r.nwords <= kRankSmallWords) {
    hipLaunchKernelGGL(k_rank_small, dim3(1), dim3(1024), 0, s, r);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_mark, dim3(1024), dim3(kBlock), 0, s, r);
  hipLaunchKernelGGL(k_scan_words, dim3((unsigned)(r.nblocks < 512 ? r.nblocks : 512)), dim3(kBlock),
                     0, s, r);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, r);
  hipLaunchKernelGGL(k_assign, dim3(1024), dim3(kBlock), 0, s, r);
  // (k_scan_blocks advances the record base / flow count; k_assign reads the staged
  //  old ones, and its blocks past n_new return before touching anything)
  return hipGetLastError();
}

#if TCBEE_VARIANTS
static void launch_count_variant(const CountArgs& c, unsigned g1, unsigned g1s, unsigned g2,
                                 hipStream_t s, int k3v) {
  const dim3 grid(g1);
  // k3v (TCBEE_K3ABL at context creation): timing-only ablation / tiling A/B
#define KC(U, A)                                                                     \
  do {                                                                               \
    if (c.pack_bits) hipLaunchKernelGGL((k_count<U, A, true>), grid, dim3(kCountBlock), 0, s, c); \
    else hipLaunchKernelGGL((k_count<U, A, false>), grid, dim3(kCountBlock), 0, s, c);            \
  } while (0)
  switch (k3v) {
    case 1: KC(8, 1); break;
    case 2: KC(8, 2); break;
    case 4: KC(8, 4); break;
    case 7: KC(8, 7); break;
    case 16: KC(16, 0); break;
    case 8: KC(8, 8); break;    // plain id stores (A/B)
    case 24: KC(16, 8); break;  // 16 records per lane, plain id stores (A/B)
    case 32: KC(4, 0); break;
    case 40:  // 16-B loads of four packed words per lane: U = 4 / 2 loads per lane
    case 42:  // (U = 8 spills 328 VGPRs)
      if (c.pack_bits && k3v == 40) hipLaunchKernelGGL((k_count<4, 0, true, true>), grid, dim3(kCountBlock), 0, s, c);
      else if (c.pack_bits) hipLaunchKernelGGL((k_count<2, 0, true, true>), grid, dim3(kCountBlock), 0, s, c);
      else KC(8, 0);
      break;
    default:
      if (c.wide_iter) KC(16, 0);
      else KC(8, 0);
      break;
  }
#undef KC
  // the two-pass scatter only where the chunked one may not cover a batch (tables
  // of >= kChunkMaxNb buckets, or the A/B hook): no empty launches otherwise
  const bool two_pass = !c.coffs || c.chunk_off || c.nb_max >= kChunkMaxNb;
  if (g2 && two_pass) {
    const dim3 gs(g1s);
    switch (k3v) {  // 64 + SABL: timing-only scatter ablations
      case 65: hipLaunchKernelGGL((k_count_scatter<8, false, 1>), gs, dim3(kCountBlock), 0, s, c); break;
      case 66: hipLaunchKernelGGL((k_count_scatter<8, false, 2>), gs, dim3(kCountBlock), 0, s, c); break;
      case 68: hipLaunchKernelGGL((k_count_scatter<8, false, 4>), gs, dim3(kCountBlock), 0, s, c); break;
      case 70: hipLaunchKernelGGL((k_count_scatter<8, false, 6>), gs, dim3(kCountBlock), 0, s, c); break;
      case 80: hipLaunchKernelGGL((k_count_scatter<16, false, 0>), gs, dim3(kCountBlock), 0, s, c); break;
      case 74: hipLaunchKernelGGL((k_count_scatter<8, false, 10>), gs, dim3(kCountBlock), 0, s, c); break;
      case 78: hipLaunchKernelGGL((k_count_scatter<8, false, 14>), gs, dim3(kCountBlock), 0, s, c); break;
      default:
        if (c.pack_bits) hipLaunchKernelGGL((k_count_scatter<8, true>), gs, dim3(kCountBlock), 0, s, c);
        else hipLaunchKernelGGL((k_count_scatter<8, false>), gs, dim3(kCountBlock), 0, s, c);
    }
    // (each of the three returns at once unless the batch's bucket count is its own)
    if (c.pack_bits) hipLaunchKernelGGL((k_count_scatter_staged<4, true>), gs, dim3(kCountBlock), 0, s, c);
    else hipLaunchKernelGGL((k_count_scatter_staged<4, false>), gs, dim3(kCountBlock), 0, s, c);
  }
  if (g2) {
    if (c.coffs && c.chunk == 8u * 1024u && k3v == 95) {  // 52 KiB: three workgroups per CU (A/B)
      const dim3 gc(g1s ? (g1s * 3 + 1) / 2 : 1);
      if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk2<true, 512, 16, 3>), gc, dim3(512), 0, s, c);
      else hipLaunchKernelGGL((k_count_chunk2<false, 512, 16, 3>), gc, dim3(512), 0, s, c);
    } else if (c.coffs && c.chunk == 12u * 1024u) {  // 76 KiB of LDS: two workgroups per CU
      const dim3 gc(g1s ? g1s : 1);
      // 512-thread workgroups, 24 records per thread (TCBEE_K3ABL=94: 1024 x 12, A/B):
      // 125M records, 125k flows (packed words): 470 vs 476 us; 1M flows (unpacked):
      // 705 vs 827 us (round 2's k_count_chunk: 607 / 868 us; profiles/r03_k3ab_*)
      if (k3v == 94) {
        if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk2<true, 1024, 12>), gc, dim3(1024), 0, s, c);
        else hipLaunchKernelGGL((k_count_chunk2<false, 1024, 12>), gc, dim3(1024), 0, s, c);
      } else if (k3v >= 101 && k3v <= 107 && c.pack_bits) {  // 100 + CABL: timing-only ablations
#define TCBEE_CABL_CASE(A) \
        case 100 + A: hipLaunchKernelGGL((k_count_chunk2<true, 512, 24, 2, A>), gc, dim3(512), 0, s, c); break;
        switch (k3v) {
          TCBEE_CABL_CASE(1) TCBEE_CABL_CASE(2) TCBEE_CABL_CASE(3) TCBEE_CABL_CASE(4) TCBEE_CABL_CASE(5)
          TCBEE_CABL_CASE(6) TCBEE_CABL_CASE(7)
        }
#undef TCBEE_CABL_CASE
      } else {
        if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk2<true, 512, 24>), gc, dim3(512), 0, s, c);
        else hipLaunchKernelGGL((k_count_chunk2<false, 512, 24>), gc, dim3(512), 0, s, c);
      }
    } else if (c.coffs && c.chunk == 16u * 1024u) {  // 132 KiB of LDS: one workgroup per CU
      const dim3 gc((g1s + 1) / 2);
      if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk<true, 1024>), gc, dim3(1024), 0, s, c);
      else hipLaunchKernelGGL((k_count_chunk<false, 1024>), gc, dim3(1024), 0, s, c);
    } else if (c.coffs) {  // 8192-record chunks, 68 KiB: two workgroups per CU
      const dim3 gc(g1s ? g1s : 1);
      if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk<true, 512>), gc, dim3(512), 0, s, c);
      else hipLaunchKernelGGL((k_count_chunk<false, 512>), gc, dim3(512), 0, s, c);
    }
    hipLaunchKernelGGL(k_count_bucket, dim3(g2), dim3(kCountBlock), 0, s, c, g1s);
  }
}
#endif

hipError_t launch_count(const CountArgs& c, unsigned g1, unsigned g1s, unsigned g2, hipStream_t s,
                        int k3v) {
#if TCBEE_VARIANTS
  // k3v (TCBEE_K3ABL at context creation): timing-only ablations / tiling A/B —
  // the variants build only
  launch_count_variant(c, g1, g1s, g2, s, k3v);
#else
  (void)k3v;
  const dim3 grid(g1);
  if (c.wide_iter) {  // large batches: 16 records per lane and iteration
    if (c.pack_bits) hipLaunchKernelGGL((k_count<16, 0, true>), grid, dim3(kCountBlock), 0, s, c);
    else hipLaunchKernelGGL((k_count<16, 0, false>), grid, dim3(kCountBlock), 0, s, c);
  } else {
    if (c.pack_bits) hipLaunchKernelGGL((k_count<8, 0, true>), grid, dim3(kCountBlock), 0, s, c);
    else hipLaunchKernelGGL((k_count<8, 0, false>), grid, dim3(kCountBlock), 0, s, c);
  }
  // the two-pass scatter only where the chunked one may not cover a batch (tables
  // of >= kChunkMaxNb buckets): no empty launches otherwise
  const bool two_pass = !c.coffs || c.nb_max >= kChunkMaxNb;
  if (g2 && two_pass) {
    const dim3 gs(g1s);
    // (each of the two returns at once unless the batch's bucket count is its own)
    if (c.pack_bits) {
      hipLaunchKernelGGL((k_count_scatter<8, true>), gs, dim3(kCountBlock), 0, s, c);
      hipLaunchKernelGGL((k_count_scatter_staged<4, true>), gs, dim3(kCountBlock), 0, s, c);
    } else {
      hipLaunchKernelGGL((k_count_scatter<8, false>), gs, dim3(kCountBlock), 0, s, c);
      hipLaunchKernelGGL((k_count_scatter_staged<4, false>), gs, dim3(kCountBlock), 0, s, c);
    }
  }
  if (g2) {
    if (c.coffs) {
      // 12288-record chunks in 76 KiB of LDS: two 512-thread workgroups per CU
      const dim3 gc(g1s ? g1s : 1);
      if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk2<true, 512, 24>), gc, dim3(512), 0, s, c);
      else hipLaunchKernelGGL((k_count_chunk2<false, 512, 24>), gc, dim3(512), 0, s, c);
    }
    hipLaunchKernelGGL(k_count_bucket, dim3(g2), dim3(kCountBlock), 0, s, c, g1s);
  }
#endif
  // mode 0 needs kCountBins threads; mode 1 up to nb_max * kBucket (grid-stride)
  // (1024-thread blocks: mode 0 takes 64 claims per block, its 16 waves split the rows)
  const unsigned gr = (g2 || c.range_ok) ? 256u : (unsigned)(kCountBins / 256);
  // (a fused-rank batch has no reduce: k_count adds its bins and advances the bases)
  if (!c.fused_rank)
    hipLaunchKernelGGL(k_count_reduce, dim3(gr), dim3(64 * kReduceWaves), 0, s, c, g1, g2);  // g1: mode-0 rows
  return hipGetLastError();
}

hipError_t launch_finalize(BatchState* b, PersistState* p, uint64_t out_cap, uint64_t* out_n,
                           tcbee_counters* ctr, int direction, hipStream_t s) {
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1), 0, s, b, p, out_cap, out_n, ctr, direction);
  return hipGetLastError();
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
  // same step time once the LDS map was u16: TCBEE_REMAP_GRID, variants build)
#if TCBEE_VARIANTS
  static const uint64_t gmax = [] {
    const char* e = getenv("TCBEE_REMAP_GRID");
    const long long v = e ? atoll(e) : 0;
    return v > 0 ? (uint64_t)v : 512ull;  // unset, 0 or garbage: the default
  }();
#else
  constexpr uint64_t gmax = 512;
#endif
  const uint64_t want = (n_max + 4ull * kRemapBlock - 1) / (4ull * kRemapBlock);
  hipLaunchKernelGGL(k_remap, dim3((unsigned)(want < gmax ? (want ? want : 1) : gmax)),
                     dim3(kRemapBlock), 0, s, ids, n_max, n_dev, map,
                     map_len);
  return hipGetLastError();
}

hipError_t launch_gen(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                      uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed,
                      hipStream_t s, const uint64_t* gidx, const uint64_t* zcdf) {
  hipLaunchKernelGGL(k_gen, dim3(grid_for(n, 8192)), dim3(kBlock), 0, s, arena, off, len, n,
                     first_index, kind, n_flows, seed, gidx, zcdf);
  return hipGetLastError();
}

}  // namespace tcbee

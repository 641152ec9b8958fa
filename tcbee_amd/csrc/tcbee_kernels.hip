// tcbee_kernels.hip — HIP kernels (gfx950) of the packet-record path, K1-K3.
//
//   K1 k_parse     one lane per frame: bounds/ethertype/proto/port checks,
//                  fixed-offset header extraction, the 74-B record, the flow
//                  key + hash + flow-table upsert (tcbee_table.h), and
//                  ORDER-PRESERVING compaction of the records (decoupled look-back
//                  over the tiles), records staged in LDS and stored as 16-B
//                  vectors. Restates xdp_hook / tc_hook (tcbee-ebpf/src/probes/
//                  xdp.rs:27-223, tc.rs:28-183) + FLOWS insert (flow_tracker.rs:
//                  17-23) + the drain task's serializer (tcbee/src/handlers/mod.rs:
//                  104-139).
//   K2 k_rank_small | k_mark / k_scan_words / k_scan_blocks / k_assign
//                  dense flow ids in first-seen order (the order in which
//                  tcbee-process creates flows, db_writer.rs:51-65).
//   K3 k_count (+ k_count_chunk2 / k_count_bucket, or the two-pass scatter, for
//                  large tables) + k_count_reduce: per record claim -> output id,
//                  pkts/bytes per flow; block 0 finalizes the counters
//                  (counters.rs:43-83).
// The N>1 exchange kernels are in tcbee_exchange.hip, the synthetic-trace
// generators in tcbee_synth.hip.
#include <cstdlib>

#include "tcbee_table.h"

namespace tcbee {

// Look-back polling bounds, in wall-clock ticks (wall_clock64: 100 MHz on MI355X,
// hipDeviceAttributeWallClockRate): a wave polls an unpublished predecessor for
// 10 us before recounting it from the input, then 1 us for each further one.
// Bounded by time, not by a poll count: a poll is an agent-scope load of a few
// hundred ns to a few us, and 4096 of them (round 1-4) let a wave spin for
// milliseconds when a predecessor's XCD had fallen behind -- with a second process's
// kernels on the GPU, K1 took 20-200x its time alone. A
// recounted aggregate is also published in the predecessor's status word (a CAS
// from "unpublished": the value is the one the predecessor itself will store).
#ifndef TCBEE_RECOUNT_TICKS
#define TCBEE_RECOUNT_TICKS 1000
#endif
#ifndef TCBEE_RECOUNT_LATE
#define TCBEE_RECOUNT_LATE 100
#endif
// K1's wave priority while a tile's index and header loads are issued (then 0):
// a starting wave issues its loads ahead of resident waves' parse / record work
// (config 3 K1 -2.6 %, round 3; priority 3 and a K3 load-phase priority measured
// no different, round 4)
constexpr int kK1LoadPrio = 2;

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

__device__ __forceinline__ void put_chunk(uint32_t (&w)[24], int c, uint4 v) {
  w[4 * c + 0] = v.x; w[4 * c + 1] = v.y; w[4 * c + 2] = v.z; w[4 * c + 3] = v.w;
}

// Header window of FPL frames: 16-B aligned chunks 0..4 from off & ~15 (all an
// IPv4 frame needs: s + 54 <= 69 < 80). When every lane's 80 B lie inside the
// arena (the common case) all FPL x 5 loads are issued unconditionally, back to
// back; otherwise each lane loads only the chunks of [off, off+min(len,54)),
// bounds-checked. Chunk 5 (IPv6 tail) is loaded later, for IPv6 frames only.
// (Explicit cache policies nt / sc0 / sc1 on these loads fill the same 128-B lines
// and were up to 20 % slower, round 2.)
template <int FPL>
__device__ __forceinline__ void load_windows(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                             const uint64_t (&off)[FPL], const uint32_t (&len)[FPL],
                                             uint32_t (&w)[FPL][24]) {
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
        if ((uint32_t)c >= c_lo && (uint32_t)c <= c_hi) v = src[c];
        q[f][c] = v;
      }
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

__device__ __forceinline__ bool parse_window(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                             uint64_t off, uint32_t caplen, uint64_t ts,
                                             uint32_t filter_port, uint32_t (&w)[24],
                                             uint32_t (&R)[19], uint64_t (&K)[5]) {
  if (caplen < kEthHdrLen) return false;  // xdp.rs:37-39
  const uint64_t abase = off & ~15ull;
  const uint32_t s = (uint32_t)(off & 15u);
  {
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
// whose word stays unpublished for TCBEE_RECOUNT_TICKS (not yet dispatched, or
// slow) has its aggregate recounted from the input by this wave (and published for
// it), so the walk always terminates; results never depend on which block
// publishes first.
template <int TILE>
__device__ uint64_t lookback_resolve(const ParseArgs& a, uint64_t tile, uint64_t count,
                                    bool withhold) {
  const uint32_t lane = __lane_id();
  if (tile == 0) return 0;
  uint64_t* status = a.tile_status;
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  int64_t wait = TCBEE_RECOUNT_TICKS;
  for (;;) {
    const int64_t idx = base - (int64_t)lane;
    uint64_t v = idx >= 0 ? ld_agent(status + idx) : kFlagInc;
    int64_t t0 = wall_clock64();
    for (;;) {
      const uint64_t inv = __ballot((v >> 62) == 0);
      if (!inv) break;
      // only the invalid lanes nearer than the nearest inclusive prefix matter
      const uint64_t inc = __ballot((v >> 62) == 2);
      const uint64_t need = inc ? (inv & ((inc & (~inc + 1)) - 1)) : inv;
      if (!need) break;
      if (wall_clock64() - t0 > wait) {
        const uint32_t j = (uint32_t)__ffsll((unsigned long long)need) - 1;
        const uint32_t cnt = tile_accept_count<TILE>(a, (uint64_t)(base - (int64_t)j));
        if (lane == j) {
          // published on the predecessor's behalf (if it still has not): the other
          // successors waiting on it stop polling instead of each recounting it
          v = kFlagAgg | cnt;
          atomicCAS(reinterpret_cast<unsigned long long*>(status + idx), 0ull,
                    (unsigned long long)v);
        }
        t0 = wall_clock64();
        wait = TCBEE_RECOUNT_LATE;
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
  load_windows<1>(arena, arena_len, o, l, w);
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
      // non-temporal (round 6: the records are written once and read by the host or
      // the next stage, never by this kernel; config 3 K1 -3.8 %, the share -1.7 %,
      // profiles/r06_store_nt_ab.log — round 1's non-temporal record stores, issued
      // lane by lane before the LDS staging existed, were slower)
      __builtin_nontemporal_store(ov, reinterpret_cast<u32x4*>(out + g));
    } else {
      const uint64_t lo = g > G0 ? g : G0;
      const uint64_t hi = (g + 16) < G1 ? (g + 16) : G1;
      for (uint64_t b = lo; b < hi; b += 2)
        *reinterpret_cast<uint16_t*>(out + b) = s16[(b - G0) >> 1];
    }
  }
}

// ---------------------------------------------------------------------------
// K1
// ---------------------------------------------------------------------------
// One tile of FPL x kBlock frames per block (tile = blockIdx.x). The tile's records
// are staged in LDS at their compacted positions and stored by the whole block
// after the look-back (a per-wave staging was slightly slower, round 2).
template <int FPL, bool FLOWS>
__global__ __launch_bounds__(kK1Block) void k_parse(ParseArgs a) {
  constexpr int TILE = kK1Block * FPL;
  constexpr int NW = kK1Block / 64;  // waves per tile
  constexpr int SREC_DW = (TILE * kRecBytes + 32) / 4;
  __shared__ __attribute__((aligned(16))) uint32_t s_rec[SREC_DW];
  __shared__ uint32_t s_wcnt[FPL][NW];
  __shared__ uint64_t s_excl;
  // per wave and frame group: the slot and record index its all-one-slot group would
  // compete with for first_seen (~0: none), merged per tile at the end
  __shared__ uint32_t s_fsl[NW * FPL], s_fsp[NW * FPL];

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
    const uint64_t i = i0 + (uint64_t)f * kK1Block + tid;
    acc[f] = false;
    slot[f] = 0xFFFFFFFFu;
    claim[f] = 0xFFFFFFFFu;
    hsh[f] = 0;
    fs_seen[f] = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < 5; ++j) K[f][j] = 0;
    const bool in = i < a.n;
    const uint64_t ic = in ? i : a.n - 1;  // loads stay unconditional (no branch per frame)
    // the streamed-once index with the non-temporal hint (round 6: config 3 K1 -1.0 %,
    // the share -0.4 %, profiles/r06_idx_nt_ab.log; the header windows keep the
    // default policy — nt there filled the same lines and was 20 % slower, round 2)
    const uint64_t o = __builtin_nontemporal_load(&a.offset[ic]);
    const uint32_t l = __builtin_nontemporal_load(&a.caplen[ic]);
    tsv[f] = __builtin_nontemporal_load(&a.ts[ic]);
    offv[f] = in ? o : 0;
    clen[f] = in ? l : 0;
  }
  uint32_t lenc[FPL];
#pragma unroll
  for (int f = 0; f < FPL; ++f) lenc[f] = clamp_caplen(offv[f], clen[f], a.arena_len);
  {
    uint32_t W[FPL][24];
    load_windows<FPL>(a.arena, a.arena_len, offv, lenc, W);
#pragma unroll
    for (int f = 0; f < FPL; ++f)
      acc[f] = parse_window(a.arena, a.arena_len, offv[f], lenc[f], tsv[f], a.filter_port, W[f],
                            R[f], K[f]);
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
  if (!withhold && tid == 0) lookback_publish(a.tile_status, tile, total);

  bool staged_early = FLOWS;
  if (FLOWS) {
    // phase B: hash, then issue the first probe's loads of every frame: an IPv4-form
    // key's 16-B compact slot + its fs32 (one line), any other key's 64-B wide slot
    u32x4 Q[FPL][4];
    uint32_t FS[FPL], S0[FPL], leader[FPL];
    bool v4k[FPL], uni[FPL], want[FPL];
    uint64_t h[FPL];
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
      // a frame group whose wave-uniform key is frame group 0's too (a hot flow):
      // no probe of its own, group 0's result below (round 6: config 2's step -2.8 %,
      // half the probes and inserts of a hot new flow; profiles/r06_config2_attempts.log)
      if (f > 0 && uni[f] && uni[0]) {
        bool eq = true;
#pragma unroll
        for (int j = 0; j < 5; ++j) eq = eq && K[f][j] == K[0][j];
        if (__all(!acc[f] || !acc[0] || eq) && __any(acc[f] && acc[0])) want[f] = false;
      }
      v4k[f] = key_is_v4form(K[f]);
      if (want[f]) {
        // Plain (cacheable) loads are exact here: a claimer stores everything a
        // reader compares (drained) before the word that publishes the slot, in the
        // same line; a stale snapshot shows EMPTY/BUSY or a mismatch, and every such
        // miss falls through to flow_upsert's coherent path.
        if (v4k[f]) {
          S0[f] = home_slot(h[f], a.tab.nlines);
          const uint32_t l = slot_line(S0[f]), pos = S0[f] - l * kSlotsPerLine;
          Q[f][0] = __builtin_amdgcn_raw_buffer_load_b128(sl_rs, l * 64u + 16u * pos, 0, 0);
          // (the slot and its fs32 share one 64-B half-line: the two halves of a
          //  128-B line can be of different ages in L1/L2 — a fresh published slot
          //  beside a stale fs32 lost first_seen values when fs32 sat in the other half)
          FS[f] = __builtin_amdgcn_raw_buffer_load_b32(sl_rs, l * 64u + 48u + 4u * pos, 0, 0);
        } else {
          S0[f] = (uint32_t)(h[f] & a.tab.wide_mask);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            Q[f][j] = __builtin_amdgcn_raw_buffer_load_b128(wd_rs, S0[f] * 64u + 16u * j, 0, 0);
        }
      }
    }
    // the records' LDS staging while the first probes are in flight, in waves whose
    // probes are all compact (IPv4-form) ones; a wave with a wide-slot probe (4 x 16-B
    // loads per frame in flight) stages after the walk, as before (round 5, A/B of 3
    // alternating rounds, K1: config 3 -2.2 %, the N=8 share -1.1 %, 1M flows -0.8 %,
    // IPv6 equal; staging early in every wave: config 3 -1.0 %, IPv6 +0.5 %)
    bool wide_wave = false;
#pragma unroll
    for (int f = 0; f < FPL; ++f) wide_wave = wide_wave || (want[f] && !v4k[f]);
    staged_early = !__any(wide_wave);
    if (staged_early) {
#pragma unroll
      for (int f = 0; f < FPL; ++f)
        if (acc[f]) lds_put_record(s_rec, rank[f] * kRecBytes, R[f]);
    }
    // phase C: resolve; a miss (new flow, busy slot, a stale snapshot) takes the full
    // upsert. Walk on with plain loads while the slots hold OTHER flows (published,
    // another key): within a batch a slot only goes EMPTY -> BUSY -> published, so a
    // published foreign slot seen in any snapshot is foreign for good; EMPTY/BUSY may
    // be stale and end the walk. A wide slot whose tag equals ours but whose key
    // differs goes to the coherent path (it may be a stale snapshot of our flow).
    // (Resolving a snapshot miss after the tile's records are stored instead was no
    //  faster, round 4.)
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
          for (uint32_t step = 0;; ++step) {
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
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(sl_rs, l * 64u + 16u * pos, 0, 0);
            fsv = __builtin_amdgcn_raw_buffer_load_b32(sl_rs, l * 64u + 48u + 4u * pos, 0, 0);
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
            for (int j = 0; j < 4; ++j) q[j] = __builtin_amdgcn_raw_buffer_load_b128(wd_rs, s * 64u + 16u * j, 0, 0);
#pragma unroll
            for (int j = 0; j < 7; ++j) {
              const u32x4 v = q[j >> 1];
              V[j] = (j & 1) ? ((uint64_t)v[2] | ((uint64_t)v[3] << 32)) : ((uint64_t)v[0] | ((uint64_t)v[1] << 32));
            }
          }
        }
        if (slow)
          sl = flow_upsert(a.tab, K[f], h[f], a.batch, a.new_list, a.persist, fbase, fs, cl,
                           kFs32Flag | (uint32_t)(i0 + (uint64_t)f * kK1Block + tid));
      }
      // a wave-uniform key: the leader's result for the whole wave
      if (f > 0 && uni[f] && !__any(want[f])) {  // group 0's flow (above)
        slot[f] = slot[0];
        claim[f] = claim[0];
        fs_seen[f] = fs_seen[0];
      } else if (uni[f]) {
        slot[f] = __shfl(sl, leader[f]);
        claim[f] = __shfl(cl, leader[f]);
        fs_seen[f] = __shfl(fs, leader[f]);
      } else if (acc[f]) {
        slot[f] = sl;
        claim[f] = sl == 0xFFFFFFFFu ? 0xFFFFFFFFu : cl;
        fs_seen[f] = fs;
      }
    }
  }
  if (!FLOWS || !staged_early) {
#pragma unroll
    for (int f = 0; f < FPL; ++f)
      if (acc[f]) lds_put_record(s_rec, rank[f] * kRecBytes, R[f]);
  }

  // (wave 0 resolving the look-back before its own probes instead — its inclusive
  //  prefix published a probe phase earlier — was 22 % slower, round 3)
  if (wave == 0) {
    const uint64_t excl = lookback_resolve<TILE>(a, tile, total, withhold);
    if (lane == 0) s_excl = excl;
  }
  __syncthreads();
  const uint64_t excl = s_excl;
  if (tid == 0 && tile == a.ntiles - 1) a.batch->n_acc = excl + total;

  // ---- records: LDS -> HBM, 16-B stores, partial chunks as 2-B stores ----
  // (non-temporal 16-B stores, see copy_out)
  {
    const uint64_t wr_lo = excl < a.out_cap ? excl : a.out_cap;
    const uint64_t wr_hi = (excl + total) < a.out_cap ? (excl + total) : a.out_cap;
    if (wr_hi > wr_lo) copy_out(a.out_rec, wr_lo * kRecBytes, wr_hi * kRecBytes, s_rec, tid, kK1Block);
  }

  // ---- per-record side outputs; first_seen = min accepted index ----
  // (pkts/bytes are NOT counted here: per-record memory-side atomics cost more
  //  than the whole parse; k_count histograms them by dense id in LDS.)
  uint32_t prev_s0 = 0xFFFFFFFFu;  // slot of the wave's last all-one-slot new-flow group
#pragma unroll
  for (int f = 0; f < FPL; ++f) {
    const uint64_t p = excl + rank[f];
    if (acc[f]) {
      // (side words non-temporal too: -0.35 % on config 3's K1, round 6)
      if (a.out_hash && p < a.out_cap) __builtin_nontemporal_store(hsh[f], &a.out_hash[p]);
      // record -> frame map (flow-hash shards of traces with rejected frames)
      if (a.out_frame && p < a.out_cap) a.out_frame[p] = (uint32_t)(i0 + (uint64_t)f * kK1Block + tid);
      if (FLOWS) {
        if (a.pack_bits) {
          // (claim, caplen) in one word; a caplen that does not fit saturates the
          // field and is stored in full beside it (K3 reads it only then)
          const uint32_t lmax = 0xFFFFFFFFu >> a.pack_bits;
          const uint32_t lq = clen[f] < lmax ? clen[f] : lmax;
          __builtin_nontemporal_store(claim[f] == 0xFFFFFFFFu ? 0xFFFFFFFFu : claim[f] | (lq << a.pack_bits),
                                      &a.acc_flow[p]);
          if (lq == lmax) a.acc_len[p] = clen[f];
        } else {
          a.acc_flow[p] = claim[f];
          a.acc_len[p] = clen[f];
        }
      }
    }
    if (FLOWS) {
      // first_seen competition: only flows new in this batch (claim >= fbase)
      const bool mine = acc[f] && slot[f] != 0xFFFFFFFFu && claim[f] >= fbase;
      const uint64_t am = __ballot(mine);
      if (lane == 0) s_fsp[wave * FPL + f] = 0xFFFFFFFFu;
      if (am) {
        const uint32_t leader = (uint32_t)__ffsll((unsigned long long)am) - 1;
        const uint32_t s0 = __shfl(slot[f], leader);
        const uint32_t p32 = (uint32_t)p;
        const uint32_t frame_i = (uint32_t)(i0 + (uint64_t)f * kK1Block + tid);
        if (__all(!mine || slot[f] == s0)) {
          // leader = lowest rank of the wave = its smallest accepted index; when the
          // wave's previous frame group was all this slot too, its earlier leader
          // competes for both (a hot new flow: one add per wave, not per group)
          const bool first = s0 != prev_s0;
          prev_s0 = s0;
          if (first && lane == leader && fs_needs_min(fs_seen[f], frame_i, p32)) {
            s_fsl[wave * FPL + f] = s0;
            s_fsp[wave * FPL + f] = p32;
          }
        } else if (mine && fs_needs_min(fs_seen[f], frame_i, p32)) {
          atomicMin(slot_fs_any(a.tab, slot[f]), p32);
        }
      }
    }
  }
  if (FLOWS) {
    // One competitor per slot and tile: the tile's smallest candidate, and only when
    // the word, re-read, is still larger. A hot flow new in the batch (config 2's one
    // flow, a Zipf head) otherwise sent one same-address device atomic per wave
    // whose frames precede the claimer's — ~2000 of them when a late wave of the first
    // dispatch round won the insert, serialized at the coherence point (round 6,
    // profiles/r06_config2_attempts.log: config 2's K1 mean 50.5-56.2 -> 44.1-44.6 us,
    // p90 63-90 -> 46-47 us, max 112-119 -> 50-51 us; with a warm table, no inserts
    // and no competition, it is 38.3 us).
    __syncthreads();
    if (tid < NW * FPL) {
      const uint32_t p0 = s_fsp[tid];
      if (p0 != 0xFFFFFFFFu) {
        const uint32_t sl0 = s_fsl[tid];
        uint32_t best = p0;
        bool owner = true;
#pragma unroll
        for (int e = 0; e < NW * FPL; ++e) {
          const uint32_t pe = s_fsp[e];
          if (pe == 0xFFFFFFFFu || s_fsl[e] != sl0 || e == (int)tid) continue;
          if (e < (int)tid) owner = false;
          best = pe < best ? pe : best;
        }
        // (an earlier tile has often lowered the word by now: a stale read is only
        //  ever larger, so the atomic is at worst redundant)
        if (owner && ld_agent32(slot_fs_any(a.tab, sl0)) > best)
          atomicMin(slot_fs_any(a.tab, sl0), best);
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

// Mode 1, phase 1 (tables past the chunked pass): ids out, bucket counts, scan, scatter.
// STAGED (nb <= kSmallNb): pass 2 counting-sorts each chunk of U x 1024 entries
// by bucket in LDS (stage / sb / ch / co) and stores them as per-bucket runs.
struct ScatterStage {
  uint32_t* stage;  // [U * kCountBlock] entries of one chunk, bucket-sorted
  uint16_t* sb;     // their buckets
  uint32_t* ch;     // [kSmallNb + 1] chunk counts per bucket (+ spare)
  uint32_t* co;     // [kSmallNb + 1] chunk offsets per bucket
};

template <int U, bool PACK, bool STAGED = false>
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
    {
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

// Bins are indexed by CLAIM (dense in [0, F)); the record's output id is
// omap[claim] (the local dense id, or — after a flow-hash exchange — the global
// one), staged in LDS; k_count_reduce maps claims to local ids for the counters.
// U records per lane and iteration: 8, or 16 on batches of >= kK3WideFrames (twice
// the loads in flight). (16-B loads of four packed words, buffer-addressed 16/24-record
// iterations and plain id stores were measured no faster, round 4: K3 mode 0 is bound
// by its id stores, which serialize with the record-word reads.)
template <int U, bool PACK>
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
  for (uint64_t base = lo; base < hi; base += (uint64_t)U * kCountBlock) {
    uint32_t s[U], len[U], id[U];
    load_acc<U, PACK>(c, base + tid, lo, hi, s, len);  // streamed once: non-temporal
    if (mode == 0) {
#pragma unroll
      for (int k = 0; k < U; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : s_map[s[k]];
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) id[k] = s[k] == 0xFFFFFFFFu ? 0xFFFFFFFFu : c.omap[s[k]];
    }
    if (c.out_id) {
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint64_t p = base + (uint64_t)k * kCountBlock + tid;
        if (p < hi && p < c.out_cap) __builtin_nontemporal_store(id[k], &c.out_id[p]);
      }
    }
    if (mode == 0) {
      // one flow in all of the wave's records this iteration (a hot flow): one add
      const uint32_t s0 = __builtin_amdgcn_readfirstlane(s[0]);
      bool same = s0 != 0xFFFFFFFFu;
      uint32_t nk = 0, sl = 0;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const bool v = s[k] != 0xFFFFFFFFu;
        same = same && (!v || (s[k] == s0 && len[k] < kBigLen));
        nk += v ? 1u : 0u;
        sl += v ? len[k] : 0u;
      }
      if (__all(same)) {
        // pk <= 64*U, by <= 64*U*(kBigLen-1) < 2^32 at U <= 32 (sums in 64 bits)
        const uint64_t pk = wave_sum64(nk), by = wave_sum64(sl);
        if (lane == 0)
          atomicAdd((unsigned long long*)&s_bin[s0], ((unsigned long long)pk << kBinPkShift) | by);
      } else {
#pragma unroll
        for (int k = 0; k < U; ++k) {
          if (s[k] == 0xFFFFFFFFu) continue;
          if (len[k] < kBigLen)
            atomicAdd((unsigned long long*)&s_bin[s[k]], (1ull << kBinPkShift) | len[k]);
          else
            global_add(s[k], 1, len[k]);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < U; ++k) {
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
    // Invariant: no block reads persist after its k3_done add. Every
    // read of rec_base / flow_count in this kernel happens before the __syncthreads
    // above, whose workgroup release waits for the block's outstanding loads, so a
    // relaxed add suffices: the last block's writes below cannot reach a read that
    // some block has not completed (no agent-scope release, which would write back
    // the XCD's L2, is needed for that ordering).
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
// the single-pass chunked scatter (k_count_chunk2) takes every mode-1 batch of up to
// kChunkMaxNb - 1 buckets when the context has its chunk offsets
__device__ __forceinline__ bool chunk_scatter(const CountArgs& c, uint64_t nflows) {
  const uint64_t nb = (nflows + kBucket - 1) >> kBucketBits;
  return c.coffs != nullptr && !c.chunk_off && nb < kChunkMaxNb;
}
__device__ __forceinline__ bool staged_scatter(const CountArgs& c, uint64_t nflows) {
  const uint64_t nb = (nflows + kBucket - 1) >> kBucketBits;
  return nb >= kStagedMinNb && nb <= kSmallNb && !chunk_scatter(c, nflows);
}

template <int U, bool PACK>
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
  count_scatter<U, PACK>(c, lo, hi, nflows, s_hist, s_cur, s_w);
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
  count_scatter<U, PACK, true>(c, lo, hi, nflows, s_hist, s_cur, s_w, st);
}

// Mode 1, single pass (nb < kChunkMaxNb): each 512-thread workgroup takes chunks of
// kChunk = 12288 accepted records (24 per thread) and
//  1. ranks them by sub-bin in LDS (counts per sub-bin, one LDS add per record or one
//     per wave when the wave's records share a sub-bin; no-flow records go to a spare
//     sub-bin nsb), scans the counts;
//  2. places every record's WORD at its sorted slot (s_srt[idx] = claim | caplen),
//     the thread keeping each of its records' slot idx in a register;
//  3. walks the sorted slots with consecutive lanes on consecutive entries: the
//     region entry (claim within the bucket | caplen) is stored coalesced at
//     region[chunk + idx] (the chunk's buckets are contiguous runs; coffs[q] = their
//     offsets for k_count_bucket), the claim -> output id gather reads omap inside a
//     few sub-bins' windows per wave (a record-order gather hits a random line of the
//     whole map per lane: 692 us per 125M records at 125k flows, tools/
//     k3_gather_floor.hip), and the id replaces the word in the slot just read;
//  4. stores the chunk's ids in record order, coalesced: each thread reads its
//     records' slots back.
// One pass over the K1 -> K3 words, no per-block cursors, no scattered stores.
// Round 6: the words themselves at their sorted slots — round 3-5 sorted u16
// positions (s_pos[idx] = pos) beside a record-order word array (s_rw[pos]), one more
// random LDS access per record (five: the ranking add, the s_co read, the position
// scatter, the walk's s_rw[pos] read and write-back; now four) and 6 B of LDS per
// record instead of 4; its scratch spill (24 B/lane) is gone too. Per 100M records,
// same box, alternating processes (profiles/r06_k3_ab.log): 125k flows 322.5 -> 296.5
// us, 1M flows 498.4 -> 480.9 us. Refuted in the same A/B: three workgroups per CU
// (6 waves/SIMD: 96 B/lane of spills, 366 / 633 us), 16384-record chunks (spills,
// 354 / 504) and 1024-thread workgroups of 24576 records (335 / 530; their longer
// bucket runs took k_count_bucket at 1M flows 156 -> 125 us, not enough).
// Every caplen of >= kLenSat (2047 B: never on an IMIX trace) goes to the flow's
// counter by a device atomic in phase 1 and its region entry carries caplen 0, so the
// walk never needs the record's position (round 5 re-read it there).
// 52 KiB of LDS and 128 VGPRs: two workgroups per CU (4 waves / SIMD).
constexpr uint32_t kLenSat = 2047;  // caplens >= kLenSat: bytes by a device atomic
template <bool PACK>
__global__ __launch_bounds__(kChunkBlock) __attribute__((amdgpu_waves_per_eu(2 * kChunkBlock / 256, 8)))
void k_count_chunk2(CountArgs c) {
  constexpr int BS = kChunkBlock, U = kChunk / kChunkBlock, CH = kChunk;
  __shared__ uint32_t s_srt[CH];
  __shared__ uint32_t s_ch[kChunkMaxNb + 1], s_co[kChunkMaxNb + 1];
  __shared__ uint32_t s_w[BS / 64];
  const uint64_t nflows = c.batch->flow_total;
  if (count_mode(c, nflows) != 1 || !chunk_scatter(c, nflows)) return;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t nb = (uint32_t)((nflows + kBucket - 1) >> kBucketBits);
  uint32_t sh = 8;
  while (sh < kBucketBits && ((nflows + (1ull << sh) - 1) >> sh) >= kChunkMaxNb) ++sh;
  const uint32_t nsb = (uint32_t)((nflows + (1ull << sh) - 1) >> sh);
  const uint32_t rsh = kBucketBits - sh;
  const uint64_t n_acc = c.batch->n_acc;
  const uint64_t nchunks = (n_acc + CH - 1) / CH;
  const uint32_t lmax = 0xFFFFFFFFu >> c.pack_bits;
  for (uint32_t b = tid; b <= nsb; b += BS) s_ch[b] = 0;
  __syncthreads();
  for (uint64_t q = blockIdx.x; q < nchunks; q += gridDim.x) {
    const uint64_t base = q * CH;
    const uint64_t hi = base + CH < n_acc ? base + CH : n_acc;
    const uint32_t nval = (uint32_t)(hi - base);
    uint32_t w[U], lp[U];
    const uint32_t* af = c.acc_flow + base;
    const uint32_t* al = c.acc_len + base;
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * BS + tid;
      w[k] = __builtin_nontemporal_load(&af[pos < nval ? pos : 0u]);
      if (!PACK) lp[k] = __builtin_nontemporal_load(&al[pos < nval ? pos : 0u]);
    }
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
    if (__any(rare)) {  // caplens of >= kLenSat: their bytes by a device atomic, field 0
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t pos = (uint32_t)k * BS + tid;
        const uint32_t cl = w[k] == 0xFFFFFFFFu ? w[k] : (w[k] & 0x1FFFFFu);
        if (cl == 0xFFFFFFFFu || (w[k] >> 21) != kLenSat) continue;
        uint32_t len = PACK ? (af[pos] >> c.pack_bits) : al[pos];
        if (PACK && len == lmax) len = al[pos];
        if ((cl >> kBucketBits) < nb)
          atomicAdd((unsigned long long*)&c.cnt[2ull * c.cmap[cl] + 1], (unsigned long long)len);
        w[k] = cl;
      }
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const bool valid = (uint32_t)k * BS + tid < nval;
      const uint32_t bk = w[k] == 0xFFFFFFFFu ? nsb : (w[k] & 0x1FFFFFu) >> sh;
      const uint32_t b0 = __builtin_amdgcn_readfirstlane(bk);
      const uint64_t vm = __ballot(valid);
      if (__all(!valid || bk == b0)) {
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
      const uint32_t off = block1024_excl_scan<BS>(tid <= nsb ? s_ch[tid] : 0u, s_w, tot);
      if (tid <= nsb) s_co[tid] = off;
      if (tid <= nsb) s_ch[tid] = 0;
    }
    __syncthreads();
    for (uint32_t j = tid; j <= nb; j += BS)
      c.coffs[q * (kChunkMaxNb + 1) + j] = s_co[j < nb ? j << rsh : nsb];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint32_t pos = (uint32_t)k * BS + tid;
      if (pos >= nval) continue;
      const uint32_t bk = w[k] == 0xFFFFFFFFu ? nsb : (w[k] & 0x1FFFFFu) >> sh;
      lp[k] += s_co[bk];  // the record's sorted slot
      s_srt[lp[k]] = w[k];
    }
    __syncthreads();
    uint32_t* rg = c.region + base;
#pragma unroll 6
    for (int k = 0; k < U; ++k) {
      const uint32_t idx = (uint32_t)k * BS + tid;
      if (idx >= nval) continue;
      const uint32_t x = s_srt[idx];
      uint32_t id = 0xFFFFFFFFu;
      const uint32_t cl = x & 0x1FFFFFu;
      if (x != 0xFFFFFFFFu && (cl >> kBucketBits) < nb) {
        // (non-temporal: 125k flows chunk +6 / bucket -7 us, 1M flows -12 / -4 us per 100M
        //  records, profiles/r06_k3_ab.log)
        __builtin_nontemporal_store((cl & (kBucket - 1u)) | (x >> 21) << kBucketBits, &rg[idx]);
        id = c.omap[cl];
      }
      s_srt[idx] = id;  // the slot this thread just read
    }
    __syncthreads();
    if (c.out_id && base < c.out_cap) {
      uint32_t* oi = c.out_id + base;
      const uint32_t lim = c.out_cap - base < nval ? (uint32_t)(c.out_cap - base) : nval;
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const uint32_t pos = (uint32_t)k * BS + tid;
        if (pos < lim) __builtin_nontemporal_store(s_srt[lp[k]], &oi[pos]);
      }
    }
    __syncthreads();  // (s_srt is rewritten by the next chunk's scatter)
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
  // segments: the two-pass scatter's g1 blocks, or k_count_chunk2's chunks
  const bool chunked = chunk_scatter(c, nflows);
  const uint64_t per = chunked ? (uint64_t)kChunk : count_per(n_acc, g1);
  const uint64_t G = chunked ? (n_acc + kChunk - 1) / kChunk : g1;
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

template <int FPL>
static hipError_t launch_parse_fpl(const ParseArgs& a, bool flows, hipStream_t s) {
  const dim3 grid((unsigned)a.ntiles);
  if (flows) hipLaunchKernelGGL((k_parse<FPL, true>), grid, dim3(kK1Block), 0, s, a);
  else hipLaunchKernelGGL((k_parse<FPL, false>), grid, dim3(kK1Block), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_parse(const ParseArgs& a, int fpl, bool flows, hipStream_t s) {
  // (FPL 2 in every product context; 1 and 4: test tilings of the variants build)
  switch (fpl) {
    case TCBEE_K1_FPL: return launch_parse_fpl<TCBEE_K1_FPL>(a, flows, s);
#if TCBEE_VARIANTS
#if TCBEE_K1_FPL != 1
    case 1: return launch_parse_fpl<1>(a, flows, s);
#endif
#if TCBEE_K1_FPL != 2
    case 2: return launch_parse_fpl<2>(a, flows, s);
#endif
#if TCBEE_K1_FPL != 4
    case 4: return launch_parse_fpl<4>(a, flows, s);
#endif
#endif
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

#if TCBEE_VARIANTS
__global__ void k_test_wait_host(const uint64_t* flag, uint64_t expect, int64_t timeout_ticks,
                                 uint64_t* state) {
  if (threadIdx.x != 0) return;
  const int64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != expect) {
    if (wall_clock64() - t0 > timeout_ticks) {
      *state = 1;
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  *state = 3;
}

hipError_t launch_test_wait_host(const uint64_t* flag_dev, uint64_t expect, uint64_t timeout_us,
                                 uint64_t* state, hipStream_t s) {
  // (wall_clock64 ticks at 100 MHz on MI355X)
  hipLaunchKernelGGL(k_test_wait_host, dim3(1), dim3(64), 0, s, flag_dev, expect,
                     (int64_t)(timeout_us * 100), state);
  return hipGetLastError();
}
#endif

hipError_t launch_rank(const RankArgs& r, hipStream_t s) {
  if (r.nwords <= kRankSmallWords) {
    hipLaunchKernelGGL(k_rank_small, dim3(1), dim3(1024), 0, s, r);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_mark, dim3(1024), dim3(kBlock), 0, s, r);
#if TCBEE_VARIANTS
  if (r.test_hold) {
    const hipError_t e = launch_test_wait_host(r.test_hold, 1, 10'000'000, r.test_hold_state, s);
    if (e != hipSuccess) return e;
  }
#endif
  hipLaunchKernelGGL(k_scan_words, dim3((unsigned)(r.nblocks < 512 ? r.nblocks : 512)), dim3(kBlock),
                     0, s, r);
  hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(kBlock), 0, s, r);
  hipLaunchKernelGGL(k_assign, dim3(1024), dim3(kBlock), 0, s, r);
  // (k_scan_blocks advances the record base / flow count; k_assign reads the staged
  //  old ones, and its blocks past n_new return before touching anything)
  return hipGetLastError();
}

hipError_t launch_count(const CountArgs& c, unsigned g1, unsigned g1s, unsigned g2, hipStream_t s) {
  const dim3 grid(g1);
  if (c.wide_iter) {  // large batches: 16 records per lane and iteration
    if (c.pack_bits) hipLaunchKernelGGL((k_count<16, true>), grid, dim3(kCountBlock), 0, s, c);
    else hipLaunchKernelGGL((k_count<16, false>), grid, dim3(kCountBlock), 0, s, c);
  } else {
    if (c.pack_bits) hipLaunchKernelGGL((k_count<8, true>), grid, dim3(kCountBlock), 0, s, c);
    else hipLaunchKernelGGL((k_count<8, false>), grid, dim3(kCountBlock), 0, s, c);
  }
  // the two-pass scatter only where the chunked one may not cover a batch (tables of
  // >= kChunkMaxNb buckets, or the test hook): no empty launches otherwise
  const bool two_pass = !c.coffs || c.chunk_off || c.nb_max >= kChunkMaxNb;
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
      // kChunk-record chunks in 52 KiB of LDS: two 512-thread workgroups per CU
      const dim3 gc(g1s ? g1s : 1);
      if (c.pack_bits) hipLaunchKernelGGL((k_count_chunk2<true>), gc, dim3(kChunkBlock), 0, s, c);
      else hipLaunchKernelGGL((k_count_chunk2<false>), gc, dim3(kChunkBlock), 0, s, c);
    }
    hipLaunchKernelGGL(k_count_bucket, dim3(g2), dim3(kCountBlock), 0, s, c, g1s);
  }
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

}  // namespace tcbee

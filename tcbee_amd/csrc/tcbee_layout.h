// tcbee_layout.h — byte layouts and pure functions shared by the HIP kernels and
// the host side of libtcbee_amd (NOT the oracle, which restates them itself).
//
// Layout contract (paths relative to the TCBee reference tree):
//   frame : eth 14 B | IPv4 20 B (proto @9, saddr @12, daddr @16) or IPv6 40 B
//           (nexthdr @6, saddr @8, daddr @24) | TCP at frame offset 34 / 54,
//           fixed (IHL / ext headers ignored: tcbee-ebpf/src/config.rs:30-33,
//           probes/xdp.rs:83,157).
//   record: 74 B = bincode(tcp_packet_trace) 70 B + FF FF FF FF
//           (tcbee/src/handlers/mod.rs:126,139; tcbee-process/src/bindings/
//           tcp_packet.rs:8-43). Field offsets in TCBEE_REC_* below.
//   key   : IpTuple repr(C) 38 B (flow.rs:4-12) + 2 zero bytes = 40 B.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define TCBEE_HD __host__ __device__ __forceinline__
#else
#define TCBEE_HD static inline
#endif

namespace tcbee {

// tcbee-ebpf/src/config.rs:22-33
constexpr uint16_t kEthertypeIPv4 = 0x0800;
constexpr uint16_t kEthertypeIPv6 = 0x86DD;
constexpr uint8_t kTcpProtocol = 6;
constexpr uint32_t kEthHdrLen = 14, kIpHdrLen = 20, kIp6HdrLen = 40, kTcpHdrLen = 20;
constexpr uint32_t kV4MinLen = kEthHdrLen + kIpHdrLen + kTcpHdrLen;   // 54
constexpr uint32_t kV6MinLen = kEthHdrLen + kIp6HdrLen + kTcpHdrLen;  // 74
// Frame bytes the record and key are built from: ethertype (12) .. TCP checksum
// (v4: 34+17 = 51, v6: 54+17 = 71). The MACs and the urgent pointer are never read.
constexpr uint32_t kFirstUsedByte = 12, kV4LastUsedByte = 51, kV6LastUsedByte = 71;

// record field offsets (bincode order of tcp_header.rs:554-572)
constexpr int kRecTime = 0, kRecSaddr = 8, kRecDaddr = 12, kRecSaddrV6 = 16,
              kRecDaddrV6 = 32, kRecSport = 48, kRecDport = 50, kRecSeq = 52,
              kRecAck = 56, kRecWindow = 60, kRecFlags = 62, kRecChecksum = 68,
              kRecMarker = 70, kRecBytes = 74;
static_assert(kRecMarker + 4 == kRecBytes, "record is 70 B + 4 B marker");
static_assert(kRecChecksum + 2 == kRecMarker, "checksum ends the bincode body");

// flow table tags
constexpr uint64_t kTagEmpty = 0, kTagBusy = 1;

// ---- tcbee flow hash v1 (DESIGN.md "Flow hash") ---------------------------
// 40-byte key read as 5 little-endian u64 words k[0..4]:
//   h = 0x7CBEE; for each word: h ^= k*C1; h = rotl(h,31)*C2;  h = fmix64(h ^ 40)
// flow_hash32 = lo32(h) ^ hi32(h); table tag = hi32(h) (bumped to >= 2), kept in
// the low half of a slot's tag word (the high half holds the flow's claim index).
TCBEE_HD uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
TCBEE_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}
TCBEE_HD uint64_t flow_hash64(uint64_t k0, uint64_t k1, uint64_t k2, uint64_t k3, uint64_t k4) {
  uint64_t h = 0x7CBEEULL;
  const uint64_t c1 = 0x87c37b91114253d5ULL, c2 = 0x4cf5ad432745937fULL;
  h ^= k0 * c1; h = rotl64(h, 31) * c2;
  h ^= k1 * c1; h = rotl64(h, 31) * c2;
  h ^= k2 * c1; h = rotl64(h, 31) * c2;
  h ^= k3 * c1; h = rotl64(h, 31) * c2;
  h ^= k4 * c1; h = rotl64(h, 31) * c2;
  return fmix64(h ^ 40u);
}
TCBEE_HD uint32_t fold32(uint64_t h) { return (uint32_t)(h ^ (h >> 32)); }
TCBEE_HD uint32_t hash_tag32(uint64_t h) {
  const uint32_t t = (uint32_t)(h >> 32);
  return t < 2 ? t + 2 : t;
}

// counter-based RNG for the synthetic generator (splitmix64)
TCBEE_HD uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

}  // namespace tcbee

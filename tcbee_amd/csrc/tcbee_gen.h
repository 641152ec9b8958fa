// tcbee_gen.h — synthetic trace frames (DESIGN.md "Synthetic traces").
// The same inline function builds the 54 header bytes of frame i on the host
// and on the device, so device-generated traces are bit-identical to the
// host-generated ones the parity tests feed the oracle. Payload bytes are zero.
#pragma once
#include "tcbee_layout.h"

namespace tcbee {

// kGenZipf: flow f drawn with P(f) ∝ 1/(f+1)^s through a caller-supplied CDF
// table (SURVEY.md §8(d) config 3 "second run", s = 1.1): zcdf[k] ≈
// 2^64 · Σ_{j≤k} p_j, non-decreasing, zcdf[n_flows-1] = 2^64-1, built on the
// host (tcbee_amd/trace.py zipf_cdf) and read identically by host and device.
// kGenMultiFlowV6: kGenMultiFlow's flow draw over IPv6/TCP frames (74 header
// bytes: eth + IPv6 without extension headers + TCP).
enum GenKind : int { kGenSingleFlow = 0, kGenMultiFlow = 1, kGenZipf = 2, kGenMultiFlowV6 = 3 };
constexpr uint32_t kGenHdrMax = 74;
TCBEE_HD uint32_t gen_header_len(int kind) { return kind == kGenMultiFlowV6 ? 74u : 54u; }

struct GenFields {
  uint64_t fh;            // the flow's hash (multi-flow kinds): IPv6 addresses
  uint32_t saddr, daddr;  // numeric (a.b.c.d = a<<24 ...)
  uint16_t sport, dport, window, check, ip_id;
  uint32_t seq, ack;
  uint8_t flags;
};

// First k with zcdf[k] > r (n ≥ 1; r = 2^64-1 maps to the last flow).
TCBEE_HD uint64_t zipf_pick(uint64_t r, const uint64_t* zcdf, uint64_t n) {
  uint64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (zcdf[mid] > r) hi = mid; else lo = mid + 1;
  }
  return lo;
}

TCBEE_HD GenFields gen_fields(uint64_t i, int kind, uint64_t n_flows, uint64_t seed,
                              const uint64_t* zcdf = nullptr) {
  GenFields g;
  g.fh = 0;
  if (kind == kGenSingleFlow) {
    // config 2 of BASELINE.json / SURVEY.md §8(d)
    g.saddr = 0x0A000001u;  // 10.0.0.1
    g.daddr = 0x0A000002u;  // 10.0.0.2
    g.sport = 40000;
    g.dport = 5201;
    g.seq = (uint32_t)(1000u + 10u * (uint32_t)i);
    g.ack = 1;
    g.flags = 0x18;
    g.window = 502;
    g.check = (uint16_t)(((uint32_t)i * 2654435761u) >> 16);
  } else {
    const uint64_t r = splitmix64(seed + 0x1000ULL + i);
    const uint64_t f = (kind == kGenZipf && zcdf && n_flows) ? zipf_pick(r, zcdf, n_flows)
                       : (n_flows ? r % n_flows : 0);
    const uint64_t fh = splitmix64((seed << 1) ^ (0xF10F10000000ULL + f));
    g.fh = fh;
    g.saddr = 0x0A000000u | (uint32_t)(fh & 0xFFFFFFu);
    g.daddr = 0xAC100000u | (uint32_t)((fh >> 24) & 0xFFFFFu);
    g.sport = (uint16_t)(1024u + (uint32_t)((fh >> 44) % 64000u));
    const uint16_t ports[4] = {80, 443, 5201, 8080};
    g.dport = ports[(fh >> 62) & 3u];
    g.seq = (uint32_t)(r >> 32);
    g.ack = (uint32_t)splitmix64(r);
    g.flags = 0x10;
    g.window = (uint16_t)(256u + (uint32_t)((fh >> 8) % 65000u));
    g.check = (uint16_t)(r >> 16);
  }
  g.ip_id = (uint16_t)i;
  return g;
}

TCBEE_HD void gen_tcp(uint8_t* t, const GenFields& g) {
  t[0] = (uint8_t)(g.sport >> 8); t[1] = (uint8_t)g.sport;
  t[2] = (uint8_t)(g.dport >> 8); t[3] = (uint8_t)g.dport;
  t[4] = (uint8_t)(g.seq >> 24); t[5] = (uint8_t)(g.seq >> 16);
  t[6] = (uint8_t)(g.seq >> 8); t[7] = (uint8_t)g.seq;
  t[8] = (uint8_t)(g.ack >> 24); t[9] = (uint8_t)(g.ack >> 16);
  t[10] = (uint8_t)(g.ack >> 8); t[11] = (uint8_t)g.ack;
  t[12] = 0x50; t[13] = g.flags;
  t[14] = (uint8_t)(g.window >> 8); t[15] = (uint8_t)g.window;
  t[16] = (uint8_t)(g.check >> 8); t[17] = (uint8_t)g.check;
  t[18] = 0; t[19] = 0;
}

// Writes the gen_header_len(kind) header bytes of a frame of `caplen` bytes:
// eth + IPv4 (IHL 5) + TCP (doff 5), or for kGenMultiFlowV6 eth + IPv6 + TCP
// (addresses 2001:db8:<flow hash> and fd00::<flow hash>, per flow).
TCBEE_HD void gen_header(uint8_t* h, uint64_t i, uint32_t caplen, int kind, uint64_t n_flows,
                         uint64_t seed, const uint64_t* zcdf = nullptr) {
  const GenFields g = gen_fields(i, kind == kGenMultiFlowV6 ? (int)kGenMultiFlow : kind, n_flows,
                                 seed, zcdf);
  // ethernet: dst 02:00:00:00:00:02, src 02:00:00:00:00:01, type IPv4 / IPv6
  h[0] = 0x02; h[1] = 0; h[2] = 0; h[3] = 0; h[4] = 0; h[5] = 0x02;
  h[6] = 0x02; h[7] = 0; h[8] = 0; h[9] = 0; h[10] = 0; h[11] = 0x01;
  if (kind == kGenMultiFlowV6) {
    h[12] = 0x86; h[13] = 0xDD;
    uint8_t* ip6 = h + 14;
    const uint32_t pl = caplen > 54 ? caplen - 54 : 0;  // payload length (TCP + data)
    ip6[0] = 0x60; ip6[1] = 0; ip6[2] = 0; ip6[3] = 0;
    ip6[4] = (uint8_t)(pl >> 8); ip6[5] = (uint8_t)pl;
    ip6[6] = kTcpProtocol; ip6[7] = 64;
    const uint64_t a = g.fh, b = splitmix64(g.fh);
    ip6[8] = 0x20; ip6[9] = 0x01; ip6[10] = 0x0d; ip6[11] = 0xb8;
    for (int k = 0; k < 4; ++k) ip6[12 + k] = (uint8_t)(a >> (8 * k));
    for (int k = 0; k < 8; ++k) ip6[16 + k] = (uint8_t)(b >> (8 * k));
    ip6[24] = 0xfd; ip6[25] = 0;
    for (int k = 0; k < 6; ++k) ip6[26 + k] = (uint8_t)(a >> (32 + 8 * (k % 4)));
    for (int k = 0; k < 8; ++k) ip6[32 + k] = (uint8_t)(b >> (8 * (7 - k)));
    gen_tcp(h + 54, g);
    return;
  }
  h[12] = 0x08; h[13] = 0x00;
  uint8_t* ip = h + 14;
  const uint32_t tot = caplen > 14 ? caplen - 14 : 0;
  ip[0] = 0x45; ip[1] = 0;
  ip[2] = (uint8_t)(tot >> 8); ip[3] = (uint8_t)tot;
  ip[4] = (uint8_t)(g.ip_id >> 8); ip[5] = (uint8_t)g.ip_id;
  ip[6] = 0x40; ip[7] = 0;  // DF
  ip[8] = 64; ip[9] = kTcpProtocol;
  ip[10] = 0; ip[11] = 0;
  ip[12] = (uint8_t)(g.saddr >> 24); ip[13] = (uint8_t)(g.saddr >> 16);
  ip[14] = (uint8_t)(g.saddr >> 8); ip[15] = (uint8_t)g.saddr;
  ip[16] = (uint8_t)(g.daddr >> 24); ip[17] = (uint8_t)(g.daddr >> 16);
  ip[18] = (uint8_t)(g.daddr >> 8); ip[19] = (uint8_t)g.daddr;
  uint32_t sum = 0;
  for (int k = 0; k < 20; k += 2) sum += ((uint32_t)ip[k] << 8) | ip[k + 1];
  while (sum >> 16) sum = (sum & 0xFFFF) + (sum >> 16);
  const uint16_t csum = (uint16_t)~sum;
  ip[10] = (uint8_t)(csum >> 8); ip[11] = (uint8_t)csum;
  gen_tcp(h + 34, g);
}

}  // namespace tcbee

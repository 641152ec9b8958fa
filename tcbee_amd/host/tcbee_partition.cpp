// Flow-hash partition of a trace over N GPUs: the receive-side-scaling step a
// NIC performs before frames reach per-queue XDP programs (the reference runs
// xdp_hook on whichever CPU services the RX queue; its per-CPU
// FLOWS maps, tcbee-ebpf/src/flow_tracker.rs:12-13, are what this partition
// makes disjoint across GPUs). Every frame the hook can key goes to the GPU
// owning its IpTuple, so each GPU's flow table holds its own flows only.
#include "tcbee_host_internal.h"

#include <algorithm>
#include <thread>
#include <vector>

#include "../csrc/tcbee_layout.h"

namespace {

using tcbee_host::ld16;
using tcbee_host::ld32;

// IpTuple key of one frame at the hook's fixed offsets (xdp.rs:37-127: ethertype
// @12, IPv4 proto @23 / IPv6 next header @20, addresses @26/@30 or @22/@38, TCP
// ports @34 or @54), or false when the hook would not key it.
bool frame_key(const uint8_t* f, uint32_t len, uint64_t (&k)[5]) {
  if (len < tcbee::kEthHdrLen) return false;
  const uint16_t et = (uint16_t)((f[12] << 8) | f[13]);
  uint8_t key[40] = {0};
  uint32_t tcp;
  if (et == tcbee::kEthertypeIPv4) {
    if (len < tcbee::kV4MinLen || f[23] != tcbee::kTcpProtocol) return false;
    std::memcpy(key + 12, f + 26, 4);  // 12 zero bytes + wire address (xdp.rs:116-119)
    std::memcpy(key + 28, f + 30, 4);
    tcp = 34;
  } else if (et == tcbee::kEthertypeIPv6) {
    if (len < tcbee::kV6MinLen || f[20] != tcbee::kTcpProtocol) return false;
    std::memcpy(key, f + 22, 16);
    std::memcpy(key + 16, f + 38, 16);
    tcp = 54;
  } else {
    return false;
  }
  const uint16_t sport = (uint16_t)((f[tcp] << 8) | f[tcp + 1]);  // host order
  const uint16_t dport = (uint16_t)((f[tcp + 2] << 8) | f[tcp + 3]);
  std::memcpy(key + 32, &sport, 2);
  std::memcpy(key + 34, &dport, 2);
  key[36] = tcbee::kTcpProtocol;
  std::memcpy(k, key, 40);
  return true;
}

// threads over [0, n): fn(lo, hi) per contiguous range (one range per 64k frames at most)
template <class F>
void parallel_ranges(uint64_t n, uint32_t threads, F fn) {
  const uint64_t t = std::max<uint64_t>(1, std::min<uint64_t>(threads ? threads : 1, n / 65536 + 1));
  if (t == 1) {
    fn(0, n, 0);
    return;
  }
  std::vector<std::thread> pool;
  for (uint64_t j = 0; j < t; ++j) pool.emplace_back(fn, n * j / t, n * (j + 1) / t, j);
  for (auto& th : pool) th.join();
}

// folded flow hash of frame i, or false when the hook would not key it
bool frame_fold(const tcbee_frames* in, uint64_t i, uint32_t& fold) {
  const uint64_t off = in->offset[i];
  uint32_t len = in->caplen[i];
  if (off >= in->arena_len) len = 0;
  else if (len > in->arena_len - off) len = (uint32_t)(in->arena_len - off);
  uint64_t k[5];
  if (!frame_key(in->arena + off, len, k)) return false;
  fold = tcbee::fold32(tcbee::flow_hash64(k[0], k[1], k[2], k[3], k[4]));
  return true;
}

}  // namespace

extern "C" int tcbee_flowhash_owner(const tcbee_frames* in, uint32_t world, uint32_t threads,
                                    uint16_t* out_owner) {
  return tcbee_flowhash_owner_rss(in, world, nullptr, 0, threads, out_owner);
}

extern "C" int tcbee_flowhash_owner_rss(const tcbee_frames* in, uint32_t world, const uint16_t* rss,
                                        uint32_t rss_len, uint32_t threads, uint16_t* out_owner) {
  if (!in || world == 0 || world > 0xFFFFu) return TCBEE_EINVAL;
  if (rss) {
    if (rss_len == 0 || rss_len > TCBEE_RSS_MAX) return TCBEE_EINVAL;
    for (uint32_t b = 0; b < rss_len; ++b)
      if (rss[b] >= world) return TCBEE_EINVAL;
  }
  const uint64_t n = in->n;
  if (n && (!in->arena || !in->offset || !in->caplen || !out_owner)) return TCBEE_EINVAL;
  parallel_ranges(n, threads, [&](uint64_t lo, uint64_t hi, uint64_t) {
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t h;
      if (frame_fold(in, i, h))
        out_owner[i] = rss ? rss[h % rss_len] : (uint16_t)(h % world);
      else
        out_owner[i] = (uint16_t)(i % world);  // no key, no record: any GPU
    }
  });
  return TCBEE_OK;
}

extern "C" int tcbee_flowhash_load(const tcbee_frames* in, uint32_t rss_len, uint32_t threads,
                                   uint64_t* out_counts) {
  if (!in || rss_len == 0 || rss_len > TCBEE_RSS_MAX || !out_counts) return TCBEE_EINVAL;
  const uint64_t n = in->n;
  if (n && (!in->arena || !in->offset || !in->caplen)) return TCBEE_EINVAL;
  const uint64_t t = std::max<uint64_t>(1, std::min<uint64_t>(threads ? threads : 1, n / 65536 + 1));
  std::vector<std::vector<uint64_t>> part(t, std::vector<uint64_t>(rss_len, 0));
  parallel_ranges(n, threads, [&](uint64_t lo, uint64_t hi, uint64_t j) {
    std::vector<uint64_t>& c = part[j];
    for (uint64_t i = lo; i < hi; ++i) {
      uint32_t h;
      if (frame_fold(in, i, h)) ++c[h % rss_len];
    }
  });
  for (uint32_t b = 0; b < rss_len; ++b) {
    uint64_t v = 0;
    for (uint64_t j = 0; j < t; ++j) v += part[j][b];
    out_counts[b] = v;
  }
  return TCBEE_OK;
}

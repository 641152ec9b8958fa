// Classic-pcap ingest: the replay source standing in for the live XDP/TC
// packet path (tcbee/src/eBPF/probes/headers.rs:67-109 drains rings fed by the
// kernel hooks; here the frames come from a recorded trace). The file is
// memory-mapped and indexed once; the tcbee_frames view points into the
// mapping, so nothing is copied until the ingest pipeline stages a chunk.
#include "tcbee_host_internal.h"

#include <cerrno>
#include <cstdio>
#include <fcntl.h>
#include <new>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <vector>

struct tcbee_pcap {
  int fd = -1;
  const uint8_t* map = nullptr;
  uint64_t len = 0;
  tcbee_pcap_info info{};
  std::vector<uint64_t> offset, ts_ns;
  std::vector<uint32_t> caplen;
};

namespace {

constexpr uint32_t kMagicUs = 0xA1B2C3D4u, kMagicNs = 0xA1B23C4Du;
constexpr uint32_t kLinkEthernet = 1;

inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

void destroy(tcbee_pcap* p) {
  if (p->map) munmap(const_cast<uint8_t*>(p->map), p->len);
  if (p->fd >= 0) ::close(p->fd);
  delete p;
}

}  // namespace

using namespace tcbee_host;

extern "C" {

int tcbee_pcap_open(tcbee_pcap** out, const char* path) {
  if (!out || !path) return TCBEE_EINVAL;
  *out = nullptr;
  tcbee_pcap* p = new (std::nothrow) tcbee_pcap;
  if (!p) return TCBEE_ENOMEM;
  p->fd = ::open(path, O_RDONLY | O_CLOEXEC);
  struct stat st;
  if (p->fd < 0 || fstat(p->fd, &st) != 0) return destroy(p), TCBEE_EIO;
  p->len = uint64_t(st.st_size);
  if (p->len < 24) return destroy(p), TCBEE_EFORMAT;
  void* m = mmap(nullptr, p->len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, p->fd, 0);
  if (m == MAP_FAILED) return destroy(p), TCBEE_EIO;
  p->map = static_cast<const uint8_t*>(m);
  madvise(m, p->len, MADV_SEQUENTIAL);

  const uint32_t magic = ld32(p->map);
  bool swapped = false, ns = false;
  if (magic == kMagicUs || magic == kMagicNs) {
    ns = magic == kMagicNs;
  } else if (bswap32(magic) == kMagicUs || bswap32(magic) == kMagicNs) {
    swapped = true;
    ns = bswap32(magic) == kMagicNs;
  } else {
    return destroy(p), TCBEE_EFORMAT;
  }
  auto u32 = [&](uint64_t off) { uint32_t v = ld32(p->map + off); return swapped ? bswap32(v) : v; };
  p->info.snaplen = u32(16);
  p->info.linktype = u32(20) & 0x0FFFFFFu;  // upper bits: FCS length flags
  p->info.nanosecond = ns;
  p->info.swapped = swapped;
  p->info.file_bytes = p->len;
  if (p->info.linktype != kLinkEthernet) return destroy(p), TCBEE_EFORMAT;

  // One sequential pass over the record headers (16 B each).
  try {
    const uint64_t guess = p->len / 96 + 16;
    p->offset.reserve(guess);
    p->caplen.reserve(guess);
    p->ts_ns.reserve(guess);
    uint64_t pos = 24;
    const uint64_t frac_mul = ns ? 1 : 1000;
    while (pos + 16 <= p->len) {
      const uint64_t sec = u32(pos), frac = u32(pos + 4);
      const uint32_t incl = u32(pos + 8);
      if (pos + 16 + incl > p->len) {
        p->info.truncated = 1;
        break;
      }
      p->offset.push_back(pos + 16);
      p->caplen.push_back(incl);
      p->ts_ns.push_back(sec * 1000000000ull + frac * frac_mul);
      pos += 16 + uint64_t(incl);
    }
    if (pos < p->len && !p->info.truncated) p->info.truncated = 1;
  } catch (const std::bad_alloc&) {
    return destroy(p), TCBEE_ENOMEM;
  }
  p->info.n = p->offset.size();
  *out = p;
  return TCBEE_OK;
}

int tcbee_pcap_frames(const tcbee_pcap* p, tcbee_frames* out) {
  if (!p || !out) return TCBEE_EINVAL;
  out->arena = p->map;
  out->arena_len = p->len;
  out->offset = p->offset.data();
  out->caplen = p->caplen.data();
  out->ts_ns = p->ts_ns.data();
  out->n = p->offset.size();
  return TCBEE_OK;
}

int tcbee_pcap_get_info(const tcbee_pcap* p, tcbee_pcap_info* out) {
  if (!p || !out) return TCBEE_EINVAL;
  *out = p->info;
  return TCBEE_OK;
}

int tcbee_pcap_close(tcbee_pcap* p) {
  if (!p) return TCBEE_EINVAL;
  destroy(p);
  return TCBEE_OK;
}

int tcbee_pcap_write(const char* path, const tcbee_frames* in, int nanosecond, uint32_t snaplen) {
  if (!path || !in || (in->n && (!in->arena || !in->offset || !in->caplen || !in->ts_ns)))
    return TCBEE_EINVAL;
  for (uint64_t i = 0; i < in->n; ++i)
    if (in->offset[i] + in->caplen[i] > in->arena_len) return TCBEE_EINVAL;
  FILE* fp = std::fopen(path, "wb");
  if (!fp) return TCBEE_EIO;
  std::vector<char> iobuf(1 << 22);
  std::setvbuf(fp, iobuf.data(), _IOFBF, iobuf.size());
  const uint32_t hdr[6] = {nanosecond ? kMagicNs : kMagicUs, 2u | (4u << 16), 0, 0,
                           snaplen ? snaplen : 262144u, kLinkEthernet};
  bool ok = std::fwrite(hdr, 24, 1, fp) == 1;
  const uint64_t div = nanosecond ? 1 : 1000;
  for (uint64_t i = 0; ok && i < in->n; ++i) {
    const uint64_t t = in->ts_ns[i];
    const uint32_t rh[4] = {uint32_t(t / 1000000000ull), uint32_t((t % 1000000000ull) / div),
                            in->caplen[i], in->caplen[i]};
    ok = std::fwrite(rh, 16, 1, fp) == 1 &&
         (in->caplen[i] == 0 || std::fwrite(in->arena + in->offset[i], in->caplen[i], 1, fp) == 1);
  }
  if (std::fclose(fp) != 0) ok = false;
  return ok ? TCBEE_OK : TCBEE_EIO;
}

}  // extern "C"

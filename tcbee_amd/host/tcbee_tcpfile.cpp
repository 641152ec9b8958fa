// .tcp record files: the append writer of tcbee-record's BufferHandler and the
// decode/validate half of tcbee-process (FileReader + TcpPacket), plus the
// metrics.json writer. See include/tcbee_host.h for the reference lines each
// function mirrors.
#include "tcbee_host_internal.h"

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <new>
#include <string>
#include <unistd.h>

namespace tcbee_host {

// bincode 1.x, legacy config: fixint little endian, fields in declaration
// order (tcp_packet.rs:8-28), bool = one byte that must be 0 or 1.
bool decode_packet(const uint8_t* r, tcbee_packet* p) {
  for (int i = 62; i < 68; ++i)
    if (r[i] > 1) {  // bincode: "invalid value for bool" -> from_buffer default
      std::memset(p, 0, sizeof(*p));
      return false;
    }
  p->time = ld64(r + 0);
  p->saddr = ld32(r + 8);
  p->daddr = ld32(r + 12);
  std::memcpy(p->saddr_v6, r + 16, 16);
  std::memcpy(p->daddr_v6, r + 32, 16);
  p->sport = ld16(r + 48);
  p->dport = ld16(r + 50);
  p->seq = ld32(r + 52);
  p->ack = ld32(r + 56);
  p->window = ld16(r + 60);
  p->flag_urg = r[62];
  p->flag_ack = r[63];
  p->flag_psh = r[64];
  p->flag_rst = r[65];
  p->flag_syn = r[66];
  p->flag_fin = r[67];
  p->checksum = ld16(r + 68);
  std::memcpy(p->div, r + 70, 4);
  return true;
}

bool marker_ok(const tcbee_packet& p) {
  return p.div[0] == 0xFF && p.div[1] == 0xFF && p.div[2] == 0xFF && p.div[3] == 0xFF;
}

// Ipv4Addr Display: dotted decimal of the big-endian octets of the u32
// (Ipv4Addr::from(u32), tcp_packet.rs:99-100).
static int fmt_v4(uint32_t v, char* out) {
  return std::snprintf(out, 48, "%u.%u.%u.%u", v >> 24, (v >> 16) & 255u, (v >> 8) & 255u,
                       v & 255u);
}

// Ipv6Addr Display of Rust's std: IPv4-mapped addresses as ::ffff:a.b.c.d,
// otherwise lowercase hex groups with the first longest run (length > 1) of
// zero groups written as "::" (RFC 5952 style).
static int fmt_v6(const uint8_t* a, char* out) {
  uint16_t g[8];
  for (int i = 0; i < 8; ++i) g[i] = uint16_t(a[2 * i] << 8 | a[2 * i + 1]);
  bool mapped = g[5] == 0xFFFF;
  for (int i = 0; i < 5; ++i) mapped = mapped && g[i] == 0;
  if (mapped)
    return std::snprintf(out, 48, "::ffff:%u.%u.%u.%u", a[12], a[13], a[14], a[15]);
  int best_s = 0, best_l = 0, cur_s = 0, cur_l = 0;
  for (int i = 0; i < 8; ++i) {
    if (g[i] == 0) {
      if (cur_l == 0) cur_s = i;
      ++cur_l;
      if (cur_l > best_l) {
        best_l = cur_l;
        best_s = cur_s;
      }
    } else {
      cur_l = 0;
    }
  }
  int n = 0;
  auto groups = [&](int lo, int hi) {
    for (int i = lo; i < hi; ++i)
      n += std::snprintf(out + n, 48 - n, i > lo ? ":%x" : "%x", g[i]);
  };
  if (best_l > 1) {
    groups(0, best_s);
    n += std::snprintf(out + n, 48 - n, "::");
    groups(best_s + best_l, 8);
  } else {
    groups(0, 8);
  }
  return n;
}

void packet_tuple(const tcbee_packet& p, tcbee_ts_tuple* t) {
  if (p.saddr != 0 && p.daddr != 0) {
    fmt_v4(p.saddr, t->src);
    fmt_v4(p.daddr, t->dst);
  } else {
    fmt_v6(p.saddr_v6, t->src);
    fmt_v6(p.daddr_v6, t->dst);
  }
  t->sport = p.sport;
  t->dport = p.dport;
  t->l4proto = 6;
}

}  // namespace tcbee_host

using namespace tcbee_host;

extern "C" {

int tcbee_host_abi_version(void) { return TCBEE_HOST_ABI_VERSION; }

int tcbee_tcp_decode(const uint8_t* rec74, uint64_t n, tcbee_packet* out, uint64_t* n_default) {
  if (n && (!rec74 || !out)) return TCBEE_EINVAL;
  uint64_t bad = 0;
  for (uint64_t i = 0; i < n; ++i) bad += !decode_packet(rec74 + i * kRec, out + i);
  if (n_default) *n_default = bad;
  return TCBEE_OK;
}

int tcbee_tcp_check(const uint8_t* rec74, uint64_t n, uint64_t* first_bad) {
  if (!first_bad || (n && !rec74)) return TCBEE_EINVAL;
  tcbee_packet p;
  for (uint64_t i = 0; i < n; ++i) {
    decode_packet(rec74 + i * kRec, &p);
    if (!marker_ok(p)) {
      *first_bad = i;
      return TCBEE_EFORMAT;
    }
  }
  *first_bad = n;
  return TCBEE_OK;
}

int tcbee_tcp_tuple(const tcbee_packet* p, tcbee_ts_tuple* out) {
  if (!p || !out) return TCBEE_EINVAL;
  std::memset(out, 0, sizeof(*out));
  packet_tuple(*p, out);
  return TCBEE_OK;
}

struct tcbee_tcpfile {
  int fd = -1;
  uint8_t* buf = nullptr;
  uint64_t cap = 0, used = 0;
  bool failed = false;
};

static int write_all(int fd, const uint8_t* p, uint64_t n) {
  while (n) {
    ssize_t w = ::write(fd, p, n > (1u << 30) ? (1u << 30) : n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return TCBEE_EIO;
    }
    p += w;
    n -= uint64_t(w);
  }
  return TCBEE_OK;
}

int tcbee_tcpfile_open(tcbee_tcpfile** out, const char* path, uint64_t buffer_bytes) {
  if (!out || !path) return TCBEE_EINVAL;
  *out = nullptr;
  tcbee_tcpfile* f = new (std::nothrow) tcbee_tcpfile;
  if (!f) return TCBEE_ENOMEM;
  f->cap = buffer_bytes ? buffer_bytes : 10000ull * 72ull;
  f->buf = new (std::nothrow) uint8_t[f->cap];
  f->fd = ::open(path, O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
  if (!f->buf || f->fd < 0) {
    int rc = f->buf ? TCBEE_EIO : TCBEE_ENOMEM;
    if (f->fd >= 0) ::close(f->fd);
    delete[] f->buf;
    delete f;
    return rc;
  }
  *out = f;
  return TCBEE_OK;
}

int tcbee_tcpfile_append(tcbee_tcpfile* f, const uint8_t* rec74, uint64_t n) {
  if (!f || (n && !rec74)) return TCBEE_EINVAL;
  if (f->failed) return TCBEE_EIO;
  uint64_t bytes = n * kRec;
  // BufWriter semantics: stage while it fits, write through when it does not.
  if (f->used + bytes > f->cap) {
    if (f->used && write_all(f->fd, f->buf, f->used)) return f->failed = true, TCBEE_EIO;
    f->used = 0;
    if (bytes >= f->cap) return write_all(f->fd, rec74, bytes) ? (f->failed = true, TCBEE_EIO)
                                                               : TCBEE_OK;
  }
  std::memcpy(f->buf + f->used, rec74, bytes);
  f->used += bytes;
  return TCBEE_OK;
}

int tcbee_tcpfile_close(tcbee_tcpfile* f) {
  if (!f) return TCBEE_EINVAL;
  int rc = TCBEE_OK;
  if (!f->failed && f->used && write_all(f->fd, f->buf, f->used)) rc = TCBEE_EIO;
  if (::close(f->fd) != 0) rc = TCBEE_EIO;
  delete[] f->buf;
  delete f;
  return rc;
}

int tcbee_metrics_write(const char* dir_prefix, const tcbee_counters* ctr,
                        uint64_t ingress_calls, uint64_t egress_calls) {
  if (!dir_prefix || !ctr) return TCBEE_EINVAL;
  std::string path = std::string(dir_prefix) + "metrics.json";
  FILE* fp = std::fopen(path.c_str(), "wb");
  if (!fp) return TCBEE_EIO;
  // serde_json::to_writer of `Metrics` (ebpf_watcher.rs:51-59): compact, no
  // trailing newline, u32 fields (the per-CPU u32 sums wrap).
  int w = std::fprintf(fp,
                       "{\"handled\":%u,\"dropped\":%u,\"ingress\":%u,\"egress\":%u,"
                       "\"ingress_calls\":%u,\"egress_calls\":%u}",
                       uint32_t(ctr->handled), uint32_t(ctr->dropped), uint32_t(ctr->ingress),
                       uint32_t(ctr->egress), uint32_t(ingress_calls), uint32_t(egress_calls));
  int rc = std::fclose(fp);
  return (w < 0 || rc != 0) ? TCBEE_EIO : TCBEE_OK;
}

}  // extern "C"

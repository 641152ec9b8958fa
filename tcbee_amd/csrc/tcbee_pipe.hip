// tcbee_pipe.hip — host-frames ingest pipeline:
// frames in host memory (a pcap mapping, a capture ring) -> pinned staging ->
// H2D -> parse -> D2H -> records on the host, with every stage of chunk i
// overlapping the others' work on chunks i-1 / i-2:
//
//   host threads   stage(i)  ─┐                     consume(i-2)
//   H2D engine                └─ H2D(i)
//   compute                            parse(i-1)
//   D2H engine                                      D2H(i-1)  (exact record count)
//
// Staging modes
//   window == 0  whole frames are gathered back to back (payload included).
//   window >= 80 "header window": only min(caplen, window) bytes of each frame
//                are shipped, at stride `window`, with the ORIGINAL caplen. The
//                record path reads at most 74 bytes of a frame and decides only
//                on bytes < min(caplen, 74) and on caplen itself (xdp.rs:37-152
//                read nothing past the TCP header), so the records, flow ids
//                and counters are identical to shipping whole frames — while
//                PCIe carries ~92 B per frame instead of the frame size.
//   window == 64 the same without the two MAC addresses, which no record field
//                uses: frame bytes [12, 76) — ethertype .. the end of an IPv6
//                TCP header — each in one whole 64-B line of staging after a
//                64-B pad (frame k's device offset = 64 + 64k - 12). Whole-line
//                streaming stores: 1.5x the gather rate of 80-B windows, whose
//                lines are written in pieces.
//
// The live source this replaces is the ring drain of the reference
// (tcbee/src/eBPF/probes/headers.rs:67-109): there the kernel hands each
// packet to the hooks; here a batch of recorded frames is streamed through
// the GPU hooks.
#include <hip/hip_runtime.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#if defined(__x86_64__)
#include <immintrin.h>  // streaming stores of the header-window gather (x86 hosts)
#define TCBEE_PIPE_HAVE_NT 1
#else
#define TCBEE_PIPE_HAVE_NT 0
#endif
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tcbee_amd.h"

namespace {

// window 64 skips the 12 MAC bytes: frame k's window holds its bytes [12, 76)
constexpr uint64_t kMacBytes = 12, kLineWindow = 64;
__host__ __device__ inline uint64_t window_skip(uint64_t window) {
  return window == kLineWindow ? kMacBytes : 0;
}
__host__ __device__ inline uint64_t window_base(uint64_t window) {
  return window == kLineWindow ? kLineWindow : 0;  // the pad before window 0
}

__global__ void k_window_offsets(uint64_t* off, uint64_t n, uint64_t window) {
  const uint64_t base = window_base(window) - window_skip(window);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    off[i] = base + i * window;
}

int map_err(hipError_t e) {
  if (e == hipSuccess) return TCBEE_OK;
  if (e == hipErrorOutOfMemory) return TCBEE_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TCBEE_ENODEV;
  if (e == hipErrorInvalidValue) return TCBEE_EINVAL;
  return TCBEE_EDEVICE;
}

#define TRY_HIP(expr)                          \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return map_err(e_);  \
  } while (0)

// Fixed pool of host threads running one parallel-for at a time.
class Pool {
 public:
  explicit Pool(unsigned n) {
    for (unsigned i = 1; i < n; ++i) th_.emplace_back([this, i] { loop(i); });
    n_ = n;
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  unsigned size() const { return n_; }
  // fn(part, parts) on the first `parts` threads (all by default; the caller is part
  // 0); returns when all are done.
  void run(const std::function<void(unsigned, unsigned)>& fn, unsigned parts = 0) {
    parts = parts == 0 || parts > n_ ? n_ : parts;
    if (parts == 1) {
      fn(0, 1);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = &fn;
      parts_ = parts;
      pending_ = n_ - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0, parts);
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop(unsigned id) {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(unsigned, unsigned)>* fn;
      unsigned parts;
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
        parts = parts_;
      }
      if (id < parts) (*fn)(id, parts);
      {
        std::lock_guard<std::mutex> g(m_);
        if (--pending_ == 0) done_cv_.notify_one();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(unsigned, unsigned)>* fn_ = nullptr;
  unsigned n_ = 1, parts_ = 1, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

struct Slot {
  // pinned host
  uint8_t* h_arena = nullptr;
  uint64_t* h_off = nullptr;
  uint32_t* h_len = nullptr;
  uint64_t* h_ts = nullptr;
  uint8_t* h_rec = nullptr;
  uint32_t* h_id = nullptr;
  uint64_t* h_meta = nullptr;  // [0] = records, [1..4] = counters
  // device
  uint8_t* d_arena = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint64_t* d_ts = nullptr;
  uint8_t* d_rec = nullptr;
  uint32_t* d_id = nullptr;
  uint64_t* d_meta = nullptr;  // same layout as h_meta
  hipEvent_t ev_h2d = nullptr, ev_parse = nullptr, ev_d2h = nullptr;
  // chunk bookkeeping
  uint64_t lo = 0, hi = 0, arena_used = 0, n_rec = 0, first_record = 0;
  bool direct = false;  // records / ids were DMA'd into the caller's registered arrays
};

}  // namespace

struct tcbee_pipe {
  int device = 0;
  tcbee_pipe_cfg cfg{};
  tcbee_ctx* ctx = nullptr;
  hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
  std::vector<Slot> slots;
  Pool* pool = nullptr;   // the gather (stage) threads, the main thread included
  Pool* cpool = nullptr;  // the copy-out (consume) threads, the consumer thread included
  unsigned gt_staged = 1;  // gather threads while the copy-out pool works (staged outputs)
  tcbee_pipe_stats st{};
  // caller output arrays registered with tcbee_pipe_register_output (page-locked):
  // chunks D2H straight into them
  uint8_t* reg_rec = nullptr;
  uint32_t* reg_id = nullptr;
  uint64_t reg_cap = 0;
  uint64_t reg_rec_bytes = 0, reg_id_bytes = 0;  // the ranges held in the registry
  uint64_t prefetch = 48;  // header-window gather: frames ahead (TCBEE_PIPE_PF, 0 = off)
  int nt_copy = 1;         // header-window gather: fixed-size 16-B loads + streaming
                           // stores into the staging (TCBEE_PIPE_NT=0: memcpy)
};

namespace {

// Page-locked output ranges, process-wide: pipes handed the same arrays
// share ONE registration. An entry is the range some pipe page-locked with
// hipHostRegister, and the pipes holding it; a pipe borrows an entry only when the
// entry covers the bytes it asks for, and the range is unregistered when its LAST
// holder releases it. Every holder syncs its own D2H stream before it releases
// (register_output, free_pipe), so by then no holder's D2H into the range is in
// flight — the owner can be released first without pulling the pages from under a
// borrower. A range the CALLER page-locked (not in the registry) is used as is when
// both of its ends are registered, and never unregistered here.
struct HostReg {
  uint8_t* base;
  uint64_t bytes;
  uint32_t holders;
};
std::mutex g_reg_mu;
std::vector<HostReg> g_regs;

// Is host byte p page-locked (hipHostRegister'd or hipHostMalloc'd)? Measured on
// this ROCm (round 6, ab/hostreg_probe): hipHostGetFlags fails for hipHostRegister'd
// ranges (it knows hipHostMalloc only), while hipPointerGetAttributes reports
// hipMemoryTypeHost for every byte of a registered range — so round 5's
// hipHostGetFlags check never saw a registration, a second pipe registered the range
// again (which HIP accepts), and the first hipHostUnregister released it for both.
bool host_locked(const void* p) {
  hipPointerAttribute_t at{};
  const bool ok = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  return ok;
}

hipError_t register_range(void* ptr, uint64_t bytes) {
  uint8_t* const b = static_cast<uint8_t*>(ptr);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (HostReg& r : g_regs) {
    if (b >= r.base && b + bytes <= r.base + r.bytes) {
      ++r.holders;
      return hipSuccess;
    }
    if (b < r.base + r.bytes && r.base < b + bytes)
      return hipErrorInvalidValue;  // overlaps a registration without being inside it
  }
  if (host_locked(b)) {
    // page-locked by the caller: borrow it if it reaches the last byte too
    if (!host_locked(b + bytes - 1)) return hipErrorInvalidValue;
    return hipSuccess;
  }
  const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterDefault);
  if (e == hipSuccess) g_regs.push_back({b, bytes, 1});
  return e;
}

void release_range(void* ptr, uint64_t bytes) {
  uint8_t* const b = static_cast<uint8_t*>(ptr);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (size_t i = 0; i < g_regs.size(); ++i) {
    HostReg& r = g_regs[i];
    if (b >= r.base && b + bytes <= r.base + r.bytes) {
      if (--r.holders == 0) {
        (void)hipHostUnregister(r.base);
        (void)hipGetLastError();  // (a failed release must not surface in a later call)
        g_regs.erase(g_regs.begin() + i);
      }
      return;
    }
  }
  // not in the registry: the caller's own registration, left as it was
}

// (the pipe's D2H stream must be idle: callers sync it first)
void unregister_output(tcbee_pipe* p) {
  if (p->reg_rec && p->reg_rec_bytes) release_range(p->reg_rec, p->reg_rec_bytes);
  if (p->reg_id && p->reg_id_bytes) release_range(p->reg_id, p->reg_id_bytes);
  p->reg_rec = nullptr;
  p->reg_id = nullptr;
  p->reg_cap = 0;
  p->reg_rec_bytes = p->reg_id_bytes = 0;
}

void free_pipe(tcbee_pipe* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  if (p->s_h2d) (void)hipStreamSynchronize(p->s_h2d);
  if (p->s_d2h) (void)hipStreamSynchronize(p->s_d2h);
  if (p->ctx) (void)tcbee_ctx_sync(p->ctx);
  unregister_output(p);
  for (Slot& s : p->slots) {
    for (void* h : {(void*)s.h_arena, (void*)s.h_off, (void*)s.h_len, (void*)s.h_ts,
                    (void*)s.h_rec, (void*)s.h_id, (void*)s.h_meta})
      if (h) (void)hipHostFree(h);
    for (void* d : {(void*)s.d_arena, (void*)s.d_off, (void*)s.d_len, (void*)s.d_ts,
                    (void*)s.d_rec, (void*)s.d_id, (void*)s.d_meta})
      if (d) (void)hipFree(d);
    for (hipEvent_t e : {s.ev_h2d, s.ev_parse, s.ev_d2h})
      if (e) (void)hipEventDestroy(e);
  }
  if (p->s_h2d) (void)hipStreamDestroy(p->s_h2d);
  if (p->s_d2h) (void)hipStreamDestroy(p->s_d2h);
  if (p->ctx) tcbee_ctx_destroy(p->ctx);
  delete p->pool;
  delete p->cpool;
  delete p;
}

template <class T>
hipError_t hpin(T** p, uint64_t count) {
  return hipHostMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T),
                       hipHostMallocDefault);
}
template <class T>
hipError_t dmal(T** p, uint64_t count) {
  return hipMalloc(reinterpret_cast<void**>(p), (count ? count : 1) * sizeof(T));
}

int alloc_slot(tcbee_pipe* p, Slot& s) {
  const uint64_t F = p->cfg.chunk_frames, B = p->cfg.chunk_bytes;
  TRY_HIP(hpin(&s.h_arena, B + 64));
  TRY_HIP(hpin(&s.h_off, F));
  TRY_HIP(hpin(&s.h_len, F));
  TRY_HIP(hpin(&s.h_ts, F));
  TRY_HIP(hpin(&s.h_rec, F * TCBEE_RECORD_BYTES));
  TRY_HIP(hpin(&s.h_id, F));
  TRY_HIP(hpin(&s.h_meta, 8));
  TRY_HIP(dmal(&s.d_arena, B + 64));
  TRY_HIP(dmal(&s.d_off, F));
  TRY_HIP(dmal(&s.d_len, F));
  TRY_HIP(dmal(&s.d_ts, F));
  TRY_HIP(dmal(&s.d_rec, F * TCBEE_RECORD_BYTES + 64));
  TRY_HIP(dmal(&s.d_id, F));
  TRY_HIP(dmal(&s.d_meta, 8));
  TRY_HIP(hipEventCreateWithFlags(&s.ev_h2d, hipEventDisableTiming));
  TRY_HIP(hipEventCreateWithFlags(&s.ev_parse, hipEventDisableTiming));
  TRY_HIP(hipEventCreateWithFlags(&s.ev_d2h, hipEventDisableTiming));
  return TCBEE_OK;
}

// Frames [lo, hi) that fit one chunk, starting at lo.
uint64_t chunk_end(const tcbee_pipe* p, const tcbee_frames* in, uint64_t lo) {
  const uint64_t F = p->cfg.chunk_frames, B = p->cfg.chunk_bytes;
  uint64_t hi = lo + F < in->n ? lo + F : in->n;
  if (p->cfg.window) return hi;  // stride window: F * window <= B by construction
  uint64_t bytes = 0, i = lo;
  for (; i < hi; ++i) {
    if (bytes + in->caplen[i] > B) break;
    bytes += in->caplen[i];
  }
  return i;
}

// Gather frames [s.lo, s.hi) into the slot's pinned staging on `gparts` of the
// gather pool's threads (pool-parallel).
void stage(tcbee_pipe* p, const tcbee_frames* in, Slot& s, unsigned gparts) {
  const uint64_t lo = s.lo, n = s.hi - s.lo, W = p->cfg.window;
  if (W) {
    const uint64_t pf = p->prefetch;
    const uint64_t skip = window_skip(W);          // frame bytes before the window
    uint8_t* const h0 = s.h_arena + window_base(W);  // window 0
    // (16-B streaming stores need a 16-B aligned staging slot per frame)
    // (streaming stores exist on x86 hosts only; elsewhere the memcpy path runs)
    const bool nt = TCBEE_PIPE_HAVE_NT && p->nt_copy && W % 16 == 0 &&
                    ((uintptr_t)s.h_arena & 15u) == 0;
    p->pool->run([&](unsigned part, unsigned parts) {
      const uint64_t a = n * part / parts, b = n * (part + 1) / parts;
      for (uint64_t k = a; k < b; ++k) {
        const uint64_t f = lo + k;
        // the windows are random lines of a multi-GB capture: fetch the lines of the
        // frame `pf` ahead while this one is copied (host-memory latency bound)
        if (pf && k + pf < b) {
          const uint64_t o2 = in->offset[f + pf] + skip;
          if (o2 + W <= in->arena_len) {
            __builtin_prefetch(in->arena + o2, 0, 0);
            __builtin_prefetch(in->arena + o2 + W - 1, 0, 0);
          }
        }
        const uint32_t len = in->caplen[f];
        const uint64_t o = in->offset[f] + skip;
#if TCBEE_PIPE_HAVE_NT
        if (nt && o + W <= in->arena_len) {
          // the whole window, whatever the caplen: the bytes past caplen are never
          // read (the kernels take caplen from h_len), so no per-frame length
          // branch; streaming stores skip the read-for-ownership of the staging line
          const __m128i* src = reinterpret_cast<const __m128i*>(in->arena + o);
          __m128i* dst = reinterpret_cast<__m128i*>(h0 + k * W);
          for (uint64_t c = 0; c < W / 16; ++c) _mm_stream_si128(dst + c, _mm_loadu_si128(src + c));
          s.h_len[k] = len;
          s.h_ts[k] = in->ts_ns[f];
          continue;
        }
#endif
        const uint64_t flen = len > skip ? len - skip : 0;  // frame bytes from the window on
        const uint64_t want = flen < W ? flen : W;
        uint64_t cp = want;
        if (o >= in->arena_len) cp = 0;
        else if (cp > in->arena_len - o) cp = in->arena_len - o;
        std::memcpy(h0 + k * W, in->arena + o, cp);
        if (cp < want) std::memset(h0 + k * W + cp, 0, want - cp);  // past the arena
        s.h_len[k] = len;
        s.h_ts[k] = in->ts_ns[f];
      }
#if TCBEE_PIPE_HAVE_NT
      if (nt) _mm_sfence();  // streaming stores visible before the H2D copy is issued
#endif
    }, gparts);
    s.arena_used = window_base(W) + n * W;
    return;
  }
  // whole frames: exclusive prefix of caplen per part, then copy
  const unsigned parts = gparts ? gparts : p->pool->size();
  std::vector<uint64_t> part_bytes(parts + 1, 0);
  p->pool->run([&](unsigned part, unsigned np) {
    const uint64_t a = n * part / np, b = n * (part + 1) / np;
    uint64_t sum = 0;
    for (uint64_t k = a; k < b; ++k) sum += in->caplen[lo + k];
    part_bytes[part + 1] = sum;
  }, parts);
  for (unsigned i = 0; i < parts; ++i) part_bytes[i + 1] += part_bytes[i];
  p->pool->run([&](unsigned part, unsigned np) {
    const uint64_t a = n * part / np, b = n * (part + 1) / np;
    uint64_t pos = part_bytes[part];
    for (uint64_t k = a; k < b; ++k) {
      const uint64_t f = lo + k;
      const uint32_t len = in->caplen[f];
      const uint64_t o = in->offset[f];
      uint64_t cp = len;
      if (o >= in->arena_len) cp = 0;
      else if (cp > in->arena_len - o) cp = in->arena_len - o;
      std::memcpy(s.h_arena + pos, in->arena + o, cp);
      if (cp < len) std::memset(s.h_arena + pos + cp, 0, len - cp);  // past the arena
      s.h_off[k] = pos;
      s.h_len[k] = len;
      s.h_ts[k] = in->ts_ns[f];
      pos += len;
    }
  }, parts);
  s.arena_used = part_bytes[parts];
}

int enqueue(tcbee_pipe* p, Slot& s, const tcbee_cfg* cfg) {
  const uint64_t n = s.hi - s.lo, W = p->cfg.window;
  // H2D
  TRY_HIP(hipMemcpyAsync(s.d_arena, s.h_arena, s.arena_used, hipMemcpyHostToDevice, p->s_h2d));
  if (!W) TRY_HIP(hipMemcpyAsync(s.d_off, s.h_off, n * 8, hipMemcpyHostToDevice, p->s_h2d));
  TRY_HIP(hipMemcpyAsync(s.d_len, s.h_len, n * 4, hipMemcpyHostToDevice, p->s_h2d));
  TRY_HIP(hipMemcpyAsync(s.d_ts, s.h_ts, n * 8, hipMemcpyHostToDevice, p->s_h2d));
  TRY_HIP(hipEventRecord(s.ev_h2d, p->s_h2d));
  // parse (in chunk order on the context's stream: the flow table is shared)
  TRY_HIP(hipStreamWaitEvent(p->s_comp, s.ev_h2d, 0));
  if (W) {
    const unsigned grid = unsigned(n / 256 + 1 < 4096 ? n / 256 + 1 : 4096);
    hipLaunchKernelGGL(k_window_offsets, dim3(grid), dim3(256), 0, p->s_comp, s.d_off, n, W);
    TRY_HIP(hipGetLastError());
  }
  TRY_HIP(hipMemsetAsync(s.d_meta, 0, 8 * sizeof(uint64_t), p->s_comp));
  tcbee_frames din{s.d_arena, s.arena_used, s.d_off, s.d_len, s.d_ts, n};
  const bool flows = !(cfg->flags & TCBEE_F_NO_FLOWS);
  int rc = tcbee_parse_batch_device(p->ctx, &din, cfg, s.d_rec, n, nullptr,
                                    flows ? s.d_id : nullptr, s.d_meta,
                                    reinterpret_cast<tcbee_counters*>(s.d_meta + 1), p->s_comp);
  if (rc) return rc;
  TRY_HIP(hipMemcpyAsync(s.h_meta, s.d_meta, 5 * sizeof(uint64_t), hipMemcpyDeviceToHost,
                         p->s_comp));
  TRY_HIP(hipEventRecord(s.ev_parse, p->s_comp));
  return TCBEE_OK;
}

// D2H of a parsed chunk's records (+ ids): straight into the caller's registered
// arrays at record `first` when the whole chunk fits below out_cap (s.direct),
// else into the slot's pinned staging. Chunks are fetched in order, so `first`
// (records of earlier chunks) is known here.
int fetch(tcbee_pipe* p, Slot& s, bool flows, uint64_t first, uint8_t* dst_rec, uint32_t* dst_id,
          uint64_t out_cap) {
  TRY_HIP(hipEventSynchronize(s.ev_parse));
  s.n_rec = s.h_meta[0];
  s.first_record = first;
  s.direct = dst_rec && first + s.n_rec <= out_cap && (!flows || dst_id);
  if (s.n_rec) {
    uint8_t* rec = s.direct ? dst_rec + first * TCBEE_RECORD_BYTES : s.h_rec;
    uint32_t* id = s.direct ? dst_id + first : s.h_id;
    TRY_HIP(hipMemcpyAsync(rec, s.d_rec, s.n_rec * TCBEE_RECORD_BYTES, hipMemcpyDeviceToHost,
                           p->s_d2h));
    if (flows) TRY_HIP(hipMemcpyAsync(id, s.d_id, s.n_rec * 4, hipMemcpyDeviceToHost, p->s_d2h));
  }
  TRY_HIP(hipEventRecord(s.ev_d2h, p->s_d2h));
  return TCBEE_OK;
}

}  // namespace

extern "C" {

int tcbee_pipe_create(tcbee_pipe** out, int device, const tcbee_pipe_cfg* pc,
                      uint64_t max_flows) {
  if (!out) return TCBEE_EINVAL;
  *out = nullptr;
  tcbee_pipe_cfg c = pc ? *pc : tcbee_pipe_cfg{};
  if (!c.chunk_frames) c.chunk_frames = 1ull << 20;
  if (!c.depth) c.depth = 3;
  if (!c.threads) c.threads = 8;
  if (c.depth < 3 || c.depth > 16 || c.threads > 256) return TCBEE_EINVAL;
  if (c.window && c.window != kLineWindow && (c.window < 80 || (c.window & 15u)))
    return TCBEE_EINVAL;
  if (c.window) c.chunk_bytes = c.chunk_frames * c.window;
  else if (!c.chunk_bytes) c.chunk_bytes = 512ull << 20;
  tcbee_pipe* p = new (std::nothrow) tcbee_pipe;
  if (!p) return TCBEE_ENOMEM;
  p->device = device;
  p->cfg = c;
#if TCBEE_VARIANTS
  // test hook (variants build only): TCBEE_PIPE_NT=0 gathers with memcpy instead of
  // streaming stores
  if (const char* e = std::getenv("TCBEE_PIPE_NT")) p->nt_copy = std::atoi(e);
#endif
  int rc = tcbee_ctx_create(&p->ctx, device, c.chunk_frames, 0, max_flows ? max_flows : 1 << 20);
  if (rc) return free_pipe(p), rc;
  void* cs = nullptr;
  tcbee_ctx_stream(p->ctx, &cs);
  p->s_comp = static_cast<hipStream_t>(cs);
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithFlags(&p->s_h2d, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&p->s_d2h, hipStreamNonBlocking) != hipSuccess)
    return free_pipe(p), TCBEE_EDEVICE;
  try {
    p->slots.resize(c.depth);
    // `threads` in all: with staged outputs a quarter copy records out while the
    // rest gather; with the caller's arrays registered (direct D2H, nothing to copy
    // out) all of them gather
    const unsigned ct = c.threads >= 4 ? c.threads / 4 : 1;
    p->gt_staged = c.threads > ct ? c.threads - ct : 1;
    p->pool = new Pool(c.threads > p->gt_staged ? c.threads : p->gt_staged);
    p->cpool = new Pool(ct);
  } catch (...) {
    return free_pipe(p), TCBEE_ENOMEM;
  }
  for (Slot& s : p->slots)
    if ((rc = alloc_slot(p, s))) return free_pipe(p), rc;
  *out = p;
  return TCBEE_OK;
}

int tcbee_pipe_register_output(tcbee_pipe* p, uint8_t* out_rec74, uint64_t cap,
                               uint32_t* out_flow_id) {
  if (!p || (cap && !out_rec74) || (!cap && (out_rec74 || out_flow_id))) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(p->device));
  TRY_HIP(hipStreamSynchronize(p->s_d2h));  // no D2H into the old arrays in flight
  unregister_output(p);
  if (!cap) return TCBEE_OK;
  TRY_HIP(register_range(out_rec74, cap * TCBEE_RECORD_BYTES));
  p->reg_rec = out_rec74;
  p->reg_rec_bytes = cap * TCBEE_RECORD_BYTES;
  if (out_flow_id) {
    const hipError_t e = register_range(out_flow_id, cap * 4);
    if (e != hipSuccess) {
      unregister_output(p);
      return map_err(e);
    }
    p->reg_id = out_flow_id;
    p->reg_id_bytes = cap * 4;
  }
  p->reg_cap = cap;
  return TCBEE_OK;
}

int tcbee_pipe_destroy(tcbee_pipe* p) {
  if (!p) return TCBEE_EINVAL;
  free_pipe(p);
  return TCBEE_OK;
}

int tcbee_pipe_ctx(tcbee_pipe* p, tcbee_ctx** ctx) {
  if (!p || !ctx) return TCBEE_EINVAL;
  *ctx = p->ctx;
  return TCBEE_OK;
}

int tcbee_pipe_get_stats(const tcbee_pipe* p, tcbee_pipe_stats* st) {
  if (!p || !st) return TCBEE_EINVAL;
  *st = p->st;
  return TCBEE_OK;
}

int tcbee_pipe_run(tcbee_pipe* p, const tcbee_frames* in, const tcbee_cfg* cfg,
                   uint8_t* out_rec74, uint64_t out_cap, uint32_t* out_flow_id,
                   tcbee_pipe_sink_fn fn, void* user, uint64_t* out_n, tcbee_counters* ctr) {
  if (!p || !in || !cfg || !out_n) return TCBEE_EINVAL;
  if (in->n && (!in->arena || !in->offset || !in->caplen || !in->ts_ns)) return TCBEE_EINVAL;
  if (out_cap && !out_rec74) return TCBEE_EINVAL;
  if (!p->cfg.window)
    for (uint64_t i = 0; i < in->n; ++i)
      if (in->caplen[i] > p->cfg.chunk_bytes) return TCBEE_ECAPACITY;
  TRY_HIP(hipSetDevice(p->device));
  const bool flows = !(cfg->flags & TCBEE_F_NO_FLOWS);
  const uint64_t D = p->slots.size();
  // the caller's arrays are the registered ones: chunks D2H straight into them
  const bool reg = p->reg_rec && out_rec74 == p->reg_rec && out_cap <= p->reg_cap &&
                   (!flows || !out_flow_id || out_flow_id == p->reg_id);
  uint8_t* const dst_rec = reg ? out_rec74 : nullptr;
  uint32_t* const dst_id = reg && flows ? out_flow_id : nullptr;
  uint64_t written = 0, records = 0, chunks = 0, fetched_records = 0;
  tcbee_counters sum{};
  int rc = TCBEE_OK;

  // consume(c): counters, records (+ ids) into the caller's arrays, the sink call.
  // It runs on a consumer thread with its own pool, in chunk order, overlapping
  // the main thread's gather of later chunks (both are host-memory bound).
  auto consume = [&](Slot& s) -> int {
    TRY_HIP(hipEventSynchronize(s.ev_d2h));
    sum.ingress += s.h_meta[1];
    sum.egress += s.h_meta[2];
    sum.handled += s.h_meta[3];
    sum.dropped += s.h_meta[4];
    const uint64_t n = s.n_rec;
    const uint8_t* rec = s.direct ? out_rec74 + records * TCBEE_RECORD_BYTES : s.h_rec;
    const uint32_t* ids = s.direct ? (out_flow_id ? out_flow_id + records : nullptr) : s.h_id;
    if (s.direct) {
      written += n;  // already in place
    } else if (out_rec74 && records < out_cap) {
      const uint64_t k = n < out_cap - records ? n : out_cap - records;
      uint8_t* dst = out_rec74 + records * TCBEE_RECORD_BYTES;
      uint32_t* did = out_flow_id ? out_flow_id + records : nullptr;
      p->cpool->run([&](unsigned part, unsigned parts) {
        const uint64_t a = k * part / parts, b = k * (part + 1) / parts;
        std::memcpy(dst + a * TCBEE_RECORD_BYTES, s.h_rec + a * TCBEE_RECORD_BYTES,
                    (b - a) * TCBEE_RECORD_BYTES);
        if (did && flows) std::memcpy(did + a, s.h_id + a, (b - a) * 4);
      });
      written += k;
    }
    records += n;
    if (fn) {
      int urc = fn(user, rec, flows ? ids : nullptr, n, s.first_record);
      if (urc) return urc;
    }
    return TCBEE_OK;
  };
  std::mutex cm;
  std::condition_variable ccv;
  uint64_t queued = 0, done = 0;  // chunks handed to / finished by the consumer
  bool closing = false;
  int crc = TCBEE_OK;
  std::thread consumer([&] {
    (void)hipSetDevice(p->device);
    for (uint64_t j = 0;; ++j) {
      {
        std::unique_lock<std::mutex> lk(cm);
        ccv.wait(lk, [&] { return j < queued || closing; });
        if (j >= queued) return;  // closing, all consumed
      }
      const int r = crc == TCBEE_OK ? consume(p->slots[j % D]) : crc;
      {
        std::lock_guard<std::mutex> g(cm);
        if (r && crc == TCBEE_OK) crc = r;
        done = j + 1;
      }
      ccv.notify_all();
    }
  });
  auto wait_done = [&](uint64_t need) -> int {
    std::unique_lock<std::mutex> lk(cm);
    ccv.wait(lk, [&] { return done >= need || crc != TCBEE_OK; });
    return crc;
  };
  auto hand_over = [&](uint64_t j) {
    {
      std::lock_guard<std::mutex> g(cm);
      queued = j + 1;
    }
    ccv.notify_all();
  };

  // Chunk c lives in slot c % D: it is staged once chunk c - D is consumed; chunk
  // c - 1's records are fetched (D2H) after chunk c is enqueued, so stage(c)
  // overlaps H2D/parse of c - 1 and the consumer's copy-out of earlier chunks.
  uint64_t lo = 0, issued = 0, fetched = 0;
  while (rc == TCBEE_OK && lo < in->n) {
    if (issued >= D && (rc = wait_done(issued - D + 1))) break;
    Slot& s = p->slots[issued % D];
    s.lo = lo;
    s.hi = chunk_end(p, in, lo);
    stage(p, in, s, reg ? 0u : p->gt_staged);
    if ((rc = enqueue(p, s, cfg))) break;
    lo = s.hi;
    ++issued;
    ++chunks;
    if (fetched + 1 < issued) {
      Slot& f = p->slots[fetched % D];
      if ((rc = fetch(p, f, flows, fetched_records, dst_rec, dst_id, out_cap))) break;
      fetched_records += f.n_rec;
      hand_over(fetched++);
    }
  }
  while (rc == TCBEE_OK && fetched < issued) {
    Slot& f = p->slots[fetched % D];
    if ((rc = fetch(p, f, flows, fetched_records, dst_rec, dst_id, out_cap))) break;
    fetched_records += f.n_rec;
    hand_over(fetched++);
  }
  {
    std::lock_guard<std::mutex> g(cm);
    closing = true;
  }
  ccv.notify_all();
  consumer.join();
  if (rc == TCBEE_OK) rc = crc;
  (void)hipStreamSynchronize(p->s_h2d);
  (void)hipStreamSynchronize(p->s_d2h);
  (void)tcbee_ctx_sync(p->ctx);
  if (rc) return rc;
  *out_n = records;
  p->st.frames += in->n;
  p->st.records += records;
  p->st.chunks += chunks;
  if (ctr) {
    ctr->ingress += sum.ingress;
    ctr->egress += sum.egress;
    ctr->handled += sum.handled;
    ctr->dropped += sum.dropped;
  }
  // records beyond out_cap were produced and handed to fn but not copied
  if (out_rec74 && records > out_cap) return TCBEE_ECAPACITY;
  return tcbee_ctx_status(p->ctx);
}

}  // extern "C"

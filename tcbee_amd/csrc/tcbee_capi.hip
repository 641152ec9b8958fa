// tcbee_capi.hip — the C ABI (include/tcbee_amd.h) over the HIP kernels.
// No exceptions cross this boundary; every entry point returns a TCBEE_* code.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>
#include <utility>
#include <vector>

#include "../../include/tcbee_amd.h"
#include "tcbee_gen.h"
#include "tcbee_internal.h"
#include "tcbee_layout.h"

using namespace tcbee;

struct tcbee_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t max_frames = 0, max_arena = 0, max_flows = 0;
  int fpl = TCBEE_K1_FPL;
  bool reset_pending = false;   // tcbee_flow_reset_device: applied by the next launch
  uint32_t withhold_every = 0;  // TCBEE_TEST_WITHHOLD (look-back recount test hook)
  int k3_no_bucket = 0;         // TCBEE_TEST_K3_NOBUCKET=1: large tables use K3 mode 2 (test hook)
  bool k3_twopass = false;      // TCBEE_TEST_K3_TWOPASS=1: mode 1 by the two-pass scatter
                                // at any bucket count (test hook; the product takes it
                                // only past kChunkMaxNb buckets)
  bool k3_wide = false;         // TCBEE_TEST_K3_WIDE=1: 16 records per lane in k_count on
                                // every batch (test hook; the product: >= kK3WideFrames)
  bool k3_range = false;        // K3 mode 3 available (part rows sized for it)
  uint32_t plain_walk = kPlainWalk;  // TCBEE_WALK: K1 plain probe walk length (test hook:
                                     // 0 sends every foreign slot to the coherent path)
  bool no_fuse_rank = false;         // TCBEE_NO_FUSE_RANK: the separate rank launch (A/B, tests)
  // TCBEE_TEST_LEGACY_INIT (test hook, variants build only): the creation path of
  // rounds 1-5 before bccf225 — creation-time memsets through hipMemset on HIP's legacy
  // default stream, and a NULL-stream call NOT ordered after that stream — so a test
  // can reproduce the round-5 all-zero-id race on purpose
  bool legacy_init = false;
#if TCBEE_VARIANTS
  const uint64_t* test_hold = nullptr;  // tcbee_test_k2_hold
  uint64_t* test_hold_state = nullptr;
#endif
  uint32_t pack_bits = 0;            // K1->K3 scratch packing (0: two words per record)

  FlowTable tab{};
  uint64_t nlines = 0;  // flow-table slot lines (6 slots of 16 B each)
  PersistState* d_persist = nullptr;
  // Small contexts (max_flows <= kFuseRankMax): two table generations (slot units,
  // wide slots, counters, persist state; the per-claim key / first_seen / id arrays
  // are shared), so that a reset is a switch to the other, already empty generation
  // and a fused batch needs no k_prep launch: its K3 empties the inactive
  // generation, zeroes the tile words and the next batch's state slot (round 4)
  bool small_gen = false;
  FlowTable tab_alt{};
  PersistState* d_persist_alt = nullptr;
  bool alt_clean = true;    // the inactive generation is empty (or being emptied in order)
  bool prepped = false;     // the last batch's K3 prepared the next one (tile words, slot)
  uint64_t tiles_hw = 0;    // tile words used since they were all last zeroed
  BatchState* d_batch = nullptr;     // = d_batch_slot[slot] of the current batch
  // two slots of what a batch's K3 reads (batch state, K1 -> K3 scratch), so that
  // with TCBEE_EX_ASYNC_IDS batch i's K3 (ids stream) runs beside batch i+1's K1;
  // the second slot is allocated on the first async call
  BatchState* d_batch_slot[2] = {nullptr, nullptr};
  uint32_t* d_slot_scratch_s[2] = {nullptr, nullptr};
  uint32_t* d_len_scratch_s[2] = {nullptr, nullptr};
  int slot = 0, nslot = 1;
  hipEvent_t ev_k2 = nullptr, ev_k3 = nullptr, ev_fin = nullptr;
  hipEvent_t ev_null = nullptr;  // a NULL-stream call: the legacy default stream's work so far
  bool k3_async = false;        // a K3 is (or may be) running on another stream
  hipStream_t pend_ids = nullptr;  // deferred + async: the ids stream
  uint64_t* d_tile_status = nullptr;
  uint64_t max_tiles = 0;
  uint64_t* d_new_list = nullptr;
  uint32_t* d_new_fs = nullptr;     // K2 scratch: new flows' local first_seen
  uint32_t* d_bitmap = nullptr;
  uint32_t* d_wprefix = nullptr;
  uint32_t* d_bprefix = nullptr;
  uint32_t* d_slot_scratch = nullptr;
  uint32_t* d_len_scratch = nullptr;
  uint64_t* d_count_part = nullptr;  // K3 mode 0 per-block partial bins [k3_g1max][kCountBins]
  uint32_t* d_k3_region = nullptr;   // K3 mode 1 (tables with > kCountBins slots only)
  uint32_t* d_k3_offs = nullptr;
  uint64_t* d_k3_lpart = nullptr;
  uint32_t* d_k3_coffs = nullptr;    // k_count_chunk2: bucket offsets per kChunk records
  uint32_t k3_nb_max = 0, k3_g2 = 0;
  uint64_t k3_g1max = 0, part_words = 0;
  int n_cu = 256;
  uint64_t max_words = 0, max_sblocks = 0;

  // host-pointer path staging (allocated on first use)
  uint8_t* d_arena = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_len = nullptr;
  uint64_t* d_ts = nullptr;
  uint8_t* d_rec = nullptr;
  uint32_t* d_hash = nullptr;
  uint32_t* d_id = nullptr;
  uint64_t* d_n = nullptr;
  tcbee_counters* d_ctr = nullptr;

  // multi-table merge scratch (allocated on first merge, grown on demand)
  uint64_t* d_mcnt = nullptr;
  uint32_t* d_mbitmap = nullptr;
  uint32_t* d_mwprefix = nullptr;
  uint32_t* d_mbprefix = nullptr;
  uint64_t m_words = 0;

  // deferred K3 (TCBEE_EX_DEFER_IDS): launched by tcbee_parse_finish_device
  bool count_pending = false;
  bool pend_empty = false;  // deferred batch had no K3 (empty / no flows): finish is a no-op
  CountArgs pend{};
  unsigned pend_g1 = 0, pend_g1s = 0, pend_g2 = 0;
  uint32_t* d_omap = nullptr;  // composed claim -> output id (allocated on first use)

  // K1 timing (tcbee_ctx_profile)
  bool profiling = false;
  std::vector<hipEvent_t> ev;  // pairs
  uint64_t ev_used = 0;
};

// A call's stream: the caller's, or (NULL) the context's own non-blocking stream,
// ordered after whatever is already queued on the legacy default stream (a caller's
// default-stream producers of the inputs, or zero-fills of the outputs, would
// otherwise race the parse: the context's stream does not wait for that stream).
// The context's device is made current first (the legacy stream recorded
// below is the CURRENT device's, so a thread driving several GPUs must not record
// another device's default stream into ev_null).
static hipError_t ctx_stream(tcbee_ctx* c, void* stream, hipStream_t& s) {
  if (hipError_t e = hipSetDevice(c->device); e != hipSuccess) return e;
  if (stream) {
    s = (hipStream_t)stream;
    return hipSuccess;
  }
  s = c->stream;
  if (c->legacy_init) return hipSuccess;  // (test hook: the unordered pre-fix path)
  hipError_t e = hipEventRecord(c->ev_null, nullptr);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ev_null, 0);
  return e;
}
// Creation-time fills: on the context's stream (create synchronizes it before it
// returns), or under the legacy-init test hook on the legacy default stream as the
// pre-fix code did.
static hipError_t init_fill(tcbee_ctx* c, void* p, int v, size_t bytes) {
  return c->legacy_init ? hipMemset(p, v, bytes) : hipMemsetAsync(p, v, bytes, c->stream);
}
static hipError_t init_fill_2d(tcbee_ctx* c, void* p, size_t pitch, int v, size_t w, size_t h) {
  return c->legacy_init ? hipMemset2D(p, pitch, v, w, h)
                        : hipMemset2DAsync(p, pitch, v, w, h, c->stream);
}
static constexpr uint64_t kMaxProfiled = 4096;

namespace {

int map_err(hipError_t e) {
  if (e == hipSuccess) return TCBEE_OK;
  if (e == hipErrorOutOfMemory) return TCBEE_ENOMEM;
  if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return TCBEE_ENODEV;
  return TCBEE_EDEVICE;
}

#define TRY_HIP(expr)                          \
  do {                                         \
    hipError_t e_ = (expr);                    \
    if (e_ != hipSuccess) return map_err(e_);  \
  } while (0)

template <class T>
hipError_t dalloc(T** p, uint64_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  return hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

uint64_t tile_frames(int fpl) { return (uint64_t)kK1Block * (uint64_t)fpl; }

int ensure_host_path(tcbee_ctx* c) {
  if (c->d_arena) return TCBEE_OK;
  TRY_HIP(dalloc(&c->d_arena, c->max_arena + 16));
  TRY_HIP(dalloc(&c->d_off, c->max_frames));
  TRY_HIP(dalloc(&c->d_len, c->max_frames));
  TRY_HIP(dalloc(&c->d_ts, c->max_frames));
  TRY_HIP(dalloc(&c->d_rec, c->max_frames * kRecBytes + 16));
  TRY_HIP(dalloc(&c->d_hash, c->max_frames));
  TRY_HIP(dalloc(&c->d_id, c->max_frames));
  TRY_HIP(dalloc(&c->d_n, 1));
  TRY_HIP(dalloc(&c->d_ctr, 1));
  return TCBEE_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Ordering against a K3 that runs on another stream (TCBEE_EX_ASYNC_IDS): host
// reads of the table wait for it; device work on `s` that reads what it writes
// (counters, ids) is queued behind it.
hipError_t k3_wait_host(tcbee_ctx* c) {
  return c->k3_async ? hipEventSynchronize(c->ev_k3) : hipSuccess;
}
hipError_t k3_wait_stream(tcbee_ctx* c, hipStream_t s) {
  return c->k3_async ? hipStreamWaitEvent(s, c->ev_k3, 0) : hipSuccess;
}

}  // namespace

extern "C" {

int tcbee_abi_version(void) { return TCBEE_ABI_VERSION; }

const char* tcbee_strerror(int code) {
  switch (code) {
    case TCBEE_OK: return "ok";
    case TCBEE_EINVAL: return "invalid argument";
    case TCBEE_ENOMEM: return "out of memory";
    case TCBEE_EDEVICE: return "HIP device error";
    case TCBEE_ECAPACITY: return "batch exceeds context capacity";
    case TCBEE_EFLOWFULL: return "flow table full";
    case TCBEE_ENODEV: return "no HIP device";
    case TCBEE_EIO: return "I/O error";
    case TCBEE_EFORMAT: return "malformed input";
    case TCBEE_ESPIN: return "in-kernel wait timed out";
    case TCBEE_EDB: return "database statement failed";
    case TCBEE_ESHARD: return "global-order export could not place a flow's first record";
    default: return "unknown error";
  }
}

int tcbee_device_count(int* n) {
  if (!n) return TCBEE_EINVAL;
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return TCBEE_OK;
}

int tcbee_ctx_destroy(tcbee_ctx* c) {
  if (!c) return TCBEE_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  dfree(c->tab.slots);
  dfree(c->tab.ent);
  dfree(c->tab.cfs);
  dfree(c->d_new_fs);
  dfree(c->tab.wide);
  dfree(c->tab.wide_used);
  dfree(c->tab.cnt);
  dfree(c->tab.cmap);
  dfree(c->d_persist);
  if (c->small_gen) {  // (the alt generation's own arrays; ent / cfs / cmap are shared)
    dfree(c->tab_alt.slots);
    dfree(c->tab_alt.wide);
    dfree(c->tab_alt.wide_used);
    dfree(c->tab_alt.cnt);
    dfree(c->d_persist_alt);
  }
  if (c->k3_async && c->ev_k3) (void)hipEventSynchronize(c->ev_k3);
  for (int i = 0; i < 2; ++i) {
    dfree(c->d_batch_slot[i]);
    if (i) {  // slot 0's scratch is d_slot_scratch / d_len_scratch, freed below
      dfree(c->d_slot_scratch_s[i]);
      dfree(c->d_len_scratch_s[i]);
    }
  }
  for (hipEvent_t e : {c->ev_k2, c->ev_k3, c->ev_fin, c->ev_null})
    if (e) (void)hipEventDestroy(e);
  dfree(c->d_tile_status);
  dfree(c->d_new_list);
  dfree(c->d_bitmap);
  dfree(c->d_wprefix);
  dfree(c->d_bprefix);
  dfree(c->d_slot_scratch);
  dfree(c->d_len_scratch);
  dfree(c->d_count_part);
  dfree(c->d_k3_region);
  dfree(c->d_k3_offs);
  dfree(c->d_k3_lpart);
  dfree(c->d_k3_coffs);
  dfree(c->d_arena);
  dfree(c->d_off);
  dfree(c->d_len);
  dfree(c->d_ts);
  dfree(c->d_rec);
  dfree(c->d_hash);
  dfree(c->d_id);
  dfree(c->d_n);
  dfree(c->d_ctr);
  dfree(c->d_mcnt);
  dfree(c->d_mbitmap);
  dfree(c->d_mwprefix);
  dfree(c->d_mbprefix);
  dfree(c->d_omap);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return TCBEE_OK;
}

int tcbee_ctx_create(tcbee_ctx** out, int device, uint64_t max_frames, uint64_t max_arena,
                     uint64_t max_flows) {
  return tcbee_ctx_create_ex(out, device, max_frames, max_arena, max_flows, max_flows);
}

int tcbee_ctx_create_ex(tcbee_ctx** out, int device, uint64_t max_frames, uint64_t max_arena,
                        uint64_t max_flows, uint64_t max_wide_flows) {
  if (!out || max_frames == 0) return TCBEE_EINVAL;
  // batch-local record / frame indices are 31-bit (the flow table's fs32 words)
  if (max_frames >= (1ull << 31)) return TCBEE_ECAPACITY;
  *out = nullptr;
  // 2^24 flows -> 2^25 slots = 2 GiB of table: K1's probe buffer resource and u32
  // slot offsets, and K3's bucketed mode (kMaxBuckets x kBucket claims), end there
  if (max_flows > kMaxTableFlows) return TCBEE_ECAPACITY;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return TCBEE_ENODEV;
  if (device < 0 || device >= ndev) return TCBEE_EINVAL;
  tcbee_ctx* c = new (std::nothrow) tcbee_ctx();
  if (!c) return TCBEE_ENOMEM;
  c->device = device;
  c->max_frames = max_frames;
  c->max_arena = max_arena;
  c->max_flows = max_flows < 16 ? 16 : max_flows;
#if TCBEE_VARIANTS
  // test hooks and A/B variants, read from the environment by the variants build
  // only (libtcbee_amd_variants.so: tests of alternative paths, tools/); the product
  // library reads no environment variable
  if (const char* e = std::getenv("TCBEE_TEST_WITHHOLD")) c->withhold_every = (uint32_t)std::atoi(e);
  if (const char* e = std::getenv("TCBEE_TEST_K3_NOBUCKET")) c->k3_no_bucket = std::atoi(e);
  if (const char* e = std::getenv("TCBEE_TEST_K3_TWOPASS")) c->k3_twopass = std::atoi(e) != 0;
  if (const char* e = std::getenv("TCBEE_TEST_K3_WIDE")) c->k3_wide = std::atoi(e) != 0;
  if (const char* e = std::getenv("TCBEE_WALK")) c->plain_walk = (uint32_t)std::atoi(e);
  if (const char* e = std::getenv("TCBEE_NO_FUSE_RANK")) c->no_fuse_rank = std::atoi(e) != 0;
  if (const char* e = std::getenv("TCBEE_TEST_LEGACY_INIT")) c->legacy_init = std::atoi(e) != 0;
  if (const char* e = std::getenv("TCBEE_FPL")) {
    const int v = std::atoi(e);
    if (v == 1 || v == 2 || v == 4) c->fpl = v;
  }
#endif
  int rc = TCBEE_OK;
  auto fail = [&](int code) {
    tcbee_ctx_destroy(c);
    return code;
  };
  if (hipSetDevice(device) != hipSuccess) return fail(TCBEE_EDEVICE);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
    return fail(TCBEE_EDEVICE);
  // kSlotsPerFlow x max_flows slots (load <= 1/8), 3 per 64-B unit
  c->nlines = (kSlotsPerFlow * c->max_flows + kSlotsPerLine - 1) / kSlotsPerLine;
  c->tab.nlines = c->nlines;
  c->tab.max_claims = c->max_flows;
  // wide-slot (non-IPv4-form: IPv6) keys: at most max_wide_flows of them (16..max_flows)
  c->tab.max_wide = max_wide_flows < 16 ? 16 : (max_wide_flows < c->max_flows ? max_wide_flows
                                                                                : c->max_flows);
  {
    // claims < max_flows: ceil(log2(max_flows)) bits + 1 (so no packed word is all
    // ones, the no-flow mark); packed while at least 11 bits remain (a standard
    // Ethernet frame's 1518 B fits the 11 bits left at b = 21, max_flows <= 2^20;
    // longer caplens saturate the field and go to the side array)
    uint32_t b = 1;
    while ((1ull << (b - 1)) < c->max_flows) ++b;
    c->pack_bits = b <= 21 ? b : 0;
#if TCBEE_VARIANTS
    if (const char* e = std::getenv("TCBEE_TEST_NOPACK")) c->pack_bits = std::atoi(e) ? 0 : c->pack_bits;
#endif
  }
  c->max_tiles = (max_frames + tile_frames(1) - 1) / tile_frames(1);
  c->max_words = (max_frames + 31) / 32;
  c->max_sblocks = (c->max_words + kScanWordsPerBlock - 1) / kScanWordsPerBlock;
  hipError_t e = hipSuccess;
  if ((e = dalloc(&c->tab.slots, 8 * c->nlines)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->tab.ent, 8 * c->max_flows)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->tab.cfs, c->max_flows)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_new_fs, c->max_flows)) != hipSuccess) return fail(map_err(e));
  // wide slots (non-IPv4-form keys): a power of two >= kSlotsPerFlow x max_wide,
  // at most 2^25 (2 GiB: K1's probe buffer resource and u32 offsets); 64 B each
  c->tab.wide_mask = 63;
  while (c->tab.wide_mask + 1 < kSlotsPerFlow * c->tab.max_wide && c->tab.wide_mask + 1 < (1ull << 25))
    c->tab.wide_mask = 2 * c->tab.wide_mask + 1;
  if ((e = dalloc(&c->tab.wide, 8 * (c->tab.wide_mask + 1))) != hipSuccess) return fail(map_err(e));
  // all ones, then every tag word zero (k_table_init sweeps the wide slots only once
  // used): fs words ~0 as a reset leaves them
  if ((e = init_fill(c, c->tab.wide, 0xFF, 64 * (c->tab.wide_mask + 1))) != hipSuccess) return fail(map_err(e));
  if ((e = init_fill_2d(c, c->tab.wide, 64, 0, 8, c->tab.wide_mask + 1)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->tab.wide_used, 1)) != hipSuccess) return fail(map_err(e));
  if ((e = init_fill(c, c->tab.wide_used, 0, 4)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->tab.cnt, 2 * c->max_flows)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->tab.cmap, c->max_flows)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_persist, 1)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_batch_slot[0], 1)) != hipSuccess) return fail(map_err(e));
  c->d_batch = c->d_batch_slot[0];
  for (hipEvent_t* ev : {&c->ev_k2, &c->ev_k3, &c->ev_fin, &c->ev_null})
    if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess)
      return fail(map_err(e));
  if ((e = dalloc(&c->d_tile_status, c->max_tiles)) != hipSuccess) return fail(map_err(e));
  // all zero between batches of small contexts (their K3 re-zeroes the words a batch used)
  if ((e = init_fill(c, c->d_tile_status, 0, c->max_tiles * sizeof(uint64_t))) != hipSuccess)
    return fail(map_err(e));
  if ((e = dalloc(&c->d_new_list, c->max_flows)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_bitmap, c->max_words)) != hipSuccess) return fail(map_err(e));
  // all zero between batches from here on (K3 clears the words a batch set)
  if ((e = init_fill(c, c->d_bitmap, 0, c->max_words * sizeof(uint32_t))) != hipSuccess)
    return fail(map_err(e));
  if ((e = dalloc(&c->d_wprefix, c->max_words)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_bprefix, c->max_sblocks)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_slot_scratch, max_frames)) != hipSuccess) return fail(map_err(e));
  if ((e = dalloc(&c->d_len_scratch, max_frames)) != hipSuccess) return fail(map_err(e));
  c->d_slot_scratch_s[0] = c->d_slot_scratch;
  c->d_len_scratch_s[0] = c->d_len_scratch;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    c->n_cu = prop.multiProcessorCount;
  // K3's grid (launch site): at most max(n_cu, blocks for < 2^24 records each),
  // one partial-bin row each
  c->k3_g1max = (max_frames + kK3MaxPer - 1) / kK3MaxPer;
  if (c->k3_g1max < (uint64_t)c->n_cu) c->k3_g1max = c->n_cu;
  // (tables past kCountBins slots also hold K3 mode 3's per-group rows: at most
  //  8 x (g1 / 8 / 2) groups x kRangeFlows claims; TCBEE_TEST_K3_NORANGE=1 keeps
  //  such tables on modes 1/2 — a test hook)
  uint64_t part_words = c->k3_g1max * kCountBins;
  c->k3_range = c->max_flows > (uint64_t)kCountBins;
#if TCBEE_VARIANTS
  if (const char* e = std::getenv("TCBEE_TEST_K3_NORANGE")) c->k3_range = c->k3_range && !std::atoi(e);
#endif
  if (c->k3_range) {
    const uint64_t rows = (uint64_t)c->n_cu / 2;  // R >= 2 in mode 3: <= g1/16 groups x 8
    if (rows * kRangeFlows > part_words) part_words = rows * kRangeFlows;
  }
  c->part_words = part_words;
  if ((e = dalloc(&c->d_count_part, part_words)) != hipSuccess)
    return fail(map_err(e));
  if (c->max_flows > (uint64_t)kCountBins && !c->k3_no_bucket) {
    // K3 mode 1 scratch: (claim, caplen) per frame, bucket offsets per K3 block,
    // partial rows of k_count_bucket (S x nb <= g2 rows of kBucket claims)
    uint64_t nb = (c->max_flows + kBucket - 1) / kBucket;
    c->k3_nb_max = (uint32_t)(nb < kMaxBuckets ? nb : kMaxBuckets);
    c->k3_g2 = c->k3_nb_max > 2u * c->n_cu ? c->k3_nb_max : 2u * c->n_cu;
    if ((e = dalloc(&c->d_k3_region, max_frames)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->d_k3_offs, 2ull * c->n_cu * (c->k3_nb_max + 1))) != hipSuccess)
      return fail(map_err(e));
    if ((e = dalloc(&c->d_k3_lpart, 2ull * c->k3_g2 * kBucket)) != hipSuccess)
      return fail(map_err(e));
    // single-pass chunked scatter (batches of < kChunkMaxNb buckets): offsets of every
    // chunk's buckets (4 B x 512 per 12288 frames)
    if ((e = dalloc(&c->d_k3_coffs, ((max_frames + kChunk - 1) / kChunk + 1) * (kChunkMaxNb + 1))) !=
        hipSuccess)
      return fail(map_err(e));
  }
  if (c->max_flows <= kFuseRankMax && c->max_frames <= kRankSmallWords * 32) {
    // the second table generation and the second batch-state slot (K1 -> K3 scratch
    // of both slots too: batches alternate slots from now on). Only for contexts whose
    // every batch can take the fused, prep-free path (<= kRankSmallWords * 32 = 1M
    // frames): a small-flow context with a larger max_frames would double
    // its 8 B/frame of scratch for batches that cannot use it
    c->small_gen = true;
    c->tab_alt = c->tab;
    c->tab_alt.slots = nullptr;
    c->tab_alt.wide = nullptr;
    c->tab_alt.wide_used = nullptr;
    c->tab_alt.cnt = nullptr;
    if ((e = dalloc(&c->tab_alt.slots, 8 * c->nlines)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->tab_alt.wide, 8 * (c->tab.wide_mask + 1))) != hipSuccess) return fail(map_err(e));
    if ((e = init_fill(c, c->tab_alt.wide, 0xFF, 64 * (c->tab.wide_mask + 1))) != hipSuccess) return fail(map_err(e));
    if ((e = init_fill_2d(c, c->tab_alt.wide, 64, 0, 8, c->tab.wide_mask + 1)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->tab_alt.wide_used, 1)) != hipSuccess) return fail(map_err(e));
    if ((e = init_fill(c, c->tab_alt.wide_used, 0, 4)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->tab_alt.cnt, 2 * c->max_flows)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->d_persist_alt, 1)) != hipSuccess) return fail(map_err(e));
    if ((e = init_fill(c, c->d_persist_alt, 0, sizeof(PersistState))) != hipSuccess) return fail(map_err(e));
    if ((e = launch_table_init(c->tab_alt, c->stream)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->d_batch_slot[1], 1)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->d_slot_scratch_s[1], c->max_frames)) != hipSuccess) return fail(map_err(e));
    if ((e = dalloc(&c->d_len_scratch_s[1], c->max_frames)) != hipSuccess) return fail(map_err(e));
    c->nslot = 2;
  }
  rc = tcbee_flow_reset(c);
  if (rc != TCBEE_OK) return fail(rc);
  *out = c;
  return TCBEE_OK;
}

int tcbee_ctx_stream(tcbee_ctx* c, void** stream) {
  if (!c || !stream) return TCBEE_EINVAL;
  *stream = (void*)c->stream;
  return TCBEE_OK;
}

int tcbee_ctx_sync(tcbee_ctx* c) {
  if (!c) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  TRY_HIP(k3_wait_host(c));
  TRY_HIP(hipStreamSynchronize(c->stream));
  return TCBEE_OK;
}

int tcbee_flow_reset(tcbee_ctx* c) {
  if (!c) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  TRY_HIP(k3_wait_host(c));
  TRY_HIP(launch_table_init(c->tab, c->stream));
  TRY_HIP(hipMemsetAsync(c->d_persist, 0, sizeof(PersistState), c->stream));
  // also the recovery point after a failed batch: the first-seen bitmap is whole-zero
  TRY_HIP(hipMemsetAsync(c->d_bitmap, 0, c->max_words * sizeof(uint32_t), c->stream));
  TRY_HIP(hipStreamSynchronize(c->stream));
  c->reset_pending = false;
  return TCBEE_OK;
}

int tcbee_flow_reset_device(tcbee_ctx* c, void* stream) {
  if (!c) return TCBEE_EINVAL;
  (void)stream;  // folded into the next parse's prep kernel (or applied before a table read)
  c->reset_pending = true;
  return TCBEE_OK;
}

namespace {
int apply_pending_reset(tcbee_ctx* c, hipStream_t s) {
  if (!c->reset_pending) return TCBEE_OK;
  TRY_HIP(launch_table_init(c->tab, s));
  TRY_HIP(hipMemsetAsync(c->d_persist, 0, sizeof(PersistState), s));
  c->reset_pending = false;
  return TCBEE_OK;
}
}  // namespace

int tcbee_parse_batch_device_ex(tcbee_ctx* c, const tcbee_frames* in, const tcbee_cfg* cfg,
                                uint8_t* out_rec74, uint64_t out_cap, uint32_t* out_flow_hash,
                                uint32_t* out_flow_id, uint64_t* out_n_dev,
                                tcbee_counters* ctr_dev, const tcbee_parse_ex* ex, void* stream) {
  if (!c || !in || !cfg) return TCBEE_EINVAL;
  if (c->count_pending) return TCBEE_EINVAL;  // tcbee_parse_finish_device first
  uint32_t* out_frame = ex ? ex->out_frame_index : nullptr;
  const bool defer = ex && (ex->flags & TCBEE_EX_DEFER_IDS);
  const bool async = ex && (ex->flags & TCBEE_EX_ASYNC_IDS);
  hipStream_t ids_stream = async ? (hipStream_t)ex->ids_stream : nullptr;
  if (ex) {
    if (ex->flags & ~(TCBEE_EX_DEFER_IDS | TCBEE_EX_ASYNC_IDS) || ex->reserved32) return TCBEE_EINVAL;
    if (async && !ids_stream) return TCBEE_EINVAL;
    if (!async && ex->ids_stream) return TCBEE_EINVAL;
    for (uint64_t r : ex->reserved)
      if (r) return TCBEE_EINVAL;
  }
  if (out_frame && in->n > 0xFFFFFFFFull) return TCBEE_EINVAL;  // u32 frame indices
  if (cfg->direction > 1) return TCBEE_EINVAL;
  if (in->n > c->max_frames) return TCBEE_ECAPACITY;
  if (in->n && (!in->arena || !in->offset || !in->caplen || !in->ts_ns)) return TCBEE_EINVAL;
  if (out_cap && !out_rec74) return TCBEE_EINVAL;
  if ((in->arena && !aligned16(in->arena)) || (out_rec74 && !aligned16(out_rec74)))
    return TCBEE_EINVAL;
  const bool flows = (cfg->flags & TCBEE_F_NO_FLOWS) == 0;
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));  // (sets c->device current)
  if (async && c->nslot < 2) {
    // first async batch: the second slot (setup, synchronous allocation)
    TRY_HIP(dalloc(&c->d_batch_slot[1], 1));
    TRY_HIP(dalloc(&c->d_slot_scratch_s[1], c->max_frames));
    TRY_HIP(dalloc(&c->d_len_scratch_s[1], c->max_frames));
    c->nslot = 2;
  }
  if (c->nslot == 2) c->slot ^= 1;  // batches alternate slots once two exist
  c->d_batch = c->d_batch_slot[c->slot];
  uint32_t* const acc_flow = c->d_slot_scratch_s[c->slot];
  uint32_t* const acc_len = c->d_len_scratch_s[c->slot];
  const int fpl = c->fpl;
  const uint64_t tf = tile_frames(fpl);
  const uint64_t ntiles = (in->n + tf - 1) / tf;
  const uint64_t nwords = flows && ntiles ? (in->n + 31) / 32 : 0;
  // a small context's batch that K2 would rank in one block: K3's blocks rank it
  // themselves (one launch fewer per batch; config 2: 1M frames of one flow)
  const bool fuse = flows && ntiles > 0 && nwords <= kRankSmallWords && c->max_flows <= kFuseRankMax &&
                    !defer && !async && !c->no_fuse_rank;
  // small contexts: no k_prep launch when the previous batch's K3 prepared this one
  // (tile words and this slot zero) and the table needs no reset, or the reset is a
  // switch to the other generation, which that K3 emptied
  const bool gen = c->small_gen && fuse;
  bool skip_prep = false;
  if (gen && c->prepped) {
    if (!c->reset_pending) {
      skip_prep = true;
    } else if (c->alt_clean) {
      std::swap(c->tab, c->tab_alt);
      std::swap(c->d_persist, c->d_persist_alt);
      c->reset_pending = false;
      c->alt_clean = false;  // the old generation: emptied by this batch's K3
      skip_prep = true;
    }
  }
  c->prepped = false;  // (set again below when this batch's K3 prepares the next one)
  if (c->tiles_hw < ntiles) c->tiles_hw = ntiles;
  if (!skip_prep) {
    PrepArgs pa{};
    pa.batch = c->d_batch;
    pa.tile_status = c->d_tile_status;
    pa.ntiles = ntiles;
    pa.reset = c->reset_pending;
    if (fuse) {
      // k_prep zeroes the counters of ids not handed out yet: after the previous
      // batch's K3, wherever that ran
      TRY_HIP(k3_wait_stream(c, s));
      pa.zero_free_counters = true;
    }
    pa.tab = c->tab;
    pa.persist = c->d_persist;
    TRY_HIP(launch_prep(pa, s));
    c->reset_pending = false;
  }
  if (ntiles > 0) {
    ParseArgs a{};
    a.arena = in->arena;
    a.arena_len = in->arena_len;
    a.offset = in->offset;
    a.caplen = in->caplen;
    a.ts = in->ts_ns;
    a.n = in->n;
    a.out_rec = out_rec74;
    a.out_cap = out_cap;
    a.out_hash = flows ? out_flow_hash : nullptr;
    a.acc_flow = acc_flow;
    a.acc_len = acc_len;
    a.tile_status = c->d_tile_status;
    a.ntiles = ntiles;
    a.batch = c->d_batch;
    a.persist = c->d_persist;
    a.new_list = c->d_new_list;
    a.tab = c->tab;
    a.filter_port = cfg->filter_port;
    a.withhold_every = c->withhold_every;
    a.plain_walk = c->plain_walk;
    a.pack_bits = c->pack_bits;
    a.out_frame = out_frame;
    const bool timed = c->profiling && c->ev_used < kMaxProfiled;
    if (timed) TRY_HIP(hipEventRecord(c->ev[2 * c->ev_used], s));
    TRY_HIP(launch_parse(a, fpl, flows, s));
    if (timed) {
      TRY_HIP(hipEventRecord(c->ev[2 * c->ev_used + 1], s));
      ++c->ev_used;
    }
  }
  if (flows && ntiles > 0) {
    RankArgs r{};
    r.new_list = c->d_new_list;
    r.new_fs = c->d_new_fs;
    r.batch = c->d_batch;
    r.persist = c->d_persist;
    r.tab = c->tab;
    r.bitmap = c->d_bitmap;
    r.wprefix = c->d_wprefix;
    r.bprefix = c->d_bprefix;
    r.nwords = nwords;
    r.nblocks = (r.nwords + kScanWordsPerBlock - 1) / kScanWordsPerBlock;
    r.update_persist = true;
#if TCBEE_VARIANTS
    r.test_hold = c->test_hold;
    r.test_hold_state = c->test_hold_state;
#endif
    // K2 rewrites claim -> id entries, zeroes new ids' counters and the bitmap K3
    // clears: after the previous batch's K3, wherever that ran
    TRY_HIP(k3_wait_stream(c, s));
    if (!fuse) TRY_HIP(launch_rank(r, s));
    CountArgs k{};
    k.fused_rank = fuse ? 1u : 0u;
    k.wide_iter = (in->n >= kK3WideFrames || c->k3_wide) ? 1u : 0u;
    k.new_list = c->d_new_list;
    k.batch_rw = c->d_batch;
    k.tab = c->tab;
    k.out_n = out_n_dev;
    k.ctr = ctr_dev;
    k.direction = cfg->direction;
    k.persist_rw = c->d_persist;
    k.acc_flow = acc_flow;
    k.pack_bits = c->pack_bits;
    k.acc_len = acc_len;
    k.out_id = out_flow_id;
    k.out_cap = out_cap;
    k.batch = c->d_batch;
    k.persist = c->d_persist;
    k.cmap = c->tab.cmap;
    k.omap = c->tab.cmap;
    k.bitmap = c->d_bitmap;
    k.cnt = c->tab.cnt;
    k.part = c->d_count_part;
    k.range_ok = c->k3_range ? 1u : 0u;
    k.part_words = c->part_words;
    k.region = c->d_k3_region;
    k.offs = c->d_k3_offs;
    k.nb_max = c->k3_nb_max;
    k.lpart = c->d_k3_lpart;
    k.coffs = c->d_k3_coffs;
    k.chunk_off = c->k3_twopass ? 1u : 0u;
    if (gen) {  // this K3 prepares the next batch (see skip_prep above)
      k.clean_tiles = c->d_tile_status;
      k.clean_ntiles = c->tiles_hw;
      k.next_batch = c->d_batch_slot[c->slot ^ 1];
      k.clean_alt = c->alt_clean ? 0u : 1u;
      k.alt = c->tab_alt;
      k.alt_persist = c->d_persist_alt;
    }
    // trade-off: more blocks = more latency hidden; each block writes a partial row
    // of every flow, so a block should see a few thousand records; and a block
    // never covers more than kK3MaxPer records (bin fields cannot overflow)
    // (16384 records per block below n_cu blocks: config 2's step -2.4 % against 8192,
    //  32768 +11 %, profiles/r06_config2_attempts.log; 4096 / 2048 were slower, round 2)
    uint64_t g1 = (in->n + 16383) / 16384;
    if (g1 > (uint64_t)c->n_cu) g1 = c->n_cu;
    const uint64_t gmin = (in->n + kK3MaxPer - 1) / kK3MaxPer;
    if (g1 < gmin) g1 = gmin;
    if (g1 == 0) g1 = 1;
    if (c->k3_range) {
      // mode 3 needs whole XCD columns of R >= 2 blocks: a multiple of 8, >= 128
      // blocks where the chip has them (each block then covers fewer records)
      const uint64_t want = (uint64_t)c->n_cu / 8 * 8 < 128 ? (uint64_t)c->n_cu / 8 * 8 : 128;
      uint64_t g = (g1 + 7) / 8 * 8;
      if (g < want) g = want;
      if (g <= c->k3_g1max) g1 = g;
    }
    k.g1 = (uint32_t)g1;
    // finalize is folded into k_count's block 0
    // mode-1 scatter: two 1024-thread workgroups per CU (its offsets rows: 2 n_cu)
    uint64_t g1s = (in->n + 8191) / 8192;
    if (g1s > 2ull * c->n_cu) g1s = 2ull * c->n_cu;
    if (g1s == 0) g1s = 1;
    if (defer) {
      c->pend = k;
      c->pend_g1 = (unsigned)g1;
      c->pend_g1s = (unsigned)g1s;
      c->pend_g2 = c->d_k3_region ? c->k3_g2 : 0u;
      c->pend_ids = ids_stream;
      c->count_pending = true;
      return TCBEE_OK;
    }
    hipStream_t ks = s;
    if (async) {  // K3 on the ids stream, after K2
      TRY_HIP(hipEventRecord(c->ev_k2, s));
      TRY_HIP(hipStreamWaitEvent(ids_stream, c->ev_k2, 0));
      ks = ids_stream;
    }
    TRY_HIP(launch_count(k, (unsigned)g1, (unsigned)g1s, c->d_k3_region ? c->k3_g2 : 0u, ks));
    if (async) TRY_HIP(hipEventRecord(c->ev_k3, ks));
    c->k3_async = async;
    if (gen) {
      c->prepped = true;
      c->alt_clean = true;  // (emptied by this K3, stream-ordered before any later use)
      c->tiles_hw = 0;
    }
  } else {
    TRY_HIP(launch_finalize(c->d_batch, c->d_persist, out_cap, out_n_dev, ctr_dev, cfg->direction, s));
    if (defer) {  // keep the parse -> finish pairing of a deferred batch
      c->count_pending = true;
      c->pend_empty = true;
    }
  }
  return TCBEE_OK;
}

int tcbee_parse_finish_device(tcbee_ctx* c, const uint32_t* id_map_dev, uint64_t map_len,
                              void* stream) {
  if (!c || !c->count_pending || (map_len && !id_map_dev)) return TCBEE_EINVAL;
  if (c->pend_empty) {
    c->count_pending = c->pend_empty = false;
    return TCBEE_OK;
  }
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  CountArgs k = c->pend;
  if (id_map_dev && !c->d_omap) TRY_HIP(dalloc(&c->d_omap, c->max_flows));
  hipStream_t ks = s;
  if (c->pend_ids) {  // async: after everything queued on `s` (K2, the id map)
    TRY_HIP(hipEventRecord(c->ev_fin, s));
    TRY_HIP(hipStreamWaitEvent(c->pend_ids, c->ev_fin, 0));
    ks = c->pend_ids;
  }
  if (id_map_dev) {
    TRY_HIP(launch_compose(c->tab.cmap, id_map_dev, map_len, k.batch, c->d_omap, c->max_flows, ks));
    k.omap = c->d_omap;
  }
  c->count_pending = false;
  TRY_HIP(launch_count(k, c->pend_g1, c->pend_g1s, c->pend_g2, ks));
  if (c->pend_ids) TRY_HIP(hipEventRecord(c->ev_k3, ks));
  c->k3_async = c->pend_ids != nullptr;
  c->pend_ids = nullptr;
  return TCBEE_OK;
}

int tcbee_flow_first_frames_device(tcbee_ctx* c, uint64_t* out_first_frame_dev, uint64_t cap,
                                   uint64_t* n_dev, const uint32_t* rec_frame_dev,
                                   const uint64_t* frame_gidx_dev, uint64_t n_frames,
                                   uint64_t rec_frame_cap, void* stream) {
  if (!c || (cap && !out_first_frame_dev) || (n_frames && !frame_gidx_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  GlobalExportArgs g{};
  g.tab = c->tab;
  g.out = out_first_frame_dev;
  g.cap = cap;
  g.persist = c->d_persist;
  g.batch = c->d_batch;
  g.n_out = n_dev;
  g.rec_frame = rec_frame_dev;
  g.frame_gidx = frame_gidx_dev;
  g.n_frames = n_frames;
  g.out_cap = rec_frame_dev ? rec_frame_cap : ~0ull;
  TRY_HIP(launch_first_frames(g, s));
  return TCBEE_OK;
}

int tcbee_owner_bucket_device(tcbee_ctx* c, uint32_t world, uint64_t seg_cap, uint64_t map_cap,
                              tcbee_flow_entry* ent_dev, uint32_t* lid_dev, uint64_t* meta_dev,
                              void* stream) {
  if (!c || world == 0 || world > kMaxOwners || !seg_cap || !ent_dev || !lid_dev || !meta_dev)
    return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  TRY_HIP(hipMemsetAsync(meta_dev, 0, (world + 2ull) * sizeof(uint64_t), s));
  OwnerArgs a{};
  a.tab = c->tab;
  a.persist = c->d_persist;
  a.world = world;
  a.seg_cap = seg_cap;
  a.map_cap = map_cap;
  a.ent = reinterpret_cast<uint64_t*>(ent_dev);
  a.lid = lid_dev;
  a.meta = meta_dev;
  a.status = &c->d_persist->status;
  TRY_HIP(launch_owner_bucket(a, s));
  return TCBEE_OK;
}

int tcbee_status_raise_device(tcbee_ctx* c, const uint64_t* v_dev, uint64_t n, uint64_t stride,
                              void* stream) {
  if (!c || (n && !v_dev) || (n > 1 && !stride)) return TCBEE_EINVAL;
  if (!n) return TCBEE_OK;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  TRY_HIP(launch_status_raise(v_dev, n, stride, &c->d_persist->status, s));
  return TCBEE_OK;
}

int tcbee_flow_first_seen_device(tcbee_ctx* c, uint64_t* out_dev, uint64_t cap, uint64_t* n_dev,
                                 void* stream) {
  if (!c || (cap && !out_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  TRY_HIP(launch_first_seen(c->tab, c->d_persist, out_dev, cap, n_dev, s));
  return TCBEE_OK;
}

int tcbee_owner_return_device(const uint32_t* ids_dev, const uint64_t* seg_meta_dev,
                              uint32_t world, uint64_t seg_cap, const uint32_t* gmap_dev,
                              uint64_t gmap_len, uint32_t* ret_dev, void* stream) {
  if (!ids_dev || !seg_meta_dev || world == 0 || !seg_cap || !ret_dev || (gmap_len && !gmap_dev))
    return TCBEE_EINVAL;
  TRY_HIP(launch_owner_return(ids_dev, seg_meta_dev, world, seg_cap, gmap_dev, gmap_len, ret_dev,
                              (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_owner_apply_device(const uint32_t* back_dev, const uint32_t* lid_dev,
                             const uint64_t* meta_dev, uint32_t world, uint64_t seg_cap,
                             uint32_t* map_dev, uint64_t map_cap, void* stream) {
  if (!back_dev || !lid_dev || !meta_dev || world == 0 || !seg_cap || (map_cap && !map_dev))
    return TCBEE_EINVAL;
  TRY_HIP(launch_owner_apply(back_dev, lid_dev, meta_dev, world, seg_cap, map_dev, map_cap,
                             (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_global_ids_device(const uint64_t* all_first_frame_dev, const uint64_t* all_n_dev,
                            uint64_t n_stride, uint32_t world, uint32_t rank, uint64_t stride,
                            uint32_t* out_map_dev, uint64_t map_cap,
                            const uint64_t* gbase_in_dev, uint64_t* gbase_out_dev, void* stream) {
  if (n_stride == 0) n_stride = 2;
  if (!all_first_frame_dev || !all_n_dev || world == 0 || rank >= world || n_stride < 2 ||
      (map_cap && !out_map_dev) || (gbase_in_dev && gbase_in_dev == gbase_out_dev))
    return TCBEE_EINVAL;
  if (!stride) return TCBEE_OK;
  TRY_HIP(launch_global_ids(all_first_frame_dev, all_n_dev, n_stride, world, rank, stride,
                            out_map_dev, map_cap, gbase_in_dev, gbase_out_dev,
                            (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_parse_batch_device(tcbee_ctx* c, const tcbee_frames* in, const tcbee_cfg* cfg,
                             uint8_t* out_rec74, uint64_t out_cap, uint32_t* out_flow_hash,
                             uint32_t* out_flow_id, uint64_t* out_n_dev, tcbee_counters* ctr_dev,
                             void* stream) {
  return tcbee_parse_batch_device_ex(c, in, cfg, out_rec74, out_cap, out_flow_hash, out_flow_id,
                                     out_n_dev, ctr_dev, nullptr, stream);
}

int tcbee_parse_batch(tcbee_ctx* c, const tcbee_frames* in, const tcbee_cfg* cfg,
                      uint8_t* out_rec74, uint64_t out_cap, uint32_t* out_flow_hash,
                      uint32_t* out_flow_id, uint64_t* out_n, tcbee_counters* ctr) {
  if (!c || !in || !cfg || !out_n) return TCBEE_EINVAL;
  if (in->n > c->max_frames) return TCBEE_ECAPACITY;
  if (in->arena_len > c->max_arena) return TCBEE_ECAPACITY;
  if (in->n && (!in->arena || !in->offset || !in->caplen || !in->ts_ns)) return TCBEE_EINVAL;
  if (out_cap && !out_rec74) return TCBEE_EINVAL;
  int rc = ensure_host_path(c);
  if (rc) return rc;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s = c->stream;
  const uint64_t n = in->n;
  if (n) {
    TRY_HIP(hipMemcpyAsync(c->d_arena, in->arena, in->arena_len, hipMemcpyHostToDevice, s));
    TRY_HIP(hipMemcpyAsync(c->d_off, in->offset, n * 8, hipMemcpyHostToDevice, s));
    TRY_HIP(hipMemcpyAsync(c->d_len, in->caplen, n * 4, hipMemcpyHostToDevice, s));
    TRY_HIP(hipMemcpyAsync(c->d_ts, in->ts_ns, n * 8, hipMemcpyHostToDevice, s));
  }
  TRY_HIP(hipMemsetAsync(c->d_ctr, 0, sizeof(tcbee_counters), s));
  tcbee_frames din{c->d_arena, in->arena_len, c->d_off, c->d_len, c->d_ts, n};
  const uint64_t cap = out_cap < n ? out_cap : n;
  rc = tcbee_parse_batch_device(c, &din, cfg, c->d_rec, cap, out_flow_hash ? c->d_hash : nullptr,
                                out_flow_id ? c->d_id : nullptr, c->d_n, c->d_ctr, s);
  if (rc) return rc;
  uint64_t nout = 0;
  tcbee_counters hc{};
  TRY_HIP(hipMemcpyAsync(&nout, c->d_n, 8, hipMemcpyDeviceToHost, s));
  TRY_HIP(hipMemcpyAsync(&hc, c->d_ctr, sizeof(hc), hipMemcpyDeviceToHost, s));
  TRY_HIP(hipStreamSynchronize(s));
  if (nout) {
    TRY_HIP(hipMemcpyAsync(out_rec74, c->d_rec, nout * kRecBytes, hipMemcpyDeviceToHost, s));
    if (out_flow_hash)
      TRY_HIP(hipMemcpyAsync(out_flow_hash, c->d_hash, nout * 4, hipMemcpyDeviceToHost, s));
    if (out_flow_id)
      TRY_HIP(hipMemcpyAsync(out_flow_id, c->d_id, nout * 4, hipMemcpyDeviceToHost, s));
    TRY_HIP(hipStreamSynchronize(s));
  }
  *out_n = nout;
  if (ctr) {
    ctr->ingress += hc.ingress;
    ctr->egress += hc.egress;
    ctr->handled += hc.handled;
    ctr->dropped += hc.dropped;
  }
  return TCBEE_OK;
}

int tcbee_flow_count(tcbee_ctx* c, uint64_t* n) {
  if (!c || !n) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  TRY_HIP(k3_wait_host(c));
  if (int rc = apply_pending_reset(c, c->stream)) return rc;
  PersistState p{};
  TRY_HIP(hipMemcpyAsync(&p, c->d_persist, sizeof(p), hipMemcpyDeviceToHost, c->stream));
  TRY_HIP(hipStreamSynchronize(c->stream));
  *n = p.flow_count;
  return TCBEE_OK;
}

int tcbee_flow_export(tcbee_ctx* c, tcbee_flow_entry* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || (cap && !out)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  TRY_HIP(k3_wait_host(c));
  if (int rc = apply_pending_reset(c, c->stream)) return rc;
  PersistState p{};
  TRY_HIP(hipMemcpyAsync(&p, c->d_persist, sizeof(p), hipMemcpyDeviceToHost, c->stream));
  TRY_HIP(hipStreamSynchronize(c->stream));
  const uint64_t nf = p.flow_count;
  std::vector<uint64_t> ent, cnt, cfs;
  std::vector<uint32_t> cmap;
  try {
    ent.resize(8 * nf + 1);
    cfs.resize(nf + 1);
    cnt.resize(2 * nf + 2);
    cmap.resize(nf + 1);
  } catch (...) {
    return TCBEE_ENOMEM;
  }
  if (nf) {
    TRY_HIP(hipMemcpyAsync(ent.data(), c->tab.ent, 8 * nf * 8, hipMemcpyDeviceToHost, c->stream));
    TRY_HIP(hipMemcpyAsync(cnt.data(), c->tab.cnt, 2 * nf * 8, hipMemcpyDeviceToHost, c->stream));
    TRY_HIP(hipMemcpyAsync(cmap.data(), c->tab.cmap, nf * 4, hipMemcpyDeviceToHost, c->stream));
    TRY_HIP(hipMemcpyAsync(cfs.data(), c->tab.cfs, nf * 8, hipMemcpyDeviceToHost, c->stream));
    TRY_HIP(hipStreamSynchronize(c->stream));
  }
  for (uint64_t cl = 0; cl < nf; ++cl) {  // claims; ids are a permutation of [0, nf)
    const uint64_t* m = &ent[8 * cl];
    const uint64_t id = cmap[cl];
    if (id >= cap || id >= nf) continue;
    tcbee_flow_entry& e = out[id];
    std::memcpy(e.tuple, m, TCBEE_KEY_BYTES);
    e.pkts = cnt[2 * id];
    e.bytes = cnt[2 * id + 1];
    e.first_seen = cfs[cl];
  }
  *n = nf < cap ? nf : cap;
  return TCBEE_OK;
}

int tcbee_flow_export_device(tcbee_ctx* c, tcbee_flow_entry* out_dev, uint64_t cap,
                             uint64_t* n_dev, void* stream) {
  if (!c || (cap && !out_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  TRY_HIP(k3_wait_stream(c, s));  // counters are K3's
  if (int rc = apply_pending_reset(c, s)) return rc;
  TRY_HIP(launch_export(c->tab, reinterpret_cast<uint64_t*>(out_dev), cap, c->d_persist, n_dev, s));
  return TCBEE_OK;
}

int tcbee_flow_export_global_device(tcbee_ctx* c, tcbee_flow_entry* out_dev, uint64_t cap,
                                    uint64_t* n_dev, const uint32_t* rec_frame_dev,
                                    const uint64_t* frame_gidx_dev, uint64_t n_frames,
                                    uint64_t rec_frame_cap, void* stream) {
  if (!c || (cap && !out_dev) || (n_frames && !frame_gidx_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  GlobalExportArgs g{};
  g.tab = c->tab;
  g.out = reinterpret_cast<uint64_t*>(out_dev);
  g.cap = cap;
  g.persist = c->d_persist;
  g.batch = c->d_batch;
  g.n_out = n_dev;
  g.rec_frame = rec_frame_dev;
  g.frame_gidx = frame_gidx_dev;
  g.n_frames = n_frames;
  g.out_cap = rec_frame_dev ? rec_frame_cap : ~0ull;
  TRY_HIP(k3_wait_stream(c, s));  // counters are K3's
  TRY_HIP(launch_export_global(g, s));
  return TCBEE_OK;
}

int tcbee_flow_records_before_device(tcbee_ctx* c, const uint32_t* rec_frame_dev,
                                     const uint64_t* frame_gidx_dev, const uint64_t* n_rec_dev,
                                     uint64_t n_rec_max, uint64_t* out_counts_dev, uint64_t cap,
                                     void* stream) {
  if (!c || (cap && !out_counts_dev) || (n_rec_max && !frame_gidx_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  TRY_HIP(launch_records_before(c->tab, c->d_persist, rec_frame_dev, frame_gidx_dev, n_rec_dev,
                                n_rec_max, out_counts_dev, cap, s));
  return TCBEE_OK;
}

int tcbee_flow_set_first_seen_device(tcbee_ctx* c, const uint64_t* fs_by_id_dev, uint64_t cap,
                                     void* stream) {
  if (!c || (cap && !fs_by_id_dev)) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  if (int rc = apply_pending_reset(c, s)) return rc;
  TRY_HIP(launch_set_first_seen(c->tab, c->d_persist, fs_by_id_dev, cap, s));
  return TCBEE_OK;
}

int tcbee_flow_merge_device(tcbee_ctx* c, const tcbee_flow_entry* ent_dev, uint64_t nseg,
                            uint64_t stride, const uint64_t* seg_meta_dev,
                            uint64_t max_total_records, uint32_t* out_ids_dev, void* stream) {
  if (c) c->prepped = false;  // (rank kernels on the current slot; the next batch preps)
  if (!c || !seg_meta_dev || (nseg * stride && (!ent_dev || !out_ids_dev))) return TCBEE_EINVAL;
  // merged first_seen values are min-reduced in the slots' 31-bit fs32 words
  if (max_total_records >= (1ull << 31)) return TCBEE_ECAPACITY;
  const uint64_t total_records = max_total_records;
  TRY_HIP(hipSetDevice(c->device));
  hipStream_t s;
  TRY_HIP(ctx_stream(c, stream, s));
  const uint64_t words = (total_records + 31) / 32 + 1;
  if (!c->d_mcnt) TRY_HIP(dalloc(&c->d_mcnt, 2 * c->max_flows));
  if (words > c->m_words) {
    // merge scratch grows with the global record count (not on the hot path)
    TRY_HIP(hipStreamSynchronize(s));
    dfree(c->d_mbitmap);
    dfree(c->d_mwprefix);
    dfree(c->d_mbprefix);
    c->d_mbitmap = nullptr;
    c->d_mwprefix = nullptr;
    c->d_mbprefix = nullptr;
    c->m_words = 0;
    TRY_HIP(dalloc(&c->d_mbitmap, words));
    TRY_HIP(dalloc(&c->d_mwprefix, words));
    TRY_HIP(dalloc(&c->d_mbprefix, (words + kScanWordsPerBlock - 1) / kScanWordsPerBlock));
    // all zero between merges from here on (each merge clears the words it set); the
    // fill completes before this call returns, so a later merge on any
    // stream finds it done
    TRY_HIP(hipMemsetAsync(c->d_mbitmap, 0, words * sizeof(uint32_t), c->stream));
    TRY_HIP(hipStreamSynchronize(c->stream));
    c->m_words = words;
  }
  // fresh table: the merge result replaces whatever this context held
  c->reset_pending = false;
  TRY_HIP(launch_table_init(c->tab, s));
  TRY_HIP(hipMemsetAsync(c->d_persist, 0, sizeof(PersistState), s));
  TRY_HIP(hipMemsetAsync(c->d_batch, 0, sizeof(BatchState), s));
  TRY_HIP(hipMemsetAsync(c->d_mcnt, 0, 2 * c->max_flows * sizeof(uint64_t), s));
  MergeArgs g{};
  g.ent = reinterpret_cast<const uint64_t*>(ent_dev);
  g.nseg = nseg;
  g.stride = stride;
  g.seg_meta = seg_meta_dev;
  g.tab = c->tab;
  g.batch = c->d_batch;
  g.persist = c->d_persist;
  g.new_list = c->d_new_list;
  g.mcnt = c->d_mcnt;
  g.out_slot = out_ids_dev;
  g.bitmap = c->d_mbitmap;
  RankArgs r{};
  r.new_list = c->d_new_list;
  r.new_fs = c->d_new_fs;
  r.batch = c->d_batch;
  r.persist = c->d_persist;
  r.tab = c->tab;
  r.bitmap = c->d_mbitmap;
  r.wprefix = c->d_mwprefix;
  r.bprefix = c->d_mbprefix;
  r.nwords = words;
  r.nblocks = (words + kScanWordsPerBlock - 1) / kScanWordsPerBlock;
  TRY_HIP(launch_merge(g, r, s));
  return TCBEE_OK;
}

int tcbee_remap_ids_device(uint32_t* ids_dev, uint64_t n_max, const uint64_t* n_dev,
                           const uint32_t* map_dev, uint64_t map_len, void* stream) {
  if (n_max && (!ids_dev || !map_dev)) return TCBEE_EINVAL;
  if (!n_max) return TCBEE_OK;
  TRY_HIP(launch_remap(ids_dev, n_max, n_dev, map_dev, map_len, (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_ctx_status(tcbee_ctx* c) {
  if (!c) return TCBEE_EINVAL;
  if (hipSetDevice(c->device) != hipSuccess) return TCBEE_EDEVICE;
  if (k3_wait_host(c) != hipSuccess) return TCBEE_EDEVICE;
  PersistState p{};
  if (hipMemcpyAsync(&p, c->d_persist, sizeof(p), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return TCBEE_EDEVICE;
  const uint32_t zero = 0;
  if (hipMemcpyAsync(&c->d_persist->status, &zero, 4, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return TCBEE_EDEVICE;
  if (p.status & kStSpin) return TCBEE_ESPIN;
  if (p.status & kStFlowFull) return TCBEE_EFLOWFULL;
  if (p.status & kStShard) return TCBEE_ESHARD;
  return TCBEE_OK;
}

int tcbee_ctx_count_mode(tcbee_ctx* c, int* mode) {
  if (!c || !mode) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  TRY_HIP(k3_wait_host(c));
  PersistState p{};
  TRY_HIP(hipMemcpyAsync(&p, c->d_persist, sizeof(p), hipMemcpyDeviceToHost, c->stream));
  TRY_HIP(hipStreamSynchronize(c->stream));
  *mode = (int)p.k3_mode - 1;
  return TCBEE_OK;
}

int tcbee_ctx_profile(tcbee_ctx* c, int enable) {
  if (!c) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  if (enable && c->ev.empty()) {
    c->ev.resize(2 * kMaxProfiled, nullptr);
    // timing-only events: no system-scope fence (its L2 writeback + invalidate is
    // measurement overhead between the kernels it brackets; elapsed times are read
    // after a stream synchronize)
    for (auto& e : c->ev) TRY_HIP(hipEventCreateWithFlags(&e, TCBEE_PROF_EVFLAGS));
  }
  c->profiling = enable != 0;
  c->ev_used = 0;
  return TCBEE_OK;
}

int tcbee_ctx_profile_read(tcbee_ctx* c, double* ms_total, uint64_t* launches) {
  if (!c || !ms_total || !launches) return TCBEE_EINVAL;
  TRY_HIP(hipSetDevice(c->device));
  double tot = 0.0;
  for (uint64_t k = 0; k < c->ev_used; ++k) {
    TRY_HIP(hipEventSynchronize(c->ev[2 * k + 1]));
    float ms = 0.f;
    TRY_HIP(hipEventElapsedTime(&ms, c->ev[2 * k], c->ev[2 * k + 1]));
    tot += ms;
  }
  *ms_total = tot;
  *launches = c->ev_used;
  return TCBEE_OK;
}

int tcbee_gen_frames_device(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                            uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed,
                            void* stream) {
  if ((n && (!arena || !off || !len)) || (kind != 0 && kind != 1 && kind != 3))
    return TCBEE_EINVAL;
  if (kind != 0 && n_flows == 0) return TCBEE_EINVAL;
  if (!n) return TCBEE_OK;
  TRY_HIP(launch_gen(arena, off, len, n, first_index, kind, n_flows, seed, (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_gen_frames_index_device(uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                  const uint64_t* gidx, uint64_t n, int kind, uint64_t n_flows,
                                  uint64_t seed, void* stream) {
  if ((n && (!arena || !off || !len || !gidx)) || (kind != 0 && kind != 1)) return TCBEE_EINVAL;
  if (kind == 1 && n_flows == 0) return TCBEE_EINVAL;
  if (!n) return TCBEE_OK;
  TRY_HIP(launch_gen(arena, off, len, n, 0, kind, n_flows, seed, (hipStream_t)stream, gidx));
  return TCBEE_OK;
}

int tcbee_gen_frames_zipf_device(uint8_t* arena, const uint64_t* off, const uint32_t* len,
                                 uint64_t n, uint64_t first_index, uint64_t n_flows,
                                 uint64_t seed, const uint64_t* zcdf, void* stream) {
  if ((n && (!arena || !off || !len)) || n_flows == 0 || !zcdf) return TCBEE_EINVAL;
  if (!n) return TCBEE_OK;
  TRY_HIP(launch_gen(arena, off, len, n, first_index, kGenZipf, n_flows, seed,
                     (hipStream_t)stream, nullptr, zcdf));
  return TCBEE_OK;
}

int tcbee_gen_frames_zipf_host(uint8_t* arena, const uint64_t* off, const uint32_t* len,
                               uint64_t n, uint64_t first_index, uint64_t n_flows, uint64_t seed,
                               const uint64_t* zcdf) {
  if ((n && (!arena || !off || !len)) || n_flows == 0 || !zcdf) return TCBEE_EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t h[54];
    gen_header(h, first_index + i, len[i], kGenZipf, n_flows, seed, zcdf);
    std::memcpy(arena + off[i], h, len[i] < 54u ? len[i] : 54u);
  }
  return TCBEE_OK;
}

uint64_t tcbee_gen_shard_scratch(uint64_t n_global) {
  const uint64_t c = (n_global + kShardChunk - 1) / kShardChunk;
  return c ? c : 1;
}

int tcbee_gen_shard_index_device(uint64_t n_global, int world, int rank, int kind,
                                 uint64_t n_flows, uint64_t seed, int imix, uint64_t* out_gidx,
                                 uint32_t* out_caplen, uint64_t cap, uint64_t* scratch,
                                 uint64_t* n_out, void* stream) {
  return tcbee_gen_shard_index_rss_device(n_global, world, rank, kind, n_flows, seed, imix,
                                          nullptr, 0, out_gidx, out_caplen, cap, scratch,
                                          n_out, stream);
}

int tcbee_gen_rss_load_device(uint64_t n_frames, int kind, uint64_t n_flows, uint64_t seed,
                              uint32_t rss_len, uint64_t* counts_dev, void* stream) {
  return tcbee_gen_rss_load_range_device(0, n_frames, kind, n_flows, seed, rss_len, counts_dev,
                                         stream);
}

int tcbee_gen_rss_load_range_device(uint64_t first_frame, uint64_t n_frames, int kind,
                                    uint64_t n_flows, uint64_t seed, uint32_t rss_len,
                                    uint64_t* counts_dev, void* stream) {
  if ((kind != 0 && kind != 1) || (kind == 1 && n_flows == 0) || rss_len == 0 ||
      rss_len > kRssMaxLen || !counts_dev)
    return TCBEE_EINVAL;
  ShardArgs a{};
  a.n_global = n_frames;
  a.first = first_frame;
  a.world = 1;
  a.kind = kind;
  a.n_flows = n_flows;
  a.seed = seed;
  a.scratch = counts_dev;
  a.rss_len = rss_len;
  TRY_HIP(launch_rss_load(a, (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_gen_shard_index_rss_device(uint64_t n_global, int world, int rank, int kind,
                                     uint64_t n_flows, uint64_t seed, int imix,
                                     const uint16_t* rss_dev, uint32_t rss_len,
                                     uint64_t* out_gidx, uint32_t* out_caplen, uint64_t cap,
                                     uint64_t* scratch, uint64_t* n_out, void* stream) {
  if (world < 1 || rank < 0 || rank >= world || (kind != 0 && kind != 1) || !scratch || !n_out ||
      (cap && (!out_gidx || !out_caplen)))
    return TCBEE_EINVAL;
  if (rss_dev && (rss_len == 0 || rss_len > kRssMaxLen)) return TCBEE_EINVAL;
  if (kind == 1 && n_flows == 0) return TCBEE_EINVAL;
  if ((n_global + kShardChunk - 1) / kShardChunk > 0x7FFFFFFFull) return TCBEE_ECAPACITY;
  ShardArgs a{};
  a.n_global = n_global;
  a.world = (uint32_t)world;
  a.rank = (uint32_t)rank;
  a.kind = kind;
  a.imix = imix;
  a.n_flows = n_flows;
  a.seed = seed;
  a.gidx = out_gidx;
  a.caplen = out_caplen;
  a.cap = cap;
  a.scratch = scratch;
  a.n_out = n_out;
  a.rss = rss_dev;
  a.rss_len = rss_dev ? rss_len : 0;
  TRY_HIP(launch_shard_index(a, (hipStream_t)stream));
  return TCBEE_OK;
}

int tcbee_gen_frames_host(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                          uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed) {
  if ((n && (!arena || !off || !len)) || (kind != 0 && kind != 1 && kind != 3))
    return TCBEE_EINVAL;
  if (kind != 0 && n_flows == 0) return TCBEE_EINVAL;
  const uint32_t hl = gen_header_len(kind);
  for (uint64_t i = 0; i < n; ++i) {
    uint8_t h[kGenHdrMax];
    gen_header(h, first_index + i, len[i], kind, n_flows, seed);
    std::memcpy(arena + off[i], h, len[i] < hl ? len[i] : hl);
  }
  return TCBEE_OK;
}

uint64_t tcbee_flow_hash64(const uint8_t key[TCBEE_KEY_BYTES]) {
  uint64_t k[5];
  std::memcpy(k, key, 40);
  return flow_hash64(k[0], k[1], k[2], k[3], k[4]);
}

}  // extern "C"

#if TCBEE_VARIANTS
// ---- test entry points of the variants build (not in include/tcbee_amd.h) ----
// The race test of DESIGN.md section 6 (round 6): host-released waits
// that pin an interleaving of the legacy default stream and a context's stream.
extern "C" {
// A page-locked, coherent host word (0), readable by kernels; the test stores to it.
int tcbee_test_flag_create(uint64_t** host_flag) {
  if (!host_flag) return TCBEE_EINVAL;
  TRY_HIP(hipHostMalloc(reinterpret_cast<void**>(host_flag), 64,
                        hipHostMallocMapped | hipHostMallocCoherent));
  **host_flag = 0;
  return TCBEE_OK;
}
int tcbee_test_flag_destroy(uint64_t* host_flag) {
  if (host_flag) TRY_HIP(hipHostFree(host_flag));
  return TCBEE_OK;
}
// Queue a wait on `stream` (NULL: HIP's legacy default stream) until *host_flag ==
// expect; wall-clock bounded (timeout_us). *state_dev = 3 released, 1 timed out.
int tcbee_test_wait_host_device(uint64_t* host_flag, uint64_t expect, uint64_t timeout_us,
                                uint64_t* state_dev, void* stream) {
  if (!host_flag || !state_dev) return TCBEE_EINVAL;
  void* dflag = nullptr;
  TRY_HIP(hipHostGetDevicePointer(&dflag, host_flag, 0));
  TRY_HIP(launch_test_wait_host(static_cast<const uint64_t*>(dflag), expect, timeout_us,
                                state_dev, (hipStream_t)stream));
  return TCBEE_OK;
}
// *registered = 1 when the host byte p lies in a page-locked range (the query
// tcbee_pipe_register_output makes: hipPointerGetAttributes type == host).
int tcbee_test_host_registered(const void* p, int* registered) {
  if (!p || !registered) return TCBEE_EINVAL;
  hipPointerAttribute_t at{};
  *registered = hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  return TCBEE_OK;
}
// Every later batch of `c` that ranks with the four-kernel K2 holds its stream between
// k_mark and k_scan_words until *host_flag == 1 (NULL: off).
int tcbee_test_k2_hold(tcbee_ctx* c, uint64_t* host_flag, uint64_t* state_dev) {
  if (!c || (host_flag && !state_dev)) return TCBEE_EINVAL;
  void* dflag = nullptr;
  if (host_flag) TRY_HIP(hipHostGetDevicePointer(&dflag, host_flag, 0));
  c->test_hold = static_cast<const uint64_t*>(dflag);
  c->test_hold_state = state_dev;
  return TCBEE_OK;
}
}  // extern "C"
#endif

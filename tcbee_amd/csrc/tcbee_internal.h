// tcbee_internal.h — device-side state shared by the kernels and the C ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tcbee_amd.h"

namespace tcbee {

// Status bits (sticky, in PersistState::status)
//   kStShard: a global-order export (tcbee_flow_export_global_device) found a flow
//   whose first record it cannot place (outside the last batch, past out_cap, or
//   rejected frames without a record -> frame map)
constexpr uint32_t kStFlowFull = 1u, kStSpin = 2u, kStShard = 4u;

// Flow table in HBM (round 3): compact slot lines probed by K1, plus dense
// per-claim entries. A flow's claim index is its insertion order over the
// context's life (fixed at insert; cmap[claim] = its dense first-seen id), so
// claims are dense in [0, flows) and bounded by max_claims (= max_flows).
//  slots: nlines units of 64 B (u64[8]; half a 128-B cache line); open addressing,
//    linear probing over slot s = unit * 3 + pos, for IPv4-form keys (12 zero bytes
//    + the address, xdp.rs:116-119):
//    words 2*pos, 2*pos + 1 (pos < 3): w0, w1 of slot pos
//      w1 = kind << 56 | claim << 32 | lo32 (w1 == 0: empty; kind 1: busy)
//      kind 2: w0 = saddr | daddr << 32 (wire bytes), lo32 = sport | dport << 16 —
//              the slot holds the whole key, so the slot alone decides a match
//      kind 4: dead (refused because the table was full): the key's w0 and lo32, no
//              claim — the flow's later frames find it and stay unclassified
//    bytes 48 + 4*pos: fs32 of slot pos: the batch-local first record index of a
//      flow new in this batch (kFs32Flag | frame while only its claimer's mark is
//      known); stale for flows of earlier batches (never read for them). A slot
//      and its fs32 share the 64-B unit: the two 64-B halves of a line can be of
//      different ages in L1/L2 (fs32 in the other half lost first_seen values)
//    One probe = one 64-B unit (16-B slot + its fs32). kSlotsPerFlow slots per
//    max_flow (load <= 1/8): ~171 B of slot units per max_flow, 176 MB at 1M flows
//    (rounds 1-2: 64-B slots, 2-16 per max_flow, 512 MiB at bench's 1M flows).
//    Measured (round 3, 125M IMIX frames, K1): load 1/2 costs 27 % at 10k flows and
//    29 % at 1M (the linear-probe walks are dependent round trips); at equal load
//    the compact slots match the 64-B slots (the cost of a large table is the
//    probe's latency, not its bytes: a 44 MB table at load 1/2 was slower than
//    176 MB at 1/8).
//  ent [claim*8 + 0..4] the 40-B key as 5 LE u64 words (5..7 spare)
//  cfs [claim]         first_seen (global accepted-record index, written by K2)
//  cnt [id*2 + 0/1]    pkts / bytes of dense flow id `id`
struct FlowTable {
  uint64_t* slots;
  uint64_t nlines;
  uint64_t* ent;
  uint64_t* cfs;         // [claim] first_seen (global accepted-record index), by K2
  // wide slots (64 B, rounds 1-2's layout) for keys that are not IPv4-form: the
  // 40-B key lives in the slot, so an IPv6 probe is one line and compares at once
  // (a compact kind-3 slot + its entry cost K1 15 % on an all-IPv6 trace: a
  // dependent load per frame). wide[s*8 + 0] tag word: 0 empty, 1 busy, else
  // hash_tag32 | claim << 32 (claim ~0: dead, the table was full); [1..5] key;
  // [6] low 32 bits: fs32 as the compact slots'
  uint64_t* wide;
  uint64_t wide_mask;    // wide slots - 1 (>= kSlotsPerFlow x max_flows, a power of 2)
  uint32_t* wide_used;   // != 0 once a wide slot was claimed: resets sweep the wide
                         // slots only then (an IPv4 capture never touches them)
  uint64_t* cnt;
  uint32_t* cmap;        // claim index -> dense id (0-based), written by K2; dense in
                         // [0, flows), so K3 stages it in LDS
  uint64_t max_claims;   // claims at or past it are refused (TCBEE_EFLOWFULL)
  uint64_t max_wide;     // claims of wide-slot (non-IPv4-form) keys past it are refused
                         // too (tcbee_ctx_create_ex; = max_claims by default)
};
constexpr uint32_t kSlotsPerLine = 3;  // compact slots per 64-B unit
constexpr uint32_t kWideSlot = 1u << 31;  // slot ids: compact s, or wide s | kWideSlot
constexpr uint64_t kSlotsPerFlow = 8;  // slots per max_flow: linear-probe load <= 1/8
constexpr uint32_t kFs32Flag = 1u << 31;

// Lives across batches of one context.
struct PersistState {
  uint64_t rec_base;    // accepted frames before this batch
  uint64_t flow_count;  // flows with ids
  uint32_t status;
  uint32_t k3_mode;     // diagnostic: K3 mode of the last batch + 1 (0: none yet)
  // rec_base / flow_count as they were before this batch's rank step: k_scan_blocks
  // (one block, before k_assign) stages them here and advances the two above, so
  // k_assign reads the old bases without any grid-wide completion count
  uint64_t rank_base;
  uint64_t rank_fbase;
  uint64_t wide_claims;  // wide-slot keys claimed (bounded by FlowTable::max_wide)
};

// Zeroed before every batch (k_prep).
struct BatchState {
  uint64_t n_acc;       // accepted frames in this batch (last tile writes it)
  uint64_t n_new;       // flows first claimed in this batch
  uint64_t flow_total;  // flows with ids after this batch (rank step writes it)
  uint64_t fs_max_word; // highest first-seen bitmap word set this batch (bounds the
                        // rank scan; the words up to it are cleared again by K3)
  uint64_t k3_done;     // (fused rank) K3 blocks finished: the last one advances the bases
};
static_assert(sizeof(BatchState) == 40, "memset size");

struct PrepArgs {
  BatchState* batch;
  uint64_t* tile_status;
  uint64_t ntiles;
  bool reset;           // also empty the flow table (a pending tcbee_flow_reset_device)
  // zero the counters of every id not yet handed out (a fused-rank batch: K3's
  // blocks add big frames to new ids' counters before any block could zero them)
  bool zero_free_counters;
  FlowTable tab;
  PersistState* persist;
};
hipError_t launch_prep(const PrepArgs& p, hipStream_t s);

struct ParseArgs {
  const uint8_t* arena;
  uint64_t arena_len;
  const uint64_t* offset;
  const uint32_t* caplen;
  const uint64_t* ts;
  uint64_t n;
  uint8_t* out_rec;
  uint64_t out_cap;
  uint32_t* out_hash;
  uint32_t* acc_flow;     // per accepted frame: the flow's claim index (ctx scratch)
  uint32_t* acc_len;      // per accepted frame: caplen (ctx scratch)
  uint64_t* tile_status;  // decoupled look-back words, one per tile
  uint64_t ntiles;
  BatchState* batch;
  PersistState* persist;
  uint64_t* new_list;     // slots first claimed this batch
  FlowTable tab;
  uint16_t filter_port;
  uint32_t withhold_every;  // test hook (TCBEE_TEST_WITHHOLD): 0 in production
  uint32_t plain_walk;      // probe steps past foreign slots with plain loads (kPlainWalk)
  uint32_t pack_bits;       // != 0: acc_flow = claim | min(caplen, lmax) << pack_bits
  uint32_t* out_frame;      // optional: batch-local frame index of record p (p < out_cap)
};
constexpr uint32_t kPlainWalk = 8;

struct RankArgs {
  const uint64_t* new_list;
  BatchState* batch;
  PersistState* persist;
  FlowTable tab;
  uint32_t* bitmap;     // one bit per accepted frame of the batch
  uint32_t* wprefix;    // per bitmap word: exclusive popcount prefix in its block
  uint32_t* bprefix;    // per scan block: exclusive popcount prefix
  uint32_t* new_fs;     // [max_claims] k_mark's copy of each new flow's local first_seen
  uint64_t nwords;
  uint64_t nblocks;
  bool update_persist;  // parse (not merge): advance rec_base / flow_count when
                        // done and zero the new ids' counters, so the batch's K3
                        // may run on another stream beside the next batch's K1
#if TCBEE_VARIANTS
  // test hook (tcbee_test_k2_hold): hold the stream between k_mark and k_scan_words
  // until a host-written flag reads 1 (the race test of DESIGN.md section 6)
  const uint64_t* test_hold = nullptr;
  uint64_t* test_hold_state = nullptr;
#endif
};

// Launchers (tcbee_kernels.hip). All asynchronous on `s`.
hipError_t launch_table_init(FlowTable t, hipStream_t s);
hipError_t launch_parse(const ParseArgs& a, int fpl, bool flows, hipStream_t s);
hipError_t launch_rank(const RankArgs& r, hipStream_t s);
#if TCBEE_VARIANTS
// test hook: one lane holds `s` until *flag_dev == expect (a page-locked coherent host
// word, system-scope loads) or timeout_us pass; *state = 3 released, 1 timed out
hipError_t launch_test_wait_host(const uint64_t* flag_dev, uint64_t expect, uint64_t timeout_us,
                                 uint64_t* state, hipStream_t s);
#endif
struct CountArgs {
  uint64_t* out_n;           // finalize (block 0): record count, counters, running bases
  tcbee_counters* ctr;
  int direction;
  PersistState* persist_rw;
  const uint32_t* acc_flow;
  uint32_t pack_bits;        // as ParseArgs::pack_bits
  const uint32_t* acc_len;
  uint32_t* out_id;
  uint64_t out_cap;
  const BatchState* batch;
  const PersistState* persist;
  const uint32_t* cmap;      // claim index -> local dense id (counters)
  const uint32_t* omap;      // claim index -> output id written to out_id (cmap, or
                             // cmap composed with a local -> global id map)
  uint32_t* bitmap;          // first-seen bitmap: words [0, fs_max_word] cleared here
  uint64_t* cnt;
  uint64_t* part;            // mode 0: [g1][kCountBins] per-block packed bins;
                             // mode 3: [groups][F] per-group packed bins by claim
  uint32_t g1;               // k_count's grid (mode 3 eligibility: count_mode)
  uint32_t range_ok;         // mode 3 allowed (0: test hook / small table)
  uint64_t part_words;       // capacity of part (u64)
  // mode 1 (large tables; region == nullptr disables it)
  uint32_t* region;          // per accepted frame: claim within its bucket | caplen
                             // << kBucketBits (0 when >= kRegLenEsc: added by a global
                             // atomic instead), bucket-sorted per block
  uint32_t* offs;            // [g1s][nb_max + 1] bucket offsets inside each block's region
  uint32_t nb_max;           // buckets the context's table can need
  uint64_t* lpart;           // [S][nb * kBucket][2] partial pkts/bytes per claim
  // mode 1, chunked (k_count_chunk2; nb < kChunkMaxNb): the region is written chunk
  // by chunk of kChunk records, bucket-sorted inside each chunk; coffs[q][0..nb] =
  // bucket offsets inside chunk q (row stride kChunkMaxNb + 1). nullptr: not used
  uint32_t* coffs;
  uint32_t chunk_off;        // 1: the two-pass scatter instead (test hook,
                             // TCBEE_TEST_K3_TWOPASS)
  // Fused rank (contexts of <= kFuseRankMax flows, batches K2 would rank in one
  // block): no rank launch — every k_count block ranks the batch's new flows itself
  // (mode 0 is certain), block 0 publishes cmap / cfs / flow_total and zeroes the new
  // ids' counters, and k_count_reduce advances the context's bases
  uint32_t fused_rank;
  // k_count: 16 records per lane and iteration instead of 8 (batches of at least
  // kK3WideFrames frames: twice the loads in flight; config 3, 100M records: K3
  // -19..-34 us per step; 1M-record batches are slower with it)
  uint32_t wide_iter;
  const uint64_t* new_list;  // (fused rank) slots first claimed this batch
  BatchState* batch_rw;      // (fused rank) the batch state K2 would have written
  FlowTable tab;             // (fused rank) slot fs32 words, cfs, cmap
  // (fused rank, small contexts: the next batch needs no k_prep launch) K3 also
  // leaves what k_prep would have prepared: tile status words [0, clean_ntiles)
  // zero, the next batch's state slot zero, and — after a reset switched the
  // context to its other table generation — the now-inactive generation empty
  uint64_t* clean_tiles;
  uint64_t clean_ntiles;
  BatchState* next_batch;
  uint32_t clean_alt;
  FlowTable alt;             // the inactive generation: slot units, wide slots, counters
  PersistState* alt_persist;
};
constexpr uint64_t kFuseRankMax = 256;
constexpr uint64_t kK3WideFrames = 16ull << 20;
// g1 = k_count blocks; g1s = k_count_scatter blocks; g2 = k_count_bucket blocks
// (g2 = 0: mode 1 impossible, neither is launched)
hipError_t launch_count(const CountArgs& c, unsigned g1, unsigned g1s, unsigned g2, hipStream_t s);

struct MergeArgs {
  const uint64_t* ent;        // nseg * stride entries, tcbee_flow_entry as u64[8]
  uint64_t nseg, stride;
  const uint64_t* seg_meta;   // per segment {valid entries, records}
  FlowTable tab;
  BatchState* batch;
  PersistState* persist;
  uint64_t* new_list;
  uint64_t* mcnt;             // per-claim pkts/bytes (2 * max_claims), zeroed
  uint32_t* out_slot;         // per entry: claim, then merged id
  uint32_t* bitmap;           // merge first-seen bitmap (cleared after use)
};
hipError_t launch_export(FlowTable t, uint64_t* out, uint64_t cap, const PersistState* p,
                         uint64_t* n_out, hipStream_t s);
// Global-order export of a table built by ONE batch (flow-hash shards): entry
// first_seen = frame_gidx[rec_frame[local record]] (rec_frame NULL: record k is
// frame k, checked against n_frames); n_out[1] = 0 (nothing to rebase).
struct GlobalExportArgs {
  FlowTable tab;
  uint64_t* out;
  uint64_t cap;
  PersistState* persist;
  const BatchState* batch;
  uint64_t* n_out;
  const uint32_t* rec_frame;
  const uint64_t* frame_gidx;
  uint64_t n_frames;
  uint64_t out_cap;  // records of the batch that have a rec_frame entry
};
hipError_t launch_export_global(const GlobalExportArgs& g, hipStream_t s);
// Merged table (first_seen = global frame index): out[id] = number of this
// rank's records whose global frame index is below the flow's first_seen.
hipError_t launch_records_before(FlowTable t, const PersistState* p, const uint32_t* rec_frame,
                                 const uint64_t* frame_gidx, const uint64_t* n_rec,
                                 uint64_t n_rec_max, uint64_t* out, uint64_t cap, hipStream_t s);
// first_seen of flow id := fs_by_id[id] (ids < cap)
hipError_t launch_set_first_seen(FlowTable t, const PersistState* p, const uint64_t* fs_by_id,
                                 uint64_t cap, hipStream_t s);
// Flow-hash exchange: first frame per local id (GlobalExportArgs.out = u64[cap]);
// global ids from the all-gathered first-frame arrays; output-id composition.
hipError_t launch_first_frames(const GlobalExportArgs& g, hipStream_t s);

// Owner exchange for contiguous shards (SURVEY.md §8(e) option 2).
constexpr uint32_t kMaxOwners = 64;
constexpr int kOwnerItems = 4;  // slots per thread of k_owner_bucket
struct OwnerArgs {
  FlowTable tab;
  const PersistState* persist;
  uint32_t world;
  uint64_t seg_cap;
  uint64_t* ent;        // [world][seg_cap] tcbee_flow_entry (u64[8])
  uint32_t* lid;        // [world][seg_cap] local id of each entry
  uint64_t* meta;       // [world + 2]: entries per owner (zeroed first; may pass
                        // seg_cap: the rest are dropped, TCBEE_ESHARD), records,
                        // entries dropped (seg_cap or map_cap)
  uint64_t map_cap;     // local ids past it have no place in the id map: ESHARD
  uint32_t* status;     // persist->status of the context (ESHARD on overflow)
};
hipError_t launch_owner_bucket(const OwnerArgs& a, hipStream_t s);
// *status |= kStShard if any v[i * stride] != 0, i < n (one block)
hipError_t launch_status_raise(const uint64_t* v, uint64_t n, uint64_t stride, uint32_t* status,
                               hipStream_t s);
// out[id] = first_seen of flow id (dense-id order: ascending), n_out = {flows, 0}
hipError_t launch_first_seen(FlowTable t, const PersistState* p, uint64_t* out, uint64_t cap,
                             uint64_t* n_out, hipStream_t s);
// ret[r*seg_cap + j] = gmap[ids[r*seg_cap + j]] for j < min(seg_meta[2r], seg_cap)
hipError_t launch_owner_return(const uint32_t* ids, const uint64_t* seg_meta, uint32_t world,
                               uint64_t seg_cap, const uint32_t* gmap, uint64_t gmap_len,
                               uint32_t* ret, hipStream_t s);
// map[lid[o*seg_cap + j]] = back[o*seg_cap + j] for j < min(meta[o], seg_cap)
hipError_t launch_owner_apply(const uint32_t* back, const uint32_t* lid, const uint64_t* meta,
                              uint32_t world, uint64_t seg_cap, uint32_t* map, uint64_t map_cap,
                              hipStream_t s);
hipError_t launch_global_ids(const uint64_t* allG, const uint64_t* alln, uint64_t nstride,
                             uint32_t world, uint32_t rank, uint64_t stride, uint32_t* gid,
                             uint64_t cap, const uint64_t* gbase_in, uint64_t* gbase_out,
                             hipStream_t s);
hipError_t launch_compose(const uint32_t* cmap, const uint32_t* id_map, uint64_t map_len,
                          const BatchState* b, uint32_t* omap, uint64_t max_flows, hipStream_t s);
hipError_t launch_merge(const MergeArgs& g, const RankArgs& r, hipStream_t s);
hipError_t launch_remap(uint32_t* ids, uint64_t n_max, const uint64_t* n_dev, const uint32_t* map,
                        uint64_t map_len, hipStream_t s);
hipError_t launch_finalize(BatchState* b, PersistState* p, uint64_t out_cap,
                           uint64_t* out_n, tcbee_counters* ctr, int direction,
                           hipStream_t s);
hipError_t launch_gen(uint8_t* arena, const uint64_t* off, const uint32_t* len, uint64_t n,
                      uint64_t first_index, int kind, uint64_t n_flows, uint64_t seed,
                      hipStream_t s, const uint64_t* gidx = nullptr,
                      const uint64_t* zcdf = nullptr);
struct ShardArgs {
  uint64_t n_global;
  uint32_t world, rank;
  int kind, imix;
  uint64_t n_flows, seed;
  uint64_t* gidx;
  uint32_t* caplen;
  uint64_t cap;
  uint64_t* scratch;  // per chunk: count, then exclusive prefix
  uint64_t* n_out;
  const uint16_t* rss;  // RSS indirection table: owner = rss[fold32 % rss_len] (NULL: % world)
  uint32_t rss_len;
  uint64_t first;       // k_rss_load: global frames [first, first + n_global)
};
constexpr uint32_t kRssMaxLen = 4096;  // RSS table entries (LDS histogram of k_rss_load)
constexpr int kShardPer = 16;  // global indices per thread
constexpr uint64_t kShardChunk = 256ull * kShardPer;  // one 256-thread block (kBlock)
hipError_t launch_shard_index(const ShardArgs& a, hipStream_t s);
// frames per RSS bucket (fold32(flow hash) % rss_len) of global frames
// [first, first + n_global), into a.scratch[0 .. rss_len)
hipError_t launch_rss_load(const ShardArgs& a, hipStream_t s);

constexpr int kBlock = 256;
// K1's block size and the product's frames per lane (build-time A/B knobs; a tile is
// kK1Block x FPL frames)
#ifndef TCBEE_K1_BS
#define TCBEE_K1_BS 256
#endif
#ifndef TCBEE_K1_FPL
#define TCBEE_K1_FPL 2
#endif
constexpr int kK1Block = TCBEE_K1_BS;
static_assert(kShardChunk == (uint64_t)kBlock * kShardPer, "shard chunk = one block");
constexpr int kScanWordsPerBlock = 2048;  // 256 threads x 8 words
constexpr uint64_t kRankSmallWords = 1024 * 32;  // single-block rank up to 1M frames
constexpr int kCountBlock = 1024;
constexpr int kCountBins = 12288;         // 96 KiB of u64 bins + 48 KiB claim->id map in LDS
// K3 mode 3: claims split into R ranges of <= kCountBins, R <= kMaxRanges; the
// R blocks of a group share one XCD (b % 8) and one record segment. Every record
// is visited R times, so it pays only for small R: vs mode 1 at 100M records
// (tools/k1_sweep.py, TCBEE_TEST_K3_NORANGE A/B) -0.36 ms at 20k flows (R 2),
// -0.08 at 30k (R 3), +0.12 at 45k (R 4), +0.42 at 60k, +2.8 at 125k (R 11)
constexpr uint32_t kMaxRanges = 3;
constexpr uint64_t kRangeFlows = (uint64_t)kCountBins * kMaxRanges;  // mode 3 up to 196608 flows
constexpr int kBinPkShift = 40;           // K3 bin: pkts in bits 63:40, bytes in 39:0
constexpr uint32_t kBigLen = 1u << 16;    // caplen >= 64 KiB: counted by device atomics
// a K3 block covers at most kK3MaxPer records (a multiple of the range granule),
// so a bin's pkts (< 2^24) and bytes (< 2^24 * kBigLen = 2^40) never overflow
constexpr uint64_t kK3Gran = 16384;
constexpr uint64_t kK3MaxPer = (1ull << 24) - kK3Gran;
constexpr int kBucketBits = 12, kBucket = 1 << kBucketBits;  // claims per mode-1 bucket
constexpr uint32_t kMaxBuckets = 4096;    // mode 1 up to 16M flows (hist + cursors: 32 KiB)
// mode 1 with kStagedMinNb..kSmallNb buckets (256k..2M flows): each chunk's
// entries are counting-sorted in LDS and stored as runs, not scattered lane by
// lane. At 100M records (TCBEE_K3ABL=90 A/B): 1M flows (245 buckets) -0.42 ms;
// 125k (31) +0.09 and 60k (15) +0.16 ms, where a wave's lanes already hit few
// bucket cursors and the per-chunk barriers cost more than they save
constexpr uint32_t kSmallNb = 512, kStagedMinNb = 64;
// k_count_chunk2's chunk: the records one 512-thread workgroup sorts by bucket in
// LDS at a time (24 per thread, 52 KiB: two workgroups per CU); the bucket pass sees
// chunk q as the segment [q * kChunk, (q+1) * kChunk). TCBEE_K3_CHUNK /
// TCBEE_K3_CHUNK_BLOCK: build-time A/B knobs (round 6: 16384 and 1024 x 24576 slower)
#ifndef TCBEE_K3_CHUNK
#define TCBEE_K3_CHUNK 12288
#endif
constexpr uint32_t kChunk = TCBEE_K3_CHUNK;
// flags of tcbee_ctx_profile's K1 timing events (A/B knob; 0 = hipEventDefault)
#ifndef TCBEE_PROF_EVFLAGS
#define TCBEE_PROF_EVFLAGS hipEventDisableSystemFence
#endif
#ifndef TCBEE_K3_CHUNK_BLOCK
#define TCBEE_K3_CHUNK_BLOCK 512
#endif
constexpr int kChunkBlock = TCBEE_K3_CHUNK_BLOCK;
// chunked mode up to kChunkMaxNb - 1 buckets: the scan of nb + 1 counts takes one
// per thread of the smaller (512-thread) workgroup
constexpr uint32_t kChunkMaxNb = 511;
constexpr uint64_t kMaxTableFlows = 1ull << 24;  // tcbee_ctx_create's max_flows limit
// mode-1 region entry: caplens from kRegLenEsc up are stored as 0 and their bytes
// added to the flow's counter by a global atomic (frames of >= 1 MiB: never on a
// real capture, but the ABI allows them)
constexpr uint32_t kRegLenEsc = (1u << (32 - kBucketBits)) - 1;

}  // namespace tcbee

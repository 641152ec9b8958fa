/*
 * tcbee_amd.h — C ABI of the MI355X-native TCBee packet-record path.
 *
 * What this replaces (all paths relative to the TCBee reference tree):
 *   - the per-packet kernel hooks  xdp_packet_tracer / tc_packet_tracer
 *       tcbee-record/tcbee-ebpf/src/main.rs:69-83
 *     which call xdp_hook / tc_hook
 *       tcbee-record/tcbee-ebpf/src/probes/xdp.rs:27-223
 *       tcbee-record/tcbee-ebpf/src/probes/tc.rs:28-183
 *   - the FLOWS flow set they insert into
 *       tcbee-record/tcbee-ebpf/src/flow_tracker.rs:12-23
 *   - the counters they bump (INGRESS/EGRESS_EVENTS, EVENTS_HANDLED/DROPPED)
 *       tcbee-record/tcbee-ebpf/src/counters.rs:5-83
 *   - the user-space serializer that turns each ring entry into the on-disk
 *     74-byte record (bincode fixint-LE 70 B + FF FF FF FF)
 *       tcbee-record/tcbee/src/handlers/mod.rs:94-146
 *
 * The kernel hook ABI is one call per packet; this ABI is one call per BATCH of
 * frames. Output is the 74-byte *file* layout (what tcbee-process reads,
 * tcbee-process/src/bindings/tcp_packet.rs:8-43), compacted, in input order.
 *
 * Conventions
 *   - Every function returns 0 (TCBEE_OK) or a negative TCBEE_E* code; nothing
 *     throws across the ABI.
 *   - All buffers are caller-owned; nothing is allocated inside a parse call.
 *   - One tcbee_ctx per host thread / HIP stream. Calls on different contexts
 *     are independent.
 *   - "_device" entry points take DEVICE pointers and a hipStream_t (as void*,
 *     NULL = the context's own stream, which then first waits for the work
 *     already queued on HIP's legacy default stream — e.g. a framework's default-
 *     stream copies of the inputs or zero-fills of the outputs) and are
 *     asynchronous unless stated. tcbee_ctx_create returns with the context's
 *     initialisation complete.
 *     Host-pointer entry points copy H2D / D2H through the context's buffers.
 */
#ifndef TCBEE_AMD_H
#define TCBEE_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TCBEE_ABI_VERSION 5  /* 5: tcbee_gen_rss_load_range_device, TCBEE_RSS_INVALID,
                                tcbee_ctx_create_ex, tcbee_pipe_register_output;
                              3: owner meta world+2 words, tcbee_status_raise_device;
                                4: RSS indirection tables for the shard generator */

/* ---- record / key layout constants (DESIGN.md "Data layout") ------------ */
#define TCBEE_RECORD_BYTES   74  /* tcp_packet.rs:42 ENTRY_SIZE            */
#define TCBEE_TRACE_BYTES    72  /* repr(C) tcp_packet_trace, tcp_header.rs:554-572 */
#define TCBEE_IPTUPLE_BYTES  38  /* repr(C) IpTuple, flow.rs:4-12          */
#define TCBEE_KEY_BYTES      40  /* IpTuple + 2 zero bytes (hash/table key) */
#define TCBEE_MAX_HDR_BYTES  74  /* eth 14 + ipv6 40 + tcp 20              */
#define TCBEE_REF_MAX_FLOWS 100  /* config.rs:19 MAX_FLOWS                  */
#define TCBEE_MAX_TABLE_FLOWS (1ull << 24) /* tcbee_ctx_create max_flows limit */

/* ---- error codes --------------------------------------------------------- */
#define TCBEE_OK                  0
#define TCBEE_EINVAL             -1  /* bad argument                          */
#define TCBEE_ENOMEM             -2  /* device / host allocation failed        */
#define TCBEE_EDEVICE            -3  /* HIP runtime error                      */
#define TCBEE_ECAPACITY          -4  /* batch larger than the context was made for */
#define TCBEE_EFLOWFULL          -5  /* flow table full (records still written) */
#define TCBEE_ENODEV             -6  /* no HIP device                           */
#define TCBEE_EIO                -7  /* file I/O error                          */
#define TCBEE_EFORMAT            -8  /* malformed input file                    */
#define TCBEE_ESPIN              -9  /* a bounded in-kernel wait timed out      */
#define TCBEE_EDB               -10  /* SQLite statement failed (sink)          */
#define TCBEE_ESHARD            -11  /* global-order export could not place a flow's
                                        first record (see tcbee_flow_export_global_device) */

/* ---- directions (which hook / which output file) ------------------------- */
#define TCBEE_DIR_INGRESS 0  /* xdp_hook  -> xdp.tcp, counts INGRESS_EVENTS */
#define TCBEE_DIR_EGRESS  1  /* tc_hook   -> tc.tcp,  counts EGRESS_EVENTS  */

/* ---- cfg flags ------------------------------------------------------------ */
#define TCBEE_F_NO_FLOWS     0x1u /* skip flow classification (hash/id/table) */

typedef struct tcbee_ctx tcbee_ctx;

/* Load-time configuration of the hook.
 * filter_port: the FILTER_PORT global (tcbee-ebpf/src/main.rs:30-31), set by
 *   EbpfLoader::set_global (tcbee/src/eBPF/ebpf_runner.rs:79-84). Host order;
 *   0 = no filter; otherwise a frame is kept only if sport or dport equals it
 *   (xdp.rs:89-92, tc.rs:72-77). */
typedef struct tcbee_cfg {
    uint16_t filter_port;
    uint8_t  direction;      /* TCBEE_DIR_*                               */
    uint8_t  reserved0;
    uint32_t flags;          /* TCBEE_F_*                                 */
} tcbee_cfg;

/* A batch of raw Ethernet frames ("the packet as XDP/TC sees it").
 * Frame i occupies arena[offset[i] .. offset[i] + caplen[i]).
 * ts_ns[i] replaces bpf_ktime_get_ns() (xdp.rs:95, tc.rs:80): a replay cannot
 * reproduce the hook-time clock, so the record carries the trace timestamp.
 * The arena may be followed by anything; the kernel never reads past
 * arena_len. */
typedef struct tcbee_frames {
    const uint8_t*  arena;
    uint64_t        arena_len;
    const uint64_t* offset;
    const uint32_t* caplen;
    const uint64_t* ts_ns;
    uint64_t        n;
} tcbee_frames;

/* Counters of counters.rs, summed over CPUs the way the TUI does
 * (tcbee/src/viz/rate_watcher.rs:52-76), widened to u64 (no wrap). */
typedef struct tcbee_counters {
    uint64_t ingress;   /* INGRESS_EVENTS: accepted TCP frames, direction 0 */
    uint64_t egress;    /* EGRESS_EVENTS:  accepted TCP frames, direction 1 */
    uint64_t handled;   /* EVENTS_HANDLED: records written                  */
    uint64_t dropped;   /* EVENTS_DROPPED: accepted but no output room      */
} tcbee_counters;

/* One flow of the context's flow table (64 B).
 * tuple = IpTuple repr(C) bytes (flow.rs:4-12; v4 address = 12 zero bytes +
 * 4 wire bytes, xdp.rs:116-119) followed by 2 zero bytes. Flow ids are dense,
 * assigned in first-seen order over the whole record stream of the context
 * (the order in which tcbee-process creates flows, db_writer.rs:51-65). */
typedef struct tcbee_flow_entry {
    uint8_t  tuple[TCBEE_KEY_BYTES];
    uint64_t pkts;        /* records of this flow                         */
    uint64_t bytes;       /* sum of caplen of those frames                */
    uint64_t first_seen;  /* global record index of its first record      */
} tcbee_flow_entry;

/* ---- library ------------------------------------------------------------- */
int         tcbee_abi_version(void);
const char* tcbee_strerror(int code);
/* Number of HIP devices visible (0 if none). Safe to call without a GPU. */
int         tcbee_device_count(int* n);

/* ---- context --------------------------------------------------------------
 * max_frames: largest batch (frames) any parse call on this ctx will pass.
 * max_arena : largest arena (bytes) the HOST entry point will copy.
 * max_flows : flow-table capacity in distinct flows, an exact bound: the claim
 *             of a flow past it is refused (TCBEE_EFLOWFULL; its frames stay
 *             unclassified, flow id ~0); at most 2^24 (TCBEE_ECAPACITY above).
 *             Device footprint per max_flow: ~171 B of compact
 *             slots (IPv4-form keys, 8 slots per flow, 3 per 64-B unit) + 104 B of
 *             per-claim state (key 64, first_seen 8, counters 16, id map 4, new-flow
 *             list 8, first-seen copy 4) — 275 MB at 1M flows — PLUS the wide slots
 *             of non-IPv4-form (IPv6) keys: a power of two >= 8 x max_wide_flows
 *             slots of 64 B (512-1024 B per wide flow: 512 MiB at 1M), allocated
 *             whatever the trace holds; tcbee_ctx_create sizes them for
 *             max_wide_flows = max_flows.
 *             Per frame of max_frames: 8 B of K1 -> K3 words (+8 B for a second
 *             slot once an asynchronous-ids batch runs), a first-seen bit, and for
 *             tables of more than 12288 flows ~4.2 B of K3 mode-1 scratch. A small
 *             context (max_flows <= 256) with max_frames <= 2^20 also keeps a
 *             second table generation and the second slot from creation (8 B per
 *             frame + ~88 KB), so that a table reset costs no launch.
 * device    : HIP device ordinal. */
int tcbee_ctx_create(tcbee_ctx** out, int device, uint64_t max_frames,
                     uint64_t max_arena, uint64_t max_flows);
/* ABI 5. The same with the wide slots sized for max_wide_flows (16..max_flows)
 * non-IPv4-form keys — an exact bound like max_flows: a wide key past it is
 * refused (TCBEE_EFLOWFULL) without taking a claim. An IPv4-only capture of 1M
 * flows needs max_wide_flows = 16 (4 KiB of wide slots instead of 512 MiB). */
int tcbee_ctx_create_ex(tcbee_ctx** out, int device, uint64_t max_frames,
                        uint64_t max_arena, uint64_t max_flows, uint64_t max_wide_flows);
int tcbee_ctx_destroy(tcbee_ctx* ctx);
/* The context's own HIP stream (hipStream_t as void*). */
int tcbee_ctx_stream(tcbee_ctx* ctx, void** stream);
int tcbee_ctx_sync(tcbee_ctx* ctx);

/* ---- the hot path (device-resident) ---------------------------------------
 * Parses in_dev->n frames that already live in HBM. Writes, in input order and
 * compacted to accepted frames only:
 *   out_rec74     [out_cap * 74] bytes  — tcbee-process record layout
 *   out_flow_hash [out_cap] u32          — tcbee flow hash v1 of the IpTuple
 *   out_flow_id   [out_cap] u32          — dense first-seen flow id
 * (flow outputs may be NULL, and are skipped entirely with TCBEE_F_NO_FLOWS).
 * out_n_dev (device u64) receives the number of records written;
 * ctr_dev (device tcbee_counters) is ACCUMULATED into (zero it once).
 * Asynchronous on `stream`; the flow table of ctx is updated in place.
 * in_dev is a host struct whose pointers are device pointers. */
int tcbee_parse_batch_device(tcbee_ctx* ctx, const tcbee_frames* in_dev,
                             const tcbee_cfg* cfg,
                             uint8_t* out_rec74, uint64_t out_cap,
                             uint32_t* out_flow_hash, uint32_t* out_flow_id,
                             uint64_t* out_n_dev, tcbee_counters* ctr_dev,
                             void* stream);

/* Extended outputs of a device-resident parse (ABI 2). */
#define TCBEE_EX_DEFER_IDS 0x1u  /* stop before K3: see tcbee_parse_finish_device */
#define TCBEE_EX_ASYNC_IDS 0x2u  /* K3 on ex->ids_stream, beside the next batch     */
typedef struct tcbee_parse_ex {
    /* [out_cap] u32: for each record written, the batch-local index of the frame
     * it came from (NULL = not written). What a flow-hash shard of a real trace
     * needs to place its flows in the global trace: rejected frames (non-TCP,
     * runts, FILTER_PORT, xdp.rs:37-92) make record k != frame k. */
    uint32_t* out_frame_index;
    /* TCBEE_EX_DEFER_IDS: records, hashes and the flow table (with local dense ids)
     * are produced; the per-record flow ids, pkts/bytes, counters and out_n are
     * written by tcbee_parse_finish_device, which must come before any other call
     * on the context except the exchanges' calls, which read only the table's keys,
     * first_seen and local ids: tcbee_flow_first_frames_device (the flow-hash
     * exchange's input), tcbee_owner_bucket_device (the owner exchange's input),
     * tcbee_status_raise_device, and tcbee_flow_export_global_device (it places
     * flows then, without counts). */
    uint32_t  flags;
    uint32_t  reserved32;    /* zero */
    /* TCBEE_EX_ASYNC_IDS: K3 — the per-record flow ids, pkts/bytes, counters and
     * out_n — runs on ids_stream (a hipStream_t) after this batch's K2, so it can
     * overlap the next batch's K1 on `stream` (batches alternate two internal
     * slots for what K3 reads). The context orders what depends on it: the next
     * batch's K2 and every table read wait for it. The CALLER orders its own
     * readers of out_flow_id / out_n / counters after ids_stream. */
    void*     ids_stream;
    uint64_t  reserved[5];   /* zero */
} tcbee_parse_ex;
int tcbee_parse_batch_device_ex(tcbee_ctx* ctx, const tcbee_frames* in_dev,
                                const tcbee_cfg* cfg,
                                uint8_t* out_rec74, uint64_t out_cap,
                                uint32_t* out_flow_hash, uint32_t* out_flow_id,
                                uint64_t* out_n_dev, tcbee_counters* ctr_dev,
                                const tcbee_parse_ex* ex, void* stream);

/* Completes a TCBEE_EX_DEFER_IDS parse (K3): out_flow_id[p] = id_map_dev[local
 * id of record p's flow] (0xFFFFFFFF past map_len), or the local id when id_map_dev
 * is NULL; counters by local id, out_n and ctr as the plain call. Asynchronous. */
int tcbee_parse_finish_device(tcbee_ctx* ctx, const uint32_t* id_map_dev, uint64_t map_len,
                              void* stream);

/* Same, host buffers in and out (H2D of frames, D2H of records), synchronous.
 * out_n / ctr are host pointers; ctr is accumulated into. */
int tcbee_parse_batch(tcbee_ctx* ctx, const tcbee_frames* in_host,
                      const tcbee_cfg* cfg,
                      uint8_t* out_rec74, uint64_t out_cap,
                      uint32_t* out_flow_hash, uint32_t* out_flow_id,
                      uint64_t* out_n, tcbee_counters* ctr);

/* ---- flow table ------------------------------------------------------------ */
/* Synchronous. Number of distinct flows seen so far / export in id order. */
int tcbee_flow_count(tcbee_ctx* ctx, uint64_t* n);
int tcbee_flow_export(tcbee_ctx* ctx, tcbee_flow_entry* out_host, uint64_t cap,
                      uint64_t* n);
/* Forget every flow (ids restart at 0, record index restarts at 0). */
int tcbee_flow_reset(tcbee_ctx* ctx);
/* Device-side export: out_dev[id] for every flow id < cap (async on stream);
 * n_dev (device u64[2], may be NULL) receives {min(flow count, cap), accepted
 * frames so far} — exactly one segment's entry of seg_meta below. */
int tcbee_flow_export_device(tcbee_ctx* ctx, tcbee_flow_entry* out_dev, uint64_t cap,
                             uint64_t* n_dev, void* stream);
/* Multi-GPU merge. ent_dev holds nseg segments of `stride`
 * entries: segment r = rank r's exported table; seg_meta_dev[2r] = its valid
 * entries, seg_meta_dev[2r+1] = its records (segments are consecutive slices of
 * one global record stream, first_seen local to the segment). The context's
 * table is REPLACED by the merge: flows equal by key are one flow, pkts/bytes
 * summed, first_seen = (records of earlier segments) + local first_seen,
 * minimised, dense ids in global first-seen order. out_ids_dev[r*stride + j] =
 * merged id of entry j of segment r (rank r's local-to-global id map).
 * max_total_records bounds the global record count. Asynchronous; the first
 * merge (or a larger bound) allocates scratch and synchronizes. */
int tcbee_flow_merge_device(tcbee_ctx* ctx, const tcbee_flow_entry* ent_dev,
                            uint64_t nseg, uint64_t stride, const uint64_t* seg_meta_dev,
                            uint64_t max_total_records, uint32_t* out_ids_dev, void* stream);
/* Global-order export for a flow-hash shard (one rank's frames are a
 * subsequence of one global trace). The context's table must
 * hold the flows of ONE batch (reset before it, as a per-window recorder does).
 * As tcbee_flow_export_device, but each entry's first_seen is the GLOBAL FRAME
 * index of the flow's first record: frame_gidx_dev[rec_frame_dev[r]] for the
 * flow's first record r of the batch (rec_frame_dev = that batch's
 * tcbee_parse_ex.out_frame_index with out_cap >= its records), or
 * frame_gidx_dev[r] when rec_frame_dev is NULL — allowed only if every one of
 * the batch's n_frames frames was accepted, which the device checks.
 * n_dev[1] = 0: the merge then rebases nothing, so flows of any partition merge
 * in global first-seen order. A first record that cannot be placed exports
 * first_seen ~0 and makes the next tcbee_ctx_status return TCBEE_ESHARD. */
int tcbee_flow_export_global_device(tcbee_ctx* ctx, tcbee_flow_entry* out_dev, uint64_t cap,
                                    uint64_t* n_dev, const uint32_t* rec_frame_dev,
                                    const uint64_t* frame_gidx_dev, uint64_t n_frames,
                                    uint64_t rec_frame_cap, void* stream);
/* The flow-hash exchange: tables of the ranks are disjoint, so
 * global first-seen ids need only each flow's global first frame.
 * Batches are WINDOWS of one global trace: window w covers the same global frame
 * range on every rank (each rank parsing its shard's frames inside it), with the
 * table kept across windows or reset before each.
 * first_frames: for the flows first seen in the last batch (local ids [fbase,
 * fbase + n_new)), out_first_frame_dev[id - fbase] = global frame index of the
 * flow's first record (placed as tcbee_flow_export_global_device places it; same
 * TCBEE_ESHARD rule, also if n_new > cap); n_dev[0] = n_new, n_dev[1] = fbase.
 * global_ids: from the all-gathered arrays (rank r's at all_first_frame_dev +
 * r*stride, its {n_new, fbase} at all_n_dev[r*n_stride], [r*n_stride+1]; n_stride
 * 0 = 2, a separate array — or n_dev placed at out_first_frame_dev + cap and the
 * two gathered as ONE array of stride cap + 2, n_stride = stride) the local -> global ids
 * of `rank`'s new flows: out_map_dev[fbase + l] = *gbase_in_dev + l + new flows of
 * the other ranks first seen earlier (entries past map_cap are not written);
 * *gbase_out_dev = *gbase_in_dev + every rank's n_new (global flows after this
 * window; keep the two words as a ping-pong pair across windows, NULL in = 0).
 * Earlier entries of out_map_dev (older flows) are left as they are. */
int tcbee_flow_first_frames_device(tcbee_ctx* ctx, uint64_t* out_first_frame_dev, uint64_t cap,
                                   uint64_t* n_dev, const uint32_t* rec_frame_dev,
                                   const uint64_t* frame_gidx_dev, uint64_t n_frames,
                                   uint64_t rec_frame_cap, void* stream);
int tcbee_global_ids_device(const uint64_t* all_first_frame_dev, const uint64_t* all_n_dev,
                            uint64_t n_stride, uint32_t world, uint32_t rank, uint64_t stride,
                            uint32_t* out_map_dev, uint64_t map_cap,
                            const uint64_t* gbase_in_dev, uint64_t* gbase_out_dev, void* stream);

/* Owner exchange for CONTIGUOUS shards (every rank may hold every flow; SURVEY.md
 * §8(e) option 2). Each flow is merged at one owner rank, owner =
 * fold32(flow_hash64(key)) % world; per batch, between K2 and K3
 * (TCBEE_EX_DEFER_IDS), all device-side and asynchronous on `stream`:
 *  tcbee_owner_bucket_device: the context's flows into `world` segments of
 *    seg_cap entries (segment o at ent_dev + o*seg_cap: key, pkts/bytes 0,
 *    first_seen local), lid_dev = local id of each entry, meta_dev[0..world) =
 *    entries per owner (the ones past seg_cap, and flows whose local id is not
 *    below map_cap — the local -> global map's size — are dropped: a map_cap drop
 *    takes no segment slot; the context's status reports TCBEE_ESHARD),
 *    meta_dev[world] = the context's records, meta_dev[world + 1] = entries dropped
 *    (ABI 3: meta_dev holds world + 2 words);
 *  -> all-gather of meta, all-to-all of the segments (rank r's segment o to o);
 *  tcbee_status_raise_device(ctx, all_meta + world + 1, world, world + 2): a peer's
 *    drops make every rank's global ids unreliable, so every rank's context then
 *    reports TCBEE_ESHARD as well (generally: ESHARD if any v_dev[i * stride],
 *    i < n, is non-zero);
 *  -> the owner merges what it received with tcbee_flow_merge_device (segment r
 *    = rank r's entries, seg_meta {count, records of rank r}: first_seen rebased
 *    to the global record stream) on a second context;
 *  tcbee_flow_first_seen_device (on that context): out_dev[id] = first_seen of
 *    flow id (ascending), n_dev = {flows, 0}: with tcbee_global_ids_device over
 *    the all-gathered arrays, the owner's id -> global id map;
 *  tcbee_owner_return_device: ret_dev[e] = gmap_dev[ids_dev[e]] for the valid
 *    received entries (ids_dev: the merge's out_ids; seg_meta_dev as the merge's);
 *  -> all-to-all back (each entry's global id returns to the place it was sent from);
 *  tcbee_owner_apply_device: map_dev[lid_dev[e]] = back_dev[e] for the valid sent
 *    entries: the local -> global id map for tcbee_parse_finish_device.
 * The context-free calls here and tcbee_global_ids_device read a NULL stream as
 * HIP's null stream, as tcbee_remap_ids_device does: pass the caller's stream. */
int tcbee_owner_bucket_device(tcbee_ctx* ctx, uint32_t world, uint64_t seg_cap, uint64_t map_cap,
                              tcbee_flow_entry* ent_dev, uint32_t* lid_dev, uint64_t* meta_dev,
                              void* stream);
int tcbee_status_raise_device(tcbee_ctx* ctx, const uint64_t* v_dev, uint64_t n, uint64_t stride,
                              void* stream);
int tcbee_flow_first_seen_device(tcbee_ctx* ctx, uint64_t* out_dev, uint64_t cap, uint64_t* n_dev,
                                 void* stream);
int tcbee_owner_return_device(const uint32_t* ids_dev, const uint64_t* seg_meta_dev,
                              uint32_t world, uint64_t seg_cap, const uint32_t* gmap_dev,
                              uint64_t gmap_len, uint32_t* ret_dev, void* stream);
int tcbee_owner_apply_device(const uint32_t* back_dev, const uint32_t* lid_dev,
                             const uint64_t* meta_dev, uint32_t world, uint64_t seg_cap,
                             uint32_t* map_dev, uint64_t map_cap, void* stream);
/* After merging global-order exports, first_seen of the merged table is a global
 * FRAME index; the reference's is the global RECORD index (accepted frames
 * before it). This rank's share: out_counts_dev[id] = number of this rank's
 * records (first min(*n_rec_dev, n_rec_max); global frame of record k =
 * frame_gidx_dev[rec_frame_dev ? rec_frame_dev[k] : k], ascending) whose global
 * frame index is below merged flow id's first_seen, for ids < cap. Summed over
 * ranks (an all-reduce) this is the global record index, which
 * tcbee_flow_set_first_seen_device writes back. Asynchronous. */
int tcbee_flow_records_before_device(tcbee_ctx* merged, const uint32_t* rec_frame_dev,
                                     const uint64_t* frame_gidx_dev, const uint64_t* n_rec_dev,
                                     uint64_t n_rec_max, uint64_t* out_counts_dev, uint64_t cap,
                                     void* stream);
int tcbee_flow_set_first_seen_device(tcbee_ctx* ctx, const uint64_t* fs_by_id_dev, uint64_t cap,
                                     void* stream);
/* ids[p] = map[ids[p]] for p < min(*n_dev, n_max) (n_dev may be NULL);
 * ids >= map_len or 0xFFFFFFFF become 0xFFFFFFFF: local ids -> merged ids.
 * No context: a NULL stream is HIP's null stream (callers that order the remap
 * after work on their own stream must pass that stream). */
int tcbee_remap_ids_device(uint32_t* ids_dev, uint64_t n_max, const uint64_t* n_dev,
                           const uint32_t* map_dev, uint64_t map_len, void* stream);
/* tcbee_flow_reset, asynchronous: applied by the next launch on the context
 * (`stream` is not used). */
int tcbee_flow_reset_device(tcbee_ctx* ctx, void* stream);
/* Sticky status of the last batches: TCBEE_OK, TCBEE_EFLOWFULL, TCBEE_ESPIN or
 * TCBEE_ESHARD.
 * Synchronous; clears the status. */
int tcbee_ctx_status(tcbee_ctx* ctx);

/* Diagnostic: how the last batch's per-flow counting (K3) ran — 0 LDS bins per
 * block, 1 claims bucketed, 2 device atomics, 3 claim ranges per XCD column,
 * -1 none yet. Synchronous. */
int tcbee_ctx_count_mode(tcbee_ctx* ctx, int* mode);

/* ---- measurement ------------------------------------------------------------
 * When enabled, every parse call records a HIP event pair around K1 (the parse
 * kernel) on the stream it is launched on. profile_read synchronizes those
 * events and returns the summed K1 time and the number of K1 launches since the
 * last enable (up to 4096 launches are kept). */
int tcbee_ctx_profile(tcbee_ctx* ctx, int enable);
int tcbee_ctx_profile_read(tcbee_ctx* ctx, double* k1_ms_total, uint64_t* k1_launches);

/* ---- synthetic trace generator (device) -----------------------------------
 * Fills the header bytes of frames whose offset/caplen are already on the
 * device (see DESIGN.md "Synthetic traces"); local frame j is global frame
 * first_index + j. kind 0 = config-2 single flow, kind 1 = multi-flow IPv4
 * (flow of frame i = splitmix64(seed + 0x1000 + i) % n_flows), kind 3 = the same
 * flows over IPv6/TCP (74 header bytes). Payload bytes are left as they are
 * (callers zero the arena). Asynchronous on stream. */
int tcbee_gen_frames_device(uint8_t* arena_dev, const uint64_t* offset_dev,
                            const uint32_t* caplen_dev, uint64_t n,
                            uint64_t first_index, int kind, uint64_t n_flows,
                            uint64_t seed, void* stream);
/* The same frames on the host (bit-identical to the device generator). */
int tcbee_gen_frames_host(uint8_t* arena, const uint64_t* offset,
                          const uint32_t* caplen, uint64_t n, uint64_t first_index,
                          int kind, uint64_t n_flows, uint64_t seed);
/* Zipf flow mix (config 3, second run): as kind 1, but frame i's flow is the
 * first k with zcdf[k] > splitmix64(seed + 0x1000 + i), zcdf = n_flows u64
 * CDF words (non-decreasing, last = 2^64-1; tcbee_amd.trace.zipf_cdf builds the
 * s = 1.1 table). zcdf_dev is a device pointer for _device, a host one for _host;
 * both generators produce identical bytes from identical tables. */
int tcbee_gen_frames_zipf_device(uint8_t* arena_dev, const uint64_t* offset_dev,
                                 const uint32_t* caplen_dev, uint64_t n, uint64_t first_index,
                                 uint64_t n_flows, uint64_t seed, const uint64_t* zcdf_dev,
                                 void* stream);
int tcbee_gen_frames_zipf_host(uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                               uint64_t n, uint64_t first_index, uint64_t n_flows,
                               uint64_t seed, const uint64_t* zcdf);
/* As tcbee_gen_frames_device, local frame j being global frame gidx_dev[j]. */
int tcbee_gen_frames_index_device(uint8_t* arena_dev, const uint64_t* offset_dev,
                                  const uint32_t* caplen_dev, const uint64_t* gidx_dev,
                                  uint64_t n, int kind, uint64_t n_flows, uint64_t seed,
                                  void* stream);
/* One GPU's flow-hash shard of the global synthetic trace [0, n_global)
 * (config 4, the NIC-RSS view): the frames whose flow hash satisfies
 * fold32(flow_hash64(key)) % world == rank, in global order. Writes
 * out_gidx_dev[k] (global index) and out_caplen_dev[k] (64 B, or IMIX 64/576/1500
 * when imix != 0, as synth_index) for k < min(count, cap), and *n_out_dev = count.
 * scratch_dev: tcbee_gen_shard_scratch(n_global) u64 words. Asynchronous. */
uint64_t tcbee_gen_shard_scratch(uint64_t n_global);
int tcbee_gen_shard_index_device(uint64_t n_global, int world, int rank, int kind,
                                 uint64_t n_flows, uint64_t seed, int imix,
                                 uint64_t* out_gidx_dev, uint32_t* out_caplen_dev, uint64_t cap,
                                 uint64_t* scratch_dev, uint64_t* n_out_dev, void* stream);
/* ABI 4. The same with a NIC's RSS indirection table: frame i goes to GPU
 * rss_dev[fold32(flow_hash64(key)) % rss_len] (entries < world; rss_len <= 4096;
 * rss_dev NULL = the modulo above), so a table can balance the GPUs' loads while
 * every flow still lands on exactly one GPU. The table lives in device memory, so
 * its entries are validated on the device: a table with an entry >= world sets
 * *n_out_dev = TCBEE_RSS_INVALID (no shard holds 2^64 - 1 frames) instead of
 * silently dropping that bucket's frames on every rank. */
#define TCBEE_RSS_INVALID (~(uint64_t)0)
int tcbee_gen_shard_index_rss_device(uint64_t n_global, int world, int rank, int kind,
                                     uint64_t n_flows, uint64_t seed, int imix,
                                     const uint16_t* rss_dev, uint32_t rss_len,
                                     uint64_t* out_gidx_dev, uint32_t* out_caplen_dev,
                                     uint64_t cap, uint64_t* scratch_dev, uint64_t* n_out_dev,
                                     void* stream);
/* ABI 4. Frames per RSS bucket (fold32(flow_hash64(key)) % rss_len) over global
 * frames [0, n_frames) of the synthetic trace: counts_dev[rss_len] u64 (overwritten),
 * the observed load a table is balanced on (tcbee_amd.trace.rss_table). Asynchronous. */
int tcbee_gen_rss_load_device(uint64_t n_frames, int kind, uint64_t n_flows, uint64_t seed,
                              uint32_t rss_len, uint64_t* counts_dev, void* stream);
/* ABI 5. The same over global frames [first_frame, first_frame + n_frames): a table
 * balanced on traffic outside the frames it then places (held out, as a NIC's RSS
 * table is rebalanced from earlier load). */
int tcbee_gen_rss_load_range_device(uint64_t first_frame, uint64_t n_frames, int kind,
                                    uint64_t n_flows, uint64_t seed, uint32_t rss_len,
                                    uint64_t* counts_dev, void* stream);

/* ---- ingest pipeline: host frames -> records on the host ----------------
 * (replaces the live ring drain of
 * tcbee/src/eBPF/probes/headers.rs:67-109.) Frames in pageable host memory (a
 * pcap mapping, a capture buffer) are gathered chunk by chunk into pinned
 * staging by `threads` host threads, copied H2D on one stream, parsed on the
 * pipe's context (flow ids continue across chunks and calls), and the exact
 * record count copied D2H on a third stream; `depth` chunks are in flight, so
 * staging, both DMA directions and the kernels overlap.
 * window == 0: whole frames are shipped. window >= 80 (multiple of 16): only
 * the first min(caplen, window) bytes of each frame are shipped, with its
 * original caplen — the record path never reads past byte 74 of a frame, so
 * outputs are identical, and PCIe carries ~window+12 bytes per frame.
 * window == 64: frame bytes [12, 76) (no record field reads the MAC addresses),
 * one whole 64-B staging line per frame — the fastest gather. */
typedef struct tcbee_pipe tcbee_pipe;
typedef struct tcbee_pipe_cfg {
    uint64_t chunk_frames;  /* frames per chunk (0 = 1<<20)                     */
    uint64_t chunk_bytes;   /* staged arena bytes per chunk, window == 0 (0 = 512 MiB) */
    uint32_t window;        /* 0 = whole frames, else header window bytes         */
    uint32_t depth;         /* chunks in flight, 3..16 (0 = 3)                     */
    uint32_t threads;       /* host staging threads (0 = 8)                        */
    uint32_t reserved;
} tcbee_pipe_cfg;
typedef struct tcbee_pipe_stats {
    uint64_t frames, records, chunks;
} tcbee_pipe_stats;
/* Called once per chunk, in order, with that chunk's records (pinned host
 * memory valid during the call); flow_id NULL with TCBEE_F_NO_FLOWS. A
 * non-zero return aborts the run with that code. */
typedef int (*tcbee_pipe_sink_fn)(void* user, const uint8_t* rec74, const uint32_t* flow_id,
                                  uint64_t n, uint64_t first_record);

int tcbee_pipe_create(tcbee_pipe** out, int device, const tcbee_pipe_cfg* cfg,
                      uint64_t max_flows);
int tcbee_pipe_destroy(tcbee_pipe* p);
/* The pipe's context (flow table export / reset, status, profiling). */
int tcbee_pipe_ctx(tcbee_pipe* p, tcbee_ctx** ctx);
int tcbee_pipe_get_stats(const tcbee_pipe* p, tcbee_pipe_stats* st);
/* Synchronous. Records (and flow ids) go to out_rec74 / out_flow_id (host,
 * may be NULL) and/or to fn. *out_n = records produced; ctr accumulated into.
 * TCBEE_ECAPACITY if more than out_cap records were produced (the first out_cap
 * are written). */
int tcbee_pipe_run(tcbee_pipe* p, const tcbee_frames* in_host, const tcbee_cfg* cfg,
                   uint8_t* out_rec74, uint64_t out_cap, uint32_t* out_flow_id,
                   tcbee_pipe_sink_fn fn, void* user, uint64_t* out_n, tcbee_counters* ctr);
/* ABI 5. Page-lock the caller's output arrays (hipHostRegister) once, so that
 * later tcbee_pipe_run calls with these same out_rec74 / out_flow_id (and an
 * out_cap <= cap) DMA each chunk's records and ids straight into them — no pinned
 * staging and no host copy-out (the copy-out read + wrote every record again,
 * ~220 B of host-memory traffic per record). A chunk whose records would pass
 * out_cap still goes through staging. The sink then receives pointers into the
 * caller's arrays. out_flow_id may be NULL (records only). Registering another
 * pair (or NULL, 0, NULL) releases the previous one; tcbee_pipe_destroy releases
 * it too. The caller keeps the arrays alive while registered. Several pipes may
 * share one pair: a range another pipe page-locked is borrowed when that
 * registration covers the requested bytes (refcounted, process-wide; the range is
 * unregistered when its last holder releases it, whichever pipe locked it), a
 * range overlapping a registration without lying inside it is TCBEE_EINVAL; a
 * range the caller page-locked itself is used as it is when both of its ends are
 * registered (else TCBEE_EINVAL) and never unregistered here. */
int tcbee_pipe_register_output(tcbee_pipe* p, uint8_t* out_rec74, uint64_t cap,
                               uint32_t* out_flow_id);

/* ---- host utilities (no GPU needed) ------------------------------------- */
/* tcbee flow hash v1 of a 40-byte key (DESIGN.md "Flow hash"). */
uint64_t tcbee_flow_hash64(const uint8_t key40[TCBEE_KEY_BYTES]);

#ifdef __cplusplus
}
#endif
#endif /* TCBEE_AMD_H */

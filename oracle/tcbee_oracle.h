/*
 * tcbee_oracle.h — CPU restatement of TCBee's packet-record path.
 *
 * TEST INFRASTRUCTURE ONLY. This is the checker, never the product: only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * PARITY UNPINNED: the reference (Rust + eBPF) cannot be built or run in this
 * image (no rustc/cargo/bpf-linker, no network, needs root + XDP/TC attach), and
 * its repository holds no tests, golden vectors or fixtures for this path
 * (SURVEY.md §0, §4, §8c). This restatement is pinned only by the
 * known-answer vectors hand-derived from the reference source
 * (tests/golden/kat_vectors.json).
 *
 * Every function cites the reference lines it restates (paths relative to the
 * TCBee tree).
 */
#ifndef TCBEE_ORACLE_H
#define TCBEE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* repr(C) tcp_packet_trace, tcbee-common/src/bindings/tcp_header.rs:551-572 */
typedef struct orc_trace {
    uint64_t time;
    uint32_t saddr;
    uint32_t daddr;
    uint8_t  saddr_v6[16];
    uint8_t  daddr_v6[16];
    uint16_t sport;
    uint16_t dport;
    uint32_t seq;
    uint32_t ack;
    uint16_t window;
    uint8_t  flag_urg, flag_ack, flag_psh, flag_rst, flag_syn, flag_fin;
    uint16_t checksum;
} orc_trace;   /* sizeof == 72 (2 bytes tail padding) */

/* repr(C) IpTuple, tcbee-common/src/bindings/flow.rs:4-12 (38 B incl. 1 pad) */
typedef struct orc_iptuple {
    uint8_t  src_ip[16];
    uint8_t  dst_ip[16];
    uint16_t sport;
    uint16_t dport;
    uint8_t  protocol;
    uint8_t  _pad;
} orc_iptuple;

typedef struct orc_counters {
    uint64_t ingress, egress, handled, dropped;
} orc_counters;

/* Decoded view of one 74-B file record, as tcbee-process sees it
 * (tcbee-process/src/bindings/tcp_packet.rs:8-29). */
typedef struct orc_packet {
    orc_trace t;
    uint8_t   div[4];
} orc_packet;

/* ts_storage::IpTuple as built by TcpPacket::get_ip_tuple (tcp_packet.rs:93-111) */
typedef struct orc_db_tuple {
    int      is_v4;
    uint8_t  src[16];   /* v4: first 4 bytes = a.b.c.d, v6: 16 bytes */
    uint8_t  dst[16];
    int64_t  sport, dport, l4proto;
} orc_db_tuple;

/* --- the hooks ----------------------------------------------------------- */
/* xdp_hook restated (probes/xdp.rs:27-223). Returns 1 and fills *out / *key when
 * the frame yields a record; 0 otherwise (XDP_PASS without a record). */
int orc_xdp_hook(const uint8_t* frame, uint32_t caplen, uint64_t ts,
                 uint16_t filter_port, orc_trace* out, orc_iptuple* key);
/* tc_hook restated (probes/tc.rs:28-183), ctx.load() bounds semantics. */
int orc_tc_hook(const uint8_t* frame, uint32_t caplen, uint64_t ts,
                uint16_t filter_port, orc_trace* out, orc_iptuple* key);

/* bincode 1.3.3 legacy serialize of tcp_packet_trace + FF FF FF FF marker
 * (handlers/mod.rs:126,139). Writes exactly 74 bytes. */
void orc_serialize(const orc_trace* t, uint8_t rec74[74]);
/* bincode::deserialize::<TcpPacket> (tcp_packet.rs:31-41): returns 1 on success,
 * 0 on a decode error (then *out is TcpPacket::default(), as the reference). */
int  orc_deserialize(const uint8_t rec74[74], orc_packet* out);
/* db_writer.rs:76-78 marker check: 1 = ok, 0 = the reference would panic. */
int  orc_marker_ok(const orc_packet* p);
void orc_get_ip_tuple(const orc_packet* p, orc_db_tuple* out);
/* TcpPacket::get_field (tcp_packet.rs:46-62): returns 1 and *value when Some. */
int  orc_get_field(const orc_packet* p, int index, int64_t* value);

/* --- flow hash v1 (the build's own function; DESIGN.md "Flow hash") ------- */
void     orc_key40(const orc_iptuple* k, uint8_t key40[40]);
uint64_t orc_flow_hash64(const uint8_t key40[40]);

/* --- batch path: parse + FLOWS + serialize + counters --------------------- */
typedef struct orc_flowtab orc_flowtab;
orc_flowtab* orc_flowtab_new(uint64_t cap_flows);
void         orc_flowtab_free(orc_flowtab* ft);
uint64_t     orc_flowtab_count(const orc_flowtab* ft);
/* Export in id (first-seen) order: 40-B key, pkts, bytes, first_seen (64 B each,
 * same layout as tcbee_flow_entry). Returns number written. */
uint64_t     orc_flowtab_export(const orc_flowtab* ft, uint8_t* out64, uint64_t cap);

/* Parses n frames in order with the hook selected by direction (0 xdp, 1 tc).
 * Appends compacted records (up to out_cap; overflow counts as dropped) and, if
 * ft != NULL, per-record flow hash (low 32 bits of hash64 folded) / dense flow
 * id; record_base = global index of the first record (for first_seen).
 * Returns the number of records written. */
/* accept[i] = 1 iff the hook emits a record for frame i (xdp.rs:37-92 /
 * tc.rs:30-119): which frames of a partitioned trace become records. */
void orc_accept_mask(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                     uint64_t n, uint16_t filter_port, int direction, uint8_t* accept);
uint64_t orc_parse_batch(const uint8_t* arena, const uint64_t* offset,
                         const uint32_t* caplen, const uint64_t* ts, uint64_t n,
                         uint16_t filter_port, int direction,
                         uint8_t* out_rec, uint64_t out_cap,
                         uint32_t* out_hash, uint32_t* out_id,
                         orc_flowtab* ft, uint64_t record_base,
                         orc_counters* ctr);

/* The CPU baseline: the reference record path over n frames on `threads`
 * pthreads (contiguous chunks, one private FLOWS set per thread like the
 * per-CPU map, flow_tracker.rs:12-13), serializing into out_rec (>= n*74 B).
 * Returns records written. */
uint64_t orc_baseline_run(const uint8_t* arena, const uint64_t* offset,
                          const uint32_t* caplen, const uint64_t* ts, uint64_t n,
                          uint16_t filter_port, int threads, uint8_t* out_rec);
/* CPU-1-file: one thread, records appended to `path` through the drain task's
 * 720 000-B buffered writer. Records written, ~0 on I/O error. */
uint64_t orc_baseline_file(const uint8_t* arena, const uint64_t* offset,
                           const uint32_t* caplen, const uint64_t* ts, uint64_t n,
                           uint16_t filter_port, const char* path);

/* Reference FLOWS semantics: the first `max` (100, config.rs:19) distinct
 * IpTuples in arrival order. Writes 40-B keys, returns count. */
uint64_t orc_ref_flows(const uint8_t* arena, const uint64_t* offset,
                       const uint32_t* caplen, uint64_t n, uint16_t filter_port,
                       int direction, uint64_t max, uint8_t* out_keys40);

#ifdef __cplusplus
}
#endif
#endif

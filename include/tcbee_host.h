/*
 * tcbee_host.h — C ABI of the host-side callers either side of the MI355X
 * record path: classic-pcap ingest, the .tcp record files,
 * the tcbee-process flow/time-series stage with its SQLite sink, and the
 * metrics.json counters file. Library: tcbee_amd/lib/libtcbee_host.so (plain
 * C++, links the system libsqlite3; no GPU needed).
 *
 * What each group replaces in the reference tree:
 *   pcap      the live XDP/TC packet source (tcbee/src/eBPF/probes/headers.rs:67-109)
 *             — a recorded trace is replayed instead of attaching hooks.
 *   tcpfile   BufferHandler's append-only writer (tcbee/src/handlers/mod.rs:65-147)
 *             and tcbee-process' FileReader + TcpPacket decode
 *             (tcbee-process/src/reader.rs:57-112, bindings/tcp_packet.rs:8-124).
 *   sink      DBWriter / FlowTracker / TsTracker (tcbee-process/src/db_writer.rs,
 *             flow_tracker.rs) on ts-storage's SQLite backend
 *             (ts-storage/src/sqlite/db.rs).
 *   metrics   EBPFWatcher's metrics.json (tcbee/src/viz/ebpf_watcher.rs:51-59,431-454).
 *
 * Conventions are those of tcbee_amd.h: 0 or a negative TCBEE_E* code, no
 * exceptions across the ABI, caller-owned buffers.
 */
#ifndef TCBEE_HOST_H
#define TCBEE_HOST_H

#include <stdint.h>
#include "tcbee_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

#define TCBEE_HOST_ABI_VERSION 2  /* 2: RSS indirection tables (tcbee_flowhash_owner_rss, _load) */
int tcbee_host_abi_version(void);

/* ---- classic pcap ---------------------------------------------------------
 * libpcap "classic" format: magic a1b2c3d4 (µs) or a1b23c4d (ns), either byte
 * order, link type 1 (Ethernet, what XDP/TC hand to the hooks). The file is
 * memory-mapped; tcbee_pcap_frames() returns a tcbee_frames view whose arena IS
 * the mapping (offsets are absolute file offsets of each packet's data), ready
 * for tcbee_parse_batch or the ingest pipeline. ts_ns = sec*1e9 + frac.
 * A truncated trailing record ends the index (counted in `truncated`). */
typedef struct tcbee_pcap tcbee_pcap;
typedef struct tcbee_pcap_info {
    uint32_t linktype;
    uint32_t snaplen;
    uint32_t nanosecond;   /* 1 if the file stores ns fractions            */
    uint32_t swapped;      /* 1 if the file is in the other byte order      */
    uint64_t n;            /* packets indexed                               */
    uint64_t truncated;    /* 1 if a partial record ended the file          */
    uint64_t file_bytes;
} tcbee_pcap_info;

int tcbee_pcap_open(tcbee_pcap** out, const char* path);
int tcbee_pcap_frames(const tcbee_pcap* p, tcbee_frames* out);
int tcbee_pcap_get_info(const tcbee_pcap* p, tcbee_pcap_info* out);
int tcbee_pcap_close(tcbee_pcap* p);
/* Writes frames as a classic pcap (link type 1, native byte order);
 * nanosecond selects the a1b23c4d magic. orig_len = caplen. */
int tcbee_pcap_write(const char* path, const tcbee_frames* in, int nanosecond,
                     uint32_t snaplen);

/* ---- flow-hash partition (the NIC's RSS step for N GPUs) -----------------
 * owner[i] = fold32(flow_hash64(key)) % world for every frame the hook can key
 * (IPv4/TCP >= 54 B, IPv6/TCP >= 74 B; IpTuple at the fixed offsets of
 * xdp.rs:37-127), so all frames of a flow reach one GPU and the per-GPU flow
 * tables are disjoint; the same function places the device
 * generator's config-4 shards. Frames without a key (non-TCP, runts) produce no
 * record on any GPU and go round robin (i % world). FILTER_PORT is left to the
 * owning GPU's hook. threads 0 = 1. */
int tcbee_flowhash_owner(const tcbee_frames* in_host, uint32_t world, uint32_t threads,
                         uint16_t* out_owner);
/* Host ABI 2. The NIC's RSS indirection table: a keyed frame goes to GPU
 * rss[fold32(flow_hash64(key)) % rss_len] (every entry < world, rss_len <=
 * TCBEE_RSS_MAX; rss NULL = the modulo above), the same placement as
 * tcbee_gen_shard_index_rss_device. A table balanced on observed bucket loads
 * (tcbee_flowhash_load, tcbee_amd.trace.rss_table) evens out the GPUs' frame
 * counts while every flow still reaches exactly one GPU. */
#define TCBEE_RSS_MAX 4096
int tcbee_flowhash_owner_rss(const tcbee_frames* in_host, uint32_t world, const uint16_t* rss,
                             uint32_t rss_len, uint32_t threads, uint16_t* out_owner);
/* Keyed frames per RSS bucket (fold32(flow_hash64(key)) % rss_len): out_counts[rss_len]. */
int tcbee_flowhash_load(const tcbee_frames* in_host, uint32_t rss_len, uint32_t threads,
                        uint64_t* out_counts);

/* ---- .tcp record files ----------------------------------------------------
 * Decoded TcpPacket (tcbee-process/src/bindings/tcp_packet.rs:8-28), the
 * struct tcbee-process builds from each 74-byte entry. */
typedef struct tcbee_packet {
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
    uint8_t  div[4];
} tcbee_packet;

/* ts_storage::IpTuple as tcbee-process derives it (tcp_packet.rs:95-111):
 * IPv4 iff saddr != 0 && daddr != 0, else IPv6 from the v6 arrays; addresses
 * rendered as Rust's std Display does (what ts-storage stores as TEXT). */
typedef struct tcbee_ts_tuple {
    char    src[48];
    char    dst[48];
    int64_t sport;
    int64_t dport;
    int64_t l4proto;   /* always 6 */
} tcbee_ts_tuple;

/* bincode 1.x decode of n 74-byte entries (TcpPacket::from_buffer,
 * tcp_packet.rs:30-41): fixint little endian, bools must be 0/1 — an entry
 * that does not decode becomes the all-zero default (n_default counts them;
 * may be NULL). */
int tcbee_tcp_decode(const uint8_t* rec74, uint64_t n, tcbee_packet* out,
                     uint64_t* n_default);
/* The DBWriter marker check (db_writer.rs:76-78) over decoded entries:
 * TCBEE_EFORMAT and *first_bad = index of the first entry whose div is not
 * FF FF FF FF (tcbee-process panics there), else 0 and *first_bad = n. */
int tcbee_tcp_check(const uint8_t* rec74, uint64_t n, uint64_t* first_bad);
int tcbee_tcp_tuple(const tcbee_packet* p, tcbee_ts_tuple* out);

/* Append-only writer with the reference's buffering (create + append, a
 * BufWriter of WRITER_BUFFER_SIZE (10000, tcbee/src/config.rs:5) x
 * size_of::<tcp_packet_trace>() (72) = 720000 bytes, handlers/mod.rs:70-90).
 * buffer_bytes 0 = that default. */
typedef struct tcbee_tcpfile tcbee_tcpfile;
int tcbee_tcpfile_open(tcbee_tcpfile** out, const char* path, uint64_t buffer_bytes);
int tcbee_tcpfile_append(tcbee_tcpfile* f, const uint8_t* rec74, uint64_t n);
int tcbee_tcpfile_close(tcbee_tcpfile* f);

/* ---- tcbee-process stage + SQLite sink ------------------------------------
 * Builds exactly the database tcbee-process builds from xdp.tcp / tc.tcp
 * (schema of ts-storage/src/sqlite/db.rs:27-104): one `flows` row per
 * downstream IpTuple in first-seen order, 46 `time_series` rows per flow
 * (10 packet + 10 probe + 25 sock + 1 cwnd, FlowTracker::new), points only for
 * values > 0, 1001-point batches (TsTracker::add_entry's `len() <= 1000`),
 * each batch atomic (one multi-row INSERT in the reference: a duplicate
 * (series, timestamp) fails the whole batch and wedges that series,
 * flow_tracker.rs:54-70), series never written deleted at close.
 *
 * flags: TCBEE_SINK_DURABLE commits every statement on its own (the
 * reference's autocommit behaviour; slow). Default: one transaction per sink,
 * committed at close — the final database content is identical. */
#define TCBEE_SINK_DURABLE 0x1u

typedef struct tcbee_sink tcbee_sink;
typedef struct tcbee_sink_stats {
    uint64_t records;         /* entries consumed                            */
    uint64_t flows;           /* flows rows created                          */
    uint64_t series_created;
    uint64_t series_deleted;  /* never-written series removed at close        */
    uint64_t points;          /* time_series_data rows inserted               */
    uint64_t batches;         /* successful batch inserts                     */
    uint64_t failed_batches;  /* batch inserts rejected (duplicate timestamp) */
    uint64_t failed_records;  /* entries whose add_event returned an error    */
} tcbee_sink_stats;

int tcbee_sink_open(tcbee_sink** out, const char* db_path, uint32_t flags);
/* DBWriter::run for a run of Packet entries, in order. TCBEE_EFORMAT (and the
 * sink refuses further input) at the first entry failing the marker check —
 * where tcbee-process panics; what was written before stays committed. */
int tcbee_sink_packets(tcbee_sink* s, const uint8_t* rec74, uint64_t n);
/* Same result, records pre-classified on the GPU: flow_id[i] = the dense
 * first-seen flow id tcbee_parse_batch produced for entry i (ids < n_ids).
 * Entries are processed flow by flow (counting sort by id on the host), which
 * leaves every table identical to the in-order path. */
int tcbee_sink_packets_grouped(tcbee_sink* s, const uint8_t* rec74,
                               const uint32_t* flow_id, uint64_t n, uint64_t n_ids);
/* FlowTracker::flush for every flow, commit, close. stats may be NULL. */
int tcbee_sink_close(tcbee_sink* s, tcbee_sink_stats* stats);
int tcbee_sink_get_stats(const tcbee_sink* s, tcbee_sink_stats* stats);

/* tcbee-process main (tcbee-process/src/main.rs): reads <prefix>xdp.tcp then
 * <prefix>tc.tcp (each if present; whole 74-byte entries, FileReader::run)
 * into a sink on db_path. The reference's other inputs (probe.tcp, *_sock.tcp,
 * *_cwnd.tcp) come from probes outside this path and are not read. */
int tcbee_process_files(const char* source_prefix, const char* db_path,
                        uint32_t flags, tcbee_sink_stats* stats);

/* ts-storage primitives the sink is built on (TSDBInterface, ts-storage/src/
 * sqlite/db.rs). value_type: 0 Int, 1 Float, 2 Boolean, 3 String
 * (DataValue::type_to_int, ts-storage/src/lib.rs:74-95). */
int tcbee_tsdb_create_flow(tcbee_sink* s, const char* src, const char* dst,
                           int64_t sport, int64_t dport, int64_t l4proto, int64_t* id);
int tcbee_tsdb_delete_flow(tcbee_sink* s, const char* src, const char* dst,
                           int64_t sport, int64_t dport, int64_t l4proto);
int tcbee_tsdb_create_series(tcbee_sink* s, int64_t flow_id, const char* name,
                             int value_type, int64_t* id);
int tcbee_tsdb_delete_series(tcbee_sink* s, int64_t flow_id, const char* name);
/* insert_multiple_points: all n points or none (TCBEE_EDB). Integer/boolean
 * series take ivalues, float series fvalues. */
int tcbee_tsdb_insert_points(tcbee_sink* s, int64_t series_id, int value_type,
                             const double* timestamps, const int64_t* ivalues,
                             const double* fvalues, uint64_t n);
/* add / set (delete + add) / delete a flow attribute (db.rs:325-407);
 * text is used for value_type 3, ivalue for 0/2, fvalue for 1. */
int tcbee_tsdb_add_attribute(tcbee_sink* s, int64_t flow_id, const char* name,
                             int value_type, int64_t ivalue, double fvalue, const char* text);
int tcbee_tsdb_set_attribute(tcbee_sink* s, int64_t flow_id, const char* name,
                             int value_type, int64_t ivalue, double fvalue, const char* text);
int tcbee_tsdb_delete_attribute(tcbee_sink* s, int64_t flow_id, const char* name);

/* ---- metrics.json -----------------------------------------------------------
 * EBPFWatcher's --metrics file (ebpf_watcher.rs:51-59,431-454): written to
 * <dir_prefix>metrics.json as compact JSON with the Metrics field order
 * {handled, dropped, ingress, egress, ingress_calls, egress_calls}; values are
 * the u32 counters of counters.rs, so they wrap mod 2^32. ingress_calls /
 * egress_calls are the tcp_recvmsg / tcp_sendmsg probe counters (not on this
 * path; pass 0). */
int tcbee_metrics_write(const char* dir_prefix, const tcbee_counters* ctr,
                        uint64_t ingress_calls, uint64_t egress_calls);

#ifdef __cplusplus
}
#endif
#endif /* TCBEE_HOST_H */

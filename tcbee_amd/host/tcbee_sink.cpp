// tcbee-process flow/time-series stage + the ts-storage SQLite backend.
//
// Mirrors, statement for statement in effect:
//   DBWriter::setup_new_stream / run        tcbee-process/src/db_writer.rs:51-82
//   FlowTracker::new / add_event / flush    tcbee-process/src/flow_tracker.rs:120-290
//   TsTracker::add_entry / flush            tcbee-process/src/flow_tracker.rs:47-110
//   SQLiteTSDB setup / create_flow / create_time_series / insert_multiple_points /
//   delete_time_series / flow attributes    ts-storage/src/sqlite/db.rs
//
// Differences in mechanics, not in the resulting database:
//   - by default the whole run is one transaction (the reference autocommits
//     every statement); TCBEE_SINK_DURABLE restores per-statement commits;
//   - row ids come from sqlite3_last_insert_rowid instead of re-SELECTing the
//     row just inserted (same value: AUTOINCREMENT ids, UNIQUE keys);
//   - a full batch (1001 points) is ONE prepared multi-row INSERT (the reference's
//     own statement shape, its parameters bound instead of formatted into the text);
//     partial batches (the flush at close) go through one prepared single-row
//     statement inside a SAVEPOINT, rolled back on a constraint failure — the
//     multi-row statement's all-or-nothing behaviour (the multi-row form: 1.9x
//     fewer seconds per record than row by row everywhere; foreign keys stay
//     enforced per row — verifying them once at close saved only 9 % more). A
//     SQLite built with fewer than 3003 host parameters per statement cannot
//     prepare it; full batches then take the SAVEPOINT path too.
#include "tcbee_host_internal.h"

#include <sqlite3.h>

#include <cstdio>
#include <fcntl.h>
#include <new>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <unordered_map>
#include <vector>

namespace {

using namespace tcbee_host;

// ---- series catalogue: FlowTracker::new creates, per flow and in this order,
// the series of TcpPacket (tcp_packet.rs:61-89), TcpProbe (tcp_probe.rs),
// sock_trace_entry (sock.rs) and cwnd_trace_entry (cwnd.rs).
enum : int { kInt = 0, kFloat = 1, kBool = 2, kText = 3 };
struct SeriesDef { const char* name; int type; };
constexpr SeriesDef kSeries[] = {
    {"SEQ_NUM", kInt}, {"ACK_NUM", kInt}, {"WINDOW", kInt}, {"FLAG_URG", kBool},
    {"FLAG_ACK", kBool}, {"FLAG_PSH", kBool}, {"FLAG_RST", kBool}, {"FLAG_SYN", kBool},
    {"FLAG_FIN", kBool}, {"CHECKSUM", kInt},
    // TcpProbe
    {"MARK", kInt}, {"DATA_LEN", kInt}, {"SND_NXT", kInt}, {"SND_UNA", kInt},
    {"SND_CWND", kInt}, {"SSTRESH", kInt}, {"SND_WND", kInt}, {"SRTT", kInt},
    {"RCV_WND", kInt}, {"SOCK_COOKIE", kInt},
    // sock_trace_entry
    {"pacing_rate", kInt}, {"max_pacing_rate", kInt}, {"backoff", kInt}, {"rto", kInt},
    {"ato", kInt}, {"rcv_mss", kInt}, {"snd_cwnd", kInt}, {"bytes_acked", kInt},
    {"snd_ssthresh", kInt}, {"total_retrans", kInt}, {"probes", kInt}, {"lost", kInt},
    {"sacked_out", kInt}, {"retrans", kInt}, {"rcv_ssthresh", kInt}, {"rttvar", kInt},
    {"advmss", kInt}, {"reordering", kInt}, {"rcv_rtt", kInt}, {"rcv_space", kInt},
    {"bytes_received", kInt}, {"segs_out", kInt}, {"segs_in", kInt}, {"snd_wscale", kInt},
    {"rcv_wscale", kInt},
    // cwnd_trace_entry
    {"perf_snd_cwnd", kInt},
};
constexpr int kNumSeries = int(sizeof(kSeries) / sizeof(kSeries[0]));
static_assert(kNumSeries == 46, "10 packet + 10 probe + 25 sock + 1 cwnd series");
constexpr int kPacketFields = 10;      // TcpPacket::get_max_index() == 9
constexpr size_t kBufferSize = 1000;   // flow_tracker.rs BUFFER_SIZE

// Schema of SQLiteTSDB::setup (ts-storage/src/sqlite/db.rs:27-104).
const char* const kSchema[] = {
    "PRAGMA foreign_keys=ON",
    "CREATE TABLE IF NOT EXISTS flows (id INTEGER PRIMARY KEY AUTOINCREMENT, "
    "src TEXT NOT NULL, dst TEXT NOT NULL, sport INTEGER NOT NULL, dport INTEGER NOT NULL, "
    "l4proto INTEGER NOT NULL, UNIQUE (src, dst, sport, dport, l4proto))",
    "CREATE TABLE IF NOT EXISTS flow_attributes (id INTEGER PRIMARY KEY AUTOINCREMENT, "
    "flow_id INTEGER, name TEXT NOT NULL, value_boolean INTEGER DEFAULT -1, value_text TEXT, "
    "value_integer INTEGER DEFAULT -1, value_float REAL DEFAULT -1, UNIQUE (flow_id, name), "
    "FOREIGN KEY (flow_id) REFERENCES flows(id))",
    "CREATE TABLE IF NOT EXISTS time_series (time_series_id INTEGER PRIMARY KEY AUTOINCREMENT, "
    "flow_id INTEGER NOT NULL, name TEXT NOT NULL, type INTEGER NOT NULL, "
    "UNIQUE (flow_id,name), FOREIGN KEY (flow_id) REFERENCES flows(id))",
    "CREATE TABLE IF NOT EXISTS time_series_data (time_series_id INTEGER NOT NULL, "
    "timestamp FLOAT NOT NULL, value_boolean INTEGER DEFAULT -1, value_text TEXT, "
    "value_integer INTEGER DEFAULT -1, value_float REAL DEFAULT -1, "
    "PRIMARY KEY (time_series_id, timestamp), FOREIGN KEY (time_series_id) REFERENCES "
    "time_series(time_series_id) ON DELETE CASCADE)",
};

const char* value_column(int type) {
  switch (type) {
    case kInt: return "value_integer";
    case kFloat: return "value_float";
    case kBool: return "value_boolean";
    default: return "value_text";
  }
}

struct Point {
  double t;
  int64_t v;
};

struct TsTracker {
  int64_t id = 0;
  int def = 0;           // index into kSeries
  uint64_t handled = 0;
  std::vector<Point> events;
};

// Downstream flow identity: ts_storage::IpTuple (IpAddr enum + ports; l4proto
// is always 6 on this path).
struct TupleKey {
  uint8_t v4;
  uint8_t src[16], dst[16];
  uint16_t sport, dport;
  bool operator==(const TupleKey& o) const { return std::memcmp(this, &o, sizeof(*this)) == 0; }
};
static_assert(sizeof(TupleKey) == 38, "packed key");
struct TupleHash {
  size_t operator()(const TupleKey& k) const {
    uint64_t h = 0xcbf29ce484222325ull;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(&k);
    for (size_t i = 0; i < sizeof(k); ++i) h = (h ^ p[i]) * 0x100000001b3ull;
    return size_t(h ^ (h >> 29));
  }
};

TupleKey key_of(const tcbee_packet& p) {
  TupleKey k;
  std::memset(&k, 0, sizeof(k));
  if (p.saddr != 0 && p.daddr != 0) {
    k.v4 = 1;
    std::memcpy(k.src, &p.saddr, 4);
    std::memcpy(k.dst, &p.daddr, 4);
  } else {
    std::memcpy(k.src, p.saddr_v6, 16);
    std::memcpy(k.dst, p.daddr_v6, 16);
  }
  k.sport = p.sport;
  k.dport = p.dport;
  return k;
}

struct FlowTracker {
  int64_t id = 0;
  tcbee_ts_tuple tuple{};
  TsTracker tr[kNumSeries];
};

}  // namespace

struct tcbee_sink {
  sqlite3* db = nullptr;
  bool durable = false;
  bool dead = false;        // a marker check failed: no further input, no flush
  sqlite3_stmt* ins_flow = nullptr;
  sqlite3_stmt* del_flow = nullptr;
  sqlite3_stmt* ins_series = nullptr;
  sqlite3_stmt* del_series = nullptr;
  sqlite3_stmt* ins_point[4] = {};
  sqlite3_stmt* ins_batch[4] = {};  // full batches: kBufferSize + 1 rows, prepared on first use
  bool batch_unprepared[4] = {};    // that prepare failed: full batches row by row
  std::vector<FlowTracker*> flows;                          // creation order
  std::unordered_map<TupleKey, uint32_t, TupleHash> index;  // DBWriter::streams
  tcbee_sink_stats st{};
  std::vector<uint32_t> gid_map;  // grouped path: 3*(GPU flow id)+class -> flows index + 1
};

namespace {

int exec(sqlite3* db, const char* sql) {
  return sqlite3_exec(db, sql, nullptr, nullptr, nullptr) == SQLITE_OK ? TCBEE_OK : TCBEE_EDB;
}

int prep(sqlite3* db, const char* sql, sqlite3_stmt** st) {
  return sqlite3_prepare_v3(db, sql, -1, SQLITE_PREPARE_PERSISTENT, st, nullptr) == SQLITE_OK
             ? TCBEE_OK
             : TCBEE_EDB;
}

// Runs a bound statement to completion and resets it.
int step_done(sqlite3_stmt* st) {
  int rc = sqlite3_step(st);
  sqlite3_reset(st);
  sqlite3_clear_bindings(st);
  return rc == SQLITE_DONE ? TCBEE_OK : TCBEE_EDB;
}

int create_flow(tcbee_sink* s, const char* src, const char* dst, int64_t sport, int64_t dport,
                int64_t l4proto, int64_t* id) {
  sqlite3_stmt* st = s->ins_flow;
  sqlite3_bind_text(st, 1, src, -1, SQLITE_TRANSIENT);
  sqlite3_bind_text(st, 2, dst, -1, SQLITE_TRANSIENT);
  sqlite3_bind_int64(st, 3, sport);
  sqlite3_bind_int64(st, 4, dport);
  sqlite3_bind_int64(st, 5, l4proto);
  if (step_done(st)) return TCBEE_EDB;
  *id = sqlite3_last_insert_rowid(s->db);
  return TCBEE_OK;
}

int create_series(tcbee_sink* s, int64_t flow_id, const char* name, int type, int64_t* id) {
  sqlite3_stmt* st = s->ins_series;
  sqlite3_bind_int64(st, 1, flow_id);
  sqlite3_bind_text(st, 2, name, -1, SQLITE_STATIC);
  sqlite3_bind_int64(st, 3, type);
  if (step_done(st)) return TCBEE_EDB;
  *id = sqlite3_last_insert_rowid(s->db);
  ++s->st.series_created;
  return TCBEE_OK;
}

int delete_series(tcbee_sink* s, int64_t flow_id, const char* name) {
  sqlite3_stmt* st = s->del_series;
  sqlite3_bind_int64(st, 1, flow_id);
  sqlite3_bind_text(st, 2, name, -1, SQLITE_STATIC);
  return step_done(st);
}

// insert_multiple_points (db.rs:548-588): all rows or none.
int insert_points(tcbee_sink* s, int64_t series_id, int type, const double* t,
                  const int64_t* iv, const double* fv, const char* const* tv, uint64_t n) {
  if (n == 0) return TCBEE_EDB;  // "INSERT ... VALUES;" is a syntax error
  sqlite3_stmt*& st = s->ins_batch[type];
  if (n == kBufferSize + 1 && !st && !s->batch_unprepared[type]) {
    std::string q = std::string("INSERT INTO time_series_data (time_series_id, timestamp, ") +
                    value_column(type) + ") VALUES ";
    for (uint64_t i = 0; i < n; ++i) q += i ? ",(?,?,?)" : "(?,?,?)";
    if (prep(s->db, q.c_str(), &st)) {
      st = nullptr;  // e.g. SQLITE_MAX_VARIABLE_NUMBER < 3003: row by row below
      s->batch_unprepared[type] = true;
    }
  }
  if (n == kBufferSize + 1 && st) {
    // a full TsTracker batch: one multi-row statement (a constraint failure rolls
    // the whole statement back: all rows or none, as the reference's)
    for (uint64_t i = 0; i < n; ++i) {
      const int b = int(3 * i);
      sqlite3_bind_int64(st, b + 1, series_id);
      sqlite3_bind_double(st, b + 2, t[i]);
      if (type == kFloat) sqlite3_bind_double(st, b + 3, fv[i]);
      else if (type == kText) sqlite3_bind_text(st, b + 3, tv[i], -1, SQLITE_STATIC);
      else sqlite3_bind_int64(st, b + 3, iv[i]);
    }
    const int rc = step_done(st);
    if (rc == TCBEE_OK) {
      s->st.points += n;
      ++s->st.batches;
    } else {
      ++s->st.failed_batches;
    }
    return rc;
  }
  if (exec(s->db, "SAVEPOINT tcbee_batch")) return TCBEE_EDB;
  sqlite3_stmt* row = s->ins_point[type];
  int rc = TCBEE_OK;
  for (uint64_t i = 0; i < n && rc == TCBEE_OK; ++i) {
    sqlite3_bind_int64(row, 1, series_id);
    sqlite3_bind_double(row, 2, t[i]);
    if (type == kFloat) sqlite3_bind_double(row, 3, fv[i]);
    else if (type == kText) sqlite3_bind_text(row, 3, tv[i], -1, SQLITE_STATIC);
    else sqlite3_bind_int64(row, 3, iv[i]);
    rc = step_done(row);
  }
  if (rc != TCBEE_OK) exec(s->db, "ROLLBACK TO tcbee_batch");
  exec(s->db, "RELEASE tcbee_batch");
  if (rc == TCBEE_OK) {
    s->st.points += n;
    ++s->st.batches;
  } else {
    ++s->st.failed_batches;
  }
  return rc;
}

int insert_tracker(tcbee_sink* s, TsTracker& tr) {
  const size_t n = tr.events.size();
  // Points are stored {t, v} interleaved; gather into the two columns.
  static thread_local std::vector<double> tt;
  static thread_local std::vector<int64_t> vv;
  tt.resize(n);
  vv.resize(n);
  for (size_t i = 0; i < n; ++i) {
    tt[i] = tr.events[i].t;
    vv[i] = tr.events[i].v;
  }
  return insert_points(s, tr.id, kSeries[tr.def].type, tt.data(), vv.data(), nullptr, nullptr, n);
}

// TsTracker::add_entry (flow_tracker.rs:47-70).
inline int add_entry(tcbee_sink* s, TsTracker& tr, double t, int64_t v) {
  ++tr.handled;
  if (tr.events.size() <= kBufferSize) {
    tr.events.push_back({t, v});
    return TCBEE_OK;
  }
  if (insert_tracker(s, tr)) return TCBEE_EDB;  // buffer kept: the series is wedged
  tr.events.clear();
  tr.events.push_back({t, v});
  return TCBEE_OK;
}

// FlowTracker::add_event for EventType::Packet: fields 0..=9 in order, a
// failing add_entry aborts the rest of this event (the `?`).
inline int add_packet(tcbee_sink* s, FlowTracker& f, const tcbee_packet& p) {
  const double t = double(p.time);
  const int64_t val[kPacketFields] = {p.seq, p.ack, p.window, p.flag_urg, p.flag_ack,
                                      p.flag_psh, p.flag_rst, p.flag_syn, p.flag_fin,
                                      p.checksum};
  for (int i = 0; i < kPacketFields; ++i) {
    if (val[i] <= 0) continue;  // get_field: values > 0 / flags when true
    if (add_entry(s, f.tr[i], t, val[i])) return TCBEE_EDB;
  }
  return TCBEE_OK;
}

// FlowTracker::new: create_flow, then the 46 series.
int new_flow(tcbee_sink* s, const tcbee_packet& p, uint32_t* idx) {
  FlowTracker* f = new (std::nothrow) FlowTracker;
  if (!f) return TCBEE_ENOMEM;
  packet_tuple(p, &f->tuple);
  if (create_flow(s, f->tuple.src, f->tuple.dst, f->tuple.sport, f->tuple.dport, 6, &f->id)) {
    delete f;
    return TCBEE_EDB;  // tcbee-process: expect("Failed to create flow entry!")
  }
  for (int i = 0; i < kNumSeries; ++i) {
    f->tr[i].def = i;
    if (i < kPacketFields) f->tr[i].events.reserve(kBufferSize + 1);
    if (create_series(s, f->id, kSeries[i].name, kSeries[i].type, &f->tr[i].id)) {
      delete f;
      return TCBEE_EDB;
    }
  }
  *idx = uint32_t(s->flows.size());
  s->flows.push_back(f);
  ++s->st.flows;
  return TCBEE_OK;
}

int lookup_or_create(tcbee_sink* s, const tcbee_packet& p, uint32_t* idx) {
  const TupleKey k = key_of(p);
  auto it = s->index.find(k);
  if (it != s->index.end()) {
    *idx = it->second;
    return TCBEE_OK;
  }
  int rc = new_flow(s, p, idx);
  if (rc == TCBEE_OK) s->index.emplace(k, *idx);
  return rc;
}

// TsTracker::flush (flow_tracker.rs:72-108).
void flush_tracker(tcbee_sink* s, FlowTracker& f, TsTracker& tr) {
  if (tr.events.empty()) {
    if (tr.handled < 1 && delete_series(s, f.id, kSeries[tr.def].name) == TCBEE_OK)
      ++s->st.series_deleted;
    return;
  }
  if (insert_tracker(s, tr) == TCBEE_OK) tr.events.clear();
}

// One decoded, marker-checked entry through DBWriter::run's Packet arm.
inline int consume(tcbee_sink* s, const tcbee_packet& p, uint32_t idx) {
  ++s->st.records;
  if (add_packet(s, *s->flows[idx], p)) ++s->st.failed_records;  // logged, not fatal
  return TCBEE_OK;
}

int fail_marker(tcbee_sink* s) {
  // tcbee-process panics in the DB thread: nothing after this entry is
  // written and no flush runs. Keep what was written so far.
  s->dead = true;
  if (!s->durable) exec(s->db, "COMMIT");
  return TCBEE_EFORMAT;
}

void free_sink(tcbee_sink* s) {
  for (FlowTracker* f : s->flows) delete f;
  sqlite3_stmt* all[] = {s->ins_flow, s->del_flow, s->ins_series, s->del_series,
                         s->ins_point[0], s->ins_point[1], s->ins_point[2], s->ins_point[3],
                         s->ins_batch[0], s->ins_batch[1], s->ins_batch[2], s->ins_batch[3]};
  for (sqlite3_stmt* st : all)
    if (st) sqlite3_finalize(st);
  if (s->db) sqlite3_close(s->db);
  delete s;
}

}  // namespace

extern "C" {

int tcbee_sink_open(tcbee_sink** out, const char* db_path, uint32_t flags) {
  if (!out || !db_path) return TCBEE_EINVAL;
  *out = nullptr;
  tcbee_sink* s = new (std::nothrow) tcbee_sink;
  if (!s) return TCBEE_ENOMEM;
  s->durable = flags & TCBEE_SINK_DURABLE;
  if (sqlite3_open_v2(db_path, &s->db, SQLITE_OPEN_READWRITE | SQLITE_OPEN_CREATE, nullptr) !=
      SQLITE_OK)
    return free_sink(s), TCBEE_EIO;
  for (const char* q : kSchema)
    if (exec(s->db, q)) return free_sink(s), TCBEE_EDB;
  int rc = prep(s->db, "INSERT INTO flows (src, dst, sport, dport, l4proto) VALUES (?1,?2,?3,?4,?5)",
                &s->ins_flow);
  rc = rc ? rc : prep(s->db, "DELETE FROM flows WHERE src = ?1 AND dst = ?2 AND sport = ?3 AND "
                             "dport = ?4 AND l4proto = ?5", &s->del_flow);
  rc = rc ? rc : prep(s->db, "INSERT INTO time_series (flow_id, name, type) VALUES (?1,?2,?3)",
                      &s->ins_series);
  rc = rc ? rc : prep(s->db, "DELETE FROM time_series WHERE flow_id = ?1 AND name = ?2",
                      &s->del_series);
  for (int t = 0; t < 4 && rc == TCBEE_OK; ++t) {
    std::string q = std::string("INSERT INTO time_series_data (time_series_id, timestamp, ") +
                    value_column(t) + ") VALUES (?1,?2,?3)";
    rc = prep(s->db, q.c_str(), &s->ins_point[t]);
  }
  if (rc) return free_sink(s), rc;
  if (!s->durable && exec(s->db, "BEGIN")) return free_sink(s), TCBEE_EDB;
  *out = s;
  return TCBEE_OK;
}

int tcbee_sink_packets(tcbee_sink* s, const uint8_t* rec74, uint64_t n) {
  if (!s || (n && !rec74)) return TCBEE_EINVAL;
  if (s->dead) return TCBEE_EFORMAT;
  tcbee_packet p;
  for (uint64_t i = 0; i < n; ++i) {
    decode_packet(rec74 + i * kRec, &p);
    if (!marker_ok(p)) return fail_marker(s);
    uint32_t idx;
    if (int rc = lookup_or_create(s, p, &idx)) return rc;
    consume(s, p, idx);
  }
  return TCBEE_OK;
}

int tcbee_sink_packets_grouped(tcbee_sink* s, const uint8_t* rec74, const uint32_t* flow_id,
                               uint64_t n, uint64_t n_ids) {
  if (!s || (n && (!rec74 || !flow_id))) return TCBEE_EINVAL;
  if (s->dead) return TCBEE_EFORMAT;
  if (n == 0) return TCBEE_OK;
  // The marker check comes first: tcbee-process would stop at the first bad
  // entry, so only the prefix before it is consumed (in-order, below).
  uint64_t first_bad = n;
  tcbee_tcp_check(rec74, n, &first_bad);
  const uint64_t m = first_bad;
  try {
    if (s->gid_map.size() < 3 * n_ids) s->gid_map.resize(3 * n_ids, 0);
    // Map each (GPU flow id, record class) to its downstream flow and group
    // entries by that flow, stable in input order (a counting sort). One GPU id
    // is one eBPF IpTuple key, but tcbee-process keys flows by the ts_storage
    // IpTuple it derives from the record (tcp_packet.rs:95-111), which also
    // depends on the record's class: v4 with both addresses set (class 0), v6
    // arrays all zero (class 1: "::" — a v4 record with a zero address), v6
    // (class 2). Within one (key, class) the derived tuple is fixed; across
    // classes one key can give two flows (v4 10.0.0.1 vs v6 ::10.0.0.1), and
    // several keys can give one flow (zero-address v4 records).
    std::vector<uint32_t> grp(m);
    std::vector<uint32_t> order_of_group;  // flows index per group, first-appearance order
    std::vector<uint32_t> group_of_flow(s->flows.size() + 1, UINT32_MAX);
    std::vector<uint64_t> count;
    tcbee_packet p;
    for (uint64_t i = 0; i < m; ++i) {
      const uint32_t g = flow_id[i];
      if (g >= n_ids) return TCBEE_EINVAL;
      const uint8_t* r = rec74 + i * kRec;
      uint32_t cls;
      if (ld32(r + 8) != 0 && ld32(r + 12) != 0) {
        cls = 0;
      } else {
        uint64_t v6 = 0;
        for (int k = 0; k < 4; ++k) v6 |= ld64(r + 16 + 8 * k);
        cls = v6 ? 2 : 1;
      }
      uint32_t& slot = s->gid_map[3 * uint64_t(g) + cls];
      uint32_t idx;
      if (slot) {
        idx = slot - 1;
      } else {
        decode_packet(r, &p);
        if (int rc = lookup_or_create(s, p, &idx)) return rc;
        slot = idx + 1;
      }
      if (idx >= group_of_flow.size()) group_of_flow.resize(s->flows.size() + 1, UINT32_MAX);
      if (group_of_flow[idx] == UINT32_MAX) {
        group_of_flow[idx] = uint32_t(order_of_group.size());
        order_of_group.push_back(idx);
        count.push_back(0);
      }
      grp[i] = group_of_flow[idx];
      ++count[grp[i]];
    }
    std::vector<uint64_t> start(count.size() + 1, 0);
    for (size_t g = 0; g < count.size(); ++g) start[g + 1] = start[g] + count[g];
    std::vector<uint64_t> perm(m);
    for (uint64_t i = 0; i < m; ++i) perm[start[grp[i]]++] = i;
    uint64_t pos = 0;
    for (size_t g = 0; g < order_of_group.size(); ++g) {
      FlowTracker& f = *s->flows[order_of_group[g]];
      for (uint64_t e = pos + count[g]; pos < e; ++pos) {
        decode_packet(rec74 + perm[pos] * kRec, &p);
        ++s->st.records;
        if (add_packet(s, f, p)) ++s->st.failed_records;
      }
    }
  } catch (const std::bad_alloc&) {
    return TCBEE_ENOMEM;
  }
  return m < n ? fail_marker(s) : TCBEE_OK;
}

int tcbee_sink_get_stats(const tcbee_sink* s, tcbee_sink_stats* stats) {
  if (!s || !stats) return TCBEE_EINVAL;
  *stats = s->st;
  return TCBEE_OK;
}

int tcbee_sink_close(tcbee_sink* s, tcbee_sink_stats* stats) {
  if (!s) return TCBEE_EINVAL;
  int rc = TCBEE_OK;
  if (!s->dead) {
    // DBWriter::run's end: FlowTracker::flush for every stream.
    for (FlowTracker* f : s->flows)
      for (TsTracker& tr : f->tr) flush_tracker(s, *f, tr);
    if (!s->durable && exec(s->db, "COMMIT")) rc = TCBEE_EDB;
  }
  if (stats) *stats = s->st;
  free_sink(s);
  return rc;
}

int tcbee_process_files(const char* source_prefix, const char* db_path, uint32_t flags,
                        tcbee_sink_stats* stats) {
  if (!source_prefix || !db_path) return TCBEE_EINVAL;
  tcbee_sink* s = nullptr;
  if (int rc = tcbee_sink_open(&s, db_path, flags)) return rc;
  int rc = TCBEE_OK;
  for (const char* name : {"xdp.tcp", "tc.tcp"}) {
    const std::string path = std::string(source_prefix) + name;
    int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
    if (fd < 0) continue;  // start_file_reader: "No Entries"
    struct stat st;
    if (fstat(fd, &st) != 0) {
      ::close(fd);
      rc = TCBEE_EIO;
      break;
    }
    const uint64_t n = uint64_t(st.st_size) / kRec;  // read_exact stops at a partial entry
    if (n) {
      void* m = mmap(nullptr, n * kRec, PROT_READ, MAP_PRIVATE, fd, 0);
      if (m == MAP_FAILED) {
        ::close(fd);
        rc = TCBEE_EIO;
        break;
      }
      madvise(m, n * kRec, MADV_SEQUENTIAL);
      rc = tcbee_sink_packets(s, static_cast<const uint8_t*>(m), n);
      munmap(m, n * kRec);
    }
    ::close(fd);
    if (rc) break;
  }
  int rc2 = tcbee_sink_close(s, stats);
  return rc ? rc : rc2;
}

// ---- ts-storage primitives ---------------------------------------------------

int tcbee_tsdb_create_flow(tcbee_sink* s, const char* src, const char* dst, int64_t sport,
                           int64_t dport, int64_t l4proto, int64_t* id) {
  if (!s || !src || !dst || !id) return TCBEE_EINVAL;
  return create_flow(s, src, dst, sport, dport, l4proto, id);
}

int tcbee_tsdb_delete_flow(tcbee_sink* s, const char* src, const char* dst, int64_t sport,
                           int64_t dport, int64_t l4proto) {
  if (!s || !src || !dst) return TCBEE_EINVAL;
  sqlite3_stmt* st = s->del_flow;
  sqlite3_bind_text(st, 1, src, -1, SQLITE_TRANSIENT);
  sqlite3_bind_text(st, 2, dst, -1, SQLITE_TRANSIENT);
  sqlite3_bind_int64(st, 3, sport);
  sqlite3_bind_int64(st, 4, dport);
  sqlite3_bind_int64(st, 5, l4proto);
  return step_done(st);
}

int tcbee_tsdb_create_series(tcbee_sink* s, int64_t flow_id, const char* name, int value_type,
                             int64_t* id) {
  if (!s || !name || !id || value_type < 0 || value_type > 3) return TCBEE_EINVAL;
  return create_series(s, flow_id, name, value_type, id);
}

int tcbee_tsdb_delete_series(tcbee_sink* s, int64_t flow_id, const char* name) {
  if (!s || !name) return TCBEE_EINVAL;
  return delete_series(s, flow_id, name);
}

int tcbee_tsdb_insert_points(tcbee_sink* s, int64_t series_id, int value_type,
                             const double* timestamps, const int64_t* ivalues,
                             const double* fvalues, uint64_t n) {
  if (!s || value_type < 0 || value_type > 2 || (n && !timestamps)) return TCBEE_EINVAL;
  if (n && value_type == kFloat ? !fvalues : (n && !ivalues)) return TCBEE_EINVAL;
  return insert_points(s, series_id, value_type, timestamps, ivalues, fvalues, nullptr, n);
}

static int bind_attr(sqlite3_stmt* st, int col, int type, int64_t iv, double fv, const char* tv) {
  switch (type) {
    case kFloat: return sqlite3_bind_double(st, col, fv);
    case kText: return sqlite3_bind_text(st, col, tv ? tv : "", -1, SQLITE_TRANSIENT);
    case kBool: return sqlite3_bind_int64(st, col, iv ? 1 : 0);
    default: return sqlite3_bind_int64(st, col, iv);
  }
}

int tcbee_tsdb_add_attribute(tcbee_sink* s, int64_t flow_id, const char* name, int value_type,
                             int64_t ivalue, double fvalue, const char* text) {
  if (!s || !name || value_type < 0 || value_type > 3) return TCBEE_EINVAL;
  const std::string q = std::string("INSERT INTO flow_attributes (flow_id, name, ") +
                        value_column(value_type) + ") VALUES (?1, ?2, ?3)";
  sqlite3_stmt* st = nullptr;
  if (prep(s->db, q.c_str(), &st)) return TCBEE_EDB;
  sqlite3_bind_int64(st, 1, flow_id);
  sqlite3_bind_text(st, 2, name, -1, SQLITE_TRANSIENT);
  bind_attr(st, 3, value_type, ivalue, fvalue, text);
  int rc = sqlite3_step(st) == SQLITE_DONE ? TCBEE_OK : TCBEE_EDB;
  sqlite3_finalize(st);
  return rc;
}

int tcbee_tsdb_delete_attribute(tcbee_sink* s, int64_t flow_id, const char* name) {
  if (!s || !name) return TCBEE_EINVAL;
  sqlite3_stmt* st = nullptr;
  if (prep(s->db, "DELETE FROM flow_attributes WHERE flow_id = ?1 AND name = ?2", &st))
    return TCBEE_EDB;
  sqlite3_bind_int64(st, 1, flow_id);
  sqlite3_bind_text(st, 2, name, -1, SQLITE_TRANSIENT);
  int rc = sqlite3_step(st) == SQLITE_DONE ? TCBEE_OK : TCBEE_EDB;
  sqlite3_finalize(st);
  return rc;
}

int tcbee_tsdb_set_attribute(tcbee_sink* s, int64_t flow_id, const char* name, int value_type,
                             int64_t ivalue, double fvalue, const char* text) {
  if (int rc = tcbee_tsdb_delete_attribute(s, flow_id, name)) return rc;
  return tcbee_tsdb_add_attribute(s, flow_id, name, value_type, ivalue, fvalue, text);
}

}  // extern "C"

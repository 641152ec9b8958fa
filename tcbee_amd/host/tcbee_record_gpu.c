/* tcbee-record-gpu — a compiled host program driving the record path through the
 * two C ABIs only (include/tcbee_amd.h, include/tcbee_host.h): no Python, no torch.
 *
 * It is what tcbee-record's user-space side (tcbee-record/tcbee/src/main.rs,
 * handlers/mod.rs:65-147) does around the XDP/TC hooks, with the hooks replaced by
 * the GPU and the live interface by a capture file:
 *   pcap (mmap, tcbee_pcap_*) -> tcbee_pipe (pinned staging, H2D, K1-K3, D2H) ->
 *   the sink callback appends each chunk's 74-B records to <prefix>xdp.tcp (or
 *   tc.tcp with --tc) through the drain task's buffered writer (tcbee_tcpfile_*) ->
 *   <prefix>metrics.json (tcbee_metrics_write) -> optionally the tcbee-process
 *   stage into SQLite (tcbee_process_files, --db).
 * The Rust binding a maintainer would add has the same shape.
 *
 *   tcbee-record-gpu [--tc] [--port P] [--db PATH] [--window W] [--threads T] PCAP PREFIX
 * Prints one JSON line: frames, records, flows, counters, seconds.
 */
#define _POSIX_C_SOURCE 199309L  /* clock_gettime */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/tcbee_amd.h"
#include "../../include/tcbee_host.h"

static int append_chunk(void* user, const uint8_t* rec74, const uint32_t* flow_id, uint64_t n,
                        uint64_t first_record) {
  (void)flow_id;
  (void)first_record;
  return tcbee_tcpfile_append((tcbee_tcpfile*)user, rec74, n);
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static int fail(const char* what, int rc) {
  fprintf(stderr, "tcbee-record-gpu: %s: %s (%d)\n", what, tcbee_strerror(rc), rc);
  return 1;
}

int main(int argc, char** argv) {
  int egress = 0;
  unsigned port = 0, window = 64, threads = 8;
  const char* db = NULL;
  int i = 1;
  for (; i < argc && argv[i][0] == '-' && argv[i][1] == '-'; ++i) {
    if (!strcmp(argv[i], "--tc")) egress = 1;
    else if (!strcmp(argv[i], "--port") && i + 1 < argc) port = (unsigned)atoi(argv[++i]);
    else if (!strcmp(argv[i], "--db") && i + 1 < argc) db = argv[++i];
    else if (!strcmp(argv[i], "--window") && i + 1 < argc) window = (unsigned)atoi(argv[++i]);
    else if (!strcmp(argv[i], "--threads") && i + 1 < argc) threads = (unsigned)atoi(argv[++i]);
    else break;
  }
  if (argc - i != 2 || port > 65535) {
    fprintf(stderr, "usage: %s [--tc] [--port P] [--db PATH] [--window W] [--threads T] PCAP PREFIX\n",
            argv[0]);
    return 2;
  }
  const char* pcap_path = argv[i];
  const char* prefix = argv[i + 1];
  char out_path[4096];
  snprintf(out_path, sizeof out_path, "%s%s", prefix, egress ? "tc.tcp" : "xdp.tcp");

  const double t0 = now_s();
  /* every path out of here releases what was opened so far (one exit below) */
  tcbee_pcap* pc = NULL;
  tcbee_pipe* pipe = NULL;
  tcbee_tcpfile* tf = NULL;
  const char* what = NULL;
  int rc = 0;
  tcbee_frames fr;
  memset(&fr, 0, sizeof fr);
  if ((rc = tcbee_pcap_open(&pc, pcap_path))) { what = "pcap_open"; goto out; }
  if ((rc = tcbee_pcap_frames(pc, &fr))) { what = "pcap_frames"; goto out; }

  tcbee_pipe_cfg pcfg;
  memset(&pcfg, 0, sizeof pcfg);
  pcfg.chunk_frames = 1u << 20;
  pcfg.window = window;
  pcfg.depth = 4;
  pcfg.threads = threads;
  if ((rc = tcbee_pipe_create(&pipe, 0, &pcfg, 1u << 20))) { what = "pipe_create"; goto out; }

  /* the drain task's writer: create + append, 10000 x 72-B entries buffered
     (handlers/mod.rs:65-139; 74-B entries here, as tcbee-process reads them) */
  if ((rc = tcbee_tcpfile_open(&tf, out_path, 10000u * TCBEE_RECORD_BYTES))) {
    what = "tcpfile_open";
    goto out;
  }

  tcbee_cfg cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.filter_port = (uint16_t)port;
  cfg.direction = egress ? TCBEE_DIR_EGRESS : TCBEE_DIR_INGRESS;
  uint64_t records = 0;
  tcbee_counters ctr;
  memset(&ctr, 0, sizeof ctr);
  rc = tcbee_pipe_run(pipe, &fr, &cfg, NULL, 0, NULL, append_chunk, tf, &records, &ctr);
  const int rc_close = tcbee_tcpfile_close(tf);
  tf = NULL;
  if (rc) { what = "pipe_run"; goto out; }
  if ((rc = rc_close)) { what = "tcpfile_close"; goto out; }

  tcbee_ctx* ctx = NULL;
  uint64_t flows = 0;
  if ((rc = tcbee_pipe_ctx(pipe, &ctx)) || (rc = tcbee_flow_count(ctx, &flows))) {
    what = "flow_count";
    goto out;
  }
  if ((rc = tcbee_metrics_write(prefix, &ctr, 0, 0))) { what = "metrics_write"; goto out; }
  tcbee_sink_stats st;
  memset(&st, 0, sizeof st);
  if (db && (rc = tcbee_process_files(prefix, db, 0, &st))) { what = "process_files"; goto out; }
  const double el = now_s() - t0;
  printf("{\"frames\": %llu, \"records\": %llu, \"flows\": %llu, \"ingress\": %llu, \"egress\": %llu, "
         "\"handled\": %llu, \"dropped\": %llu, \"db_records\": %llu, \"seconds\": %.6f}\n",
         (unsigned long long)fr.n, (unsigned long long)records, (unsigned long long)flows,
         (unsigned long long)ctr.ingress, (unsigned long long)ctr.egress,
         (unsigned long long)ctr.handled, (unsigned long long)ctr.dropped,
         (unsigned long long)st.records, el);
out:
  if (tf) (void)tcbee_tcpfile_close(tf);
  if (pipe) tcbee_pipe_destroy(pipe);
  if (pc) tcbee_pcap_close(pc);
  return what ? fail(what, rc) : 0;
}

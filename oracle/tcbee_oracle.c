/*
 * tcbee_oracle.c — CPU restatement of TCBee's packet-record path.
 *
 * TEST INFRASTRUCTURE ONLY (the checker, never the thing measured or shipped).
 * PARITY UNPINNED: no reference fixtures exist for this path and the reference
 * cannot run here; pinned by hand-derived KATs only (see tcbee_oracle.h).
 *
 * Paths cited are relative to the TCBee reference tree.
 */
#include "tcbee_oracle.h"

#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* config.rs:22-33 */
enum {
    ETHERTYPE_IPV4 = 0x0800,
    ETHERTYPE_IPV6 = 0x86DD,
    TCP_PROTOCOL = 0x06,
    ETH_HDR_LEN = 14, /* sizeof(ethhdr), eth_header.rs:9-13 */
    IP_HDR_LEN = 20,  /* sizeof(iphdr),  ip4_header.rs:148-160 */
    IP6_HDR_LEN = 40, /* sizeof(ipv6hdr), ip6_header.rs:160-169 */
    TCP_HDR_LEN = 20, /* sizeof(tcphdr), tcp_header.rs:150-160 */
    MAX_FLOWS = 100,  /* config.rs:19 */
};

/* ---- byte-order helpers: a little-endian host reading wire bytes --------- */
/* A field declared __be16/__be32 is loaded natively (LE) from the wire bytes;
 * `.to_be()` on a little-endian target byte-swaps it, i.e. the result is the
 * big-endian (network-order) numeric value of those bytes. */
static uint16_t ld_le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static uint32_t ld_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint16_t swap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }
static uint32_t swap32(uint32_t v) {
    return (v >> 24) | ((v >> 8) & 0xFF00u) | ((v << 8) & 0xFF0000u) | (v << 24);
}
/* u16::to_be / u32::to_be on a little-endian target (bpfel; x86 user space) */
static uint16_t to_be16(uint16_t v) { return swap16(v); }
static uint32_t to_be32(uint32_t v) { return swap32(v); }

/* tcphdr bitfield accessors (tcp_header.rs:22-30 extract_bit on LE:
 * bit index % 8 within storage byte index/8; storage = tcp bytes 12..13).
 * fin=bit 8, syn=9, rst=10, psh=11, ack=12, urg=13 (tcp_header.rs:229-425);
 * each returns __u16 (0/1). */
static uint16_t tcp_bit(const uint8_t* tcp, int index) {
    const uint8_t byte = tcp[12 + index / 8];
    const uint8_t mask = (uint8_t)(1u << (index % 8));
    return (uint16_t)((byte & mask) == mask);
}

/* Builds the tcp_packet_trace fields common to v4/v6 from the TCP header
 * (xdp.rs:100-111 / xdp.rs:174-185 / tc.rs:85-96 / tc.rs:137-148). */
static void fill_tcp(const uint8_t* tcp, orc_trace* t) {
    t->sport = to_be16(ld_le16(tcp + 0));
    t->dport = to_be16(ld_le16(tcp + 2));
    t->seq = to_be32(ld_le32(tcp + 4));
    t->ack = to_be32(ld_le32(tcp + 8));
    t->window = to_be16(ld_le16(tcp + 14));
    /* `tcp_hdr.urg().to_be() == 1`: urg() is a u16 0/1; to_be() of 1 is 0x0100
     * on a little-endian target, so every flag compares false. Restated
     * literally, not simplified. */
    t->flag_urg = to_be16(tcp_bit(tcp, 13)) == 1;
    t->flag_ack = to_be16(tcp_bit(tcp, 12)) == 1;
    t->flag_psh = to_be16(tcp_bit(tcp, 11)) == 1;
    t->flag_rst = to_be16(tcp_bit(tcp, 10)) == 1;
    t->flag_fin = to_be16(tcp_bit(tcp, 8)) == 1;
    t->flag_syn = to_be16(tcp_bit(tcp, 9)) == 1;
    t->checksum = to_be16(ld_le16(tcp + 16));
}

/* FILTER_PORT check, xdp.rs:89-92 / tc.rs:72-77 (host-order ports). */
static int port_filtered(const uint8_t* tcp, uint16_t filter_port) {
    return filter_port != 0 && to_be16(ld_le16(tcp + 0)) != filter_port &&
           to_be16(ld_le16(tcp + 2)) != filter_port;
}

static void v4_fill(const uint8_t* f, uint64_t ts, orc_trace* out, orc_iptuple* key) {
    const uint8_t* ip = f + ETH_HDR_LEN;
    const uint8_t* tcp = f + ETH_HDR_LEN + IP_HDR_LEN; /* IHL ignored: xdp.rs:83 */
    memset(out, 0, sizeof(*out));
    out->time = ts; /* bpf_ktime_get_ns() at xdp.rs:95 -> trace timestamp */
    out->saddr = to_be32(ld_le32(ip + 12)); /* xdp.rs:96 */
    out->daddr = to_be32(ld_le32(ip + 16)); /* xdp.rs:97 */
    fill_tcp(tcp, out);
    /* IpTuple, xdp.rs:116-127: 12 zero bytes + saddr.to_le_bytes() (= wire bytes) */
    memset(key, 0, sizeof(*key));
    memcpy(key->src_ip + 12, ip + 12, 4);
    memcpy(key->dst_ip + 12, ip + 16, 4);
    key->sport = out->sport;
    key->dport = out->dport;
    key->protocol = 6;
}

static void v6_fill(const uint8_t* f, uint64_t ts, orc_trace* out, orc_iptuple* key) {
    const uint8_t* ip6 = f + ETH_HDR_LEN;
    const uint8_t* tcp = f + ETH_HDR_LEN + IP6_HDR_LEN; /* no ext-hdr walk: xdp.rs:157 */
    memset(out, 0, sizeof(*out));
    out->time = ts;
    out->saddr = 0; /* xdp.rs:170-171 */
    out->daddr = 0;
    memcpy(out->saddr_v6, ip6 + 8, 16); /* in6_u.u6_addr8, xdp.rs:172-173 */
    memcpy(out->daddr_v6, ip6 + 24, 16);
    fill_tcp(tcp, out);
    memset(key, 0, sizeof(*key)); /* xdp.rs:189-195 */
    memcpy(key->src_ip, ip6 + 8, 16);
    memcpy(key->dst_ip, ip6 + 24, 16);
    key->sport = out->sport;
    key->dport = out->dport;
    key->protocol = 6;
}

/* xdp_hook, probes/xdp.rs:27-223 (direct packet pointers + data_end checks). */
int orc_xdp_hook(const uint8_t* f, uint32_t len, uint64_t ts, uint16_t filter_port,
                 orc_trace* out, orc_iptuple* key) {
    if (ETH_HDR_LEN > len) return 0;                          /* xdp.rs:37-39 */
    const uint16_t ethertype = to_be16(ld_le16(f + 12));      /* xdp.rs:49   */
    if (ethertype != ETHERTYPE_IPV4 && ethertype != ETHERTYPE_IPV6) return 0; /* :52 */
    if (ethertype == ETHERTYPE_IPV4) {
        if (ETH_HDR_LEN + IP_HDR_LEN > len) return 0;         /* xdp.rs:60-62 */
        if (f[ETH_HDR_LEN + 9] != TCP_PROTOCOL) return 0;     /* xdp.rs:73-75 iphdr.protocol @9 */
        if (ETH_HDR_LEN + IP_HDR_LEN + TCP_HDR_LEN > len) return 0; /* xdp.rs:78-80 */
        if (port_filtered(f + ETH_HDR_LEN + IP_HDR_LEN, filter_port)) return 0; /* :90 */
        v4_fill(f, ts, out, key);
    } else {
        if (ETH_HDR_LEN + IP6_HDR_LEN > len) return 0;        /* xdp.rs:134-136 */
        if (f[ETH_HDR_LEN + 6] != TCP_PROTOCOL) return 0;     /* xdp.rs:147 ipv6hdr.nexthdr @6 */
        if (ETH_HDR_LEN + IP6_HDR_LEN + TCP_HDR_LEN > len) return 0; /* xdp.rs:152-154 */
        if (port_filtered(f + ETH_HDR_LEN + IP6_HDR_LEN, filter_port)) return 0; /* :164 */
        v6_fill(f, ts, out, key);
    }
    return 1;
}

/* bpf_skb_load_bytes(ctx, off, .., n) fails when off + n > skb->len. */
static int skb_can_load(uint32_t len, uint32_t off, uint32_t n) { return off + n <= len; }

/* tc_hook, probes/tc.rs:28-183 (ctx.load bounds-checked loads). */
int orc_tc_hook(const uint8_t* f, uint32_t len, uint64_t ts, uint16_t filter_port,
                orc_trace* out, orc_iptuple* key) {
    if (!skb_can_load(len, 12, 2)) return 0;                  /* tc.rs:30-33 h_proto @12 */
    const uint16_t ethertype = to_be16(ld_le16(f + 12));
    uint8_t protocol;
    if (ethertype == ETHERTYPE_IPV4) {
        if (!skb_can_load(len, ETH_HDR_LEN + 9, 1)) return 0; /* tc.rs:40-42 */
        protocol = f[ETH_HDR_LEN + 9];
    } else if (ethertype == ETHERTYPE_IPV6) {
        if (!skb_can_load(len, ETH_HDR_LEN + 6, 1)) return 0; /* tc.rs:46-48 */
        protocol = f[ETH_HDR_LEN + 6];
    } else {
        return 0;                                             /* tc.rs:49-52 */
    }
    if (protocol != TCP_PROTOCOL) return 0;                   /* tc.rs:55-57 */
    if (ethertype == ETHERTYPE_IPV4) {
        if (!skb_can_load(len, ETH_HDR_LEN, IP_HDR_LEN)) return 0;              /* tc.rs:63 */
        if (!skb_can_load(len, ETH_HDR_LEN + IP_HDR_LEN, TCP_HDR_LEN)) return 0; /* :66-68 */
        if (port_filtered(f + ETH_HDR_LEN + IP_HDR_LEN, filter_port)) return 0;  /* :72-77 */
        v4_fill(f, ts, out, key);                             /* tc.rs:79-110 */
    } else {
        if (!skb_can_load(len, ETH_HDR_LEN, IP6_HDR_LEN)) return 0;             /* tc.rs:114 */
        if (!skb_can_load(len, ETH_HDR_LEN + IP6_HDR_LEN, TCP_HDR_LEN)) return 0; /* :117-119 */
        if (port_filtered(f + ETH_HDR_LEN + IP6_HDR_LEN, filter_port)) return 0; /* :123-128 */
        v6_fill(f, ts, out, key);                             /* tc.rs:131-158 */
    }
    return 1;
}

/* ---- bincode 1.3.3 legacy (fixint, little-endian) ------------------------ */
/* bincode::serialize of tcp_packet_trace (handlers/mod.rs:126): fields in
 * declaration order (tcp_header.rs:554-572), integers LE at their own width,
 * [u8; 16] as a tuple (no length prefix), bool as one byte 0/1; then the
 * marker `writer.write(&[255,255,255,255])` (handlers/mod.rs:139). */
static uint8_t* put16(uint8_t* p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); return p + 2; }
static uint8_t* put32(uint8_t* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = (uint8_t)(v >> (8 * i));
    return p + 4;
}
static uint8_t* put64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
    return p + 8;
}

void orc_serialize(const orc_trace* t, uint8_t rec[74]) {
    uint8_t* p = rec;
    p = put64(p, t->time);
    p = put32(p, t->saddr);
    p = put32(p, t->daddr);
    memcpy(p, t->saddr_v6, 16); p += 16;
    memcpy(p, t->daddr_v6, 16); p += 16;
    p = put16(p, t->sport);
    p = put16(p, t->dport);
    p = put32(p, t->seq);
    p = put32(p, t->ack);
    p = put16(p, t->window);
    *p++ = t->flag_urg ? 1 : 0;
    *p++ = t->flag_ack ? 1 : 0;
    *p++ = t->flag_psh ? 1 : 0;
    *p++ = t->flag_rst ? 1 : 0;
    *p++ = t->flag_syn ? 1 : 0;
    *p++ = t->flag_fin ? 1 : 0;
    p = put16(p, t->checksum);
    /* 70 bytes so far */
    p[0] = p[1] = p[2] = p[3] = 0xFF;
}

static uint16_t get16(const uint8_t** p) { uint16_t v = ld_le16(*p); *p += 2; return v; }
static uint32_t get32(const uint8_t** p) { uint32_t v = ld_le32(*p); *p += 4; return v; }
static uint64_t get64(const uint8_t** p) {
    uint64_t v = (uint64_t)ld_le32(*p) | ((uint64_t)ld_le32(*p + 4) << 32);
    *p += 8;
    return v;
}
static int getbool(const uint8_t** p, uint8_t* out) {
    const uint8_t b = **p;
    *p += 1;
    if (b > 1) return 0; /* bincode: InvalidBoolEncoding */
    *out = b;
    return 1;
}

/* tcp_packet.rs:31-41: bincode::deserialize::<TcpPacket>; error -> default() */
int orc_deserialize(const uint8_t rec[74], orc_packet* out) {
    orc_packet tmp;
    memset(&tmp, 0, sizeof(tmp));
    const uint8_t* p = rec;
    tmp.t.time = get64(&p);
    tmp.t.saddr = get32(&p);
    tmp.t.daddr = get32(&p);
    memcpy(tmp.t.saddr_v6, p, 16); p += 16;
    memcpy(tmp.t.daddr_v6, p, 16); p += 16;
    tmp.t.sport = get16(&p);
    tmp.t.dport = get16(&p);
    tmp.t.seq = get32(&p);
    tmp.t.ack = get32(&p);
    tmp.t.window = get16(&p);
    int ok = 1;
    ok &= getbool(&p, &tmp.t.flag_urg);
    ok &= getbool(&p, &tmp.t.flag_ack);
    ok &= getbool(&p, &tmp.t.flag_psh);
    ok &= getbool(&p, &tmp.t.flag_rst);
    ok &= getbool(&p, &tmp.t.flag_syn);
    ok &= getbool(&p, &tmp.t.flag_fin);
    tmp.t.checksum = get16(&p);
    memcpy(tmp.div, p, 4);
    if (!ok) {
        memset(out, 0, sizeof(*out)); /* TcpPacket::default() */
        return 0;
    }
    *out = tmp;
    return 1;
}

/* db_writer.rs:76-78 */
int orc_marker_ok(const orc_packet* p) {
    return p->div[0] == 0xFF && p->div[1] == 0xFF && p->div[2] == 0xFF && p->div[3] == 0xFF;
}

/* tcp_packet.rs:93-111; Ipv4Addr::from(u32) takes the u32 as big-endian octets */
void orc_get_ip_tuple(const orc_packet* p, orc_db_tuple* out) {
    memset(out, 0, sizeof(*out));
    if (p->t.saddr != 0 && p->t.daddr != 0) {
        out->is_v4 = 1;
        for (int i = 0; i < 4; ++i) {
            out->src[i] = (uint8_t)(p->t.saddr >> (24 - 8 * i));
            out->dst[i] = (uint8_t)(p->t.daddr >> (24 - 8 * i));
        }
    } else {
        out->is_v4 = 0;
        memcpy(out->src, p->t.saddr_v6, 16);
        memcpy(out->dst, p->t.daddr_v6, 16);
    }
    out->sport = p->t.sport;
    out->dport = p->t.dport;
    out->l4proto = 6;
}

/* tcp_packet.rs:46-62 (flags are Boolean(true) -> value 1) */
int orc_get_field(const orc_packet* p, int index, int64_t* value) {
    const orc_trace* t = &p->t;
    switch (index) {
        case 0: if (t->seq > 0) { *value = t->seq; return 1; } return 0;
        case 1: if (t->ack > 0) { *value = t->ack; return 1; } return 0;
        case 2: if (t->window > 0) { *value = t->window; return 1; } return 0;
        case 3: if (t->flag_urg) { *value = 1; return 1; } return 0;
        case 4: if (t->flag_ack) { *value = 1; return 1; } return 0;
        case 5: if (t->flag_psh) { *value = 1; return 1; } return 0;
        case 6: if (t->flag_rst) { *value = 1; return 1; } return 0;
        case 7: if (t->flag_syn) { *value = 1; return 1; } return 0;
        case 8: if (t->flag_fin) { *value = 1; return 1; } return 0;
        case 9: if (t->checksum > 0) { *value = t->checksum; return 1; } return 0;
        default: return 0;
    }
}

/* ---- flow hash v1 (the build's own definition; DESIGN.md "Flow hash") ---- */
void orc_key40(const orc_iptuple* k, uint8_t key40[40]) {
    memset(key40, 0, 40);
    memcpy(key40, k->src_ip, 16);
    memcpy(key40 + 16, k->dst_ip, 16);
    put16(key40 + 32, k->sport);
    put16(key40 + 34, k->dport);
    key40[36] = k->protocol;
}

static uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static uint64_t fmix64(uint64_t k) {
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdULL;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL;
    k ^= k >> 33;
    return k;
}
uint64_t orc_flow_hash64(const uint8_t key40[40]) {
    uint64_t h = 0x7CBEEULL;
    for (int i = 0; i < 5; ++i) {
        uint64_t w = 0;
        for (int b = 0; b < 8; ++b) w |= (uint64_t)key40[8 * i + b] << (8 * b);
        h ^= w * 0x87c37b91114253d5ULL;
        h = rotl64(h, 31) * 0x4cf5ad432745937fULL;
    }
    return fmix64(h ^ 40u);
}
static uint32_t fold32(uint64_t h) { return (uint32_t)(h ^ (h >> 32)); }

/* ---- exact flow table: dense ids in first-seen order -------------------- */
typedef struct orc_flow {
    uint8_t key[40];
    uint64_t pkts, bytes, first_seen;
} orc_flow;

struct orc_flowtab {
    orc_flow* flows; /* in id order */
    uint64_t n, cap_flows;
    uint64_t* slots; /* id+1, 0 = empty */
    uint64_t nslots;
};

orc_flowtab* orc_flowtab_new(uint64_t cap) {
    orc_flowtab* ft = (orc_flowtab*)calloc(1, sizeof(*ft));
    if (!ft) return NULL;
    ft->cap_flows = cap < 16 ? 16 : cap;
    ft->flows = (orc_flow*)malloc(ft->cap_flows * sizeof(orc_flow));
    ft->nslots = 32;
    while (ft->nslots < 2 * ft->cap_flows) ft->nslots <<= 1;
    ft->slots = (uint64_t*)calloc(ft->nslots, sizeof(uint64_t));
    if (!ft->flows || !ft->slots) { orc_flowtab_free(ft); return NULL; }
    return ft;
}
void orc_flowtab_free(orc_flowtab* ft) {
    if (!ft) return;
    free(ft->flows);
    free(ft->slots);
    free(ft);
}
uint64_t orc_flowtab_count(const orc_flowtab* ft) { return ft->n; }

static void ft_grow(orc_flowtab* ft) {
    const uint64_t ncap = ft->cap_flows * 2;
    ft->flows = (orc_flow*)realloc(ft->flows, ncap * sizeof(orc_flow));
    ft->cap_flows = ncap;
    free(ft->slots);
    ft->nslots <<= 1;
    ft->slots = (uint64_t*)calloc(ft->nslots, sizeof(uint64_t));
    for (uint64_t id = 0; id < ft->n; ++id) {
        uint64_t s = orc_flow_hash64(ft->flows[id].key) & (ft->nslots - 1);
        while (ft->slots[s]) s = (s + 1) & (ft->nslots - 1);
        ft->slots[s] = id + 1;
    }
}

/* returns dense id; inserts with first_seen on a miss */
static uint64_t ft_upsert(orc_flowtab* ft, const uint8_t key[40], uint64_t h,
                          uint64_t first_seen, uint32_t bytes) {
    uint64_t s = h & (ft->nslots - 1);
    for (;;) {
        const uint64_t v = ft->slots[s];
        if (!v) break;
        orc_flow* f = &ft->flows[v - 1];
        if (!memcmp(f->key, key, 40)) {
            f->pkts += 1;
            f->bytes += bytes;
            return v - 1;
        }
        s = (s + 1) & (ft->nslots - 1);
    }
    if (ft->n == ft->cap_flows) {
        ft_grow(ft);
        return ft_upsert(ft, key, h, first_seen, bytes);
    }
    const uint64_t id = ft->n++;
    memcpy(ft->flows[id].key, key, 40);
    ft->flows[id].pkts = 1;
    ft->flows[id].bytes = bytes;
    ft->flows[id].first_seen = first_seen;
    ft->slots[s] = id + 1;
    return id;
}

uint64_t orc_flowtab_export(const orc_flowtab* ft, uint8_t* out, uint64_t cap) {
    const uint64_t n = ft->n < cap ? ft->n : cap;
    for (uint64_t i = 0; i < n; ++i) {
        uint8_t* e = out + 64 * i;
        memcpy(e, ft->flows[i].key, 40);
        put64(e + 40, ft->flows[i].pkts);
        put64(e + 48, ft->flows[i].bytes);
        put64(e + 56, ft->flows[i].first_seen);
    }
    return n;
}

/* ---- batch: hook per frame, ring (= compacted output), FLOWS, counters --- */
void orc_accept_mask(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                     uint64_t n, uint16_t filter_port, int direction, uint8_t* accept) {
    for (uint64_t i = 0; i < n; ++i) {
        orc_trace t;
        orc_iptuple k;
        const uint8_t* f = arena + offset[i];
        accept[i] = (uint8_t)(direction ? orc_tc_hook(f, caplen[i], 0, filter_port, &t, &k)
                                        : orc_xdp_hook(f, caplen[i], 0, filter_port, &t, &k));
    }
}

uint64_t orc_parse_batch(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                         const uint64_t* ts, uint64_t n, uint16_t filter_port, int direction,
                         uint8_t* out_rec, uint64_t out_cap, uint32_t* out_hash,
                         uint32_t* out_id, orc_flowtab* ft, uint64_t record_base,
                         orc_counters* ctr) {
    uint64_t written = 0, accepted = 0;
    for (uint64_t i = 0; i < n; ++i) {
        orc_trace t;
        orc_iptuple k;
        const uint8_t* f = arena + offset[i];
        const int ok = direction ? orc_tc_hook(f, caplen[i], ts[i], filter_port, &t, &k)
                                 : orc_xdp_hook(f, caplen[i], ts[i], filter_port, &t, &k);
        if (!ok) continue;
        /* FLOWS insert happens before the ring reserve (xdp.rs:121 vs :204), so
         * every accepted frame is classified, written or dropped. */
        uint8_t key[40];
        orc_key40(&k, key);
        const uint64_t h = orc_flow_hash64(key);
        uint64_t id = 0;
        if (ft) id = ft_upsert(ft, key, h, record_base + accepted, caplen[i]);
        accepted++;
        /* ring reserve/submit or drop (xdp.rs:204-218) */
        if (written < out_cap) {
            orc_serialize(&t, out_rec + 74 * written);
            if (out_hash) out_hash[written] = fold32(h);
            if (out_id) out_id[written] = (uint32_t)id;
            written++;
        }
    }
    if (ctr) {
        if (direction) ctr->egress += accepted; /* try_egress_counter, tc.rs:167 */
        else ctr->ingress += accepted;          /* try_ingress_counter, xdp.rs:207 */
        ctr->handled += written;                /* xdp.rs:214 */
        ctr->dropped += accepted - written;     /* xdp.rs:217 */
    }
    return written;
}

/* ---- reference FLOWS: first MAX_FLOWS distinct tuples (flow_tracker.rs:17-23)
 * A BPF hash map with max_entries 100 rejects new keys once full; existing keys
 * update in place (BPF_ANY). */
uint64_t orc_ref_flows(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                       uint64_t n, uint16_t filter_port, int direction, uint64_t max,
                       uint8_t* out_keys) {
    uint64_t cnt = 0;
    for (uint64_t i = 0; i < n; ++i) {
        orc_trace t;
        orc_iptuple k;
        const uint8_t* f = arena + offset[i];
        const int ok = direction ? orc_tc_hook(f, caplen[i], 0, filter_port, &t, &k)
                                 : orc_xdp_hook(f, caplen[i], 0, filter_port, &t, &k);
        if (!ok) continue;
        uint8_t key[40];
        orc_key40(&k, key);
        int seen = 0;
        for (uint64_t j = 0; j < cnt && !seen; ++j) seen = !memcmp(out_keys + 40 * j, key, 40);
        if (!seen && cnt < max) memcpy(out_keys + 40 * cnt++, key, 40);
    }
    return cnt;
}

/* ---- CPU baseline: the reference record path on host threads ------------ */
typedef struct {
    const uint8_t* arena;
    const uint64_t* offset;
    const uint32_t* caplen;
    const uint64_t* ts;
    uint64_t lo, hi;
    uint16_t filter_port;
    uint8_t* out;
    uint64_t written;
} base_job;

/* One thread = one CPU running xdp_hook into a private FLOWS set (PerCpuHashMap,
 * 100 entries, flow_tracker.rs:12-13) + the drain task's bincode serialization
 * (handlers/mod.rs:104-139) into memory. */
static void* base_worker(void* arg) {
    base_job* j = (base_job*)arg;
    uint8_t keys[MAX_FLOWS][40];
    uint64_t nkeys = 0, w = 0;
    uint8_t* out = j->out + 74 * j->lo;
    for (uint64_t i = j->lo; i < j->hi; ++i) {
        orc_trace t;
        orc_iptuple k;
        if (!orc_xdp_hook(j->arena + j->offset[i], j->caplen[i], j->ts[i], j->filter_port, &t, &k))
            continue;
        uint8_t key[40];
        orc_key40(&k, key);
        int seen = 0;
        for (uint64_t q = 0; q < nkeys && !seen; ++q) seen = !memcmp(keys[q], key, 40);
        if (!seen && nkeys < MAX_FLOWS) memcpy(keys[nkeys++], key, 40);
        orc_serialize(&t, out + 74 * w);
        w++;
    }
    j->written = w;
    return NULL;
}

uint64_t orc_baseline_run(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                          const uint64_t* ts, uint64_t n, uint16_t filter_port, int threads,
                          uint8_t* out_rec) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    base_job jobs[256];
    pthread_t th[256];
    for (int t = 0; t < threads; ++t) {
        jobs[t].arena = arena;
        jobs[t].offset = offset;
        jobs[t].caplen = caplen;
        jobs[t].ts = ts;
        jobs[t].lo = n * (uint64_t)t / (uint64_t)threads;
        jobs[t].hi = n * (uint64_t)(t + 1) / (uint64_t)threads;
        jobs[t].filter_port = filter_port;
        jobs[t].out = out_rec;
        jobs[t].written = 0;
    }
    if (threads == 1) {
        base_worker(&jobs[0]);
    } else {
        for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, base_worker, &jobs[t]);
        for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    }
    uint64_t total = 0;
    for (int t = 0; t < threads; ++t) total += jobs[t].written;
    return total;
}

/* CPU-1-file baseline: one thread, xdp_hook + FLOWS(100) as above,
 * and the drain task's file path: the file opened create|append|O_NONBLOCK
 * (handlers/mod.rs:70-76), a BufWriter of size_of::<tcp_packet_trace>() x
 * WRITER_BUFFER_SIZE = 72 x 10000 B (mod.rs:86-89, config.rs:5), and per record
 * two writes into it — the 70-B bincode body, then FF FF FF FF (mod.rs:126-139)
 * — a write(2) of the buffer whenever the next piece does not fit, and a final
 * flush. Returns records written, or ~0 on an I/O error. */
static int base_put(int fd, uint8_t* buf, size_t* len, size_t cap, const uint8_t* p, size_t k) {
    if (*len + k > cap) {
        size_t off = 0;
        while (off < *len) {
            const ssize_t w = write(fd, buf + off, *len - off);
            if (w < 0) {
                if (errno == EAGAIN || errno == EINTR) continue;
                return -1;
            }
            off += (size_t)w;
        }
        *len = 0;
    }
    if (k) memcpy(buf + *len, p, k);
    *len += k;
    return 0;
}

uint64_t orc_baseline_file(const uint8_t* arena, const uint64_t* offset, const uint32_t* caplen,
                           const uint64_t* ts, uint64_t n, uint16_t filter_port,
                           const char* path) {
    enum { kCap = 72 * 10000 };
    const int fd = open(path, O_CREAT | O_WRONLY | O_APPEND | O_NONBLOCK, 0644);
    if (fd < 0) return ~0ull;
    uint8_t* buf = (uint8_t*)malloc(kCap);
    if (!buf) {
        close(fd);
        return ~0ull;
    }
    uint8_t keys[MAX_FLOWS][40];
    uint64_t nkeys = 0, w = 0;
    size_t len = 0;
    int err = 0;
    for (uint64_t i = 0; i < n && !err; ++i) {
        orc_trace t;
        orc_iptuple k;
        if (!orc_xdp_hook(arena + offset[i], caplen[i], ts[i], filter_port, &t, &k)) continue;
        uint8_t key[40];
        orc_key40(&k, key);
        int seen = 0;
        for (uint64_t q = 0; q < nkeys && !seen; ++q) seen = !memcmp(keys[q], key, 40);
        if (!seen && nkeys < MAX_FLOWS) memcpy(keys[nkeys++], key, 40);
        uint8_t rec[74];
        orc_serialize(&t, rec);  /* body [0,70) + marker [70,74) */
        err = base_put(fd, buf, &len, kCap, rec, 70) || base_put(fd, buf, &len, kCap, rec + 70, 4);
        w++;
    }
    if (!err) err = base_put(fd, buf, &len, 0, NULL, 0);  /* cap 0: flush what is left */
    free(buf);
    close(fd);
    return err ? ~0ull : w;
}

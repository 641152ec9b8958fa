"""Frame traces: the input side of the path (a NIC ring / trace file replayed).

A :class:`Trace` is the host view of ``tcbee_frames`` (include/tcbee_amd.h):
frame ``i`` is ``arena[offset[i] : offset[i] + caplen[i]]`` with timestamp
``ts_ns[i]`` (which stands in for ``bpf_ktime_get_ns()``,
tcbee-ebpf/src/probes/xdp.rs:95).

Synthetic traces follow BASELINE.json configs 2-4; the header
bytes come from the library's generator (tcbee_amd/csrc/tcbee_gen.h) so the
host and device versions of a trace are bit-identical.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib

TS_BASE_NS = 1_000_000_000
TS_STEP_NS = 1_000
IMIX_SIZES = (64, 576, 1500)  # 7 : 4 : 1
DEFAULT_SEED = 0x7CBEE

GEN_SINGLE = 0
GEN_MULTI = 1
GEN_ZIPF = 2     # config 3 "second run": flows drawn Zipf(ZIPF_S)
GEN_MULTI_V6 = 3  # GEN_MULTI's flow draw over IPv6/TCP frames (74 header bytes)
ZIPF_S = 1.1


@dataclass
class Trace:
    arena: np.ndarray   # uint8
    offset: np.ndarray  # uint64
    caplen: np.ndarray  # uint32
    ts_ns: np.ndarray   # uint64

    def __post_init__(self):
        self.arena = np.ascontiguousarray(self.arena, dtype=np.uint8)
        self.offset = np.ascontiguousarray(self.offset, dtype=np.uint64)
        self.caplen = np.ascontiguousarray(self.caplen, dtype=np.uint32)
        self.ts_ns = np.ascontiguousarray(self.ts_ns, dtype=np.uint64)
        n = len(self.offset)
        if len(self.caplen) != n or len(self.ts_ns) != n:
            raise ValueError("offset/caplen/ts_ns length mismatch")

    @property
    def n(self) -> int:
        return len(self.offset)

    def frame(self, i: int) -> bytes:
        o = int(self.offset[i])
        return self.arena[o:o + int(self.caplen[i])].tobytes()

    def slice(self, lo: int, hi: int) -> "Trace":
        """Frames [lo, hi) with a re-based, compact arena."""
        off = self.offset[lo:hi]
        ln = self.caplen[lo:hi]
        if hi <= lo:
            return Trace(np.zeros(0, np.uint8), off, ln, self.ts_ns[lo:hi])
        a0 = int(off.min())
        a1 = int((off + ln).max())
        return Trace(self.arena[a0:a1].copy(), off - np.uint64(a0), ln.copy(),
                     self.ts_ns[lo:hi].copy())

    def select(self, idx: np.ndarray) -> "Trace":
        """Frames idx (ascending), sharing this trace's arena (zero-copy: the
        offsets still point into it) — one GPU's part of a partitioned trace."""
        idx = np.asarray(idx, dtype=np.int64)
        return Trace(self.arena, self.offset[idx], self.caplen[idx], self.ts_ns[idx])

    @staticmethod
    def from_frames(frames, ts_ns=None) -> "Trace":
        """Pack a list of byte strings back to back."""
        lens = np.array([len(f) for f in frames], dtype=np.uint32)
        off = np.zeros(len(frames), dtype=np.uint64)
        if len(frames):
            off[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        arena = np.frombuffer(b"".join(frames), dtype=np.uint8).copy()
        if ts_ns is None:
            ts_ns = TS_BASE_NS + TS_STEP_NS * np.arange(len(frames), dtype=np.uint64)
        return Trace(arena, off, lens, np.asarray(ts_ns, dtype=np.uint64))


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 (== tcbee::splitmix64 in tcbee_layout.h)."""
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def synth_index(n: int, sizes: str = "64", seed: int = DEFAULT_SEED, first_index: int = 0):
    """offset/caplen/ts_ns of a synthetic trace and its arena length.

    sizes="64": every frame 64 B (config 2); sizes="imix": 64/576/1500 at 7:4:1
    drawn per frame from splitmix64(seed ^ 0x1M1X + i) % 12 (config 3/4);
    sizes="imix6": the same draw with 78/576/1500 (IPv6/TCP needs 74 bytes).
    Frames are packed back to back (no padding), as in a capture file.
    """
    i = np.arange(first_index, first_index + n, dtype=np.uint64)
    if sizes == "64":
        caplen = np.full(n, 64, dtype=np.uint32)
    elif sizes in ("imix", "imix6"):
        r = splitmix64(np.uint64(seed ^ 0x1A1E) + i) % np.uint64(12)
        small = 64 if sizes == "imix" else 78
        caplen = np.where(r < 7, small, np.where(r < 11, 576, 1500)).astype(np.uint32)
    else:
        raise ValueError(sizes)
    offset = np.zeros(n, dtype=np.uint64)
    if n:
        np.cumsum(caplen[:-1], dtype=np.uint64, out=offset[1:])
    ts = np.uint64(TS_BASE_NS) + np.uint64(TS_STEP_NS) * i
    arena_len = int(offset[-1]) + int(caplen[-1]) if n else 0
    return offset, caplen, ts, arena_len


_ZIPF_CACHE: dict = {}


def zipf_cdf(n_flows: int, s: float = ZIPF_S) -> np.ndarray:
    """CDF table of the Zipf flow mix (tcbee_gen.h kGenZipf): u64 word k ≈
    2^64 · P(flow ≤ k) with P(flow = k) ∝ (k + 1)^-s, non-decreasing, last word
    2^64 - 1. Frame i takes the first flow whose word exceeds its 64-bit draw."""
    key = (int(n_flows), float(s))
    z = _ZIPF_CACHE.get(key)
    if z is None:
        if n_flows < 1:
            raise ValueError("n_flows must be >= 1")
        p = np.arange(1, n_flows + 1, dtype=np.float64) ** -float(s)
        c = np.cumsum(p)
        c /= c[-1]
        # 2^64 - 4096: the largest float64 below 2^64 (the cast of 2^64 is undefined)
        z = np.minimum(c * 2.0 ** 64, 2.0 ** 64 - 4096.0).astype(np.uint64)
        z[-1] = np.uint64(0xFFFFFFFFFFFFFFFF)
        z.setflags(write=False)
        _ZIPF_CACHE[key] = z
    return z


def gen_frames_host(arena: np.ndarray, offset: np.ndarray, caplen: np.ndarray,
                    kind: int, n_flows: int, seed: int, first_index: int = 0) -> None:
    """Writes the header bytes of every frame into ``arena`` (payload untouched)."""
    if kind == GEN_ZIPF:
        z = zipf_cdf(n_flows)
        rc = _lib.lib().tcbee_gen_frames_zipf_host(
            arena.ctypes.data_as(C.c_void_p), offset.ctypes.data_as(C.c_void_p),
            caplen.ctypes.data_as(C.c_void_p), C.c_uint64(len(offset)),
            C.c_uint64(first_index), C.c_uint64(n_flows), C.c_uint64(seed),
            z.ctypes.data_as(C.c_void_p))
        _lib.check(rc, "tcbee_gen_frames_zipf_host")
        return
    rc = _lib.lib().tcbee_gen_frames_host(
        arena.ctypes.data_as(C.c_void_p), offset.ctypes.data_as(C.c_void_p),
        caplen.ctypes.data_as(C.c_void_p), C.c_uint64(len(offset)), C.c_uint64(first_index),
        kind, C.c_uint64(n_flows), C.c_uint64(seed))
    _lib.check(rc, "tcbee_gen_frames_host")


def synth_trace(n: int, sizes: str = "64", kind: int = GEN_SINGLE, n_flows: int = 1,
                seed: int = DEFAULT_SEED, first_index: int = 0) -> Trace:
    """A synthetic trace on the host (configs 2/3 of BASELINE.json): global frames
    [first_index, first_index + n), arena re-based to the first of them."""
    offset, caplen, ts, arena_len = synth_index(n, sizes, seed, first_index)
    arena = np.zeros(arena_len + 16, dtype=np.uint8)
    gen_frames_host(arena, offset, caplen, kind, n_flows, seed, first_index)
    return Trace(arena[:arena_len] if arena_len else arena[:0], offset, caplen, ts)


RSS_BUCKETS = 4096  # entries of the RSS indirection tables (TCBEE_RSS_MAX)


def rss_table(load, world: int) -> np.ndarray:
    """An RSS indirection table (NIC receive-side scaling: hash bucket -> GPU)
    balanced on observed per-bucket frame counts: longest-processing-time greedy
    (buckets by load, largest first, each to the least loaded GPU; ties by bucket
    and GPU number), so every rank computes the same table from the same counts.
    Every flow's frames share one bucket, so a flow still reaches exactly one GPU;
    only the mapping of buckets to GPUs is chosen. uint16[len(load)]."""
    load = np.asarray(load, dtype=np.int64)
    if world < 1 or world > 0xFFFF or load.ndim != 1 or len(load) == 0:
        raise ValueError("rss_table: 1 <= world <= 65535 and a non-empty 1-D load")
    order = np.lexsort((np.arange(len(load)), -load))  # load descending, bucket ascending
    table = np.empty(len(load), dtype=np.uint16)
    tot = [0] * world
    import heapq
    heap = [(0, g) for g in range(world)]
    for b in order:
        t, g = heapq.heappop(heap)
        table[b] = g
        tot[g] = t + int(load[b])
        heapq.heappush(heap, (tot[g], g))
    return table



def flow_hash64_np(k0, k1, k2, k3, k4) -> np.ndarray:
    """Vectorised flow hash v1 (== tcbee::flow_hash64 in tcbee_layout.h) of keys given
    as five LE u64 word arrays."""
    c1, c2 = np.uint64(0x87C37B91114253D5), np.uint64(0x4CF5AD432745937F)
    s31, s33 = np.uint64(31), np.uint64(33)
    h = np.full(np.shape(k0), 0x7CBEE, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for k in (k0, k1, k2, k3, k4):
            h ^= np.asarray(k, dtype=np.uint64) * c1
            h = ((h << s31) | (h >> s33)) * c2
        h ^= np.uint64(40)
        h ^= h >> s33
        h *= np.uint64(0xFF51AFD7ED558CCD)
        h ^= h >> s33
        h *= np.uint64(0xC4CEB9FE1A85EC53)
        h ^= h >> s33
    return h


def synth_flow_folds(n_flows: int, seed: int = DEFAULT_SEED) -> np.ndarray:
    """fold32(flow_hash64(IpTuple)) of every flow f < n_flows of the multi-flow
    synthetic trace (tcbee_gen.h gen_fields: the flow's addresses and ports from
    splitmix64((seed << 1) ^ (0xF10F10000000 + f)); the key K1 builds, xdp.rs:116-127)
    — the value a NIC's RSS (and the device shard generator, gen_fold) buckets a
    flow's frames by. uint32[n_flows]."""
    f = np.arange(n_flows, dtype=np.uint64)
    with np.errstate(over="ignore"):
        fh = splitmix64(np.uint64((seed << 1) & 0xFFFFFFFFFFFFFFFF) ^ (np.uint64(0xF10F10000000) + f))
    m24, m20 = np.uint64(0xFFFFFF), np.uint64(0xFFFFF)
    saddr = (np.uint64(0x0A000000) | (fh & m24)).astype(np.uint32)
    daddr = (np.uint64(0xAC100000) | ((fh >> np.uint64(24)) & m20)).astype(np.uint32)
    sport = np.uint64(1024) + (fh >> np.uint64(44)) % np.uint64(64000)
    dport = np.array([80, 443, 5201, 8080], dtype=np.uint64)[(fh >> np.uint64(62)).astype(np.int64)]
    k1 = saddr.byteswap().astype(np.uint64) << np.uint64(32)
    k3 = daddr.byteswap().astype(np.uint64) << np.uint64(32)
    k4 = sport | (dport << np.uint64(16)) | (np.uint64(6) << np.uint64(32))
    zero = np.zeros(n_flows, dtype=np.uint64)
    h = flow_hash64_np(zero, k1, zero, k3, k4)
    return (h ^ (h >> np.uint64(32))).astype(np.uint32)


def rss_flows_per_rank(n_flows: int, world: int, seed: int = DEFAULT_SEED,
                       table: np.ndarray | None = None) -> np.ndarray:
    """Flows each rank of a flow-hash partition holds at most (exactly, once every
    flow has appeared): flows f < n_flows routed through the RSS indirection table
    (bucket fold32 % len(table)) or, without one, the modulo placement fold32 % world.
    Known before any frame is parsed, so shard capacities come from it. int64[world]."""
    folds = synth_flow_folds(n_flows, seed)
    if table is None:
        owner = folds % np.uint32(world)
    else:
        t = np.asarray(table)
        owner = t[(folds % np.uint32(len(t))).astype(np.int64)]
    return np.bincount(owner.astype(np.int64), minlength=world).astype(np.int64)

"""Host-frames ingest pipeline over ``tcbee_pipe``.

:class:`Pipeline` streams frames that live in host memory (a pcap mapping, a
numpy trace) through the GPU record path with pinned staging and overlapped
H2D / parse / D2H (tcbee_amd/csrc/tcbee_pipe.hip). :func:`replay_pcap` is the
end-to-end replay the reference performs live: frames -> ``<dir>xdp.tcp`` /
``<dir>tc.tcp`` (BufferHandler append semantics) -> optionally the
tcbee-process SQLite database -> ``<dir>metrics.json``.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from .parser import PacketParser, _ptr
from .trace import Trace


@dataclass
class PipeResult:
    n: int
    records: np.ndarray | None   # uint8 [n, 74] when collected
    flow_id: np.ndarray | None   # uint32 [n] when collected with flows
    counters: dict = field(default_factory=dict)


class Pipeline:
    def __init__(self, device: int = 0, chunk_frames: int = 1 << 20, window: int = 64,
                 depth: int = 3, threads: int = 8, chunk_bytes: int = 0,
                 max_flows: int = 1 << 20, variants: bool = False):
        """variants=True: a pipe of the variants build (TCBEE_PIPE_* A/B settings
        read from the environment; tests of those paths only)."""
        cfg = _lib.PipeCfg(chunk_frames, chunk_bytes, window, depth, threads, 0)
        h = C.c_void_p()
        self._L = _lib.lib(variants)
        _lib.check(self._L.tcbee_pipe_create(C.byref(h), device, C.byref(cfg), max_flows),
                   "tcbee_pipe_create")
        self._h = h
        ctx = C.c_void_p()
        _lib.check(self._L.tcbee_pipe_ctx(h, C.byref(ctx)), "tcbee_pipe_ctx")
        self.parser = PacketParser._borrow(ctx, device, chunk_frames, max_flows, self._L)
        self.window = window
        self._registered = None  # (out_rec, out_id) page-locked for direct D2H
        # "registered" (direct D2H into the registered arrays) or "staged"
        # (calibrate_output chooses per box)
        self.output_mode = "staged"

    def register_output(self, out_rec, out_id=None) -> None:
        """Page-lock the caller's output arrays once (tcbee_pipe_register_output):
        later run(..., out_rec=out_rec, out_id=out_id) calls DMA each chunk's records
        and ids straight into them instead of staging + a host copy-out. The arrays
        are kept referenced while registered; register_output(None) releases them."""
        if out_rec is None:
            _lib.check(self._L.tcbee_pipe_register_output(self._h, None, 0, None),
                       "tcbee_pipe_register_output")
            self._registered = None
            self.output_mode = "staged"
            return
        if (out_rec.dtype != np.uint8 or out_rec.ndim != 2 or out_rec.shape[1] != _lib.RECORD_BYTES
                or not out_rec.flags.c_contiguous):
            raise ValueError("out_rec: a C-contiguous uint8 [n, 74] array")
        if out_id is not None and (out_id.dtype != np.uint32 or not out_id.flags.c_contiguous
                                   or len(out_id) < len(out_rec)):
            raise ValueError("out_id: a C-contiguous uint32 array of at least len(out_rec)")
        _lib.check(self._L.tcbee_pipe_register_output(self._h, _ptr(out_rec), len(out_rec),
                                                      _ptr(out_id)),
                   "tcbee_pipe_register_output")
        self._registered = (out_rec, out_id)
        self.output_mode = "registered"

    def calibrate_output(self, trace: Trace, frames: int = 4_000_000, reps: int = 2) -> dict:
        """Choose how this pipe returns records for the caller's registered arrays:
        straight into them (direct D2H) or through pinned staging + a host copy-out.
        Which is faster depends on the box's host memory (round 4: 515 vs 343 Mpkt/s on
        one box, 438 vs 452 on another), so a short calibration on a prefix of `trace`
        decides: both modes alternate (ABBA order) `reps` times over the first
        `frames` frames and the faster median is kept — the pipe stays registered, or
        releases its registration and stages. Returns the timings and the choice
        (also in self.output_mode). register_output() first.

        Side effects: the timed runs write the first `frames` records and
        ids of `trace` into the registered arrays (their previous contents are
        overwritten), and the pipe's flow table is reset before each run and once
        more at the end. A pipe that already holds flows is refused (ValueError)
        rather than silently losing its table: calibrate before the first run, or
        reset_flows() first."""
        import time
        if self._registered is None:
            raise ValueError("calibrate_output: register_output() first")
        if self.parser.flow_count():
            raise ValueError("calibrate_output: the pipe's flow table holds flows that "
                             "the calibration would reset (calibrate first, or reset_flows())")
        rec, ids = self._registered
        m = min(frames, trace.n, len(rec))
        sub = trace.slice(0, m)
        ts = {"registered": [], "staged": []}
        order = ["registered", "staged", "staged", "registered"] * reps
        for mode in order:
            if mode == "registered" and self._registered is None:
                self.register_output(rec, ids)
            elif mode == "staged" and self._registered is not None:
                self.register_output(None)
            self.reset_flows()
            t0 = time.perf_counter()
            self.run(sub, out_rec=rec[:m], out_id=None if ids is None else ids[:m])
            ts[mode].append(time.perf_counter() - t0)
        med = {k: float(np.median(v)) for k, v in ts.items()}
        self.output_mode = min(med, key=med.get)
        if self.output_mode == "registered" and self._registered is None:
            self.register_output(rec, ids)
        elif self.output_mode == "staged" and self._registered is not None:
            self.register_output(None)
        self.reset_flows()
        return {"frames": m, "reps": len(order) // 2,
                "registered_mpkts": round(m / med["registered"] / 1e6, 1),
                "staged_mpkts": round(m / med["staged"] / 1e6, 1), "chosen": self.output_mode}

    def run(self, trace: Trace, filter_port: int = 0, direction: int = _lib.DIR_INGRESS,
            flows: bool = True, collect: bool = True, sink=None, out_rec=None,
            out_id=None) -> PipeResult:
        """Parse every frame of `trace`. collect: gather records (and flow ids) into
        arrays (or into the caller's out_rec [n,74] / out_id [n]). sink(rec, ids,
        first_record): called per chunk with numpy views valid during the call."""
        n = trace.n
        rec = out_rec
        ids = out_id
        if collect and rec is None:
            rec = np.empty((max(n, 1), _lib.RECORD_BYTES), dtype=np.uint8)
        if collect and flows and ids is None:
            ids = np.empty(max(n, 1), dtype=np.uint32)
        cap = (len(rec) if rec is not None else 0)
        err = []

        def _cb(user, prec, pid, k, first):
            try:
                r = np.ctypeslib.as_array(C.cast(prec, C.POINTER(C.c_uint8)),
                                          shape=(k * _lib.RECORD_BYTES,)).reshape(k, -1) \
                    if k else np.zeros((0, _lib.RECORD_BYTES), np.uint8)
                i = (np.ctypeslib.as_array(C.cast(pid, C.POINTER(C.c_uint32)), shape=(k,))
                     if (pid and k) else None)
                sink(r, i, int(first))
                return 0
            except Exception as e:  # surfaced after the run
                err.append(e)
                return _lib.EINVAL
        cb = _lib.PIPE_SINK_FN(_cb) if sink is not None else _lib.PIPE_SINK_FN()
        fr = _lib.Frames(_ptr(trace.arena) if len(trace.arena) else 0, len(trace.arena),
                         _ptr(trace.offset), _ptr(trace.caplen), _ptr(trace.ts_ns), n)
        cfg = _lib.Cfg(filter_port, direction, 0, 0 if flows else _lib.F_NO_FLOWS)
        nout = C.c_uint64(0)
        ctr = _lib.Counters()
        rc = self._L.tcbee_pipe_run(self._h, C.byref(fr), C.byref(cfg), _ptr(rec), cap,
                                       _ptr(ids) if flows else 0, cb, None, C.byref(nout),
                                       C.byref(ctr))
        if err:
            raise err[0]
        _lib.check(rc, "tcbee_pipe_run")
        k = int(nout.value)
        return PipeResult(k, rec[:k] if rec is not None else None,
                          ids[:k] if (ids is not None and flows) else None, ctr.as_dict())

    def flows(self) -> np.ndarray:
        return self.parser.flows()

    def reset_flows(self) -> None:
        self.parser.reset_flows()

    def stats(self) -> dict:
        st = _lib.PipeStats()
        _lib.check(self._L.tcbee_pipe_get_stats(self._h, C.byref(st)), "tcbee_pipe_get_stats")
        return {k: int(getattr(st, k)) for k, _ in st._fields_}

    def close(self) -> None:
        if self._h:
            self.parser.close()
            self._L.tcbee_pipe_destroy(self._h)  # (releases a registered output too)
            self._h = None
            self._registered = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def replay_pcap(pcap_path: str, out_prefix: str, direction: int = _lib.DIR_INGRESS,
                filter_port: int = 0, db_path: str | None = None, metrics: bool = True,
                device: int = 0, window: int = 64, chunk_frames: int = 1 << 20,
                threads: int = 8) -> dict:
    """pcap -> GPU record path -> <out_prefix>xdp.tcp|tc.tcp (appended), optionally
    the tcbee-process SQLite database at db_path (records pre-grouped by the GPU's
    flow ids), and <out_prefix>metrics.json. Returns counters and sink stats."""
    from . import host
    name = "tc.tcp" if direction == _lib.DIR_EGRESS else "xdp.tcp"
    out = {}
    with host.Pcap(pcap_path) as pc, Pipeline(device=device, window=window,
                                              chunk_frames=chunk_frames,
                                              threads=threads) as pipe:
        tf = host.TcpFile(out_prefix + name)
        sk = host.Sink(db_path) if db_path else None
        try:
            def sink(rec, ids, first):
                tf.append(rec)
                if sk is not None:
                    sk.packets_grouped(rec, ids, int(ids.max()) + 1 if len(ids) else 0)
            res = pipe.run(pc.trace(), filter_port=filter_port, direction=direction,
                           flows=True, collect=False, sink=sink)
        finally:
            tf.close()
            if sk is not None:
                out["sink"] = sk.close()
        out["records"] = res.n
        out["frames"] = pc.n
        out["counters"] = res.counters
        out["flows"] = int(pipe.parser.flow_count())
    if metrics:
        host.write_metrics(out_prefix, out["counters"])
    return out

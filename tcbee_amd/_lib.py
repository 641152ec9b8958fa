"""ctypes binding of libtcbee_amd.so (the C ABI in include/tcbee_amd.h).

The shared library is built in-tree (tcbee_amd/lib/libtcbee_amd.so) by
``__graft_entry__.build()`` / ``make -C tcbee_amd/csrc``. There is no fallback:
if the library is missing, importing the product path raises.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libtcbee_amd.so")
# The variants build of the same sources (-DTCBEE_VARIANTS=1): test hooks and the
# timing-only ablations / A/B variants selected by TCBEE_* environment variables.
# Loaded only on request (PacketParser(variants=True): tests of those alternative
# paths); the product library reads no environment variable.
VARIANTS_LIB_PATH = os.path.join(_HERE, "lib", "libtcbee_amd_variants.so")
# A/B tooling only (tools/lib_ab.sh: the same workload against an older build of the
# kernels, or the variants build, in another process); the product and the tests
# load the in-tree library. The swap needs an explicit second opt-in
# (TCBEE_AB_OPTIN=1, set by the A/B scripts): a stray TCBEE_AB_LIB alone must not
# silently replace the product under a bench or a test.
AB_LIB = None
if os.environ.get("TCBEE_AB_LIB"):
    if os.environ.get("TCBEE_AB_OPTIN") != "1":
        raise ImportError("TCBEE_AB_LIB is set without TCBEE_AB_OPTIN=1: refusing to load "
                          f"{os.environ['TCBEE_AB_LIB']} in place of the product library "
                          "(A/B tooling sets both; unset TCBEE_AB_LIB otherwise)")
    AB_LIB = LIB_PATH = os.path.abspath(os.environ["TCBEE_AB_LIB"])

RECORD_BYTES = 74
TRACE_BYTES = 72
KEY_BYTES = 40
DIR_INGRESS = 0
DIR_EGRESS = 1
F_NO_FLOWS = 0x1

OK = 0
EINVAL = -1
ENOMEM = -2
EDEVICE = -3
ECAPACITY = -4
EFLOWFULL = -5
ENODEV = -6
EIO = -7
EFORMAT = -8
ESPIN = -9
EDB = -10
ESHARD = -11


class TcbeeError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _strerror(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class Cfg(C.Structure):
    _fields_ = [("filter_port", C.c_uint16), ("direction", C.c_uint8),
                ("reserved0", C.c_uint8), ("flags", C.c_uint32)]


class Frames(C.Structure):
    _fields_ = [("arena", C.c_void_p), ("arena_len", C.c_uint64),
                ("offset", C.c_void_p), ("caplen", C.c_void_p),
                ("ts_ns", C.c_void_p), ("n", C.c_uint64)]


class Counters(C.Structure):
    _fields_ = [("ingress", C.c_uint64), ("egress", C.c_uint64),
                ("handled", C.c_uint64), ("dropped", C.c_uint64)]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class FlowEntry(C.Structure):
    _fields_ = [("tuple", C.c_uint8 * KEY_BYTES), ("pkts", C.c_uint64),
                ("bytes", C.c_uint64), ("first_seen", C.c_uint64)]


EX_DEFER_IDS = 0x1
EX_ASYNC_IDS = 0x2


class ParseEx(C.Structure):
    _fields_ = [("out_frame_index", C.c_void_p), ("flags", C.c_uint32),
                ("reserved32", C.c_uint32), ("ids_stream", C.c_void_p),
                ("reserved", C.c_uint64 * 5)]


class PipeCfg(C.Structure):
    _fields_ = [("chunk_frames", C.c_uint64), ("chunk_bytes", C.c_uint64),
                ("window", C.c_uint32), ("depth", C.c_uint32), ("threads", C.c_uint32),
                ("reserved", C.c_uint32)]


class PipeStats(C.Structure):
    _fields_ = [("frames", C.c_uint64), ("records", C.c_uint64), ("chunks", C.c_uint64)]


# int (*)(void* user, const uint8_t* rec74, const uint32_t* flow_id, uint64_t n, uint64_t first)
PIPE_SINK_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64)

assert C.sizeof(Cfg) == 8 and C.sizeof(Frames) == 48 and C.sizeof(PipeCfg) == 32
assert C.sizeof(Counters) == 32 and C.sizeof(FlowEntry) == 64 and C.sizeof(ParseEx) == 64

# every symbol declared in include/tcbee_amd.h, with its ctypes signature
_SIGS = {
    "tcbee_abi_version": (C.c_int, []),
    "tcbee_strerror": (C.c_char_p, [C.c_int]),
    "tcbee_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "tcbee_ctx_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_uint64,
                                   C.c_uint64, C.c_uint64]),
    "tcbee_ctx_create_ex": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.c_uint64,
                                      C.c_uint64, C.c_uint64, C.c_uint64]),
    "tcbee_ctx_destroy": (C.c_int, [C.c_void_p]),
    "tcbee_ctx_stream": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "tcbee_ctx_sync": (C.c_int, [C.c_void_p]),
    "tcbee_parse_batch_device": (C.c_int, [C.c_void_p, C.POINTER(Frames), C.POINTER(Cfg),
                                           C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    "tcbee_parse_batch_device_ex": (C.c_int, [C.c_void_p, C.POINTER(Frames), C.POINTER(Cfg),
                                              C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p, C.POINTER(ParseEx),
                                              C.c_void_p]),
    "tcbee_parse_finish_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tcbee_flow_first_frames_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64,
                                                 C.c_void_p, C.c_void_p, C.c_void_p,
                                                 C.c_uint64, C.c_uint64, C.c_void_p]),
    "tcbee_owner_bucket_device": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "tcbee_status_raise_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                            C.c_void_p]),
    "tcbee_flow_first_seen_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                               C.c_void_p]),
    "tcbee_owner_return_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint64,
                                            C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "tcbee_owner_apply_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                           C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tcbee_global_ids_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32,
                                          C.c_uint32, C.c_uint64, C.c_void_p, C.c_uint64,
                                          C.c_void_p, C.c_void_p, C.c_void_p]),
    "tcbee_parse_batch": (C.c_int, [C.c_void_p, C.POINTER(Frames), C.POINTER(Cfg),
                                    C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                    C.POINTER(C.c_uint64), C.POINTER(Counters)]),
    "tcbee_flow_count": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64)]),
    "tcbee_flow_export": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64,
                                    C.POINTER(C.c_uint64)]),
    "tcbee_flow_reset": (C.c_int, [C.c_void_p]),
    "tcbee_flow_reset_device": (C.c_int, [C.c_void_p, C.c_void_p]),
    "tcbee_ctx_status": (C.c_int, [C.c_void_p]),
    "tcbee_flow_export_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                           C.c_void_p]),
    "tcbee_flow_merge_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64,
                                          C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "tcbee_flow_export_global_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64,
                                                  C.c_void_p, C.c_void_p, C.c_void_p,
                                                  C.c_uint64, C.c_uint64, C.c_void_p]),
    "tcbee_flow_records_before_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_void_p, C.c_uint64, C.c_void_p,
                                                   C.c_uint64, C.c_void_p]),
    "tcbee_flow_set_first_seen_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64,
                                                   C.c_void_p]),
    "tcbee_remap_ids_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_uint64, C.c_void_p]),
    "tcbee_ctx_profile": (C.c_int, [C.c_void_p, C.c_int]),
    "tcbee_ctx_count_mode": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "tcbee_ctx_profile_read": (C.c_int, [C.c_void_p, C.POINTER(C.c_double),
                                         C.POINTER(C.c_uint64)]),
    "tcbee_gen_frames_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                          C.c_uint64, C.c_int, C.c_uint64, C.c_uint64,
                                          C.c_void_p]),
    "tcbee_gen_frames_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                        C.c_uint64, C.c_int, C.c_uint64, C.c_uint64]),
    "tcbee_gen_frames_index_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_uint64, C.c_int, C.c_uint64, C.c_uint64,
                                                C.c_void_p]),
    "tcbee_gen_frames_zipf_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                               C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p,
                                               C.c_void_p]),
    "tcbee_gen_frames_zipf_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                             C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]),
    "tcbee_gen_shard_scratch": (C.c_uint64, [C.c_uint64]),
    "tcbee_gen_shard_index_device": (C.c_int, [C.c_uint64, C.c_int, C.c_int, C.c_int,
                                               C.c_uint64, C.c_uint64, C.c_int, C.c_void_p,
                                               C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                               C.c_void_p]),
    "tcbee_gen_shard_index_rss_device": (C.c_int, [C.c_uint64, C.c_int, C.c_int, C.c_int,
                                                   C.c_uint64, C.c_uint64, C.c_int, C.c_void_p,
                                                   C.c_uint32, C.c_void_p, C.c_void_p,
                                                   C.c_uint64, C.c_void_p, C.c_void_p,
                                                   C.c_void_p]),
    "tcbee_gen_rss_load_device": (C.c_int, [C.c_uint64, C.c_int, C.c_uint64, C.c_uint64,
                                            C.c_uint32, C.c_void_p, C.c_void_p]),
    "tcbee_gen_rss_load_range_device": (C.c_int, [C.c_uint64, C.c_uint64, C.c_int, C.c_uint64,
                                                  C.c_uint64, C.c_uint32, C.c_void_p,
                                                  C.c_void_p]),
    "tcbee_flow_hash64": (C.c_uint64, [C.c_void_p]),
    "tcbee_pipe_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(PipeCfg),
                                    C.c_uint64]),
    "tcbee_pipe_destroy": (C.c_int, [C.c_void_p]),
    "tcbee_pipe_register_output": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "tcbee_pipe_ctx": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "tcbee_pipe_get_stats": (C.c_int, [C.c_void_p, C.POINTER(PipeStats)]),
    "tcbee_pipe_run": (C.c_int, [C.c_void_p, C.POINTER(Frames), C.POINTER(Cfg), C.c_void_p,
                                 C.c_uint64, C.c_void_p, PIPE_SINK_FN, C.c_void_p,
                                 C.POINTER(C.c_uint64), C.POINTER(Counters)]),
}
EXPORTED = tuple(_SIGS)
# test entry points of the variants build only (not in include/tcbee_amd.h)
_VARIANT_SIGS = {
    "tcbee_test_flag_create": (C.c_int, [C.POINTER(C.c_void_p)]),
    "tcbee_test_flag_destroy": (C.c_int, [C.c_void_p]),
    "tcbee_test_wait_host_device": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                              C.c_void_p]),
    "tcbee_test_k2_hold": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "tcbee_test_host_registered": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
}

_libs: dict = {}


def lib(variants: bool = False) -> C.CDLL:
    """The loaded libtcbee_amd.so (variants=True: libtcbee_amd_variants.so). Raises
    if it has not been built."""
    path = VARIANTS_LIB_PATH if variants else LIB_PATH
    L = _libs.get(path)
    if L is None:
        if not os.path.exists(path):
            raise ImportError(
                f"{path} is missing: build it with `make -C tcbee_amd/csrc` "
                "or __graft_entry__.build() (no CPU fallback exists)")
        _share_hip_runtime_with_torch()
        L = C.CDLL(path)
        sigs = dict(_SIGS, **_VARIANT_SIGS) if variants else _SIGS
        for name, (res, args) in sigs.items():
            # (an older build under TCBEE_AB_LIB may predate some entry points)
            if (AB_LIB or variants) and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _libs[path] = L
    return L


def lib_identity(variants: bool = False) -> dict:
    """Path and sha256 prefix of the library lib(variants) loads (the bench line
    records which binary it measured)."""
    import hashlib
    path = VARIANTS_LIB_PATH if variants else LIB_PATH
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return {"lib_path": os.path.relpath(path, os.path.dirname(_HERE)) if not AB_LIB else path,
            "lib_sha256_16": h.hexdigest()[:16], "ab_lib": bool(AB_LIB)}


def _share_hip_runtime_with_torch() -> None:
    """libtcbee_amd.so needs libamdhip64.so.7, and torch-ROCm bundles its own copy
    under the same soname: only one can live in a process. If torch is installed,
    load it first so both share torch's runtime (loading /opt/rocm's first makes
    torch report "No HIP GPUs are available")."""
    if "torch" in sys.modules or os.environ.get("TCBEE_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _strerror(code: int) -> str:
    try:
        return lib().tcbee_strerror(code).decode()
    except Exception:  # library absent while formatting an error
        return f"tcbee error {code}"


def check(rc: int, what: str = "") -> None:
    if rc != OK:
        raise TcbeeError(rc, what)


def device_count() -> int:
    n = C.c_int(0)
    check(lib().tcbee_device_count(C.byref(n)), "tcbee_device_count")
    return n.value

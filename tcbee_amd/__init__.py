"""tcbee_amd — MI355X-native TCBee packet-record path.

Hot path: Eth/IPv4/IPv6/TCP fixed-offset header parse + 5-tuple flow
classification of raw frames, emitting TCBee's 74-byte ``*.tcp`` records
(see DESIGN.md). The compute runs in hand-written HIP kernels for gfx950 in
``tcbee_amd/lib/libtcbee_amd.so``, reached through the C ABI of
``include/tcbee_amd.h``.
"""
from ._lib import (DIR_EGRESS, DIR_INGRESS, EXPORTED, F_NO_FLOWS, KEY_BYTES, LIB_PATH,
                   RECORD_BYTES, TcbeeError, device_count, lib)
from .parser import (FLOW_DTYPE, PacketParser, ParseResult, flow_hash64, gen_frames_device,
                     gen_frames_index_device, gen_rss_load_device, gen_shard_index_device,
                     gen_shard_scratch_words)
from .trace import (RSS_BUCKETS, Trace, rss_flows_per_rank, rss_table, splitmix64, synth_flow_folds,
                    synth_index, synth_trace)

__all__ = [
    "DIR_EGRESS", "DIR_INGRESS", "EXPORTED", "F_NO_FLOWS", "KEY_BYTES", "LIB_PATH",
    "RECORD_BYTES", "TcbeeError", "device_count", "lib", "FLOW_DTYPE", "PacketParser",
    "ParseResult", "flow_hash64", "gen_frames_device", "gen_frames_index_device",
    "gen_rss_load_device", "gen_shard_index_device", "gen_shard_scratch_words", "RSS_BUCKETS",
    "Trace", "rss_flows_per_rank", "rss_table", "splitmix64", "synth_flow_folds", "synth_index",
    "synth_trace",
]

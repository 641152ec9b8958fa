// Shared helpers of libtcbee_host (not part of the ABI).
#pragma once
#include <cstdint>
#include <cstring>

#include "../../include/tcbee_host.h"

namespace tcbee_host {

constexpr uint64_t kRec = TCBEE_RECORD_BYTES;

inline uint16_t ld16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }
inline uint32_t ld32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return v; }
inline uint64_t ld64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return v; }

// TcpPacket::from_buffer; false (and *p zeroed) if bincode rejects the entry.
bool decode_packet(const uint8_t* rec74, tcbee_packet* p);
// db_writer.rs:76-78
bool marker_ok(const tcbee_packet& p);
// TcpPacket::get_ip_tuple with Rust's address Display
void packet_tuple(const tcbee_packet& p, tcbee_ts_tuple* t);

}  // namespace tcbee_host

// frame_codec_core.hpp -- the payload parse of Frame::read (everything after the CRC gate), written
// once for the host codec (frame_codec.cpp) and the GPU batch parse (frame_parse.hip).
//
// Restates src/frame/serial/mod.rs:694-705 (dispatch on the frame id) and read_*_payload :54-434,
// read_datagram :183-309.  A byte reader abstracts the frame: rd(i) = frame byte i (i < len).
// Only bytes the reference reads are read, in the order it checks lengths, so a rejected frame
// never reads past its end.  rd.head3(i) = bytes i, i + 1, i + 2 packed little-endian (the caller has
// checked that at least 6 bytes remain from i; a reader may read byte i + 3 with them).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/uflow_frame_codec.h"

namespace ufc_codec {

#define UFC_HD __host__ __device__ __forceinline__

constexpr uint32_t kMaxFrameSize = 1472;                  // src/lib.rs:286-294
constexpr uint32_t kSynPayload = kMaxFrameSize - 5;       // serial/mod.rs:25
constexpr uint32_t kDataPayloadHeader = 5;                // serial/mod.rs:41
constexpr uint32_t kAckPayloadHeader = 10;                // serial/mod.rs:49

template <class Rd>
UFC_HD uint32_t be32(const Rd& rd, uint32_t i) {
  return (rd(i) << 24) | (rd(i + 1) << 16) | (rd(i + 2) << 8) | rd(i + 3);
}
template <class Rd>
UFC_HD uint32_t be16(const Rd& rd, uint32_t i) {
  return (rd(i) << 8) | rd(i + 1);
}

// src/half_connection/packet_receiver/mod.rs:12-30 `datagram_is_valid` on a decoded datagram
// (CHANNEL_COUNT = MAX_CHANNELS = 64, src/lib.rs:278; MAX_FRAGMENT_SIZE, src/lib.rs:297).
UFC_HD bool datagram_is_valid(const ufc_item& d) {
  if (d.channel_id >= UFC_MAX_CHANNELS) return false;
  if (d.channel_parent_lead != 0 && (d.window_parent_lead == 0 || d.channel_parent_lead < d.window_parent_lead))
    return false;
  if (d.fragment_id > d.fragment_id_last) return false;
  if (d.fragment_id < d.fragment_id_last && d.data_len != UFC_MAX_FRAGMENT_SIZE) return false;
  if (d.data_len > UFC_MAX_FRAGMENT_SIZE) return false;
  return true;
}

// A datagram header (read_datagram, serial/mod.rs:183-309) from a header reader h(c) = byte c of
// the header: its size hs (micro 6, small 9, large 14) and payload length dl (bytes 0..2) ...
// The three bytes are read together (one dependent step per datagram in a walk, not two): the
// callers have checked that at least 6 header bytes remain.
template <class H>
UFC_HD void datagram_size(const H& h, uint32_t& hs, uint32_t& dl) {
  const uint32_t b0 = h(0), b1 = h(1), b2 = h(2);
  if ((b0 & 0x80) == 0) {  // micro (:190-229)
    hs = 6;
    dl = b0 & 0x3F;
  } else if ((b0 & 0x40) == 0) {  // small (:230-268)
    hs = 9;
    dl = b1;
  } else {  // large (:269-308)
    hs = 14;
    dl = (b1 << 8) | b2;
  }
}

// ... and its fields, once the frame is known to hold hs + dl bytes from the header on.
// data_offset is left to the caller (the header's frame offset + hs).
template <class H>
UFC_HD void decode_datagram(const H& h, uint32_t hs, ufc_item& it) {
  const uint32_t b0 = h(0);
  if (hs == 6) {  // micro
    const uint32_t b1 = h(1), b4d = h(4);
    it.channel_id = (uint8_t)(((b4d >> 2) & 0x20) | ((b0 >> 2) & 0x10) | (b1 & 0x0F));
    it.id = ((b1 & 0xF0) << 12) | (h(2) << 8) | h(3);
    it.window_parent_lead = (uint16_t)(b4d & 0x7F);
    it.channel_parent_lead = (uint16_t)h(5);
    it.form = 0;
    it.data_len = b0 & 0x3F;
  } else if (hs == 9) {  // small
    it.channel_id = (uint8_t)(b0 & 0x3F);
    it.id = ((h(2) & 0x0F) << 16) | (h(3) << 8) | h(4);
    it.window_parent_lead = (uint16_t)((h(5) << 8) | h(6));
    it.channel_parent_lead = (uint16_t)((h(7) << 8) | h(8));
    it.form = 1;
    it.data_len = h(1);
  } else {  // large
    it.channel_id = (uint8_t)(b0 & 0x3F);
    it.id = ((h(3) & 0x0F) << 16) | (h(4) << 8) | h(5);
    it.window_parent_lead = (uint16_t)((h(6) << 8) | h(7));
    it.channel_parent_lead = (uint16_t)((h(8) << 8) | h(9));
    it.fragment_id = (uint16_t)((h(10) << 8) | h(11));
    it.fragment_id_last = (uint16_t)((h(12) << 8) | h(13));
    it.form = 2;
    it.data_len = (h(1) << 8) | h(2);
  }
  it.flags = datagram_is_valid(it) ? UFC_ITEM_VALID : 0;
}

// An ack group (serial/mod.rs:395-417) from h(c) = byte c of the group.
template <class H>
UFC_HD void decode_ack_group(const H& h, ufc_item& it) {
  it.id = (h(0) << 24) | (h(1) << 16) | (h(2) << 8) | h(3);
  it.data_offset = (h(4) << 24) | (h(5) << 16) | (h(6) << 8) | h(7);  // bitfield
  it.channel_id = (uint8_t)(h(8) != 0 ? 1 : 0);
  it.form = 3;
}

// Where the items go: sink(k, item) for k < cap, when sink.on().  PtrSink: a plain array.
// kDecode false: the sink only takes each datagram header's frame offset, header(k, off).
struct PtrSink {
  static constexpr bool kDecode = true;
  ufc_item* p;
  UFC_HD bool on() const { return p != nullptr; }
  UFC_HD void operator()(uint32_t k, const ufc_item& it) const { p[k] = it; }
  UFC_HD void header(uint32_t, uint32_t) const {}
};

// Parse the payload of a frame of `len` bytes (len >= 5) whose CRC gate passed.  Fills `info`
// (kind, aux, f[], item_count) and, when the sink is on, the first `cap` items.  Returns
// whether Frame::read returns Some.
template <class Rd, class Sink>
UFC_HD bool parse_payload(const Rd& rd, uint32_t len, ufc_frame_info& info, const Sink& items, uint32_t cap) {
  const uint32_t plen = len - 5;  // payload = frame[1 .. len - 4]
  auto p = [&](uint32_t i) -> uint32_t { return rd(1 + i); };
  auto p32 = [&](uint32_t i) -> uint32_t { return be32(rd, 1 + i); };
  auto p16 = [&](uint32_t i) -> uint32_t { return be16(rd, 1 + i); };
  info.item_count = 0;
  switch (info.kind) {
    case UFC_FRAME_HANDSHAKE_SYN:  // :54-87
      if (plen != kSynPayload) return false;
      info.aux = (uint8_t)p(0);
      info.f[0] = p32(1); info.f[1] = p32(5); info.f[2] = p32(9); info.f[3] = p32(13);
      return true;
    case UFC_FRAME_HANDSHAKE_SYN_ACK:  // :89-126
      if (plen != 20) return false;
      info.f[0] = p32(0); info.f[1] = p32(4); info.f[2] = p32(8); info.f[3] = p32(12); info.f[4] = p32(16);
      return true;
    case UFC_FRAME_HANDSHAKE_ACK:  // :128-141
      if (plen != 4) return false;
      info.f[0] = p32(0);
      return true;
    case UFC_FRAME_HANDSHAKE_ERROR: {  // :143-165
      if (plen != 5) return false;
      const uint32_t e = p(4);
      if (e > 2) return false;
      info.f[0] = p32(0);
      info.aux = (uint8_t)e;
      return true;
    }
    case UFC_FRAME_DISCONNECT:      // :167-173
    case UFC_FRAME_DISCONNECT_ACK:  // :175-181
      return plen == 0;
    case UFC_FRAME_DATA: {  // :311-340
      if (plen < kDataPayloadHeader) return false;
      info.f[0] = p32(0);
      const uint32_t b4 = p(4);
      info.aux = (uint8_t)(b4 >> 7);
      const uint32_t cnt = b4 & 0x7F;
      uint32_t pos = kDataPayloadHeader;
      for (uint32_t k = 0; k < cnt; k++) {  // read_datagram, :183-309
        const uint32_t rem = plen - pos;
        if (rem < 6) return false;
        auto h = [&](uint32_t c) -> uint32_t { return p(pos + c); };
        // the header's first three bytes at once (rd.head3: one read where the reader can, so the
        // sizes of small and large datagrams do not wait on a second read after the first byte's)
        const uint32_t h3 = rd.head3(1 + pos);
        uint32_t hs, dl;
        datagram_size([&](uint32_t c) -> uint32_t { return (h3 >> (8 * c)) & 0xFFu; }, hs, dl);
        if (rem < hs + dl) return false;
        if (items.on() && k < cap) {
          if (Sink::kDecode) {
            ufc_item it{};
            decode_datagram(h, hs, it);
            it.data_offset = 1 + pos + hs;
            items(k, it);
          } else {
            items.header(k, 1 + pos);  // the header's frame offset only
          }
        }
        pos += hs + dl;
      }
      if (pos != plen) return false;  // :335-337
      info.item_count = cnt;
      return true;
    }
    case UFC_FRAME_SYNC: {  // :342-367
      if (plen != 9) return false;
      const uint32_t mode = p(0);
      info.aux = (uint8_t)(mode & 3u);
      info.f[0] = (mode & 1u) ? p32(1) : 0u;
      info.f[1] = (mode & 2u) ? p32(5) : 0u;
      return true;
    }
    case UFC_FRAME_ACK: {  // :369-434
      if (plen < kAckPayloadHeader) return false;
      const uint32_t cnt = p16(8);
      // each group needs 9 bytes (:395-397, :412-417) and nothing may remain (:425-427)
      if (plen - kAckPayloadHeader != UFC_ACK_GROUP_SIZE * cnt) return false;
      info.f[0] = p32(0);
      info.f[1] = p32(4);
      if (items.on() && Sink::kDecode) {  // (ack groups sit at fixed offsets: no header hook)
        for (uint32_t k = 0; k < cnt && k < cap; k++) {
          const uint32_t o = kAckPayloadHeader + UFC_ACK_GROUP_SIZE * k;
          ufc_item it{};
          decode_ack_group([&](uint32_t c) -> uint32_t { return p(o + c); }, it);
          items(k, it);
        }
      }
      info.item_count = cnt;
      return true;
    }
    default:
      return false;  // unknown id (:704)
  }
}

// Frame::read given the CRC gate's verdict for the frame (crc_ok = len >= 5 && trailer matches).
template <class Rd, class Sink>
UFC_HD bool read_frame_to(const Rd& rd, uint32_t len, bool crc_ok, ufc_frame_info& info, const Sink& items,
                          uint32_t cap) {
  info.kind = len >= 1 ? (uint8_t)rd(0) : (uint8_t)0xFF;
  info.ok = 0;
  info.aux = 0;
  info.crc_ok = (crc_ok && len >= 5) ? 1 : 0;
  for (int i = 0; i < 5; i++) info.f[i] = 0;
  info.item_count = 0;
  if (!info.crc_ok) return false;
  const bool ok = parse_payload(rd, len, info, items, cap);
  if (!ok) info.item_count = 0;
  info.ok = ok ? 1 : 0;
  return ok;
}

template <class Rd>
UFC_HD bool read_frame(const Rd& rd, uint32_t len, bool crc_ok, ufc_frame_info& info, ufc_item* items,
                       uint32_t cap) {
  return read_frame_to(rd, len, crc_ok, info, PtrSink{items}, cap);
}

}  // namespace ufc_codec

// frame_codec.cpp -- host side of uflow's frame codec (include/uflow_frame_codec.h): Frame::read,
// the fixed-size writers, DataFrameBuilder / AckFrameBuilder, and the batched host parse that
// follows the batched CRC gate.  The payload parse is frame_codec_core.hpp (shared with the GPU).
#include <algorithm>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/uflow_frame_codec.h"
#include "crc_math.hpp"
#include "frame_codec_core.hpp"

namespace {

struct HostBytes {
  const uint8_t* p;
  uint32_t operator()(uint32_t i) const { return p[i]; }
  uint32_t head3(uint32_t i) const { return p[i] | (p[i + 1] << 8) | ((uint32_t)p[i + 2] << 16); }
};

inline void put32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

inline bool crc_gate(const uint8_t* f, size_t len) {  // serial/mod.rs:676-690
  if (len < 5) return false;
  const uint32_t rx = ((uint32_t)f[len - 4] << 24) | ((uint32_t)f[len - 3] << 16) | ((uint32_t)f[len - 2] << 8) |
                      (uint32_t)f[len - 1];
  return ufc::host_extend(0u, f, len - 4) == rx;
}

// Trailer: BE32 CRC of everything before it (serial/mod.rs:463-470, build.rs:151-159), or zeros
// for a later batched seal.
inline void trailer(uint8_t* f, size_t body, int seal) {
  put32(f + body, seal ? ufc::host_extend(0u, f, body) : 0u);
}

constexpr uint32_t kPacketIdMask = (1u << 20) - 1;  // src/packet_id.rs

}  // namespace

extern "C" {

int ufc_frame_read(const uint8_t* frame, size_t len, ufc_frame_info* info, ufc_item* items, size_t items_cap) {
  if (!info || (!frame && len)) return UFC_ERR_INVALID_ARG;
  if (len > 0xFFFFFFFFu) len = 0xFFFFFFFFu;
  const bool gate = frame && crc_gate(frame, len);
  const bool ok = ufc_codec::read_frame(HostBytes{frame}, (uint32_t)len, gate, *info, items,
                                        (uint32_t)std::min<size_t>(items_cap, 0xFFFFFFFFu));
  info->item_first = 0;
  if (ok && info->item_count > items_cap && items) return UFC_ERR_NOMEM;
  return ok ? 1 : 0;
}

int ufc_frame_parse(const uint8_t* frame, size_t len, int crc_ok, ufc_frame_info* info, ufc_item* items,
                    size_t items_cap) {
  if (!info || (!frame && len)) return UFC_ERR_INVALID_ARG;
  if (len > 0xFFFFFFFFu) len = 0xFFFFFFFFu;
  const bool ok = ufc_codec::read_frame(HostBytes{frame}, (uint32_t)len, crc_ok != 0 && frame, *info, items,
                                        (uint32_t)std::min<size_t>(items_cap, 0xFFFFFFFFu));
  info->item_first = 0;
  if (ok && info->item_count > items_cap && items) return UFC_ERR_NOMEM;
  return ok ? 1 : 0;
}

int ufc_datagram_is_valid(const ufc_item* datagram) {  // packet_receiver/mod.rs:12-30
  if (!datagram) return UFC_ERR_INVALID_ARG;
  return ufc_codec::datagram_is_valid(*datagram) ? 1 : 0;
}

size_t ufc_frame_write_fixed(const ufc_frame_info* info, uint8_t* out, size_t cap, int seal) {
  if (!info || !out) return 0;
  size_t len;
  switch (info->kind) {
    case UFC_FRAME_HANDSHAKE_SYN: len = ufc_codec::kMaxFrameSize; break;  // :437-473, zero-padded
    case UFC_FRAME_HANDSHAKE_SYN_ACK: len = 25; break;                   // :475-514
    case UFC_FRAME_HANDSHAKE_ACK: len = 9; break;                        // :516-539
    case UFC_FRAME_HANDSHAKE_ERROR: len = 10; break;                     // :541-569
    case UFC_FRAME_DISCONNECT:                                           // :571-590
    case UFC_FRAME_DISCONNECT_ACK: len = 5; break;                       // :592-611
    case UFC_FRAME_SYNC: len = 14; break;                                // :623-657
    default: return 0;
  }
  if (cap < len) return 0;
  std::memset(out, 0, len);
  out[0] = info->kind;
  switch (info->kind) {
    case UFC_FRAME_HANDSHAKE_SYN:
      out[1] = info->aux;
      for (int i = 0; i < 4; i++) put32(out + 2 + 4 * i, info->f[i]);
      break;
    case UFC_FRAME_HANDSHAKE_SYN_ACK:
      for (int i = 0; i < 5; i++) put32(out + 1 + 4 * i, info->f[i]);
      break;
    case UFC_FRAME_HANDSHAKE_ACK:
      put32(out + 1, info->f[0]);
      break;
    case UFC_FRAME_HANDSHAKE_ERROR:
      if (info->aux > 2) return 0;  // HandshakeErrorType has three values (:551-555)
      put32(out + 1, info->f[0]);
      out[5] = info->aux;
      break;
    case UFC_FRAME_SYNC: {
      const uint8_t mode = info->aux & 3u;
      out[1] = mode;
      put32(out + 2, (mode & 1u) ? info->f[0] : 0u);
      put32(out + 6, (mode & 2u) ? info->f[1] : 0u);
      break;
    }
    default:
      break;
  }
  trailer(out, len - 4, seal);
  return len;
}

// ---- DataFrameBuilder (build.rs:47-181) ----
int ufc_data_frame_builder_init(ufc_builder* b, uint8_t* buf, size_t cap, uint32_t sequence_id, int nonce) {
  if (!b || !buf || cap < 6 + 4) return UFC_ERR_INVALID_ARG;
  b->buf = buf;
  b->cap = cap;
  buf[0] = UFC_FRAME_DATA;  // :56-66
  put32(buf + 1, sequence_id);
  buf[5] = (uint8_t)((nonce ? 1 : 0) << 7);
  b->len = 6;
  b->count = 0;
  b->kind = UFC_FRAME_DATA;
  return UFC_OK;
}

size_t ufc_data_frame_encoded_size(const ufc_datagram_ref* d) {  // :173-181
  if (!d) return 0;
  if (d->fragment_id_last == 0) {
    if (d->data_len < 64 && d->window_parent_lead < 128 && d->channel_parent_lead < 256) return 6 + d->data_len;
    if (d->data_len < 256) return 9 + d->data_len;
  }
  return 14 + d->data_len;
}

int ufc_data_frame_builder_add(ufc_builder* b, const ufc_datagram_ref* d) {
  if (!b || !d || b->kind != UFC_FRAME_DATA) return UFC_ERR_INVALID_ARG;
  // build.rs:74-77 (debug_assert!): channel, 20-bit sequence id, u16 length, count limit
  if (d->channel_id >= UFC_MAX_CHANNELS || d->sequence_id > kPacketIdMask || d->data_len > 0xFFFF ||
      b->count >= UFC_DATA_FRAME_MAX_DATAGRAM_COUNT || (d->data_len && !d->data))
    return UFC_ERR_INVALID_ARG;
  if (d->fragment_id_last == 0 && d->fragment_id != 0) return UFC_ERR_INVALID_ARG;  // :82
  const size_t need = ufc_data_frame_encoded_size(d);
  if (b->len + need + 4 > b->cap) return UFC_ERR_INVALID_ARG;
  uint8_t* h = b->buf + b->len;
  const uint32_t dl = (uint32_t)d->data_len, ch = d->channel_id, seq = d->sequence_id;
  const size_t hs = need - d->data_len;  // header form chosen as in :80-121
  if (hs == 6) {  // micro, :84-100
    h[0] = (uint8_t)(dl | ((ch & 0x10) << 2));
    h[1] = (uint8_t)(((seq >> 12) & 0xF0) | (ch & 0x0F));
    h[2] = (uint8_t)(seq >> 8);
    h[3] = (uint8_t)seq;
    h[4] = (uint8_t)(d->window_parent_lead | ((ch & 0x20) << 2));
    h[5] = (uint8_t)d->channel_parent_lead;
  } else if (hs == 9) {  // small, :101-119
    h[0] = (uint8_t)(ch | 0x80);
    h[1] = (uint8_t)dl;
    h[2] = (uint8_t)(seq >> 16);
    h[3] = (uint8_t)(seq >> 8);
    h[4] = (uint8_t)seq;
    h[5] = (uint8_t)(d->window_parent_lead >> 8);
    h[6] = (uint8_t)d->window_parent_lead;
    h[7] = (uint8_t)(d->channel_parent_lead >> 8);
    h[8] = (uint8_t)d->channel_parent_lead;
  } else {  // large, :123-143
    h[0] = (uint8_t)(ch | 0xC0);
    h[1] = (uint8_t)(dl >> 8);
    h[2] = (uint8_t)dl;
    h[3] = (uint8_t)(seq >> 16);
    h[4] = (uint8_t)(seq >> 8);
    h[5] = (uint8_t)seq;
    h[6] = (uint8_t)(d->window_parent_lead >> 8);
    h[7] = (uint8_t)d->window_parent_lead;
    h[8] = (uint8_t)(d->channel_parent_lead >> 8);
    h[9] = (uint8_t)d->channel_parent_lead;
    h[10] = (uint8_t)(d->fragment_id >> 8);
    h[11] = (uint8_t)d->fragment_id;
    h[12] = (uint8_t)(d->fragment_id_last >> 8);
    h[13] = (uint8_t)d->fragment_id_last;
  }
  if (dl) std::memcpy(h + hs, d->data, dl);
  b->len += hs + dl;
  b->count++;
  return UFC_OK;
}

// ---- AckFrameBuilder (build.rs:183-256) ----
int ufc_ack_frame_builder_init(ufc_builder* b, uint8_t* buf, size_t cap, uint32_t frame_window_base_id,
                               uint32_t packet_window_base_id) {
  if (!b || !buf || cap < 11 + 4) return UFC_ERR_INVALID_ARG;
  b->buf = buf;
  b->cap = cap;
  buf[0] = UFC_FRAME_ACK;  // :189-205
  put32(buf + 1, frame_window_base_id);
  put32(buf + 5, packet_window_base_id);
  buf[9] = buf[10] = 0;
  b->len = 11;
  b->count = 0;
  b->kind = UFC_FRAME_ACK;
  return UFC_OK;
}

int ufc_ack_frame_builder_add(ufc_builder* b, uint32_t base_id, uint32_t bitfield, int nonce) {
  if (!b || b->kind != UFC_FRAME_ACK || b->count >= 0xFFFF || b->len + 9 + 4 > b->cap) return UFC_ERR_INVALID_ARG;
  uint8_t* h = b->buf + b->len;  // :213-228
  put32(h, base_id);
  put32(h + 4, bitfield);
  h[8] = (uint8_t)(nonce ? 1 : 0);
  b->len += 9;
  b->count++;
  return UFC_OK;
}

size_t ufc_builder_size(const ufc_builder* b) { return b ? b->len + 4 : 0; }

size_t ufc_builder_build(ufc_builder* b, int seal) {
  if (!b || !b->buf || b->len + 4 > b->cap) return 0;
  if (b->kind == UFC_FRAME_DATA) {
    b->buf[5] |= (uint8_t)b->count;  // :148-149
  } else if (b->kind == UFC_FRAME_ACK) {
    b->buf[9] = (uint8_t)(b->count >> 8);  // :231-234
    b->buf[10] = (uint8_t)b->count;
  } else {
    return 0;
  }
  trailer(b->buf, b->len, seal);
  return b->len + 4;
}

// ---- batched host parse ----
int ufc_parse_batch_host(const uint8_t* bytes, const uint64_t* offsets, size_t n, const uint8_t* valid,
                         ufc_frame_info* infos, ufc_item* items, size_t items_cap, size_t* items_used,
                         int nthreads) {
  if (items_used) *items_used = 0;
  if (n == 0) return UFC_OK;
  if (!bytes || !offsets || !infos) return UFC_ERR_INVALID_ARG;
  for (size_t i = 0; i < n; i++)
    if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 0xFFFFFFFFull) return UFC_ERR_INVALID_ARG;
  int T = nthreads > 0 ? nthreads : 1;
  T = (int)std::min<size_t>((size_t)T, (n + 1023) / 1024);
  if (T < 1) T = 1;
  // Pass 1 (parallel over contiguous frame ranges): gate + parse into infos, count items.
  std::vector<uint64_t> part(T + 1, 0);
  auto pass1 = [&](int t) {
    const size_t a = n * t / T, b = n * (t + 1) / T;
    uint64_t c = 0;
    for (size_t i = a; i < b; i++) {
      const uint8_t* f = bytes + offsets[i];
      const size_t len = (size_t)(offsets[i + 1] - offsets[i]);
      const bool gate = valid ? valid[i] != 0 : crc_gate(f, len);
      ufc_codec::read_frame(HostBytes{f}, (uint32_t)len, gate, infos[i], nullptr, 0);
      infos[i].item_first = (uint32_t)c;  // local, rebased in pass 2
      c += infos[i].item_count;
    }
    part[t + 1] = c;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(pass1, t);
  pass1(0);
  for (auto& x : th) x.join();
  th.clear();
  for (int t = 0; t < T; t++) part[t + 1] += part[t];
  const uint64_t total = part[T];
  if (items_used) *items_used = (size_t)total;
  const bool fill = items && total <= items_cap;
  // Pass 2: global item indices, items written by re-parsing accepted frames.
  auto pass2 = [&](int t) {
    const size_t a = n * t / T, b = n * (t + 1) / T;
    for (size_t i = a; i < b; i++) {
      const uint64_t first = part[t] + infos[i].item_first;
      infos[i].item_first = (uint32_t)first;
      if (fill && infos[i].ok && infos[i].item_count) {
        ufc_frame_info tmp;
        const uint8_t* f = bytes + offsets[i];
        ufc_codec::read_frame(HostBytes{f}, (uint32_t)(offsets[i + 1] - offsets[i]), true, tmp, items + first,
                              infos[i].item_count);
      }
    }
  };
  for (int t = 1; t < T; t++) th.emplace_back(pass2, t);
  pass2(0);
  for (auto& x : th) x.join();
  return (items && !fill) ? UFC_ERR_NOMEM : UFC_OK;
}

}  // extern "C"

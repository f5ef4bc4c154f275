/*
 * uflow_frame_codec.h -- C ABI of libuflowcrc.so for uflow's frame codec around the CRC gate:
 * the rest of Frame::read (type dispatch and payload parse), the frame writers and builders, and
 * batched parses that consume the batched CRC gate's valid flags.
 *
 * Reference (lowquark/uflow v0.7.1, Rust) interfaces each entry point replaces:
 *   ufc_frame_read             <- src/frame/serial/mod.rs:674-706  `Frame::read` (Serialize::read), with
 *                                 read_*_payload :54-434 and read_datagram :183-309
 *   ufc_frame_write_fixed      <- src/frame/serial/mod.rs:437-611, 623-657  write_handshake_*,
 *                                 write_disconnect[_ack], write_sync
 *   ufc_data_frame_builder_*   <- src/frame/serial/build.rs:47-181  DataFrameBuilder::{new, add, build,
 *                                 count, size, encoded_size}
 *   ufc_ack_frame_builder_*    <- src/frame/serial/build.rs:183-256  AckFrameBuilder::{new, add, build, size}
 *   ufc_parse_batch_host       <- the receive loops' Frame::read of every datagram (src/server/mod.rs:
 *                                 591-602, src/client/mod.rs:615-623), after the batched CRC gate
 *   ufc_parse_batch_varlen     <- the same parse on the GPU, device-resident frames
 *   ufc_datagram_is_valid, UFC_ITEM_VALID
 *                              <- src/half_connection/packet_receiver/mod.rs:12-30 `datagram_is_valid`,
 *                                 applied by handle_datagram (:147-150) to every received datagram
 *
 * Conventions: as uflow_frame_crc.h.  A frame the reference would reject is data (ok = 0), never
 * an error; nothing is allocated per call except where stated (the device parse's scan scratch
 * grows inside the context).  Decoded datagrams point into the frame (data_offset, data_len);
 * nothing is copied.
 */
#ifndef UFLOW_FRAME_CODEC_H
#define UFLOW_FRAME_CODEC_H

#include <stddef.h>
#include <stdint.h>

#include "uflow_frame_crc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Frame ids (src/frame/serial/mod.rs:15-23). */
#define UFC_FRAME_HANDSHAKE_SYN 0
#define UFC_FRAME_HANDSHAKE_SYN_ACK 1
#define UFC_FRAME_HANDSHAKE_ACK 2
#define UFC_FRAME_HANDSHAKE_ERROR 3
#define UFC_FRAME_DISCONNECT 4
#define UFC_FRAME_DISCONNECT_ACK 5
#define UFC_FRAME_DATA 10
#define UFC_FRAME_SYNC 11
#define UFC_FRAME_ACK 12
/* Wire constants (src/frame/serial/mod.rs:25-44). */
#define UFC_DATA_FRAME_MAX_DATAGRAM_COUNT 127
#define UFC_ACK_GROUP_SIZE 9
#define UFC_MAX_CHANNELS 64

/* One decoded frame (32 bytes).  Fields by kind (f[] in wire order):
 *   handshake_syn      aux = version; f = nonce, max_receive_rate, max_packet_size, max_receive_alloc
 *   handshake_syn_ack  f = nonce_ack, nonce, max_receive_rate, max_packet_size, max_receive_alloc
 *   handshake_ack      f = nonce_ack
 *   handshake_error    f = nonce_ack; aux = error (0 Version, 1 Config, 2 ServerFull)
 *   disconnect[_ack]   -
 *   data               f = sequence_id; aux = nonce (0/1); item_count = datagrams
 *   sync               aux = mode (bit 0: next_frame_id present, bit 1: next_packet_id present);
 *                      f = next_frame_id, next_packet_id (0 when absent)
 *   ack                f = frame_window_base_id, packet_window_base_id; item_count = ack groups
 * ok = 1 exactly when Frame::read returns Some; with ok = 0 the other fields are unspecified
 * except kind (byte 0 of the frame, or 0xFF for frames shorter than 1 byte). */
typedef struct ufc_frame_info {
  uint8_t kind;
  uint8_t ok;
  uint8_t aux;
  uint8_t crc_ok;      /* the CRC gate alone (len >= 5 and the trailer matches) */
  uint32_t f[5];
  uint32_t item_count;
  uint32_t item_first; /* batched parses: index of the frame's first item in the item array */
} ufc_frame_info;

/* One datagram of a data frame, or one ack group of an ack frame (24 bytes). */
typedef struct ufc_item {
  uint32_t id;                  /* datagram: sequence_id; ack group: base_id */
  uint8_t channel_id;           /* datagram: channel_id; ack group: nonce (0/1) */
  uint8_t form;                 /* datagram header: 0 micro, 1 small, 2 large; 3 = ack group */
  uint16_t window_parent_lead;
  uint16_t channel_parent_lead;
  uint16_t fragment_id;
  uint16_t fragment_id_last;
  uint16_t flags;               /* datagram: UFC_ITEM_VALID if datagram_is_valid (below); ack group: 0 */
  uint32_t data_offset;         /* datagram: payload offset in the frame; ack group: bitfield */
  uint32_t data_len;            /* datagram: payload bytes; ack group: 0 */
} ufc_item;

/* ufc_item.flags bit: the datagram passes the receive side's content check,
 * src/half_connection/packet_receiver/mod.rs:12-30 `datagram_is_valid` (channel < 64; a nonzero
 * channel_parent_lead needs window_parent_lead != 0 and channel_parent_lead >= window_parent_lead;
 * fragment_id <= fragment_id_last; every fragment but the last exactly UFC_MAX_FRAGMENT_SIZE bytes;
 * no payload over UFC_MAX_FRAGMENT_SIZE).  handle_datagram (:147-150) drops datagrams without it. */
#define UFC_ITEM_VALID 1
/* MAX_FRAGMENT_SIZE = MAX_FRAME_SIZE - DATA_FRAME_OVERHEAD - MAX_DATAGRAM_OVERHEAD (src/lib.rs:297). */
#define UFC_MAX_FRAGMENT_SIZE 1448

/* ---- scalar host entry points ---- */
/* Frame::read: 1 = Some, 0 = None.  info is always written; up to items_cap items are written
 * (info->item_count says how many the frame holds; UFC_ERR_NOMEM if items_cap is smaller). */
int ufc_frame_read(const uint8_t* frame, size_t len, ufc_frame_info* info, ufc_item* items, size_t items_cap);

/* The rest of Frame::read after an external CRC gate (e.g. the batched GPU gate): crc_ok is the
 * gate's verdict for this frame.  Returns and fills as ufc_frame_read. */
int ufc_frame_parse(const uint8_t* frame, size_t len, int crc_ok, ufc_frame_info* info, ufc_item* items,
                    size_t items_cap);

/* datagram_is_valid (src/half_connection/packet_receiver/mod.rs:12-30) of a decoded datagram
 * (form 0..2): 1 valid, 0 not (the parses store the same verdict in flags & UFC_ITEM_VALID). */
int ufc_datagram_is_valid(const ufc_item* datagram);

/* Fixed-size frames (every kind but data and ack) from info; writes the BE32 CRC trailer when
 * seal != 0, else 4 zero bytes (for a batched seal on the GPU).  Returns the frame length, 0 if
 * cap is too small or the kind is data/ack/unknown. */
size_t ufc_frame_write_fixed(const ufc_frame_info* info, uint8_t* out, size_t cap, int seal);

/* Builders over a caller-owned buffer. */
typedef struct ufc_builder {
  uint8_t* buf;
  size_t cap;
  size_t len;      /* bytes written so far (header + items, no trailer) */
  uint32_t count;  /* datagrams or ack groups added */
  uint32_t kind;   /* UFC_FRAME_DATA or UFC_FRAME_ACK */
} ufc_builder;

typedef struct ufc_datagram_ref {
  uint32_t sequence_id;
  uint8_t channel_id;
  uint8_t reserved;
  uint16_t window_parent_lead;
  uint16_t channel_parent_lead;
  uint16_t fragment_id;
  uint16_t fragment_id_last;
  const uint8_t* data;
  size_t data_len;
} ufc_datagram_ref;

int ufc_data_frame_builder_init(ufc_builder* b, uint8_t* buf, size_t cap, uint32_t sequence_id, int nonce);
/* UFC_ERR_INVALID_ARG for what build.rs debug_asserts (channel >= 64, sequence id >= 2^20,
 * data > 65535 B, already 127 datagrams) and when the buffer would overflow (trailer included). */
int ufc_data_frame_builder_add(ufc_builder* b, const ufc_datagram_ref* d);
size_t ufc_data_frame_encoded_size(const ufc_datagram_ref* d);
int ufc_ack_frame_builder_init(ufc_builder* b, uint8_t* buf, size_t cap, uint32_t frame_window_base_id,
                               uint32_t packet_window_base_id);
int ufc_ack_frame_builder_add(ufc_builder* b, uint32_t base_id, uint32_t bitfield, int nonce);
/* Frame size once built: len + 4 (build.rs:169-171, 249-251). */
size_t ufc_builder_size(const ufc_builder* b);
/* Patches the count (build.rs:148-149 / 231-234) and appends the trailer: BE32 CRC if seal != 0,
 * else 4 zero bytes.  Returns the frame length. */
size_t ufc_builder_build(ufc_builder* b, int seal);

/* ---- batched parses (CSR batch: frame i = bytes[offsets[i] .. offsets[i+1])) ----
 * valid: the batched CRC gate's flags (ufc_crc_batch_varlen / ufc_validate_host_varlen); NULL =
 * check the CRC here.  infos[n]; items in frame order, infos[i].item_first the first of frame i;
 * *items_used = total items of accepted frames (items of rejected frames are not emitted); if it
 * exceeds items_cap only infos are complete and UFC_ERR_NOMEM is returned. */
int ufc_parse_batch_host(const uint8_t* bytes, const uint64_t* offsets, size_t n, const uint8_t* valid,
                         ufc_frame_info* infos, ufc_item* items, size_t items_cap, size_t* items_used,
                         int nthreads);
/* Device-resident, asynchronous on `stream`: d_valid is required (the gate's output), d_items_used
 * is one device word.  Items beyond items_cap are dropped (compare *d_items_used with the cap). */
int ufc_parse_batch_varlen(ufc_ctx* ctx, const uint8_t* d_bytes, const uint64_t* d_offsets, size_t n,
                           const uint8_t* d_valid, ufc_frame_info* d_infos, ufc_item* d_items, size_t items_cap,
                           uint64_t* d_items_used, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* UFLOW_FRAME_CODEC_H */

"""Expected outputs of the batched parse (ufc_parse_batch_varlen / ufc_parse_batch_host) built from the
codec oracle alone (test infrastructure, not a test module).

`oracle_records(frames)` decodes each frame with oracle/codec.py `frame_read` (serial/mod.rs:675-706;
datagram_is_valid of packet_receiver/mod.rs:12-30) and lays the result out as the C ABI's records
(include/uflow_frame_codec.h: ufc_frame_info, ufc_item).  `tile_records` expands the records of a few
distinct frames to a batch that repeats them, so a million-frame GPU parse is compared with the oracle
without decoding a million frames in Python (the full-size parse pinned to the oracle,
not to the product's own host parse).
"""
import numpy as np

import oracle
from oracle import codec as C
from uflow_amd.frame import FRAME_INFO_DTYPE, ITEM_DTYPE

ITEM_VALID = 1   # UFC_ITEM_VALID
FORM_ACK = 3     # ufc_item.form of an ack group


def _info_of(fb, ref, crc_ok):
    info = np.zeros(1, dtype=FRAME_INFO_DTYPE)[0]
    info["kind"] = fb[0] if len(fb) >= 1 else 0xFF
    info["crc_ok"] = 1 if crc_ok else 0
    items = []
    if ref is None:
        return info, items
    info["ok"] = 1
    k, f = ref["kind"], [0] * 5
    if k == "handshake_syn":
        info["aux"] = ref["version"]
        f[:4] = [ref["nonce"], ref["max_receive_rate"], ref["max_packet_size"], ref["max_receive_alloc"]]
    elif k == "handshake_syn_ack":
        f = [ref["nonce_ack"], ref["nonce"], ref["max_receive_rate"], ref["max_packet_size"], ref["max_receive_alloc"]]
    elif k == "handshake_ack":
        f[0] = ref["nonce_ack"]
    elif k == "handshake_error":
        f[0] = ref["nonce_ack"]
        info["aux"] = C.ERRORS.index(ref["error"])
    elif k == "data":
        f[0] = ref["sequence_id"]
        info["aux"] = 1 if ref["nonce"] else 0
        for dg in ref["datagrams"]:
            it = np.zeros(1, dtype=ITEM_DTYPE)[0]
            it["id"], it["channel_id"], it["form"] = dg["sequence_id"], dg["channel_id"], dg["header"]
            it["window_parent_lead"], it["channel_parent_lead"] = dg["window_parent_lead"], dg["channel_parent_lead"]
            it["fragment_id"], it["fragment_id_last"] = dg["fragment_id"], dg["fragment_id_last"]
            it["flags"] = ITEM_VALID if C.datagram_is_valid(dg) else 0
            it["data_offset"], it["data_len"] = dg["data_offset"], dg["data_len"]
            items.append(it)
    elif k == "sync":
        info["aux"] = (1 if ref["next_frame_id"] is not None else 0) | (2 if ref["next_packet_id"] is not None else 0)
        f[0] = ref["next_frame_id"] or 0
        f[1] = ref["next_packet_id"] or 0
    elif k == "ack":
        f[:2] = [ref["frame_window_base_id"], ref["packet_window_base_id"]]
        for g in ref["frame_acks"]:
            it = np.zeros(1, dtype=ITEM_DTYPE)[0]
            it["id"], it["channel_id"], it["form"], it["data_offset"] = g["base_id"], 1 if g["nonce"] else 0, FORM_ACK, \
                g["bitfield"]
            items.append(it)
    info["f"] = f
    info["item_count"] = len(items)
    return info, items


def oracle_records(frames):
    """(infos, items) of a batch of frames (bytes each) as the C ABI lays them out, from the oracle."""
    infos = np.zeros(len(frames), dtype=FRAME_INFO_DTYPE)
    items = []
    first = 0
    for i, fb in enumerate(frames):
        fb = bytes(fb)
        info, its = _info_of(fb, C.frame_read(fb), oracle.frame_validate(fb)[0] and len(fb) >= 5)
        info["item_first"] = first
        infos[i] = info
        items.extend(its)
        first += len(its)
    return infos, (np.array(items, dtype=ITEM_DTYPE) if items else np.zeros(0, ITEM_DTYPE))


def tile_records(base_infos, base_items, tile, dead):
    """Records of a batch whose frame i is base frame tile[i], except frames with dead[i] set (a bit
    flipped: the CRC gate fails, Frame::read returns None, no items)."""
    cnt = base_infos["item_count"].astype(np.int64)
    bfirst = base_infos["item_first"].astype(np.int64)
    infos = base_infos[tile].copy()
    if dead.any():
        d = infos[dead]
        d["ok"] = 0
        d["crc_ok"] = 0
        d["aux"] = 0
        d["f"] = 0
        d["item_count"] = 0
        infos[dead] = d
    n_items = np.where(dead, 0, cnt[tile])
    first = np.zeros(tile.size, dtype=np.int64)
    first[1:] = np.cumsum(n_items)[:-1]
    infos["item_first"] = first.astype(np.uint32)
    total = int(n_items.sum())
    # item j of frame i comes from base item bfirst[tile[i]] + j
    src = np.repeat(bfirst[tile] - first, n_items) + np.arange(total, dtype=np.int64)
    return infos, base_items[src]


def compare(got_infos, got_items, exp_infos, exp_items):
    """Every field of every frame Frame::read accepts, kind / ok / crc_ok / item_count / item_first of
    the others (their other fields are unspecified, include/uflow_frame_codec.h), and every item."""
    n = exp_infos.size
    assert got_infos.size == n
    ok = exp_infos["ok"] == 1
    raw_g = got_infos.view(np.uint8).reshape(n, -1)
    raw_e = exp_infos.view(np.uint8).reshape(n, -1)
    bad = np.nonzero(ok & (raw_g != raw_e).any(1))[0]
    assert bad.size == 0, f"{bad.size} accepted frames' infos differ from the oracle, first {bad[:8]}"
    for fld in ("kind", "ok", "crc_ok", "item_count", "item_first"):
        bad = np.nonzero(got_infos[fld] != exp_infos[fld])[0]
        assert bad.size == 0, f"{fld}: {bad.size} frames differ from the oracle, first {bad[:8]}"
    bad = np.nonzero(~ok & (got_infos["ok"] == 1))[0]
    assert bad.size == 0
    k = exp_items.size
    assert got_items.size >= k
    bad = np.nonzero((got_items[:k].view(np.uint8).reshape(k, -1) != exp_items.view(np.uint8).reshape(k, -1)).any(1))[0]
    assert bad.size == 0, f"{bad.size} items differ from the oracle, first {bad[:8]}"

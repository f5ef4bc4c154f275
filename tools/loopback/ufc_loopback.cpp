// ufc_loopback -- uflow frames over UDP loopback with the batched CRC gate in the receive path.
//
// Two modes (BASELINE.json configs 1 and 5):
//   --echo        a restatement of examples/echo_server.rs + echo_client.rs as frame plumbing:
//                 the client sends data frames carrying "Hello world!" packets to 127.0.0.1:8888,
//                 the server gates them on the CPU (ufc_frame_read = Frame::read), echoes each
//                 packet on channel 0 and its reverse on channel 1 (echo_server.rs:23-32), and the
//                 client gates and checks the echoes.  No connection protocol: frames only.
//   (default)     tests/ideal_transfer.rs at saturation: a sender thread streams data frames of one
//                 MAX_FRAGMENT_SIZE (1448 B) datagram each (1472-B frames, 4 channels) with
//                 sendmmsg; the receiver takes batches with recvmmsg into fixed 1472-B slots (pinned
//                 host memory) and hands each batch to a worker that runs the CRC gate -- on the GPU
//                 (ufc_validate_host_slots: H2D + kernel + D2H) or on the CPU (--gate cpu) -- then
//                 the rest of Frame::read (ufc_frame_parse) and checks every payload byte.  The
//                 reference does one recv_from + Frame::read per datagram (server/mod.rs:591-602).
//                 --send-seal cpu|gpu: the sender builds every flush's frames with zero trailers and
//                 seals them in one batch (per frame on the CPU, or ufc_seal_host_slots on the GPU)
//                 before sendmmsg, the batched form of emit.rs:114-125 + build.rs:151-159.
//   --rx-threads R   the server loop of server/mod.rs:591-602 (receive, gate, handle in one thread)
//                 on R threads, each with its own socket (port + r) fed by its own sender: per
//                 batch the thread receives into one of two pinned slot buffers; with the GPU gate
//                 it queues the batch's gate (ufc_validate_host_slots_async) and, while that runs,
//                 parses and checks the previous batch, then receives the next; with --gate cpu it
//                 gates each frame itself (ufc_frame_validate) before parsing.
// Output: one JSON line (frames/s and GB/s of frame bytes received, gated and parsed).
#include <arpa/inet.h>
#include <hip/hip_runtime.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/uflow_frame_codec.h"

namespace {

constexpr size_t kFrame = 1472;              // MAX_FRAME_SIZE (src/lib.rs:294)
constexpr size_t kFragment = 1448;           // MAX_FRAGMENT_SIZE (src/lib.rs:297)
constexpr int kChannels = 4;                 // tests/ideal_transfer.rs:10

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int udp_socket(uint16_t port, bool bind_it, int rcvbuf) {
  int fd = socket(AF_INET, SOCK_DGRAM, 0);
  if (fd < 0) {
    perror("socket");
    exit(2);
  }
  if (rcvbuf) setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf));
  int sndbuf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof(sndbuf));
  if (bind_it) {
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(port);
    a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
    if (bind(fd, (sockaddr*)&a, sizeof(a)) != 0) {
      perror("bind");
      exit(2);
    }
  }
  return fd;
}

sockaddr_in loopback(uint16_t port) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(port);
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  return a;
}

void set_timeout(int fd, int ms) {
  timeval tv{ms / 1000, (ms % 1000) * 1000};
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

// Payload byte i of packet p on channel c (ideal_transfer.rs:76-84 puts the channel and a BE
// packet id first; the rest is a pattern the receiver can recompute).
inline uint8_t payload_byte(uint32_t c, uint32_t p, size_t i) {
  if (i == 0) return (uint8_t)c;
  if (i < 5) return (uint8_t)(p >> (8 * (4 - i)));
  return (uint8_t)(p * 131u + (uint32_t)i * 7u + c);
}

// One frame of the stream: data frame `seq` = packet seq / 4 of channel seq % 4.
size_t build_stream_frame(uint8_t* out, uint32_t seq, bool seal) {
  const uint32_t c = seq % kChannels, p = seq / kChannels;
  static thread_local std::vector<uint8_t> pay(kFragment);
  for (size_t i = 0; i < kFragment; i++) pay[i] = payload_byte(c, p, i);
  ufc_builder b;
  ufc_data_frame_builder_init(&b, out, kFrame, seq, 0);
  ufc_datagram_ref d{};
  d.sequence_id = p & 0xFFFFF;
  d.channel_id = (uint8_t)c;
  d.data = pay.data();
  d.data_len = kFragment;
  if (ufc_data_frame_builder_add(&b, &d) != UFC_OK) abort();
  return ufc_builder_build(&b, seal ? 1 : 0);
}

struct Args {
  bool echo = false;
  bool gpu = true;
  uint64_t frames = 2000000;
  int batch = 4096;
  uint16_t port = 8888;
  uint64_t corrupt_every = 0;  // flip one bit in every k-th frame (must be rejected)
  bool verify = true;
  int send_seal = 0;  // 0: frames built once and re-sent; 1: built per flush, sealed on the CPU; 2: ... on the GPU
  int rx_threads = 0;  // > 0: the inline receive loop on that many threads (run_stream_inline)
  int tx_per_rx = 1;   // sender threads per receive thread (inline mode)
  double rate_gbps = 0;  // inline mode: offered rate of frame bytes, all senders together (0 = unpaced)
};

// Sender pacing: block until `bytes` may leave at `rate` B/s counted from t0 (spin for short waits).
void pace(double t0, double bytes, double rate) {
  if (rate <= 0) return;
  const double due = t0 + bytes / rate;
  for (;;) {
    const double d = due - now_s();
    if (d <= 0) return;
    if (d > 200e-6) std::this_thread::sleep_for(std::chrono::duration<double>(d - 100e-6));
    else std::this_thread::yield();
  }
}

// ---------------- config 1: echo plumbing ----------------
int run_echo(const Args& a) {
  const int srv = udp_socket(a.port, true, 1 << 20);
  const int cli = udp_socket(0, false, 1 << 20);
  set_timeout(srv, 2000);
  set_timeout(cli, 2000);
  const int kMsgs = 10;
  std::atomic<int> served{0};
  std::thread server([&] {
    uint8_t buf[kFrame], out[kFrame];
    ufc_frame_info info;
    ufc_item items[UFC_DATA_FRAME_MAX_DATAGRAM_COUNT];
    for (int k = 0; k < kMsgs; k++) {
      sockaddr_in from{};
      socklen_t fl = sizeof(from);
      const ssize_t n = recvfrom(srv, buf, sizeof(buf), 0, (sockaddr*)&from, &fl);
      if (n < 0) return;
      if (ufc_frame_read(buf, (size_t)n, &info, items, UFC_DATA_FRAME_MAX_DATAGRAM_COUNT) != 1 ||
          info.kind != UFC_FRAME_DATA)
        continue;  // Frame::read returned None: dropped silently (server/mod.rs:598)
      for (uint32_t j = 0; j < info.item_count; j++) {
        const uint8_t* msg = buf + items[j].data_offset;
        const uint32_t len = items[j].data_len;
        std::string s((const char*)msg, len), r(s.rbegin(), s.rend());
        printf("[server] received \"%s\"\n", s.c_str());
        ufc_builder b;
        ufc_data_frame_builder_init(&b, out, sizeof(out), info.f[0], 0);
        ufc_datagram_ref d0{};  // echo on channel 0 (echo_server.rs:29)
        d0.sequence_id = items[j].id;
        d0.channel_id = 0;
        d0.data = msg;
        d0.data_len = len;
        ufc_datagram_ref d1 = d0;  // reversed on channel 1 (echo_server.rs:32)
        d1.channel_id = 1;
        d1.data = (const uint8_t*)r.data();
        ufc_data_frame_builder_add(&b, &d0);
        ufc_data_frame_builder_add(&b, &d1);
        const size_t fl2 = ufc_builder_build(&b, 1);
        sendto(srv, out, fl2, 0, (sockaddr*)&from, fl);
      }
      served++;
    }
  });
  const sockaddr_in to = loopback(a.port);
  int ok = 0;
  uint8_t buf[kFrame], out[kFrame];
  for (int k = 0; k < kMsgs; k++) {
    char msg[64];
    snprintf(msg, sizeof(msg), "Hello world! #%d", k);  // echo_client.rs sends "Hello world!"
    ufc_builder b;
    ufc_data_frame_builder_init(&b, out, sizeof(out), (uint32_t)k, 0);
    ufc_datagram_ref d{};
    d.sequence_id = (uint32_t)k;
    d.data = (const uint8_t*)msg;
    d.data_len = strlen(msg);
    ufc_data_frame_builder_add(&b, &d);
    const size_t fl = ufc_builder_build(&b, 1);
    sendto(cli, out, fl, 0, (const sockaddr*)&to, sizeof(to));
    const ssize_t n = recv(cli, buf, sizeof(buf), 0);
    ufc_frame_info info;
    ufc_item items[4];
    if (n > 0 && ufc_frame_read(buf, (size_t)n, &info, items, 4) == 1 && info.item_count == 2) {
      std::string e0((const char*)buf + items[0].data_offset, items[0].data_len);
      std::string e1((const char*)buf + items[1].data_offset, items[1].data_len);
      std::string want(msg), rev(want.rbegin(), want.rend());
      printf("[client] received \"%s\" / \"%s\"\n", e0.c_str(), e1.c_str());
      if (e0 == want && e1 == rev && items[0].channel_id == 0 && items[1].channel_id == 1) ok++;
    }
  }
  server.join();
  close(srv);
  close(cli);
  printf("{\"config\": \"1: echo_client + echo_server over loopback, CPU CRC gate (frame plumbing)\", "
         "\"messages\": %d, \"echoes_ok\": %d, \"served\": %d}\n",
         kMsgs, ok, served.load());
  return ok == kMsgs ? 0 : 1;
}

// ---------------- config 5: saturation with the gate in the receive path ----------------
struct Batch {
  uint8_t* slots = nullptr;  // batch * kFrame bytes (pinned when the gate is on the GPU)
  std::vector<uint32_t> lens;
  std::vector<uint32_t> crc;
  std::vector<uint8_t> valid;
  size_t n = 0;
};

int run_stream(const Args& a) {
  ufc_ctx* ctx = nullptr;
  if (a.gpu) {
    const int rc = ufc_ctx_create(&ctx, 0);
    if (rc != UFC_OK) {
      fprintf(stderr, "ufc_ctx_create: %s\n", ufc_error_string(rc));
      return 2;
    }
  }
  const int rx = udp_socket(a.port, true, 256 << 20);
  set_timeout(rx, 300);
  const int tx = udp_socket(0, false, 0);
  const size_t B = (size_t)a.batch;
  // Sender: frames are built once (a ring of distinct frames, re-sent by sequence number).
  const uint32_t kRing = 8192;
  std::vector<uint8_t> ring((size_t)kRing * kFrame);
  for (uint32_t s = 0; s < kRing; s++) build_stream_frame(ring.data() + (size_t)s * kFrame, s, true);
  std::atomic<bool> sender_done{false};
  std::atomic<uint64_t> sent{0};
  // Send-side seal modes: every flush of F frames is laid out by the
  // builder with zero trailers (payloads copied from a pool), sealed in one batch -- per frame on
  // the CPU (ufc_frame_seal) or on the GPU (ufc_seal_host_slots) -- then sent with sendmmsg.
  double t_send_seal = 0, t_send_total = 0;
  ufc_ctx* sctx = nullptr;
  if (a.send_seal == 2 && ufc_ctx_create(&sctx, 0) != UFC_OK) return 2;
  std::thread sender([&] {
    const sockaddr_in to = loopback(a.port);
    const double t0 = now_s();
    if (a.send_seal) {
      const size_t F = 4096;
      uint8_t* slab = nullptr;
      if (sctx) {
        if (hipHostMalloc((void**)&slab, F * kFrame, hipHostMallocDefault) != hipSuccess) abort();
      } else {
        slab = (uint8_t*)malloc(F * kFrame);
      }
      std::vector<uint32_t> lens(F), crcs(F);
      std::vector<mmsghdr> msgs(F);
      std::vector<iovec> iov(F);
      uint64_t s = 0;
      while (s < a.frames) {
        const size_t m = (size_t)std::min<uint64_t>(F, a.frames - s);
        for (size_t i = 0; i < m; i++) {
          const uint32_t seq = (uint32_t)((s + i) % kRing);
          uint8_t* f = slab + i * kFrame;
          ufc_builder b;  // DataFrameBuilder::new + add (payload from the pool) with a zero trailer
          ufc_data_frame_builder_init(&b, f, kFrame, seq, 0);
          ufc_datagram_ref d{};
          d.sequence_id = (seq / kChannels) & 0xFFFFF;
          d.channel_id = (uint8_t)(seq % kChannels);
          d.data = ring.data() + (size_t)seq * kFrame + 20;  // pool payload (6-B frame + 14-B datagram header)
          d.data_len = kFragment;
          ufc_data_frame_builder_add(&b, &d);
          lens[i] = (uint32_t)ufc_builder_build(&b, 0);
        }
        const double ts = now_s();
        if (sctx) {
          if (ufc_seal_host_slots(sctx, slab, kFrame, lens.data(), m, crcs.data()) != UFC_OK) abort();
        } else {
          for (size_t i = 0; i < m; i++) ufc_frame_seal(slab + i * kFrame, lens[i]);
        }
        t_send_seal += now_s() - ts;
        for (size_t i = 0; i < m; i++) {
          const uint64_t q = s + i;
          if (a.corrupt_every && q % a.corrupt_every == a.corrupt_every - 1) slab[i * kFrame + 100 + q % 1000] ^= 0x10;
          iov[i].iov_base = slab + i * kFrame;
          iov[i].iov_len = lens[i];
          msgs[i].msg_hdr = msghdr{};
          msgs[i].msg_hdr.msg_name = (void*)&to;
          msgs[i].msg_hdr.msg_namelen = sizeof(to);
          msgs[i].msg_hdr.msg_iov = &iov[i];
          msgs[i].msg_hdr.msg_iovlen = 1;
        }
        for (size_t done = 0; done < m;) {
          const int r = sendmmsg(tx, msgs.data() + done, (unsigned)std::min<size_t>(64, m - done), 0);
          if (r > 0) done += (size_t)r;
        }
        s += m;
      }
      if (sctx)
        (void)hipHostFree(slab);
      else
        free(slab);
      t_send_total = now_s() - t0;
      sent = s;
      sender_done = true;
      return;
    }
    const int M = 64;
    std::vector<mmsghdr> msgs(M);
    std::vector<iovec> iov(M);
    std::vector<uint8_t> scratch((size_t)M * kFrame);
    uint64_t s = 0;
    while (s < a.frames) {
      const int m = (int)std::min<uint64_t>(M, a.frames - s);
      for (int i = 0; i < m; i++) {
        const uint64_t q = s + i;
        uint8_t* f = ring.data() + (size_t)(q % kRing) * kFrame;
        if (a.corrupt_every && q % a.corrupt_every == a.corrupt_every - 1) {  // one flipped bit
          memcpy(scratch.data() + (size_t)i * kFrame, f, kFrame);
          f = scratch.data() + (size_t)i * kFrame;
          f[100 + q % 1000] ^= 0x10;
        }
        iov[i].iov_base = f;
        iov[i].iov_len = kFrame;
        msgs[i].msg_hdr = msghdr{};
        msgs[i].msg_hdr.msg_name = (void*)&to;
        msgs[i].msg_hdr.msg_namelen = sizeof(to);
        msgs[i].msg_hdr.msg_iov = &iov[i];
        msgs[i].msg_hdr.msg_iovlen = 1;
      }
      const int r = sendmmsg(tx, msgs.data(), m, 0);
      if (r > 0) s += r;
    }
    sent = s;
    sender_done = true;
  });
  // Two batches: the receiver fills one while the worker gates and parses the other.
  Batch bufs[2];
  for (Batch& b : bufs) {
    if (a.gpu) {
      if (hipHostMalloc((void**)&b.slots, B * kFrame, hipHostMallocDefault) != hipSuccess) return 2;
    } else {
      b.slots = (uint8_t*)malloc(B * kFrame);
    }
    b.lens.resize(B);
    b.crc.resize(B);
    b.valid.resize(B);
  }
  std::mutex mu;
  std::condition_variable cv;
  int full = -1;           // index of the batch waiting for the worker
  bool free_slot[2] = {true, true};
  bool stop = false;
  uint64_t n_valid = 0, n_invalid = 0, n_parsed = 0, n_payload_bad = 0, bytes_in = 0;
  double t_gate = 0;
  std::thread worker([&] {
    std::vector<ufc_item> items(UFC_DATA_FRAME_MAX_DATAGRAM_COUNT);
    for (;;) {
      int k;
      {
        std::unique_lock<std::mutex> l(mu);
        cv.wait(l, [&] { return full >= 0 || stop; });
        if (full < 0 && stop) return;
        k = full;
        full = -1;
      }
      Batch& b = bufs[k];
      const double t0 = now_s();
      if (a.gpu) {
        if (ufc_validate_host_slots(ctx, b.slots, kFrame, b.lens.data(), b.n, b.crc.data(), b.valid.data()) != UFC_OK)
          abort();
      } else {
        for (size_t i = 0; i < b.n; i++) b.valid[i] = (uint8_t)ufc_frame_validate(b.slots + i * kFrame, b.lens[i]);
      }
      t_gate += now_s() - t0;
      for (size_t i = 0; i < b.n; i++) {
        const uint8_t* f = b.slots + i * kFrame;
        bytes_in += b.lens[i];
        if (!b.valid[i]) {
          n_invalid++;
          continue;
        }
        n_valid++;
        ufc_frame_info info;
        if (ufc_frame_parse(f, b.lens[i], 1, &info, items.data(), items.size()) != 1) continue;
        n_parsed++;
        if (a.verify && info.kind == UFC_FRAME_DATA && info.item_count == 1) {
          const uint32_t seq = info.f[0], c = seq % kChannels, p = seq / kChannels;
          if (items[0].channel_id != c || items[0].id != (p & 0xFFFFF) || items[0].data_len != kFragment) {
            n_payload_bad++;
            continue;
          }
          if (memcmp(f + items[0].data_offset, ring.data() + (size_t)(seq % kRing) * kFrame + items[0].data_offset,
                     kFragment) != 0)
            n_payload_bad++;
        }
      }
      std::lock_guard<std::mutex> l(mu);
      free_slot[k] = true;
      cv.notify_all();
    }
  });
  uint64_t received = 0;
  double t_first = 0, t_last = 0;
  std::vector<mmsghdr> msgs(B);
  std::vector<iovec> iov(B);
  int cur = 0;
  for (;;) {
    {
      std::unique_lock<std::mutex> l(mu);
      cv.wait(l, [&] { return free_slot[cur]; });
      free_slot[cur] = false;
    }
    Batch& b = bufs[cur];
    b.n = 0;
    bool idle = false;
    while (b.n < B) {
      const size_t want = B - b.n;
      for (size_t i = 0; i < want; i++) {
        iov[i].iov_base = b.slots + (b.n + i) * kFrame;
        iov[i].iov_len = kFrame;
        msgs[i].msg_hdr = msghdr{};
        msgs[i].msg_hdr.msg_iov = &iov[i];
        msgs[i].msg_hdr.msg_iovlen = 1;
      }
      const int r = recvmmsg(rx, msgs.data(), (unsigned)want, MSG_WAITFORONE, nullptr);
      if (r <= 0) {  // 300 ms without a datagram: the stream is over
        idle = sender_done.load();
        if (idle || received == 0) {
          if (idle) break;
          continue;
        }
        break;
      }
      if (received == 0) t_first = now_s();
      for (int i = 0; i < r; i++) b.lens[b.n + i] = msgs[i].msg_len;
      b.n += (size_t)r;
      received += (uint64_t)r;
      t_last = now_s();
    }
    {
      std::unique_lock<std::mutex> l(mu);
      if (b.n) {
        cv.wait(l, [&] { return full < 0; });
        full = cur;
      } else {
        free_slot[cur] = true;
      }
      cv.notify_all();
    }
    cur ^= 1;
    if (idle) break;
  }
  {
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [&] { return full < 0 && free_slot[0] && free_slot[1]; });
    stop = true;
    cv.notify_all();
  }
  worker.join();
  sender.join();
  const double secs = now_s() - t_first;
  const double span = std::max(t_last - t_first, 1e-9);
  printf("{\"config\": \"5: ideal_transfer-style loopback at saturation, %s CRC gate in the receive path\", "
         "\"frame_bytes\": %zu, \"sent\": %llu, \"received\": %llu, \"lost\": %llu, \"loss_frac\": %.5f, "
         "\"valid\": %llu, \"invalid\": %llu, "
         "\"parsed\": %llu, \"payload_mismatch\": %llu, \"receive_seconds\": %.4f, \"frames_per_s\": %.0f, "
         "\"GB_s\": %.3f, \"gate_seconds\": %.4f, \"gate_GB_s\": %.3f, \"batch\": %d, \"total_seconds\": %.4f, "
         "\"send_seal\": \"%s\", \"send_seal_seconds\": %.4f, \"send_seal_GB_s\": %.3f, \"send_seconds\": %.4f}\n",
         a.gpu ? "GPU (ufc_validate_host_slots: H2D + kernel + D2H)" : "CPU (ufc_frame_validate, 1 thread)", kFrame,
         (unsigned long long)sent.load(), (unsigned long long)received,
         (unsigned long long)(sent.load() - std::min<uint64_t>(sent.load(), received)),
         sent.load() ? 1.0 - (double)received / (double)sent.load() : 0.0, (unsigned long long)n_valid,
         (unsigned long long)n_invalid, (unsigned long long)n_parsed, (unsigned long long)n_payload_bad, span,
         received / span, bytes_in / span / 1e9, t_gate, t_gate > 0 ? bytes_in / t_gate / 1e9 : 0.0, a.batch, secs,
         a.send_seal == 0 ? "none (prebuilt frames)" : a.send_seal == 1 ? "cpu (ufc_frame_seal per frame)"
                                                                       : "gpu (ufc_seal_host_slots per flush)",
         t_send_seal, t_send_seal > 0 ? (double)sent.load() * kFrame / t_send_seal / 1e9 : 0.0, t_send_total);
  for (Batch& b : bufs) {
    if (a.gpu)
      (void)hipHostFree(b.slots);
    else
      free(b.slots);
  }
  close(rx);
  close(tx);
  if (ctx) ufc_ctx_destroy(ctx);
  if (sctx) ufc_ctx_destroy(sctx);
  return (n_payload_bad == 0 && received > 0) ? 0 : 1;
}

// ---------------- config 5, inline receive loops on R threads ----------------
struct LaneStats {
  uint64_t received = 0, valid = 0, invalid = 0, parsed = 0, payload_bad = 0, bytes = 0;
  double t_first = 0, t_last = 0, t_gate = 0, t_recv = 0, t_handle = 0, t_sync = 0;
};

int run_stream_inline(const Args& a) {
  const int R = a.rx_threads;
  const size_t B = (size_t)a.batch;
  const uint32_t kRing = 8192;
  std::vector<uint8_t> ring((size_t)kRing * kFrame);
  for (uint32_t s = 0; s < kRing; s++) build_stream_frame(ring.data() + (size_t)s * kFrame, s, true);
  std::vector<LaneStats> st(R);
  std::vector<std::thread> threads;
  std::atomic<int> senders_done{0};
  std::atomic<int> failed{0};
  std::vector<int> rx(R);
  int rcvbuf = 0;
  for (int r = 0; r < R; r++) {
    rx[r] = udp_socket((uint16_t)(a.port + r), true, 64 << 20);
    set_timeout(rx[r], 300);
    socklen_t sl = sizeof(rcvbuf);
    getsockopt(rx[r], SOL_SOCKET, SO_RCVBUF, &rcvbuf, &sl);
  }
  const int TX = R * std::max(1, a.tx_per_rx);
  const double rate_tx = a.rate_gbps > 0 ? a.rate_gbps * 1e9 / TX : 0.0;  // B/s per sender
  std::atomic<uint64_t> sent_total{0};
  // Senders start once every receiver is ready (GPU context, pinned buffers and the staging warm-up
  // take a fresh process up to seconds, which unstarted receivers would otherwise lose as datagrams).
  std::atomic<int> rx_ready{0};
  std::atomic<double> t_send0{0.0};  // (pacing clock and the sender-clock goodput start)
  std::vector<double> t_send_end(TX, 0.0);
  for (int t = 0; t < TX; t++) {
    // sender t: frames [F t / TX, F (t+1) / TX) to port + t % R
    threads.emplace_back([&, t] {
      while (rx_ready.load() < R) std::this_thread::sleep_for(std::chrono::microseconds(200));
      if (t == 0) t_send0.store(now_s());
      while (t_send0.load() == 0.0) std::this_thread::yield();
      const int tx = udp_socket(0, false, 0);
      const sockaddr_in to = loopback((uint16_t)(a.port + t % R));
      const uint64_t lo = a.frames * t / TX, hi = a.frames * (t + 1) / TX;
      const int M = 64;
      std::vector<mmsghdr> msgs(M);
      std::vector<iovec> iov(M);
      std::vector<uint8_t> scratch((size_t)M * kFrame);
      for (uint64_t s = lo; s < hi;) {
        const int m = (int)std::min<uint64_t>(M, hi - s);
        pace(t_send0.load(), (double)(s - lo) * kFrame, rate_tx);
        for (int i = 0; i < m; i++) {
          const uint64_t q = s + i;
          uint8_t* f = ring.data() + (size_t)(q % kRing) * kFrame;
          if (a.corrupt_every && q % a.corrupt_every == a.corrupt_every - 1) {
            memcpy(scratch.data() + (size_t)i * kFrame, f, kFrame);
            f = scratch.data() + (size_t)i * kFrame;
            f[100 + q % 1000] ^= 0x10;
          }
          iov[i].iov_base = f;
          iov[i].iov_len = kFrame;
          msgs[i].msg_hdr = msghdr{};
          msgs[i].msg_hdr.msg_name = (void*)&to;
          msgs[i].msg_hdr.msg_namelen = sizeof(to);
          msgs[i].msg_hdr.msg_iov = &iov[i];
          msgs[i].msg_hdr.msg_iovlen = 1;
        }
        const int k = sendmmsg(tx, msgs.data(), m, 0);
        if (k > 0) {
          s += (uint64_t)k;
          sent_total += (uint64_t)k;
        }
      }
      t_send_end[t] = now_s();
      close(tx);
      senders_done++;
    });
  }
  for (int r = 0; r < R; r++) {
    // receiver r: receive, gate, parse + check, in one thread
    threads.emplace_back([&, r] {
      LaneStats& S = st[r];
      ufc_ctx* ctx = nullptr;
      hipStream_t streams[2] = {nullptr, nullptr};
      struct Buf {
        uint8_t* slots = nullptr;
        uint32_t* lens = nullptr;
        uint32_t* crc = nullptr;
        uint8_t* valid = nullptr;
        size_t n = 0;
      } bufs[2];
      bool counted = false;
      auto fail = [&](const char* what) {
        fprintf(stderr, "receiver %d: %s\n", r, what);
        failed++;
        if (!counted) rx_ready++;  // (never leave the senders waiting)
        counted = true;
      };
      if (a.gpu) {
        if (ufc_ctx_create(&ctx, 0) != UFC_OK) return fail("ufc_ctx_create");
        for (int k = 0; k < 2; k++) {
          if (hipStreamCreateWithFlags(&streams[k], hipStreamNonBlocking) != hipSuccess ||
              hipHostMalloc((void**)&bufs[k].slots, B * kFrame, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&bufs[k].lens, B * 4, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&bufs[k].crc, B * 4, hipHostMallocDefault) != hipSuccess ||
              hipHostMalloc((void**)&bufs[k].valid, B, hipHostMallocDefault) != hipSuccess)
            return fail("pinned buffers");
        }
        // size the context's per-stream staging for a full batch now (a first small batch would
        // otherwise grow it mid-stream, and freeing device memory waits for the whole device)
        for (int k = 0; k < 2; k++) {
          memset(bufs[k].lens, 0, B * 4);
          if (ufc_validate_host_slots_async(ctx, bufs[k].slots, kFrame, bufs[k].lens, B, bufs[k].crc, bufs[k].valid,
                                            streams[k]) != UFC_OK ||
              hipStreamSynchronize(streams[k]) != hipSuccess)
            return fail("staging warm-up");
        }
      } else {
        for (int k = 0; k < 2; k++) {
          bufs[k].slots = (uint8_t*)malloc(B * kFrame);
          bufs[k].lens = (uint32_t*)malloc(B * 4);
          bufs[k].crc = (uint32_t*)malloc(B * 4);
          bufs[k].valid = (uint8_t*)malloc(B);
        }
      }
      std::vector<ufc_item> items(UFC_DATA_FRAME_MAX_DATAGRAM_COUNT);
      std::vector<mmsghdr> msgs(B);
      std::vector<iovec> iov(B);
      rx_ready++;
      counted = true;
      // parse + payload check of a gated batch (the rest of Frame::read and the application)
      auto handle = [&](const Buf& b) {
        for (size_t i = 0; i < b.n; i++) {
          const uint8_t* f = b.slots + i * kFrame;
          S.bytes += b.lens[i];
          if (!b.valid[i]) {
            S.invalid++;
            continue;
          }
          S.valid++;
          ufc_frame_info info;
          if (ufc_frame_parse(f, b.lens[i], 1, &info, items.data(), items.size()) != 1) continue;
          S.parsed++;
          if (a.verify && info.kind == UFC_FRAME_DATA && info.item_count == 1) {
            const uint32_t seq = info.f[0], c = seq % kChannels, p = seq / kChannels;
            if (items[0].channel_id != c || items[0].id != (p & 0xFFFFF) || items[0].data_len != kFragment ||
                memcmp(f + items[0].data_offset, ring.data() + (size_t)(seq % kRing) * kFrame + items[0].data_offset,
                       kFragment) != 0)
              S.payload_bad++;
          }
        }
      };
      int cur = 0, pending = -1;
      bool idle = false;
      while (!idle) {
        Buf& b = bufs[cur];
        b.n = 0;
        while (b.n < B) {
          const size_t want = B - b.n;
          for (size_t i = 0; i < want; i++) {
            iov[i].iov_base = b.slots + (b.n + i) * kFrame;
            iov[i].iov_len = kFrame;
            msgs[i].msg_hdr = msghdr{};
            msgs[i].msg_hdr.msg_iov = &iov[i];
            msgs[i].msg_hdr.msg_iovlen = 1;
          }
          const double tr0 = now_s();
          const int k = recvmmsg(rx[r], msgs.data(), (unsigned)want, MSG_WAITFORONE, nullptr);
          if (k > 0) S.t_recv += now_s() - tr0;
          if (k <= 0) {  // 300 ms without a datagram
            if (senders_done.load() == TX) {
              idle = true;
              break;
            }
            if (S.received == 0) continue;
            break;
          }
          if (S.received == 0) S.t_first = now_s();
          for (int i = 0; i < k; i++) b.lens[b.n + i] = msgs[i].msg_len;
          b.n += (size_t)k;
          S.received += (uint64_t)k;
          S.t_last = now_s();
        }
        if (a.gpu) {
          const double t0 = now_s();
          if (b.n && ufc_validate_host_slots_async(ctx, b.slots, kFrame, b.lens, b.n, b.crc, b.valid, streams[cur]) != UFC_OK)
            return fail("ufc_validate_host_slots_async");
          if (pending >= 0) {
            const double ts = now_s();
            if (hipStreamSynchronize(streams[pending]) != hipSuccess) return fail("hipStreamSynchronize");
            S.t_sync += now_s() - ts;
            S.t_gate += now_s() - t0;  // (queueing + waiting: the gate's cost to this thread)
            const double th = now_s();
            handle(bufs[pending]);
            S.t_handle += now_s() - th;
          } else {
            S.t_gate += now_s() - t0;
          }
          pending = b.n ? cur : -1;
          cur ^= 1;
        } else {
          const double t0 = now_s();
          for (size_t i = 0; i < b.n; i++) b.valid[i] = (uint8_t)ufc_frame_validate(b.slots + i * kFrame, b.lens[i]);
          S.t_gate += now_s() - t0;
          const double th = now_s();
          handle(b);
          S.t_handle += now_s() - th;
        }
      }
      if (pending >= 0) {
        if (hipStreamSynchronize(streams[pending]) != hipSuccess) return fail("hipStreamSynchronize");
        handle(bufs[pending]);
      }
      for (int k = 0; k < 2; k++) {
        if (a.gpu) {
          (void)hipHostFree(bufs[k].slots);
          (void)hipHostFree(bufs[k].lens);
          (void)hipHostFree(bufs[k].crc);
          (void)hipHostFree(bufs[k].valid);
          (void)hipStreamDestroy(streams[k]);
        } else {
          free(bufs[k].slots);
          free(bufs[k].lens);
          free(bufs[k].crc);
          free(bufs[k].valid);
        }
      }
      if (ctx) ufc_ctx_destroy(ctx);
    });
  }
  for (auto& t : threads) t.join();
  for (int r = 0; r < R; r++) close(rx[r]);
  LaneStats T;
  T.t_first = 1e300;
  double gate_max = 0;
  for (const LaneStats& S : st) {
    T.received += S.received;
    T.valid += S.valid;
    T.invalid += S.invalid;
    T.parsed += S.parsed;
    T.payload_bad += S.payload_bad;
    T.bytes += S.bytes;
    if (S.received) {
      T.t_first = std::min(T.t_first, S.t_first);
      T.t_last = std::max(T.t_last, S.t_last);
    }
    T.t_gate += S.t_gate;
    T.t_recv += S.t_recv;
    T.t_handle += S.t_handle;
    T.t_sync += S.t_sync;
    gate_max = std::max(gate_max, S.t_gate);
  }
  const double span = std::max(T.t_last - T.t_first, 1e-9);
  const double t_start = t_send0.load();
  double send_end = t_start;
  for (double t : t_send_end) send_end = std::max(send_end, t);
  const uint64_t sent = sent_total.load();
  // Goodput on the senders' clock: frame bytes received / (last datagram received - first sent):
  // comparable between gates whatever each one dropped (ideal_transfer.rs).
  const double span_tx = std::max((T.received ? T.t_last : send_end) - t_start, 1e-9);
  printf("{\"config\": \"5: ideal_transfer-style loopback, inline receive loops (receive + %s gate + "
         "parse + payload check per thread)\", \"rx_threads\": %d, \"frame_bytes\": %zu, \"sent\": %llu, "
         "\"received\": %llu, \"lost\": %llu, \"loss_frac\": %.5f, \"offered_GB_s\": %.3f, "
         "\"valid\": %llu, \"invalid\": %llu, \"parsed\": %llu, \"payload_mismatch\": %llu, "
         "\"receive_seconds\": %.4f, \"frames_per_s\": %.0f, \"GB_s\": %.3f, \"goodput_GB_s_sender_clock\": %.3f, "
         "\"send_seconds\": %.4f, \"gate_thread_seconds\": %.4f, "
         "\"gate_share_of_thread_time\": %.3f, \"recv_call_seconds\": %.4f, \"sync_wait_seconds\": %.4f, "
         "\"handle_seconds\": %.4f, \"batch\": %d, \"failed_threads\": %d, \"tx_threads\": %d, "
         "\"so_rcvbuf\": %d}\n",
         a.gpu ? "GPU (ufc_validate_host_slots_async, overlapped with the next receive)" : "CPU (ufc_frame_validate)", R,
         kFrame, (unsigned long long)sent, (unsigned long long)T.received,
         (unsigned long long)(sent - std::min(sent, T.received)), sent ? 1.0 - (double)T.received / (double)sent : 0.0,
         a.rate_gbps, (unsigned long long)T.valid,
         (unsigned long long)T.invalid, (unsigned long long)T.parsed, (unsigned long long)T.payload_bad, span,
         T.received / span, T.bytes / span / 1e9, T.bytes / span_tx / 1e9, send_end - t_start, T.t_gate,
         T.t_gate / (span * R), T.t_recv, T.t_sync, T.t_handle, a.batch, failed.load(), TX, rcvbuf);
  return (T.payload_bad == 0 && T.received > 0 && failed.load() == 0) ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; i++) {
    const std::string s = argv[i];
    auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (s == "--echo") a.echo = true;
    else if (s == "--gate") a.gpu = std::string(next()) != "cpu";
    else if (s == "--frames") a.frames = strtoull(next(), nullptr, 10);
    else if (s == "--batch") a.batch = atoi(next());
    else if (s == "--port") a.port = (uint16_t)atoi(next());
    else if (s == "--corrupt-every") a.corrupt_every = strtoull(next(), nullptr, 10);
    else if (s == "--no-verify") a.verify = false;
    else if (s == "--rx-threads") a.rx_threads = atoi(next());
    else if (s == "--tx-per-rx") a.tx_per_rx = atoi(next());
    else if (s == "--rate-gbps") a.rate_gbps = atof(next());
    else if (s == "--send-seal") {
      const std::string v = next();
      a.send_seal = v == "gpu" ? 2 : v == "cpu" ? 1 : 0;
    }
    else {
      fprintf(stderr, "usage: %s [--echo] [--gate gpu|cpu] [--frames N] [--batch B] [--port P] "
                      "[--corrupt-every K] [--no-verify] [--send-seal none|cpu|gpu] [--rx-threads R] [--tx-per-rx T] "
                      "[--rate-gbps G]\n", argv[0]);
      return 2;
    }
  }
  if (a.echo) return run_echo(a);
  return a.rx_threads > 0 ? run_stream_inline(a) : run_stream(a);
}

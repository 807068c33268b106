// Batched UDP socket I/O for the codec's host boundary.
//
// The reference moves one datagram per system call: sendto (utils/
// reliableUDP.py:61, :92, :146, :161) and recvfrom(1024) (:67, :118, :167;
// proxy.py:129).  These entry points move up to 1024 datagrams per call with
// sendmmsg / recvmmsg, straight between the socket and caller-owned host
// buffers (pinned, so they feed hipMemcpyAsync without a bounce), in the
// packed-frames + offsets layout rudp_encode_varlen writes and rudp_decode
// (variable-length) reads.  Host code only: no HIP calls in this file.
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <string.h>
#include <sys/socket.h>

#include <vector>

#include "../../include/rudp.h"

namespace {

constexpr unsigned kMaxVec = 1024;  // datagrams per recvmmsg/sendmmsg call

thread_local std::vector<mmsghdr> t_msgs;
thread_local std::vector<iovec> t_iov;
thread_local std::vector<sockaddr_in> t_names;

void reserve(unsigned n) {
  if (t_msgs.size() < n) {
    t_msgs.resize(n);
    t_iov.resize(n);
    t_names.resize(n);
  }
}

}  // namespace

extern "C" {

// Source / destination of a datagram as one integer: IPv4 address (host byte
// order) << 16 | port.
static uint64_t addr_key(const sockaddr_in& a) {
  return ((uint64_t)ntohl(a.sin_addr.s_addr) << 16) | ntohs(a.sin_port);
}

static sockaddr_in key_addr(uint64_t k) {
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)(k & 0xFFFFu));
  a.sin_addr.s_addr = htonl((uint32_t)(k >> 16));
  return a;
}

int rudp_udp_recv_batch(int fd, uint8_t* h_frames, uint64_t cap_bytes, uint32_t slot_bytes,
                        uint32_t max_msgs, uint64_t* h_frame_off, int timeout_ms) {
  return rudp_udp_recv_batch_from(fd, h_frames, cap_bytes, slot_bytes, max_msgs, h_frame_off, nullptr,
                                  timeout_ms);
}

int rudp_udp_recv_batch_from(int fd, uint8_t* h_frames, uint64_t cap_bytes, uint32_t slot_bytes,
                             uint32_t max_msgs, uint64_t* h_frame_off, uint64_t* h_src_or_null,
                             int timeout_ms) {
  if (fd < 0 || !h_frames || !h_frame_off || slot_bytes == 0) return RUDP_EINVAL;
  uint64_t want = cap_bytes / slot_bytes;
  if (want > max_msgs) want = max_msgs;
  h_frame_off[0] = 0;
  if (want == 0) return 0;
  if (timeout_ms != 0) {  // wait for the first datagram (-1: forever)
    pollfd pfd{fd, POLLIN, 0};
    int pr;
    do {
      pr = poll(&pfd, 1, timeout_ms);
    } while (pr < 0 && errno == EINTR);
    if (pr < 0) return -errno;
    if (pr == 0) return 0;
  }
  // Receive into fixed slots (a datagram longer than slot_bytes is truncated,
  // as recvfrom(1024) truncates in the reference), then pack the frames to
  // the front in order: packed offsets never pass slot offsets.
  uint64_t got = 0, packed = 0;
  while (got < want) {
    const unsigned chunk = (unsigned)((want - got) < kMaxVec ? (want - got) : kMaxVec);
    reserve(chunk);
    for (unsigned i = 0; i < chunk; ++i) {
      t_iov[i].iov_base = h_frames + (got + i) * (uint64_t)slot_bytes;
      t_iov[i].iov_len = slot_bytes;
      memset(&t_msgs[i], 0, sizeof(mmsghdr));
      t_msgs[i].msg_hdr.msg_iov = &t_iov[i];
      t_msgs[i].msg_hdr.msg_iovlen = 1;
      if (h_src_or_null) {
        t_names[i] = sockaddr_in{};
        t_msgs[i].msg_hdr.msg_name = &t_names[i];
        t_msgs[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
      }
    }
    int r;
    do {
      r = recvmmsg(fd, t_msgs.data(), chunk, MSG_DONTWAIT, nullptr);
    } while (r < 0 && errno == EINTR);
    if (r < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      if (got == 0) return -errno;
      break;
    }
    for (int i = 0; i < r; ++i) {
      const uint64_t len = t_msgs[i].msg_len;
      uint8_t* src = h_frames + (got + i) * (uint64_t)slot_bytes;
      if (h_frames + packed != src) memmove(h_frames + packed, src, len);
      packed += len;
      h_frame_off[got + i + 1] = packed;
      if (h_src_or_null)
        h_src_or_null[got + i] = t_names[i].sin_family == AF_INET ? addr_key(t_names[i]) : 0;
    }
    got += (uint64_t)r;
    if ((unsigned)r < chunk) break;  // socket drained
  }
  return (int)got;
}

int rudp_udp_send_batch(int fd, const uint8_t* h_frames, const uint64_t* h_frame_off, uint64_t n,
                        const char* ip, uint16_t port) {
  if (!ip) return RUDP_EINVAL;
  sockaddr_in dst{};
  dst.sin_family = AF_INET;
  dst.sin_port = htons(port);
  if (inet_pton(AF_INET, ip, &dst.sin_addr) != 1) return RUDP_EINVAL;
  const uint64_t key = addr_key(dst);
  return rudp_udp_send_batch_to(fd, h_frames, h_frame_off, n, &key, 0);
}

int rudp_udp_send_batch_to(int fd, const uint8_t* h_frames, const uint64_t* h_frame_off, uint64_t n,
                           const uint64_t* h_dst, int per_datagram) {
  if (fd < 0 || (n && (!h_frames || !h_frame_off)) || !h_dst) return RUDP_EINVAL;
  uint64_t sent = 0;
  while (sent < n) {
    const unsigned chunk = (unsigned)((n - sent) < kMaxVec ? (n - sent) : kMaxVec);
    reserve(chunk);
    for (unsigned i = 0; i < chunk; ++i) {
      const uint64_t k = sent + i;
      t_iov[i].iov_base = const_cast<uint8_t*>(h_frames + h_frame_off[k]);
      t_iov[i].iov_len = h_frame_off[k + 1] - h_frame_off[k];
      memset(&t_msgs[i], 0, sizeof(mmsghdr));
      t_names[i] = key_addr(h_dst[per_datagram ? k : 0]);
      t_msgs[i].msg_hdr.msg_name = &t_names[i];
      t_msgs[i].msg_hdr.msg_namelen = sizeof(sockaddr_in);
      t_msgs[i].msg_hdr.msg_iov = &t_iov[i];
      t_msgs[i].msg_hdr.msg_iovlen = 1;
    }
    int r;
    do {
      r = sendmmsg(fd, t_msgs.data(), chunk, 0);
    } while (r < 0 && errno == EINTR);
    if (r < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK || errno == ENOBUFS) {
        pollfd pfd{fd, POLLOUT, 0};
        poll(&pfd, 1, 100);
        continue;
      }
      return sent ? (int)sent : -errno;
    }
    sent += (uint64_t)r;
  }
  return (int)sent;
}

}  // extern "C"

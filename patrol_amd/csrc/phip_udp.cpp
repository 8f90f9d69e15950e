// The socket edge of the batched Receive pipeline: host
// code only, no GPU.  The reference reads one datagram per loop iteration
// into a 256-byte buffer under a 3-second read deadline (repo.go:54-73,
// 108-120) and answers an incast with one WriteTo per reply (repo.go:86-90,
// 160-169).  Here one call moves a whole batch:
//
//   phip_udp_recv_batch    recvmmsg into a caller buffer (a pinned ring slot),
//                          datagrams packed back to back in the wire layout
//                          phip_receive_datagrams / phip_ring_receive take;
//   phip_incast_replies    MarshalBinary of every INCAST_REPLY the batch
//                          produced, with the peer each one goes back to;
//   phip_udp_send_batch    sendmmsg of a run of datagrams (replies, or the
//                          phip_export_datagrams egress batch to one peer).
#include <errno.h>
#include <poll.h>
#include <sys/socket.h>
#include <netinet/in.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstring>

#include "patrolhip.h"

namespace {

constexpr uint32_t kVec = 256;   // datagrams per recvmmsg / sendmmsg call

socklen_t peer_len(const uint8_t* p) {
  sa_family_t fam;
  std::memcpy(&fam, p + offsetof(sockaddr_storage, ss_family), sizeof fam);
  if (fam == AF_INET) return sizeof(sockaddr_in);
  if (fam == AF_INET6) return sizeof(sockaddr_in6);
  return sizeof(sockaddr_storage);
}

}  // namespace

extern "C" {

int phip_udp_recv_batch(int fd, uint8_t* bytes, uint64_t cap, uint64_t* offs, uint32_t max_msgs,
                        uint8_t* peers, int timeout_ms, uint32_t* n_out) {
  static_assert(sizeof(sockaddr_storage) == PHIP_PEER_BYTES, "peer record size");
  if (!n_out) return PHIP_ERR_INVALID;
  *n_out = 0;
  if (fd < 0 || !bytes || !offs) return PHIP_ERR_INVALID;
  offs[0] = 0;
  // The first datagram may wait up to the deadline (repo.go:109: a Timeout
  // net.Error makes the Go loop continue, so it is not an error here).
  pollfd p{fd, POLLIN, 0};
  int pr;
  do pr = poll(&p, 1, timeout_ms); while (pr < 0 && errno == EINTR);
  if (pr < 0) return PHIP_ERR_IO;
  if (pr == 0) return PHIP_OK;
  mmsghdr hdr[kVec];
  iovec iov[kVec];
  uint64_t pos = 0;
  uint32_t n = 0;
  while (n < max_msgs) {
    // Each datagram lands in its own 256-byte window (Go's buffer: a longer
    // datagram is cut to bucketPacketSize bytes, repo.go:56), then is packed
    // down to the end of the previous one.
    const uint64_t fit = (cap - pos) / PHIP_BUCKET_PACKET_SIZE;
    const uint32_t want = (uint32_t)std::min<uint64_t>(std::min<uint32_t>(kVec, max_msgs - n), fit);
    if (!want) break;
    std::memset(hdr, 0, sizeof(mmsghdr) * want);
    for (uint32_t k = 0; k < want; ++k) {
      iov[k].iov_base = bytes + pos + (uint64_t)k * PHIP_BUCKET_PACKET_SIZE;
      iov[k].iov_len = PHIP_BUCKET_PACKET_SIZE;
      hdr[k].msg_hdr.msg_iov = &iov[k];
      hdr[k].msg_hdr.msg_iovlen = 1;
      if (peers) {
        hdr[k].msg_hdr.msg_name = peers + (uint64_t)(n + k) * PHIP_PEER_BYTES;
        hdr[k].msg_hdr.msg_namelen = PHIP_PEER_BYTES;
      }
    }
    const int got = recvmmsg(fd, hdr, want, MSG_DONTWAIT, nullptr);
    if (got < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      return PHIP_ERR_IO;
    }
    const uint64_t base = pos;
    for (int k = 0; k < got; ++k) {
      const uint32_t len = std::min<uint32_t>(hdr[k].msg_len, PHIP_BUCKET_PACKET_SIZE);
      const uint64_t from = base + (uint64_t)k * PHIP_BUCKET_PACKET_SIZE;
      if (from != pos) std::memmove(bytes + pos, bytes + from, len);   // pos <= from
      pos += len;
      offs[++n] = pos;
    }
    if ((uint32_t)got < want) break;
  }
  *n_out = n;
  return PHIP_OK;
}

int phip_incast_replies(const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                        const uint8_t* status, const phip_state* reply, const uint8_t* peers,
                        uint8_t* out, uint64_t cap, uint64_t* out_offs, uint8_t* out_peers,
                        uint32_t* n_out) {
  if (!n_out) return PHIP_ERR_INVALID;
  *n_out = 0;
  if (n && (!bytes || !offs || !status || !reply || !out || !out_offs)) return PHIP_ERR_INVALID;
  uint64_t pos = 0;
  uint32_t m = 0;
  out_offs[0] = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if ((status[i] & 0x7F) != PHIP_ST_INCAST_REPLY) continue;
    // The name as UnmarshalBinary read it (bucket.go:84-88); the datagram
    // passed the length check, or the status would not be a reply.
    const uint8_t* d = bytes + offs[i];
    const uint32_t len = d[24];
    if (cap - pos < PHIP_BUCKET_FIXED_SIZE + (uint64_t)len) return PHIP_ERR_INVALID;
    const int sz = phip_marshal(d + PHIP_BUCKET_FIXED_SIZE, len, &reply[i], out + pos);
    if (sz < 0) return sz;
    if (peers && out_peers)
      std::memmove(out_peers + (uint64_t)m * PHIP_PEER_BYTES, peers + (uint64_t)i * PHIP_PEER_BYTES,
                  PHIP_PEER_BYTES);
    pos += (uint64_t)sz;
    out_offs[++m] = pos;
  }
  *n_out = m;
  return PHIP_OK;
}

int phip_udp_send_batch(int fd, const uint8_t* bytes, const uint64_t* offs, uint32_t n,
                        const uint8_t* peers, uint32_t peer_stride, uint32_t* sent_out) {
  if (sent_out) *sent_out = 0;
  if (fd < 0 || (n && (!bytes || !offs))) return PHIP_ERR_INVALID;
  mmsghdr hdr[kVec];
  iovec iov[kVec];
  uint32_t done = 0;
  while (done < n) {
    const uint32_t want = std::min<uint32_t>(kVec, n - done);
    std::memset(hdr, 0, sizeof(mmsghdr) * want);
    for (uint32_t k = 0; k < want; ++k) {
      const uint32_t i = done + k;
      iov[k].iov_base = const_cast<uint8_t*>(bytes + offs[i]);
      iov[k].iov_len = offs[i + 1] - offs[i];
      hdr[k].msg_hdr.msg_iov = &iov[k];
      hdr[k].msg_hdr.msg_iovlen = 1;
      if (peers) {
        const uint8_t* pa = peers + (uint64_t)i * peer_stride;
        hdr[k].msg_hdr.msg_name = const_cast<uint8_t*>(pa);
        hdr[k].msg_hdr.msg_namelen = peer_len(pa);
      }
    }
    const int got = sendmmsg(fd, hdr, want, 0);
    if (got < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN || errno == EWOULDBLOCK) {
        pollfd p{fd, POLLOUT, 0};
        poll(&p, 1, 1000);
        continue;
      }
      if (sent_out) *sent_out = done;
      return PHIP_ERR_IO;
    }
    done += (uint32_t)got;
  }
  if (sent_out) *sent_out = done;
  return PHIP_OK;
}

}  // extern "C"

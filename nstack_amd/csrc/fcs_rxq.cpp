// fcs_rxq.cpp — batched RX call site (include/nstack_rxq.h).
//
// Mirrors ether_receive (/root/reference/src/linux/ether.c:180-212) per call while the frames
// arrive in recvmmsg batches and, with FCS_RXQ_TRAILER, are verified on the GPU (CRC residue over
// frame + trailer). Two buffers alternate: while the GPU checks one batch, the next recvmmsg fills
// the other. The CRC itself is never computed here.
#include <arpa/inet.h>
#include <sys/socket.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/nstack_fcs.h"
#include "../../include/nstack_rxq.h"
#include "fcs_device.hpp"

namespace {
constexpr uint32_t kHeaderLen = 14;     // ETHER_HEADER_LEN (src/nstack_ether.h:27)
constexpr uint32_t kFcsLen = 4;         // ETHER_FCS_LEN
constexpr uint32_t kMaxLen = 1514;      // ETHER_MAXLEN: ether_receive's buffer (:183)
constexpr uint32_t kSlot = 2048;        // receive slot: a longer frame shows up as truncated
constexpr uint32_t kMaxBatch = 4096;
}  // namespace

// One receive buffer: recvmmsg slots plus the frame list the verify kernel reads. With the
// trailer flag and pinned memory, every array lives in fcs_host_alloc memory, so the GPU reads
// the list and writes ok[] in place while the host goes on receiving into the other buffer.
struct RxBuf {
    uint8_t *arena = nullptr;           // cap slots of kSlot bytes
    uint64_t *off = nullptr;
    uint32_t *len = nullptr;
    uint8_t *ok = nullptr;
    bool pinned = false;                // all four from fcs_host_alloc
    uint32_t n = 0, next = 0;           // frames in the buffer, next one to hand out
    uint64_t ticket = 0;
    enum State { kEmpty, kInFlight, kReady } state = kEmpty;
};

struct fcs_rxq {
    int fd = -1;
    uint8_t mac[6];
    uint32_t cap = 0, flags = 0;
    bool pipelined = false;             // trailer check overlapped with the next recvmmsg
    RxBuf b[2];
    int cur = 0;                        // the buffer being handed out
    std::vector<mmsghdr> msgs;
    std::vector<iovec> iov;
    uint64_t n_frames = 0, n_bad = 0, n_echo = 0, n_drop = 0, n_batches = 0;
    std::mutex mu;
};

namespace {
void free_buf(RxBuf &B) {
    void *p[4] = {B.arena, B.off, B.len, B.ok};
    for (void *x : p)
        if (x) {
            if (B.pinned) fcs_host_free(x);
            else std::free(x);
        }
    B = RxBuf{};
}

bool alloc_buf(RxBuf &B, uint32_t cap, bool pinned) {
    const uint64_t sz[4] = {(uint64_t)cap * kSlot, (uint64_t)cap * 8, (uint64_t)cap * 4, cap};
    void *p[4] = {};
    for (int i = 0; i < 4; i++) {
        p[i] = pinned ? fcs_host_alloc(sz[i]) : std::malloc(sz[i]);
        if (!p[i]) {
            for (int k = 0; k < i; k++) pinned ? fcs_host_free(p[k]) : std::free(p[k]);
            return false;
        }
    }
    B.arena = (uint8_t *)p[0];
    B.off = (uint64_t *)p[1];
    B.len = (uint32_t *)p[2];
    B.ok = (uint8_t *)p[3];
    B.pinned = pinned;
    return true;
}

// One recvmmsg into B; returns frames received (> 0), 0 for nothing queued, or -errno.
int recv_into(fcs_rxq *q, RxBuf &B, int flags) {
    for (uint32_t i = 0; i < q->cap; i++) {
        q->iov[i] = iovec{B.arena + (uint64_t)i * kSlot, kSlot};
        q->msgs[i] = mmsghdr{};
        q->msgs[i].msg_hdr.msg_iov = &q->iov[i];
        q->msgs[i].msg_hdr.msg_iovlen = 1;
    }
    int r;
    do {
        r = recvmmsg(q->fd, q->msgs.data(), q->cap, flags, nullptr);
    } while (r < 0 && errno == EINTR);
    if (r < 0) {
        if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINPROGRESS) return 0;   // :196-198
        return -errno;
    }
    const uint32_t n = (uint32_t)r;
    const uint32_t tail = (q->flags & FCS_RXQ_TRAILER) ? kFcsLen : 0u;
    for (uint32_t i = 0; i < n; i++) {
        uint32_t L = q->msgs[i].msg_len;
        if ((q->msgs[i].msg_hdr.msg_flags & MSG_TRUNC) || L > kMaxLen + tail || L < kHeaderLen + tail) L = 0;
        B.off[i] = (uint64_t)i * kSlot;
        B.len[i] = L;   // 0: runt or oversize, dropped when handed out
        B.ok[i] = 1;
    }
    q->n_frames += n;
    q->n_batches++;
    B.n = n;
    B.next = 0;
    return (int)n;
}

// Start B's trailer check (pipelined: launch only), or do it at once. No unchecked frame is
// handed out: on failure the batch is dropped and -errno returned.
int start_check(fcs_rxq *q, RxBuf &B) {
    if (!(q->flags & FCS_RXQ_TRAILER)) {
        B.state = RxBuf::kReady;
        return 0;
    }
    if (q->pipelined) {
        const int rc = fcs::mapped_submit(B.arena, (uint64_t)B.n * kSlot, B.off, B.len, B.ok, B.n, &B.ticket);
        if (rc) {
            B.state = RxBuf::kEmpty;
            return rc;
        }
        B.state = RxBuf::kInFlight;
        return 0;
    }
    const int64_t bad = ether_fcs_verify_host(B.arena, (uint64_t)B.n * kSlot, B.off, B.len, B.ok, B.n);
    if (bad < 0) {
        B.state = RxBuf::kEmpty;
        return (int)bad;
    }
    B.state = RxBuf::kReady;
    return 0;
}

int finish_check(RxBuf &B) {
    if (B.state != RxBuf::kInFlight) return 0;
    const int rc = fcs::mapped_wait(B.ticket);
    B.state = rc ? RxBuf::kEmpty : RxBuf::kReady;
    return rc;
}
}  // namespace

extern "C" {

fcs_rxq_t *fcs_rxq_create(int fd, const uint8_t own_mac[6], uint32_t max_batch, uint32_t flags) {
    if (fd < 0 || !own_mac || max_batch == 0 || max_batch > kMaxBatch || (flags & ~FCS_RXQ_TRAILER)) return nullptr;
    fcs_rxq *q = new (std::nothrow) fcs_rxq;
    if (!q) return nullptr;
    q->fd = fd;
    std::memcpy(q->mac, own_mac, 6);
    q->cap = max_batch;
    q->flags = flags;
    // pinned buffers let the GPU read the frames and the list in place; two of them overlap the
    // check of one batch with the recvmmsg of the next
    bool pinned = alloc_buf(q->b[0], max_batch, true) && alloc_buf(q->b[1], max_batch, true);
    if (!pinned) {
        free_buf(q->b[0]);
        free_buf(q->b[1]);
        if (!alloc_buf(q->b[0], max_batch, false) || !alloc_buf(q->b[1], max_batch, false)) {
            free_buf(q->b[0]);
            delete q;
            return nullptr;
        }
    }
    q->pipelined = pinned && (flags & FCS_RXQ_TRAILER);
    q->msgs.resize(max_batch);
    q->iov.resize(max_batch);
    return q;
}

int fcs_rxq_receive(fcs_rxq_t *q, struct fcs_ether_hdr *hdr, uint8_t *buf, size_t bsize) {
    if (!q || !hdr || (!buf && bsize)) return -EINVAL;
    std::lock_guard<std::mutex> lk(q->mu);
    const uint32_t tail = (q->flags & FCS_RXQ_TRAILER) ? kFcsLen : 0u;
    for (;;) {
        RxBuf &B = q->b[q->cur];
        if (B.state == RxBuf::kReady) {
            while (B.next < B.n) {
                const uint32_t i = B.next++;
                const uint32_t L = B.len[i];
                const uint8_t *f = B.arena + B.off[i];
                if (L == 0) { q->n_drop++; continue; }
                if (!std::memcmp(f + 6, q->mac, 6)) { q->n_echo++; continue; }   // own echo (:202)
                if (!B.ok[i]) { q->n_bad++; continue; }
                std::memcpy(hdr->h_dst, f, 6);                                     // :204-206
                std::memcpy(hdr->h_src, f + 6, 6);
                hdr->h_proto = (uint16_t)((f[12] << 8) | f[13]);                   // ntohs
                const uint32_t payload = L - kHeaderLen - tail;
                if (bsize) std::memcpy(buf, f + kHeaderLen, std::min<size_t>(payload, bsize));   // :208-209
                return (int)payload;                                               // :211
            }
            B.state = RxBuf::kEmpty;
        }
        RxBuf &O = q->b[1 - q->cur];
        if (O.state == RxBuf::kInFlight) {
            // the GPU checks O: meanwhile take whatever is already queued into B (no waiting, so
            // O's frames are not held back by a quiet link), then hand out O
            const int r = recv_into(q, B, MSG_DONTWAIT);
            if (r < 0) return r;
            if (r > 0) {
                const int rc = start_check(q, B);
                if (rc) return rc;
            }
            const int rc = finish_check(O);
            if (rc) return rc;
            q->cur = 1 - q->cur;
            continue;
        }
        const int r = recv_into(q, B, MSG_WAITFORONE);   // the socket's own blocking mode
        if (r <= 0) return r;   // 0: nothing queued (:196-198); -errno
        int rc = start_check(q, B);
        if (rc) return rc;
        if (q->pipelined) {   // the next batch, if one is already queued, goes to the GPU behind B
            const int r2 = recv_into(q, O, MSG_DONTWAIT);
            if (r2 > 0 && (rc = start_check(q, O))) {
                finish_check(B);
                B.state = RxBuf::kEmpty;
                return rc;
            }
        }
        if ((rc = finish_check(B))) return rc;
    }
}

void fcs_rxq_stats(const fcs_rxq_t *q, uint64_t *frames, uint64_t *bad_fcs, uint64_t *echoes, uint64_t *dropped,
                   uint64_t *batches) {
    if (!q) return;
    fcs_rxq *m = const_cast<fcs_rxq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (frames) *frames = m->n_frames;
    if (bad_fcs) *bad_fcs = m->n_bad;
    if (echoes) *echoes = m->n_echo;
    if (dropped) *dropped = m->n_drop;
    if (batches) *batches = m->n_batches;
}

void fcs_rxq_destroy(fcs_rxq_t *q) {
    if (!q) return;
    for (RxBuf &B : q->b) {
        finish_check(B);   // the GPU may still be writing ok[] of an in-flight batch
        free_buf(B);
    }
    delete q;
}

}  // extern "C"

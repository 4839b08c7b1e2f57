// fcs_rxq.cpp — batched RX call site (include/nstack_rxq.h).
//
// Mirrors ether_receive (/root/reference/src/linux/ether.c:180-212) per call while the frames
// arrive in recvmmsg batches and, with FCS_RXQ_TRAILER, are verified on the GPU one batch at a
// time (ether_fcs_verify_host: CRC residue over frame + trailer). The CRC itself is never computed
// here.
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

namespace {
constexpr uint32_t kHeaderLen = 14;     // ETHER_HEADER_LEN (src/nstack_ether.h:27)
constexpr uint32_t kFcsLen = 4;         // ETHER_FCS_LEN
constexpr uint32_t kMaxLen = 1514;      // ETHER_MAXLEN: ether_receive's buffer (:183)
constexpr uint32_t kSlot = 2048;        // receive slot: a longer frame shows up as truncated
constexpr uint32_t kMaxBatch = 4096;
}  // namespace

struct fcs_rxq {
    int fd = -1;
    uint8_t mac[6];
    uint32_t cap = 0, flags = 0;
    uint8_t *arena = nullptr;           // cap slots of kSlot bytes, pinned (fcs_host_alloc) if possible
    bool pinned = false;
    std::vector<mmsghdr> msgs;
    std::vector<iovec> iov;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len;
    std::vector<uint8_t> ok;
    uint32_t n = 0, next = 0;           // the batch being handed out
    uint64_t n_frames = 0, n_bad = 0, n_echo = 0, n_drop = 0, n_batches = 0;
    std::mutex mu;
};

namespace {
// One recvmmsg into the arena; returns frames received (> 0), 0 for nothing queued, or -errno.
int refill(fcs_rxq *q) {
    for (uint32_t i = 0; i < q->cap; i++) {
        q->iov[i] = iovec{q->arena + (uint64_t)i * kSlot, kSlot};
        q->msgs[i] = mmsghdr{};
        q->msgs[i].msg_hdr.msg_iov = &q->iov[i];
        q->msgs[i].msg_hdr.msg_iovlen = 1;
    }
    int r;
    do {
        r = recvmmsg(q->fd, q->msgs.data(), q->cap, MSG_WAITFORONE, nullptr);
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
        q->off[i] = (uint64_t)i * kSlot;
        q->len[i] = L;   // 0: runt or oversize, dropped when handed out
        q->ok[i] = 1;
    }
    q->n_frames += n;
    q->n_batches++;
    if (tail) {   // one GPU call verifies the whole batch (frame + trailer must leave the residue)
        const int64_t bad = ether_fcs_verify_host(q->arena, (uint64_t)n * kSlot, q->off.data(), q->len.data(),
                                                  q->ok.data(), n);
        if (bad < 0) return (int)bad;   // no unchecked frame is handed out
    }
    q->n = n;
    q->next = 0;
    return (int)n;
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
    const uint64_t bytes = (uint64_t)max_batch * kSlot;
    q->arena = (uint8_t *)fcs_host_alloc(bytes);   // pinned: the verify DMA reads it directly
    q->pinned = q->arena != nullptr;
    if (!q->arena) q->arena = (uint8_t *)std::malloc(bytes);
    if (!q->arena) {
        delete q;
        return nullptr;
    }
    q->msgs.resize(max_batch);
    q->iov.resize(max_batch);
    q->off.resize(max_batch);
    q->len.resize(max_batch);
    q->ok.resize(max_batch);
    return q;
}

int fcs_rxq_receive(fcs_rxq_t *q, struct fcs_ether_hdr *hdr, uint8_t *buf, size_t bsize) {
    if (!q || !hdr || (!buf && bsize)) return -EINVAL;
    std::lock_guard<std::mutex> lk(q->mu);
    const uint32_t tail = (q->flags & FCS_RXQ_TRAILER) ? kFcsLen : 0u;
    for (;;) {
        while (q->next < q->n) {
            const uint32_t i = q->next++;
            const uint32_t L = q->len[i];
            const uint8_t *f = q->arena + q->off[i];
            if (L == 0) { q->n_drop++; continue; }
            if (!std::memcmp(f + 6, q->mac, 6)) { q->n_echo++; continue; }   // own echo (:202)
            if (!q->ok[i]) { q->n_bad++; continue; }
            std::memcpy(hdr->h_dst, f, 6);                                     // :204-206
            std::memcpy(hdr->h_src, f + 6, 6);
            hdr->h_proto = (uint16_t)((f[12] << 8) | f[13]);                   // ntohs
            const uint32_t payload = L - kHeaderLen - tail;
            if (bsize) std::memcpy(buf, f + kHeaderLen, std::min<size_t>(payload, bsize));   // :208-209
            return (int)payload;                                               // :211
        }
        const int r = refill(q);
        if (r <= 0) return r;   // 0: nothing queued (:196-198); -errno
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
    if (q->arena) {
        if (q->pinned) fcs_host_free(q->arena);
        else std::free(q->arena);
    }
    delete q;
}

}  // extern "C"

// fcs_rxq.cpp — batched RX call site (include/nstack_rxq.h).
//
// Mirrors ether_receive (/root/reference/src/linux/ether.c:180-212) per call while the frames
// arrive in recvmmsg batches and, with FCS_RXQ_TRAILER, are verified on the GPU (CRC residue over
// frame + trailer). Two buffers alternate: while the GPU checks one batch, the next recvmmsg fills
// the other. ether_receive never fails or drops frames for FCS reasons, so when the GPU check of a
// batch fails (HIP error, timeout, no GPU) the library's host CRC checks it instead
// (fcs_host_crc.cpp), counted per queue and in fcs_engine_host_batches: the
// synchronous ether_fcs_verify_host answers a failed GPU step itself; a failed pipelined check
// (mapped_submit / mapped_wait) or no usable GPU at all is answered here.
//
// A batch whose frames total at most host_max bytes is checked by the host CRC on the receiving
// thread, by design (counted in fcs_rxq_small_batches, not as a failure): recvmmsg has just copied
// its frames there, so they are cache-hot, and the host CRC (four-lane carry-less folding, ~32 ns
// per 1518-B frame on one MI355X-box core) beats a GPU step's launch and completion round trip on
// small batches. Larger batches go to the GPU, whose check overlaps the next recvmmsg. The scan of
// tools/rxq_host_max_scan.sh (profiles/r06_rxq_host_max_scan.jsonl, medians of three, M frames/s):
// 64 x 1518 B (97 KB) 2.85 on the host against 2.69 on the GPU; 256 x 1518 B (389 KB) 2.93 with
// 256 KiB against 2.73 with 1 MiB (the batch on the host); 46-B payloads flat from 64 KiB up.
// Hence 256 KiB.
#include <arpa/inet.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <utility>
#include <vector>

#include "../../include/nstack_fcs.h"
#include "../../include/nstack_rxq.h"
#include "fcs_device.hpp"
#include "fcs_host_crc.hpp"

namespace {
constexpr uint32_t kHeaderLen = 14;     // ETHER_HEADER_LEN (src/nstack_ether.h:27)
constexpr uint32_t kFcsLen = 4;         // ETHER_FCS_LEN
constexpr uint32_t kMaxLen = 1514;      // ETHER_MAXLEN: ether_receive's buffer (:183)
constexpr uint32_t kSlot = 2048;        // receive slot: a longer frame shows up as truncated
constexpr uint32_t kMaxBatch = 4096;
constexpr uint32_t kResidue = 0x2144DF1Cu;   // CRC-32 of any frame followed by its own LE FCS
constexpr size_t kMaxPinnedSpares = 64;   // pinned ok arrays taken to replace set-aside ones (then malloc'd)
constexpr uint64_t kRxHostMaxDefault = 256 * 1024;   // see the file comment
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
    bool ok_pinned = false;             // ok from fcs_host_alloc (it may be replaced, see host_check)
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
    uint64_t n_host_batches = 0, n_host_frames = 0;   // batches the host CRC checked after a failure
    uint64_t n_small_batches = 0, n_small_frames = 0, n_gpu_batches = 0;   // by design / on the GPU
    std::atomic<uint64_t> host_max{kRxHostMaxDefault};   // see fcs_rxq_set_host_max
    // ok arrays of pipelined batches whose check failed after its launch: the kernel may still write
    // them, so they are never reused before fcs_rxq_destroy, whatever else fails (every one is set
    // aside; their number is bounded because the engine stops launching after repeated failures).
    std::vector<std::pair<uint8_t *, bool>> quarantine;   // (array, from fcs_host_alloc)
    size_t pinned_spares = 0;
    // One malloc'd ok array per buffer, taken when no fresh array can be allocated: a buffer that
    // gets a non-pinned array is checked synchronously from then on, so it needs at most one.
    uint8_t *spare[2] = {nullptr, nullptr};
    std::mutex mu;
};

namespace {
void free_buf(RxBuf &B) {
    void *p[4] = {B.arena, B.off, B.len, B.ok};
    for (int i = 0; i < 4; i++)
        if (p[i]) {
            if (i == 3 ? B.ok_pinned : B.pinned) fcs_host_free(p[i]);
            else std::free(p[i]);
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
    B.ok_pinned = pinned;
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

void count_host(fcs_rxq *q, RxBuf &B) {
    q->n_host_batches++;
    q->n_host_frames += B.n;
}

// The GPU check of B failed or could not run: check it with the host CRC instead (SURVEY.md §8b;
// ether_receive never drops a frame for FCS reasons). launched: a pipelined check of B was launched
// and its wait failed, so that kernel may still write B.ok: the array is set aside in every case
// and B gets a fresh one (pinned while spares last, so B stays pipelined; else malloc'd, and B's
// later checks go through the synchronous ether_fcs_verify_host, which never lets a kernel write
// into the caller's array).
void host_check(fcs_rxq *q, RxBuf &B, bool launched) {
    const char *why = fcs_last_error();
    if (launched) {
        uint8_t *fresh = nullptr;
        if (B.ok_pinned && q->pinned_spares < kMaxPinnedSpares && (fresh = (uint8_t *)fcs_host_alloc(q->cap)))
            q->pinned_spares++;
        const bool fresh_pinned = fresh != nullptr;
        if (!fresh) fresh = (uint8_t *)std::malloc(q->cap);
        q->quarantine.emplace_back(B.ok, B.ok_pinned);
        if (!fresh) std::swap(fresh, q->spare[&B == &q->b[1]]);   // allocation failed: the buffer's spare
        B.ok = fresh;
        B.ok_pinned = fresh_pinned;
    }
    for (uint32_t i = 0; i < B.n; i++) {
        const uint32_t L = B.len[i];   // 0: runt or oversize, dropped anyway
        B.ok[i] = L >= kFcsLen && fcs::host_crc32(B.arena + B.off[i], L) == kResidue;
    }
    fcs::host_batch_answered("fcs_rxq_receive", why);
    count_host(q, B);
    B.state = RxBuf::kReady;
}

// Start B's trailer check (pipelined: launch only), or do it at once. Every frame handed out has
// been checked, by the GPU or the host CRC (by design below the GPU minimum, or when a GPU step
// failed).
void start_check(fcs_rxq *q, RxBuf &B) {
    if (!(q->flags & FCS_RXQ_TRAILER)) {
        B.state = RxBuf::kReady;
        return;
    }
    uint64_t bytes = 0;
    for (uint32_t i = 0; i < B.n; i++) bytes += B.len[i];
    if (bytes <= q->host_max.load(std::memory_order_relaxed)) {   // below the GPU minimum: the frames are cache-hot on this thread
        for (uint32_t i = 0; i < B.n; i++) {
            const uint32_t L = B.len[i];   // 0: runt or oversize, dropped anyway
            B.ok[i] = L >= kFcsLen && fcs::host_crc32(B.arena + B.off[i], L) == kResidue;
        }
        q->n_small_batches++;
        q->n_small_frames += B.n;
        B.state = RxBuf::kReady;
        return;
    }
    q->n_gpu_batches++;
    if (q->pipelined && B.ok_pinned) {
        if (fcs::mapped_submit(B.arena, (uint64_t)B.n * kSlot, B.off, B.len, B.ok, B.n, &B.ticket))
            return host_check(q, B, false);   // nothing launched
        B.state = RxBuf::kInFlight;
        return;
    }
    const int64_t bad = ether_fcs_verify_host(B.arena, (uint64_t)B.n * kSlot, B.off, B.len, B.ok, B.n);
    if (bad < 0) return host_check(q, B, false);   // no usable GPU: nothing ran
    if (fcs::last_call_host_answered()) count_host(q, B);   // the engine answered a failed GPU step
    B.state = RxBuf::kReady;
}

void finish_check(fcs_rxq *q, RxBuf &B) {
    if (B.state != RxBuf::kInFlight) return;
    if (fcs::mapped_wait(B.ticket)) return host_check(q, B, true);
    B.state = RxBuf::kReady;
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
    if (const char *e = std::getenv("NSTACK_RXQ_HOST_MAX_BYTES")) q->host_max.store(std::strtoull(e, nullptr, 0));
    for (uint8_t *&sp : q->spare)
        if (!(sp = (uint8_t *)std::malloc(max_batch))) {
            fcs_rxq_destroy(q);
            return nullptr;
        }
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
        if (O.state == RxBuf::kReady) {   // received after B and already checked (by the host CRC)
            q->cur = 1 - q->cur;
            continue;
        }
        if (O.state == RxBuf::kInFlight) {
            // the GPU checks O: meanwhile take whatever is already queued into B (no waiting, so
            // O's frames are not held back by a quiet link), then hand out O
            const int r = recv_into(q, B, MSG_DONTWAIT);
            if (r < 0) {
                finish_check(q, O);   // O's frames stay queued for the next call
                q->cur = 1 - q->cur;
                return r;
            }
            if (r > 0) start_check(q, B);
            finish_check(q, O);
            q->cur = 1 - q->cur;
            continue;
        }
        const int r = recv_into(q, B, MSG_WAITFORONE);   // the socket's own blocking mode
        if (r <= 0) return r;   // 0: nothing queued (:196-198); -errno
        start_check(q, B);
        if (q->pipelined) {   // the next batch, if one is already queued, goes to the GPU behind B
            const int r2 = recv_into(q, O, MSG_DONTWAIT);
            if (r2 > 0) start_check(q, O);
        }
        finish_check(q, B);
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

uint64_t fcs_rxq_set_host_max(fcs_rxq_t *q, uint64_t bytes) {
    if (!q) return 0;
    return q->host_max.exchange(bytes);   // not under mu: a receive may be blocked in recvmmsg
}

void fcs_rxq_small_batches(const fcs_rxq_t *q, uint64_t *small_batches, uint64_t *small_frames,
                           uint64_t *gpu_batches) {
    if (!q) return;
    fcs_rxq *m = const_cast<fcs_rxq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (small_batches) *small_batches = m->n_small_batches;
    if (small_frames) *small_frames = m->n_small_frames;
    if (gpu_batches) *gpu_batches = m->n_gpu_batches;
}

void fcs_rxq_fallbacks(const fcs_rxq_t *q, uint64_t *host_batches, uint64_t *host_frames) {
    if (!q) return;
    fcs_rxq *m = const_cast<fcs_rxq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (host_batches) *host_batches = m->n_host_batches;
    if (host_frames) *host_frames = m->n_host_frames;
}

void fcs_rxq_destroy(fcs_rxq_t *q) {
    if (!q) return;
    for (RxBuf &B : q->b) {
        finish_check(q, B);   // the GPU may still be writing ok[] of an in-flight batch
        free_buf(B);
    }
    for (auto &x : q->quarantine) x.second ? fcs_host_free(x.first) : std::free(x.first);
    for (uint8_t *sp : q->spare) std::free(sp);
    delete q;
}

}  // extern "C"

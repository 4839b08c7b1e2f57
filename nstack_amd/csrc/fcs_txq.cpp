// fcs_txq.cpp — batched TX call site (include/nstack_txq.h).
//
// Mirrors ether_send (/root/reference/src/linux/ether.c:214-272) per call — frame layout
// (:257-263), -EMSGSIZE rule (:222-224, :234-237), per-call return value (:265-269) — while the
// FCS of every frame queued by any thread is computed in one GPU batch (ether_fcs_tx_host) and
// the batch is handed to the sink at once (sendmmsg). The CRC itself is never computed here.
#include <arpa/inet.h>
#include <linux/if_packet.h>
#include <sys/socket.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/nstack_fcs.h"
#include "../../include/nstack_txq.h"

namespace {

constexpr uint32_t kHeaderLen = 14;     // ETHER_HEADER_LEN (src/nstack_ether.h:27)
constexpr uint32_t kMinPayload = 56;    // ETHER_MINLEN - ETHER_FCS_LEN (:28-31; ether.c:223)
constexpr uint32_t kFcsLen = 4;         // ETHER_FCS_LEN
constexpr uint32_t kSlot = 1518;        // ETHER_MAXLEN + ETHER_FCS_LEN: largest frame_size
constexpr uint32_t kMaxBatch = 65536;

using Clock = std::chrono::steady_clock;

struct Waiter {
    int result = 0;
    std::atomic<bool> done{false};   // set last by the flusher; the producer may be spinning on it
};

// Hand-offs spin this long before sleeping on a condition variable: a futex wake-up costs tens of
// microseconds, more than the GPU step of a small batch.
constexpr auto kSpin = std::chrono::microseconds(50);

inline void cpu_relax() { __builtin_ia32_pause(); }

struct Batch {
    uint8_t *arena = nullptr;            // cap slots of kSlot bytes (pinned when possible)
    bool pinned = false;
    std::vector<uint32_t> covered;       // FCS-covered bytes (frame_size - 4) per slot
    std::vector<uint32_t> sizes;         // frame_size per slot
    std::vector<uint8_t *> frames;
    std::vector<int> res;
    std::vector<Waiter *> waiters;
    uint32_t reserved = 0;               // slots handed out (under fcs_txq::mu)
    std::atomic<uint32_t> ready{0};      // slots fully assembled by their producers
    uint64_t seq = 0;
    Clock::time_point first;
};

}  // namespace

struct fcs_txq {
    uint8_t mac[6];
    uint32_t cap = 0, flush_usec = 0;
    fcs_txq_sink_fn sink = nullptr;
    void *ctx = nullptr;
    std::mutex mu;
    std::condition_variable cv_flusher;   // producers / flush() -> flusher
    std::condition_variable cv_prod;      // flusher -> producers (batch swapped, results ready)
    Batch b[2];
    int open = 0;                         // producers fill b[open]
    uint64_t seq_done = 0;                // last batch handed to the sink
    uint64_t flush_target = 0;            // flush() wants batches <= this closed now
    bool stop = false;
    uint64_t n_frames = 0, n_batches = 0, n_errors = 0;
    uint64_t ns_ready = 0, ns_gpu = 0, ns_sink = 0, ns_busy = 0;   // flusher time split
    uint64_t ns_pickup = 0;               // first frame of a batch queued -> batch closed
    std::atomic<uint32_t> queued{0};      // frames reserved in the open batch (mirror, for spinning)
    std::atomic<bool> stop_req{false};    // mirror of stop for the spinning flusher
    std::thread th;
};

namespace {

void flusher(fcs_txq *q) {
    std::unique_lock<std::mutex> lk(q->mu);
    for (;;) {
        Batch *B = &q->b[q->open];
        for (;;) {
            if (B->reserved == q->cap || q->stop) break;
            if (B->reserved > 0 && (q->flush_usec == 0 || q->flush_target >= B->seq)) break;
            if (B->reserved > 0) {
                // linger for company. Short lingers spin: a timed futex sleep is rounded up by the
                // kernel's timer slack (50 us by default), longer than the whole GPU step.
                const auto deadline = B->first + std::chrono::microseconds(q->flush_usec);
                if (q->flush_usec <= 1000) {
                    lk.unlock();
                    while (Clock::now() < deadline && q->queued.load(std::memory_order_acquire) < q->cap &&
                           !q->stop_req.load(std::memory_order_acquire))
                        cpu_relax();
                    lk.lock();
                } else {
                    q->cv_flusher.wait_until(lk, deadline);
                }
                if (B->reserved == q->cap || q->stop || Clock::now() >= deadline || q->flush_target >= B->seq) break;
                continue;
            }
            // idle: spin a little for the next frame, then sleep until a producer or flush() calls
            lk.unlock();
            const auto until = Clock::now() + kSpin;
            while (q->queued.load(std::memory_order_acquire) == 0 && Clock::now() < until &&
                   !q->stop_req.load(std::memory_order_acquire))
                cpu_relax();
            lk.lock();
            if (B->reserved == 0 && !q->stop && q->flush_target < B->seq) q->cv_flusher.wait(lk);
        }
        if (B->reserved == 0) {   // stop requested and nothing left
            q->seq_done = B->seq - 1;
            q->cv_prod.notify_all();
            break;
        }
        // close B; producers move on to the other buffer
        const uint32_t n = B->reserved;
        q->ns_pickup += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - B->first).count();
        q->open ^= 1;
        Batch &N = q->b[q->open];
        N.reserved = 0;
        N.ready.store(0, std::memory_order_relaxed);
        N.seq = B->seq + 1;
        q->queued.store(0, std::memory_order_relaxed);
        q->cv_prod.notify_all();
        lk.unlock();

        const auto t0 = Clock::now();
        while (B->ready.load(std::memory_order_acquire) < n) std::this_thread::yield();
        const auto t1 = Clock::now();
        // FCS of every frame, written little-endian after its covered bytes (ether.c:262-263)
        const int rc = ether_fcs_tx_host(B->arena, kSlot, B->covered.data(), n);
        const auto t2 = Clock::now();
        if (rc == 0) {
            for (uint32_t i = 0; i < n; i++) {
                B->frames[i] = B->arena + (uint64_t)i * kSlot;
                B->sizes[i] = B->covered[i] + kFcsLen;
                B->res[i] = -EIO;   // a sink that forgets a frame reports it as failed
            }
            q->sink(q->ctx, B->frames.data(), B->sizes.data(), B->res.data(), n);
        } else {
            for (uint32_t i = 0; i < n; i++) B->res[i] = rc;   // nothing leaves unchecked
        }
        const auto t3 = Clock::now();

        lk.lock();
        auto ns = [](Clock::duration d) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
        q->ns_ready += ns(t1 - t0);
        q->ns_gpu += ns(t2 - t1);
        q->ns_sink += ns(t3 - t2);
        q->ns_busy += ns(Clock::now() - t0);
        for (uint32_t i = 0; i < n; i++) {
            if (B->res[i] != (int)(B->covered[i] + kFcsLen)) q->n_errors++;
            if (Waiter *w = B->waiters[i]) {   // null: fcs_txq_send_async
                w->result = B->res[i];
                w->done.store(true, std::memory_order_release);   // last touch: w may vanish now
            }
        }
        q->seq_done = B->seq;
        q->n_frames += n;
        q->n_batches++;
        q->cv_prod.notify_all();
    }
}

}  // namespace

extern "C" {

fcs_txq_t *fcs_txq_create(const uint8_t src_mac[6], uint32_t max_batch, uint32_t flush_usec,
                          fcs_txq_sink_fn sink, void *sink_ctx) {
    if (!src_mac || !sink || max_batch == 0 || max_batch > kMaxBatch) return nullptr;
    fcs_txq *q = new (std::nothrow) fcs_txq;
    if (!q) return nullptr;
    std::memcpy(q->mac, src_mac, 6);
    q->cap = max_batch;
    q->flush_usec = flush_usec;
    q->sink = sink;
    q->ctx = sink_ctx;
    for (int k = 0; k < 2; k++) {
        Batch &B = q->b[k];
        const uint64_t bytes = (uint64_t)max_batch * kSlot;
        B.arena = (uint8_t *)fcs_host_alloc(bytes);   // pinned: direct H2D
        B.pinned = B.arena != nullptr;
        if (!B.arena) B.arena = (uint8_t *)std::malloc(bytes);   // no GPU runtime: sends will fail
        if (!B.arena) {
            fcs_txq_destroy(q);
            return nullptr;
        }
        B.covered.assign(max_batch, 0);
        B.sizes.assign(max_batch, 0);
        B.frames.assign(max_batch, nullptr);
        B.res.assign(max_batch, 0);
        B.waiters.assign(max_batch, nullptr);
    }
    q->b[0].seq = 1;
    q->th = std::thread(flusher, q);
    return q;
}

}  // extern "C"

namespace {
// Reserve a slot in the open batch, assemble the frame there (outside the lock) and mark it
// ready. w == nullptr: fire-and-forget (the result only feeds the error counter).
int enqueue(fcs_txq *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize, Waiter *w) {
    if (!q || !dst || (!buf && bsize)) return -EINVAL;
    const size_t frame_size = kHeaderLen + std::max<size_t>(bsize, kMinPayload) + kFcsLen;   // :222-224
    if (frame_size > kSlot) return -EMSGSIZE;                                                // :234-237
    std::unique_lock<std::mutex> lk(q->mu);
    while (!q->stop && q->b[q->open].reserved == q->cap) {   // batch full: wait for the swap
        q->cv_flusher.notify_one();
        q->cv_prod.wait(lk);
    }
    if (q->stop) return -ESHUTDOWN;
    Batch &B = q->b[q->open];
    const uint32_t slot = B.reserved++;
    if (slot == 0) B.first = Clock::now();
    B.waiters[slot] = w;
    q->queued.store(B.reserved, std::memory_order_release);
    if (slot == 0 || B.reserved == q->cap) q->cv_flusher.notify_one();
    lk.unlock();

    // assemble exactly as ether_send (:257-261): dst, src, htons(proto), payload, zero pad and
    // zeroed FCS slot; the engine fills the FCS (:262-263)
    uint8_t *f = B.arena + (uint64_t)slot * kSlot;
    std::memcpy(f, dst, 6);
    std::memcpy(f + 6, q->mac, 6);
    f[12] = (uint8_t)(proto >> 8);
    f[13] = (uint8_t)proto;
    if (bsize) std::memcpy(f + kHeaderLen, buf, bsize);
    std::memset(f + kHeaderLen + bsize, 0, frame_size - kHeaderLen - bsize);
    B.covered[slot] = (uint32_t)(frame_size - kFcsLen);
    B.ready.fetch_add(1, std::memory_order_release);
    return (int)frame_size;
}
}  // namespace

extern "C" {

int fcs_txq_send(fcs_txq_t *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize) {
    Waiter w;
    const int rc = enqueue(q, dst, proto, buf, bsize, &w);
    if (rc < 0) return rc;
    const auto until = Clock::now() + kSpin;
    while (!w.done.load(std::memory_order_acquire) && Clock::now() < until) cpu_relax();
    if (!w.done.load(std::memory_order_acquire)) {
        std::unique_lock<std::mutex> lk(q->mu);
        while (!w.done.load(std::memory_order_acquire)) q->cv_prod.wait(lk);
    }
    return w.result;
}

int fcs_txq_send_async(fcs_txq_t *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize) {
    return enqueue(q, dst, proto, buf, bsize, nullptr);
}

int fcs_txq_flush(fcs_txq_t *q) {
    if (!q) return -EINVAL;
    std::unique_lock<std::mutex> lk(q->mu);
    const Batch &B = q->b[q->open];
    const uint64_t target = B.reserved ? B.seq : B.seq - 1;   // the open batch, else the one in flight
    q->flush_target = std::max(q->flush_target, target);
    q->cv_flusher.notify_one();
    while (q->seq_done < target) q->cv_prod.wait(lk);
    return 0;
}

void fcs_txq_destroy(fcs_txq_t *q) {
    if (!q) return;
    if (q->th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(q->mu);
            q->stop = true;
            q->stop_req.store(true, std::memory_order_release);
        }
        q->cv_flusher.notify_one();
        q->th.join();
    }
    for (int k = 0; k < 2; k++) {
        Batch &B = q->b[k];
        if (B.arena) {
            if (B.pinned) fcs_host_free(B.arena);
            else std::free(B.arena);
        }
    }
    delete q;
}

void fcs_txq_stats(const fcs_txq_t *q, uint64_t *frames, uint64_t *batches, uint64_t *errors) {
    if (!q) return;
    fcs_txq *m = const_cast<fcs_txq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (frames) *frames = m->n_frames;
    if (batches) *batches = m->n_batches;
    if (errors) *errors = m->n_errors;
}

void fcs_txq_timing(const fcs_txq_t *q, uint64_t *ns_ready, uint64_t *ns_gpu, uint64_t *ns_sink,
                    uint64_t *ns_busy, uint64_t *ns_pickup) {
    if (!q) return;
    fcs_txq *m = const_cast<fcs_txq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (ns_ready) *ns_ready = m->ns_ready;
    if (ns_gpu) *ns_gpu = m->ns_gpu;
    if (ns_sink) *ns_sink = m->ns_sink;
    if (ns_busy) *ns_busy = m->ns_busy;
    if (ns_pickup) *ns_pickup = m->ns_pickup;
}

// ---- sinks ----
namespace {
void send_batch(int fd, std::vector<mmsghdr> &m, uint32_t n, int *res) {
    uint32_t i = 0;
    while (i < n) {
        const int r = sendmmsg(fd, &m[i], n - i, 0);
        if (r < 0) {
            if (errno == EINTR) continue;
            res[i] = -errno;   // as ether_send's sendto failure (:267-269); go on with the rest
            i++;
            continue;
        }
        for (int k = 0; k < r; k++) res[i + k] = (int)m[i + k].msg_len;
        i += (uint32_t)r;
    }
}
}  // namespace

void fcs_txq_sink_fd(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n) {
    const int fd = *(const int *)ctx;
    static thread_local std::vector<mmsghdr> m;
    static thread_local std::vector<iovec> iov;
    m.assign(n, mmsghdr{});
    iov.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        iov[i] = iovec{frames[i], sizes[i]};
        m[i].msg_hdr.msg_iov = &iov[i];
        m[i].msg_hdr.msg_iovlen = 1;
    }
    send_batch(fd, m, n, res);
}

void fcs_txq_sink_packet(void *ctx, uint8_t *const *frames, const uint32_t *sizes, int *res, uint32_t n) {
    const fcs_txq_packet_ctx *pc = (const fcs_txq_packet_ctx *)ctx;
    static thread_local std::vector<mmsghdr> m;
    static thread_local std::vector<iovec> iov;
    static thread_local std::vector<sockaddr_ll> sa;
    m.assign(n, mmsghdr{});
    iov.resize(n);
    sa.assign(n, sockaddr_ll{});
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *f = frames[i];
        sockaddr_ll &a = sa[i];   // as ether_send's socket_address (:241-253), from the header
        a.sll_family = AF_PACKET;
        a.sll_protocol = htons((uint16_t)((f[12] << 8) | f[13]));
        a.sll_ifindex = pc->ifindex;
        a.sll_halen = 6;
        std::memcpy(a.sll_addr, f, 6);
        iov[i] = iovec{frames[i], sizes[i]};
        m[i].msg_hdr.msg_name = &a;
        m[i].msg_hdr.msg_namelen = sizeof(sockaddr_ll);
        m[i].msg_hdr.msg_iov = &iov[i];
        m[i].msg_hdr.msg_iovlen = 1;
    }
    send_batch(pc->fd, m, n, res);
}

}  // extern "C"

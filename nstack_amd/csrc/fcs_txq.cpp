// fcs_txq.cpp — batched TX call site (include/nstack_txq.h).
//
// Mirrors ether_send (/root/reference/src/linux/ether.c:214-272) per call — frame layout
// (:257-263), -EMSGSIZE rule (:222-224, :234-237), per-call return value (:265-269) — while the
// FCS of every frame queued by any thread is computed in one GPU batch (ether_fcs_tx_batch_host)
// and the batch is handed to the sink at once (sendmmsg). ether_send never fails for FCS reasons, so
// when the GPU step fails the batch's FCSs come from the library's host CRC (fcs_host_crc.cpp,
// SURVEY.md §8b): ether_fcs_tx_batch_host answers a failed GPU step itself, and without any usable
// GPU (-ENODEV) the queue does; either way counted per queue and in fcs_engine_host_batches, and the
// frames still leave. The engine never leaves a kernel that can write into the arena after a failed
// call (its results go through the library's own mapped memory), so arenas are always reused.
//
// Where the GPU does not pay, the host CRC (fcs_host_crc.cpp, carry-less folding, ~47 GB/s on 1518-B
// frames on one MI355X-box core) computes the FCS by design (counted in fcs_txq_small_batches, not as a failure).
// Measured on MI355X boxes (profiles/r06_txq_vs_reference.jsonl): a GPU step costs a launch and a
// completion round trip (9-12 us) whatever it holds, and a hand-off between threads costs 1-2 us,
// while the reference's own per-frame CRC costs 4.8 us per 1518-B frame and 0.2 us per 60-B one.
// - A synchronous caller (fcs_txq_send) with none of its own frames still queued sends its frame
//   itself: ether_send's body with the host CRC, the sink called with a batch of one on its own
//   thread (sinks are thread-safe, as the reference's concurrent sendto calls are). Its frames keep
//   their order (nothing of its own is queued), and it never waits for a batch it has no use for.
//   A synchronous caller with fire-and-forget frames still queued joins the batch behind them and
//   computes its own frame's FCS there (cache-hot, in parallel with the other callers).
//   fcs_txq_set_sync_host(q, 0) sends synchronous frames through the batch and its GPU step instead.
// - Fire-and-forget frames (fcs_txq_send_async) take one GPU step per batch when their covered bytes
//   exceed host_max, the GPU minimum; at or below it the flusher computes them. Its frames are cold
//   in the flusher's cache (the producers wrote them), and a fast host answer keeps the next batch
//   small, so the in-queue scan favours the GPU from about ten full frames up: the default is 16 KiB.
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
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/nstack_fcs.h"
#include "../../include/nstack_txq.h"
#include "fcs_device.hpp"
#include "fcs_host_crc.hpp"

namespace {

constexpr uint32_t kHeaderLen = 14;     // ETHER_HEADER_LEN (src/nstack_ether.h:27)
constexpr uint32_t kMinPayload = 56;    // ETHER_MINLEN - ETHER_FCS_LEN (:28-31; ether.c:223)
constexpr uint32_t kFcsLen = 4;         // ETHER_FCS_LEN
constexpr uint32_t kSlot = 1518;        // ETHER_MAXLEN + ETHER_FCS_LEN: largest frame_size
constexpr uint32_t kStride = 1536;      // arena slot pitch: whole cache lines, so producers filling
                                        // neighbouring slots never share a line
constexpr uint32_t kMaxBatch = 65536;
// Fire-and-forget batches of at most this many covered bytes take the host CRC (see the file
// comment). tools/tx_crossover.c puts the crossover at ~500 KB when the host CRC reads cache-hot
// frames; in the queue they are cold, and batches that take the host path stay small. The scan of
// fire-and-forget producers (tools/txq_vs_reference.sh, profiles/r06_txq_vs_reference.jsonl):
// 1518-B frames as fast at 4-32 KiB as with every batch on the GPU, slower from 128 KiB; 78-B
// frames 3x faster at 8-32 KiB (small batches answered at once, large ones on the GPU).
constexpr uint64_t kHostMaxDefault = 16 * 1024;

using Clock = std::chrono::steady_clock;

struct Waiter {
    int result = 0;
    std::atomic<bool> done{false};   // set last by the flusher; the producer may be spinning on it
};

// Hand-offs spin this long before sleeping on a condition variable: a futex wake-up costs tens of
// microseconds, more than the GPU step of a small batch.
constexpr auto kSpin = std::chrono::microseconds(50);

inline void cpu_relax() { __builtin_ia32_pause(); }

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch()).count();
}

// What a producer leaves for the flusher in its slot. `ready` = the batch sequence number once
// the frame is assembled, so the flag needs no reset between uses of the buffer.
struct alignas(64) SlotMeta {
    Waiter *w = nullptr;                 // null: fcs_txq_send_async
    uint32_t covered = 0;
    bool has_fcs = false;                // the sync caller computed it (host CRC, frame cache-hot)
    std::atomic<uint64_t> ready{0};
};

struct Batch {
    uint8_t *arena = nullptr;            // cap slots of kStride bytes (pinned when possible);
    bool pinned = false;                 //   shard k owns slots [k * per, (k + 1) * per)
    std::vector<SlotMeta> meta;          // per slot, one cache line each (written by its producer)
    // the frames that leave, in shard order (filled by the flusher)
    std::vector<uint32_t> slot;          // arena slot of each
    std::vector<uint64_t> off;           // its byte offset in the arena
    std::vector<uint32_t> covered;       // FCS-covered bytes (frame_size - 4)
    std::vector<uint64_t> need_off;      // the frames that still need their FCS (the GPU step's list)
    std::vector<uint32_t> need_len;
    std::vector<uint32_t> sizes;         // frame_size
    std::vector<uint8_t *> frames;
    std::vector<int> res;
    std::atomic<int64_t> first_ns{0};    // when the batch's first frame was reserved (0: not yet)
};

// A shard's open batch and its fill level in one word, so producers reserve slots with one atomic
// add and no lock: bits 63..32 = batch sequence number (the batch lives in b[seq & 1]), 31..0 =
// slots reserved. The flusher closes a batch by swapping (seq + 1, 0) into every shard.
inline uint64_t st_pack(uint64_t seq, uint32_t r) { return (seq << 32) | r; }
inline uint64_t st_seq(uint64_t s) { return s >> 32; }
inline uint32_t st_res(uint64_t s) { return (uint32_t)s; }

constexpr uint32_t kMaxShards = 16;
constexpr uint32_t kMinShardSlots = 64;
struct alignas(64) Shard {
    std::atomic<uint64_t> st{0};
};

// Home shard of the calling thread: threads are numbered in the order they first send.
std::atomic<uint32_t> g_thread_count{0};
// The calling thread's last reservation on a queue (its floor, see enqueue), keyed by the queue's
// unique id so a queue created at a freed one's address starts from no floor.
struct Floor {
    uint64_t seq = 0;
    uint32_t shard = 0;
};
std::atomic<uint64_t> g_queue_ids{0};

uint32_t thread_number() {
    thread_local const uint32_t t = g_thread_count.fetch_add(1, std::memory_order_relaxed);
    return t;
}

}  // namespace

struct fcs_txq {
    uint64_t id = g_queue_ids.fetch_add(1, std::memory_order_relaxed);   // never reused (Floor)
    uint8_t mac[6];
    uint32_t cap = 0, flush_usec = 0;
    fcs_txq_sink_fn sink = nullptr;
    void *ctx = nullptr;
    uint32_t nsh = 1, per = 0;            // shards, slots per shard (cap = nsh * per)
    Batch b[2];
    Shard sh[kMaxShards];                 // (open batch seq, slots reserved) per shard: see st_pack
    std::atomic<bool> idle{false};        // flusher asleep waiting for a first frame
    std::atomic<bool> blocked{false};     // a producer found every shard it may use full
    std::atomic<bool> stop_req{false};
    // slow paths (sleeping, flush(), statistics) take mu
    std::mutex mu;
    std::condition_variable cv_flusher;   // producers / flush() -> flusher
    std::condition_variable cv_prod;      // flusher -> producers (batch swapped, results ready)
    uint64_t seq_done = 0;                // last batch handed to the sink
    std::atomic<uint64_t> seq_sunk{0};    // the same, readable without mu (fcs_txq_send's direct path)
    struct alignas(64) DirectCount {      // frames synchronous callers sent themselves, per thread shard
        std::atomic<uint64_t> frames{0}, errors{0};   //   (one shared line would bounce between cores)
    } direct[kMaxShards];
    uint64_t flush_target = 0;            // flush() wants batches <= this closed now
    uint64_t n_frames = 0, n_batches = 0, n_errors = 0;
    uint64_t n_host_batches = 0, n_host_frames = 0;   // failed GPU steps answered by the host CRC
    uint64_t n_small_batches = 0, n_small_frames = 0; // no GPU step / frames on the host CRC, by design
    uint64_t n_gpu_batches = 0;                       // batches the GPU computed
    std::atomic<uint64_t> host_max{kHostMaxDefault};  // see fcs_txq_set_host_max
    std::atomic<bool> sync_host{true};                // see fcs_txq_set_sync_host
    uint64_t ns_ready = 0, ns_gpu = 0, ns_sink = 0, ns_busy = 0;   // flusher time split
    uint64_t ns_pickup = 0;               // first frame of a batch queued -> batch closed
    std::string last_error;               // fcs_last_error() of the latest failed GPU step
    std::thread th;
};

namespace {

uint64_t flush_target(fcs_txq *q) {
    std::lock_guard<std::mutex> lk(q->mu);
    return q->flush_target;
}

// Slots reserved in the open batch over all shards (each capped at its size).
uint32_t reserved(fcs_txq *q, std::memory_order mo) {
    uint32_t r = 0;
    for (uint32_t k = 0; k < q->nsh; k++) r += std::min(st_res(q->sh[k].st.load(mo)), q->per);
    return r;
}

enum class Leave { kStop, kSend };

// Wait until the open batch has a frame to leave with; kStop when stopping with nothing left.
// Leaves when full (or a producer is stuck behind a full home shard), when flush() asks, at once
// when flush_usec == 0, else after the oldest frame has lingered flush_usec. *closed_empty gets
// the shards the stop path sealed while still empty (they hold no frames).
Leave wait_for_batch(fcs_txq *q, uint64_t seq, uint32_t *closed_empty) {
    *closed_empty = 0;
    for (;;) {
        uint32_t r = reserved(q, std::memory_order_seq_cst);
        const bool stop = q->stop_req.load(std::memory_order_acquire);
        if (r == 0) {
            // stopping: mark every empty shard full so no producer can slip a frame in after we
            // leave (it then sees stop_req and returns -ESHUTDOWN); lost a race: send what came
            if (stop) {
                bool all = true;
                for (uint32_t k = 0; k < q->nsh; k++) {
                    uint64_t s = st_pack(seq, 0);
                    if (q->sh[k].st.compare_exchange_strong(s, st_pack(seq, q->per), std::memory_order_seq_cst))
                        *closed_empty |= 1u << k;
                    else
                        all = false;
                }
                if (all) return Leave::kStop;
                return Leave::kSend;
            }
            // idle: spin a little for the next frame, then sleep until a producer, flush() or
            // destroy wakes us (a producer taking a shard's slot 0 notifies when it sees idle set)
            const auto until = Clock::now() + kSpin;
            while (reserved(q, std::memory_order_acquire) == 0 && Clock::now() < until &&
                   !q->stop_req.load(std::memory_order_acquire))
                cpu_relax();
            std::unique_lock<std::mutex> lk(q->mu);
            q->idle.store(true, std::memory_order_seq_cst);
            while (reserved(q, std::memory_order_seq_cst) == 0 && !q->stop_req.load(std::memory_order_seq_cst))
                q->cv_flusher.wait(lk);
            q->idle.store(false, std::memory_order_relaxed);
            continue;
        }
        if (r >= q->cap || stop || q->flush_usec == 0 || q->blocked.load(std::memory_order_acquire) ||
            flush_target(q) >= seq)
            return Leave::kSend;
        // linger for company. Short lingers spin: a timed futex sleep is rounded up by the kernel's
        // timer slack (50 us by default), longer than the whole GPU step.
        Batch &B = q->b[seq & 1];
        int64_t f = B.first_ns.load(std::memory_order_acquire);
        if (f == 0) f = now_ns();   // the first frame's producer has not stamped it yet
        const int64_t deadline = f + (int64_t)q->flush_usec * 1000;
        if (q->flush_usec <= 1000) {
            while (now_ns() < deadline && reserved(q, std::memory_order_acquire) < q->cap &&
                   !q->blocked.load(std::memory_order_acquire) && !q->stop_req.load(std::memory_order_acquire))
                cpu_relax();
        } else {
            std::unique_lock<std::mutex> lk(q->mu);
            const auto left = std::chrono::nanoseconds(std::max<int64_t>(0, deadline - now_ns()));
#ifdef FCS_TXQ_TSAN   // tools/tsan: GCC 11's libtsan misses pthread_cond_clockwait (steady-clock waits)
            q->cv_flusher.wait_until(lk, std::chrono::system_clock::now() + left);
#else
            q->cv_flusher.wait_for(lk, left);
#endif
        }
        if (now_ns() >= deadline) return Leave::kSend;
    }
}

void flusher(fcs_txq *q) {
    for (;;) {
        const uint64_t seq = st_seq(q->sh[0].st.load(std::memory_order_acquire));
        uint32_t closed_empty = 0;
        if (wait_for_batch(q, seq, &closed_empty) == Leave::kStop) {   // stopping, nothing queued
            std::lock_guard<std::mutex> lk(q->mu);
            q->seq_done = seq - 1;
            q->seq_sunk.store(seq - 1, std::memory_order_release);
            q->cv_prod.notify_all();
            return;
        }
        // close batch seq: producers move on to b[(seq + 1) & 1], which the previous iteration
        // finished with (its results were delivered before we got here). Shards are closed from
        // the lowest up, so a thread that climbs from its home shard (because it is full) finds no
        // closed shard above an open one; enqueue's per-thread floor keeps the order in any case.
        Batch *B = &q->b[seq & 1];
        Batch &N = q->b[(seq + 1) & 1];
        N.first_ns.store(0, std::memory_order_relaxed);
        uint32_t nk[kMaxShards];
        for (uint32_t k = 0; k < q->nsh; k++) {
            const uint64_t old = q->sh[k].st.exchange(st_pack(seq + 1, 0), std::memory_order_acq_rel);
            nk[k] = (closed_empty >> k) & 1 ? 0 : std::min(st_res(old), q->per);   // past per: no slot
        }
        q->blocked.store(false, std::memory_order_release);
        {
            std::lock_guard<std::mutex> lk(q->mu);   // producers waiting for a free slot
            q->cv_prod.notify_all();
        }
        const int64_t f = B->first_ns.load(std::memory_order_acquire);
        const uint64_t pickup = f ? (uint64_t)std::max<int64_t>(0, now_ns() - f) : 0;

        const auto t0 = Clock::now();
        uint32_t n = 0, nn = 0;   // frames; frames still without an FCS (fire-and-forget ones, or all)
        uint64_t bytes = 0;       // covered bytes of those
        for (uint32_t k = 0; k < q->nsh; k++) {
            for (uint32_t j = 0; j < nk[k]; j++, n++) {   // every reserved slot assembled by its producer
                const uint32_t slot = k * q->per + j;
                SlotMeta &m = B->meta[slot];
                while (m.ready.load(std::memory_order_acquire) != seq) std::this_thread::yield();
                B->slot[n] = slot;
                B->off[n] = (uint64_t)slot * kStride;
                B->covered[n] = m.covered;
                if (!m.has_fcs) {
                    B->need_off[nn] = B->off[n];
                    B->need_len[nn] = m.covered;
                    bytes += m.covered;
                    nn++;
                }
            }
        }
        const auto t1 = Clock::now();
        // FCS of every frame that has none yet, written little-endian after its covered bytes
        // (ether.c:262-263): the host CRC at or below the GPU minimum, else one GPU step
        const bool small = bytes <= q->host_max.load(std::memory_order_relaxed);
        int rc = 0;
        bool host = false;
        auto host_fcs = [&] {
            for (uint32_t i = 0; i < nn; i++) {
                uint8_t *f = B->arena + B->need_off[i];
                const uint32_t c = fcs::host_crc32(f, B->need_len[i]);
                std::memcpy(f + B->need_len[i], &c, 4);   // little-endian, as ether.c:263
            }
        };
        if (nn && small) {   // below the GPU minimum: the host CRC by design, not a failure answer
            host_fcs();
        } else if (nn) {
            // the span the frames occupy (not the whole arena): it decides the engine's in-place path
            const uint64_t span = B->need_off[nn - 1] + kStride;
            rc = ether_fcs_tx_batch_host(B->arena, span, B->need_off.data(), B->need_len.data(), nn);
            host = rc != 0 || fcs::last_call_host_answered();   // the engine answered a failed GPU step
        }
        if (rc != 0) {
            // no usable GPU at all: ether_send cannot fail for FCS reasons (src/linux/ether.c:234-269),
            // so the host CRC computes this batch's FCSs, counted and reported
            host_fcs();
            fcs::host_batch_answered("fcs_txq flusher", fcs_last_error());
        }
        const auto t2 = Clock::now();
        for (uint32_t i = 0; i < n; i++) {
            B->frames[i] = B->arena + B->off[i];
            B->sizes[i] = B->covered[i] + kFcsLen;
            B->res[i] = -EIO;   // a sink that forgets a frame reports it as failed
        }
        q->sink(q->ctx, B->frames.data(), B->sizes.data(), B->res.data(), n);
        const auto t3 = Clock::now();

        std::lock_guard<std::mutex> lk(q->mu);
        if (host) {
            q->last_error = fcs_last_error() ? fcs_last_error() : "";
            q->n_host_batches++;
            q->n_host_frames += nn;
        }
        if (n && small) q->n_small_batches++;       // no GPU step: every FCS from the host CRC by design
        if (nn && !small && !host) q->n_gpu_batches++;
        q->n_small_frames += (n - nn) + (small ? nn : 0);
        auto ns = [](Clock::duration d) { return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count(); };
        q->ns_ready += ns(t1 - t0);
        q->ns_gpu += ns(t2 - t1);
        q->ns_sink += ns(t3 - t2);
        q->ns_busy += ns(Clock::now() - t0);
        q->ns_pickup += pickup;
        for (uint32_t i = 0; i < n; i++) {
            if (B->res[i] != (int)(B->covered[i] + kFcsLen)) q->n_errors++;
            if (Waiter *w = B->meta[B->slot[i]].w) {   // null: fcs_txq_send_async
                w->result = B->res[i];
                w->done.store(true, std::memory_order_release);   // last touch: w may vanish now
            }
        }
        q->seq_done = seq;
        q->seq_sunk.store(seq, std::memory_order_release);
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
    // as many shards (a power of two, at most 16) as split the batch into equal parts of at
    // least kMinShardSlots slots
    q->nsh = 1;
    while (q->nsh < kMaxShards && max_batch % (2 * q->nsh) == 0 && max_batch / (2 * q->nsh) >= kMinShardSlots)
        q->nsh *= 2;
    q->per = max_batch / q->nsh;
    q->flush_usec = flush_usec;
    if (const char *e = std::getenv("NSTACK_TXQ_HOST_MAX_BYTES")) q->host_max.store(std::strtoull(e, nullptr, 0));
    q->sink = sink;
    q->ctx = sink_ctx;
    for (int k = 0; k < 2; k++) {
        Batch &B = q->b[k];
        const uint64_t bytes = (uint64_t)max_batch * kStride;
        B.arena = (uint8_t *)fcs_host_alloc(bytes);   // pinned: direct H2D
        B.pinned = B.arena != nullptr;
        if (!B.arena) B.arena = (uint8_t *)std::malloc(bytes);   // no GPU runtime: the host CRC answers
        if (!B.arena) {
            fcs_txq_destroy(q);
            return nullptr;
        }
        B.meta = std::vector<SlotMeta>(max_batch);
        B.slot.assign(max_batch, 0);
        B.off.assign(max_batch, 0);
        B.covered.assign(max_batch, 0);
        B.need_off.assign(max_batch, 0);
        B.need_len.assign(max_batch, 0);
        B.sizes.assign(max_batch, 0);
        B.frames.assign(max_batch, nullptr);
        B.res.assign(max_batch, 0);
    }
    for (uint32_t k = 0; k < q->nsh; k++) q->sh[k].st.store(st_pack(1, 0));
    q->th = std::thread(flusher, q);
    return q;
}

}  // extern "C"

namespace {
// Assemble exactly as ether_send (:257-261): dst, src, htons(proto), payload, zero pad and zeroed
// FCS slot; the FCS is filled in afterwards (:262-263).
inline void assemble(uint8_t *f, const uint8_t *mac, const uint8_t dst[6], uint16_t proto, const uint8_t *buf,
                     size_t bsize, size_t frame_size) {
    std::memcpy(f, dst, 6);
    std::memcpy(f + 6, mac, 6);
    f[12] = (uint8_t)(proto >> 8);
    f[13] = (uint8_t)proto;
    if (bsize) std::memcpy(f + kHeaderLen, buf, bsize);
    std::memset(f + kHeaderLen + bsize, 0, frame_size - kHeaderLen - bsize);
}

Floor &thread_floor(const fcs_txq *q) {
    thread_local std::unordered_map<uint64_t, Floor> floors;   // nodes: references stay valid
    thread_local uint64_t last_id = ~0ull;
    thread_local Floor *last = nullptr;
    if (q->id != last_id) {   // the usual case is one queue per thread (one per ether handle)
        last = &floors[q->id];
        last_id = q->id;
    }
    return *last;
}

// Reserve a slot in the open batch (one fetch_add on the home shard's word, no lock), assemble the
// frame there and mark it ready.
// w == nullptr: fire-and-forget (the result only feeds the error counter).
//
// Per-thread order: batches leave in sequence and a batch's frames leave in (shard, slot) order, so
// a thread's frames leave in the order it queued them if each of its reservations comes after the
// previous one in (batch, shard) order: the thread keeps that pair per queue (its floor) and skips
// any shard word that names an earlier batch, or the same batch and a lower shard. Climbing alone
// does not guarantee it: a thread whose home shard was full may reserve in a higher shard of the
// next batch, and its next frame would find its home shard open in that same batch (seen under
// ThreadSanitizer as one frame in ~10 runs out of order before the floor existed). A fetch_add
// result names the batch the slot is in; it can only be later than the word loaded before it.
int enqueue(fcs_txq *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize, Waiter *w) {
    if (!q || !dst || (!buf && bsize)) return -EINVAL;
    const size_t frame_size = kHeaderLen + std::max<size_t>(bsize, kMinPayload) + kFcsLen;   // :222-224
    if (frame_size > kSlot) return -EMSGSIZE;                                                // :234-237
    const uint32_t home = thread_number() % q->nsh;
    Floor &fl = thread_floor(q);
    uint64_t s = 0;
    uint32_t k = home;
    for (;;) {
        if (q->stop_req.load(std::memory_order_acquire)) return -ESHUTDOWN;
        const uint64_t seq0 = st_seq(q->sh[home].st.load(std::memory_order_acquire));
        bool got = false;
        for (k = home; k < q->nsh && !got; k++) {
            s = q->sh[k].st.load(std::memory_order_acquire);
            if (st_seq(s) < fl.seq || (st_seq(s) == fl.seq && k < fl.shard)) continue;   // before the last frame
            if (st_res(s) < q->per) {
                // one fetch_add; a producer that overshoots a full shard got no slot and moves on
                // (the flusher takes min(reserved, per))
                s = q->sh[k].st.fetch_add(1, std::memory_order_seq_cst);
                got = st_res(s) < q->per;
            }
        }
        if (got) {
            k--;
            fl.seq = st_seq(s);
            fl.shard = k;
            break;
        }
        // every shard from home up is full: have the flusher close the batch and wait for it
        q->blocked.store(true, std::memory_order_release);
        const auto until = Clock::now() + kSpin;
        while (st_seq(q->sh[home].st.load(std::memory_order_acquire)) == seq0 && Clock::now() < until) cpu_relax();
        std::unique_lock<std::mutex> lk(q->mu);
        while (st_seq(q->sh[home].st.load(std::memory_order_acquire)) == seq0 &&
               !q->stop_req.load(std::memory_order_acquire)) {
            q->cv_flusher.notify_one();
            q->cv_prod.wait(lk);
        }
    }
    const uint64_t seq = st_seq(s);
    const uint32_t slot = k * q->per + st_res(s);
    Batch &B = q->b[seq & 1];
    if (st_res(s) == 0) {
        int64_t zero = 0;
        B.first_ns.compare_exchange_strong(zero, now_ns(), std::memory_order_acq_rel);
        if (q->idle.load(std::memory_order_seq_cst)) {   // the flusher went to sleep: wake it
            std::lock_guard<std::mutex> lk(q->mu);
            q->cv_flusher.notify_one();
        }
    }
    if (st_res(s) + 1 == q->per && q->flush_usec > 1000) {   // a long linger sleeps: a full shard may end it
        std::lock_guard<std::mutex> lk(q->mu);
        q->cv_flusher.notify_one();
    }

    uint8_t *f = B.arena + (uint64_t)slot * kStride;
    assemble(f, q->mac, dst, proto, buf, bsize, frame_size);
    SlotMeta &m = B.meta[slot];
    m.w = w;
    m.covered = (uint32_t)(frame_size - kFcsLen);
    // A synchronous caller blocks for its batch anyway: it computes its own frame's FCS here, on its
    // own core where the frame is cache-hot, in parallel with the other callers (unless sync_host is off)
    m.has_fcs = w && q->sync_host.load(std::memory_order_relaxed);
    if (m.has_fcs) {
        const uint32_t c = fcs::host_crc32(f, m.covered);
        std::memcpy(f + m.covered, &c, 4);   // little-endian, as ether.c:263
    }
    m.ready.store(seq, std::memory_order_release);
    return (int)frame_size;
}
// ether_send's body (src/linux/ether.c:222-269) for one frame on the calling thread: assembled in a
// stack buffer, its FCS from the host CRC, handed to the sink as a batch of one (concurrently with
// other senders and the flusher, as the reference's threads call sendto concurrently).
int send_direct(fcs_txq *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize) {
    if (!dst || (!buf && bsize)) return -EINVAL;
    const size_t frame_size = kHeaderLen + std::max<size_t>(bsize, kMinPayload) + kFcsLen;   // :222-224
    if (frame_size > kSlot) return -EMSGSIZE;                                                // :234-237
    if (q->stop_req.load(std::memory_order_acquire)) return -ESHUTDOWN;
    alignas(64) uint8_t f[kStride];
    assemble(f, q->mac, dst, proto, buf, bsize, frame_size);
    const uint32_t covered = (uint32_t)(frame_size - kFcsLen);
    const uint32_t c = fcs::host_crc32(f, covered);
    std::memcpy(f + covered, &c, 4);   // little-endian, as ether.c:263
    uint8_t *fp = f;
    uint32_t sz = (uint32_t)frame_size;
    int res = -EIO;   // a sink that forgets the frame reports it as failed
    q->sink(q->ctx, &fp, &sz, &res, 1);
    fcs_txq::DirectCount &dc = q->direct[thread_number() % kMaxShards];
    dc.frames.fetch_add(1, std::memory_order_relaxed);
    if (res != (int)frame_size) dc.errors.fetch_add(1, std::memory_order_relaxed);
    return res;
}
}  // namespace

extern "C" {

int fcs_txq_send(fcs_txq_t *q, const uint8_t dst[6], uint16_t proto, const uint8_t *buf, size_t bsize) {
    // A synchronous caller with no frame of its own still queued sends its frame itself (see the file
    // comment); one with queued fire-and-forget frames, or with sync_host off, goes through the batch.
    if (q && q->sync_host.load(std::memory_order_relaxed) &&
        thread_floor(q).seq <= q->seq_sunk.load(std::memory_order_acquire))
        return send_direct(q, dst, proto, buf, bsize);
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
    // per shard: the open batch if it holds frames, else the one before it; the latest of these.
    // A frame this thread queued is in a shard whose word now names its batch with res > 0, or a
    // later batch: either way the target covers it, even while a close is half way through.
    uint64_t target = 0;
    for (uint32_t k = 0; k < q->nsh; k++) {
        const uint64_t s = q->sh[k].st.load(std::memory_order_seq_cst);
        target = std::max(target, st_res(s) ? st_seq(s) : st_seq(s) - 1);
    }
    std::unique_lock<std::mutex> lk(q->mu);
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
            q->stop_req.store(true, std::memory_order_seq_cst);
            q->cv_flusher.notify_one();
            q->cv_prod.notify_all();
        }
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

void fcs_txq_fallbacks(const fcs_txq_t *q, uint64_t *host_batches, uint64_t *host_frames) {
    if (!q) return;
    fcs_txq *m = const_cast<fcs_txq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    if (host_batches) *host_batches = m->n_host_batches;
    if (host_frames) *host_frames = m->n_host_frames;
}

uint64_t fcs_txq_set_host_max(fcs_txq_t *q, uint64_t bytes) {
    if (!q) return 0;
    return q->host_max.exchange(bytes);
}

int fcs_txq_set_sync_host(fcs_txq_t *q, int on) {
    if (!q) return -EINVAL;
    return q->sync_host.exchange(on != 0) ? 1 : 0;
}

void fcs_txq_small_batches(const fcs_txq_t *q, uint64_t *small_batches, uint64_t *small_frames,
                           uint64_t *gpu_batches) {
    if (!q) return;
    fcs_txq *m = const_cast<fcs_txq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    uint64_t direct = 0;
    for (const fcs_txq::DirectCount &dc : m->direct) direct += dc.frames.load(std::memory_order_relaxed);
    if (small_batches) *small_batches = m->n_small_batches + direct;
    if (small_frames) *small_frames = m->n_small_frames + direct;
    if (gpu_batches) *gpu_batches = m->n_gpu_batches;
}

void fcs_txq_stats(const fcs_txq_t *q, uint64_t *frames, uint64_t *batches, uint64_t *errors) {
    if (!q) return;
    fcs_txq *m = const_cast<fcs_txq *>(q);
    std::lock_guard<std::mutex> lk(m->mu);
    uint64_t direct = 0, derr = 0;   // batches of one
    for (const fcs_txq::DirectCount &dc : m->direct) {
        direct += dc.frames.load(std::memory_order_relaxed);
        derr += dc.errors.load(std::memory_order_relaxed);
    }
    if (frames) *frames = m->n_frames + direct;
    if (batches) *batches = m->n_batches + direct;
    if (errors) *errors = m->n_errors + derr;
}

const char *fcs_txq_last_error(const fcs_txq_t *q) {
    if (!q) return "";
    fcs_txq *m = const_cast<fcs_txq *>(q);
    static thread_local std::string copy;
    std::lock_guard<std::mutex> lk(m->mu);
    copy = m->last_error;
    return copy.c_str();
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
    if (n == 1) {   // a synchronous sender's own frame: one send, as ether_send's one sendto
        ssize_t r;
        do r = send(fd, frames[0], sizes[0], 0); while (r < 0 && errno == EINTR);
        res[0] = r < 0 ? -errno : (int)r;
        return;
    }
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
    if (n == 1) {   // one frame: sendto with the frame's sockaddr_ll, exactly as ether_send (:241-265)
        sockaddr_ll a{};
        const uint8_t *f = frames[0];
        a.sll_family = AF_PACKET;
        a.sll_protocol = htons((uint16_t)((f[12] << 8) | f[13]));
        a.sll_ifindex = pc->ifindex;
        a.sll_halen = 6;
        std::memcpy(a.sll_addr, f, 6);
        ssize_t r;
        do r = sendto(pc->fd, f, sizes[0], 0, (const sockaddr *)&a, sizeof a); while (r < 0 && errno == EINTR);
        res[0] = r < 0 ? -errno : (int)r;
        return;
    }
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

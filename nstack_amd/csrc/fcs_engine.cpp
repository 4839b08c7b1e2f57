// fcs_engine.cpp — the C ABI (include/nstack_fcs.h) around the gfx950 FCS kernel.
//
// Replaces ether_fcs() (/root/reference/src/ether_fcs.c:4-19, prototype src/nstack_ether.h:80)
// and provides the batched forms its TX call site (src/linux/ether.c:262-263) needs.
// Per-device state (constant tables in HBM, staging buffers, streams) is created lazily and is
// safe to use from many threads. Every entry point computes on the GPU; a missing GPU or code object
// is reported as -ENODEV and bad arguments as -EINVAL. SURVEY.md §8b ("on any HIP error, fall back
// to the CPU path so results never differ"): the host batch forms answer any other failure of their
// GPU step from the host CRC of fcs_host_crc.cpp (with_host_answer; counted, announced on stderr),
// and the error-less drop-in ether_fcs does so after its GPU attempt and the retry on a fresh lane
// have both failed. The device forms return the HIP error (their frames are in device memory).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>
#include <initializer_list>

#include "../../include/nstack_fcs.h"
#include "fcs_device.hpp"
#include "fcs_error.hpp"
#include "fcs_host_crc.hpp"
#include "fcs_launch.hpp"
#include "fcs_tables.hpp"

namespace {

thread_local std::string g_last_error;

int fail(int err, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return -err;
}

int hip_fail(hipError_t e, const char *what) {
    const int err = (e == hipErrorNoDevice || e == hipErrorInvalidDevice ||
                     e == hipErrorNoBinaryForGpu || e == hipErrorInvalidDeviceFunction ||
                     e == hipErrorInvalidImage || e == hipErrorSharedObjectInitFailed)
                        ? ENODEV
                        : (e == hipErrorOutOfMemory ? ENOMEM : EIO);
    return fail(err, "%s: %s", what, hipGetErrorString(e));
}

#define HIPTRY(expr, what)                        \
    do {                                          \
        hipError_t e_ = (expr);                   \
        if (e_ != hipSuccess) return hip_fail(e_, what); \
    } while (0)

// Makes `dev` current for the scope and restores the caller's device on exit (a host-batch call
// must not leave a multi-GPU caller's thread on another device: its next *_dev call resolves the
// device from the thread's current one).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        err = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// Drop-in ether_fcs health counters (fcs_engine_stats).
std::atomic<uint64_t> g_dropin_calls{0}, g_dropin_retries{0}, g_dropin_recovered{0}, g_lane_resets{0};
std::atomic<uint64_t> g_host_fallbacks{0};   // drop-in calls answered by the host CRC (fcs_host_crc.cpp)

#ifdef FCS_FAULT_HOOK
// Test-only build (libnstack_fcs_faults.so): the calling thread's next N drop-in attempts fail as
// if the GPU step had returned an error, so the recovery path can be exercised on a healthy GPU.
thread_local int g_inject_faults = 0;
bool injected_fault() {
    if (g_inject_faults <= 0) return false;
    g_inject_faults--;
    return true;
}
// ... and the next N single-frame attempts give up right after the launch, as if the 10 s wait had
// run out, while their kernel is still in flight (the quarantine path).
thread_local int g_inject_timeouts = 0;
bool injected_timeout() {
    if (g_inject_timeouts <= 0) return false;
    g_inject_timeouts--;
    return true;
}
// ... and of the host batch calls (the five ether_fcs_*_host forms, which the TX/RX queues use, and
// the mapped-list submit and wait of the RX queue), whichever thread makes them (the TX queue's GPU
// step runs on its flusher thread), the next `skip` run normally and the `calls` after them fail:
// at entry, before anything is launched (fcs_debug_fail_batches; a failed mapped-list wait leaves
// its kernel in flight), or at the call's first wait after a launch, giving up with the kernel
// still in flight as a timeout would (fcs_debug_late_batches).
struct Injector {
    std::mutex mu;
    int skip = 0, calls = 0;
    bool take() {
        std::lock_guard<std::mutex> lk(mu);
        if (skip > 0) {
            skip--;
            return false;
        }
        if (calls <= 0) return false;
        calls--;
        return true;
    }
    void arm(int s, int c) {
        std::lock_guard<std::mutex> lk(mu);
        skip = s;
        calls = c;
    }
    int left() {
        std::lock_guard<std::mutex> lk(mu);
        return skip + calls;
    }
};
Injector g_inject_batch, g_inject_late;
bool injected_batch_fault() { return g_inject_batch.take(); }
bool injected_late_fault() { return g_inject_late.take(); }
// ... and the next small-batch launch (TX/verify in mapped memory) is queued behind hold_kernel,
// which keeps its stream busy until the host word (fcs_host_alloc memory) turns nonzero or 20 s
// pass: a kernel that really stays in flight after its call gave up (fcs_debug_hold_small).
std::atomic<const uint32_t *> g_hold_word{nullptr};
const uint32_t *take_hold() { return g_hold_word.exchange(nullptr); }
#else
inline bool injected_fault() { return false; }
inline bool injected_timeout() { return false; }
inline bool injected_batch_fault() { return false; }
inline bool injected_late_fault() { return false; }
inline const uint32_t *take_hold() { return nullptr; }
#endif

// Device-wide synchronisations the engine has issued (fcs_debug_device_syncs): a hung kernel on a
// retired stream would block every one of them, so the paths a failed call leaves behind avoid them.
std::atomic<uint64_t> g_device_syncs{0};
hipError_t device_sync() {
    g_device_syncs.fetch_add(1, std::memory_order_relaxed);
    return hipDeviceSynchronize();
}

// Host batch calls (ether_fcs_*_host, and the TX/RX queues' batches, which go through them)
// answered by the host CRC because their GPU step failed.
std::atomic<uint64_t> g_host_batches{0};
// Set when the calling thread's last host batch call was answered by the host CRC (the queues read
// it to count their own batches: fcs::last_call_host_answered).
thread_local bool t_host_answered = false;
// Failed host batch calls that may have left a kernel in flight retire the resources that kernel
// can still write (pipeline staging, the small-batch stream, its mapped words and counters): they
// are set aside until fcs_engine_fini, never reused. After kMaxRetired such calls the host batch
// forms stop calling the GPU and answer from the host CRC (counted, reported once).
constexpr uint32_t kMaxRetired = 16;
std::atomic<uint32_t> g_retired{0};
bool host_only() { return g_retired.load(std::memory_order_relaxed) >= kMaxRetired; }

// Host pipeline resources of one device: kDepth chunks in flight (double-buffered by default).
#ifndef FCS_PIPE_DEPTH   // measurement-only override (chunks in flight per device)
#define FCS_PIPE_DEPTH 2
#endif
struct Pipe {
    static constexpr int kDepth = FCS_PIPE_DEPTH;
    hipStream_t stream = nullptr;     // copies to the device, chunk after chunk at the full PCIe rate
    hipStream_t cstream = nullptr;    // each chunk's kernel and its D2H, once its H2D has landed, so they
                                      // overlap the next chunk's H2D (two H2D streams halved the rate)
    hipEvent_t done[kDepth] = {};
    hipEvent_t landed[kDepth] = {};
    uint8_t *d_in[kDepth] = {};
    uint8_t *h_in[kDepth] = {};     // pinned staging
    uint64_t *d_off[kDepth] = {};   // a chunk's n offsets, then its n lengths
    uint32_t *d_out[kDepth] = {};
    uint64_t *h_off[kDepth] = {};   // pinned; as d_off (one H2D per chunk)
    uint32_t *h_out[kDepth] = {};   // pinned
    uint64_t cap_bytes = 0, cap_frames = 0;
};

struct DevState {
    int dev = -1;
    int cus = 0;
    uint32_t *d_blob = nullptr;
    uint32_t *d_one_blob = nullptr;   // tables of the single-frame kernel (drop-in ether_fcs)
    uint32_t *d_kinit = nullptr;      // kinit_table() in device memory (mapped-list kernel)
    // Dynamic-tail counters of the LDS-DMA kernel: a ring of kCtrSlots, one 64-B line each; a
    // large fixed launch takes the next slot and zeroes it on its own stream before the kernel.
    // A slot is reused only after the kernel that last used it has finished: the reuser's stream
    // waits for that kernel's completion event before zeroing the slot (ctr_mu[slot] is held from
    // taking the slot until the event is recorded behind the new launch).
    static constexpr uint32_t kCtrSlots = 256;
    unsigned long long *d_ctr = nullptr;
    std::atomic<uint32_t> ctr_seq{0};
    std::mutex ctr_mu[kCtrSlots];
    hipEvent_t ctr_done[kCtrSlots] = {};
    // Per-slot device scratch for launches that need some besides the counter (the arena-stream
    // kernel's list of units for fcs_flat_kernel), guarded by the same slot lease.
    uint32_t *ctr_scr[kCtrSlots] = {};
    uint64_t ctr_scr_words[kCtrSlots] = {};
    uint32_t *d_last_listed = nullptr;   // the last arena-stream launch's unit-list length (in d_ctr's last line)
    // Streams and mapped result words of drop-in lanes given up while a kernel may still be in
    // flight on them (timeout, lost completion, device error): never reused or freed before
    // fcs_engine_fini, so a late kernel cannot write into memory that serves another call.
    std::mutex q_mu;
    std::vector<hipStream_t> q_streams;
    std::vector<void *> q_host;
    std::vector<void *> q_dev;   // device buffers of retired resources (hipFree at fini)
    std::mutex pipe_mu;      // one host pipeline at a time per device
    Pipe pipe;
    std::mutex tx_mu;        // small-batch zero-copy TX (ether_fcs_tx_host on pinned frames)
    hipStream_t tx_stream = nullptr;
    uint32_t *tx_len = nullptr, *tx_out = nullptr;   // pinned, device-mapped
    uint32_t *tx_dlen = nullptr, *tx_dout = nullptr; //   ... their device addresses
    uint64_t *tx_off = nullptr, *tx_doff = nullptr;  // frame offsets (ether_fcs_tx_batch_host)
    uint64_t *tx_flag = nullptr, *tx_dflag = nullptr; // completion word (signal_kernel), mapped
    uint64_t tx_seq = 0;
    uint64_t tx_first_seq = 1;   // first completion number of the current tx_stream (earlier ones
                                 // belong to a retired stream: retire_small)
    struct OldGen {              // a retired small-batch stream: completions [first, last] were
        uint64_t first, last;    // issued on it; its stream and word are quarantined, not freed, so
        hipStream_t st;          // a batch issued before the retirement can still be waited for
        const uint64_t *flag;
    };
    std::vector<OldGen> tx_old;
    unsigned long long *tx_dcount = nullptr;        // small-batch kernel: frames done (device memory)
    uint64_t tx_count = 0;                           //   ... its value once every launch so far is done
    uint64_t *vz_off = nullptr, *vz_doff = nullptr;  // small RX verify batches (same stream and lock):
    uint32_t *vz_len = nullptr, *vz_dlen = nullptr;  //   offsets, lengths, ok flags and the bad count,
    uint8_t *vz_ok = nullptr, *vz_dok = nullptr;     //   pinned and device-mapped; the kernel's bad
    unsigned long long *vz_dbad = nullptr;           //   count goes to device scratch (no PCIe atomics)
    uint64_t vz_cap = 0;
    uint64_t tx_cap = 0;
    std::mutex one_mu;       // single-frame (drop-in ether_fcs) staging
    hipStream_t one_stream = nullptr;
    uint8_t *one_h = nullptr, *one_hd = nullptr;      // pinned, device-mapped frame staging
    uint32_t *one_hout = nullptr, *one_dout = nullptr;
    uint64_t *one_flag = nullptr, *one_dflag = nullptr;
    uint64_t one_seq = 0;
    uint64_t one_cap = 0;
    // Single-frame kernel (drop-in ether_fcs, one-frame TX): a few independent lanes, each with its
    // own stream and result word, so concurrent callers (nstack calls ether_fcs from its main,
    // ingress, egress and timer threads) do not queue behind one another. A thread keeps its lane.
    struct OneLane {
        std::mutex mu;
        hipStream_t st = nullptr;
        uint64_t *flag = nullptr, *dflag = nullptr;   // mapped result word: (seq << 32) | FCS
        uint32_t seq = 0;
    };
    static constexpr int kOneLanes = 4;   // HIP maps streams onto 4 hardware queues per process
    OneLane one_lane[kOneLanes];
};

std::mutex g_mu;
std::vector<std::unique_ptr<DevState>> g_dev;   // indexed by HIP device ordinal
std::vector<int> g_engine_devs;                  // devices used by the host batch APIs
const fcs::Tables &tables() {
    static const fcs::Tables t;
    return t;
}

// A_L(0xFFFFFFFF) for L = 0 .. kOneBytes: the all-ones CRC start carried over L bytes (the
// single-frame kernels start from a zero register and add this back).
const std::vector<uint32_t> &kinit_table() {
    static const std::vector<uint32_t> k = [] {
        std::vector<uint32_t> v(fcs::kOneBytes + 1);
        v[0] = 0xFFFFFFFFu;
        for (uint32_t L = 1; L <= fcs::kOneBytes; L++) v[L] = tables().zstep(v[L - 1]);
        return v;
    }();
    return k;
}

// A device's state: the table images, counters and (lazily) its streams and staging buffers.
int make_dev_state(int dev, std::unique_ptr<DevState> *out) {
    auto st = std::make_unique<DevState>();
    st->dev = dev;
    int cur = 0;
    HIPTRY(hipGetDevice(&cur), "hipGetDevice");
    HIPTRY(hipSetDevice(dev), "hipSetDevice");
    hipDeviceProp_t prop;
    hipError_t pe = hipGetDeviceProperties(&prop, dev);
    if (pe != hipSuccess) { hipSetDevice(cur); return hip_fail(pe, "hipGetDeviceProperties"); }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        hipSetDevice(cur);
        return fail(ENODEV, "device %d is %s; this engine is built for gfx950 only", dev, prop.gcnArchName);
    }
    st->cus = prop.multiProcessorCount;
    const std::vector<uint32_t> blob = tables().blob();
    hipError_t ae = hipMalloc(&st->d_blob, blob.size() * 4);
    if (ae == hipSuccess) ae = hipMemcpy(st->d_blob, blob.data(), blob.size() * 4, hipMemcpyHostToDevice);
    const std::vector<uint32_t> one = tables().one_blob();
    if (ae == hipSuccess) ae = hipMalloc(&st->d_one_blob, one.size() * 4);
    if (ae == hipSuccess) ae = hipMemcpy(st->d_one_blob, one.data(), one.size() * 4, hipMemcpyHostToDevice);
    const std::vector<uint32_t> &ki = kinit_table();
    if (ae == hipSuccess) ae = hipMalloc(&st->d_kinit, ki.size() * 4);
    if (ae == hipSuccess) ae = hipMemcpy(st->d_kinit, ki.data(), ki.size() * 4, hipMemcpyHostToDevice);
    // the counter ring plus one line for the last arena-stream launch's unit-list length
    if (ae == hipSuccess) ae = hipMalloc(&st->d_ctr, (DevState::kCtrSlots + 1) * 64);
    if (ae == hipSuccess) ae = hipMemset(st->d_ctr, 0, (DevState::kCtrSlots + 1) * 64);
    if (ae == hipSuccess) st->d_last_listed = (uint32_t *)(st->d_ctr + 8 * DevState::kCtrSlots);
    hipSetDevice(cur);
    if (ae != hipSuccess) return hip_fail(ae, "uploading FCS tables");
    *out = std::move(st);
    return 0;
}

int dev_state(int dev, DevState **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return fail(ENODEV, "no HIP device visible (%s)", hipGetErrorString(e));
    if (dev < 0 || dev >= ndev) return fail(EINVAL, "device %d out of range (%d devices)", dev, ndev);
    if ((int)g_dev.size() < ndev) g_dev.resize(ndev);
    if (!g_dev[dev]) {
        int rc = make_dev_state(dev, &g_dev[dev]);
        if (rc) return rc;
    }
    *out = g_dev[dev].get();
    return 0;
}

// Engine device ids at or past the device count (only with NSTACK_FCS_ALIAS_DEVICES=1, a test
// hook): a state of their own on HIP device id mod count, so the multi-device host path (shard
// plan, one thread and pipeline per device, result assembly) runs on a one-GPU box.
std::map<int, std::unique_ptr<DevState>> g_alias;
std::vector<std::unique_ptr<DevState>> g_alias_retired;   // dropped by a later init; freed at fini

int alias_state(int id, int ndev, DevState **out) {
    std::lock_guard<std::mutex> lk(g_mu);
    auto &slot = g_alias[id];
    if (!slot) {
        int rc = make_dev_state(id % ndev, &slot);
        if (rc) return rc;
    }
    *out = slot.get();
    return 0;
}

bool alias_devices_enabled() {
    const char *e = std::getenv("NSTACK_FCS_ALIAS_DEVICES");
    return e && std::atoi(e) != 0;
}

int current_dev_state(DevState **out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    return dev_state(dev, out);
}

inline uint64_t floor4(uint64_t x) { return x & ~3ull; }
inline uint64_t ceil4(uint64_t x) { return (x + 3) & ~3ull; }

uint32_t segments(uint32_t len) { return len ? (len + fcs::kSegBytes - 1) / fcs::kSegBytes : 1u; }

// Bound for the kernel's front-masking loop (words 0 .. ceil(zmax/4)-1 get masked): the leading
// zero bytes of the front lane of segment 0, or the whole chunk (48) when segment 0 leaves lanes
// with no frame bytes at all (those lanes' loads are not zero-filled and must be masked entirely).
uint32_t mask_bound(uint32_t len) {
    if (!len) return fcs::kChunkBytes;
    const uint32_t l0 = len - fcs::kSegBytes * (segments(len) - 1);
    if (l0 <= fcs::kSegBytes - fcs::kChunkBytes) return fcs::kChunkBytes;
    return fcs::kChunkBytes * ((l0 + fcs::kChunkBytes - 1) / fcs::kChunkBytes) - l0;
}

int grid_for(const DevState *ds, uint64_t n, int threads) {
    // frame slots (quarter-waves) per workgroup of the kernel launch_fcs picks
    const uint64_t slots = (uint64_t)threads / fcs::kGroup;
    const uint64_t want = (n + slots - 1) / slots;
#ifdef FCS_GRID_CUS   // measurement-only build: run the persistent grid on fewer CUs
    const uint64_t cus = std::min<uint64_t>((uint64_t)ds->cus, FCS_GRID_CUS);
#else
    const uint64_t cus = (uint64_t)ds->cus;
#endif
    return (int)std::max<uint64_t>(1, std::min<uint64_t>(cus, want));
}

uint64_t *g_dbg = nullptr;   // FCS_STAMPS builds only

// Variable-length batches of at most this many frames take the quarter-wave-per-frame kernel
// (every frame in flight at once: lowest latency); larger ones the windowed kernel (throughput).
// 16384 = 4 frames x 16 waves x 256 CUs: one item per quarter-wave on a full chip.
std::atomic<uint64_t> g_var_threshold{16384};

// The device whose d_last_listed holds the unit-list length of the last arena-stream launch
// (fcs_debug_stream_listed). DevStates live until fcs_engine_fini, so the pointer stays valid.
std::atomic<DevState *> g_last_stream_dev{nullptr};

// A zeroed work counter for one launch (Dispenser in fcs_kernel.hip): the next slot of the
// device's ring, cleared on the launch's own stream just before the kernel, after the slot's
// previous kernel (on any stream) has finished. The lease holds the slot until the new launch's
// completion event is recorded (CounterLease::~CounterLease, after the launch).
struct CounterLease {
    DevState *ds = nullptr;
    hipStream_t st = nullptr;
    int slot = -1;
    CounterLease() = default;
    CounterLease(const CounterLease &) = delete;
    CounterLease &operator=(const CounterLease &) = delete;
    ~CounterLease() {
        if (slot < 0) return;
        (void)hipEventRecord(ds->ctr_done[slot], st);
        ds->ctr_mu[slot].unlock();
    }
};

// Device scratch of `words` u32 that belongs to a held slot lease (grown on the host once the
// slot's last kernel has finished).
int lease_scratch(CounterLease &lease, uint64_t words, uint32_t **out) {
    DevState *ds = lease.ds;
    const int s = lease.slot;
    if (ds->ctr_scr_words[s] < words) {
        if (ds->ctr_scr[s]) {
            HIPTRY(hipEventSynchronize(ds->ctr_done[s]), "waiting for the counter slot's last kernel");
            HIPTRY(hipFree(ds->ctr_scr[s]), "hipFree(slot scratch)");
            ds->ctr_scr[s] = nullptr;
            ds->ctr_scr_words[s] = 0;
        }
        const uint64_t w = std::max<uint64_t>(words, 1u << 16);
        HIPTRY(hipMalloc(&ds->ctr_scr[s], w * 4), "hipMalloc(slot scratch)");
        ds->ctr_scr_words[s] = w;
    }
    *out = ds->ctr_scr[s];
    return 0;
}

// words: how many u64 counters of the slot's 64-B line the launch(es) use (1..8), all zeroed.
int take_counter(DevState *ds, hipStream_t st, fcs::KParams &p, CounterLease &lease, uint32_t words = 1) {
    const uint32_t slot = ds->ctr_seq.fetch_add(1, std::memory_order_relaxed) % DevState::kCtrSlots;
    ds->ctr_mu[slot].lock();
    lease.ds = ds;
    lease.st = st;
    lease.slot = (int)slot;
    if (!ds->ctr_done[slot]) {
        HIPTRY(hipEventCreateWithFlags(&ds->ctr_done[slot], hipEventDisableTiming), "hipEventCreate(counter)");
    } else {
        HIPTRY(hipStreamWaitEvent(st, ds->ctr_done[slot], 0), "waiting for the counter slot's last kernel");
    }
    p.ctr = ds->d_ctr + 8 * slot;
    HIPTRY(hipMemsetAsync(p.ctr, 0, 8 * words, st), "zeroing the work counter");
    return 0;
}

// The fixed-length route (fcs::route_fixed, the one place that decides it), its grid, its work
// counter, and the launch of exactly that kernel (fcs::launch_fixed_route).
fcs::KParams fixed_params(const DevState *ds, const void *base, uint64_t stride, uint32_t len, uint64_t n) {
    fcs::KParams p{};
    p.base = (uint64_t)base;
    p.stride = stride;
    p.n = n;
    p.lo4 = floor4((uint64_t)base);
    p.hi4 = ceil4((uint64_t)base + (n - 1) * stride + len);
    p.flen = len;
    p.fseg = segments(len);
    p.zmax = mask_bound(len);
    p.blob = ds ? ds->d_blob : nullptr;
    return p;
}

int launch_fixed(DevState *ds, const void *base, uint64_t stride, uint32_t len, uint64_t n,
                 uint32_t *out, hipStream_t st, uint8_t *ok = nullptr, unsigned long long *bad = nullptr) {
    CounterLease lease;   // declared first: released (event recorded) after the launch below
    fcs::KParams p = fixed_params(ds, base, stride, len, n);
    p.ok = ok;
    p.bad = bad;
    p.out = out;
    p.dbg = g_dbg;
    const fcs::FixedRoute r = fcs::route_fixed(p, n > g_var_threshold.load(std::memory_order_relaxed));
    p.zmax = r.zmax;
    // short frames: one lane per frame, 64 frames per wave item; the others: the route's slots
    const int grid = r.kernel == fcs::FixedKernel::kShort
                         ? FCS_SHORT_WG_PER_CU * grid_for(ds, (n + 15) / 16, r.threads)
                         : grid_for(ds, n, r.threads);
    const uint64_t items = (n + r.item_frames - 1) / r.item_frames, waves = (uint64_t)grid * (r.threads / 64);
    if (r.dyn_min && items >= r.dyn_min * waves) {   // large batch: dynamic schedule
        const int rc = take_counter(ds, st, p, lease);
        if (rc) return rc;
    }
    HIPTRY(fcs::launch_fixed_route(r, p, grid, st), "launching a fixed-length FCS kernel");
    return 0;
}

// off == nullptr: frame i starts at arena + i * stride (TX slots of variable covered length).
int launch_var(DevState *ds, const void *arena, uint64_t arena_bytes, const uint64_t *off,
               const uint32_t *len, uint32_t *out, uint64_t n, hipStream_t st, uint8_t *ok = nullptr,
               unsigned long long *bad = nullptr, uint64_t stride = 0) {
    CounterLease lease;
    fcs::KParams p{};
    p.ok = ok;
    p.bad = bad;
    p.stride = stride;
    p.base = (uint64_t)arena;
    p.off = off;
    p.len = len;
    p.out = out;
    p.n = n;
    p.lo4 = floor4((uint64_t)arena);
    p.hi4 = ceil4((uint64_t)arena + arena_bytes);
    p.zmax = fcs::kChunkBytes;
    p.blob = ds->d_blob;
#ifdef FCS_STAMPS
    p.dbg = g_dbg;
#endif
    const bool windowed = n > g_var_threshold.load(std::memory_order_relaxed);
    const int grid = grid_for(ds, n, fcs::kWgThreads);
#ifndef FCS_NO_STREAM   // measurement-only: every windowed batch through fcs_flat_kernel alone
    if (windowed && off != nullptr && p.hi4 - p.lo4 >= 2 * (uint64_t)fcs::kChunkBytes) {
        // arena stream for units of packed 64..1536-B frames, then fcs_flat_kernel for the units it
        // listed (it returns at once when there are none)
        // one lease serves both kernels: the flat kernel's counter is the second word of the same
        // 64-B counter line (taking a second slot while holding the first could land on the held
        // slot once the ring wraps)
        int rc = take_counter(ds, st, p, lease, 2);
        if (rc) return rc;
        const uint64_t units = (n + fcs::kStUnitFrames - 1) / fcs::kStUnitFrames;
        uint32_t *scr = nullptr;
        if ((rc = lease_scratch(lease, units + 1, &scr))) return rc;
        p.ucount = scr;
        p.ulist = scr + 1;
        HIPTRY(hipMemsetAsync(p.ucount, 0, 4, st), "zeroing the unit list");
        HIPTRY(fcs::launch_stream(p, (int)std::min<uint64_t>((uint64_t)ds->cus, units), st), "launching fcs_stream_kernel");
        // the flat kernel stores the unit-list length for fcs_debug_stream_listed (the slot scratch
        // is reused and may be regrown once the lease is released)
        g_last_stream_dev.store(ds, std::memory_order_relaxed);
        fcs::KParams q = p;
        q.ctr = p.ctr + 1;
        q.listed_out = ds->d_last_listed;
        HIPTRY(fcs::launch_fcs(true, true, q, grid, st), "launching fcs_flat_kernel<listed units>");
        return 0;
    }
#endif
    if (windowed && (n + 63) / 64 >= fcs::kFlatDynMinWindowsPerWave * (uint64_t)grid * (fcs::kWgThreads / 64)) {
        const int rc = take_counter(ds, st, p, lease);
        if (rc) return rc;
    }
    HIPTRY(fcs::launch_fcs(true, windowed, p, grid, st), "launching fcs_kernel<var>");
    return 0;
}

// Set aside a stream and pinned words that a kernel may still use: neither destroyed nor freed
// (hipHostFree could block behind a hung kernel, and a late kernel must not write into a word that
// serves another call by then) until fcs_engine_fini.
void quarantine(DevState *ds, hipStream_t st, std::initializer_list<void *> host,
                std::initializer_list<void *> dev = {}) {
    std::lock_guard<std::mutex> lk(ds->q_mu);
    if (st) ds->q_streams.push_back(st);
    for (void *h : host)
        if (h) ds->q_host.push_back(h);
    for (void *d : dev)
        if (d) ds->q_dev.push_back(d);
}

// hipFree and hipHostFree synchronise the device. While a retired stream may still run a kernel
// (one that never finishes would block them for good), arrays that a growth path replaces join the
// quarantine instead of being freed; no live kernel uses them any more either way.
bool quarantine_busy(DevState *ds) {
    std::lock_guard<std::mutex> lk(ds->q_mu);
    bool busy = false;
    for (hipStream_t st : ds->q_streams)
        if (hipStreamQuery(st) == hipErrorNotReady) {
            busy = true;
            break;
        }
    (void)hipGetLastError();
    return busy;
}

void release(DevState *ds, std::initializer_list<void *> host, std::initializer_list<void *> dev = {}) {
    if (quarantine_busy(ds)) {
        quarantine(ds, nullptr, host, dev);
        return;
    }
    for (void *h : host)
        if (h) (void)hipHostFree(h);
    for (void *d : dev)
        if (d) (void)hipFree(d);
}

// A host batch call failed after launching on the pipeline (a chunk's kernel or copies may still
// run): its streams, events and staging are set aside and recreated on next use, so a late kernel or
// D2H copy cannot write into staging that serves a later call. Caller holds pipe_mu.
void retire_pipe(DevState *ds) {
    Pipe &pp = ds->pipe;
    quarantine(ds, pp.stream, {}, {});
    quarantine(ds, pp.cstream, {}, {});
    for (int b = 0; b < Pipe::kDepth; b++) {
        quarantine(ds, nullptr, {pp.h_in[b], pp.h_off[b], pp.h_out[b]}, {pp.d_in[b], pp.d_off[b], pp.d_out[b]});
        // events are only recorded and waited on; a fresh pipe creates its own
    }
    ds->pipe = Pipe{};
    (void)hipGetLastError();
    g_retired.fetch_add(1, std::memory_order_relaxed);
}

int ensure_pipe(DevState *ds, uint64_t bytes, uint64_t frames) {
    Pipe &pp = ds->pipe;
    if (!pp.stream) {
        HIPTRY(hipStreamCreateWithFlags(&pp.stream, hipStreamNonBlocking), "hipStreamCreate");
        HIPTRY(hipStreamCreateWithFlags(&pp.cstream, hipStreamNonBlocking), "hipStreamCreate");
        for (int b = 0; b < Pipe::kDepth; b++) {
            HIPTRY(hipEventCreateWithFlags(&pp.done[b], hipEventDisableTiming), "hipEventCreate");
            HIPTRY(hipEventCreateWithFlags(&pp.landed[b], hipEventDisableTiming), "hipEventCreate");
        }
    }
    if (bytes > pp.cap_bytes) {
        for (int b = 0; b < Pipe::kDepth; b++) {
            release(ds, {pp.h_in[b]}, {pp.d_in[b]});
            pp.d_in[b] = nullptr;
            pp.h_in[b] = nullptr;
        }
        pp.cap_bytes = 0;
        for (int b = 0; b < Pipe::kDepth; b++) {
            HIPTRY(hipMalloc(&pp.d_in[b], bytes + 64), "hipMalloc(staging)");
            HIPTRY(hipHostMalloc(&pp.h_in[b], bytes + 64, hipHostMallocDefault), "hipHostMalloc(staging)");
        }
        pp.cap_bytes = bytes;
    }
    if (frames > pp.cap_frames) {
        for (int b = 0; b < Pipe::kDepth; b++) {
            release(ds, {pp.h_off[b], pp.h_out[b]}, {pp.d_off[b], pp.d_out[b]});
            pp.d_off[b] = nullptr; pp.d_out[b] = nullptr;
            pp.h_off[b] = nullptr; pp.h_out[b] = nullptr;
        }
        pp.cap_frames = 0;
        for (int b = 0; b < Pipe::kDepth; b++) {
            HIPTRY(hipMalloc(&pp.d_off[b], frames * 12), "hipMalloc(off, len)");
            HIPTRY(hipMalloc(&pp.d_out[b], frames * 4), "hipMalloc(out)");
            HIPTRY(hipHostMalloc(&pp.h_off[b], frames * 12, hipHostMallocDefault), "hipHostMalloc(off, len)");
            HIPTRY(hipHostMalloc(&pp.h_out[b], frames * 4, hipHostMallocDefault), "hipHostMalloc(out)");
        }
        pp.cap_frames = frames;
    }
    return 0;
}

// Ranges from fcs_host_alloc (the TX queue's arenas): host address -> device address without a
// HIP query per small batch. Entries leave in fcs_host_free, before the memory is released.
struct PinnedRange {
    uint64_t bytes;
    uint8_t *dev;
};
std::mutex g_pin_mu;
std::map<uintptr_t, PinnedRange> g_pinned;

uint8_t *pinned_dev_ptr(const void *p, uint64_t bytes) {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    const uintptr_t a = (uintptr_t)p;
    auto it = g_pinned.upper_bound(a);
    if (it == g_pinned.begin()) return nullptr;
    --it;
    if (a < it->first || a + bytes > it->first + it->second.bytes) return nullptr;
    return it->second.dev + (a - it->first);
}

// A small batch completes when signal_kernel, queued behind its FCS kernel, stores `v` into the
// mapped completion word: the host spins on that word (a stream synchronisation costs ~3 us more
// per round trip, tools/microbench/launch_lat.hip). Errors and stalls are still caught by
// polling the stream now and then.
// Completion words only grow: every launch that stores one is numbered under its stream's lock
// in stream order, so a later launch may already have overwritten `v` with a larger value.
int wait_flag(hipStream_t st, const uint64_t *flag, uint64_t v, const char *what) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; i++) {
        if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= v) return 0;
        __builtin_ia32_pause();
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(st);
            if (q == hipSuccess) {
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) >= v) return 0;
                return fail(EIO, "%s: stream idle but no completion signal", what);
            }
            if (q != hipErrorNotReady) return hip_fail(q, what);
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10))
                return fail(ETIMEDOUT, "%s: no completion after 10 s", what);
        }
    }
}

bool is_pinned(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// A chunk of host frames handed to one device: frames [i0, i1) of the caller's arrays.
struct HostJob {
    const uint8_t *arena;          // var: arena base; fixed/tx: frame 0
    uint64_t arena_bytes;
    const uint64_t *off;           // var only (nullptr: frame i at i*stride)
    const uint32_t *len;           // var/tx lengths (nullptr: fixed len)
    uint64_t stride;
    uint32_t flen;
    uint32_t *out;                 // crc per frame (nullptr in TX mode)
    uint8_t *tx_base;              // TX: write FCS after each frame
    uint64_t i0, i1;
    uint8_t *ok;                   // verify: ok[i] = frame i (FCS trailer included) checks
    std::atomic<uint64_t> *bad;    //   ... count of frames that do not
};

constexpr uint32_t kResidue = 0x2144DF1Cu;   // ether_fcs(frame || LE32(ether_fcs(frame)))

constexpr uint64_t kChunkBytesHost = 128ull << 20;   // per pipeline slot
constexpr uint64_t kChunkFramesMax = 1ull << 20;

int run_host_job_body(DevState *ds, const HostJob &job, bool &launched);

// Runs the chunked H2D -> kernel -> D2H pipeline of one device over frames [i0, i1). A failure after
// anything was enqueued retires the pipeline (retire_pipe): a chunk's kernel or copy may still run.
int run_host_job(DevState *ds, const HostJob &job) {
    std::lock_guard<std::mutex> lk(ds->pipe_mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    bool launched = false;
    const int rc = run_host_job_body(ds, job, launched);
    if (rc && launched) retire_pipe(ds);
    return rc;
}

int run_host_job_body(DevState *ds, const HostJob &job, bool &launched) {
    int rc = ensure_pipe(ds, kChunkBytesHost + 2 * fcs::kSegBytes, kChunkFramesMax);
    if (rc) return rc;
    Pipe &pp = ds->pipe;
    const bool var = job.off || job.len;
    const bool src_pinned = is_pinned(job.arena);

    struct Pending { bool live = false; uint64_t i0 = 0, n = 0; } pend[Pipe::kDepth];
    auto drain = [&](int b) -> int {
        if (!pend[b].live) return 0;
        if (injected_late_fault()) return fail(ETIMEDOUT, "host pipeline: injected late fault (FCS_FAULT_HOOK build)");
        HIPTRY(hipEventSynchronize(pp.done[b]), "hipEventSynchronize");
        if (job.out && !job.ok && !job.tx_base) {   // plain CRCs: one copy
            std::memcpy(job.out + pend[b].i0, pp.h_out[b], pend[b].n * 4);
            pend[b].live = false;
            return 0;
        }
        for (uint64_t q = 0; q < pend[b].n; q++) {
            const uint64_t i = pend[b].i0 + q;
            const uint32_t c = pp.h_out[b][q];
            if (job.out) job.out[i] = c;
            if (job.ok) {
                job.ok[i] = c == kResidue;
                if (c != kResidue) job.bad->fetch_add(1, std::memory_order_relaxed);
            }
            if (job.tx_base) {   // src/linux/ether.c:263 — memcpy of the host-order u32
                uint8_t *dst = job.tx_base + (job.off ? job.off[i] : i * job.stride) + job.len[i];
                std::memcpy(dst, &c, 4);
            }
        }
        pend[b].live = false;
        return 0;
    };

    uint64_t i = job.i0;
    int slot = 0;
    uint64_t est = kChunkFramesMax;   // frames per chunk to try first (variable-length batches)
#ifdef FCS_HOST_TRACE   // measurement-only: where the host thread's time goes, per call
    using hclk = std::chrono::steady_clock;
    double tr[5] = {0, 0, 0, 0, 0};   // drain wait, chunk plan, staging, enqueue, final drain
    const auto tr0 = hclk::now();
    auto trs = [&](int k, hclk::time_point a) { tr[k] += std::chrono::duration<double, std::milli>(hclk::now() - a).count(); };
#define FCS_TR(k, a) trs(k, a)
#define FCS_TR_AT(a) const auto a = hclk::now()
#else
#define FCS_TR(k, a)
#define FCS_TR_AT(a)
#endif
    while (i < job.i1) {
        const int b = slot % Pipe::kDepth;
        FCS_TR_AT(ta);
        if ((rc = drain(b))) return rc;
        FCS_TR(0, ta);
        FCS_TR_AT(tb);
        // ---- choose the chunk [i, e) and the host byte span it needs ----
        uint64_t e = i, lo = 0, hi = 0, sum = 0;
        if (!job.off) {
            // frame q at arena + q*stride; span [i*stride, (e-1)*stride + len_q)
            const uint64_t per = std::max<uint64_t>(job.stride, 1);
            uint64_t cnt = std::min<uint64_t>(std::max<uint64_t>(1, kChunkBytesHost / per), kChunkFramesMax);
            e = std::min(job.i1, i + cnt);
            lo = i * job.stride;
            uint32_t lastlen = job.len ? job.len[e - 1] : job.flen;
            hi = (e - 1) * job.stride + lastlen;
            if (job.len)
                for (uint64_t q = i; q < e; q++) hi = std::max<uint64_t>(hi, q * job.stride + job.len[q]);
            if (hi - lo > kChunkBytesHost + 2 * fcs::kSegBytes) {   // a single giant frame
                if (e - i > 1) { e = i + 1; hi = i * job.stride + (job.len ? job.len[i] : job.flen); }
                else return fail(EINVAL, "frame %llu of %llu bytes exceeds the %llu-byte host chunk",
                                 (unsigned long long)i, (unsigned long long)(hi - lo),
                                 (unsigned long long)kChunkBytesHost);
            }
        } else {
            // frames [i, i + cnt) whose span and byte sum both fit the chunk: one branch-free
            // min/max/sum pass over a candidate count (the previous chunk's, grown), shrunk by the
            // overshoot until it fits (a frame-by-frame walk with an early exit was the host path's
            // bottleneck on IMIX: ~3 ns per frame against ~6 ns of PCIe time)
            uint64_t cnt = std::min<uint64_t>(job.i1 - i, std::min<uint64_t>(kChunkFramesMax, est));
            for (;;) {
                uint64_t l = UINT64_MAX, h = 0, sm = 0;
                const uint64_t *op = job.off + i;
                const uint32_t *lp = job.len + i;
                for (uint64_t q = 0; q < cnt; q++) {
                    const uint64_t a = op[q], z = a + lp[q];
                    l = a < l ? a : l;
                    h = z > h ? z : h;
                    sm += lp[q];
                }
                // a span far larger than the frames' bytes (shuffled or sparse offsets) is gathered
                // into the staging buffer instead, so only the bytes must fit
                const bool sparse = h - l > 2 * sm;
                const uint64_t need = sparse ? sm : std::max(h - l, sm);
                if (need <= kChunkBytesHost || cnt == 1) {
                    lo = l;
                    hi = h;
                    sum = sm;
                    e = i + cnt;
                    // next candidate: this count scaled to the chunk size (at most 1/8 more)
                    const uint64_t g = need ? (uint64_t)((double)cnt * (double)kChunkBytesHost / (double)need) : cnt * 2;
                    est = std::max<uint64_t>(1, std::min<uint64_t>(g, cnt + cnt / 8 + 1));
                    break;
                }
                cnt = std::max<uint64_t>(1, std::min<uint64_t>(cnt - 1, (uint64_t)((double)cnt * (double)kChunkBytesHost / (double)need * 0.98)));
            }
            if (hi - lo > kChunkBytesHost + 2 * fcs::kSegBytes && e - i == 1)
                return fail(EINVAL, "frame %llu of %llu bytes exceeds the %llu-byte host chunk",
                            (unsigned long long)i, (unsigned long long)job.len[i],
                            (unsigned long long)kChunkBytesHost);
        }
        FCS_TR(1, tb);
        FCS_TR_AT(tc);
        const uint64_t n = e - i;
        uint64_t *ho = pp.h_off[b];
        uint32_t *hl = reinterpret_cast<uint32_t *>(ho + n);   // lengths right after the offsets
        uint64_t span = hi - lo;
        const bool gather = job.off && (span > kChunkBytesHost || span > 2 * sum);   // sparse: pack frames
        const uint8_t *src = job.arena + lo;
        if (gather) {
            uint64_t w = 0;
            for (uint64_t q = 0; q < n; q++) {
                std::memcpy(pp.h_in[b] + w, job.arena + job.off[i + q], job.len[i + q]);
                ho[q] = w;
                hl[q] = job.len[i + q];
                w += job.len[i + q];
            }
            span = w;
            src = pp.h_in[b];
        } else {
            if (var) {
                const uint32_t *lp = job.len + i;
                if (job.off) {
                    const uint64_t *op = job.off + i;
                    for (uint64_t q = 0; q < n; q++) {
                        ho[q] = op[q] - lo;
                        hl[q] = lp[q];
                    }
                } else {
                    for (uint64_t q = 0; q < n; q++) {
                        ho[q] = (i + q) * job.stride - lo;
                        hl[q] = lp[q];
                    }
                }
            }
            if (!src_pinned) {
                fcs::staging_copy(pp.h_in[b], src, span);
                src = pp.h_in[b];
            }
        }
        FCS_TR(2, tc);
        FCS_TR_AT(td);
        launched = true;
        HIPTRY(hipMemcpyAsync(pp.d_in[b], src, span, hipMemcpyHostToDevice, pp.stream), "H2D frames");
        if (var) {
            HIPTRY(hipMemcpyAsync(pp.d_off[b], ho, n * 12, hipMemcpyHostToDevice, pp.stream), "H2D off, len");
        }
        HIPTRY(hipEventRecord(pp.landed[b], pp.stream), "hipEventRecord");
        HIPTRY(hipStreamWaitEvent(pp.cstream, pp.landed[b], 0), "hipStreamWaitEvent");
        if (var)
            rc = launch_var(ds, pp.d_in[b], span, pp.d_off[b], reinterpret_cast<const uint32_t *>(pp.d_off[b] + n),
                            pp.d_out[b], n, pp.cstream);
        else
            rc = launch_fixed(ds, pp.d_in[b], job.stride, job.flen, n, pp.d_out[b], pp.cstream);
        if (rc) return rc;
        HIPTRY(hipMemcpyAsync(pp.h_out[b], pp.d_out[b], n * 4, hipMemcpyDeviceToHost, pp.cstream), "D2H crc");
        HIPTRY(hipEventRecord(pp.done[b], pp.cstream), "hipEventRecord");
        pend[b].live = true;
        pend[b].i0 = i;
        pend[b].n = n;
        i = e;
        slot++;
        FCS_TR(3, td);
    }
    FCS_TR_AT(te);
    for (int b = 0; b < Pipe::kDepth; b++)
        if ((rc = drain(b))) return rc;
    FCS_TR(4, te);
#ifdef FCS_HOST_TRACE
    std::fprintf(stderr, "host_trace var=%d chunks=%d total_ms=%.3f drain_ms=%.3f plan_ms=%.3f stage_ms=%.3f enqueue_ms=%.3f final_ms=%.3f\n",
                 (int)var, slot, std::chrono::duration<double, std::milli>(hclk::now() - tr0).count(), tr[0], tr[1], tr[2], tr[3], tr[4]);
#endif
#undef FCS_TR
#undef FCS_TR_AT
    return 0;
}

// Small TX batches in pinned memory (the TX queue's arenas): no staging copies — the kernel reads
// the frames and writes the FCSs through device-mapped pinned memory, one launch, one sync; the
// host then stores each FCS little-endian after its covered bytes (src/linux/ether.c:263).
#ifndef FCS_ZC_MAX_MB   // measurement builds (tools/variants.sh) move the limit
#define FCS_ZC_MAX_MB 64
#endif
constexpr uint64_t kZeroCopyMaxBytes = (uint64_t)FCS_ZC_MAX_MB << 20;

// Small-batch resources on the TX/verify stream (caller holds tx_mu).
int ensure_small(DevState *ds) {
    if (!ds->tx_stream) {
        HIPTRY(hipStreamCreateWithFlags(&ds->tx_stream, hipStreamNonBlocking), "hipStreamCreate");
        HIPTRY(hipHostMalloc(&ds->tx_flag, 64, hipHostMallocMapped), "hipHostMalloc(tx flag)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->tx_dflag, ds->tx_flag, 0), "hipHostGetDevicePointer(flag)");
        *ds->tx_flag = 0;
    }
    if (!ds->tx_dcount) {
        // zeroed on tx_stream itself, ahead of every launch on it: a device-wide sync here would wait
        // on a retired stream whose kernel may never finish (the case retire_small isolates)
        HIPTRY(hipMalloc(&ds->tx_dcount, 64), "hipMalloc(small batch counter)");
        HIPTRY(hipMemsetAsync(ds->tx_dcount, 0, 64, ds->tx_stream), "hipMemsetAsync(small batch counter)");
        ds->tx_count = 0;
    }
    return 0;
}

// A call on the small-batch stream failed after its launch (a timeout, a lost completion): the
// kernel may still run and write the stream's mapped results (tx_out, vz_ok), its completion word
// and the frame counter whose value later launches' completion test relies on. All of them are set
// aside and recreated on next use; completions numbered before the new stream's first one
// (tx_first_seq) are waited for on the retired stream's own word (tx_old). Caller holds tx_mu.
void retire_small(DevState *ds) {
    if (ds->tx_stream && ds->tx_seq >= ds->tx_first_seq)
        ds->tx_old.push_back({ds->tx_first_seq, ds->tx_seq, ds->tx_stream, ds->tx_flag});
    quarantine(ds, ds->tx_stream, {ds->tx_flag, ds->tx_len, ds->tx_out, ds->tx_off, ds->vz_off, ds->vz_len, ds->vz_ok},
               {ds->tx_dcount, ds->vz_dbad});
    ds->tx_stream = nullptr;
    ds->tx_flag = ds->tx_dflag = nullptr;
    ds->tx_len = ds->tx_out = ds->tx_dlen = ds->tx_dout = nullptr;
    ds->tx_off = ds->tx_doff = nullptr;
    ds->vz_off = ds->vz_doff = nullptr;
    ds->vz_len = ds->vz_dlen = nullptr;
    ds->vz_ok = ds->vz_dok = nullptr;
    ds->vz_dbad = nullptr;
    ds->tx_dcount = nullptr;
    ds->tx_count = 0;
    ds->tx_cap = ds->vz_cap = 0;
    ds->tx_first_seq = ds->tx_seq + 1;
    (void)hipGetLastError();
    g_retired.fetch_add(1, std::memory_order_relaxed);
}


int run_tx_zero_copy(DevState *ds, uint8_t *base, uint64_t bytes, uint64_t stride, const uint64_t *off,
                     const uint32_t *len, uint64_t n) {
    std::lock_guard<std::mutex> lk(ds->tx_mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    int rc = ensure_small(ds);
    if (rc) return rc;
    if (n > ds->tx_cap) {
        const uint64_t cap = std::max<uint64_t>({n, 2 * ds->tx_cap, 4096});   // few growths, few kept arrays
        release(ds, {ds->tx_len, ds->tx_out, ds->tx_off});
        ds->tx_len = ds->tx_out = nullptr;
        ds->tx_off = nullptr;
        ds->tx_cap = 0;
        HIPTRY(hipHostMalloc(&ds->tx_len, cap * 4, hipHostMallocMapped), "hipHostMalloc(tx len)");
        HIPTRY(hipHostMalloc(&ds->tx_out, cap * 4, hipHostMallocMapped), "hipHostMalloc(tx out)");
        HIPTRY(hipHostMalloc(&ds->tx_off, cap * 8, hipHostMallocMapped), "hipHostMalloc(tx off)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->tx_dlen, ds->tx_len, 0), "hipHostGetDevicePointer(len)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->tx_dout, ds->tx_out, 0), "hipHostGetDevicePointer(out)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->tx_doff, ds->tx_off, 0), "hipHostGetDevicePointer(off)");
        ds->tx_cap = cap;
    }
    void *dbase = pinned_dev_ptr(base, bytes);   // our own arenas: no HIP query
    if (!dbase && hipHostGetDevicePointer(&dbase, base, 0) != hipSuccess) {   // pinned but not mapped
        (void)hipGetLastError();
        return 1;
    }
    bool small = n <= fcs::kTxSmallMax;
    for (uint64_t i = 0; small && i < n; i++) small = len[i] <= fcs::kOneBytes;
    if (const uint32_t *hw = take_hold()) {   // FCS_FAULT_HOOK builds only
        const uint32_t *dw = reinterpret_cast<const uint32_t *>(pinned_dev_ptr(hw, 4));
        if (dw) HIPTRY(fcs::launch_hold(dw, 20ull * 100000000ull, ds->tx_stream), "launching the hold kernel");
    }
    uint64_t v = 0;
    if (small) {   // everything the kernel needs rides in its arguments; it writes the FCSs to tx_out
        const std::vector<uint32_t> &kinit = kinit_table();
        fcs::TxSmallArgs a;
        a.flag = ds->tx_dflag;
        a.ok = nullptr;
        a.out = ds->tx_dout;
        a.count = ds->tx_dcount;
        a.count_base = ds->tx_count;
        a.blob = ds->d_one_blob;
        a.base = (uint8_t *)dbase;
        a.seq = v = ++ds->tx_seq;
        a.n = (uint32_t)n;
        a.pad = 0;
        for (uint64_t i = 0; i < n; i++) {
            a.off[i] = off ? off[i] : i * stride;
            a.len[i] = len[i];
            a.kinit[i] = kinit[len[i]];
        }
        HIPTRY(fcs::launch_tx_small(a, ds->tx_stream), "launching the small TX kernel");
        ds->tx_count += n;
    } else {
        std::memcpy(ds->tx_len, len, n * 4);
        if (off) std::memcpy(ds->tx_off, off, n * 8);
        if ((rc = launch_var(ds, dbase, bytes, off ? ds->tx_doff : nullptr, ds->tx_dlen, ds->tx_dout, n, ds->tx_stream,
                             nullptr, nullptr, off ? 0 : stride))) {
            retire_small(ds);   // the arena-stream kernel may have started before a later launch failed
            return rc;
        }
        v = ++ds->tx_seq;
        if (const hipError_t e = fcs::launch_signal(ds->tx_dflag, v, ds->tx_stream); e != hipSuccess) {
            rc = hip_fail(e, "launching signal");
            retire_small(ds);   // the FCS kernel is in flight
            return rc;
        }
    }
    // the kernel is in flight: a failed wait leaves it so, and it may still write tx_out
    rc = injected_late_fault() ? fail(ETIMEDOUT, "small TX batch: injected late fault (FCS_FAULT_HOOK build)")
                               : wait_flag(ds->tx_stream, ds->tx_flag, v, "small TX batch");
    if (rc) {
        retire_small(ds);
        return rc;
    }
    for (uint64_t i = 0; i < n; i++) std::memcpy(base + (off ? off[i] : i * stride) + len[i], &ds->tx_out[i], 4);
    return 0;
}

// One frame of at most kOneBytes through fcs_one_kernel: the frame rides in the kernel arguments
// and the FCS comes back in the calling thread's lane's mapped result word. Any host memory.
uint32_t my_lane() {
    static std::atomic<uint32_t> next_thread{0};
    thread_local const uint32_t me = next_thread.fetch_add(1, std::memory_order_relaxed);
    return me % DevState::kOneLanes;
}

// Drop a lane whose last call failed: its stream and result word are recreated on next use, so a
// stream left in an error state or a result word a stuck kernel may still write is never reused.
void reset_lane(DevState *ds, DevState::OneLane &L) {
    quarantine(ds, L.st, {L.flag});
    L.st = nullptr;
    L.flag = L.dflag = nullptr;
    L.seq = 0;
    (void)hipGetLastError();
    g_lane_resets.fetch_add(1, std::memory_order_relaxed);
}

int run_one(DevState *ds, const void *data, size_t bsize, uint32_t *crc, uint32_t lane, bool batch = false) {
    DevState::OneLane &L = ds->one_lane[lane % DevState::kOneLanes];
    std::lock_guard<std::mutex> lk(L.mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    if (injected_fault()) {
        reset_lane(ds, L);
        return fail(EIO, "single-frame kernel: injected fault (FCS_FAULT_HOOK build)");
    }
    if (!L.st) {
        HIPTRY(hipStreamCreateWithFlags(&L.st, hipStreamNonBlocking), "hipStreamCreate");
        HIPTRY(hipHostMalloc(&L.flag, 64, hipHostMallocMapped), "hipHostMalloc(result word)");
        HIPTRY(hipHostGetDevicePointer((void **)&L.dflag, L.flag, 0), "hipHostGetDevicePointer(result word)");
        *L.flag = 0;
    }
    fcs::OneArgs a;
    a.flag = L.dflag;
    a.blob = ds->d_one_blob;
    if (++L.seq == 0) L.seq = 1;   // 0 never names a completion
    a.seq = L.seq;
    a.kinit = kinit_table()[bsize];
    uint8_t *win = reinterpret_cast<uint8_t *>(a.data);
    std::memset(win, 0, fcs::kOneBytes - bsize);
    if (bsize) std::memcpy(win + fcs::kOneBytes - bsize, data, bsize);
    if (const hipError_t le = fcs::launch_one(a, L.st); le != hipSuccess) {
        const int r = hip_fail(le, "launching the single-frame kernel");
        reset_lane(ds, L);
        return r;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 1;; i++) {
        const uint64_t v = __atomic_load_n(L.flag, __ATOMIC_ACQUIRE);
        if ((uint32_t)(v >> 32) == a.seq) {
            *crc = (uint32_t)v;
            return 0;
        }
        // FCS_FAULT_HOOK builds only: give up with the kernel in flight (drop-in, or a one-frame host batch)
        if (i == 1) {
            const bool late = batch && injected_late_fault();
            if (late || injected_timeout()) {
                reset_lane(ds, L);
                return fail(ETIMEDOUT, "single-frame kernel: injected %s (FCS_FAULT_HOOK build)",
                            late ? "late fault" : "timeout");
            }
        }
        __builtin_ia32_pause();
        if ((i & 4095) == 0) {
            const hipError_t q = hipStreamQuery(L.st);
            if (q == hipSuccess && (uint32_t)(__atomic_load_n(L.flag, __ATOMIC_ACQUIRE) >> 32) != a.seq) {
                reset_lane(ds, L);
                return fail(EIO, "single-frame kernel finished without a result");
            }
            if (q != hipSuccess && q != hipErrorNotReady) {
                const int r = hip_fail(q, "single-frame kernel");
                reset_lane(ds, L);
                return r;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                reset_lane(ds, L);
                return fail(ETIMEDOUT, "single-frame kernel: no result after 10 s");
            }
        }
    }
}

// Small RX verify batches in fcs_host_alloc memory (the RX queue's arena): the kernel reads the
// frames and writes the ok flags and the bad count through mapped memory, one launch and a
// completion word, as run_tx_zero_copy does for TX. Returns the bad count or -errno.
int64_t run_verify_zero_copy(DevState *ds, const uint8_t *darena, uint64_t arena_bytes, const uint64_t *off,
                             const uint32_t *len, uint8_t *ok, uint64_t n) {
    std::lock_guard<std::mutex> lk(ds->tx_mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    int rc = ensure_small(ds);
    if (rc) return rc;
    if (n > ds->vz_cap) {
        const uint64_t cap = std::max<uint64_t>({n, 2 * ds->vz_cap, 4096});
        release(ds, {ds->vz_off, ds->vz_len, ds->vz_ok});
        ds->vz_off = nullptr;
        ds->vz_len = nullptr;
        ds->vz_ok = nullptr;
        ds->vz_cap = 0;
        HIPTRY(hipHostMalloc(&ds->vz_off, cap * 8, hipHostMallocMapped), "hipHostMalloc(verify off)");
        HIPTRY(hipHostMalloc(&ds->vz_len, cap * 4, hipHostMallocMapped), "hipHostMalloc(verify len)");
        HIPTRY(hipHostMalloc(&ds->vz_ok, cap, hipHostMallocMapped), "hipHostMalloc(verify ok)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->vz_doff, ds->vz_off, 0), "hipHostGetDevicePointer(off)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->vz_dlen, ds->vz_len, 0), "hipHostGetDevicePointer(len)");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->vz_dok, ds->vz_ok, 0), "hipHostGetDevicePointer(ok)");
        ds->vz_cap = cap;
    }
    if (!ds->vz_dbad) HIPTRY(hipMalloc(&ds->vz_dbad, 64), "hipMalloc(verify bad scratch)");
    bool small = n <= fcs::kTxSmallMax;
    for (uint64_t i = 0; small && i < n; i++) small = len[i] <= fcs::kOneBytes;
    uint64_t v = 0;
    if (small) {   // the small-batch kernel in verify mode: frame list in its arguments
        const std::vector<uint32_t> &kinit = kinit_table();
        fcs::TxSmallArgs a;
        a.flag = ds->tx_dflag;
        a.blob = ds->d_one_blob;
        a.base = (uint8_t *)darena;
        a.ok = ds->vz_dok;
        a.out = nullptr;
        a.count = ds->tx_dcount;
        a.count_base = ds->tx_count;
        a.seq = v = ++ds->tx_seq;
        a.n = (uint32_t)n;
        a.pad = 0;
        for (uint64_t i = 0; i < n; i++) {
            a.off[i] = off[i];
            a.len[i] = len[i];
            a.kinit[i] = kinit[len[i]];
        }
        HIPTRY(fcs::launch_tx_small(a, ds->tx_stream), "launching the small verify kernel");
        ds->tx_count += n;
    } else {
        std::memcpy(ds->vz_off, off, n * 8);
        std::memcpy(ds->vz_len, len, n * 4);
        if ((rc = launch_var(ds, darena, arena_bytes, ds->vz_doff, ds->vz_dlen, nullptr, n, ds->tx_stream, ds->vz_dok,
                             ds->vz_dbad))) {
            retire_small(ds);   // the arena-stream kernel may have started before a later launch failed
            return rc;
        }
        v = ++ds->tx_seq;
        if (const hipError_t e = fcs::launch_signal(ds->tx_dflag, v, ds->tx_stream); e != hipSuccess) {
            rc = hip_fail(e, "launching signal");
            retire_small(ds);   // the verify kernel is in flight
            return rc;
        }
    }
    // the kernel is in flight: a failed wait leaves it so, and it may still write vz_ok
    rc = injected_late_fault() ? fail(ETIMEDOUT, "small verify batch: injected late fault (FCS_FAULT_HOOK build)")
                               : wait_flag(ds->tx_stream, ds->tx_flag, v, "small verify batch");
    if (rc) {
        retire_small(ds);
        return rc;
    }
    std::memcpy(ok, ds->vz_ok, n);
    int64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) bad += ok[i] == 0;
    return bad;
}

int engine_devices(std::vector<DevState *> *out) {
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (g_engine_devs.empty()) {
            int ndev = 0;
            hipError_t e = hipGetDeviceCount(&ndev);
            if (e != hipSuccess || ndev <= 0) return fail(ENODEV, "no HIP device visible (%s)", hipGetErrorString(e));
            for (int d = 0; d < ndev; d++) g_engine_devs.push_back(d);
        }
    }
    std::vector<int> devs;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        devs = g_engine_devs;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return fail(ENODEV, "no HIP device visible (%s)", hipGetErrorString(e));
    out->clear();
    for (int d : devs) {
        DevState *ds = nullptr;
        int rc = d < ndev ? dev_state(d, &ds) : alias_state(d, ndev, &ds);
        if (rc) return rc;
        out->push_back(ds);
    }
    return 0;
}

// A TX batch of one frame (a sync ether_send caller on its own): the single-frame kernel, from any
// host memory, and the FCS stored here (src/linux/ether.c:263).
int tx_one(uint8_t *frame, uint32_t len) {
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    uint32_t c = 0;
    if ((rc = run_one(devs[0], frame, len, &c, my_lane(), true))) return rc;
    std::memcpy(frame + len, &c, 4);
    return 0;
}


// Every frame [off, off + len + tail) inside [0, arena_bytes): -EINVAL naming the first that is not.
// The host-inclusive calls check the whole batch before anything runs, so nothing is written on an
// error. The check is branch-free and, from 1 M frames up, split over 8 threads: one thread
// walking IMIX offsets and lengths took ~4 % of a 4 GiB host-inclusive call (tools/ab_host.py).
int check_frames(const uint64_t *off, const uint32_t *len, uint64_t n, uint64_t arena_bytes, uint32_t tail,
                 const char *what) {
    auto bad_in = [=](uint64_t a, uint64_t z) {
        uint64_t bad = 0;
        for (uint64_t i = a; i < z; i++) {
            const uint64_t o = off[i], l = (uint64_t)len[i] + tail;
            bad |= (uint64_t)(o > arena_bytes) | (uint64_t)(l > arena_bytes - o);
        }
        return bad != 0;
    };
    constexpr uint64_t kSplit = 1ull << 20;
    constexpr int kThreads = 8;
    bool bad = false;
    if (n < kSplit) {
        bad = bad_in(0, n);
    } else {
        bool part_bad[kThreads] = {};
        std::thread th[kThreads - 1];
        const uint64_t per = (n + kThreads - 1) / kThreads;
        for (int t = 1; t < kThreads; t++)
            th[t - 1] = std::thread([&, t] { part_bad[t] = bad_in(std::min(n, per * t), std::min(n, per * (t + 1))); });
        part_bad[0] = bad_in(0, std::min(n, per));
        for (auto &x : th) x.join();
        for (int t = 0; t < kThreads; t++) bad |= part_bad[t];
    }
    if (!bad) return 0;
    for (uint64_t i = 0; i < n; i++)
        if (off[i] > arena_bytes || (uint64_t)len[i] + tail > arena_bytes - off[i])
            return fail(EINVAL, "frame %llu [%llu, +%u)%s outside the %llu-byte arena", (unsigned long long)i,
                        (unsigned long long)off[i], len[i], tail ? " and its FCS" : "", (unsigned long long)arena_bytes);
    return fail(EINVAL, "%s: frame check", what);   // not reached
}

std::atomic<uint64_t> g_sharded_calls{0}, g_shard_jobs{0};

// Shard [0, n) over the engine devices (contiguous ranges, byte-balanced when lengths are known:
// fcs_shard_plan).
int run_host_sharded(HostJob job, uint64_t n) {
    if (n == 0) return 0;
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    const uint64_t G = std::min<uint64_t>(devs.size(), std::max<uint64_t>(1, n / 1024));
    std::vector<uint64_t> cut(G + 1, 0);
    if (G > 1 && (rc = fcs_shard_plan(job.len, n, (uint32_t)G, cut.data()))) return rc;
    if (G == 1) {
        job.i0 = 0;
        job.i1 = n;
        return run_host_job(devs[0], job);
    }
    g_sharded_calls.fetch_add(1, std::memory_order_relaxed);
    g_shard_jobs.fetch_add(G, std::memory_order_relaxed);
    std::vector<int> rcs(G, 0);
    std::vector<std::string> errs(G);
    std::vector<std::thread> th;
    for (uint64_t g = 0; g < G; g++) {
        th.emplace_back([&, g] {
            HostJob jj = job;
            jj.i0 = cut[g];
            jj.i1 = cut[g + 1];
            rcs[g] = jj.i0 < jj.i1 ? run_host_job(devs[g], jj) : 0;
            errs[g] = g_last_error;
        });
    }
    for (auto &t : th) t.join();
    for (uint64_t g = 0; g < G; g++)
        if (rcs[g]) {
            g_last_error = errs[g];
            return rcs[g];
        }
    return 0;
}

// The host CRC's answer to a host batch call ("on any HIP error, fall back to the CPU
// path so results never differ"): fcs_host_crc.cpp, the product's own slice-by-16 (never the oracle).
// Plain CRCs, TX mode (the FCS stored little-endian after each frame, src/linux/ether.c:263) or RX
// verify (ok[i]; returns the count of failing frames). Large batches are split over 8 threads.
int64_t host_answer(const HostJob &job, uint64_t n) {
    auto part = [&job](uint64_t a, uint64_t z) -> uint64_t {
        uint64_t bad = 0;
        for (uint64_t i = a; i < z; i++) {
            const uint64_t o = job.off ? job.off[i] : i * job.stride;
            const uint32_t L = job.len ? job.len[i] : job.flen;
            const uint32_t c = fcs::host_crc32(job.arena + o, L);
            if (job.out) job.out[i] = c;
            if (job.ok) {
                job.ok[i] = c == kResidue;   // no input of 0..3 bytes has the residue as its CRC
                bad += c != kResidue;
            }
            if (job.tx_base) std::memcpy(job.tx_base + o + L, &c, 4);
        }
        return bad;
    };
    constexpr uint64_t kSplit = 1ull << 16;
    constexpr int kThreads = 8;
    if (n < kSplit) return (int64_t)part(0, n);
    uint64_t bad[kThreads] = {};
    std::thread th[kThreads - 1];
    const uint64_t per = (n + kThreads - 1) / kThreads;
    for (int t = 1; t < kThreads; t++)
        th[t - 1] = std::thread([&, t] { bad[t] = part(std::min(n, per * t), std::min(n, per * (t + 1))); });
    bad[0] = part(0, std::min(n, per));
    uint64_t sum = 0;
    for (auto &x : th) x.join();
    for (uint64_t b : bad) sum += b;
    return (int64_t)sum;
}

// A host batch form's GPU step, answered by the host CRC when it fails with a runtime error: -EIO,
// -ETIMEDOUT, -ENOMEM or any other errno but -EINVAL (bad arguments, nothing written) and -ENODEV
// (no usable gfx950 GPU or code object at all: the batch forms fail loudly then, they never turn
// into a CPU library). Such calls are counted in fcs_engine_host_batches, the first is reported on
// stderr, and fcs_last_error() keeps the GPU step's error. A failed GPU step never leaves a kernel
// that can still write into the caller's memory: results go through the library's own staging or
// mapped arrays, which are retired on such a failure (retire_pipe, retire_small). After kMaxRetired
// retirements the forms answer from the host CRC without calling the GPU (host_only).
template <class F>
int64_t with_host_answer(const char *site, const HostJob &job, uint64_t n, F gpu) {
    t_host_answered = false;
    int64_t rc;
    if (injected_batch_fault()) rc = fail(EIO, "%s: injected fault (FCS_FAULT_HOOK build)", site);
    else if (host_only()) rc = fail(EIO, "%s: the host batch forms stopped using the GPU after %u failed calls", site, kMaxRetired);
    else rc = gpu();
    if (rc >= 0 || rc == -EINVAL || rc == -ENODEV) return rc;
    const std::string why = g_last_error;
    fcs::host_batch_answered(site, why.c_str());
    t_host_answered = true;
    const int64_t r = host_answer(job, n);
    g_last_error = std::string(site) + " answered by the host CRC after: " + why;
    return job.ok ? r : 0;
}

// Frames over kOneBytes (no Ethernet frame is): copied into pinned, device-mapped staging and run
// through the fixed-length kernels on the device's staging stream. On an error the staging stream
// and words are dropped, so a retry starts from fresh ones.
int run_staged(DevState *ds, const void *data, size_t bsize, uint32_t *crc) {
    std::lock_guard<std::mutex> lk(ds->one_mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    auto reset = [ds] {   // the staging buffer one_h is kept: no kernel writes it
        quarantine(ds, ds->one_stream, {ds->one_hout, ds->one_flag});
        ds->one_stream = nullptr;
        ds->one_hout = ds->one_dout = nullptr;
        ds->one_flag = ds->one_dflag = nullptr;
        (void)hipGetLastError();
        g_lane_resets.fetch_add(1, std::memory_order_relaxed);
    };
    if (injected_fault()) {
        reset();
        return fail(EIO, "staged ether_fcs: injected fault (FCS_FAULT_HOOK build)");
    }
    int rc = 0;
    hipError_t e = hipSuccess;
    if (!ds->one_stream) {   // zero-copy: the kernel reads the frame and writes the FCS in pinned memory
        if ((e = hipStreamCreateWithFlags(&ds->one_stream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipHostMalloc(&ds->one_hout, 64, hipHostMallocMapped)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void **)&ds->one_dout, ds->one_hout, 0)) != hipSuccess ||
            (e = hipHostMalloc(&ds->one_flag, 64, hipHostMallocMapped)) != hipSuccess ||
            (e = hipHostGetDevicePointer((void **)&ds->one_dflag, ds->one_flag, 0)) != hipSuccess) {
            rc = hip_fail(e, "staged ether_fcs: stream and result words");
            reset();
            return rc;
        }
        ds->one_flag[0] = ds->one_flag[1] = 0;
        ds->one_seq = 0;
    }
    if (bsize > ds->one_cap) {
        release(ds, {ds->one_h});
        ds->one_h = ds->one_hd = nullptr;
        ds->one_cap = 0;
        const uint64_t cap = std::max<uint64_t>(4096, bsize + 64);
        HIPTRY(hipHostMalloc(&ds->one_h, cap, hipHostMallocMapped), "staged ether_fcs: hipHostMalloc");
        HIPTRY(hipHostGetDevicePointer((void **)&ds->one_hd, ds->one_h, 0), "staged ether_fcs: map");
        ds->one_cap = cap - 64;
    }
    std::memcpy(ds->one_h, data, bsize);
    rc = launch_fixed(ds, ds->one_hd, bsize, (uint32_t)bsize, 1, ds->one_dout, ds->one_stream);
    const uint64_t v = ++ds->one_seq;
    if (!rc && (e = fcs::launch_signal(ds->one_dflag, v, ds->one_stream)) != hipSuccess)
        rc = hip_fail(e, "staged ether_fcs: signal");
    if (!rc) rc = wait_flag(ds->one_stream, ds->one_flag, v, "ether_fcs");
    if (rc) {
        reset();
        return rc;
    }
    *crc = ds->one_hout[0];
    return 0;
}

int dropin_attempt(const void *data, size_t bsize, uint32_t lane, uint32_t *crc) {
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    if (bsize <= fcs::kOneBytes) return run_one(devs[0], data, bsize, crc, lane);
    return run_staged(devs[0], data, bsize, crc);
}

}  // namespace

// Pageable host bytes are copied into pinned staging before their DMA; one core copies
// ~28 GB/s, below PCIe Gen5 x16, so large spans are split over a few threads.
int fcs::mapped_submit(uint8_t *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len, uint8_t *ok,
                       uint64_t n, uint64_t *ticket) {
    if (!arena || !off || !len || !ok || !ticket || n == 0) return fail(EINVAL, "mapped_submit: bad arguments");
    for (uint64_t i = 0; i < n; i++)
        if (len[i] > fcs::kOneBytes || off[i] > arena_bytes || len[i] > arena_bytes - off[i])
            return fail(EINVAL, "mapped_submit: frame %llu out of range", (unsigned long long)i);
    const uint8_t *da = pinned_dev_ptr(arena, arena_bytes);
    const uint8_t *doff = pinned_dev_ptr(off, n * 8), *dlen = pinned_dev_ptr(len, n * 4);
    uint8_t *dok = pinned_dev_ptr(ok, n);
    if (!da || !doff || !dlen || !dok) return fail(EINVAL, "mapped_submit: buffers not from fcs_host_alloc");
    if (injected_batch_fault()) return fail(EIO, "mapped_submit: injected fault (FCS_FAULT_HOOK build)");
    if (host_only()) return fail(EIO, "mapped_submit: the host batch forms stopped using the GPU after %u failed calls", kMaxRetired);
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    DevState *ds = devs[0];
    std::lock_guard<std::mutex> lk(ds->tx_mu);
    DeviceGuard dg(ds->dev);
    HIPTRY(dg.err, "hipSetDevice");
    if ((rc = ensure_small(ds))) return rc;
    if (n <= fcs::kTxSmallMax) {   // the list fits the kernel arguments: one PCIe round trip less
        const std::vector<uint32_t> &kinit = kinit_table();
        fcs::TxSmallArgs a;
        a.flag = ds->tx_dflag;
        a.blob = ds->d_one_blob;
        a.base = (uint8_t *)da;
        a.ok = dok;
        a.out = nullptr;
        a.count = ds->tx_dcount;
        a.count_base = ds->tx_count;
        a.seq = ds->tx_seq + 1;
        a.n = (uint32_t)n;
        a.pad = 0;
        for (uint64_t i = 0; i < n; i++) {
            a.off[i] = off[i];
            a.len[i] = len[i];
            a.kinit[i] = kinit[len[i]];
        }
        HIPTRY(fcs::launch_tx_small(a, ds->tx_stream), "launching the small-batch kernel");
        ds->tx_seq++;
        ds->tx_count += n;
        *ticket = a.seq;
        return 0;
    }
    fcs::ListArgs a;
    a.flag = ds->tx_dflag;
    a.blob = ds->d_one_blob;
    a.kinit = ds->d_kinit;
    a.base = (uint8_t *)da;
    a.off = (const uint64_t *)doff;
    a.len = (const uint32_t *)dlen;
    a.ok = dok;
    a.out = nullptr;
    a.count = ds->tx_dcount;
    a.count_base = ds->tx_count;
    a.seq = ds->tx_seq + 1;
    a.n = (uint32_t)n;
    a.pad = 0;
    HIPTRY(fcs::launch_small_list(a, ds->tx_stream), "launching the mapped-list kernel");
    ds->tx_seq++;
    ds->tx_count += n;
    *ticket = a.seq;
    return 0;
}

int fcs::mapped_wait(uint64_t ticket) {
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    DevState *ds = devs[0];
    hipStream_t st = nullptr;
    const uint64_t *flag = nullptr;
    {
        std::lock_guard<std::mutex> lk(ds->tx_mu);
        if (ticket >= ds->tx_first_seq && ds->tx_stream) {
            st = ds->tx_stream;
            flag = ds->tx_flag;
        } else {   // issued on a stream retired since (another batch's wait failed): wait on its word
            for (const DevState::OldGen &g : ds->tx_old)
                if (g.first <= ticket && ticket <= g.last) {
                    st = g.st;
                    flag = g.flag;
                }
            if (!st) return fail(EIO, "mapped_wait: no small-batch stream issued batch %llu", (unsigned long long)ticket);
        }
    }
    // injected: give up at once, as if the wait had timed out, with the kernel still in flight
    rc = injected_batch_fault() ? fail(ETIMEDOUT, "mapped_wait: injected fault (FCS_FAULT_HOOK build)")
                                : wait_flag(st, flag, ticket, "mapped-list batch");
    if (rc) {
        std::lock_guard<std::mutex> lk(ds->tx_mu);
        if (ds->tx_stream == st) retire_small(ds);   // not retired by another failed call meanwhile
    }
    return rc;
}

void fcs::host_batch_answered(const char *site, const char *why) {
    static std::atomic<bool> told{false};
    if (!told.exchange(true))
        std::fprintf(stderr, "nstack_fcs: %s: GPU step failed (%s); the batch is answered by the host CRC "
                             "(counted in fcs_engine_host_batches; reported once)\n", site, why ? why : "");
    g_host_batches.fetch_add(1, std::memory_order_relaxed);
}

bool fcs::last_call_host_answered() { return t_host_answered; }

void fcs::staging_copy(uint8_t *dst, const uint8_t *src, uint64_t bytes) {
    constexpr uint64_t kCopySplitBytes = 16ull << 20;
    constexpr int kCopyThreads = 4;
    if (bytes < kCopySplitBytes) {
        std::memcpy(dst, src, bytes);
        return;
    }
    const uint64_t part = ((bytes + kCopyThreads - 1) / kCopyThreads + 4095) & ~4095ull;
    std::thread th[kCopyThreads - 1];
    for (int t = 1; t < kCopyThreads; t++) {
        const uint64_t a = std::min(bytes, part * t), z = std::min(bytes, part * (t + 1));
        th[t - 1] = std::thread([=] { if (z > a) std::memcpy(dst + a, src + a, z - a); });
    }
    std::memcpy(dst, src, std::min(bytes, part));
    for (auto &x : th) x.join();
}

int fcs::current_device(int *dev, int *cus) {
    DevState *ds = nullptr;
    const int rc = current_dev_state(&ds);
    if (rc) return rc;
    *dev = ds->dev;
    *cus = ds->cus;
    return 0;
}

int fcs::launch_with_counter(int dev, void *stream, const std::function<int(unsigned long long *)> &launch) {
    hipStream_t st = (hipStream_t)stream;
    DevState *ds = nullptr;
    int rc = dev_state(dev, &ds);
    if (rc) return rc;
    CounterLease lease;   // released (completion event recorded) after the launch
    fcs::KParams p{};
    if ((rc = take_counter(ds, st, p, lease))) return rc;
    return launch(p.ctr);
}

int fcs::engine_device0(int *dev, int *cus) {
    std::vector<DevState *> devs;
    const int rc = engine_devices(&devs);
    if (rc) return rc;
    *dev = devs[0]->dev;
    *cus = devs[0]->cus;
    return 0;
}

int fcs::set_error(int err, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return -err;
}

// Release everything a device state holds (engine shutdown, or an alias state that is no longer an
// engine device). Caller holds g_mu.
static void destroy_state(DevState *ds) {
    hipSetDevice(ds->dev);
    Pipe &pp = ds->pipe;
    for (int b = 0; b < Pipe::kDepth; b++) {
        if (pp.done[b]) hipEventDestroy(pp.done[b]);
        if (pp.landed[b]) hipEventDestroy(pp.landed[b]);
        if (pp.d_in[b]) hipFree(pp.d_in[b]);
        if (pp.h_in[b]) hipHostFree(pp.h_in[b]);
        if (pp.d_off[b]) hipFree(pp.d_off[b]);
        if (pp.d_out[b]) hipFree(pp.d_out[b]);
        if (pp.h_off[b]) hipHostFree(pp.h_off[b]);
        if (pp.h_out[b]) hipHostFree(pp.h_out[b]);
    }
    if (pp.stream) hipStreamDestroy(pp.stream);
    if (pp.cstream) hipStreamDestroy(pp.cstream);
    if (ds->tx_stream) hipStreamDestroy(ds->tx_stream);
    if (ds->tx_len) hipHostFree(ds->tx_len);
    if (ds->tx_out) hipHostFree(ds->tx_out);
    if (ds->tx_off) hipHostFree(ds->tx_off);
    if (ds->tx_flag) hipHostFree(ds->tx_flag);
    if (ds->tx_dcount) hipFree(ds->tx_dcount);
    if (ds->vz_off) hipHostFree(ds->vz_off);
    if (ds->vz_len) hipHostFree(ds->vz_len);
    if (ds->vz_ok) hipHostFree(ds->vz_ok);
    if (ds->vz_dbad) hipFree(ds->vz_dbad);
    if (ds->one_stream) hipStreamDestroy(ds->one_stream);
    if (ds->one_h) hipHostFree(ds->one_h);
    if (ds->one_hout) hipHostFree(ds->one_hout);
    if (ds->one_flag) hipHostFree(ds->one_flag);
    for (DevState::OneLane &L : ds->one_lane) {
        if (L.st) hipStreamDestroy(L.st);
        if (L.flag) hipHostFree(L.flag);
    }
    if (!ds->q_streams.empty() || !ds->q_host.empty() || !ds->q_dev.empty()) (void)device_sync();
    for (hipStream_t q : ds->q_streams) hipStreamDestroy(q);
    for (void *h : ds->q_host) hipHostFree(h);
    for (void *d : ds->q_dev) hipFree(d);
    for (hipEvent_t ev : ds->ctr_done)
        if (ev) hipEventDestroy(ev);
    if (ds->d_blob) hipFree(ds->d_blob);
    if (ds->d_one_blob) hipFree(ds->d_one_blob);
    if (ds->d_kinit) hipFree(ds->d_kinit);
    if (ds->d_ctr) hipFree(ds->d_ctr);
    for (uint32_t *scr : ds->ctr_scr)
        if (scr) hipFree(scr);
}

extern "C" {

const char *fcs_last_error(void) { return g_last_error.c_str(); }

const char *fcs_engine_version(void) {
    return "nstack-fcs 0.6 gfx950: quarter-wave/frame, 96B lane windows as 2 slice-by-4 chains, v_perm "
           "addressing, DPP reduce; 1496-1524B: LDS-DMA (nt global_load_lds) 6KiB slot/wave, 16 waves/CU, "
           "32KiB 8-replica tables, guided dynamic items; 130-399B: 4 lanes x 36-104B, 400-868B: 8 lanes x 44-112B windows/frame, 870-1476B: 16 lanes x 60-96B windows, 6-7KiB LDS-DMA slots; <=128B: lane/frame; 1477-1495B, 1525-1988B: 104/120/128B-window LDS-DMA, 7/8KiB slots; "
           ">1524B otherwise: frame-interleaved LDS-DMA segments of 900-1988B (least m*(WD+8)); var: "
           "packed 64-1536B units as an arena stream (4KiB LDS-DMA items, taps at frame boundaries, XOR "
           "scan), other units as a flat chunk stream per 64-frame window";
}

int fcs_engine_init(int ndev) {
    int total = 0;
    hipError_t e = hipGetDeviceCount(&total);
    if (e != hipSuccess || total <= 0) return fail(ENODEV, "no HIP device visible (%s)", hipGetErrorString(e));
    const int use = ndev <= 0 ? total : ((ndev > total && !alias_devices_enabled()) ? total : ndev);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_engine_devs.clear();
        for (int d = 0; d < use; d++) g_engine_devs.push_back(d);
        // alias states (NSTACK_FCS_ALIAS_DEVICES test hook) of ids that are no longer engine
        // devices are retired, not destroyed: a concurrent host call may still hold a raw pointer
        // to one (taken from engine_devices before this init). fcs_engine_fini frees them.
        for (auto it = g_alias.begin(); it != g_alias.end();) {
            if (it->first >= use) {
                g_alias_retired.push_back(std::move(it->second));
                it = g_alias.erase(it);
            } else {
                ++it;
            }
        }
    }
    std::vector<DevState *> devs;
    int rc = engine_devices(&devs);
    if (rc) return rc;
    return use;
}

void fcs_engine_fini(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (auto &up : g_dev)
        if (up) destroy_state(up.get());
    for (auto &kv : g_alias)
        if (kv.second) destroy_state(kv.second.get());
    for (auto &up : g_alias_retired)
        if (up) destroy_state(up.get());
    g_last_stream_dev.store(nullptr, std::memory_order_relaxed);
    g_dev.clear();
    g_alias.clear();
    g_alias_retired.clear();
    g_engine_devs.clear();
    g_retired.store(0, std::memory_order_relaxed);   // the retired resources are freed with their states
    hipSetDevice(cur);
}

uint64_t fcs_engine_set_var_threshold(uint64_t frames) {
    return g_var_threshold.exchange(frames);
}

int fcs_engine_device_count(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_engine_devs.empty()) return (int)g_engine_devs.size();
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess) return 0;
    return total;
}

int ether_fcs_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                        uint32_t *out, void *stream) {
    if (n == 0) return 0;
    if (!base || !out) return fail(EINVAL, "null pointer");
    if (n > 1 && stride < len) return fail(EINVAL, "stride %llu < len %u", (unsigned long long)stride, len);
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    return launch_fixed(ds, base, stride, len, n, out, (hipStream_t)stream);
}

int ether_fcs_batch_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                        const uint32_t *len, uint32_t *out, uint64_t n, void *stream) {
    if (n == 0) return 0;
    if (!arena || !off || !len || !out) return fail(EINVAL, "null pointer");
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    return launch_var(ds, arena, arena_bytes, off, len, out, n, (hipStream_t)stream);
}

int ether_fcs_batch_host(const void *arena, uint64_t arena_bytes, const uint64_t *off,
                         const uint32_t *len, uint32_t *out, uint64_t n) {
    t_host_answered = false;   // early returns below must not report the previous call
    if (n == 0) return 0;
    if (!arena || !off || !len || !out) return fail(EINVAL, "null pointer");
    if (int rc = check_frames(off, len, n, arena_bytes, 0, __func__)) return rc;
    HostJob job{(const uint8_t *)arena, arena_bytes, off, len, 0, 0, out, nullptr, 0, n, nullptr, nullptr};
    return (int)with_host_answer(__func__, job, n, [&] { return (int64_t)run_host_sharded(job, n); });
}

int ether_fcs_fixed_host(const void *base, uint64_t stride, uint32_t len, uint64_t n,
                         uint32_t *out) {
    t_host_answered = false;   // early returns below must not report the previous call
    if (n == 0) return 0;
    if (!base || !out) return fail(EINVAL, "null pointer");
    if (n > 1 && stride < len) return fail(EINVAL, "stride %llu < len %u", (unsigned long long)stride, len);
    HostJob job{(const uint8_t *)base, (n - 1) * stride + len, nullptr, nullptr, n > 1 ? stride : len, len,
                out, nullptr, 0, n, nullptr, nullptr};
    return (int)with_host_answer(__func__, job, n, [&] { return (int64_t)run_host_sharded(job, n); });
}

int ether_fcs_tx_host(void *base, uint64_t stride, const uint32_t *len, uint64_t n) {
    t_host_answered = false;   // early returns below must not report the previous call
    if (n == 0) return 0;
    if (!base || !len) return fail(EINVAL, "null pointer");
    for (uint64_t i = 0; i < n; i++)
        if ((uint64_t)len[i] + 4 > stride)
            return fail(EINVAL, "frame %llu: len %u + FCS does not fit stride %llu", (unsigned long long)i,
                        len[i], (unsigned long long)stride);
    HostJob job{(const uint8_t *)base, n * stride, nullptr, len, stride, 0, nullptr, (uint8_t *)base, 0, n,
                nullptr, nullptr};
    return (int)with_host_answer(__func__, job, n, [&]() -> int64_t {
        if (n == 1 && len[0] <= fcs::kOneBytes) return tx_one((uint8_t *)base, len[0]);
        if (n * stride <= kZeroCopyMaxBytes && (pinned_dev_ptr(base, n * stride) || is_pinned(base))) {
            std::vector<DevState *> devs;
            int rc = engine_devices(&devs);
            if (rc) return rc;
            rc = run_tx_zero_copy(devs[0], (uint8_t *)base, n * stride, stride, nullptr, len, n);
            if (rc <= 0) return rc;   // 1: the frames are not device-mapped; take the staged pipeline
        }
        return run_host_sharded(job, n);
    });
}

int ether_fcs_tx_batch_host(void *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len,
                            uint64_t n) {
    t_host_answered = false;   // early returns below must not report the previous call
    if (n == 0) return 0;
    if (!arena || !off || !len) return fail(EINVAL, "null pointer");
    if (int rc = check_frames(off, len, n, arena_bytes, 4, __func__)) return rc;
    HostJob job{(const uint8_t *)arena, arena_bytes, off, len, 0, 0, nullptr, (uint8_t *)arena, 0, n, nullptr,
                nullptr};
    return (int)with_host_answer(__func__, job, n, [&]() -> int64_t {
        if (n == 1 && len[0] <= fcs::kOneBytes) return tx_one((uint8_t *)arena + off[0], len[0]);
        if (arena_bytes <= kZeroCopyMaxBytes && (pinned_dev_ptr(arena, arena_bytes) || is_pinned(arena))) {
            std::vector<DevState *> devs;
            int rc = engine_devices(&devs);
            if (rc) return rc;
            rc = run_tx_zero_copy(devs[0], (uint8_t *)arena, arena_bytes, 0, off, len, n);
            if (rc <= 0) return rc;
        }
        return run_host_sharded(job, n);
    });
}

// ---- RX verification: frames that carry their FCS trailer ----
int ether_fcs_verify_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len,
                         uint8_t *ok, uint64_t *bad, uint64_t n, void *stream) {
    if (!bad) return fail(EINVAL, "null pointer");
    HIPTRY(hipMemsetAsync(bad, 0, 8, (hipStream_t)stream), "zeroing bad count");
    if (n == 0) return 0;
    if (!arena || !off || !len || !ok) return fail(EINVAL, "null pointer");
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    return launch_var(ds, arena, arena_bytes, off, len, nullptr, n, (hipStream_t)stream, ok,
                      (unsigned long long *)bad);
}

int ether_fcs_verify_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n, uint8_t *ok,
                               uint64_t *bad, void *stream) {
    if (!bad) return fail(EINVAL, "null pointer");
    HIPTRY(hipMemsetAsync(bad, 0, 8, (hipStream_t)stream), "zeroing bad count");
    if (n == 0) return 0;
    if (!base || !ok) return fail(EINVAL, "null pointer");
    if (n > 1 && stride < len) return fail(EINVAL, "stride %llu < len %u", (unsigned long long)stride, len);
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    return launch_fixed(ds, base, stride, len, n, nullptr, (hipStream_t)stream, ok, (unsigned long long *)bad);
}

int64_t ether_fcs_verify_host(const void *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len,
                              uint8_t *ok, uint64_t n) {
    t_host_answered = false;   // early returns below must not report the previous call
    if (n == 0) return 0;
    if (!arena || !off || !len || !ok) return fail(EINVAL, "null pointer");
    if (int rc = check_frames(off, len, n, arena_bytes, 0, __func__)) return rc;
    HostJob job{(const uint8_t *)arena, arena_bytes, off, len, 0, 0, nullptr, nullptr, 0, n, ok, nullptr};
    return with_host_answer(__func__, job, n, [&]() -> int64_t {
        if (arena_bytes <= kZeroCopyMaxBytes) {
            if (const uint8_t *darena = pinned_dev_ptr(arena, arena_bytes)) {   // the RX queue's arena
                std::vector<DevState *> devs;
                const int rc = engine_devices(&devs);
                if (rc) return rc;
                return run_verify_zero_copy(devs[0], darena, arena_bytes, off, len, ok, n);
            }
        }
        std::atomic<uint64_t> bad{0};
        HostJob jb = job;
        jb.bad = &bad;
        const int rc = run_host_sharded(jb, n);
        return rc ? rc : (int64_t)bad.load();
    });
}

// Drop-in for src/ether_fcs.c:4. Synchronous, reentrant. The reference cannot fail and has no
// error channel (SURVEY.md §8b Errors), so an attempt that fails (HIP error, lost completion,
// 10 s timeout) is retried once: the failed lane's stream and result word are quarantined and the
// frame goes through the next lane, freshly created. When the retry fails too (no GPU, a sticky
// device error), or the buffer is too long for the kernels' 32-bit frame lengths, the call is
// answered by the host CRC (fcs_host_crc.cpp): counted in fcs_engine_host_fallbacks and reported
// on stderr the first time, never a wrong FCS and never an abort. Counters: fcs_engine_stats.
uint32_t ether_fcs(const void *data, size_t bsize) {
    if (bsize == 0) return 0;   // src/ether_fcs.c: the loop does not run, crc stays 0
    g_dropin_calls.fetch_add(1, std::memory_order_relaxed);
    auto host = [&](const char *why) {
        static std::atomic<bool> told{false};
        if (!told.exchange(true))
            std::fprintf(stderr, "nstack_fcs: ether_fcs: %s; answering from the host CRC (counted in "
                                 "fcs_engine_host_fallbacks; reported once)\n", why);
        g_host_fallbacks.fetch_add(1, std::memory_order_relaxed);
        return fcs::host_crc32(data, bsize);
    };
    if (bsize > 0xFFFFFFFFull) return host("buffer of 4 GiB or more (the kernels take 32-bit frame lengths)");
    const uint32_t lane = my_lane();
    uint32_t c = 0;
    if (dropin_attempt(data, bsize, lane, &c) == 0) return c;
    const std::string first = g_last_error;
    g_dropin_retries.fetch_add(1, std::memory_order_relaxed);
    if (dropin_attempt(data, bsize, lane + 1, &c) == 0) {
        g_dropin_recovered.fetch_add(1, std::memory_order_relaxed);
        g_last_error = "ether_fcs recovered after: " + first;
        return c;
    }
    const std::string why = "no usable GPU engine (" + g_last_error + "; first attempt: " + first + ")";
    g_last_error = "ether_fcs answered by the host CRC after: " + why;
    return host(why.c_str());
}

uint64_t fcs_engine_host_fallbacks(void) { return g_host_fallbacks.load(std::memory_order_relaxed); }

uint32_t fcs_debug_stream_unit_frames(void) { return fcs::kStUnitFrames; }

// The name of a fixed-length route (fcs_debug_fixed_route, fcs_debug_last_fixed_launch).
static std::string route_name(const fcs::FixedRoute &r) {
    switch (r.kernel) {
        case fcs::FixedKernel::kShort: return "short:" + std::to_string(r.wd);
        case fcs::FixedKernel::kFlat: return "flat";
        case fcs::FixedKernel::kWide4: return "wide4:" + std::to_string(r.wd);
        case fcs::FixedKernel::kWide8: return "wide8:" + std::to_string(r.wd);
        case fcs::FixedKernel::kWide16: return "wide16:" + std::to_string(r.wd);
        case fcs::FixedKernel::kSegment: return r.wd == 24 ? "segment" : "segment:" + std::to_string(r.wd);
        case fcs::FixedKernel::kDma: return "lds-dma";
        case fcs::FixedKernel::kTiny: return "tiny";
        case fcs::FixedKernel::kSingle: return "single";
        case fcs::FixedKernel::kGeneric: return "generic";
    }
    return "?";
}

static int copy_name(const std::string &r, char *out, uint64_t cap) {
    if (!out || cap == 0) return -EINVAL;
    const uint64_t k = std::min<uint64_t>(r.size(), cap - 1);
    std::memcpy(out, r.data(), k);
    out[k] = 0;
    return (int)k;
}

// fcs::route_fixed's decision for a batch, named (no device call).
int fcs_debug_fixed_route(uint64_t base, uint64_t stride, uint32_t len, uint64_t n, char *out, uint64_t cap) {
    if (n == 0) return copy_name("none", out, cap);
    const fcs::KParams p = fixed_params(nullptr, (const void *)base, stride, len, n);
    return copy_name(route_name(fcs::route_fixed(p, n > g_var_threshold.load(std::memory_order_relaxed))), out, cap);
}

// The kernel the last fixed-length launch of this process actually launched (launch_fixed_route
// records it in the case that launches), with its workgroup size: "<route name>/<threads>".
int fcs_debug_last_fixed_launch(char *out, uint64_t cap) {
    const fcs::FixedRoute r = fcs::last_fixed_launch();
    if (r.threads == 0) return copy_name("none", out, cap);
    return copy_name(route_name(r) + "/" + std::to_string(r.threads), out, cap);
}

int64_t fcs_debug_stream_listed(void) {
    DevState *ds = g_last_stream_dev.load(std::memory_order_relaxed);
    if (!ds) return -1;
    DeviceGuard dg(ds->dev);   // read on the device that ran the launch
    HIPTRY(dg.err, "hipSetDevice");
    HIPTRY(device_sync(), "hipDeviceSynchronize");
    uint32_t v = 0;
    HIPTRY(hipMemcpy(&v, ds->d_last_listed, 4, hipMemcpyDeviceToHost), "reading the unit-list length");
    return (int64_t)v;
}

void fcs_engine_host_stats(uint64_t *sharded_calls, uint64_t *shard_jobs) {
    if (sharded_calls) *sharded_calls = g_sharded_calls.load(std::memory_order_relaxed);
    if (shard_jobs) *shard_jobs = g_shard_jobs.load(std::memory_order_relaxed);
}

void fcs_engine_stats(uint64_t *dropin_calls, uint64_t *dropin_retries, uint64_t *dropin_recovered,
                      uint64_t *lane_resets) {
    if (dropin_calls) *dropin_calls = g_dropin_calls.load(std::memory_order_relaxed);
    if (dropin_retries) *dropin_retries = g_dropin_retries.load(std::memory_order_relaxed);
    if (dropin_recovered) *dropin_recovered = g_dropin_recovered.load(std::memory_order_relaxed);
    if (lane_resets) *lane_resets = g_lane_resets.load(std::memory_order_relaxed);
}

uint64_t fcs_engine_host_batches(void) { return g_host_batches.load(std::memory_order_relaxed); }

uint64_t fcs_debug_device_syncs(void) { return g_device_syncs.load(std::memory_order_relaxed); }

#ifdef FCS_FAULT_HOOK
void fcs_debug_hold_small(const uint32_t *word) { g_hold_word.store(word); }
void fcs_debug_fail_next(int attempts) { g_inject_faults = attempts; }
void fcs_debug_timeout_next(int attempts) { g_inject_timeouts = attempts; }
void fcs_debug_fail_batches(int skip, int calls) { g_inject_batch.arm(skip, calls); }
void fcs_debug_late_batches(int skip, int calls) { g_inject_late.arm(skip, calls); }
int fcs_debug_batch_faults_left(void) { return g_inject_batch.left() + g_inject_late.left(); }
// Resources retired after failed host batch calls so far (host-only from kMaxRetired on).
uint32_t fcs_debug_retired(void) { return g_retired.load(std::memory_order_relaxed); }
#endif

int fcs_shard_plan(const uint32_t *len, uint64_t n, uint32_t parts, uint64_t *cut) {
    if (!cut || parts == 0) return fail(EINVAL, "fcs_shard_plan: bad arguments");
    const uint64_t G = parts;
    cut[0] = 0;
    cut[G] = n;
    if (len) {   // byte-balanced: cut g is the first index where the prefix reaches g/G of the bytes
        uint64_t tot = 0;
        for (uint64_t i = 0; i < n; i++) tot += len[i];
        uint64_t acc = 0, g = 1;
        for (uint64_t i = 0; i < n && g < G; i++) {
            acc += len[i];
            while (g < G && (unsigned __int128)acc * G >= (unsigned __int128)tot * g) cut[g++] = i + 1;
        }
        for (; g < G; g++) cut[g] = n;
    } else {
        for (uint64_t g = 1; g < G; g++) cut[g] = (uint64_t)((unsigned __int128)n * g / G);
    }
    return 0;
}

void *fcs_host_alloc(uint64_t bytes) {
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
        fail(ENOMEM, "hipHostMalloc(%llu) failed", (unsigned long long)bytes);
        return nullptr;
    }
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) == hipSuccess && d) {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        g_pinned[(uintptr_t)p] = PinnedRange{bytes, (uint8_t *)d};
    } else {
        (void)hipGetLastError();
    }
    return p;
}

// A kernel set aside by a failed call (quarantined stream) may still read pinned memory the caller
// now frees: wait for the quarantined streams to drain, at most 10 s, and keep the memory mapped (a
// leak, never a GPU page fault) if one is still busy. A stream that has already outlived one such
// wait is remembered as stuck and not waited for again (the memory is kept at once), so a queue's
// teardown after a hung kernel does not cost 10 s per array.
namespace {
std::mutex g_stuck_mu;
std::set<hipStream_t> g_stuck;
}  // namespace

void fcs_host_free(void *p) {
    if (!p) return;
    std::vector<hipStream_t> busy;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto take = [&busy](DevState *ds) {
            std::lock_guard<std::mutex> ql(ds->q_mu);
            busy.insert(busy.end(), ds->q_streams.begin(), ds->q_streams.end());
        };
        for (auto &up : g_dev)
            if (up) take(up.get());
        for (auto &kv : g_alias)
            if (kv.second) take(kv.second.get());
    }
    {
        std::lock_guard<std::mutex> lk(g_stuck_mu);
        for (hipStream_t st : busy)
            if (g_stuck.count(st) && hipStreamQuery(st) == hipErrorNotReady) {
                (void)hipGetLastError();
                return;   // kept: a kernel known to be stuck may still read it
            }
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (hipStream_t st : busy)
        while (hipStreamQuery(st) == hipErrorNotReady) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                (void)hipGetLastError();
                std::lock_guard<std::mutex> lk(g_stuck_mu);
                g_stuck.insert(st);
                return;   // kept: a kernel of a failed call may still read it
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    (void)hipGetLastError();
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        g_pinned.erase((uintptr_t)p);
    }
    hipHostFree(p);
}

int fcs_fill_splitmix64_dev(void *p, uint64_t bytes, uint64_t seed, uint64_t byte_offset, void *stream) {
    if (!bytes) return 0;
    if (!p) return fail(EINVAL, "null pointer");
    HIPTRY(fcs::launch_fill(p, bytes, seed, byte_offset, (hipStream_t)stream), "launching fill");
    return 0;
}

int fcs_read_stream_dev(const void *p, uint64_t bytes, uint32_t *sink, void *stream) {
    if (!p || !sink) return fail(EINVAL, "null pointer");
    HIPTRY(fcs::launch_read_stream(p, bytes, sink, (hipStream_t)stream), "launching read stream");
    return 0;
}

int fcs_dma_stream_dev(const void *p, uint64_t bytes, uint32_t *sink, void *stream) {
    if (!p || !sink) return fail(EINVAL, "null pointer");
    constexpr uint32_t L = 1518;   // the headline kernel's geometry over the same bytes
    if (bytes < 4 * fcs::kDmaItemBytes) return fail(EINVAL, "fcs_dma_stream_dev: at least 24 KiB");
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    fcs::KParams k{};
    k.base = (uint64_t)p;
    k.stride = L;
    k.flen = L;
    k.fseg = 1;
    k.n = bytes / L;
    k.lo4 = floor4((uint64_t)p);
    k.hi4 = ceil4((uint64_t)p + k.n * L);
    k.zmax = fcs::kDmaCover - L;
    k.blob = ds->d_blob;
    k.out = sink;
    const hipStream_t st = (hipStream_t)stream;
    const int grid = grid_for(ds, k.n, fcs::kDmaWgThreads);
    CounterLease lease;
    if ((rc = take_counter(ds, st, k, lease))) return rc;
    HIPTRY(fcs::launch_dma_stream(k, grid, st), "launching the LDS-DMA read stream");
    return 0;
}

int fcs_stream_load_dev(const void *arena, uint64_t arena_bytes, const uint64_t *off, const uint32_t *len,
                        uint64_t n, uint32_t *sink, void *stream) {
    if (!arena || !off || !len || !sink) return fail(EINVAL, "null pointer");
    if (n == 0) return 0;
    DevState *ds = nullptr;
    int rc = current_dev_state(&ds);
    if (rc) return rc;
    fcs::KParams k{};
    k.base = (uint64_t)arena;
    k.off = off;
    k.len = len;
    k.n = n;
    k.lo4 = floor4((uint64_t)arena);
    k.hi4 = ceil4((uint64_t)arena + arena_bytes);
    k.zmax = fcs::kChunkBytes;
    k.blob = ds->d_blob;
    k.out = sink;
    const hipStream_t st = (hipStream_t)stream;
    const uint64_t units = (n + fcs::kStUnitFrames - 1) / fcs::kStUnitFrames;
    CounterLease lease;
    if ((rc = take_counter(ds, st, k, lease))) return rc;
    HIPTRY(fcs::launch_stream(k, (int)std::min<uint64_t>((uint64_t)ds->cus, units), st, true),
           "launching the arena-stream load walk");
    return 0;
}

#ifdef FCS_STAMPS
// Diagnostic stamp sink for FCS_STAMPS measurement builds (tools/stamps.py); not in product builds.
extern "C" int fcs_debug_set_sink(void *p) { g_dbg = (uint64_t *)p; return 0; }
#endif

int fcs_timed_fixed_dev(const void *base, uint64_t stride, uint32_t len, uint64_t n, uint32_t *out,
                        void *stream, int reps, float *ms_per_launch) {
    if (reps <= 0 || !ms_per_launch) return fail(EINVAL, "bad reps/out");
    hipEvent_t a, b;
    HIPTRY(hipEventCreate(&a), "hipEventCreate");
    HIPTRY(hipEventCreate(&b), "hipEventCreate");
    hipStream_t st = (hipStream_t)stream;
    HIPTRY(hipEventRecord(a, st), "hipEventRecord");
    for (int r = 0; r < reps; r++) {
        int rc = ether_fcs_fixed_dev(base, stride, len, n, out, stream);
        if (rc) return rc;
    }
    HIPTRY(hipEventRecord(b, st), "hipEventRecord");
    HIPTRY(hipEventSynchronize(b), "hipEventSynchronize");
    float ms = 0;
    HIPTRY(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
    hipEventDestroy(a);
    hipEventDestroy(b);
    *ms_per_launch = ms / (float)reps;
    return 0;
}

// Introspection for the CPU test-suite: copy the constant table blob the kernel stages into LDS.
// (Table construction is host code; it checksums no frame data.)
int fcs_tables_blob(uint32_t *out, uint64_t words) {
    const std::vector<uint32_t> b = tables().blob();
    if (!out || words < b.size()) return fail(EINVAL, "need %zu words", b.size());
    std::memcpy(out, b.data(), b.size() * 4);
    return (int)b.size();
}

}  // extern "C"

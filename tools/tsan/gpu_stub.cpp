// gpu_stub.cpp — host-only stand-ins for the engine entry points the TX and RX queues call, so the
// queue logic (nstack_amd/csrc/fcs_txq.cpp, fcs_rxq.cpp) can run under the sanitizers without a GPU.
// TX: the "FCS" is a placeholder word and each batch takes 20 us, like a small GPU step. RX: the
// check is the real residue test (the library's host CRC), so dropped frames are the right ones.
// STUB_FAIL_EVERY=k makes every k-th RX submit / wait / synchronous check fail (the queue's
// recovery paths). Test tool only.
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <chrono>
#include <mutex>
#include <deque>
#include <cerrno>
#include "../../nstack_amd/csrc/fcs_host_crc.hpp"

static bool stub_fail() {   // STUB_FAIL_EVERY=k: every k-th call fails
    static const long every = std::getenv("STUB_FAIL_EVERY") ? std::atol(std::getenv("STUB_FAIL_EVERY")) : 0;
    static std::atomic<long> calls{0};
    return every > 0 && ++calls % every == 0;
}
static uint8_t residue_ok(const uint8_t *f, uint32_t len) {
    return len >= 4 && fcs::host_crc32(f, len) == 0x2144DF1Cu;
}
extern "C" {
int ether_fcs_tx_host(void *base, uint64_t stride, const uint32_t *len, uint64_t n) {
    for (uint64_t i = 0; i < n; i++) { uint32_t c = 0xA5A5A5A5u ^ len[i]; std::memcpy((uint8_t*)base + i*stride + len[i], &c, 4); }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    return 0;
}
int ether_fcs_tx_batch_host(void *arena, uint64_t bytes, const uint64_t *off, const uint32_t *len, uint64_t n) {
    (void)bytes;
    for (uint64_t i = 0; i < n; i++) { uint32_t c = 0xA5A5A5A5u ^ len[i]; std::memcpy((uint8_t*)arena + off[i] + len[i], &c, 4); }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
    return 0;
}
int64_t ether_fcs_verify_host(const void *arena, uint64_t, const uint64_t *off, const uint32_t *len, uint8_t *ok,
                              uint64_t n) {
    if (stub_fail()) return -EIO;
    int64_t bad = 0;
    for (uint64_t i = 0; i < n; i++) bad += !(ok[i] = residue_ok((const uint8_t *)arena + off[i], len[i]));
    return bad;
}
const char *fcs_last_error(void) { return "stub"; }
void *fcs_host_alloc(uint64_t b) { return std::malloc(b); }
void fcs_host_free(void *p) { std::free(p); }
}

// Asynchronous form (fcs_device.hpp): the "GPU step" completes 20 us after its submission,
// tickets in order.
namespace fcs {
static std::mutex g_mu;
static uint64_t g_next = 0;
static std::deque<std::pair<uint64_t, std::chrono::steady_clock::time_point>> g_due;
int mapped_submit(uint8_t *arena, uint64_t, const uint64_t *off, const uint32_t *len, uint8_t *ok, uint64_t n,
                  uint64_t *ticket) {
    if (ok && stub_fail()) return -EIO;
    for (uint64_t i = 0; i < n; i++) {
        if (ok) { ok[i] = residue_ok(arena + off[i], len[i]); continue; }
        uint32_t c = 0xA5A5A5A5u ^ len[i];
        std::memcpy(arena + off[i] + len[i], &c, 4);
    }
    std::lock_guard<std::mutex> lk(g_mu);
    *ticket = ++g_next;
    g_due.emplace_back(*ticket, std::chrono::steady_clock::now() + std::chrono::microseconds(20));
    return 0;
}
void host_batch_answered(const char *, const char *) {}
bool last_call_host_answered() { return false; }
int mapped_wait(uint64_t ticket) {
    if (stub_fail()) return -ETIMEDOUT;
    for (;;) {
        std::chrono::steady_clock::time_point t;
        {
            std::lock_guard<std::mutex> lk(g_mu);
            while (!g_due.empty() && g_due.front().first < ticket) g_due.pop_front();
            if (g_due.empty() || g_due.front().first != ticket) return 0;
            t = g_due.front().second;
        }
        std::this_thread::sleep_until(t);
        std::lock_guard<std::mutex> lk(g_mu);
        if (!g_due.empty() && g_due.front().first == ticket) g_due.pop_front();
        return 0;
    }
}
}  // namespace fcs

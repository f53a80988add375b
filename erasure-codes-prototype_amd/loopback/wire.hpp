// The proxy-to-proxy wire format of the reference, carried over in-process channels.
//
// utils.cpp:125-157 int_to_bytes / double_to_bytes copy the host representation (4-byte little-endian int,
// 8-byte IEEE double on x86-64).  A helper proxy's message to the main proxy (handle_repair.cpp:589-603,
// handle_merge.cpp:500-515) is
//     [int cluster_id][int flag = 1][int n][n x block_size bytes][double seconds]
// (flag 0, [int n][(int idx, block) x n][double]: original blocks forwarded through the proxy, only used
// when IF_DIRECT_FROM_NODE is false, metadata.h:14; not exercised by the reference's default build).
// The harness adds one frame of its own, [int cluster_id][int -1]: a helper that failed says so instead
// of leaving the main proxy waiting on its socket.
// The loopback harness replaces the asio socket with a Channel holding whole framed messages.
#pragma once
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <vector>

namespace ecg_loopback {

using Bytes = std::vector<uint8_t>;

inline void put_int(Bytes& b, int v) {
    uint8_t t[sizeof(int)];
    memcpy(t, &v, sizeof(int));
    b.insert(b.end(), t, t + sizeof(int));
}

inline void put_double(Bytes& b, double v) {
    uint8_t t[sizeof(double)];
    memcpy(t, &v, sizeof(double));
    b.insert(b.end(), t, t + sizeof(double));
}

inline void put_bytes(Bytes& b, const char* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }

class Reader {
public:
    explicit Reader(const Bytes& b) : b_(b) {}
    int get_int() {
        int v;
        take(&v, sizeof(int));
        return v;
    }
    double get_double() {
        double v;
        take(&v, sizeof(double));
        return v;
    }
    void get_bytes(char* out, size_t n) { take(out, n); }
    // true when every field was present and the message is fully consumed
    bool done() const { return good_ && at_ == b_.size(); }

private:
    void take(void* out, size_t n) {  // a short message zero-fills and marks the reader bad
        if (at_ + n > b_.size()) {
            memset(out, 0, n);
            good_ = false;
            return;
        }
        memcpy(out, b_.data() + at_, n);
        at_ += n;
    }
    const Bytes& b_;
    size_t at_ = 0;
    bool good_ = true;
};

// One listening endpoint of the main proxy (acceptor_ + SOCKET_PORT_OFFSET, proxy.h): helpers send whole
// framed messages; the main proxy accepts them in arrival order.
class Channel {
public:
    void send(Bytes msg) {
        {
            std::lock_guard<std::mutex> g(mu_);
            q_.push_back(std::move(msg));
        }
        cv_.notify_one();
    }
    // Empty message = nothing arrived within `timeout_s` (a helper died): the caller fails the call.
    Bytes accept(double timeout_s = 120.0) {
        std::unique_lock<std::mutex> g(mu_);
        if (!cv_.wait_for(g, std::chrono::duration<double>(timeout_s), [&] { return !q_.empty(); })) return {};
        Bytes m = std::move(q_.front());
        q_.pop_front();
        return m;
    }

private:
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<Bytes> q_;
};

}  // namespace ecg_loopback

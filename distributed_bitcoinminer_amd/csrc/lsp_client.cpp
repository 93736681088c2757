// lsp_client.cpp -- see lsp_client.hpp.
#include "lsp_client.hpp"

#include <arpa/inet.h>
#include <netdb.h>
#include <poll.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>

#include "wire.hpp"

namespace hm {

static int env_int(const char* name, int dflt) {
    const char* v = getenv(name);
    return (v && *v) ? atoi(v) : dflt;
}

LspParams LspParams::from_env() {
    LspParams p;
    p.epoch_limit = env_int("HM_LSP_EPOCH_LIMIT", p.epoch_limit);
    p.epoch_millis = env_int("HM_LSP_EPOCH_MS", p.epoch_millis);
    p.window_size = env_int("HM_LSP_WINDOW", p.window_size);
    p.max_backoff = env_int("HM_LSP_MAX_BACKOFF", p.max_backoff);
    if (p.epoch_limit < 1) p.epoch_limit = 1;
    if (p.epoch_millis < 1) p.epoch_millis = 1;
    if (p.window_size < 1) p.window_size = 1;
    if (p.max_backoff < 0) p.max_backoff = 0;
    return p;
}

namespace lsp {

static uint32_t int_sum(int v) {  // checksum.go:4-19 (uint32 of a Go int)
    const uint32_t u = (uint32_t)v;
    return (u & 0xFFFFu) + (u >> 16);
}

uint16_t checksum(int conn_id, int seq, int size, const std::string& payload) {
    uint32_t sum = int_sum(conn_id) + int_sum(seq) + int_sum(size);
    for (size_t i = 0; i < payload.size(); i += 2) {  // little-endian 16-bit words
        const uint32_t lo = (uint8_t)payload[i];
        const uint32_t hi = i + 1 < payload.size() ? (uint8_t)payload[i + 1] : 0u;
        sum += lo | (hi << 8);
    }
    while (sum > 0xFFFFu) sum = (sum >> 16) + (sum & 0xFFFFu);  // end-around carry
    return (uint16_t)sum;
}

std::string encode(const Msg& m) {
    char head[160];
    snprintf(head, sizeof head, "{\"Type\":%d,\"ConnID\":%d,\"SeqNum\":%d,\"Size\":%d,\"Checksum\":%u,\"Payload\":",
             m.type, m.conn_id, m.seq, m.size, (unsigned)m.checksum);
    std::string out = head;
    if (m.has_payload) {
        out += '"';
        out += wire::b64_encode(m.payload);
        out += '"';
    } else {
        out += "null";
    }
    out += '}';
    return out;
}

static bool as_int(const wire::JVal& v, int* out) {
    if (v.kind != wire::JVal::NUM || !v.int_ok || v.mag > 0x7fffffffull) return false;
    *out = v.neg ? -(int)v.mag : (int)v.mag;
    return true;
}

bool decode(const std::string& bytes, Msg* m) {
    std::map<std::string, wire::JVal> o;
    if (!wire::parse_object(bytes, &o)) return false;
    *m = Msg();
    auto it = o.find("type");
    if (it != o.end()) as_int(it->second, &m->type);
    if ((it = o.find("connid")) != o.end()) as_int(it->second, &m->conn_id);
    if ((it = o.find("seqnum")) != o.end()) as_int(it->second, &m->seq);
    if ((it = o.find("size")) != o.end()) as_int(it->second, &m->size);
    if ((it = o.find("checksum")) != o.end()) {
        const wire::JVal& v = it->second;
        if (v.kind == wire::JVal::NUM && v.int_ok && !v.neg && v.mag <= 0xFFFF)
            m->checksum = (uint16_t)v.mag;
    }
    if ((it = o.find("payload")) != o.end() && it->second.kind == wire::JVal::STR) {
        if (!wire::b64_decode(it->second.str, &m->payload)) return false;
        m->has_payload = true;
    }
    return true;
}

bool intact(Msg* m) {
    if (m->type == kConnect || m->type == kAck) return true;
    if (m->size < 0) return false;
    const size_t want = (size_t)m->size;
    if (m->payload.size() < want) return false;
    if (m->payload.size() > want) m->payload.resize(want);
    return checksum(m->conn_id, m->seq, m->size, m->payload) == m->checksum;
}

}  // namespace lsp

using Clock = std::chrono::steady_clock;

static int open_udp(const std::string& hostport, std::string* err) {
    const size_t colon = hostport.rfind(':');
    if (colon == std::string::npos) { *err = "bad host:port"; return -1; }
    std::string host = hostport.substr(0, colon), port = hostport.substr(colon + 1);
    if (host.empty() || host == "localhost") host = "127.0.0.1";
    addrinfo hints{};
    hints.ai_family = AF_UNSPEC;
    hints.ai_socktype = SOCK_DGRAM;
    addrinfo* res = nullptr;
    if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) != 0 || !res) {
        *err = "cannot resolve " + hostport;
        return -1;
    }
    int fd = socket(res->ai_family, SOCK_DGRAM, 0);
    if (fd < 0 || ::connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
        *err = "cannot open UDP socket to " + hostport;
        if (fd >= 0) ::close(fd);
        freeaddrinfo(res);
        return -1;
    }
    freeaddrinfo(res);
    return fd;
}

std::unique_ptr<LspClient> LspClient::connect(const std::string& hostport, const LspParams& p,
                                              std::string* err) {
    std::unique_ptr<LspClient> c(new LspClient());
    c->p_ = p;
    c->fd_ = open_udp(hostport, err);
    if (c->fd_ < 0) return nullptr;
    lsp::Msg conn;
    conn.type = lsp::kConnect;
    const std::string cbytes = lsp::encode(conn);
    char buf[65536];
    for (int epoch = 0; epoch < p.epoch_limit; ++epoch) {
        c->send_raw(cbytes);
        const auto deadline = Clock::now() + std::chrono::milliseconds(p.epoch_millis);
        for (;;) {
            const int ms = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                               deadline - Clock::now()).count();
            if (ms <= 0) break;
            pollfd pf{c->fd_, POLLIN, 0};
            if (poll(&pf, 1, ms) <= 0) continue;
            const ssize_t n = recv(c->fd_, buf, sizeof buf, 0);
            if (n <= 0) continue;
            lsp::Msg m;
            if (!lsp::decode(std::string(buf, (size_t)n), &m) || !lsp::intact(&m)) continue;
            if (m.type == lsp::kAck && m.seq == 0) {
                c->conn_id_ = m.conn_id;
                c->th_ = std::thread(&LspClient::loop, c.get());
                return c;
            }
        }
    }
    *err = "connection couldn't be made";
    return nullptr;
}

LspClient::~LspClient() {
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
    if (fd_ >= 0) ::close(fd_);
}

void LspClient::send_raw(const std::string& bytes) {
    (void)!::send(fd_, bytes.data(), bytes.size(), 0);
    last_tx_ = Clock::now();
}

// Move backlog into the window: every seq below (lowest unacked + WindowSize).
void LspClient::pump_window_locked() {
    while (!backlog_.empty()) {
        const int lowest = inflight_.empty() ? backlog_.front().first : inflight_.begin()->first;
        const int seq = backlog_.front().first;
        if (seq >= lowest + p_.window_size) break;
        Out o;
        o.bytes = std::move(backlog_.front().second);
        backlog_.pop_front();
        send_raw(o.bytes);
        inflight_[seq] = std::move(o);
    }
}

bool LspClient::write(const std::string& payload) {
    std::lock_guard<std::mutex> g(mu_);
    if (lost_ || stop_) return false;
    lsp::Msg m;
    m.type = lsp::kData;
    m.conn_id = conn_id_;
    m.seq = next_seq_++;
    m.size = (int)payload.size();
    m.payload = payload;
    m.has_payload = true;
    m.checksum = lsp::checksum(m.conn_id, m.seq, m.size, m.payload);
    backlog_.emplace_back(m.seq, lsp::encode(m));
    pump_window_locked();
    return true;
}

bool LspClient::read(std::string* payload) {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return !ready_.empty() || lost_ || stop_; });
    if (ready_.empty()) return false;
    *payload = std::move(ready_.front());
    ready_.pop_front();
    return true;
}

void LspClient::close() {
    std::unique_lock<std::mutex> g(mu_);
    cv_.wait(g, [&] { return (inflight_.empty() && backlog_.empty()) || lost_; });
    stop_ = true;
    g.unlock();
    cv_.notify_all();
    if (th_.joinable()) th_.join();
}

void LspClient::loop() {
    char buf[65536];
    lsp::Msg hb;
    hb.type = lsp::kAck;
    hb.conn_id = conn_id_;
    const std::string heartbeat = lsp::encode(hb);
    const auto epoch = std::chrono::milliseconds(p_.epoch_millis);
    // Liveness follows the reference's timers (lsp/client_impl.go:257-286,
    // server_impl.go:397-420): the peer is lost after EpochLimit epochs with
    // nothing received.  The reference server resets its timers on every
    // message, ACK(0) included, and sends its own reminder only after a
    // silent epoch.  So this side keeps quiet for 1.5 epochs before its
    // keepalive: the server's reminder fires first and each side keeps
    // hearing the other while idle.  A client that beats every epoch would
    // keep the server silent and then declare it lost.  With EpochLimit 1 the
    // server must hear from us every epoch, hence half an epoch.
    const auto keepalive = p_.epoch_limit >= 2 ? epoch * 3 / 2 : epoch / 2;
    const auto drop_after = epoch * p_.epoch_limit;
    auto last_rx = Clock::now();
    auto next_tick = last_rx + epoch;  // data resend schedule
    for (;;) {
        Clock::time_point wake;
        {
            std::lock_guard<std::mutex> g(mu_);
            if (stop_) return;
            wake = std::min({next_tick, last_tx_ + keepalive, last_rx + drop_after});
        }
        const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(wake - Clock::now());
        pollfd pf{fd_, POLLIN, 0};
        const int pr = poll(&pf, 1, (int)std::max<int64_t>(0, std::min<int64_t>(ms.count() + 1, 50)));
        if (pr > 0) {
            const ssize_t n = recv(fd_, buf, sizeof buf, 0);
            lsp::Msg m;
            if (n > 0 && lsp::decode(std::string(buf, (size_t)n), &m) && lsp::intact(&m)) {
                last_rx = Clock::now();
                std::lock_guard<std::mutex> g(mu_);
                if (m.type == lsp::kData) {
                    lsp::Msg ack;
                    ack.type = lsp::kAck;
                    ack.conn_id = conn_id_;
                    ack.seq = m.seq;
                    send_raw(lsp::encode(ack));
                    if (m.seq == expected_) {
                        ready_.push_back(std::move(m.payload));
                        ++expected_;
                        for (auto it = pending_.find(expected_); it != pending_.end();
                             it = pending_.find(expected_)) {
                            ready_.push_back(std::move(it->second));
                            pending_.erase(it);
                            ++expected_;
                        }
                        cv_.notify_all();
                    } else if (m.seq > expected_) {
                        pending_.emplace(m.seq, std::move(m.payload));
                    }
                } else if (m.type == lsp::kAck && m.seq > 0) {
                    if (inflight_.erase(m.seq)) {
                        pump_window_locked();
                        cv_.notify_all();
                    }
                }
            }
        }
        const auto now = Clock::now();
        std::lock_guard<std::mutex> g(mu_);
        if (now - last_rx >= drop_after) {
            lost_ = true;
            cv_.notify_all();
            return;
        }
        if (now >= next_tick) {
            next_tick += epoch;
            for (auto& kv : inflight_) {  // resend with capped exponential back-off
                Out& o = kv.second;
                if (o.waited >= o.back_off) {
                    o.waited = 0;
                    send_raw(o.bytes);
                    o.back_off = o.back_off == 0 ? std::min(1, p_.max_backoff)
                                                 : std::min(2 * o.back_off, p_.max_backoff);
                } else {
                    ++o.waited;
                }
            }
        }
        if (now - last_tx_ >= keepalive) send_raw(heartbeat);
    }
}

}  // namespace hm
